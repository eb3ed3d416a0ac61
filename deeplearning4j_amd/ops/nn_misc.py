"""LRN, dropout family, embedding lookup, depthwise / separable / transposed convolution — HIP kernels of
``csrc/nn_misc.hip`` on the GPU (plus the implicit-GEMM conv kernels for the transposed conv), torch reference code
on CPU. Every op has an explicit backward (no autograd).

Reference: CudnnLocalResponseNormalizationHelper.java:160,199 / LocalResponseNormalization.java:47,187;
NN:nn/conf/dropout/{Dropout.java:84, AlphaDropout.java:113, GaussianDropout.java:66, GaussianNoise.java:53};
EmbeddingLayer.java:71,111; Deconvolution2DLayer.java:112-225; SeparableConvolution2DLayer.java:126-236;
DepthwiseConvolution2DLayer.java.
"""
import ctypes

import torch
import torch.nn.functional as F

from .dispatch import use_native
from .fallback import note

c_void_p, c_int, c_ll, c_float, c_ull = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, \
    ctypes.c_ulonglong

_SIGS = {
    "dl4j_lrn_fwd": [c_int, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_int, c_ll, c_ll, c_ll, c_int, c_float,
                     c_float, c_float, c_int, c_void_p],
    "dl4j_lrn_bwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_int, c_ll, c_ll, c_ll, c_int,
                     c_float, c_float, c_int, c_void_p],
    "dl4j_dropout": [c_int, c_void_p, c_void_p, c_ll, c_ull, c_void_p, c_int, c_int, c_float, c_float, c_float,
                     c_float, c_float, c_void_p],
    "dl4j_emb_gather": [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_ll, c_ll, c_int, c_void_p],
    "dl4j_emb_scatter_add": [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_ll, c_ll, c_int, c_void_p],
    "dl4j_bert_embed_fwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_ll, c_ll,
                            c_int, c_void_p],
    "dl4j_bert_embed_bwd_pt": [c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_ll, c_ll, c_int, c_ll,
                               c_ll, c_void_p],
    "dl4j_dwconv_fwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "dl4j_dwconv_bwd_data": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "dl4j_dwconv_bwd_weight": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
}


def _lib():
    from . import native
    lib = native.load()
    for n, a in _SIGS.items():
        native.register_sig(n, a)
    return lib


def _dt(t):
    return {torch.bfloat16: 1, torch.float32: 0, torch.float16: 2}.get(t.dtype)


def _p(t):
    return None if t is None else c_void_p(t.data_ptr())


def _s():
    from .native import _stream
    return c_void_p(_stream())


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"HIP kernel {what} failed with code {rc}")


def _dense(x):
    """x itself when its strides are a permutation of a dense layout (so empty_like reproduces them)."""
    return x if x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last) else x.contiguous()


# ------------------------------------------------------------------------------------------------ LRN
def _lrn_geom(x):
    N, C = x.shape[0], x.shape[1]
    P = x[0, 0].numel()
    sn, sc = x.stride(0), x.stride(1)
    sp = x.stride(-1) if x.dim() > 2 else 1
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        sp = x.stride(3)                                         # = C; the spatial index p = h*W + w
    elif x.dim() == 4:
        sp = x.stride(3)                                         # = 1 for NCHW-contiguous
    return N, C, P, sn, sc, sp, int(sc == 1)


def lrn_forward(x, n, k, alpha, beta):
    """Cross-channel LRN over a window of ``n`` channels centred on each channel. Returns (y, ctx)."""
    half = int(n) // 2
    if use_native(x, "lrn") and _dt(x) is not None and x.dim() in (2, 4):
        x = _dense(x)
        lib = _lib()
        y = torch.empty_like(x)
        unit = torch.empty_like(x, dtype=torch.float32)
        N, C, P, sn, sc, sp, cf = _lrn_geom(x)
        _check(lib.dl4j_lrn_fwd(_dt(x), _p(x), _p(y), _p(unit), x.numel(), C, P, sn, sc, sp, half, float(k),
                                float(alpha), float(beta), cf, _s()), "lrn_fwd")
        return y, ("native", x, unit, half, float(alpha), float(beta))
    note(x, "lrn", f"{x.dtype} {x.dim()}-D")
    xf = x.float() if x.dtype != torch.float64 else x
    sq = xf * xf
    pad = F.pad(sq.unsqueeze(0), (0, 0) * (x.dim() - 2) + (half, half)).squeeze(0) if x.dim() > 2 else \
        F.pad(sq, (half, half))
    s = sum(pad[:, i:i + x.shape[1]] for i in range(2 * half + 1))
    unit = k + alpha * s
    return (xf * unit.pow(-beta)).to(x.dtype), ("ref", xf, unit, half, float(alpha), float(beta))


def lrn_backward(g, ctx):
    kind, x, unit, half, alpha, beta = ctx
    if kind == "native":
        g = g.to(x.dtype)
        if g.stride() != x.stride():
            g = torch.empty_like(x).copy_(g)
        dx = torch.empty_like(x)
        N, C, P, sn, sc, sp, cf = _lrn_geom(x)
        _check(_lib().dl4j_lrn_bwd(_dt(x), _p(x), _p(g), _p(unit), _p(dx), x.numel(), C, P, sn, sc, sp, half,
                                   alpha, beta, cf, _s()), "lrn_bwd")
        return dx
    gf = g.to(x.dtype)
    t = gf * x * unit.pow(-beta - 1)
    pad = F.pad(t.unsqueeze(0), (0, 0) * (x.dim() - 2) + (half, half)).squeeze(0) if x.dim() > 2 else \
        F.pad(t, (half, half))
    s = sum(pad[:, i:i + x.shape[1]] for i in range(2 * half + 1))
    return gf * unit.pow(-beta) - 2 * alpha * beta * x * s


# ------------------------------------------------------------------------------------------------ dropout
MODES = {"dropout": 0, "alpha": 1, "gaussian_dropout": 2, "gaussian_noise": 3}


class PhiloxStream:
    """Per-layer counter-based RNG state: a fixed 64-bit key and a device-resident call counter. ``advance()``
    bumps the counter with one device op (so HIP-graph replays draw fresh masks); forward and backward of the
    same call read the same counter value and regenerate identical random numbers."""

    def __init__(self, device):
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.offset = torch.zeros(1, dtype=torch.int64, device=device)

    def advance(self):
        self.offset.add_(1)


def dropout_native(x, mode, stream, bwd, p=1.0, a=1.0, b=0.0, alpha_p=0.0, sd=0.0):
    """y = f(x) for the dropout family on the GPU (None when the dtype is not covered)."""
    if _dt(x) is None:
        return None
    x = _dense(x)
    y = torch.empty_like(x)
    _check(_lib().dl4j_dropout(_dt(x), _p(x), _p(y), x.numel(), c_ull(stream.seed), _p(stream.offset),
                               MODES[mode], int(bwd), float(p), float(a), float(b), float(alpha_p), float(sd),
                               _s()), "dropout")
    return y


def dropout_grad_native(g, like, mode, stream, **kw):
    """Backward of ``dropout_native`` for gradient ``g`` laid out like the forward input ``like``."""
    g = g.to(like.dtype)
    if g.stride() != _dense(like).stride():
        g = torch.empty_like(_dense(like)).copy_(g)
    return dropout_native(g, mode, stream, True, **kw)


# ------------------------------------------------------------------------------------------------ embedding
def embedding_forward(W, idx):
    """Rows of W [V, D] for integer ``idx`` (any shape) -> [*idx.shape, D]."""
    flat = idx.reshape(-1)
    if use_native(W, "embedding") and _dt(W) is not None and W.dim() == 2:
        fi = flat.to(torch.int64).contiguous()
        out = torch.empty((fi.numel(), W.shape[1]), dtype=W.dtype, device=W.device)
        _check(_lib().dl4j_emb_gather(_dt(W), _p(W), _p(fi), _p(out), fi.numel(), W.shape[1], W.stride(0),
                                      W.stride(1), W.shape[0], _s()), "emb_gather")
        return out.reshape(tuple(idx.shape) + (W.shape[1],))
    note(W, "embedding", f"gather {W.dtype}")
    return W.index_select(0, flat.long()).reshape(tuple(idx.shape) + (W.shape[1],))


def embedding_backward_(dW, idx, g):
    """dW [V, D] (fp32 gradient view) += scatter of g [*idx.shape, D] rows at ``idx``."""
    flat = idx.reshape(-1)
    D = dW.shape[1]
    g2 = g.reshape(-1, D)
    if use_native(g, "embedding") and _dt(g2) is not None and dW.dtype == torch.float32:
        fi = flat.to(torch.int64).contiguous()
        g2 = g2.contiguous()
        _check(_lib().dl4j_emb_scatter_add(_dt(g2), _p(g2), _p(fi), _p(dW), fi.numel(), D, dW.stride(0),
                                           dW.stride(1), dW.shape[0], _s()), "emb_scatter_add")
        return dW
    note(g, "embedding", f"scatter {g.dtype}")
    dW.index_add_(0, flat.long(), g2.to(dW.dtype))
    return dW


def bert_embed_forward(Ww, Wp, Wt, idx):
    """[B*T, E] = Wword[idx] + Wpos[t] + Wtype[0] for token ids ``idx`` [B, T] in one HIP pass (fp32 sum, one rounding);
    None when the kernel does not take these operands (the caller sums with torch)."""
    B, T = idx.shape
    E = Ww.shape[1]
    if not (use_native(Ww, "embedding") and _dt(Ww) is not None and Ww.dtype == Wp.dtype == Wt.dtype and
            Ww.dim() == Wp.dim() == Wt.dim() == 2 and Ww.stride(1) == Wp.stride(1) == Wt.stride(1) == 1 and
            Wp.shape[0] >= T and Wp.shape[1] == Wt.shape[1] == E):
        return None
    fi = idx.reshape(-1).to(torch.int64).contiguous()
    out = torch.empty((B * T, E), dtype=Ww.dtype, device=Ww.device)
    rc = _lib().dl4j_bert_embed_fwd(_dt(Ww), _p(Ww), _p(Wp), _p(Wt), _p(fi), _p(out), B * T, T, E, Ww.stride(0),
                                    Wp.stride(0), Ww.shape[0], _s())
    return out if rc == 0 else None


def bert_embed_backward_pt(de, gpos, gtype, B, T):
    """Position gradient gpos [Tmax, E] (rows >= T zeroed) and token-type gradient gtype [ntype, E] (row 0 = sum of
    every row of de [B*T, E], other rows zeroed), written into fp32 gradient views; False when not taken."""
    if not (use_native(de, "embedding") and _dt(de) is not None and de.is_contiguous() and
            gpos.dtype == gtype.dtype == torch.float32 and gpos.dim() == gtype.dim() == 2 and
            gpos.shape[1] == gtype.shape[1] == de.shape[1] and gpos.shape[0] >= T):
        return False
    rc = _lib().dl4j_bert_embed_bwd_pt(_dt(de), _p(de), _p(gpos), _p(gtype), B, T, gpos.shape[0], de.shape[1],
                                       gpos.stride(0), gpos.stride(1), gtype.shape[0], gtype.stride(0),
                                       gtype.stride(1), _s())
    return rc == 0


# ------------------------------------------------------------------------------------------------ depthwise conv
def _out_size(H, k, s, pt, pb, d):
    return (H + pt + pb - d * (k - 1) - 1) // s + 1


def _dw_geom(x, w, stride, pad4, dilation):
    N, C, H, W_ = x.shape
    dm, Cw, KH, KW = w.shape
    OH = _out_size(H, KH, stride[0], pad4[0], pad4[1], dilation[0])
    OW = _out_size(W_, KW, stride[1], pad4[2], pad4[3], dilation[1])
    gi = (ctypes.c_int * 15)(N, H, W_, C, dm, OH, OW, KH, KW, stride[0], stride[1], pad4[0], pad4[2],
                             dilation[0], dilation[1])
    return gi, OH, OW


def _dw_native_ok(x, w):
    return use_native(x, "depthwise") and _dt(x) is not None and x.dim() == 4 and w.shape[1] == x.shape[1]


def depthwise_forward(x, w, b, stride, pad4, dilation):
    """Depthwise conv: x [N, C, H, W], w [dm, C, kh, kw] (reference layout) -> [N, C*dm, OH, OW]."""
    dm, C, KH, KW = w.shape
    if _dw_native_ok(x, w):
        x = x.contiguous(memory_format=torch.channels_last)
        gi, OH, OW = _dw_geom(x, w, stride, pad4, dilation)
        wr = w.float().permute(2, 3, 1, 0).reshape(KH * KW, C * dm).contiguous()
        bias = b.float().reshape(-1).contiguous() if b is not None else None
        y = torch.empty((x.shape[0], C * dm, OH, OW), dtype=x.dtype, device=x.device,
                        memory_format=torch.channels_last)
        _check(_lib().dl4j_dwconv_fwd(_dt(x), _p(x), _p(wr), _p(bias), _p(y), gi, _s()), "dwconv_fwd")
        return y
    note(x, "depthwise", f"fwd {x.dtype}")
    wg = w.permute(1, 0, 2, 3).reshape(C * dm, 1, KH, KW).to(x.dtype)
    xp = F.pad(x, (pad4[2], pad4[3], pad4[0], pad4[1]))
    return F.conv2d(xp, wg, b.reshape(-1).to(x.dtype) if b is not None else None, tuple(stride), 0,
                    tuple(dilation), groups=C)


def depthwise_backward(x, w, dy, stride, pad4, dilation, need_dx=True, need_db=False):
    """Returns (dx, dW [dm, C, kh, kw] fp32 (fp64 for fp64 inputs), db fp32 or None)."""
    dm, C, KH, KW = w.shape
    if _dw_native_ok(x, w) and dy.dtype == x.dtype:
        x = x.contiguous(memory_format=torch.channels_last)
        dy = dy.contiguous(memory_format=torch.channels_last)
        gi, OH, OW = _dw_geom(x, w, stride, pad4, dilation)
        lib = _lib()
        wr = w.float().permute(2, 3, 1, 0).reshape(KH * KW, C * dm).contiguous()
        dx = None
        if need_dx:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            _check(lib.dl4j_dwconv_bwd_data(_dt(x), _p(dy), _p(wr), _p(dx), gi, _s()), "dwconv_bwd_data")
        dwr = torch.zeros((KH * KW, C * dm), dtype=torch.float32, device=x.device)
        _check(lib.dl4j_dwconv_bwd_weight(_dt(x), _p(x), _p(dy), _p(dwr), gi, _s()), "dwconv_bwd_weight")
        dW = dwr.reshape(KH, KW, C, dm).permute(3, 2, 0, 1)
        db = None
        if need_db:
            from . import native
            rows = dy.permute(0, 2, 3, 1).reshape(-1, C * dm)
            db = native.channel_sum(rows) if (C * dm) % 8 == 0 else None
            if db is None:
                db = rows.float().sum(0)
        return dx, dW, db
    note(x, "depthwise", f"bwd {x.dtype}")
    wg = w.permute(1, 0, 2, 3).reshape(C * dm, 1, KH, KW).to(x.dtype)
    xp = F.pad(x, (pad4[2], pad4[3], pad4[0], pad4[1]))
    dxp, dwg, _ = torch.ops.aten.convolution_backward(dy.to(x.dtype), xp, wg, None, list(stride), [0, 0],
                                                      list(dilation), False, [0, 0], C, [need_dx, True, False])
    dx = dxp[:, :, pad4[0]:pad4[0] + x.shape[2], pad4[2]:pad4[2] + x.shape[3]] if need_dx else None
    acc = torch.float64 if x.dtype == torch.float64 else torch.float32
    dW = dwg.reshape(C, dm, KH, KW).permute(1, 0, 2, 3).to(acc)
    db = dy.to(acc).sum((0, 2, 3)) if need_db else None
    return dx, dW, db


# ------------------------------------------------------------------------------------------------ transposed conv
def deconv_forward(x, w, b, stride, pad, dilation=(1, 1)):
    """Transposed conv, w [nIn, nOut, kh, kw]. On the GPU it is the conv bwd-data path (ops/conv_native.py; strided
    deconvs phase-split), i.e. the transposed conv of ``Deconvolution2DLayer`` on MFMA."""
    from .conv import conv2d_backward
    N, Cin, H, W_ = x.shape
    _, Cout, R, S = w.shape
    s0, s1 = stride
    OH = (H - 1) * s0 - 2 * pad[0] + dilation[0] * (R - 1) + 1
    OW = (W_ - 1) * s1 - 2 * pad[1] + dilation[1] * (S - 1) + 1
    if use_native(x, "deconv") and x.dtype == torch.bfloat16 and tuple(dilation) == (1, 1) and Cin % 8 == 0 and \
            Cout % 8 == 0 and pad[0] <= R - 1 and pad[1] <= S - 1:
        # transposed conv = bwd-data of the conv with the same stride: strided cases run phase-split (one stride-1
        # sub-conv per output phase), not on a zero-interleaved input
        xz = x.contiguous(memory_format=torch.channels_last)
        shape_x = torch.empty((N, Cout, OH, OW), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        y, _, _ = conv2d_backward(shape_x, w.to(x.dtype), xz, (s0, s1), (pad[0], pad[0], pad[1], pad[1]), (1, 1),
                                  True, False, False)
        if b is not None:
            y = y + b.reshape(1, -1, 1, 1).to(y.dtype)
        return y
    note(x, "deconv", f"fwd {x.dtype}")
    return F.conv_transpose2d(x, w.to(x.dtype), b.reshape(-1).to(x.dtype) if b is not None else None, tuple(stride),
                              tuple(pad), 0, 1, tuple(dilation))


def deconv_backward(x, w, g, stride, pad, dilation=(1, 1), need_db=True, gW=None, gb=None):
    """Returns (dx, dW, db): dx is the forward conv of g (stride s), dW the conv weight gradient with the roles of
    input and output gradient swapped, db the channel sums of g."""
    from .conv import conv2d_backward, conv2d_forward
    pad4 = (pad[0], pad[0], pad[1], pad[1])
    if x.is_cuda:
        g = g.to(x.dtype).contiguous(memory_format=torch.channels_last)
        xc = x.contiguous(memory_format=torch.channels_last)
        dx = conv2d_forward(g, w.to(x.dtype), None, stride, pad4, dilation)
        _, dW, db = conv2d_backward(g, w.to(x.dtype), xc, stride, pad4, dilation, False, True, False,
                                    gW=gW, grads_zeroed=False)
        if dW is None:
            dW = gW
        db = None
        if need_db:
            from . import native
            Cout = g.shape[1]
            rows = g.permute(0, 2, 3, 1).reshape(-1, Cout)
            db = native.channel_sum(rows, out=gb) if use_native(g, "conv") and Cout % 8 == 0 else None
            if db is None:
                db = rows.float().sum(0)
        return dx, dW, db
    wt = w.to(x.dtype)
    dx, dW, db = torch.ops.aten.convolution_backward(g.to(x.dtype), x, wt, [w.shape[1]] if need_db else None,
                                                     list(stride), list(pad), list(dilation), True, [0, 0], 1,
                                                     [True, True, need_db])
    return dx, dW, db
