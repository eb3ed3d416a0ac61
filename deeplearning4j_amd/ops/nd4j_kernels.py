"""ND4J op surface on the HIP kernels of ``csrc/nd4j_ops.hip`` (reference: libnd4j's transform / pairwise /
broadcast / reduce / indexreduce families and the reverse / space_to_depth / depth_to_space / space_to_batch /
upsampling2d / mergemax custom ops).

Every entry point takes CUDA tensors of float32 / bfloat16 / float16 and returns ``None`` when the kernel does not
apply (CPU tensor, other dtype, autograd tracking); callers then use the torch expression they always had, so CPU
behaviour is unchanged. ``materialize`` turns ANY strided view (permute / expand / negative-step reverse) into a
contiguous tensor with one kernel, which is how the shape-only layers (space<->depth, space<->batch, upsampling)
run on the GPU without a library copy kernel.
"""
import ctypes

import torch

from . import native
from .native import _ptr, _stream, c_int, c_ll, c_void_p

native.register_sig("dl4j_transform", [c_int, c_int, c_void_p, c_void_p, c_ll, ctypes.c_float, ctypes.c_float,
                                       c_void_p])
native.register_sig("dl4j_transform_bp", [c_int, c_int, c_void_p, c_void_p, c_void_p, c_ll, ctypes.c_float, c_void_p])
native.register_sig("dl4j_binary", [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                    c_int, c_void_p])
native.register_sig("dl4j_reduce_segments", [c_ll, c_ll, c_ll])
native.register_sig("dl4j_reduce_ws_bytes", [c_ll, c_ll, c_ll], restype=c_ll)
native.register_sig("dl4j_reduce", [c_int, c_int, c_void_p, c_void_p, c_void_p, c_ll, c_ll, c_ll, c_int, c_void_p,
                                    c_void_p])
native.register_sig("dl4j_strided_copy", [c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_ll, c_void_p])
native.register_sig("dl4j_strided_copy2", [c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_ll, c_void_p])
native.register_sig("dl4j_col2im", [c_int, c_void_p, c_void_p] + [c_int] * 12 + [c_void_p])
native.register_sig("dl4j_mergemax", [c_int, c_void_p, c_int, c_void_p, c_void_p, c_ll, c_void_p])
native.register_sig("dl4j_mergemax_bp", [c_int, c_void_p, c_void_p, c_void_p, c_int, c_ll, c_void_p])
native.register_sig("dl4j_fill", [c_void_p, c_ll, ctypes.c_uint, c_void_p])
native.register_sig("dl4j_axpy", [c_int, c_void_p, c_void_p, c_ll, ctypes.c_float, c_void_p])
native.register_sig("dl4j_im2col_rows", [c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p])
native.register_sig("dl4j_col2im_rows", [c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p])

DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
CALLS = __import__("collections").Counter()     # kernel launches per entry point (tests check the GPU path ran)

# unary op codes (csrc/nd4j_ops.hip)
OPS = {
    "identity": 0, "relu": 1, "relu6": 2, "leakyrelu": 3, "elu": 4, "selu": 5, "sigmoid": 6, "hardsigmoid": 7,
    "tanh": 8, "hardtanh": 9, "rationaltanh": 10, "rectifiedtanh": 11, "softplus": 12, "softsign": 13, "cube": 14,
    "swish": 15, "gelu_tanh": 16, "gelu": 17, "rrelu": 18,
    "exp": 30, "log": 31, "abs": 32, "neg": 33, "sqrt": 34, "square": 35, "sign": 36, "pow": 37, "reciprocal": 38,
    "floor": 39, "ceil": 40, "round": 41, "sin": 42, "cos": 43, "clip": 44, "step": 45, "add_s": 46, "mul_s": 47,
    "rsub_s": 48, "rdiv_s": 49, "max_s": 50, "min_s": 51, "log1p": 52, "expm1": 53, "rsqrt": 54, "atan": 55,
    "asin": 56, "acos": 57, "sinh": 58, "cosh": 59, "erf": 60, "sub_s": 61, "div_s": 62,
}
ACT_MAX = 18            # ops 0..18 have a derivative kernel
BIN = {"add": 0, "sub": 1, "mul": 2, "div": 3, "rsub": 4, "rdiv": 5, "max": 6, "min": 7, "pow": 8, "sqdiff": 9,
       "eq": 10, "neq": 11, "gt": 12, "gte": 13, "lt": 14, "lte": 15, "fmod": 16, "atan2": 17, "remainder": 18}
RED = {"sum": 0, "mean": 1, "max": 2, "min": 3, "prod": 4, "norm1": 5, "norm2": 6, "normmax": 7, "sumsq": 8,
       "amax": 9, "amin": 10, "var": 11, "std": 12, "argmax": 13, "argmin": 14, "logsumexp": 15}


def enabled():
    import os
    return os.environ.get("DL4J_AMD_ND4J_KERNELS", "1") == "1"


def ok(*ts):
    """All tensors on the GPU in a kernel dtype, nothing tracked by autograd, native library present."""
    if not enabled():
        return False
    for t in ts:
        if not torch.is_tensor(t) or not t.is_cuda or t.dtype not in DT:
            return False
        if t.requires_grad and torch.is_grad_enabled():
            return False
    try:
        native.load()
    except Exception:
        return False
    return True


def _dense(t):
    """Memory-dense layout: contiguous, or channels-last contiguous (elementwise kernels walk the storage)."""
    if t.is_contiguous():
        return True
    if t.dim() == 4:
        return t.is_contiguous(memory_format=torch.channels_last)
    if t.dim() == 5:
        return t.is_contiguous(memory_format=torch.channels_last_3d)
    return False


def _arr(vals):
    return (ctypes.c_longlong * max(1, len(vals)))(*[int(v) for v in vals])


def _check(rc, what):
    native._check(rc, what)
    CALLS[what] += 1


# ------------------------------------------------------------------------------------------------------ transforms
def transform(x, op, a0=0.0, a1=0.0, out=None):
    if not ok(x):
        return None
    code = OPS[op] if isinstance(op, str) else int(op)
    if not _dense(x):
        x = x.contiguous()
    y = out if out is not None else torch.empty_like(x)             # same (dense) strides as x
    if y.stride() != x.stride():
        return None
    _check(native.load().dl4j_transform(DT[x.dtype], code, _ptr(x), _ptr(y), x.numel(), float(a0), float(a1),
                                        _stream()), "transform")
    return y


def transform_bp(z, eps, op, a0=0.0):
    """eps * f'(z) for the activation ops."""
    code = OPS[op] if isinstance(op, str) else int(op)
    if code > ACT_MAX or not ok(z, eps) or z.dtype != eps.dtype or z.shape != eps.shape:
        return None
    if not (_dense(z) and z.stride() == eps.stride()):
        z, eps = z.contiguous(), eps.contiguous()
    out = torch.empty_like(z)
    _check(native.load().dl4j_transform_bp(DT[z.dtype], code, _ptr(z), _ptr(eps), _ptr(out), z.numel(), float(a0),
                                           _stream()), "transform_bp")
    return out


# ------------------------------------------------------------------------------------------------------ broadcast
def binary(a, b, op, out=None):
    """op(a, b) with numpy/ND4J broadcasting; scalars (python numbers) go through the scalar transform ops."""
    code = BIN[op] if isinstance(op, str) else int(op)
    if not torch.is_tensor(b):
        scal = {"add": "add_s", "sub": "sub_s", "mul": "mul_s", "div": "div_s", "rsub": "rsub_s", "rdiv": "rdiv_s",
                "max": "max_s", "min": "min_s", "pow": "pow"}.get(op)
        if scal is None or not ok(a):
            return None
        return transform(a, scal, float(b), out=out)
    if not ok(a, b) or a.dtype != b.dtype:
        return None
    shape = torch.broadcast_shapes(a.shape, b.shape)
    if len(shape) > 8:
        return None
    if out is not None:
        y = out
    elif tuple(a.shape) == tuple(shape) and _dense(a):
        y = torch.empty_like(a)                                     # keep a channels-last operand's layout
    else:
        y = torch.empty(shape, dtype=a.dtype, device=a.device)
    if tuple(y.shape) != tuple(shape) or not _dense(y):
        return None
    lib = native.load()
    if tuple(a.shape) == tuple(shape) == tuple(b.shape) and _dense(a) and a.stride() == b.stride() and \
            a.stride() == y.stride():
        _check(lib.dl4j_binary(DT[a.dtype], code, _ptr(a), _ptr(b), _ptr(y), len(shape), _arr(shape), None, None, 1,
                               _stream()), "binary")
        return y
    if not y.is_contiguous():
        return None
    ea, eb = a.expand(shape), b.expand(shape)
    # expanded views keep the operands' storage offsets: hand the kernel the first element's address
    _check(lib.dl4j_binary(DT[a.dtype], code, _ptr(ea), _ptr(eb), _ptr(y), len(shape), _arr(shape),
                           _arr(ea.stride()), _arr(eb.stride()), 0, _stream()), "binary")
    return y


# ------------------------------------------------------------------------------------------------------ reductions
_ws = {}


def _red_ws(nbytes, device):
    key = (str(device), torch.cuda.current_stream(device).stream_id)
    t = _ws.get(key)
    if t is None or t.numel() < nbytes:
        t = _ws[key] = torch.empty(max(int(nbytes), 64), dtype=torch.uint8, device=device)
    return t


def reduce(x, op, dims=None, keepdims=False, bias_corrected=True):
    """Reduce over ``dims`` (None = all), fp32 accumulation; value ops return x.dtype (as ND4J returns the input
    type), argmax / argmin return int64 indices into the flattened reduced dims."""
    if not ok(x):
        return None
    code = RED[op]
    nd = x.dim()
    dims = list(range(nd)) if dims is None else sorted(d % nd for d in (dims if isinstance(dims, (list, tuple))
                                                                          else [dims]))
    if nd == 0:
        return None
    shape = list(x.shape)
    contiguous_block = dims == list(range(dims[0], dims[-1] + 1))
    if contiguous_block and x.is_contiguous():
        O = 1
        for s in shape[:dims[0]]:
            O *= s
        R = 1
        for s in shape[dims[0]:dims[-1] + 1]:
            R *= s
        I = 1
        for s in shape[dims[-1] + 1:]:
            I *= s
        src = x
    else:
        keep = [d for d in range(nd) if d not in dims]
        src = materialize(x.permute(*keep, *dims))
        if src is None:
            return None
        O = 1
        for d in keep:
            O *= shape[d]
        R = 1
        for d in dims:
            R *= shape[d]
        I = 1
    if O * R * I == 0:
        return None
    lib = native.load()
    is_arg = op in ("argmax", "argmin")
    out = torch.empty(O * I, dtype=torch.int64 if is_arg else torch.float32, device=x.device)
    ws = _red_ws(lib.dl4j_reduce_ws_bytes(O, R, I), x.device)
    _check(lib.dl4j_reduce(DT[x.dtype], code, _ptr(src), None if is_arg else _ptr(out), _ptr(out) if is_arg else None,
                           O, R, I, int(bool(bias_corrected)), _ptr(ws), _stream()), "reduce")
    oshape = [1 if d in dims else shape[d] for d in range(nd)] if keepdims else [shape[d] for d in range(nd)
                                                                               if d not in dims]
    out = out.reshape(oshape)
    return out if is_arg else out.to(x.dtype)


# ------------------------------------------------------------------------------------------------------ data movement
def _copy(src, shape, strides, base, dtype, pad_before=None, src_extent=None):
    """Kernel call: contiguous [shape] from ``src``'s storage at element offset ``base`` and ``strides``."""
    y = torch.empty(tuple(shape), dtype=dtype, device=src.device)
    if y.numel() == 0:
        return y
    off = None if pad_before is None else _arr([-p for p in pad_before])
    lim = None if src_extent is None else _arr(src_extent)
    rc = native.load().dl4j_strided_copy(DT[dtype], ctypes.c_void_p(src.untyped_storage().data_ptr()), _ptr(y),
                                         len(shape), _arr(shape), _arr(strides), off, lim, int(base), _stream())
    _check(rc, "strided_copy")
    return y


def materialize(v):
    """Contiguous copy of the strided view ``v`` (any strides, incl. 0 from expand) on one kernel."""
    if not ok(v) or v.dim() > 8 or v.dim() == 0:
        return None
    return _copy(v, v.shape, v.stride(), v.storage_offset(), v.dtype)


def cast_pad_last(v, dtype, K8, out=None):
    """Contiguous ``dtype`` copy of the strided view ``v`` (any strides, any kernel dtype) with its last dimension
    zero-padded from K to ``K8`` — permute + cast + pad of a GEMM operand in ONE launch (dl4j_strided_copy2).
    ``out``: optional contiguous destination of that shape (e.g. from the open arena)."""
    if not ok(v) or dtype not in DT or v.dim() > 8 or v.dim() == 0:
        return None
    shape = tuple(v.shape[:-1]) + (K8,)
    y = out if out is not None else torch.empty(shape, dtype=dtype, device=v.device)
    if y.numel() == 0:
        return y
    lim = [0] * (v.dim() - 1) + [v.shape[-1]]
    rc = native.load().dl4j_strided_copy2(DT[v.dtype], DT[dtype], ctypes.c_void_p(v.untyped_storage().data_ptr()),
                                          _ptr(y), v.dim(), _arr(shape), _arr(v.stride()), None, _arr(lim),
                                          int(v.storage_offset()), _stream())
    _check(rc, "strided_copy2")
    CALLS["cast_pad_last"] += 1
    return y


def channels_last_copy(x, C=None):
    """Channels-last copy of the 4-D ``x`` (any strides) with its channel dimension zero-padded (C > channels) or
    truncated (C < channels) to ``C``, in one strided-copy launch; None when the kernel does not take x."""
    if not ok(x) or x.dim() != 4:
        return None
    c = x.shape[1]
    C = c if C is None else int(C)
    src = x[:, :C] if C < c else x
    y = cast_pad_last(src.permute(0, 2, 3, 1), x.dtype, C)
    return None if y is None else y.permute(0, 3, 1, 2)


def pad2d(x, pads):
    """Zero padding of the last two dims of an NCHW tensor: pads = (top, bottom, left, right)."""
    if not ok(x) or x.dim() != 4:
        return None
    pt, pb, pl, pr = pads
    n, c, h, w = x.shape
    return _copy(x, (n, c, h + pt + pb, w + pl + pr), x.stride(), x.storage_offset(), x.dtype,
                 pad_before=(0, 0, pt, pl), src_extent=(0, 0, h, w))


def reverse(x, dims):
    """Flip along ``dims`` (negative strides from the last element)."""
    if not ok(x) or x.dim() == 0 or x.dim() > 8:
        return None
    dims = [d % x.dim() for d in (dims if isinstance(dims, (list, tuple)) else [dims])]
    st = list(x.stride())
    base = x.storage_offset()
    for d in dims:
        base += (x.shape[d] - 1) * st[d]
        st[d] = -st[d]
    return _copy(x, x.shape, st, base, x.dtype)


def upsample_nearest2d(x, sh, sw):
    """NCHW nearest upsampling (DL4J Upsampling2D)."""
    if not ok(x) or x.dim() != 4:
        return None
    n, c, h, w = x.shape
    v = x[:, :, :, None, :, None].expand(n, c, h, sh, w, sw)
    y = materialize(v)
    return None if y is None else y.reshape(n, c, h * sh, w * sw)


def upsample_nearest2d_bp(eps, sh, sw):
    if not ok(eps) or eps.dim() != 4:
        return None
    n, c, H, W = eps.shape
    v = eps.reshape(n, c, H // sh, sh, W // sw, sw).permute(0, 1, 2, 4, 3, 5)
    t = materialize(v)
    if t is None:
        return None
    r = reduce(t.reshape(-1, sh * sw), "sum", [1])
    return None if r is None else r.reshape(n, c, H // sh, W // sw)


def space_to_depth(x, b):
    """NCHW, TensorFlow depth order (output channel = (dy*b + dx)*C + c)."""
    if not ok(x) or x.dim() != 4:
        return None
    n, c, H, W = x.shape
    y = materialize(x.reshape(n, c, H // b, b, W // b, b).permute(0, 3, 5, 1, 2, 4))
    return None if y is None else y.reshape(n, b * b * c, H // b, W // b)


def depth_to_space(x, b):
    if not ok(x) or x.dim() != 4:
        return None
    n, cc, h, w = x.shape
    c = cc // (b * b)
    y = materialize(x.reshape(n, b, b, c, h, w).permute(0, 3, 4, 1, 5, 2))
    return None if y is None else y.reshape(n, c, h * b, w * b)


def space_to_batch(x, blocks, pads):
    """NCHW; blocks (bh, bw); pads ((pt, pb), (pl, pr)); output batch index = (oy*bw + ox)*N + n."""
    if not ok(x) or x.dim() != 4:
        return None
    (pt, pb), (pl, pr) = pads
    bh, bw = blocks
    xp = pad2d(x, (pt, pb, pl, pr)) if any((pt, pb, pl, pr)) else x
    if xp is None:
        return None
    n, c, H, W = xp.shape
    y = materialize(xp.reshape(n, c, H // bh, bh, W // bw, bw).permute(3, 5, 0, 1, 2, 4))
    return None if y is None else y.reshape(bh * bw * n, c, H // bh, W // bw)


def batch_to_space(x, blocks, crops):
    if not ok(x) or x.dim() != 4:
        return None
    (ct, cb), (cl, cr) = crops
    bh, bw = blocks
    nb, c, h, w = x.shape
    n = nb // (bh * bw)
    y = materialize(x.reshape(bh, bw, n, c, h, w).permute(2, 3, 4, 0, 5, 1))
    if y is None:
        return None
    y = y.reshape(n, c, h * bh, w * bw)
    if any((ct, cb, cl, cr)):
        y = materialize(y[:, :, ct:h * bh - cb, cl:w * bw - cr])
    return y


def mergemax(xs):
    """Elementwise max over 1..8 same-shape tensors; returns (max, argmax bytes)."""
    if not (1 <= len(xs) <= 8) or not ok(*xs) or any(t.shape != xs[0].shape or t.dtype != xs[0].dtype for t in xs):
        return None
    xs = [t.contiguous() for t in xs]
    y = torch.empty_like(xs[0])
    am = torch.empty(xs[0].shape, dtype=torch.uint8, device=y.device)
    ptrs = (ctypes.c_void_p * len(xs))(*[t.data_ptr() for t in xs])
    _check(native.load().dl4j_mergemax(DT[y.dtype], ptrs, len(xs), _ptr(y), _ptr(am), y.numel(), _stream()),
           "mergemax")
    return y, am


def mergemax_bp(eps, am, n):
    if not ok(eps) or not (1 <= n <= 8):
        return None
    eps = eps.contiguous()
    outs = [torch.empty_like(eps) for _ in range(n)]
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in outs])
    _check(native.load().dl4j_mergemax_bp(DT[eps.dtype], _ptr(eps), _ptr(am), ptrs, n, eps.numel(), _stream()),
           "mergemax_bp")
    return outs


def im2col(x, R, S, stride, pad4, dilation):
    """[N, C*R*S, OH*OW] columns (F.unfold layout) of an NCHW image: zero-pad kernel + one strided copy."""
    if not ok(x) or x.dim() != 4:
        return None
    pt, pb, pl, pr = pad4
    xp = pad2d(x, (pt, pb, pl, pr)) if any(pad4) else x
    if xp is None:
        return None
    N, C, Hp, Wp = xp.shape
    sh, sw = stride
    dh, dw = dilation
    OH = (Hp - dh * (R - 1) - 1) // sh + 1
    OW = (Wp - dw * (S - 1) - 1) // sw + 1
    sN, sC, sH, sW = xp.stride()
    v = xp.as_strided((N, C, R, S, OH, OW), (sN, sC, sH * dh, sW * dw, sH * sh, sW * sw), xp.storage_offset())
    cols = materialize(v)
    return None if cols is None else cols.reshape(N, C * R * S, OH * OW)


def col2im(cols, N, C, Hp, Wp, R, S, stride, dilation, OH, OW):
    """Adjoint of ``im2col`` onto the padded image [N, C, Hp, Wp] (overlapping windows summed, gather form)."""
    if not ok(cols):
        return None
    cols = cols.contiguous()
    x = torch.empty((N, C, Hp, Wp), dtype=cols.dtype, device=cols.device)
    _check(native.load().dl4j_col2im(DT[cols.dtype], _ptr(cols), _ptr(x), N, C, Hp, Wp, R, S, stride[0], stride[1],
                                     dilation[0], dilation[1], OH, OW, _stream()), "col2im")
    return x


def _rows_geom(H, W, R, S, stride, pad_tl, dilation, OH, OW):
    return (ctypes.c_int * 12)(R, S, stride[0], stride[1], pad_tl[0], pad_tl[1], dilation[0], dilation[1], OH, OW, H,
                               W)


def im2col_rows(x, R, S, stride, pad4, dilation, OH, OW):
    """[N*OH*OW, C*R*S] im2col rows (column order c, r, s) of the NCHW-logical ``x`` at any strides, zero padding in
    the same launch; None when the kernel does not take x."""
    if not ok(x) or x.dim() != 4:
        return None
    N, C, H, W = x.shape
    cols = torch.empty((N * OH * OW, C * R * S), dtype=x.dtype, device=x.device)
    g = _rows_geom(H, W, R, S, stride, (pad4[0], pad4[2]), dilation, OH, OW)
    _check(native.load().dl4j_im2col_rows(DT[x.dtype], _ptr(x), _ptr(cols), N, C, _arr(x.stride()), g, _stream()),
           "im2col_rows")
    return cols


def col2im_rows(dcols, N, C, H, W, R, S, stride, pad4, dilation, OH, OW):
    """Adjoint of ``im2col_rows``: the [N, C, H, W] image gradient, channels-last, overlapping taps summed."""
    if not ok(dcols):
        return None
    dcols = dcols.contiguous()
    dx = torch.empty((N, H, W, C), dtype=dcols.dtype, device=dcols.device)
    g = _rows_geom(H, W, R, S, stride, (pad4[0], pad4[2]), dilation, OH, OW)
    _check(native.load().dl4j_col2im_rows(DT[dcols.dtype], _ptr(dcols), _ptr(dx), N, C, g, _stream()), "col2im_rows")
    return dx.permute(0, 3, 1, 2)


def fill_(t, value=0.0):
    """In-place fill of a contiguous (any memory format, dense storage) CUDA tensor with the in-tree fill kernel;
    torch's fill elsewhere (CPU tensors, non-dense views). Returns t."""
    import struct
    if not (t.is_cuda and t.numel() and t.dtype in DT and enabled() and
            (t.is_contiguous() or t.is_contiguous(memory_format=torch.channels_last))):
        return t.fill_(value)
    if t.dtype == torch.float32:
        pat = struct.unpack("<I", struct.pack("<f", float(value)))[0]
    else:
        h = torch.tensor([float(value)], dtype=t.dtype).view(torch.int16).item() & 0xFFFF
        pat = h | (h << 16)
    native._check(native.load().dl4j_fill(_ptr(t), t.numel() * t.element_size(), pat, _stream()), "fill")
    CALLS["fill"] += 1
    return t


def zero_(t):
    return fill_(t, 0.0)


def axpy_(y, x, alpha):
    """y += alpha * x for a dense fp32 CUDA ``y`` and an ``x`` of y's element count (fp32 / bf16 / fp16) with the
    in-tree kernel; torch elsewhere. Returns y."""
    if not (y.is_cuda and y.dtype == torch.float32 and x.dtype in DT and enabled() and y.is_contiguous() and
            x.is_contiguous() and x.numel() == y.numel()):
        return y.add_(x.reshape(y.shape).to(y.dtype), alpha=alpha)
    native._check(native.load().dl4j_axpy(DT[x.dtype], _ptr(x), _ptr(y), y.numel(), float(alpha), _stream()), "axpy")
    CALLS["axpy"] += 1
    return y
