"""Convolution ops (reference ConvolutionLayer.java:131-265,290-428 im2col+GEMM path and the
CudnnConvolutionHelper contract, CUDA:convolution/CudnnConvolutionHelper.java:297-306,424-470).

``conv2d_forward(x, w, b, stride, pad4, dilation, act)`` — NCHW logical, channels-last physical on GPU.
``conv2d_backward(...)`` -> (dx, dw, db).  pad4 = (top, bottom, left, right) so Same mode's
asymmetric padding is exact.

GPU: bf16 / fp16 implicit-GEMM HIP kernels on MFMA (``csrc/conv_gemm.hip``, ``conv_igemm.hip``, ``conv_wrw.hip``)
when the shape is supported; fp32 convs as row-per-pixel im2col / col2im kernels (``csrc/nd4j_ops.hip``) + one
in-tree exact-fp32 MFMA GEMM per product; anything else takes the library path and is counted
(ops/fallback.py).
CPU: torch reference (fp32/fp64).
"""
import torch
import torch.nn.functional as F

from .dispatch import use_native


def _sym(pad4):
    pt, pb, pl, pr = pad4
    return pt == pb and pl == pr


def _fp32_gemm_ok(x, groups):
    return x.is_cuda and x.dtype == torch.float32 and groups == 1 and x.dim() == 4 and use_native(x, "conv")


def _out_hw(x, R, S, stride, pad4, dilation):
    pt, pb, pl, pr = pad4
    OH = (x.shape[2] + pt + pb - dilation[0] * (R - 1) - 1) // stride[0] + 1
    OW = (x.shape[3] + pl + pr - dilation[1] * (S - 1) - 1) // stride[1] + 1
    return OH, OW


def _fp32_conv_fwd(x, w, b, stride, pad4, dilation):
    """fp32 conv on the GPU without the library: row-per-pixel im2col (one in-tree kernel, padding included) and ONE
    exact-fp32 MFMA GEMM over every image, ``[N*OH*OW, C*R*S] x [C*R*S, K]`` with the bias in its epilogue; the
    output is that product viewed channels-last (no layout copy). Reference: ConvolutionLayer.java:290-428 (im2col +
    gemm, one GEMM per minibatch)."""
    from . import nd4j_kernels as K
    from .gemm import mmul
    Kc, C, R, S = w.shape
    N = x.shape[0]
    OH, OW = _out_hw(x, R, S, stride, pad4, dilation)
    if OH < 1 or OW < 1:
        return None
    cols = K.im2col_rows(x, R, S, stride, pad4, dilation, OH, OW)
    if cols is None:
        return None
    y = mmul(cols, w.reshape(Kc, -1).to(torch.float32).t(),
             bias=None if b is None else b.reshape(-1).to(torch.float32))                     # [N*OH*OW, K]
    return y.reshape(N, OH, OW, Kc).permute(0, 3, 1, 2)


def _fp32_conv_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db):
    """Backward of ``_fp32_conv_fwd``: dX = col2im_rows(dY · W) (gather form, channels-last, no atomics),
    dW = dYᵀ · im2col_rows(X) (one GEMM, the pixel dimension is its K), db = column sums of dY."""
    from . import nd4j_kernels as K
    from .gemm import mmul
    N, C, H, W = x.shape
    Kc, _, R, S = w.shape
    OH, OW = dy.shape[2], dy.shape[3]
    if dy.dtype != torch.float32:
        return None
    dyr = dy.permute(0, 2, 3, 1)
    if not dyr.is_contiguous():
        dyr = K.materialize(dyr)
        if dyr is None:
            return None
    dy2 = dyr.reshape(N * OH * OW, Kc)
    w2 = w.reshape(Kc, -1).to(torch.float32)
    dx = dw = db = None
    if need_dx:
        dx = K.col2im_rows(mmul(dy2, w2), N, C, H, W, R, S, stride, pad4, dilation, OH, OW)
        if dx is None:
            return None
    if need_dw:
        cols = K.im2col_rows(x, R, S, stride, pad4, dilation, OH, OW)
        if cols is None:
            return None
        dw = mmul(dy2.t(), cols).reshape(w.shape)
    if need_db:
        from . import native
        db = native.channel_sum(dy2)
        if db is None:
            db = K.reduce(dy2, "sum", [0])
    return dx, dw, db


def conv2d_forward(x, w, b, stride, pad4, dilation=(1, 1), groups=1, want_stats=False):
    if use_native(x, "conv") and groups == 1:
        from . import native
        y = native.conv2d_fwd(x, w, b, stride, pad4, dilation, want_stats)
        if y is not None:
            return y
    if _fp32_gemm_ok(x, groups):
        y = _fp32_conv_fwd(x, w, b, stride, pad4, dilation)
        if y is not None:
            return y
    from .fallback import note
    note(x, "conv", f"fwd {x.dtype} groups={groups}")
    pt, pb, pl, pr = pad4
    if b is not None:
        b = b.to(x.dtype)
    if _sym(pad4):
        return F.conv2d(x, w, b, tuple(stride), (pt, pl), tuple(dilation), groups)
    xp = F.pad(x, (pl, pr, pt, pb))
    return F.conv2d(xp, w, b, tuple(stride), 0, tuple(dilation), groups)


def conv2d_backward(x, w, dy, stride, pad4, dilation=(1, 1), need_dx=True, need_dw=True, need_db=True,
                    groups=1, gW=None, gb=None, grads_zeroed=False, dx_accum=None):
    """Returns (dx, dW, db). When the native kernels run and fp32 gradient views ``gW``/``gb`` are given,
    dW/db are written straight into them (fp32 accumulation) and returned as None."""
    if use_native(x, "conv") and groups == 1:
        from . import native
        r = native.conv2d_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db, gW, gb,
                               grads_zeroed, dx_accum)
        if r is not None:
            return r
    if _fp32_gemm_ok(x, groups):
        r = _fp32_conv_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db)
        if r is not None:
            return r
    from .fallback import note
    note(x, "conv", f"bwd {x.dtype} groups={groups}")
    pt, pb, pl, pr = pad4
    sym = _sym(pad4)
    xin = x if sym else F.pad(x, (pl, pr, pt, pb))
    padding = [pt, pl] if sym else [0, 0]
    dy = dy.contiguous(memory_format=torch.channels_last) if x.is_cuda and dy.dim() == 4 else dy
    own_db = need_db and dy.is_cuda and dy.dim() == 4
    dx, dw, db = torch.ops.aten.convolution_backward(
        dy, xin, w, [w.shape[0]] if need_db and not own_db else None, list(stride), padding, list(dilation), False,
        [0, 0], groups, [need_dx, need_dw, need_db and not own_db])
    if own_db:
        # bias gradient as a column sum of the contiguous channels-last [N*H*W, K] view (the library reduces over
        # strided N,H,W dims: ~4x slower on the 411 MB ResNet stem gradient)
        K = dy.shape[1]
        rows = dy.permute(0, 2, 3, 1).reshape(-1, K)
        from . import native
        db = native.channel_sum(rows) if use_native(dy, "conv") else None
        if db is None:
            db = rows.sum(0, dtype=torch.float32)
    if need_dx and not sym:
        dx = dx[:, :, pt:pt + x.shape[2], pl:pl + x.shape[3]]
    return dx, dw, db


def conv_transpose2d_forward(x, w, b, stride, padding, dilation=(1, 1)):
    from .fallback import note
    note(x, "deconv", "library transposed convolution")
    return F.conv_transpose2d(x, w, b, tuple(stride), tuple(padding), 0, 1, tuple(dilation))


def depthwise_conv2d_forward(x, w, b, stride, pad4, dilation, depth_mult):
    """w: [dm, C, kh, kw] (reference sconv2d layout) -> grouped conv with C groups."""
    C = x.shape[1]
    wg = w.permute(1, 0, 2, 3).reshape(C * depth_mult, 1, w.shape[2], w.shape[3])
    return conv2d_forward(x, wg, b, stride, pad4, dilation, groups=C)
