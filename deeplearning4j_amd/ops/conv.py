"""Convolution ops (reference ConvolutionLayer.java:131-265,290-428 im2col+GEMM path and the
CudnnConvolutionHelper contract, CUDA:convolution/CudnnConvolutionHelper.java:297-306,424-470).

``conv2d_forward(x, w, b, stride, pad4, dilation, act)`` — NCHW logical, channels-last physical on GPU.
``conv2d_backward(...)`` -> (dx, dw, db).  pad4 = (top, bottom, left, right) so Same mode's
asymmetric padding is exact.

GPU: bf16 / fp16 implicit-GEMM HIP kernels on MFMA (``csrc/conv_gemm.hip``, ``conv_igemm.hip``, ``conv_wrw.hip``)
when the shape is supported; fp32 convs as im2col / col2im on the in-tree strided-copy and gather kernels
(``csrc/nd4j_ops.hip``) + the in-tree exact-fp32 MFMA GEMM; anything else takes the library path and is counted
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


def _fp32_conv_fwd(x, w, b, stride, pad4, dilation):
    """fp32 conv on the GPU without the library: im2col (zero-pad + strided-copy kernels, ops/nd4j_kernels.py) + the
    in-tree exact-fp32 MFMA GEMM (ops/gemm.py) + the broadcast-add kernel for the bias."""
    from . import nd4j_kernels as K
    from .gemm import mmul
    Kc, _, R, S = w.shape
    cols = K.im2col(x, R, S, stride, pad4, dilation)
    if cols is None:
        return None
    N = x.shape[0]
    pt, pb, pl, pr = pad4
    OH = (x.shape[2] + pt + pb - dilation[0] * (R - 1) - 1) // stride[0] + 1
    OW = (x.shape[3] + pl + pr - dilation[1] * (S - 1) - 1) // stride[1] + 1
    y = mmul(w.reshape(Kc, -1).to(torch.float32), cols)                                          # [N, K, L]
    y = y.reshape(N, Kc, OH, OW)
    if b is not None:
        yb = K.binary(y, b.reshape(1, -1, 1, 1).to(y.dtype).contiguous(), "add")
        y = yb if yb is not None else y + b.reshape(1, -1, 1, 1).to(y.dtype)
    return y


def _fp32_conv_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db):
    from . import nd4j_kernels as K
    from .gemm import mmul
    pt, pb, pl, pr = pad4
    N, C, H, W = x.shape
    Hp, Wp = H + pt + pb, W + pl + pr
    Kc, _, R, S = w.shape
    OH, OW = dy.shape[2], dy.shape[3]
    L = OH * OW
    dy3 = dy.reshape(N, Kc, L).to(torch.float32).contiguous()
    dx = dw = db = None
    if need_dx:
        dcols = mmul(w.reshape(Kc, -1).t().to(torch.float32), dy3)                              # [N, CRS, L]
        dxp = K.col2im(dcols, N, C, Hp, Wp, R, S, stride, dilation, OH, OW)
        if dxp is None:
            return None
        dx = K.materialize(dxp[:, :, pt:pt + H, pl:pl + W]) if any(pad4) else dxp
    if need_dw:
        cols = K.im2col(x, R, S, stride, pad4, dilation)
        if cols is None:
            return None
        dw = mmul(dy3.permute(1, 0, 2).reshape(Kc, N * L), cols.permute(0, 2, 1).reshape(N * L, -1)).reshape(w.shape)
    if need_db:
        db = K.reduce(dy3, "sum", [0, 2])
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
