"""2D pooling (reference SubsamplingLayer.java:207-263,341-358; CudnnSubsamplingHelper MAX /
AVERAGE_COUNT_INCLUDE_PADDING). MAX saves the argmax for the backward scatter.

GPU: NHWC HIP kernels (``csrc/pool.hip``) for MAX/AVG bf16/fp32; CPU: torch reference.
"""
import torch
import torch.nn.functional as F

from .dispatch import use_native
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


def _cl_channels(t, C):
    """The first C channels of the 4-D ``t`` as a channels-last tensor (one in-tree strided copy on the GPU)."""
    from . import nd4j_kernels as NK
    y = NK.channels_last_copy(t, C)
    return y if y is not None else t[:, :C].contiguous(memory_format=torch.channels_last)


def pool2d_forward(x, ptype, kernel, stride, pad4, dilation=(1, 1), pnorm=2, eps=1e-8):
    """Returns (y, ctx). ptype in {'MAX','AVG','SUM','PNORM'}."""
    pt, pb, pl, pr = pad4
    if use_native(x, "pool") and ptype in ("MAX", "AVG") and tuple(dilation) == (1, 1):
        from . import native
        C = x.shape[1] if x.dim() == 4 else 0
        if x.dim() == 4 and C % 8:
            # channel counts off the 8-wide vector (LeNet's 20 / 50): zero-padded channels through the same kernel
            from .conv_native import _pad_ch, _r8
            r = native.pool2d_fwd(_pad_ch(x, _r8(C), cl=True), ptype, kernel, stride, pad4)
            if r is not None:
                y, ctx = r
                return _cl_channels(y, C), ("PADC", C, ctx)
        r = native.pool2d_fwd(x, ptype, kernel, stride, pad4)
        if r is not None:
            return r
    from .fallback import note
    note(x, "pool", f"{ptype} {x.dtype}")
    if ptype == "MAX":
        xp = F.pad(x, (pl, pr, pt, pb), value=float("-inf")) if any(pad4) else x
        y, idx = F.max_pool2d(xp, tuple(kernel), tuple(stride), 0, tuple(dilation), return_indices=True)
        return y, ("MAX", x.shape, xp.shape, idx, kernel, stride, pad4, dilation)
    xp = F.pad(x, (pl, pr, pt, pb)) if any(pad4) else x
    if ptype in ("AVG", "SUM"):
        y = F.avg_pool2d(xp, tuple(kernel), tuple(stride), 0, ceil_mode=False, count_include_pad=True)
        if ptype == "SUM":
            y = y * (kernel[0] * kernel[1])
        return y, (ptype, x.shape, xp.shape, None, kernel, stride, pad4, dilation)
    if ptype == "PNORM":
        xa = torch.abs(_acc(xp)) ** pnorm
        s = F.avg_pool2d(xa, tuple(kernel), tuple(stride), 0) * (kernel[0] * kernel[1])
        y = s ** (1.0 / pnorm)
        return y.to(x.dtype), ("PNORM", x.shape, xp.shape, (xp, y), kernel, stride, pad4, dilation, pnorm, eps)
    raise ValueError(ptype)


def pool2d_backward(dy, ctx):
    kind = ctx[0]
    if kind == "PADC":
        from .conv_native import _pad_ch, _r8
        C, inner = ctx[1], ctx[2]
        dx = pool2d_backward(_pad_ch(dy, _r8(C), cl=True), inner)
        return _cl_channels(dx, C)
    if kind == "NATIVE":
        from . import native
        return native.pool2d_bwd(dy, ctx)
    _, xshape, xpshape, aux, kernel, stride, pad4, dilation = ctx[:8]
    pt, pb, pl, pr = pad4
    if kind == "MAX":
        dxp = torch.ops.aten.max_pool2d_with_indices_backward(
            dy, torch.empty(xpshape, dtype=dy.dtype, device=dy.device), list(kernel), list(stride), [0, 0],
            list(dilation), False, aux)
    elif kind in ("AVG", "SUM"):
        dxp = torch.ops.aten.avg_pool2d_backward(
            dy, torch.empty(xpshape, dtype=dy.dtype, device=dy.device), list(kernel), list(stride), [0, 0], False,
            True, None)
        if kind == "SUM":
            dxp = dxp * (kernel[0] * kernel[1])
    elif kind == "PNORM":
        pnorm, eps = ctx[8], ctx[9]
        xp, y = aux
        # d/dx (sum |x|^p)^(1/p) = |x|^(p-1) sign(x) * y^(1-p)
        g = _acc(dy) * torch.clamp(_acc(y), min=eps) ** (1 - pnorm)
        up = torch.ops.aten.avg_pool2d_backward(g, _acc(xp), list(kernel), list(stride), [0, 0], False, True,
                                                None) * (kernel[0] * kernel[1])
        dxp = (up * torch.abs(_acc(xp)) ** (pnorm - 1) * torch.sign(_acc(xp))).to(dy.dtype)
    else:
        raise ValueError(kind)
    if any(pad4):
        dxp = dxp[:, :, pt:pt + xshape[2], pl:pl + xshape[3]]
    return dxp
