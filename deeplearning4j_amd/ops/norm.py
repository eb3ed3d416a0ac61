"""Batch normalization ops (reference nn/layers/normalization/BatchNormalization.java:131-210 backward,
:250-370 forward; CudnnBatchNormalizationHelper SPATIAL mode).

Numerics contract (reference): batch var is the *biased* variance; eps is added before the sqrt and
the running variance tracks (var + eps), so inference uses std = sqrt(running_var):
    running_mean = decay*running_mean + (1-decay)*mean
    running_var  = decay*running_var  + (1-decay)*(var + eps)
``relu=True`` fuses the following ActivationLayer(ReLU) (forward max(0,.), backward mask) — the
HIP kernel does it in the same pass (``csrc/batchnorm.hip``).
"""
import torch

from .dispatch import use_native
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


def _dims(x):
    return (0,) if x.dim() == 2 else (0, 2, 3)


def _bshape(x):
    return (1, -1) if x.dim() == 2 else (1, -1, 1, 1)


def bn_forward(x, gamma, beta, run_mean, run_var, training, decay, eps, relu=False, residual=None, rctx=None,
               stats_only=False):
    """Returns (y, ctx). gamma/beta may be python floats (lockGammaBeta). Running stats updated in place
    when training. ``residual``: fused shortcut, y = relu(bn(x) + residual) (relu implied).
    HIP-only fusions (None when the kernel path cannot take them; the caller then runs the unfused layers):
    ``stats_only`` returns (x, ctx) after the statistics / running-stat update (the apply is done by the residual
    consumer), ``rctx`` (a stats_only context) applies that shortcut BN to the raw ``residual`` inside this pass."""
    if residual is not None:
        relu = True
    if stats_only or rctx is not None:
        if not (use_native(x, "bn") and x.dim() in (2, 4) and torch.is_tensor(gamma)):
            return None
        from . import native
        return native.bn_fwd(x, gamma, beta, run_mean, run_var, training, decay, eps, relu, residual, rctx=rctx,
                             stats_only=stats_only)
    if use_native(x, "bn") and x.dim() in (2, 4) and torch.is_tensor(gamma):
        from . import native
        r = native.bn_fwd(x, gamma, beta, run_mean, run_var, training, decay, eps, relu, residual)
        if r is not None:
            return r
    from .fallback import note
    note(x, "bn", f"torch path ({x.dtype}, dim {x.dim()})")
    xf = _acc(x)
    dims = _dims(x)
    bs = _bshape(x)
    if training:
        mean = xf.mean(dim=dims)
        var = xf.var(dim=dims, unbiased=False) + eps
        with torch.no_grad():
            run_mean.mul_(decay).add_(mean.reshape(run_mean.shape).to(run_mean.dtype) * (1 - decay))
            run_var.mul_(decay).add_(var.reshape(run_var.shape).to(run_var.dtype) * (1 - decay))
    else:
        mean = _acc(run_mean.reshape(-1))
        var = _acc(run_var.reshape(-1))
    invstd = torch.rsqrt(var)
    g = _acc(gamma.reshape(-1)) if torch.is_tensor(gamma) else torch.full_like(mean, float(gamma))
    b = _acc(beta.reshape(-1)) if torch.is_tensor(beta) else torch.full_like(mean, float(beta))
    xhat = (xf - mean.reshape(bs)) * invstd.reshape(bs)
    y = xhat * g.reshape(bs) + b.reshape(bs)
    if residual is not None:
        y = y + _acc(residual)
    if relu:
        y = torch.relu(y)
    y = y.to(x.dtype)
    if x.dim() == 4 and x.is_cuda:
        y = y.contiguous(memory_format=torch.channels_last)
    return y, ("REF", x, mean, invstd, g, b, relu, y if relu else None, residual is not None)


def bn_backward(dy, ctx, dgamma_out=None, dbeta_out=None, rgrads=None):
    """Returns (dx, dgamma, dbeta, dresidual) — dgamma/dbeta are sums over the batch (not averaged);
    dresidual is None unless the forward fused a residual. The native kernel writes dgamma/dbeta straight
    into ``dgamma_out``/``dbeta_out`` (the layer's fp32 gradient views) when given. With a folded-in shortcut BN
    (forward ``rctx``) dresidual is the gradient w.r.t. that BN's input and ``rgrads`` = its (dgamma, dbeta) views."""
    if ctx[0] == "NATIVE":
        from . import native
        return native.bn_bwd(dy, ctx, dgamma_out, dbeta_out, rgrads=rgrads)
    _, x, mean, invstd, g, b, relu, y, has_res = ctx
    dims = _dims(x)
    bs = _bshape(x)
    dyf = _acc(dy)
    if relu:
        dyf = dyf * (y > 0).to(dyf.dtype)
    xhat = (_acc(x) - mean.reshape(bs)) * invstd.reshape(bs)
    m = x.numel() // x.shape[1]
    dbeta = dyf.sum(dim=dims)
    dgamma = (dyf * xhat).sum(dim=dims)
    dx = (g * invstd).reshape(bs) * (dyf - dbeta.reshape(bs) / m - xhat * (dgamma.reshape(bs) / m))
    dx = dx.to(dy.dtype)
    if x.dim() == 4 and x.is_cuda:
        dx = dx.contiguous(memory_format=torch.channels_last)
    dres = dyf.to(dy.dtype) if has_res else None
    return dx, dgamma, dbeta, dres


def bn_pool_forward(x, gamma, beta, run_mean, run_var, training, decay, eps, kernel, stride, pad4):
    """Fused BatchNorm -> ReLU -> max pool (the ResNet stem tail). Returns (y_pooled, ctx). On the GPU one HIP
    pass applies BN+ReLU and pools (the BN output is never materialised); elsewhere it composes the reference
    ops, so results are identical up to rounding."""
    if use_native(x, "bn") and x.dim() == 4 and torch.is_tensor(gamma):
        from . import native
        r = native.bn_pool_fwd(x, gamma, beta, run_mean, run_var, training, decay, eps, kernel, stride, pad4)
        if r is not None:
            return r
    from .pool import pool2d_forward
    y_bn, bctx = bn_forward(x, gamma, beta, run_mean, run_var, training, decay, eps, relu=True)
    y, pctx = pool2d_forward(y_bn, "MAX", kernel, stride, pad4)
    return y, ("COMPOSED", bctx, pctx, tuple(x.shape))


def bn_pool_backward(dy, ctx, dgamma_out=None, dbeta_out=None):
    """Returns (dx, dgamma, dbeta) for bn_pool_forward."""
    if ctx[0] == "NATIVE_POOL":
        from . import native
        return native.bn_pool_bwd(dy, ctx, dgamma_out, dbeta_out)
    from .pool import pool2d_backward
    _, bctx, pctx, xshape = ctx
    d = pool2d_backward(dy, pctx)
    if tuple(d.shape[2:]) != tuple(xshape[2:]):                 # truncated windows: rows/cols never pooled
        full = torch.zeros(xshape, dtype=d.dtype, device=d.device)
        full[:, :, :d.shape[2], :d.shape[3]] = d
        d = full
    dx, dgamma, dbeta, _ = bn_backward(d, bctx, dgamma_out, dbeta_out)
    return dx, dgamma, dbeta


def bn_forward_inference_only(x, gamma, beta, run_mean, run_var, relu=False):
    y, _ = bn_forward(x, gamma, beta, run_mean, run_var, False, 0.0, 0.0, relu)
    return y


def layer_norm_forward(x, gamma, beta, eps):
    """LayerNorm over dim 1 of [mb, n] (or [mb, n, T]); returns (y, ctx)."""
    xf = _acc(x)
    if x.dim() == 3:
        xf = xf.transpose(1, 2)
    mean = xf.mean(dim=-1, keepdim=True)
    var = xf.var(dim=-1, unbiased=False, keepdim=True)
    invstd = torch.rsqrt(var + eps)
    xhat = (xf - mean) * invstd
    y = xhat * _acc(gamma.reshape(-1)) + _acc(beta.reshape(-1))
    if x.dim() == 3:
        y = y.transpose(1, 2)
    return y.to(x.dtype), (xhat, invstd, _acc(gamma.reshape(-1)), x.dim())


def layer_norm_backward(dy, ctx):
    xhat, invstd, g, nd = ctx
    d = _acc(dy)
    if nd == 3:
        d = d.transpose(1, 2)
    n = xhat.shape[-1]
    red = tuple(range(d.dim() - 1))
    dgamma = (d * xhat).sum(dim=red)
    dbeta = d.sum(dim=red)
    dxhat = d * g
    dx = invstd * (dxhat - dxhat.mean(dim=-1, keepdim=True) - xhat * (dxhat * xhat).mean(dim=-1, keepdim=True))
    if nd == 3:
        dx = dx.transpose(1, 2)
    _ = n
    return dx.to(dy.dtype), dgamma, dbeta
