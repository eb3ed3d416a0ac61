"""Dropout variants, weight noise and parameter constraints.

Reference: nn/conf/dropout/{Dropout,AlphaDropout,GaussianDropout,GaussianNoise}.java (Dropout.java:84
uses inverted dropout with *retain* probability p), nn/conf/weightnoise/{DropConnect,WeightNoise}.java,
nn/conf/constraint/{MaxNorm,MinMaxNorm,NonNegative,UnitNorm}Constraint.java.
"""
import math

import torch

from .base import Config
from .weights import Distribution, NormalDistribution


class IDropout(Config):
    """applyDropout(x, iteration, epoch, inPlace) -> x'; backprop(grad) uses the saved mask. As in the reference it is
    called only for training passes; ``inPlace`` is accepted for signature parity (the input is never overwritten).

    On the GPU the whole family runs on one counter-based Philox kernel (csrc/nn_misc.hip): no mask is stored, the
    backward regenerates it from the layer's (seed, device counter), and the counter advance is a device op, so
    captured HIP-graph steps draw a fresh mask every replay. CPU tensors use torch's generator and a saved mask."""

    def applyDropout(self, x, iteration=0, epoch=0, inPlace=False):
        raise NotImplementedError

    def backprop(self, grad):
        raise NotImplementedError

    def clear(self):
        self._mask = None
        self._native = None

    def _gpu(self, x, mode, **kw):
        """Native forward when x is a bf16/fp32 CUDA tensor; returns None otherwise."""
        from ...ops.dispatch import use_native
        if not use_native(x, "dropout") or x.dtype not in (torch.bfloat16, torch.float32, torch.float16):
            self._native = None
            return None
        from ...ops import nn_misc
        rng = getattr(self, "_rng", None)
        if rng is None or rng.offset.device != x.device:
            rng = self._rng = nn_misc.PhiloxStream(x.device)
        rng.advance()
        y = nn_misc.dropout_native(x, mode, rng, False, **kw)
        self._native = (y, mode, kw)
        return y

    def _gpu_backprop(self, grad):
        nat = getattr(self, "_native", None)
        if nat is None or not grad.is_cuda:
            return None
        from ...ops import nn_misc
        like, mode, kw = nat
        return nn_misc.dropout_grad_native(grad, like, mode, self._rng, **kw).to(grad.dtype)


def _pval(p, iteration, epoch):
    return p.valueAt(iteration, epoch) if hasattr(p, "valueAt") else p


class Dropout(IDropout):
    """Inverted dropout, p = probability of RETAINING an activation (reference Dropout.java:84)."""
    FIELDS = {"p": 0.5}

    def __init__(self, p=0.5, **kw):
        super().__init__(p=p, **kw)

    def applyDropout(self, x, iteration=0, epoch=0, inPlace=False):
        p = _pval(self.p, iteration, epoch)
        if p >= 1.0:
            self._mask = self._native = None
            return x
        y = self._gpu(x, "dropout", p=p)
        if y is not None:
            return y
        self._mask = (torch.rand_like(x, dtype=torch.float32) < p).to(x.dtype) / p
        return x * self._mask

    def backprop(self, grad):
        g = self._gpu_backprop(grad)
        if g is not None:
            return g
        m = getattr(self, "_mask", None)
        return grad if m is None else grad * m


class AlphaDropout(IDropout):
    """Alpha dropout for SELU networks (Klambauer et al. 2017), reference AlphaDropout.java:113."""
    FIELDS = {"p": 0.5}
    ALPHA = 1.6732632423543772848170429916717
    LAMBDA = 1.0507009873554804934193349852946

    def __init__(self, p=0.5, **kw):
        super().__init__(p=p, **kw)

    def a(self, p):
        alpha_p = -self.LAMBDA * self.ALPHA
        return 1.0 / math.sqrt(p + alpha_p * alpha_p * p * (1 - p))

    def b(self, p):
        return -self.a(p) * (1 - p) * (-self.LAMBDA * self.ALPHA)

    def applyDropout(self, x, iteration=0, epoch=0, inPlace=False):
        p = _pval(self.p, iteration, epoch)
        alpha_p = -self.LAMBDA * self.ALPHA
        a, b = self.a(p), self.b(p)
        y = self._gpu(x, "alpha", p=p, a=a, b=b, alpha_p=alpha_p)
        if y is not None:
            return y
        keep = (torch.rand_like(x, dtype=torch.float32) < p).to(x.dtype)
        self._mask = keep * a
        return a * (x * keep + alpha_p * (1 - keep)) + b

    def backprop(self, grad):
        g = self._gpu_backprop(grad)
        return g if g is not None else grad * self._mask


class GaussianDropout(IDropout):
    """Multiplicative N(1, rate/(1-rate)) noise (reference GaussianDropout.java:66)."""
    FIELDS = {"rate": 0.5}

    def __init__(self, rate=0.5, **kw):
        super().__init__(rate=rate, **kw)

    def applyDropout(self, x, iteration=0, epoch=0, inPlace=False):
        r = _pval(self.rate, iteration, epoch)
        std = math.sqrt(r / (1 - r))
        y = self._gpu(x, "gaussian_dropout", sd=std)
        if y is not None:
            return y
        self._mask = (torch.randn_like(x, dtype=torch.float32) * std + 1.0).to(x.dtype)
        return x * self._mask

    def backprop(self, grad):
        g = self._gpu_backprop(grad)
        return g if g is not None else grad * self._mask


class GaussianNoise(IDropout):
    """Additive zero-mean Gaussian noise (reference GaussianNoise.java:53)."""
    FIELDS = {"stddev": 0.1}

    def __init__(self, stddev=0.1, **kw):
        super().__init__(stddev=stddev, **kw)

    def applyDropout(self, x, iteration=0, epoch=0, inPlace=False):
        s = _pval(self.stddev, iteration, epoch)
        y = self._gpu(x, "gaussian_noise", sd=s)
        return y if y is not None else x + torch.randn_like(x) * s

    def backprop(self, grad):
        return grad


def to_dropout(d):
    if d is None or isinstance(d, IDropout):
        return d
    d = float(d)
    if d == 0.0 or d == 1.0:     # reference: dropOut(0) and dropOut(1) both mean "no dropout"
        return None
    return Dropout(d)


# ------------------------------------------------------------------------------- weight noise
class IWeightNoise(Config):
    def getParameter(self, layer, key, param, iteration, epoch, training):
        raise NotImplementedError


class DropConnect(IWeightNoise):
    FIELDS = {"weightRetainProb": 0.5, "applyToBiases": False}

    def __init__(self, weightRetainProb=0.5, **kw):
        super().__init__(weightRetainProb=weightRetainProb, **kw)

    def getParameter(self, layer, key, param, iteration, epoch, training):
        if not training or (key == "b" and not self.applyToBiases):
            return param
        p = _pval(self.weightRetainProb, iteration, epoch)
        return param * (torch.rand_like(param, dtype=torch.float32) < p).to(param.dtype)


class WeightNoise(IWeightNoise):
    FIELDS = {"distribution": None, "applyToBias": False, "additive": True}

    def __init__(self, distribution=None, **kw):
        super().__init__(distribution=distribution or NormalDistribution(0, 1), **kw)

    def getParameter(self, layer, key, param, iteration, epoch, training):
        if not training or (key == "b" and not self.applyToBias):
            return param
        noise = torch.empty(param.shape, dtype=torch.float32)
        self.distribution.sample_(noise)
        noise = noise.to(param.device, param.dtype)
        return param + noise if self.additive else param * noise


# --------------------------------------------------------------------------------- constraints
class LayerConstraint(Config):
    FIELDS = {"params": None, "dimensions": [1]}

    def apply_(self, key, p):
        raise NotImplementedError

    def applies_to(self, key, is_bias):
        if self.params:
            return key in self.params
        return not is_bias

    def _norm_dims(self, p):
        dims = [d for d in (self.dimensions or [1]) if d < p.dim()]
        return dims or list(range(1, p.dim())) or [0]


class MaxNormConstraint(LayerConstraint):
    FIELDS = {"maxNorm": 1.0}

    def __init__(self, maxNorm=1.0, *dims, **kw):
        if dims:
            kw["dimensions"] = list(dims)
        super().__init__(maxNorm=maxNorm, **kw)

    def apply_(self, key, p):
        # reference MaxNormConstraint: norms along the configured dimensions (1 for [nIn, nOut] dense / RNN weights,
        # [1, 2, 3] for [out, in, kH, kW] conv weights)
        n = p.norm(dim=self._norm_dims(p), keepdim=True)
        scale = torch.clamp(self.maxNorm / (n + 1e-6), max=1.0)
        p.mul_(scale)


class MinMaxNormConstraint(LayerConstraint):
    FIELDS = {"min": 0.0, "max": 1.0, "rate": 1.0}

    def __init__(self, min=0.0, max=1.0, rate=1.0, *dims, **kw):
        if dims:
            kw["dimensions"] = list(dims)
        super().__init__(min=min, max=max, rate=rate, **kw)

    def apply_(self, key, p):
        n = p.norm(dim=self._norm_dims(p), keepdim=True)
        clipped = torch.clamp(n, self.min, self.max)
        target = self.rate * clipped + (1 - self.rate) * n
        p.mul_(target / (n + 1e-6))


class NonNegativeConstraint(LayerConstraint):
    def apply_(self, key, p):
        p.clamp_(min=0)


class UnitNormConstraint(LayerConstraint):
    def __init__(self, *dims, **kw):
        if dims:
            kw["dimensions"] = list(dims)
        super().__init__(**kw)

    def apply_(self, key, p):
        p.div_(p.norm(dim=self._norm_dims(p), keepdim=True) + 1e-6)


_ = Distribution  # re-export convenience
