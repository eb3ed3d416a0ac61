"""Wrapper / utility runtime layers: FrozenLayer, MaskLayer, MaskZeroLayer
(reference nn/layers/FrozenLayer.java:472, nn/layers/util/{MaskLayer,MaskZeroLayer}.java)."""
import torch

from .base import LayerImpl


class FrozenLayerImpl(LayerImpl):
    """Delegates forward to the wrapped layer (always in inference mode for dropout); backprop stops here:
    zero parameter gradient and no epsilon for earlier layers (reference FrozenLayer.java:80-82)."""

    def __init__(self, conf, index=0, net=None):
        super().__init__(conf, index, net)
        self.inner = conf.underlying.instantiate(index=index, net=net)

    def bind(self):
        self.inner.params, self.inner.cparams, self.inner.grads = self.params, self.cparams, self.grads
        self.inner.net = self.net

    def getInsideLayer(self):
        return self.inner

    def activate(self, x, training=False, mask=None, **kw):
        self.bind()
        return self.inner.activate(x, False, mask)

    def backpropGradient(self, eps, **kw):
        for v in self.grads.values():
            v.zero_()
        return self.make_gradient(), None

    def __getattr__(self, name):
        if name in ("inner",):
            raise AttributeError(name)
        return getattr(self.inner, name)


class FrozenLayerWithBackpropImpl(FrozenLayerImpl):
    """Frozen parameters, but the epsilon still flows to earlier layers (so layers below a frozen block keep
    training): the wrapped layer's backprop runs for its input gradient and its parameter gradient is discarded."""

    def backpropGradient(self, eps, **kw):
        self.bind()
        _, eps_in = self.inner.backpropGradient(eps, **kw)
        for v in self.grads.values():
            v.zero_()
        return self.make_gradient(), eps_in


class MaskLayerImpl(LayerImpl):
    """Applies the current feature mask to activations (and to epsilons in backprop)."""

    def _apply(self, x, mask):
        if mask is None:
            return x
        if x.dim() == 3:
            return x * mask.reshape(mask.shape[0], 1, -1).to(x.dtype)
        if x.dim() == 2:
            return x * mask.reshape(-1, 1).to(x.dtype)
        return x * mask.reshape(mask.shape[0], 1, 1, 1).to(x.dtype)

    def activate(self, x, training=False, mask=None, **kw):
        self.maskArray = mask
        return self._apply(x, mask)

    def backpropGradient(self, eps, **kw):
        return self.make_gradient(), self._apply(eps, self.maskArray)


class MaskZeroLayerImpl(LayerImpl):
    """Derives a [mb, T] mask from time steps whose features all equal maskingValue, then runs the
    wrapped recurrent layer with that mask."""

    def __init__(self, conf, index=0, net=None):
        super().__init__(conf, index, net)
        self.inner = conf.underlying.instantiate(index=index, net=net)

    def getUnderlying(self):
        self.inner.params, self.inner.cparams, self.inner.grads = self.params, self.cparams, self.grads
        return self.inner

    def activate(self, x, training=False, mask=None, **kw):
        self.inner.params, self.inner.cparams, self.inner.grads = self.params, self.cparams, self.grads
        m = (x != self.conf.maskingValue).any(dim=1).to(x.dtype)      # [mb, T]
        return self.inner.activate(x, training, m)

    def backpropGradient(self, eps, **kw):
        return self.inner.backpropGradient(eps)

    def rnnClearPreviousState(self):
        if hasattr(self.inner, "rnnClearPreviousState"):
            self.inner.rnnClearPreviousState()


_ = torch
