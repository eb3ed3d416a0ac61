"""SameDiff layer runtime (reference nn/layers/samediff/SameDiffLayer.java, conf/layers/samediff/SDLayerParams.java).

Forward runs the user's ``defineLayer(sd, input, paramTable)`` on the layer's parameter views; backward
re-uses the recorded autograd graph of the last training forward (or re-runs the forward under
``enable_grad``) and writes the parameter gradients straight into the flat gradient views.
"""
import torch

from ..nn.layers.base import LayerImpl
from . import SameDiff


class SDLayerParams:
    def __init__(self):
        self.weights = {}
        self.biases = {}

    def clear(self):
        self.weights.clear()
        self.biases.clear()

    def addWeightParam(self, key, shape):
        self.weights[key] = [int(s) for s in shape]

    def addBiasParam(self, key, shape):
        self.biases[key] = [int(s) for s in shape]

    def getParameterKeys(self):
        return list(self.weights) + list(self.biases)

    def getParamShapes(self):
        return {**self.weights, **self.biases}


class SameDiffLayerImpl(LayerImpl):
    def _run(self, x, grad):
        sd = SameDiff()
        keys = list(self.params.keys())
        leaves = {}
        for k in keys:
            p = self.params[k].detach().to(x.dtype if x.is_floating_point() else self.params[k].dtype)
            leaves[k] = p.requires_grad_(grad)
        xin = x.detach().requires_grad_(grad)
        with torch.set_grad_enabled(grad):
            inp = sd.var("input", xin)
            table = {k: sd.var(k, v) for k, v in leaves.items()}
            out = self.conf.defineLayer(sd, inp, table)
            if isinstance(out, (list, tuple)):
                out = out[0]
        return out.value, xin, leaves

    def activate(self, x, training=False, mask=None, **kw):
        self.input = x
        if training:
            self._out, self._xin, self._leaves = self._run(x, True)
            return self._out.detach()
        with torch.no_grad():
            out, _, _ = self._run(x, False)
        return out

    def backpropGradient(self, eps, **kw):
        if getattr(self, "_out", None) is None:
            self._out, self._xin, self._leaves = self._run(self.input, True)
        keys = list(self._leaves)
        grads = torch.autograd.grad(self._out, [self._xin] + [self._leaves[k] for k in keys], eps.to(self._out.dtype),
                                    allow_unused=True)
        dx = grads[0]
        for k, g in zip(keys, grads[1:]):
            if g is None:
                self.grads[k].zero_()
            else:
                self.grads[k].copy_(g.reshape(self.grads[k].shape))
        self._out = None
        return self.make_gradient(), dx
