"""SameDiff layer runtime (reference nn/layers/samediff/SameDiffLayer.java, conf/layers/samediff/SDLayerParams.java).

Forward records the user's ``defineLayer(sd, input, paramTable)`` into a SameDiff graph over the layer's parameter
views; backward runs that graph's reverse pass (each op's explicit derivative, samediff/autodiff.py) seeded with the
layer's epsilon, and writes the parameter gradients straight into the flat gradient views.
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
    def _run(self, x):
        sd = SameDiff()
        inp = sd.placeHolder("input", x.detach())
        table = {}
        for k in self.params.keys():
            p = self.params[k].detach()
            table[k] = sd.var(k, p.to(x.dtype) if x.is_floating_point() else p)
        out = self.conf.defineLayer(sd, inp, table)
        if isinstance(out, (list, tuple)):
            out = out[0]
        return sd, out

    def activate(self, x, training=False, mask=None, **kw):
        self.input = x
        sd, out = self._run(x)
        self._sd, self._outv = (sd, out) if training else (None, None)
        return out.value

    def backpropGradient(self, eps, **kw):
        if getattr(self, "_sd", None) is None:
            self._sd, self._outv = self._run(self.input)
        sd, out = self._sd, self._outv
        keys = list(self.params.keys())
        grads = sd._backward({out.name: eps.to(out.value.dtype)}, ["input"] + keys, [out.name])
        dx = grads["input"]
        for k in keys:
            g = grads[k]
            if g is None:
                self.grads[k].zero_()
            else:
                self.grads[k].copy_(g.reshape(self.grads[k].shape))
        self._sd = self._outv = None
        if dx is None:
            dx = torch.zeros_like(self.input)
        return self.make_gradient(), dx
