"""Feed-forward runtime layers: Dense, Activation, Dropout, Embedding, ElementWiseMultiplication.

Dense (reference nn/layers/BaseLayer.java:86,97,334-336): z = xW + b; a = act(z);
backward: delta = act'(z)*eps; dW = x^T delta; db = sum(delta); eps_prev = delta W^T.
The GEMMs run on the in-tree MFMA kernels (ops/gemm.py): bias fused into the forward epilogue, dW accumulated in
fp32 straight into the 'f'-ordered gradient view; the bf16 path keeps W as a bf16 shadow.
"""
import torch

from .base import LayerImpl, add_row, bias_grad_, copy_grad_, matmul, weight_grad_
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


class DenseLayerImpl(LayerImpl):
    def preOutput(self, x, training=False):
        W = self.W("W")
        return matmul(x.to(W.dtype), W, bias=self.Wbias("b") if "b" in self.params else None)

    def activate(self, x, training=False, mask=None):
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        z = self.preOutput(x, training)
        self._z = z
        a = self.conf.activation.getActivation(z, training)
        if mask is not None and a.dim() == 2 and mask.dim() == 2 and mask.shape[1] == 1:
            a = a * mask.to(a.dtype)
        return a

    def backpropGradient(self, eps):
        delta = self.conf.activation.backprop(self._z, eps.to(self._z.dtype))
        x = self.input.to(delta.dtype)
        if "W" in self.grads:
            weight_grad_(self.grads["W"], x.t(), delta)
        if "b" in self.grads:
            bias_grad_(self.grads["b"], delta)
        if not getattr(self, "need_input_grad", True):
            return self.make_gradient(), None
        W = self.W("W")
        eps_prev = matmul(delta.to(W.dtype), W.t())
        eps_prev = self.backpropDropOut(eps_prev)
        return self.make_gradient(), eps_prev


class ElementWiseMultiplicationLayerImpl(LayerImpl):
    """out = act(x * w + b) elementwise (reference nn/layers/feedforward/elementwise)."""

    def activate(self, x, training=False, mask=None):
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        self._z = x * self.W("W").reshape(1, -1) + self.W("b").reshape(1, -1)
        return self.conf.activation.getActivation(self._z, training)

    def backpropGradient(self, eps):
        delta = self.conf.activation.backprop(self._z, eps)
        copy_grad_(self.grads["W"], _acc((delta * self.input)).sum(dim=0))
        copy_grad_(self.grads["b"], _acc(delta).sum(dim=0))
        return self.make_gradient(), self.backpropDropOut(delta * self.W("W").reshape(1, -1))


class ActivationLayerImpl(LayerImpl):
    def activate(self, x, training=False, mask=None):
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self._z = x
        return self.conf.activation.getActivation(x, training)

    def backpropGradient(self, eps):
        d = self.conf.activation.backprop(self._z, eps)
        return self.make_gradient(), self.backpropDropOut(d)


class DropoutLayerImpl(LayerImpl):
    def activate(self, x, training=False, mask=None):
        self.training = training
        return self.applyDropOutIfNecessary(x, training)

    def backpropGradient(self, eps):
        return self.make_gradient(), self.backpropDropOut(eps)


class EmbeddingLayerImpl(LayerImpl):
    """Row gather forward (reference EmbeddingLayer.java:111 pullRows), scatter-add backward (:71); HIP gather /
    atomic scatter-add kernels on the GPU (csrc/nn_misc.hip)."""

    def activate(self, x, training=False, mask=None):
        from ...ops.nn_misc import embedding_forward
        self.training = training
        idx = x.reshape(-1).long()
        self._idx = idx
        W = self.W("W")
        z = embedding_forward(W, idx)
        if "b" in self.params:
            z = add_row(z, self.W("b"))
        self._z = z
        return self.conf.activation.getActivation(z, training)

    def backpropGradient(self, eps):
        from ...ops.nn_misc import embedding_backward_
        delta = self.conf.activation.backprop(self._z, eps)
        gW = self.grads["W"]
        gW.zero_()
        embedding_backward_(gW, self._idx, delta)
        if "b" in self.grads:
            bias_grad_(self.grads["b"], delta)
        return self.make_gradient(), None


class EmbeddingSequenceLayerImpl(EmbeddingLayerImpl):
    """[mb, T] (or [mb,1,T]) indices -> [mb, nOut, T]."""

    def activate(self, x, training=False, mask=None):
        self.training = training
        if x.dim() == 3:
            x = x[:, 0, :]
        mb, T = x.shape
        self._shape = (mb, T)
        out = super().activate(x.reshape(-1), training)           # [mb*T, nOut] (example-major)
        out = out.reshape(mb, T, -1).permute(0, 2, 1)
        if mask is not None:
            out = out * mask.reshape(mb, 1, T).to(out.dtype)
        return out

    def backpropGradient(self, eps):
        mb, T = self._shape
        e = eps.permute(0, 2, 1).reshape(mb * T, -1)
        return super().backpropGradient(e)
