"""Output / loss layers (reference nn/layers/BaseOutputLayer.java:82-92,147-178, LossLayer.java,
RnnOutputLayer, RnnLossLayer, CnnLossLayer, CenterLossOutputLayer).

score = (sum_examples loss + fullNetworkL1 + fullNetworkL2) / minibatch  (BaseOutputLayer.computeScore)
MCXENT/NLL + softmax goes through the fused softmax-cross-entropy kernel (ops.softmax_xent).
"""
import torch

from ...ops import softmax_xent
from ..conf.activations import ActivationSoftmax
from ..conf.losses import LossMCXENT
from ..conf.validation import check_labels
from .base import LayerImpl, add_row, bias_grad_, copy_grad_, matmul, weight_grad_
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


def _rnn_to_2d(x):
    mb, n, T = x.shape
    return x.permute(2, 0, 1).reshape(T * mb, n)


def _2d_to_rnn(x, mb):
    n = x.shape[1]
    T = x.shape[0] // mb
    return x.reshape(T, mb, n).permute(1, 2, 0)


def _mask_rnn_to_2d(mask):
    """[mb, T] per-time-step mask -> [T*mb, 1]; [mb, nOut, T] per-output mask (reference
    GradientCheckTestsMasking.testPerOutputMaskingRnn) -> [T*mb, nOut], rows ordered like _rnn_to_2d."""
    if mask is None:
        return None
    if mask.dim() == 3:
        return _rnn_to_2d(mask)
    return mask.t().reshape(-1, 1) if mask.dim() == 2 else mask


class BaseOutputLayerImpl(LayerImpl):
    has_params = True

    def __init__(self, conf, index=0, net=None):
        super().__init__(conf, index, net)
        self.labels = None

    def setLabels(self, labels):
        self.labels = labels

    def getLabels(self):
        return self.labels

    def _fused(self):
        return isinstance(self.conf.lossFn, LossMCXENT) and isinstance(self.conf.activation, ActivationSoftmax) \
            and self.conf.lossFn.weights is None

    def preOutput2d(self, x):
        if not self.has_params:
            return x
        W = self.W("W")
        return matmul(x.to(W.dtype), W, bias=self.Wbias("b") if "b" in self.params else None)

    # 2d views of input / labels / mask -------------------------------------------------------
    def _in2d(self, x):
        return x

    def _lab2d(self, y):
        # 3d time-series labels after an RNN->FF preprocessor (e.g. TBPTT windows): [mb, n, T] -> [mb*T, n], the row
        # order RnnToFeedForwardPreProcessor gives the activations (reference BaseOutputLayer.getLabels2d)
        if y is not None and y.dim() == 3:
            return y.permute(0, 2, 1).reshape(-1, y.shape[1])
        return y

    def _mask2d(self, m):
        return m

    def _out_from2d(self, a):
        return a

    def activate(self, x, training=False, mask=None):
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        self.maskArray = mask
        x2 = self._in2d(x)
        self._x2 = x2
        z = self.preOutput2d(x2)
        self._z = z
        self._cache = None
        if training and getattr(self, "_skip_train_output", False) and self._fused():
            # training step whose output activation nobody reads (the fused loss recomputes the softmax from z):
            # the pre-activation stands in for it
            return self._out_from2d(z)
        return self._out_from2d(self.conf.activation.getActivation(z, training))

    def output(self, x, training=False):
        return self.activate(x, training)

    def _lab_strided(self, y):
        """(mb, (per-example, per-time-step, per-class) strides) addressing the 2-D label rows inside ``y`` in place,
        or None when the rows are not a strided view of it."""
        if y.dim() == 2:
            return y.shape[0], (y.stride(0), 0, y.stride(1))
        return None

    def _loss_and_grad_strided(self):
        """GPU fused softmax-MCXENT straight from the layer's label tensor (no 2-D label copy); the gradient comes
        back as a zero-K-padded GEMM operand when nOut % 8 != 0."""
        z = self._z
        if not (z.is_cuda and z.dim() == 2 and self.maskArray is None and self.labels is not None):
            return None
        from ... import ops
        if not ops.use_native(z, "softmax_xent"):
            return None
        y = self.labels
        if y.device != z.device or y.dtype != torch.float32:
            y = y.to(device=z.device, dtype=torch.float32)
        ls = self._lab_strided(y)
        if ls is None:
            return None
        from ...ops import native
        return native.softmax_xent_strided(z, y, ls[0], ls[1], self.conf.lossFn.softmaxClipEps)

    def _loss_and_grad(self):
        if self._cache is not None:
            return self._cache
        if self.has_params:
            check_labels(self.conf, self.labels, self.index)
        if self._fused():
            r = self._loss_and_grad_strided()
            if r is not None:
                self._cache = r
                return r
        y = self._lab2d(self.labels)
        mask = self._mask2d(self.maskArray)
        if self._fused():
            s, g, _ = softmax_xent(self._z, y.to(self._z.device), mask, self.conf.lossFn.softmaxClipEps)
        else:
            s = self.conf.lossFn.computeScoreArray(y, self._z, self.conf.activation, mask)
            g = self.conf.lossFn.computeGradient(y, self._z, self.conf.activation, mask)
        self._cache = (s, g)
        return self._cache

    def _score_mb(self):
        """The score is averaged over the NETWORK's input minibatch (reference BaseOutputLayer.computeScore divides
        by getInputMiniBatchSize()), which the updater also divides the gradient by; it differs from this layer's
        own input rows after a minibatch-changing layer such as SpaceToBatch."""
        mb = getattr(self, "inputMiniBatchSize", None)
        return mb if mb else self.input.shape[0]

    def computeScore(self, fullNetworkL1=0.0, fullNetworkL2=0.0, training=True):
        s, _ = self._loss_and_grad()
        if s.is_cuda and s.dtype == torch.float32 and s.is_contiguous() and \
                not torch.is_tensor(fullNetworkL1) and not torch.is_tensor(fullNetworkL2):
            from ...ops import native
            if native.load() is not None:
                # (sum + l1 + l2) / minibatch in one in-tree block (fixed order)
                return native.score_reduce(s, float(fullNetworkL1) + float(fullNetworkL2), 1.0 / self._score_mb())
        return (s.sum() + fullNetworkL1 + fullNetworkL2) / self._score_mb()

    def computeScoreForExamples(self, fullNetworkL1=0.0, fullNetworkL2=0.0):
        s, _ = self._loss_and_grad()
        return s + (fullNetworkL1 + fullNetworkL2)

    def backpropGradient(self, eps=None):
        _, delta = self._loss_and_grad()
        if self.has_params:
            x = self._x2.to(delta.dtype)
            weight_grad_(self.grads["W"], x.t(), delta)
            if "b" in self.grads:
                bias_grad_(self.grads["b"], delta)
            W = self.W("W")
            eps2 = matmul(delta.to(W.dtype), W.t())
        else:
            eps2 = delta
        return self.make_gradient(), self.backpropDropOut(self._eps_from2d(eps2))

    def _eps_from2d(self, e):
        return e

    def clear(self):
        super().clear()
        self.labels = None
        self._cache = None


class OutputLayerImpl(BaseOutputLayerImpl):
    GRADS_OVERWRITE = True


class LossLayerImpl(BaseOutputLayerImpl):
    has_params = False


class RnnOutputLayerImpl(BaseOutputLayerImpl):
    GRADS_OVERWRITE = True        # weight_grad_ / bias_grad_ write the whole W / b views
    def _in2d(self, x):
        self._mb = x.shape[0]
        return _rnn_to_2d(x) if x.dim() == 3 else x

    def _lab2d(self, y):
        return _rnn_to_2d(y) if y.dim() == 3 else y

    def _lab_strided(self, y):
        if y.dim() == 3:                                   # [mb, V, T]: row t*mb + b
            return y.shape[0], (y.stride(0), y.stride(2), y.stride(1))
        return super()._lab_strided(y)

    def _mask2d(self, m):
        return _mask_rnn_to_2d(m)

    def _out_from2d(self, a):
        return _2d_to_rnn(a, self._mb) if self.input.dim() == 3 else a

    def _eps_from2d(self, e):
        return _2d_to_rnn(e, self._mb) if self.input.dim() == 3 else e

    def computeScoreForExamples(self, fullNetworkL1=0.0, fullNetworkL2=0.0):
        s, _ = self._loss_and_grad()
        if self.input.dim() == 3:
            s = s.reshape(-1, self._mb).sum(dim=0)
        return s + (fullNetworkL1 + fullNetworkL2)


class RnnLossLayerImpl(RnnOutputLayerImpl):
    has_params = False


class CnnLossLayerImpl(BaseOutputLayerImpl):
    has_params = False

    def _in2d(self, x):
        self._shape = x.shape
        return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1])

    def _lab2d(self, y):
        return y.permute(0, 2, 3, 1).reshape(-1, y.shape[1])

    def _mask2d(self, m):
        if m is None:
            return None
        return m.reshape(-1, 1) if m.dim() == 3 or (m.dim() == 4 and m.shape[1] == 1) else m.permute(
            0, 2, 3, 1).reshape(-1, m.shape[1])

    def _out_from2d(self, a):
        n, c, h, w = self._shape
        return a.reshape(n, h, w, c).permute(0, 3, 1, 2)

    def _eps_from2d(self, e):
        return self._out_from2d(e)

    def computeScoreForExamples(self, fullNetworkL1=0.0, fullNetworkL2=0.0):
        s, _ = self._loss_and_grad()
        n = self._shape[0]
        return s.reshape(n, -1).sum(dim=1) + (fullNetworkL1 + fullNetworkL2)


class CenterLossOutputLayerImpl(BaseOutputLayerImpl):
    """Adds lambda/2 * ||x - c_y||^2 to the score; centers move toward class means with rate alpha."""

    def activate(self, x, training=False, mask=None):
        self._center_sq = None
        return super().activate(x, training, mask)

    def computeScore(self, fullNetworkL1=0.0, fullNetworkL2=0.0, training=True):
        base = super().computeScore(fullNetworkL1, fullNetworkL2, training)
        sq = getattr(self, "_center_sq", None)
        if sq is None:
            c = self.params["cL"]
            d = _acc(self._x2) - _acc(self.labels) @ _acc(c)
            sq = (d * d).sum()
        # with the centers as they were for this forward pass: backprop moves them afterwards, the reference moves
        # them in the update that follows the score (CenterLossOutputLayer.computeScore)
        return base + 0.5 * self.conf.lambda_ * sq / self._score_mb()

    def backpropGradient(self, eps=None):
        g, eps_prev = super().backpropGradient(eps)
        c = self.params["cL"]
        y = _acc(self.labels)
        x = _acc(self._x2)
        d = x - y @ _acc(c)
        self._center_sq = (d * d).sum()
        eps_prev = eps_prev + (self.conf.lambda_ * d).to(eps_prev.dtype)
        if self.conf.gradientCheck:
            # the exact gradient of the center term w.r.t. the centers; the centers themselves stay put
            if "cL" in self.grads:
                self.grads["cL"].copy_((self.conf.lambda_ * (y.t() @ (-d))).to(self.grads["cL"].dtype))
            return g, eps_prev
        with torch.no_grad():
            counts = y.sum(dim=0).clamp(min=1).reshape(-1, 1)
            delta_c = (y.t() @ (-d)) / (counts + 1)
            c.sub_((self.conf.alpha * delta_c).to(c.dtype))
        if "cL" in self.grads:
            self.grads["cL"].zero_()
        return g, eps_prev
