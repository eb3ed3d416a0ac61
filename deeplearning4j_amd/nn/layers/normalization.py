"""Normalization runtime layers: BatchNormalization (+ fused ReLU), LocalResponseNormalization,
LayerNormalization.

BatchNormalization: reference nn/layers/normalization/BatchNormalization.java (forward :250-370,
backward :131-210; mean/var "gradients" are zero :164-167,205-208). The HIP helper
(csrc/batchnorm.hip) does stats + normalize + affine (+ReLU when the network planner fused the
following ActivationLayer(ReLU) into this layer) in NHWC, and the backward in two passes.
"""
import torch

from ... import ops
from .base import LayerImpl, copy_grad_
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


class BatchNormalizationImpl(LayerImpl):
    def __init__(self, conf, index=0, net=None):
        super().__init__(conf, index, net)
        self.fuse_relu = False

    def type(self):
        return "NORMALIZATION"

    def _gb(self):
        c = self.conf
        if c.lockGammaBeta:
            return c.gamma, c.beta
        return self.params["gamma"], self.params["beta"]

    def activate(self, x, training=False, mask=None):
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        if x.dim() not in (2, 4):
            raise ValueError(f"BatchNormalization on activations of rank {x.dim()} not supported {self.layerId()}")
        g, b = self._gb()
        c = self.conf
        pool = getattr(self, "fuse_pool", None)
        if pool is not None and x.dim() == 4:
            # planner fused the following ReLU and max SubsamplingLayer: BN -> ReLU -> pool in one pass
            from .convolution import compute_pad4
            pc = pool.conf
            pad4 = compute_pad4(pc, x.shape[2], x.shape[3], pc.kernelSize, pc.stride, pc.dilation)
            y, self._ctx = ops.bn_pool_forward(x, g, b, self.params["mean"], self.params["var"], training, c.decay,
                                               c.eps, tuple(pc.kernelSize), tuple(pc.stride), pad4)
            self._pool_fused = True
            self._track_deferred_bias(training)
            return y
        self._pool_fused = False
        self._apply_deferred = False
        if getattr(self, "defer_apply", False) and training:
            # shortcut BN folded into its residual consumer (planner): statistics only, the raw input flows on and
            # the consumer applies this layer's normalisation (and runs its backward)
            r = ops.bn_forward(x, g, b, self.params["mean"], self.params["var"], training, c.decay, c.eps,
                               stats_only=True)
            if r is not None:
                self._apply_deferred = True
                y, self._ctx = r
                self._track_deferred_bias(training)
                return y
        # the reference BN layer applies no activation function of its own (BatchNormalization.java:225,398)
        res = getattr(self, "residual", None)
        rbn = getattr(self, "residual_bn", None)
        self._rbn_active = None
        if res is not None and rbn is not None and getattr(rbn, "_apply_deferred", False):
            r = ops.bn_forward(x, g, b, self.params["mean"], self.params["var"], training, c.decay, c.eps,
                               relu=True, residual=res, rctx=rbn._ctx[2])
            if r is None:
                raise RuntimeError(f"{self.layerId()}: fused shortcut BatchNormalization could not run")
            y, self._ctx = r
            self._rbn_active = rbn
        else:
            y, self._ctx = ops.bn_forward(x, g, b, self.params["mean"], self.params["var"], training, c.decay, c.eps,
                                          relu=self.fuse_relu, residual=res)
        self.residual = None
        self._track_deferred_bias(training)
        return y

    def _track_deferred_bias(self, training):
        c = self.conf
        db = getattr(self, "deferred_bias", None)
        if training and db is not None:
            # the producing conv skipped its bias (it cancels in the batch statistics): the running mean must
            # still track E[conv + bias]
            from ...ops.nd4j_kernels import axpy_
            with torch.no_grad():
                axpy_(self.params["mean"], db.params["b"], 1.0 - c.decay)

    def backpropGradient(self, eps):
        gg, gb = self.grads.get("gamma"), self.grads.get("beta")
        if getattr(self, "_apply_deferred", False):
            # the residual consumer already wrote this layer's gamma / beta gradients and hands back the gradient
            # w.r.t. this layer's input
            self._apply_deferred = False
            self._zero_stat_grads()
            return self.make_gradient(), self.backpropDropOut(eps)
        if getattr(self, "_pool_fused", False):
            dx, dgamma, dbeta = ops.bn_pool_backward(eps, self._ctx, gg, gb)
            self.dresidual = None
        elif getattr(self, "_rbn_active", None) is not None:
            rbn = self._rbn_active
            self._rbn_active = None
            dx, dgamma, dbeta, self.dresidual = ops.bn_backward(eps, self._ctx, gg, gb,
                                                                rgrads=(rbn.grads.get("gamma"), rbn.grads.get("beta")))
        else:
            dx, dgamma, dbeta, self.dresidual = ops.bn_backward(eps, self._ctx, gg, gb)
        if gg is not None:
            if dgamma is not gg:
                copy_grad_(gg, dgamma)
            if dbeta is not gb:
                copy_grad_(gb, dbeta)
        self._zero_stat_grads()
        return self.make_gradient(), self.backpropDropOut(dx)

    def _zero_stat_grads(self):
        if not getattr(self, "_stat_grads_zero", False):
            # running-stat "gradients" are zero (reference :164-167,205-208); their NoOp update keeps them so
            self.grads["mean"].zero_()
            self.grads["var"].zero_()
            self._stat_grads_zero = True


def _is_identity(a):
    from ..conf.activations import ActivationIdentity
    return a is None or isinstance(a, ActivationIdentity)


class LocalResponseNormalizationImpl(LayerImpl):
    """Cross-channel LRN: y = x / (k + alpha * sum_{window n} x^2)^beta (reference
    LocalResponseNormalization.java:47,187; cudnnLRNCrossChannel semantics without the /n). HIP kernels
    (csrc/nn_misc.hip) on the GPU in both directions, torch reference on CPU; explicit backward."""

    def activate(self, x, training=False, mask=None):
        from ...ops.nn_misc import lrn_forward
        self.input = x
        c = self.conf
        y, self._ctx = lrn_forward(x, c.n, c.k, c.alpha, c.beta)
        return y.to(x.dtype)

    def backpropGradient(self, eps):
        from ...ops.nn_misc import lrn_backward
        return self.make_gradient(), lrn_backward(eps, self._ctx).to(eps.dtype)


class LayerNormalizationImpl(LayerImpl):
    def activate(self, x, training=False, mask=None):
        self.input = x
        y, self._ctx = ops.layer_norm_forward(x, self.params["gamma"], self.params["beta"], self.conf.eps)
        self._pre = y
        return self.conf.activation.getActivation(y, training) if not _is_identity(self.conf.activation) else y

    def backpropGradient(self, eps):
        if not _is_identity(self.conf.activation):
            eps = self.conf.activation.backprop(self._pre, eps)
        dx, dg, db = ops.layer_norm_backward(eps, self._ctx)
        copy_grad_(self.grads["gamma"], dg)
        copy_grad_(self.grads["beta"], db)
        return self.make_gradient(), dx
