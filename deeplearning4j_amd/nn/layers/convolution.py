"""Convolution-family runtime layers (reference nn/layers/convolution/*).

ConvolutionLayer: forward = conv + bias (+activation), backward = (dW, db, dx)
(ConvolutionLayer.java:131-265,290-428; helper SPI :173-200,345-375). Same mode pads
top/left = floor(total/2) exactly like ConvolutionUtils.getSameModeTopLeftPadding.
Activations are NCHW logically; on GPU they are kept channels-last in memory (NHWC) so the HIP
implicit-GEMM kernels read contiguous channel vectors.
"""
import torch
import torch.nn.functional as F

from ... import ops
from ..conf.enums import ConvolutionMode
from ..conf.layers import conv_out_size, same_padding
from .base import LayerImpl, copy_grad_
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


def _cl(x):
    if x.is_cuda and x.dim() == 4:
        if x.is_contiguous(memory_format=torch.channels_last):
            return x
        from ...ops import nd4j_kernels as NK
        y = NK.channels_last_copy(x)                              # in-tree strided copy, no library kernel
        return y if y is not None else x.contiguous(memory_format=torch.channels_last)
    return x


def compute_pad4(conf, h, w, kernel=None, stride=None, dilation=None):
    kernel = kernel or conf.kernelSize
    stride = stride or conf.stride
    dilation = dilation or getattr(conf, "dilation", [1, 1]) or [1, 1]
    if conf.convolutionMode == ConvolutionMode.Same:
        oh = conv_out_size(h, kernel[0], stride[0], 0, dilation[0], ConvolutionMode.Same)
        ow = conv_out_size(w, kernel[1], stride[1], 0, dilation[1], ConvolutionMode.Same)
        pt, pb = same_padding(h, oh, kernel[0], stride[0], dilation[0])
        pl, pr = same_padding(w, ow, kernel[1], stride[1], dilation[1])
        return (pt, pb, pl, pr)
    p = conf.padding
    # validate (raises for Strict mode mismatches, as the reference does)
    conv_out_size(h, kernel[0], stride[0], p[0], dilation[0], conf.convolutionMode)
    conv_out_size(w, kernel[1], stride[1], p[1], dilation[1], conf.convolutionMode)
    return (p[0], p[0], p[1], p[1])


def _truncate_input(conf, x, kernel, stride, pad4, dilation):
    """Truncate mode: crop rows/cols that no window reaches so the library conv sees an exact fit."""
    if conf.convolutionMode == ConvolutionMode.Same:
        return x
    h, w = x.shape[2], x.shape[3]
    oh = conv_out_size(h, kernel[0], stride[0], pad4[0], dilation[0], ConvolutionMode.Truncate)
    ow = conv_out_size(w, kernel[1], stride[1], pad4[2], dilation[1], ConvolutionMode.Truncate)
    need_h = (oh - 1) * stride[0] + (kernel[0] - 1) * dilation[0] + 1 - 2 * pad4[0]
    need_w = (ow - 1) * stride[1] + (kernel[1] - 1) * dilation[1] + 1 - 2 * pad4[2]
    if need_h < h or need_w < w:
        return x[:, :, :max(need_h, 0) if need_h < h else h, :max(need_w, 0) if need_w < w else w]
    return x


class ConvolutionLayerImpl(LayerImpl):
    def type(self):
        return "CONVOLUTIONAL"

    extra_pad4 = None     # set by the graph planner when a preceding ZeroPaddingLayer is folded into this conv
    defer_bias = False    # set by the graph planner when a training-mode BatchNormalization absorbs the bias
    dx_accum = None       # set by the graph for one backward call: existing gradient of x to accumulate into
    emit_bn_stats = False  # set by the graph planner when a training-mode BatchNormalization consumes the output

    def _geom(self, x):
        c = self.conf
        pad4 = compute_pad4(c, x.shape[2], x.shape[3])
        if self.extra_pad4 is not None:
            pad4 = tuple(a + b for a, b in zip(pad4, self.extra_pad4))
        return list(c.kernelSize), list(c.stride), pad4, list(c.dilation)

    def preOutput(self, x, training=False):
        k, s, pad4, d = self._geom(x)
        W = self.W("W")
        b = self.params["b"].reshape(-1) if "b" in self.params else None      # master-precision bias
        if self.defer_bias and training:
            b = None
        xt = x     # Truncate mode needs no cropping: output sizes use floor division everywhere
        self._xt = xt
        self._geom_cache = (s, pad4, d)
        return ops.conv2d_forward(_cl(xt.to(W.dtype)), W, b, s, pad4, d,
                                  want_stats=bool(training and self.emit_bn_stats))

    def activate(self, x, training=False, mask=None):
        if x.dim() != 4:
            raise ValueError(f"Got rank {x.dim()} array as input to ConvolutionLayer {self.layerId()}; "
                             "expected rank 4 [minibatch, channels, height, width]")
        if x.shape[1] != self.conf.nIn:
            raise ValueError(f"Cannot do forward pass in Convolution layer {self.layerId()}: input depth "
                             f"{x.shape[1]} does not match nIn {self.conf.nIn}")
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        z = self.preOutput(x, training)
        self._z = z
        return self.conf.activation.getActivation(z, training)

    def backpropGradient(self, eps):
        delta = self.conf.activation.backprop(self._z, eps.to(self._z.dtype))
        s, pad4, d = self._geom_cache
        W = self.W("W")
        xt = _cl(self._xt.to(W.dtype))
        need_dx = getattr(self, "need_input_grad", True)
        acc = getattr(self, "dx_accum", None)       # set by the graph when x already has a gradient (fan-out)
        self.dx_accum = None
        dx, dW, db = ops.conv2d_backward(xt, W, _cl(delta.to(W.dtype)), s, pad4, d, need_dx, True,
                                         "b" in self.grads, gW=self.grads["W"], gb=self.grads.get("b"),
                                         grads_zeroed=getattr(self.net, "_grads_zeroed", False),
                                         dx_accum=acc if need_dx and self.conf.idropout is None else None)
        if dW is not None:
            copy_grad_(self.grads["W"], dW)
        if "b" in self.grads and db is not None:
            copy_grad_(self.grads["b"], db)
        if not need_dx:
            return self.make_gradient(), None
        if dx.shape[2:] != self.input.shape[2:]:
            full = torch.zeros(self.input.shape, dtype=dx.dtype, device=dx.device)
            full[:, :, :dx.shape[2], :dx.shape[3]] = dx
            dx = full
        return self.make_gradient(), self.backpropDropOut(dx)


class Convolution1DLayerImpl(ConvolutionLayerImpl):
    """[mb, nIn, T] -> conv over T with a [k,1] kernel."""

    def activate(self, x, training=False, mask=None):
        self._was3d = x.dim() == 3
        x4 = x.unsqueeze(3) if x.dim() == 3 else x
        out = super().activate(x4, training, None)
        out = out.squeeze(3)
        if mask is not None:
            out = out * mask.unsqueeze(1).to(out.dtype)[:, :, :out.shape[2]]
        return out

    def backpropGradient(self, eps):
        g, dx = super().backpropGradient(eps.unsqueeze(3))
        return g, (dx.squeeze(3) if dx is not None else None)


class Deconvolution2DImpl(ConvolutionLayerImpl):
    """Transposed convolution (reference Deconvolution2DLayer.java:112-225): forward is the conv bwd-data kernel on
    the zero-interleaved input, backward is a forward conv (dx) plus a weight-gradient conv (dW) — all on the
    implicit-GEMM HIP kernels for bf16 on the GPU; explicit backward everywhere (ops/nn_misc.py)."""

    def _pad(self):
        c = self.conf
        return [0, 0] if c.convolutionMode == ConvolutionMode.Same else list(c.padding)

    def preOutput(self, x, training=False):
        from ...ops.nn_misc import deconv_forward
        c = self.conf
        W = self.W("W")
        b = self.W("b").reshape(-1) if "b" in self.params else None
        self._xt = x
        out = deconv_forward(_cl(x.to(W.dtype)), W, b, list(c.stride), self._pad(), list(c.dilation))
        self._full_hw = out.shape[2:]
        if c.convolutionMode == ConvolutionMode.Same:
            out = out[:, :, :x.shape[2] * c.stride[0], :x.shape[3] * c.stride[1]]
        return out

    def backpropGradient(self, eps):
        from ...ops.nn_misc import deconv_backward
        c = self.conf
        delta = self.conf.activation.backprop(self._z, eps.to(self._z.dtype))
        W = self.W("W")
        if tuple(delta.shape[2:]) != tuple(self._full_hw):
            full = torch.zeros(delta.shape[:2] + tuple(self._full_hw), dtype=delta.dtype, device=delta.device)
            full[:, :, :delta.shape[2], :delta.shape[3]] = delta
            delta = full
        gW = self.grads["W"] if self.grads["W"].dtype == torch.float32 and self.grads["W"].is_contiguous() else None
        dx, dW, db = deconv_backward(self._xt.to(W.dtype), W, delta.to(W.dtype), list(c.stride), self._pad(),
                                     list(c.dilation), "b" in self.grads, gW=gW,
                                     gb=self.grads["b"].reshape(-1) if "b" in self.grads else None)
        if dW is not None and dW is not gW:
            copy_grad_(self.grads["W"], _acc(dW))
        if "b" in self.grads and db is not None:
            copy_grad_(self.grads["b"], _acc(db))
        return self.make_gradient(), self.backpropDropOut(dx)


class DepthwiseConvolution2DImpl(ConvolutionLayerImpl):
    """Depthwise conv, weights [depthMultiplier, C, kh, kw]; direct HIP stencil kernels (fwd, bwd-data,
    bwd-weight) on the GPU, grouped library conv on CPU; explicit backward."""

    def preOutput(self, x, training=False):
        from ...ops.nn_misc import depthwise_forward
        c = self.conf
        W = self.W("W")
        pad4 = compute_pad4(c, x.shape[2], x.shape[3])
        self._xt = _cl(x.to(W.dtype))
        self._geom_cache = (list(c.stride), pad4, list(c.dilation))
        b = self.params["b"].reshape(-1) if "b" in self.params else None
        return depthwise_forward(self._xt, W, b, *self._geom_cache)

    def backpropGradient(self, eps):
        from ...ops.nn_misc import depthwise_backward
        delta = self.conf.activation.backprop(self._z, eps.to(self._z.dtype))
        W = self.W("W")
        dx, dW, db = depthwise_backward(self._xt, W, _cl(delta.to(W.dtype)), *self._geom_cache,
                                        need_db="b" in self.grads)
        copy_grad_(self.grads["W"], dW)
        if "b" in self.grads:
            copy_grad_(self.grads["b"], db)
        return self.make_gradient(), self.backpropDropOut(dx)


class SeparableConvolution2DImpl(DepthwiseConvolution2DImpl):
    """Depthwise conv (no bias) followed by a pointwise 1x1 conv with the bias (reference
    SeparableConvolution2DLayer.java:126-236); the pointwise part runs on the conv/GEMM kernels."""

    def preOutput(self, x, training=False):
        from ...ops.nn_misc import depthwise_forward
        c = self.conf
        W = self.W("W")
        pad4 = compute_pad4(c, x.shape[2], x.shape[3])
        self._xt = _cl(x.to(W.dtype))
        self._geom_cache = (list(c.stride), pad4, list(c.dilation))
        self._y1 = _cl(depthwise_forward(self._xt, W, None, *self._geom_cache))
        b = self.params["b"].reshape(-1) if "b" in self.params else None
        return ops.conv2d_forward(self._y1, self.W("pW"), b, (1, 1), (0, 0, 0, 0), (1, 1))

    def backpropGradient(self, eps):
        from ...ops.nn_misc import depthwise_backward
        delta = self.conf.activation.backprop(self._z, eps.to(self._z.dtype))
        W, pW = self.W("W"), self.W("pW")
        dy1, dpW, db = ops.conv2d_backward(self._y1, pW, _cl(delta.to(pW.dtype)), (1, 1), (0, 0, 0, 0), (1, 1),
                                           True, True, "b" in self.grads, gW=self.grads["pW"],
                                           gb=self.grads.get("b"))
        if dpW is not None:
            copy_grad_(self.grads["pW"], _acc(dpW))
        if "b" in self.grads and db is not None:
            copy_grad_(self.grads["b"], _acc(db))
        dx, dW, _ = depthwise_backward(self._xt, W, _cl(dy1.to(W.dtype)), *self._geom_cache, need_db=False)
        copy_grad_(self.grads["W"], dW)
        return self.make_gradient(), self.backpropDropOut(dx)


class SubsamplingLayerImpl(LayerImpl):
    def type(self):
        return "SUBSAMPLING"

    def activate(self, x, training=False, mask=None):
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        c = self.conf
        pad4 = compute_pad4(c, x.shape[2], x.shape[3], c.kernelSize, c.stride, c.dilation)
        xt = x     # floor-division output sizes already implement Truncate mode
        self._xshape = x.shape
        y, self._ctx = ops.pool2d_forward(_cl(xt), c.poolingType.value, c.kernelSize, c.stride, pad4, c.dilation,
                                          c.pnorm, c.eps)
        return y

    def backpropGradient(self, eps):
        dx = ops.pool2d_backward(_cl(eps), self._ctx)
        if dx.shape[2:] != self._xshape[2:]:
            full = torch.zeros(self._xshape, dtype=dx.dtype, device=dx.device)
            full[:, :, :dx.shape[2], :dx.shape[3]] = dx
            dx = full
        return self.make_gradient(), self.backpropDropOut(dx)


class Subsampling1DLayerImpl(SubsamplingLayerImpl):
    def activate(self, x, training=False, mask=None):
        out = super().activate(x.unsqueeze(3), training, None).squeeze(3)
        if mask is not None:
            from ..util.time_series import reverse_time_series  # noqa: F401 (keeps import graph simple)
        return out

    def backpropGradient(self, eps):
        g, dx = super().backpropGradient(eps.unsqueeze(3))
        return g, dx.squeeze(3)


class ZeroPaddingLayerImpl(LayerImpl):
    def activate(self, x, training=False, mask=None):
        t, b, l, r = self.conf.padding
        self._pad = (t, b, l, r)
        return _cl(F.pad(x, (l, r, t, b)))

    def backpropGradient(self, eps):
        t, b, l, r = self._pad
        H, W = eps.shape[2], eps.shape[3]
        return self.make_gradient(), eps[:, :, t:H - b, l:W - r]


class ZeroPadding1DLayerImpl(LayerImpl):
    def activate(self, x, training=False, mask=None):
        l, r = self.conf.padding
        self._pad = (l, r)
        return F.pad(x, (l, r))

    def backpropGradient(self, eps):
        l, r = self._pad
        return self.make_gradient(), eps[:, :, l:eps.shape[2] - r]


class Cropping2DImpl(LayerImpl):
    def activate(self, x, training=False, mask=None):
        t, b, l, r = self.conf.cropping
        self._shape = x.shape
        return x[:, :, t:x.shape[2] - b, l:x.shape[3] - r]

    def backpropGradient(self, eps):
        t, b, l, r = self.conf.cropping
        g = torch.zeros(self._shape, dtype=eps.dtype, device=eps.device)
        g[:, :, t:self._shape[2] - b, l:self._shape[3] - r] = eps
        return self.make_gradient(), g


def _nd4j():
    from ...ops import nd4j_kernels
    return nd4j_kernels


class Upsampling2DImpl(LayerImpl):
    """GPU: one broadcast-copy kernel forward, one permute-copy + row-sum reduction backward (csrc/nd4j_ops.hip)."""

    def activate(self, x, training=False, mask=None):
        s = self.conf.size
        if x.is_cuda:
            y = _nd4j().upsample_nearest2d(x, s[0], s[1])
            if y is not None:
                return y
        return x.repeat_interleave(s[0], dim=2).repeat_interleave(s[1], dim=3)

    def backpropGradient(self, eps):
        s = self.conf.size
        n, c, h, w = eps.shape
        if eps.is_cuda:
            g = _nd4j().upsample_nearest2d_bp(eps, s[0], s[1])
            if g is not None:
                return self.make_gradient(), g
        return self.make_gradient(), eps.reshape(n, c, h // s[0], s[0], w // s[1], s[1]).sum(dim=(3, 5))


class Upsampling1DImpl(LayerImpl):
    def activate(self, x, training=False, mask=None):
        return x.repeat_interleave(self.conf.size[0], dim=2)

    def backpropGradient(self, eps):
        s = self.conf.size[0]
        n, c, T = eps.shape
        return self.make_gradient(), eps.reshape(n, c, T // s, s).sum(dim=3)


class SpaceToDepthImpl(LayerImpl):
    """TensorFlow depth ordering: output channel = (dy * b + dx) * C + c (block offset major), the layout the
    reference's space_to_depth op and Keras-imported models use."""

    def activate(self, x, training=False, mask=None):
        b = self.conf.blockSize
        n, c, H, W = x.shape
        if x.is_cuda:
            y = _nd4j().space_to_depth(x, b)
            if y is not None:
                return y
        y = x.reshape(n, c, H // b, b, W // b, b).permute(0, 3, 5, 1, 2, 4)
        return y.reshape(n, b * b * c, H // b, W // b)

    def backpropGradient(self, eps):
        b = self.conf.blockSize
        if eps.is_cuda:
            g = _nd4j().depth_to_space(eps, b)
            if g is not None:
                return self.make_gradient(), g
        n, cc, h, w = eps.shape
        c = cc // (b * b)
        g = eps.reshape(n, b, b, c, h, w).permute(0, 3, 4, 1, 5, 2)
        return self.make_gradient(), g.reshape(n, c, h * b, w * b)


class SpaceToBatchImpl(LayerImpl):
    def activate(self, x, training=False, mask=None):
        (pt, pb), (pl, pr) = self.conf.padding
        bh, bw = self.conf.blocks
        if x.is_cuda:
            y = _nd4j().space_to_batch(x, (bh, bw), ((pt, pb), (pl, pr)))
            if y is not None:
                self._shape = (x.shape, (x.shape[0], x.shape[1], x.shape[2] + pt + pb, x.shape[3] + pl + pr))
                return y
        xp = F.pad(x, (pl, pr, pt, pb))
        n, c, H, W = xp.shape
        self._shape = (x.shape, xp.shape)
        y = xp.reshape(n, c, H // bh, bh, W // bw, bw).permute(3, 5, 0, 1, 2, 4)
        return y.reshape(bh * bw * n, c, H // bh, W // bw)

    def backpropGradient(self, eps):
        (pt, pb), (pl, pr) = self.conf.padding
        bh, bw = self.conf.blocks
        xs, xps = self._shape
        n, c, H, W = xps
        if eps.is_cuda:
            g = _nd4j().batch_to_space(eps, (bh, bw), ((pt, pb), (pl, pr)))
            if g is not None:
                return self.make_gradient(), g
        g = eps.reshape(bh, bw, n, c, H // bh, W // bw).permute(2, 3, 4, 0, 5, 1).reshape(n, c, H, W)
        return self.make_gradient(), g[:, :, pt:pt + xs[2], pl:pl + xs[3]]
