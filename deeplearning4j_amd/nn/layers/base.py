"""Runtime layer base (reference nn/api/Layer.java:54-288, nn/layers/AbstractLayer.java, BaseLayer.java).

A runtime layer owns *views* into the network's flat parameter vector (master precision), the flat
gradient vector, and — for reduced-precision compute — the flat bf16/fp16 shadow of the parameters.
``activate`` runs the forward pass and caches what backprop needs; ``backpropGradient(eps)`` writes
dL/dparam into the gradient views (sums over the minibatch, not means) and returns dL/dinput.
"""
import torch

from ..gradient import Gradient
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


class ParamTable(dict):
    """Parameter (or gradient) views by key. Calling it returns the layer's flat segment of the network's parameter
    vector, as the reference's ``Layer.params()`` (a view when the network laid the layer out, else a copy)."""
    flat = None

    def __call__(self):
        if self.flat is not None:
            return self.flat
        if not self:
            return torch.zeros(0)
        return torch.cat([v.reshape(-1) for v in self.values()])


class LayerImpl:
    def __init__(self, conf, index=0, net=None):
        self.conf = conf
        self.index = index
        self.net = net
        self.params = ParamTable()   # key -> master view (fp32/fp64); params() -> flat segment
        self.cparams = {}     # key -> compute-dtype view (shadow) ; == params when no shadow
        self.grads = {}       # key -> gradient view
        self.input = None
        self.maskArray = None
        self.maskState = None
        self.training = False
        self.iteration = 0
        self.epoch = 0
        self.listeners = []
        self.helperCountFail = 0
        self.dropoutApplied = False

    # -------------------------------------------------------------------------- listeners
    def getListeners(self):
        """The layer's training listeners: its own, else those of the network that owns it (the reference sets the
        network's listeners on every layer, whether they are set before or after init)."""
        if self.listeners:
            return self.listeners
        return list(getattr(self.net, "listeners", None) or [])

    def setListeners(self, *ls):
        self.listeners = [x for l in ls for x in (l if isinstance(l, (list, tuple)) else [l])]

    # -------------------------------------------------------------------------- params
    def numParams(self):
        return self.conf.numParams()

    def paramTable(self):
        return dict(self.params)

    def getParam(self, key):
        return self.params[key]

    def setParam(self, key, val):
        with torch.no_grad():
            self.params[key].copy_(val.reshape(self.params[key].shape))
            if self.cparams.get(key) is not None and self.cparams[key] is not self.params[key]:
                self.cparams[key].copy_(self.params[key])

    def setParamTable(self, table):
        for k, v in table.items():
            self.setParam(k, v)

    def setParams(self, flat):
        """Overwrite all of this layer's parameters from one flat vector (reference Layer.setParams)."""
        flat = flat.reshape(-1)
        if flat.numel() != self.numParams():
            raise ValueError(f"{self.numParams()} parameters expected, got {flat.numel()}")
        with torch.no_grad():
            if self.params.flat is not None:
                self.params.flat.copy_(flat.to(self.params.flat.dtype))
            else:
                o = 0
                for k, v in self.params.items():
                    v.copy_(flat[o:o + v.numel()].reshape(v.shape).to(v.dtype))
                    o += v.numel()
        if self.net is not None:
            self.net._params_changed()
        else:
            for k in self.params:
                if self.cparams.get(k) is not None and self.cparams[k] is not self.params[k]:
                    self.cparams[k].copy_(self.params[k])

    def update(self, gradient, paramType=None):
        """Add a gradient (an already-computed update) to the parameters, reference BaseLayer.update(Gradient) /
        update(INDArray, String) (nn/layers/BaseLayer.java:167-176: ``param.addi(gradient)``)."""
        if paramType is None:
            for k, g in gradient.gradientForVariable().items():
                self.update(g, k)
            return
        with torch.no_grad():
            p = self.params[paramType]
            self.setParam(paramType, p + gradient.reshape(p.shape).to(p.dtype))

    def W(self, key="W"):
        """Compute-dtype view of parameter ``key`` (with weight noise / DropConnect applied when training)."""
        p = self.cparams.get(key, self.params.get(key))
        wn = getattr(self.conf, "weightNoise", None)
        if wn is not None and self.training:
            p = wn.getParameter(self, key, p, self.iteration, self.epoch, True)
        return p

    def Wbias(self, key="b"):
        """Bias for a GEMM epilogue: the fp32 master parameter itself when nothing perturbs it (the epilogue adds
        fp32 bias, so a 16-bit shadow would only cost a conversion launch per call and precision), else W(key)."""
        p = self.params.get(key)
        if p is not None and p.dtype == torch.float32 and getattr(self.conf, "weightNoise", None) is None:
            return p
        return self.W(key)

    def type(self):
        return "FEED_FORWARD"

    def layerId(self):
        return f"(layer name: {self.conf.layerName}, index: {self.index}, type: {type(self).__name__})"

    @property
    def compute_dtype(self):
        return self.net.compute_dtype if self.net is not None else torch.float32

    # -------------------------------------------------------------------------- forward/backward
    def applyDropOutIfNecessary(self, x, training):
        d = getattr(self.conf, "idropout", None)
        if training and d is not None:
            self.dropoutApplied = True
            return d.applyDropout(x, self.iteration, self.epoch, False)
        self.dropoutApplied = False
        return x

    def backpropDropOut(self, eps):
        d = getattr(self.conf, "idropout", None)
        if self.dropoutApplied and d is not None:
            return d.backprop(eps)
        return eps

    def activate(self, x, training=False, mask=None):
        raise NotImplementedError

    def backpropGradient(self, epsilon):
        raise NotImplementedError

    def preOutput(self, x, training=False):
        raise NotImplementedError(f"preOutput not supported by {type(self).__name__}")

    def make_gradient(self):
        g = Gradient()
        for k, v in self.grads.items():
            g.setGradientFor(k, v)
        return g

    def clear(self):
        self.input = None
        self.maskArray = None

    def setInput(self, x):
        self.input = x

    def getInput(self):
        return self.input

    # -------------------------------------------------------------------------- masks
    def setMaskArray(self, m):
        self.maskArray = m

    def feedForwardMaskArray(self, mask, state, mb):
        self.maskArray = mask
        self.maskState = state
        return mask, state

    # -------------------------------------------------------------------------- misc
    def isPretrainLayer(self):
        return False

    def calcL1(self, backprop_params_only=True):
        s = 0.0
        for k, p in self.params.items():
            l1 = self.conf.l1For(k)
            if l1 > 0:
                s += l1 * p.abs().sum().item()
        return s

    def calcL2(self, backprop_params_only=True):
        s = 0.0
        for k, p in self.params.items():
            l2 = self.conf.l2For(k)
            if l2 > 0:
                s += 0.5 * l2 * (_acc(p) * _acc(p)).sum().item()
        return s

    def applyConstraints(self, iteration, epoch):
        cs = getattr(self.conf, "constraints", None)
        if not cs:
            return
        with torch.no_grad():
            for c in cs:
                for k, p in self.params.items():
                    if c.params == ["*"] or (c.params and k in c.params) or \
                            (not c.params and not self.conf.is_bias(k)):
                        if p.numel() == 0:
                            continue
                        c.apply_(k, p)
                        if self.cparams.get(k) is not None and self.cparams[k] is not p:
                            self.cparams[k].copy_(p)


def matmul(a, b, bias=None, out_dtype=None, act=None, z=None):
    """``a @ b (+ bias)`` on the in-tree MFMA GEMM (ops/gemm.py); torch reference on CPU."""
    from ...ops.gemm import bias_vec, mmul
    return mmul(a, b, bias=bias_vec(bias), out_dtype=out_dtype, act=act, z=z)


def weight_grad_(view, a, b):
    """Gradient view <- a @ b, accumulated in fp32 by the GEMM and written straight into the (possibly 'f'-ordered)
    flat-gradient view — no bf16 rounding of the product before the master-precision gradient."""
    from ...ops.gemm import mmul
    if view.dim() == 2 and tuple(view.shape) == (a.shape[-2], b.shape[-1]) and view.device == a.device:
        mmul(a, b, out=view)
    else:
        copy_grad_(view, mmul(a, b, out_dtype=torch.float64 if view.dtype == torch.float64 else torch.float32))


def bias_grad_(view, delta):
    """Bias gradient = column sums of delta [M, N] (fp32), on the channel-sum HIP kernel when on the GPU."""
    K8 = getattr(delta, "_dl4j_kz", 0)
    if K8 and delta.is_cuda and delta.dim() == 2 and delta.stride() == (K8, 1) and view.dtype == torch.float32:
        # zero-padded operand view (ops/gemm.py kz_view): column sums over the whole padded buffer, padding dropped
        from ...ops import native
        full = delta.as_strided((delta.shape[0], K8), (K8, 1))
        tmp = native.channel_sum(full)
        if tmp is not None:
            view.copy_(tmp[:delta.shape[1]].reshape(view.shape))
            return
    if delta.is_cuda and delta.dim() == 2 and delta.dtype in (torch.float32, torch.bfloat16, torch.float16) \
            and delta.is_contiguous() \
            and view.dtype == torch.float32 and view.is_contiguous():
        from ...ops import native
        if native.channel_sum(delta, out=view.reshape(-1)) is not None:
            return
    copy_grad_(view, _acc(delta).sum(dim=0))


def add_row(z, b):
    return z + b.reshape(1, -1).to(z.dtype)


def copy_grad_(view, value):
    """Write a gradient into a (possibly 'f'-ordered) gradient view."""
    view.copy_(value.reshape(view.shape))
