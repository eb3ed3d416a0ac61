"""ComputationGraph vertex configurations with their (stateless) forward/backward.

Reference: nn/conf/graph/*.java (configs) and nn/graph/vertex/impl/**.java (runtime), e.g.
ElementWiseVertex.java:44-45 (ops Add/Subtract/Product/Average/Max; Max uses mergemax +
mergemaxindex for backprop, ElementWiseVertex.java:105,155), MergeVertex.java:118-156 (concat on
dim 1), L2Vertex.java:78, L2NormalizeVertex.java:81-88, rnn/{LastTimeStep,DuplicateToTimeSeries,
ReverseTimeSeries}Vertex.java.

``forward(inputs, training, masks) -> (out, ctx)`` and ``backward(eps, ctx) -> [eps_i]``.
"""
import torch

from .base import Config, int_list
from .inputs import InputType, InputTypeConvolutional, InputTypeFeedForward, InputTypeRecurrent
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


class GraphVertex(Config):
    def numParams(self, backprop=True):
        """Parameter count (the reference's numParams(boolean backprop); the flag does not change it here)."""
        return 0

    def getOutputType(self, layerIndex, *inputTypes):
        return inputTypes[0]

    def forward(self, inputs, training=False, masks=None):
        raise NotImplementedError

    def backward(self, eps, ctx):
        raise NotImplementedError

    def feedForwardMask(self, masks):
        for m in masks or []:
            if m is not None:
                return m
        return None


class ElementWiseVertex(GraphVertex):
    FIELDS = {"op": "Add"}

    class Op:
        Add = "Add"
        Subtract = "Subtract"
        Product = "Product"
        Average = "Average"
        Max = "Max"

    def __init__(self, op="Add", **kw):
        super().__init__(op=str(op), **kw)

    def forward(self, inputs, training=False, masks=None):
        op = self.op
        if op == "Add":
            out = inputs[0]
            for x in inputs[1:]:
                out = out + x
            return out, len(inputs)
        if op == "Subtract":
            if len(inputs) != 2:
                raise ValueError("ElementWiseVertex(Subtract) requires exactly 2 inputs")
            return inputs[0] - inputs[1], 2
        if op == "Product":
            out = inputs[0]
            for x in inputs[1:]:
                out = out * x
            return out, list(inputs)
        if op == "Average":
            out = inputs[0]
            for x in inputs[1:]:
                out = out + x
            return out / len(inputs), len(inputs)
        if op == "Max":
            if inputs[0].is_cuda:
                from deeplearning4j_amd.ops import nd4j_kernels as K
                r = K.mergemax(list(inputs))                        # mergemax kernel (csrc/nd4j_ops.hip)
                if r is not None:
                    return r[0], ("mergemax", r[1], len(inputs))
            st = torch.stack(list(inputs), 0)
            out, idx = st.max(dim=0)
            return out, (idx, len(inputs))
        raise ValueError(op)

    def backward(self, eps, ctx):
        op = self.op
        if op == "Add":
            return [eps] * ctx
        if op == "Subtract":
            return [eps, -eps]
        if op == "Product":
            xs = ctx
            outs = []
            for i in range(len(xs)):
                g = eps
                for j, x in enumerate(xs):
                    if j != i:
                        g = g * x
                outs.append(g)
            return outs
        if op == "Average":
            return [eps / ctx] * ctx
        if op == "Max":
            if isinstance(ctx[0], str):
                from deeplearning4j_amd.ops import nd4j_kernels as K
                _, am, n = ctx
                r = K.mergemax_bp(eps.to(am.device), am, n) if eps.is_cuda else None
                if r is not None:
                    return r
                return [eps * (am == i).to(eps.dtype) for i in range(n)]
            idx, n = ctx
            return [eps * (idx == i).to(eps.dtype) for i in range(n)]
        raise ValueError(op)


class MergeVertex(GraphVertex):
    """Concatenate along dimension 1 (features / channels)."""

    def getOutputType(self, layerIndex, *inputTypes):
        t0 = inputTypes[0]
        if isinstance(t0, InputTypeConvolutional):
            return InputType.convolutional(t0.height, t0.width, sum(t.channels for t in inputTypes))
        if isinstance(t0, InputTypeRecurrent):
            return InputType.recurrent(sum(t.size for t in inputTypes), t0.timeSeriesLength)
        return InputType.feedForward(sum(t.arrayElementsPerExample() for t in inputTypes))

    def forward(self, inputs, training=False, masks=None):
        if len(inputs) == 1:
            return inputs[0], [inputs[0].shape[1]]
        return torch.cat(list(inputs), dim=1), [x.shape[1] for x in inputs]

    def backward(self, eps, ctx):
        return list(torch.split(eps, ctx, dim=1))


class SubsetVertex(GraphVertex):
    """Features [from, to] inclusive along dim 1."""
    FIELDS = {"from_": 0, "to": 0}
    _ALIASES = {"from": "from_"}

    def __init__(self, from_=0, to=0, **kw):
        super().__init__(from_=from_, to=to, **kw)

    def getOutputType(self, layerIndex, *inputTypes):
        n = self.to - self.from_ + 1
        t = inputTypes[0]
        if isinstance(t, InputTypeConvolutional):
            return InputType.convolutional(t.height, t.width, n)
        if isinstance(t, InputTypeRecurrent):
            return InputType.recurrent(n, t.timeSeriesLength)
        return InputType.feedForward(n)

    def forward(self, inputs, training=False, masks=None):
        x = inputs[0]
        return x[:, self.from_:self.to + 1], x.shape

    def backward(self, eps, ctx):
        g = torch.zeros(ctx, dtype=eps.dtype, device=eps.device)
        g[:, self.from_:self.to + 1] = eps
        return [g]


class StackVertex(GraphVertex):
    """Stack along dim 0 (minibatch)."""

    def forward(self, inputs, training=False, masks=None):
        """Time series of different lengths are zero-padded to the longest (reference StackVertex.doForward); the
        stacked mask marks the padding."""
        inputs = list(inputs)
        self._mask_shapes = [(x.shape[0], x.shape[2] if x.dim() == 3 else None) for x in inputs]
        if inputs[0].dim() == 3:
            T = max(x.shape[2] for x in inputs)
            if any(x.shape[2] != T for x in inputs):
                self._Tmax = T
                padded = [torch.nn.functional.pad(x, (0, T - x.shape[2])) for x in inputs]
                return torch.cat(padded, dim=0), ([x.shape[0] for x in inputs], [x.shape[2] for x in inputs])
        self._Tmax = None
        return torch.cat(inputs, dim=0), [x.shape[0] for x in inputs]

    def backward(self, eps, ctx):
        if isinstance(ctx, tuple):
            ns, Ts = ctx
            return [e[:, :, :T] for e, T in zip(torch.split(eps, ns, dim=0), Ts)]
        return list(torch.split(eps, ctx, dim=0))

    def feedForwardMask(self, masks):
        """Masks are stacked like the activations (reference StackVertex.feedForwardMaskArrays): an input without a
        mask contributes ones; no mask at all stays None."""
        masks = list(masks or [])
        if not any(m is not None for m in masks):
            return None
        ref = next(m for m in masks if m is not None)
        shapes = getattr(self, "_mask_shapes", None) or [(ref.shape[0], ref.shape[1])] * len(masks)
        out = [m if m is not None else torch.ones(n, T if T is not None else ref.shape[1], dtype=ref.dtype,
                                                  device=ref.device) for m, (n, T) in zip(masks, shapes)]
        Tmax = max(m.shape[1] for m in out)
        out = [torch.nn.functional.pad(m, (0, Tmax - m.shape[1])) if m.shape[1] != Tmax else m for m in out]
        return torch.cat(out, dim=0)


class UnstackVertex(GraphVertex):
    FIELDS = {"from_": 0, "stackSize": 1}

    def __init__(self, from_=0, stackSize=1, **kw):
        super().__init__(from_=from_, stackSize=stackSize, **kw)

    def forward(self, inputs, training=False, masks=None):
        x = inputs[0]
        n = x.shape[0] // self.stackSize
        return x[self.from_ * n:(self.from_ + 1) * n], (x.shape, n)

    def feedForwardMask(self, masks):
        m = (masks or [None])[0]
        if m is None:
            return None
        n = m.shape[0] // self.stackSize
        return m[self.from_ * n:(self.from_ + 1) * n]

    def backward(self, eps, ctx):
        shape, n = ctx
        g = torch.zeros(shape, dtype=eps.dtype, device=eps.device)
        g[self.from_ * n:(self.from_ + 1) * n] = eps
        return [g]


class ReshapeVertex(GraphVertex):
    FIELDS = {"newShape": None, "order": "c"}

    def __init__(self, *shape, **kw):
        if shape:
            kw["newShape"] = list(shape[0]) if len(shape) == 1 and isinstance(shape[0], (list, tuple)) else list(shape)
        super().__init__(**kw)

    def getOutputType(self, layerIndex, *inputTypes):
        s = self.newShape
        if len(s) == 2:
            return InputType.feedForward(s[1])
        if len(s) == 3:
            return InputType.recurrent(s[1], s[2])
        return InputType.convolutional(s[2], s[3], s[1])

    def forward(self, inputs, training=False, masks=None):
        x = inputs[0]
        shape = list(self.newShape)
        if shape[0] in (-1, 0) or shape[0] != x.shape[0]:
            shape[0] = x.shape[0]
        return x.reshape(shape), x.shape

    def backward(self, eps, ctx):
        return [eps.reshape(ctx)]


class ScaleVertex(GraphVertex):
    FIELDS = {"scaleFactor": 1.0}

    def __init__(self, scaleFactor=1.0, **kw):
        super().__init__(scaleFactor=scaleFactor, **kw)

    def forward(self, inputs, training=False, masks=None):
        return inputs[0] * self.scaleFactor, None

    def backward(self, eps, ctx):
        return [eps * self.scaleFactor]


class ShiftVertex(GraphVertex):
    FIELDS = {"shiftFactor": 0.0}

    def __init__(self, shiftFactor=0.0, **kw):
        super().__init__(shiftFactor=shiftFactor, **kw)

    def forward(self, inputs, training=False, masks=None):
        return inputs[0] + self.shiftFactor, None

    def backward(self, eps, ctx):
        return [eps]


class L2Vertex(GraphVertex):
    """Euclidean distance between two inputs per example -> [mb, 1]."""
    FIELDS = {"eps": 1e-8}

    def getOutputType(self, layerIndex, *inputTypes):
        return InputType.feedForward(1)

    def forward(self, inputs, training=False, masks=None):
        a, b = inputs
        d = (a - b).reshape(a.shape[0], -1)
        n = torch.sqrt((d * d).sum(dim=1, keepdim=True))
        return n, (d, n, a.shape)

    def backward(self, eps, ctx):
        d, n, shape = ctx
        g = d / torch.clamp(n, min=self.eps) * eps.reshape(-1, 1)
        g = g.reshape(shape)
        return [g, -g]


class L2NormalizeVertex(GraphVertex):
    FIELDS = {"dimension": None, "eps": 1e-8}

    def forward(self, inputs, training=False, masks=None):
        x = inputs[0]
        dims = self.dimension or list(range(1, x.dim()))
        n = torch.sqrt((x * x).sum(dim=dims, keepdim=True))
        n = torch.clamp(n, min=self.eps)
        return x / n, (x, n, dims)

    def backward(self, eps, ctx):
        x, n, dims = ctx
        y = x / n
        return [(eps - y * (eps * y).sum(dim=dims, keepdim=True)) / n]


class PoolHelperVertex(GraphVertex):
    """Strips the first row and column of a CNN activation (Keras GoogLeNet import helper)."""

    def getOutputType(self, layerIndex, *inputTypes):
        t = inputTypes[0]
        return InputType.convolutional(t.height - 1, t.width - 1, t.channels)

    def forward(self, inputs, training=False, masks=None):
        x = inputs[0]
        return x[:, :, 1:, 1:], x.shape

    def backward(self, eps, ctx):
        g = torch.zeros(ctx, dtype=eps.dtype, device=eps.device)
        g[:, :, 1:, 1:] = eps
        return [g]


class PreprocessorVertex(GraphVertex):
    FIELDS = {"preProcessor": None}

    def __init__(self, preProcessor=None, **kw):
        super().__init__(preProcessor=preProcessor, **kw)

    def getOutputType(self, layerIndex, *inputTypes):
        return self.preProcessor.getOutputType(inputTypes[0])

    def forward(self, inputs, training=False, masks=None):
        x = inputs[0]
        return self.preProcessor.preProcess(x, x.shape[0], training), x.shape[0]

    def backward(self, eps, ctx):
        return [self.preProcessor.backprop(eps, ctx)]


class LastTimeStepVertex(GraphVertex):
    FIELDS = {"maskArrayInputName": None}

    def __init__(self, maskArrayInputName=None, **kw):
        super().__init__(maskArrayInputName=maskArrayInputName, **kw)

    def getOutputType(self, layerIndex, *inputTypes):
        return InputType.feedForward(inputTypes[0].size)

    def forward(self, inputs, training=False, masks=None):
        x = inputs[0]
        mask = masks[0] if masks else None
        if mask is None:
            return x[:, :, -1], (x.shape, None)
        idx = (mask.shape[1] - 1 - torch.argmax(_acc(torch.flip(mask, [1])), dim=1)).long()
        out = x[torch.arange(x.shape[0], device=x.device), :, idx]
        return out, (x.shape, idx)

    def backward(self, eps, ctx):
        shape, idx = ctx
        g = torch.zeros(shape, dtype=eps.dtype, device=eps.device)
        if idx is None:
            g[:, :, -1] = eps
        else:
            g[torch.arange(shape[0], device=eps.device), :, idx] = eps
        return [g]

    def feedForwardMask(self, masks):
        return None


class DuplicateToTimeSeriesVertex(GraphVertex):
    """[mb, n] -> [mb, n, T] where T is taken from the named input's time dimension."""
    FIELDS = {"inputName": None}

    def __init__(self, inputName=None, **kw):
        super().__init__(inputName=inputName, **kw)

    def getOutputType(self, layerIndex, *inputTypes):
        return InputType.recurrent(inputTypes[0].arrayElementsPerExample())

    def forward(self, inputs, training=False, masks=None, T=None):
        x = inputs[0]
        T = T if T is not None else self._T
        return x.unsqueeze(2).expand(x.shape[0], x.shape[1], T).contiguous(), None

    def backward(self, eps, ctx):
        return [eps.sum(dim=2)]


class ReverseTimeSeriesVertex(GraphVertex):
    FIELDS = {"maskArrayInputName": None}

    def __init__(self, maskArrayInputName=None, **kw):
        super().__init__(maskArrayInputName=maskArrayInputName, **kw)

    def forward(self, inputs, training=False, masks=None):
        from ..util.time_series import reverse_time_series
        mask = masks[0] if masks else None
        return reverse_time_series(inputs[0], mask), mask

    def backward(self, eps, ctx):
        from ..util.time_series import reverse_time_series
        return [reverse_time_series(eps, ctx)]


class LayerVertex(GraphVertex):
    """Graph node holding a layer config (+ optional preprocessor)."""
    FIELDS = {"layerConf": None, "preProcessor": None}

    def numParams(self, backprop=True):
        return self.layerConf.numParams()

    def getLayerConf(self):
        """The reference's per-layer NeuralNetConfiguration view: ``getLayerConf().getLayer()`` is the layer
        configuration (a FrozenLayer wrapper stays a FrozenLayer)."""
        from .network import LayerConfiguration
        return LayerConfiguration(self.layerConf)

    def getOutputType(self, layerIndex, *inputTypes):
        t = inputTypes[0]
        if self.preProcessor is not None:
            t = self.preProcessor.getOutputType(t)
        return self.layerConf.getOutputType(layerIndex, t)


_ = (InputTypeFeedForward, int_list)
