"""Layer configurations (reference nn/conf/layers/*, 45+ classes).

Each config:
  * holds hyper-parameters (DL4J field names; inherited from the global NeuralNetConfiguration
    builder when left unset — reference NeuralNetConfiguration.Builder / configureLayer),
  * infers output shapes (``getOutputType``) and nIn (``setNIn``) from an InputType,
  * declares its **flat parameter layout** (``param_specs``) — the order and memory order of each
    parameter inside the layer's slice of the network-wide flat [1, P] vector. These layouts are the
    reference's ParamInitializers (reference nn/params/*: Dense W 'f'[nIn,nOut] then b
    DefaultParamInitializer.java:114-146; conv b then W c[out,in,kh,kw]
    ConvolutionParamInitializer.java:118-122; LSTM W,RW,b LSTMParamInitializer.java:126-167;
    BN gamma,beta,mean,var BatchNormalizationParamInitializer.java:88-102),
  * instantiates its runtime layer (``deeplearning4j_amd.nn.layers``).
"""
import importlib
import math

from .activations import to_activation
from .base import Config, int_list, int_pair
from .enums import AlgoMode, ConvolutionMode, GradientNormalization, PoolingType
from .inputs import (InputType, InputTypeConvolutional, InputTypeConvolutionalFlat, InputTypeFeedForward,
                     InputTypeRecurrent)
from .losses import to_loss
from .regularization import to_dropout
from .updaters import to_updater
from .validation import validate_kernel_geometry
from ...exceptions import DL4JInvalidConfigException, InvalidInputTypeException
from .weights import to_weight_init


class ParamSpec:
    """One parameter inside a layer's flat slice."""
    __slots__ = ("key", "shape", "order", "kind", "fan_in", "fan_out", "value", "trainable")

    def __init__(self, key, shape, order="c", kind="weight", fan_in=1.0, fan_out=1.0, value=0.0,
                 trainable=True):
        self.key, self.shape, self.order, self.kind = key, list(shape), order, kind
        self.fan_in, self.fan_out, self.value, self.trainable = fan_in, fan_out, value, trainable

    @property
    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n


# Global-inheritable properties (reference BaseLayer fields, nn/conf/layers/BaseLayer.java:42-54)
INHERITABLE = ("activation", "weightInit", "biasInit", "dist", "l1", "l2", "l1Bias", "l2Bias", "updater",
               "biasUpdater", "weightNoise", "gradientNormalization", "gradientNormalizationThreshold",
               "idropout", "convolutionMode", "cudnnAlgoMode", "constraints")


class Layer(Config):
    FIELDS = {"layerName": None, "idropout": None, "constraints": None}
    _ALIASES = {"name": "layerName", "dropOut": "idropout", "dropout": "idropout"}
    _CONVERTERS = {"idropout": to_dropout}

    def getIDropout(self):
        return self.idropout
    RUNTIME = None      # "module:Class" of the runtime implementation

    # ---- builder hooks ---------------------------------------------------------------------
    @staticmethod
    def _builder_hook_constrainWeights(kw, v):
        kw.setdefault("constraints", [])
        for c in (v if isinstance(v, list) else [v]):
            c = c.clone()
            c.params = ["W"]
            kw["constraints"].append(c)

    @staticmethod
    def _builder_hook_constrainBias(kw, v):
        kw.setdefault("constraints", [])
        for c in (v if isinstance(v, list) else [v]):
            c = c.clone()
            c.params = ["b"]
            kw["constraints"].append(c)

    @staticmethod
    def _builder_hook_constrainRecurrent(kw, v):
        # recurrent weights of LSTM / GravesLSTM / SimpleRnn (reference BaseRecurrentLayer.Builder.constrainRecurrent)
        kw.setdefault("constraints", [])
        for c in (v if isinstance(v, list) else [v]):
            c = c.clone()
            c.params = ["RW"]
            kw["constraints"].append(c)

    @staticmethod
    def _builder_hook_constrainAllParameters(kw, v):
        kw.setdefault("constraints", [])
        for c in (v if isinstance(v, list) else [v]):
            c = c.clone()
            c.params = ["*"]
            kw["constraints"].append(c)

    # ---- shape inference -----------------------------------------------------------------------
    def getOutputType(self, layerIndex, inputType):
        return inputType

    def setNIn(self, inputType, override=False):
        pass

    def getPreProcessorForInputType(self, inputType):
        return None

    # ---- params ----------------------------------------------------------------------------------
    def param_specs(self):
        return []

    def numParams(self):
        return sum(p.numel for p in self.param_specs())

    def paramKeys(self):
        return [p.key for p in self.param_specs()]

    def isPretrainParam(self, key):
        return False

    def is_bias(self, key):
        return key in ("b", "beta", "vb", "bias")

    def updaterFor(self, key):
        if self.is_bias(key) and getattr(self, "biasUpdater", None) is not None:
            return self.biasUpdater
        return getattr(self, "updater", None)

    def getL1ByParam(self, key):
        return self.l1For(key)

    def getL2ByParam(self, key):
        return self.l2For(key)

    def getUpdaterByParam(self, key):
        """The updater of parameter ``key``: the bias updater for bias parameters when one is set (reference
        BaseLayer.getUpdaterByParam)."""
        return self.updaterFor(key)

    def l1For(self, key):
        if self.is_bias(key):
            return getattr(self, "l1Bias", 0.0) or 0.0
        return getattr(self, "l1", 0.0) or 0.0

    def l2For(self, key):
        if self.is_bias(key):
            return getattr(self, "l2Bias", 0.0) or 0.0
        return getattr(self, "l2", 0.0) or 0.0

    def applyGlobal(self, g):
        """Fill unset inheritable fields from the global builder dict ``g``."""
        fields = self._all_fields()
        for k in INHERITABLE:
            if k in fields and getattr(self, k) is None and g.get(k) is not None:
                v = g[k]
                conv = self._CONVERTERS.get(k)
                import copy as _c
                setattr(self, k, conv(_c.deepcopy(v)) if conv else _c.deepcopy(v))

    def instantiate(self, **kw):
        rt = self.RUNTIME
        if not isinstance(rt, str):               # a user layer may name its runtime class directly
            return rt(self, **kw)
        mod, cls = rt.split(":")
        return getattr(importlib.import_module(mod), cls)(self, **kw)

    def getLayerName(self):
        return self.layerName

    def __call__(self):
        """``layer.conf()`` as in the reference (a runtime layer's conf() is its per-layer NeuralNetConfiguration,
        whose getLayer() is this config): runtime layers keep the config itself in ``.conf``."""
        from .network import LayerConfiguration
        return LayerConfiguration(self)

    def getActivationFn(self):
        """The layer's activation function object (inherited from the global config when not set on the layer)."""
        return getattr(self, "activation", None)


class NoParamLayer(Layer):
    pass


class BaseLayer(Layer):
    FIELDS = {"activation": None, "weightInit": None, "biasInit": None, "dist": None, "l1": None, "l2": None,
              "l1Bias": None, "l2Bias": None, "updater": None, "biasUpdater": None, "weightNoise": None,
              "gradientNormalization": None, "gradientNormalizationThreshold": None}
    _ALIASES = dict(Layer._ALIASES, activationFn="activation", iUpdater="updater")
    _CONVERTERS = dict(Layer._CONVERTERS, activation=to_activation, weightInit=to_weight_init,
                       updater=to_updater, biasUpdater=to_updater,
                       gradientNormalization=GradientNormalization.of)

    def _post_init(self):
        pass

    def finalize_defaults(self):
        """Apply the reference's hard defaults for anything still unset after inheritance."""
        from .activations import ActivationSigmoid
        from .updaters import Sgd
        from .weights import WeightInit
        if self.activation is None:
            self.activation = ActivationSigmoid()
        if self.weightInit is None:
            self.weightInit = WeightInit.XAVIER
        if self.weightInit == WeightInit.DISTRIBUTION and self.dist is None:
            from .weights import NormalDistribution
            self.dist = NormalDistribution(0, 1)      # the reference builder's default distribution
        if self.biasInit is None:
            self.biasInit = 0.0
        for k in ("l1", "l2", "l1Bias", "l2Bias"):
            if getattr(self, k) is None:
                setattr(self, k, 0.0)
        if self.updater is None:
            self.updater = Sgd(1e-3)
        if self.gradientNormalization is None:
            self.gradientNormalization = GradientNormalization.None_
        if self.gradientNormalizationThreshold is None:
            self.gradientNormalizationThreshold = 1.0


class FeedForwardLayer(BaseLayer):
    FIELDS = {"nIn": 0, "nOut": 0}

    @classmethod
    def _builder_positional(cls, kw, *args):
        raise TypeError(f"{cls.__name__}.Builder takes no positional arguments")

    def getOutputType(self, layerIndex, inputType):
        return InputType.feedForward(self.nOut)

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        if isinstance(inputType, InputTypeFeedForward):
            self.nIn = inputType.size
        elif isinstance(inputType, InputTypeRecurrent):
            self.nIn = inputType.size
        elif isinstance(inputType, InputTypeConvolutional):
            self.nIn = inputType.channels * inputType.height * inputType.width
        elif isinstance(inputType, InputTypeConvolutionalFlat):
            self.nIn = inputType.getFlattenedSize()

    def getPreProcessorForInputType(self, inputType):
        from .preprocessors import CnnToFeedForwardPreProcessor, FeedForwardToCnnPreProcessor, \
            RnnToFeedForwardPreProcessor
        if isinstance(inputType, InputTypeConvolutional):
            return CnnToFeedForwardPreProcessor(inputHeight=inputType.height, inputWidth=inputType.width,
                                                numChannels=inputType.channels)
        if isinstance(inputType, InputTypeRecurrent):
            return RnnToFeedForwardPreProcessor()
        return None


class DenseLayer(FeedForwardLayer):
    FIELDS = {"hasBias": True}
    RUNTIME = "deeplearning4j_amd.nn.layers.feedforward:DenseLayerImpl"

    def param_specs(self):
        specs = [ParamSpec("W", [self.nIn, self.nOut], "f", "weight", self.nIn, self.nOut)]
        if self.hasBias:
            specs.append(ParamSpec("b", [1, self.nOut], "c", "bias"))
        return specs


class ElementWiseMultiplicationLayer(FeedForwardLayer):
    RUNTIME = "deeplearning4j_amd.nn.layers.feedforward:ElementWiseMultiplicationLayerImpl"

    def param_specs(self):
        return [ParamSpec("W", [1, self.nOut], "c", "weight", self.nIn, self.nOut),
                ParamSpec("b", [1, self.nOut], "c", "bias")]


class EmbeddingLayer(FeedForwardLayer):
    """Index -> row lookup; input is [mb,1] of integer indices (reference EmbeddingLayer.java:71,111)."""
    FIELDS = {"hasBias": True}
    RUNTIME = "deeplearning4j_amd.nn.layers.feedforward:EmbeddingLayerImpl"

    def param_specs(self):
        # 'f' like every DefaultParamInitializer weight (DefaultParamInitializer.java:139 reshape('f', nIn, nOut)):
        # the coefficients.bin segment then matches a reference checkpoint element for element
        specs = [ParamSpec("W", [self.nIn, self.nOut], "f", "weight", self.nIn, self.nOut)]
        if self.hasBias:
            specs.append(ParamSpec("b", [1, self.nOut], "c", "bias"))
        return specs


class EmbeddingSequenceLayer(EmbeddingLayer):
    """[mb, T] indices -> [mb, nOut, T] (RNN format)."""
    FIELDS = {"inputLength": 1}
    RUNTIME = "deeplearning4j_amd.nn.layers.feedforward:EmbeddingSequenceLayerImpl"

    def getOutputType(self, layerIndex, inputType):
        return InputType.recurrent(self.nOut, self.inputLength)

    def getPreProcessorForInputType(self, inputType):
        return None


class BaseOutputLayer(FeedForwardLayer):
    FIELDS = {"lossFn": None, "hasBias": True}
    _ALIASES = dict(FeedForwardLayer._ALIASES, lossFunction="lossFn")
    _CONVERTERS = dict(FeedForwardLayer._CONVERTERS, lossFn=to_loss)

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["lossFn"] = to_loss(args[0])

    def param_specs(self):
        specs = [ParamSpec("W", [self.nIn, self.nOut], "f", "weight", self.nIn, self.nOut)]
        if self.hasBias:
            specs.append(ParamSpec("b", [1, self.nOut], "c", "bias"))
        return specs

    def finalize_defaults(self):
        super().finalize_defaults()
        if self.lossFn is None:
            from .losses import LossMCXENT
            self.lossFn = LossMCXENT()


class OutputLayer(BaseOutputLayer):
    RUNTIME = "deeplearning4j_amd.nn.layers.output:OutputLayerImpl"


class CenterLossOutputLayer(BaseOutputLayer):
    """Softmax output + center loss (Wen et al. 2016), reference nn/conf/layers/CenterLossOutputLayer.java."""
    FIELDS = {"alpha": 0.05, "lambda_": 2e-4, "gradientCheck": False}
    _ALIASES = dict(BaseOutputLayer._ALIASES, **{"lambda": "lambda_"})
    RUNTIME = "deeplearning4j_amd.nn.layers.output:CenterLossOutputLayerImpl"

    def param_specs(self):
        # gradientCheck: the centers are checked like any parameter (dL/dc = lambda * sum(c_y - x)) and are not
        # moved by the forward-backward pass (reference CenterLossOutputLayer.java:217-223)
        return super().param_specs() + [ParamSpec("cL", [self.nOut, self.nIn], "c", "zero",
                                                  trainable=bool(self.gradientCheck))]


class LossLayer(FeedForwardLayer):
    """No-parameter loss layer (reference LossLayer.java)."""
    FIELDS = {"lossFn": None}
    _ALIASES = dict(FeedForwardLayer._ALIASES, lossFunction="lossFn")
    _CONVERTERS = dict(FeedForwardLayer._CONVERTERS, lossFn=to_loss)
    RUNTIME = "deeplearning4j_amd.nn.layers.output:LossLayerImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["lossFn"] = to_loss(args[0])

    def getOutputType(self, layerIndex, inputType):
        return inputType

    def setNIn(self, inputType, override=False):
        super().setNIn(inputType, override)
        self.nOut = self.nIn

    def finalize_defaults(self):
        super().finalize_defaults()
        if self.lossFn is None:
            from .losses import LossMCXENT
            self.lossFn = LossMCXENT()


class RnnOutputLayer(BaseOutputLayer):
    RUNTIME = "deeplearning4j_amd.nn.layers.output:RnnOutputLayerImpl"

    def getOutputType(self, layerIndex, inputType):
        T = inputType.timeSeriesLength if isinstance(inputType, InputTypeRecurrent) else -1
        return InputType.recurrent(self.nOut, T)

    def getPreProcessorForInputType(self, inputType):
        from .preprocessors import CnnToRnnPreProcessor, FeedForwardToRnnPreProcessor
        if isinstance(inputType, InputTypeFeedForward):
            return FeedForwardToRnnPreProcessor()
        if isinstance(inputType, InputTypeConvolutional):
            return CnnToRnnPreProcessor(inputHeight=inputType.height, inputWidth=inputType.width,
                                        numChannels=inputType.channels)
        return None


class RnnLossLayer(LossLayer):
    RUNTIME = "deeplearning4j_amd.nn.layers.output:RnnLossLayerImpl"

    def getOutputType(self, layerIndex, inputType):
        if isinstance(inputType, InputTypeFeedForward):
            return InputType.recurrent(inputType.size)
        return inputType

    def getPreProcessorForInputType(self, inputType):
        # feed-forward / CNN activations are reshaped back to time series first, as for the RNN layers (reference
        # RnnLossLayer.getPreProcessorForInputType -> InputTypeUtil.getPreprocessorForInputTypeRnnLayers)
        return RnnOutputLayer.getPreProcessorForInputType(self, inputType)


class CnnLossLayer(LossLayer):
    """Per-pixel loss over NCHW activations (reference CnnLossLayer.java)."""
    RUNTIME = "deeplearning4j_amd.nn.layers.output:CnnLossLayerImpl"

    def getPreProcessorForInputType(self, inputType):
        return None

    def setNIn(self, inputType, override=False):
        if isinstance(inputType, InputTypeConvolutional):
            self.nIn = self.nOut = inputType.channels


# ---------------------------------------------------------------------------------- convolution
def conv_out_size(in_size, k, s, p, d, mode):
    """Reference nn/util/ConvolutionUtils.java:getOutputSize (Strict / Truncate / Same)."""
    k_eff = k + (k - 1) * (d - 1)
    if mode == ConvolutionMode.Same:
        return int(math.ceil(in_size / s))
    num = in_size - k_eff + 2 * p
    if num < 0:
        raise InvalidInputTypeException(f"Invalid input size {in_size} for kernel {k_eff}, padding {p}: the "
                                         f"kernel is larger than the padded input")
    if mode == ConvolutionMode.Strict and num % s != 0:
        raise DL4JInvalidConfigException(
            f"Invalid input/configuration for ConvolutionMode.Strict: (in={in_size} - k={k_eff} + 2*p={p})"
            f" / s={s} is not an integer. Use ConvolutionMode.Truncate or Same.")
    return num // s + 1


def same_padding(in_size, out_size, k, s, d):
    """Top/left padding for Same mode; returns (before, after)."""
    k_eff = k + (k - 1) * (d - 1)
    total = max(0, (out_size - 1) * s + k_eff - in_size)
    return total // 2, total - total // 2


class ConvolutionLayer(FeedForwardLayer):
    FIELDS = {"kernelSize": [5, 5], "stride": [1, 1], "padding": [0, 0], "dilation": [1, 1],
              "convolutionMode": None, "cudnnAlgoMode": None, "hasBias": True,
              "cudnnFwdAlgo": None, "cudnnBwdFilterAlgo": None, "cudnnBwdDataAlgo": None}
    _CONVERTERS = dict(FeedForwardLayer._CONVERTERS, kernelSize=int_pair, stride=int_pair, padding=int_pair,
                       dilation=int_pair, convolutionMode=ConvolutionMode.of, cudnnAlgoMode=AlgoMode.of)
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:ConvolutionLayerImpl"
    _GEOM_DIMS = 2

    @classmethod
    def _geom_hook(cls, kw, name, v):
        """Builder setter of a 2-D geometry field: exactly two values (reference ConvolutionLayer.Builder /
        SubsamplingLayer.Builder -> ValidationUtils.validate2NonNegative; IllegalStateException)."""
        if cls._GEOM_DIMS == 2 and not isinstance(v, (list, tuple)):
            raise DL4JInvalidConfigException(f"{cls.__name__}: {name} needs 2 values, got the single value {v}")
        kw[name] = int_pair(v)

    @classmethod
    def _builder_hook_kernelSize(cls, kw, v):
        cls._geom_hook(kw, "kernelSize", v)

    @classmethod
    def _builder_hook_stride(cls, kw, v):
        cls._geom_hook(kw, "stride", v)

    @classmethod
    def _builder_hook_padding(cls, kw, v):
        cls._geom_hook(kw, "padding", v)

    @classmethod
    def _builder_positional(cls, kw, *args):
        names = ["kernelSize", "stride", "padding"]
        if len(args) >= 1 and isinstance(args[0], int) and all(isinstance(a, int) for a in args):
            # Builder(kh, kw) or Builder(kh, kw, sh, sw, ...)
            vals = list(args)
            args = [vals[i:i + 2] for i in range(0, len(vals), 2)]
        for n, a in zip(names, args):
            kw[n] = int_pair(a)

    def _post_init(self):
        validate_kernel_geometry(self)

    def finalize_defaults(self):
        super().finalize_defaults()
        if self.convolutionMode is None:
            self.convolutionMode = ConvolutionMode.Truncate
        if self.cudnnAlgoMode is None:
            self.cudnnAlgoMode = AlgoMode.PREFER_FASTEST

    def _out_hw(self, inputType):
        mode = self.convolutionMode or ConvolutionMode.Truncate
        oh = conv_out_size(inputType.height, self.kernelSize[0], self.stride[0], self.padding[0],
                           self.dilation[0], mode)
        ow = conv_out_size(inputType.width, self.kernelSize[1], self.stride[1], self.padding[1],
                           self.dilation[1], mode)
        return oh, ow

    def getOutputType(self, layerIndex, inputType):
        if isinstance(inputType, InputTypeConvolutionalFlat):
            inputType = inputType.getUnflattenedType()
        if not isinstance(inputType, InputTypeConvolutional):
            raise ValueError(f"Invalid input for {type(self).__name__} (layer {layerIndex}): expected CNN "
                             f"input, got {inputType}")
        oh, ow = self._out_hw(inputType)
        return InputType.convolutional(oh, ow, self.nOut)

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        if isinstance(inputType, InputTypeConvolutional):
            self.nIn = inputType.channels
        elif isinstance(inputType, InputTypeConvolutionalFlat):
            self.nIn = inputType.depth

    def getPreProcessorForInputType(self, inputType):
        from .preprocessors import FeedForwardToCnnPreProcessor
        if isinstance(inputType, InputTypeConvolutionalFlat):
            return FeedForwardToCnnPreProcessor(inputHeight=inputType.height, inputWidth=inputType.width,
                                                numChannels=inputType.depth)
        return None

    def param_specs(self):
        kh, kw = self.kernelSize
        fan_in = self.nIn * kh * kw
        fan_out = self.nOut * kh * kw
        specs = []
        if self.hasBias:
            specs.append(ParamSpec("b", [1, self.nOut], "c", "bias"))
        specs.append(ParamSpec("W", [self.nOut, self.nIn, kh, kw], "c", "weight", fan_in, fan_out))
        return specs


class Convolution2D(ConvolutionLayer):
    pass


class Deconvolution2D(ConvolutionLayer):
    """Transposed convolution; weights [nIn, nOut, kh, kw] (reference Deconvolution2D.java:78)."""
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:Deconvolution2DImpl"

    def _out_hw(self, inputType):
        mode = self.convolutionMode or ConvolutionMode.Truncate
        res = []
        for i, n in enumerate((inputType.height, inputType.width)):
            k, s, p, d = self.kernelSize[i], self.stride[i], self.padding[i], self.dilation[i]
            if mode == ConvolutionMode.Same:
                res.append(n * s)
            else:
                res.append(s * (n - 1) + (k + (k - 1) * (d - 1)) - 2 * p)
        return tuple(res)

    def param_specs(self):
        kh, kw = self.kernelSize
        specs = []
        if self.hasBias:
            specs.append(ParamSpec("b", [1, self.nOut], "c", "bias"))
        specs.append(ParamSpec("W", [self.nIn, self.nOut, kh, kw], "c", "weight", self.nIn * kh * kw,
                               self.nOut * kh * kw))
        return specs


class SeparableConvolution2D(ConvolutionLayer):
    """Depthwise (depthMultiplier) then pointwise 1x1 (reference SeparableConvolution2D.java:148)."""
    FIELDS = {"depthMultiplier": 1}
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:SeparableConvolution2DImpl"

    def param_specs(self):
        kh, kw = self.kernelSize
        dm = self.depthMultiplier
        specs = []
        if self.hasBias:
            specs.append(ParamSpec("b", [1, self.nOut], "c", "bias"))
        specs.append(ParamSpec("W", [dm, self.nIn, kh, kw], "c", "weight", self.nIn * kh * kw, dm * kh * kw))
        specs.append(ParamSpec("pW", [self.nOut, self.nIn * dm, 1, 1], "c", "weight", self.nIn * dm, self.nOut))
        return specs


class DepthwiseConvolution2D(ConvolutionLayer):
    FIELDS = {"depthMultiplier": 1}
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:DepthwiseConvolution2DImpl"

    def getOutputType(self, layerIndex, inputType):
        t = super().getOutputType(layerIndex, inputType)
        return InputType.convolutional(t.height, t.width, self.nIn * self.depthMultiplier)

    def setNIn(self, inputType, override=False):
        super().setNIn(inputType, override)
        self.nOut = self.nIn * self.depthMultiplier

    def param_specs(self):
        kh, kw = self.kernelSize
        dm = self.depthMultiplier
        specs = []
        if self.hasBias:
            specs.append(ParamSpec("b", [1, self.nIn * dm], "c", "bias"))
        specs.append(ParamSpec("W", [dm, self.nIn, kh, kw], "c", "weight", kh * kw, dm * kh * kw))
        return specs


class Convolution1DLayer(ConvolutionLayer):
    """1D conv over RNN-format input [mb, nIn, T] (reference Convolution1DLayer.java:50)."""
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:Convolution1DLayerImpl"
    _GEOM_DIMS = 1

    @classmethod
    def _builder_positional(cls, kw, *args):
        names = ["kernelSize", "stride", "padding"]
        for n, a in zip(names, args):
            a = a[0] if isinstance(a, (list, tuple)) else a
            kw[n] = [int(a), 1]

    def _post_init(self):
        for n in ("kernelSize", "stride", "padding", "dilation"):
            v = getattr(self, n)
            if v is not None and len(v) == 2 and n != "padding" and v[1] != 1 and v[0] == v[1]:
                setattr(self, n, [v[0], 1])
            elif v is not None and len(v) == 2 and n == "padding" and v[0] == v[1] and v[1] != 0:
                setattr(self, n, [v[0], 0])
        validate_kernel_geometry(self)

    def getOutputType(self, layerIndex, inputType):
        mode = self.convolutionMode or ConvolutionMode.Truncate
        T = inputType.timeSeriesLength
        oT = conv_out_size(T, self.kernelSize[0], self.stride[0], self.padding[0], self.dilation[0], mode) \
            if T and T > 0 else -1
        return InputType.recurrent(self.nOut, oT)

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        if isinstance(inputType, InputTypeRecurrent):
            self.nIn = inputType.size

    def getPreProcessorForInputType(self, inputType):
        from .preprocessors import FeedForwardToRnnPreProcessor
        if isinstance(inputType, InputTypeFeedForward):
            return FeedForwardToRnnPreProcessor()
        return None

    def param_specs(self):
        k = self.kernelSize[0]
        specs = []
        if self.hasBias:
            specs.append(ParamSpec("b", [1, self.nOut], "c", "bias"))
        specs.append(ParamSpec("W", [self.nOut, self.nIn, k, 1], "c", "weight", self.nIn * k, self.nOut * k))
        return specs


class Convolution1D(Convolution1DLayer):
    pass


class SubsamplingLayer(Layer):
    FIELDS = {"poolingType": PoolingType.MAX, "kernelSize": [1, 1], "stride": [2, 2], "padding": [0, 0],
              "dilation": [1, 1], "convolutionMode": None, "pnorm": 2, "eps": 1e-8, "cudnnAllowFallback": True}
    _CONVERTERS = dict(Layer._CONVERTERS, kernelSize=int_pair, stride=int_pair, padding=int_pair,
                       dilation=int_pair, convolutionMode=ConvolutionMode.of, poolingType=PoolingType.of)
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:SubsamplingLayerImpl"
    PoolingType = PoolingType                      # the reference's nested SubsamplingLayer.PoolingType
    _GEOM_DIMS = 2
    _geom_hook = ConvolutionLayer.__dict__["_geom_hook"]
    _builder_hook_kernelSize = ConvolutionLayer.__dict__["_builder_hook_kernelSize"]
    _builder_hook_stride = ConvolutionLayer.__dict__["_builder_hook_stride"]
    _builder_hook_padding = ConvolutionLayer.__dict__["_builder_hook_padding"]

    @classmethod
    def _builder_positional(cls, kw, *args):
        args = list(args)
        if args and isinstance(args[0], (PoolingType, str)) and not isinstance(args[0], list):
            kw["poolingType"] = PoolingType.of(args.pop(0))
        for n, a in zip(["kernelSize", "stride", "padding"], args):
            kw[n] = int_pair(a)

    def _post_init(self):
        validate_kernel_geometry(self)

    def finalize_defaults(self):
        if self.convolutionMode is None:
            self.convolutionMode = ConvolutionMode.Truncate

    def applyGlobal(self, g):
        if self.convolutionMode is None and g.get("convolutionMode") is not None:
            self.convolutionMode = g["convolutionMode"]

    def getOutputType(self, layerIndex, inputType):
        if isinstance(inputType, InputTypeConvolutionalFlat):
            inputType = inputType.getUnflattenedType()
        mode = self.convolutionMode or ConvolutionMode.Truncate
        oh = conv_out_size(inputType.height, self.kernelSize[0], self.stride[0], self.padding[0],
                           self.dilation[0], mode)
        ow = conv_out_size(inputType.width, self.kernelSize[1], self.stride[1], self.padding[1],
                           self.dilation[1], mode)
        return InputType.convolutional(oh, ow, inputType.channels)

    def getPreProcessorForInputType(self, inputType):
        from .preprocessors import FeedForwardToCnnPreProcessor
        if isinstance(inputType, InputTypeConvolutionalFlat):
            return FeedForwardToCnnPreProcessor(inputHeight=inputType.height, inputWidth=inputType.width,
                                                numChannels=inputType.depth)
        return None


class Pooling2D(SubsamplingLayer):
    pass


class Subsampling1DLayer(SubsamplingLayer):
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:Subsampling1DLayerImpl"
    _GEOM_DIMS = 1

    @classmethod
    def _builder_positional(cls, kw, *args):
        args = list(args)
        if args and isinstance(args[0], (PoolingType, str)):
            kw["poolingType"] = PoolingType.of(args.pop(0))
        for n, a in zip(["kernelSize", "stride", "padding"], args):
            a = a[0] if isinstance(a, (list, tuple)) else a
            kw[n] = [int(a), 1] if n != "padding" else [int(a), 0]

    def _post_init(self):
        # setter-built sizes (.kernelSize(2).stride(1)) arrive as square 2-D pairs: the second dim is the dummy
        # width of the [mb, C, T, 1] view
        for n in ("kernelSize", "stride", "padding", "dilation"):
            v = getattr(self, n, None)
            if v is None or len(v) != 2 or v[0] != v[1]:
                continue
            if n == "padding":
                if v[1] != 0:
                    setattr(self, n, [v[0], 0])
            elif v[1] != 1:
                setattr(self, n, [v[0], 1])
        validate_kernel_geometry(self)

    def getOutputType(self, layerIndex, inputType):
        mode = self.convolutionMode or ConvolutionMode.Truncate
        T = inputType.timeSeriesLength
        oT = conv_out_size(T, self.kernelSize[0], self.stride[0], self.padding[0], 1, mode) if T > 0 else -1
        return InputType.recurrent(inputType.size, oT)


class Pooling1D(Subsampling1DLayer):
    pass


class BatchNormalization(FeedForwardLayer):
    FIELDS = {"decay": 0.9, "eps": 1e-5, "isMinibatch": True, "lockGammaBeta": False, "gamma": 1.0,
              "beta": 0.0}
    RUNTIME = "deeplearning4j_amd.nn.layers.normalization:BatchNormalizationImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        if args:
            kw["decay"] = float(args[0])
        if len(args) > 1:
            kw["isMinibatch"] = bool(args[1])

    def getOutputType(self, layerIndex, inputType):
        return inputType

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        if isinstance(inputType, InputTypeConvolutional):
            self.nIn = inputType.channels
        elif isinstance(inputType, InputTypeConvolutionalFlat):
            self.nIn = inputType.depth
        elif isinstance(inputType, InputTypeRecurrent):
            self.nIn = inputType.size
        else:
            self.nIn = inputType.size
        self.nOut = self.nIn

    def getPreProcessorForInputType(self, inputType):
        if isinstance(inputType, InputTypeConvolutionalFlat):
            from .preprocessors import FeedForwardToCnnPreProcessor
            return FeedForwardToCnnPreProcessor(inputHeight=inputType.height, inputWidth=inputType.width,
                                                numChannels=inputType.depth)
        return None

    def finalize_defaults(self):
        super().finalize_defaults()
        from .activations import ActivationIdentity
        # BN has no activation of its own in the zoo nets unless set explicitly
        if self.activation is None:
            self.activation = ActivationIdentity()

    def param_specs(self):
        n = self.nOut or self.nIn
        specs = []
        if not self.lockGammaBeta:
            specs += [ParamSpec("gamma", [1, n], "c", "const", value=self.gamma),
                      ParamSpec("beta", [1, n], "c", "const", value=self.beta)]
        specs += [ParamSpec("mean", [1, n], "c", "const", value=0.0, trainable=False),
                  ParamSpec("var", [1, n], "c", "const", value=1.0, trainable=False)]
        return specs

    def is_bias(self, key):
        return key == "beta"

    def updaterFor(self, key):
        if key in ("mean", "var"):
            from .updaters import NoOp
            return NoOp()
        return super().updaterFor(key)

    def l1For(self, key):
        # no BatchNormalization parameter is regularised (reference BatchNormalization.getL1ByParam :132-135)
        return 0.0

    def l2For(self, key):
        return 0.0


class LocalResponseNormalization(Layer):
    FIELDS = {"k": 2.0, "n": 5.0, "alpha": 1e-4, "beta": 0.75, "cudnnAllowFallback": True}
    RUNTIME = "deeplearning4j_amd.nn.layers.normalization:LocalResponseNormalizationImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        """Builder(k, n, alpha, beta) or Builder(alpha, beta) (LocalResponseNormalization.java Builder ctors)."""
        names = ["k", "n", "alpha", "beta"] if len(args) != 2 else ["alpha", "beta"]
        for n, v in zip(names, args):
            kw[n] = float(v)


class LayerNormalization(FeedForwardLayer):
    """LayerNorm over the feature dim (new; needed by the BERT-base config of BASELINE.json)."""
    FIELDS = {"eps": 1e-12}
    RUNTIME = "deeplearning4j_amd.nn.layers.normalization:LayerNormalizationImpl"

    def getOutputType(self, layerIndex, inputType):
        return inputType

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        self.nIn = inputType.size
        self.nOut = self.nIn

    def getPreProcessorForInputType(self, inputType):
        return None

    def param_specs(self):
        return [ParamSpec("gamma", [1, self.nIn], "c", "const", value=1.0),
                ParamSpec("beta", [1, self.nIn], "c", "const", value=0.0)]

    def is_bias(self, key):
        return key == "beta"


class ActivationLayer(NoParamLayer):
    FIELDS = {"activation": None}
    _CONVERTERS = dict(NoParamLayer._CONVERTERS, activation=to_activation)
    RUNTIME = "deeplearning4j_amd.nn.layers.feedforward:ActivationLayerImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["activation"] = to_activation(args[0])

    def __init__(self, activation=None, **kw):
        super().__init__(activation=activation, **kw)

    def applyGlobal(self, g):
        if self.activation is None and g.get("activation") is not None:
            self.activation = to_activation(g["activation"])

    def finalize_defaults(self):
        if self.activation is None:
            from .activations import ActivationSigmoid
            self.activation = ActivationSigmoid()


class DropoutLayer(FeedForwardLayer):
    RUNTIME = "deeplearning4j_amd.nn.layers.feedforward:DropoutLayerImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["idropout"] = to_dropout(args[0])

    def getOutputType(self, layerIndex, inputType):
        return inputType

    def getPreProcessorForInputType(self, inputType):
        return None

    def setNIn(self, inputType, override=False):
        pass


class GlobalPoolingLayer(NoParamLayer):
    FIELDS = {"poolingType": PoolingType.MAX, "poolingDimensions": None, "pnorm": 2, "collapseDimensions": True}
    _CONVERTERS = dict(NoParamLayer._CONVERTERS, poolingType=PoolingType.of, poolingDimensions=int_list)
    RUNTIME = "deeplearning4j_amd.nn.layers.pooling:GlobalPoolingLayerImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["poolingType"] = PoolingType.of(args[0])

    def getOutputType(self, layerIndex, inputType):
        if isinstance(inputType, InputTypeConvolutional):
            if self.collapseDimensions:
                return InputType.feedForward(inputType.channels)
            return InputType.convolutional(1, 1, inputType.channels)
        if isinstance(inputType, InputTypeRecurrent):
            if self.collapseDimensions:
                return InputType.feedForward(inputType.size)
            return InputType.recurrent(inputType.size, 1)
        return inputType


class ZeroPaddingLayer(NoParamLayer):
    """padding = [top, bottom, left, right] (reference ZeroPaddingLayer.java:58)."""
    FIELDS = {"padding": [0, 0, 0, 0]}
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:ZeroPaddingLayerImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        if len(args) == 1:
            a = args[0]
            args = tuple(a) if isinstance(a, (list, tuple)) else (a,)
        if len(args) == 1:
            kw["padding"] = [args[0]] * 4
        elif len(args) == 2:
            kw["padding"] = [args[0], args[0], args[1], args[1]]
        else:
            kw["padding"] = [int(x) for x in args]

    def _post_init(self):
        p = self.padding
        if isinstance(p, int):
            self.padding = [p] * 4
        elif len(p) == 2:
            self.padding = [p[0], p[0], p[1], p[1]]

    def getOutputType(self, layerIndex, inputType):
        t, b, l, r = self.padding
        return InputType.convolutional(inputType.height + t + b, inputType.width + l + r, inputType.channels)


class ZeroPadding1DLayer(NoParamLayer):
    FIELDS = {"padding": [0, 0]}
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:ZeroPadding1DLayerImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["padding"] = [args[0], args[0]] if len(args) == 1 and isinstance(args[0], int) else list(
            args[0] if len(args) == 1 else args)

    def getOutputType(self, layerIndex, inputType):
        T = inputType.timeSeriesLength
        return InputType.recurrent(inputType.size, T + sum(self.padding) if T > 0 else -1)


class Cropping2D(NoParamLayer):
    FIELDS = {"cropping": [0, 0, 0, 0]}
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:Cropping2DImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        ZeroPaddingLayer._builder_positional(kw, *args)
        kw["cropping"] = kw.pop("padding")

    def getOutputType(self, layerIndex, inputType):
        t, b, l, r = self.cropping
        return InputType.convolutional(inputType.height - t - b, inputType.width - l - r, inputType.channels)


class Upsampling2D(NoParamLayer):
    FIELDS = {"size": [2, 2]}
    _CONVERTERS = dict(NoParamLayer._CONVERTERS, size=int_pair)
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:Upsampling2DImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["size"] = int_pair(args[0])

    def getOutputType(self, layerIndex, inputType):
        return InputType.convolutional(inputType.height * self.size[0], inputType.width * self.size[1],
                                       inputType.channels)


class Upsampling1D(NoParamLayer):
    FIELDS = {"size": [2]}
    _CONVERTERS = dict(NoParamLayer._CONVERTERS, size=int_list)
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:Upsampling1DImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["size"] = int_list(args[0])

    def getOutputType(self, layerIndex, inputType):
        T = inputType.timeSeriesLength
        return InputType.recurrent(inputType.size, T * self.size[0] if T > 0 else -1)


class SpaceToDepthLayer(NoParamLayer):
    FIELDS = {"blockSize": 2, "dataFormat": "NCHW"}
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:SpaceToDepthImpl"

    class DataFormat:                              # the reference's nested SpaceToDepthLayer.DataFormat
        NCHW = "NCHW"
        NHWC = "NHWC"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["blockSize"] = int(args[0])
        if len(args) > 1:
            kw["dataFormat"] = str(getattr(args[1], "value", args[1]))

    def getOutputType(self, layerIndex, inputType):
        b = self.blockSize
        return InputType.convolutional(inputType.height // b, inputType.width // b, inputType.channels * b * b)


class SpaceToBatchLayer(NoParamLayer):
    FIELDS = {"blocks": [2, 2], "padding": [[0, 0], [0, 0]]}
    RUNTIME = "deeplearning4j_amd.nn.layers.convolution:SpaceToBatchImpl"

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["blocks"] = int_pair(args[0])
        if len(args) > 1:
            kw["padding"] = args[1]

    def getOutputType(self, layerIndex, inputType):
        (pt, pb), (pl, pr) = self.padding
        return InputType.convolutional((inputType.height + pt + pb) // self.blocks[0],
                                       (inputType.width + pl + pr) // self.blocks[1], inputType.channels)


# ---------------------------------------------------------------------------------- recurrent
class BaseRecurrentLayer(FeedForwardLayer):
    FIELDS = {"weightInitRecurrent": None, "distRecurrent": None}
    _CONVERTERS = dict(FeedForwardLayer._CONVERTERS, weightInitRecurrent=to_weight_init)

    def getOutputType(self, layerIndex, inputType):
        T = inputType.timeSeriesLength if isinstance(inputType, InputTypeRecurrent) else -1
        return InputType.recurrent(self.nOut, T)

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        if isinstance(inputType, InputTypeRecurrent):
            self.nIn = inputType.size
        else:
            super().setNIn(inputType, override)

    def getPreProcessorForInputType(self, inputType):
        from .preprocessors import CnnToRnnPreProcessor, FeedForwardToRnnPreProcessor
        if isinstance(inputType, InputTypeFeedForward):
            return FeedForwardToRnnPreProcessor()
        if isinstance(inputType, InputTypeConvolutional):
            return CnnToRnnPreProcessor(inputHeight=inputType.height, inputWidth=inputType.width,
                                        numChannels=inputType.channels)
        return None


class AbstractLSTM(BaseRecurrentLayer):
    FIELDS = {"forgetGateBiasInit": 1.0, "gateActivationFn": None}
    _CONVERTERS = dict(BaseRecurrentLayer._CONVERTERS, gateActivationFn=to_activation)
    _ALIASES = dict(BaseRecurrentLayer._ALIASES, gateActivationFunction="gateActivationFn")
    PEEPHOLE = False

    def finalize_defaults(self):
        super().finalize_defaults()
        if self.gateActivationFn is None:
            from .activations import ActivationSigmoid
            self.gateActivationFn = ActivationSigmoid()

    def param_specs(self):
        H = self.nOut
        rw_cols = 4 * H + (3 if self.PEEPHOLE else 0)
        return [ParamSpec("W", [self.nIn, 4 * H], "f", "weight", self.nIn, 4 * H),
                ParamSpec("RW", [H, rw_cols], "f", "recurrent", H, 4 * H),
                ParamSpec("b", [1, 4 * H], "c", "lstm_bias", value=self.forgetGateBiasInit)]


class LSTM(AbstractLSTM):
    """LSTM without peepholes, gate order IFOG (reference LSTM.java:80, LSTMHelpers.java)."""
    RUNTIME = "deeplearning4j_amd.nn.layers.recurrent:LSTMImpl"


class GravesLSTM(AbstractLSTM):
    """LSTM with peephole connections (Graves 2013), RW has 3 extra peephole columns."""
    PEEPHOLE = True
    RUNTIME = "deeplearning4j_amd.nn.layers.recurrent:GravesLSTMImpl"


class GravesBidirectionalLSTM(AbstractLSTM):
    PEEPHOLE = True
    RUNTIME = "deeplearning4j_amd.nn.layers.recurrent:GravesBidirectionalLSTMImpl"

    def param_specs(self):
        H = self.nOut
        out = []
        for d in ("F", "B"):
            out += [ParamSpec("W" + d, [self.nIn, 4 * H], "f", "weight", self.nIn, 4 * H),
                    ParamSpec("RW" + d, [H, 4 * H + 3], "f", "recurrent", H, 4 * H),
                    ParamSpec("b" + d, [1, 4 * H], "c", "lstm_bias", value=self.forgetGateBiasInit)]
        return out

    def is_bias(self, key):
        return key in ("bF", "bB")


class SimpleRnn(BaseRecurrentLayer):
    """h_t = act(x_t W + h_{t-1} RW + b) (reference layers/recurrent/SimpleRnn.java:44)."""
    RUNTIME = "deeplearning4j_amd.nn.layers.recurrent:SimpleRnnImpl"

    def param_specs(self):
        return [ParamSpec("W", [self.nIn, self.nOut], "f", "weight", self.nIn, self.nOut),
                ParamSpec("RW", [self.nOut, self.nOut], "f", "recurrent", self.nOut, self.nOut),
                ParamSpec("b", [1, self.nOut], "c", "bias")]


class BaseWrapperLayer(Layer):
    FIELDS = {"underlying": None}

    def getOutputType(self, layerIndex, inputType):
        return self.underlying.getOutputType(layerIndex, inputType)

    def setNIn(self, inputType, override=False):
        self.underlying.setNIn(inputType, override)

    def getPreProcessorForInputType(self, inputType):
        return self.underlying.getPreProcessorForInputType(inputType)

    def param_specs(self):
        return self.underlying.param_specs()

    def applyGlobal(self, g):
        self.underlying.applyGlobal(g)

    def finalize_defaults(self):
        if hasattr(self.underlying, "finalize_defaults"):
            self.underlying.finalize_defaults()

    def updaterFor(self, key):
        return self.underlying.updaterFor(key)

    def l1For(self, key):
        return self.underlying.l1For(key)

    def l2For(self, key):
        return self.underlying.l2For(key)

    def is_bias(self, key):
        return self.underlying.is_bias(key)


class Bidirectional(BaseWrapperLayer):
    """Wraps a recurrent layer; forward + time-reversed copies, merged by ``mode``
    (reference nn/conf/layers/recurrent/Bidirectional.java). Params: 'f'+key, 'b'+key."""
    FIELDS = {"mode": "CONCAT"}
    RUNTIME = "deeplearning4j_amd.nn.layers.recurrent:BidirectionalImpl"

    class Mode:
        """Bidirectional.Mode.CONCAT / ADD / MUL / AVERAGE (reference Bidirectional.Mode)."""
        CONCAT, ADD, MUL, AVERAGE = "CONCAT", "ADD", "MUL", "AVERAGE"

    @classmethod
    def _builder_positional(cls, kw, *args):
        if len(args) == 1:
            kw["underlying"] = args[0]
        else:
            kw["mode"] = str(args[0]).upper()
            kw["underlying"] = args[1]

    def __init__(self, *args, **kw):
        if args:
            self._builder_positional(kw, *args)
        super().__init__(**kw)

    def getOutputType(self, layerIndex, inputType):
        t = self.underlying.getOutputType(layerIndex, inputType)
        if self.mode == "CONCAT":
            return InputType.recurrent(t.size * 2, t.timeSeriesLength)
        return t

    def param_specs(self):
        out = []
        for d in ("f", "b"):
            for p in self.underlying.param_specs():
                q = ParamSpec(d + p.key, p.shape, p.order, p.kind, p.fan_in, p.fan_out, p.value, p.trainable)
                out.append(q)
        return out

    def _strip(self, key):
        return key[1:]

    def updaterFor(self, key):
        return self.underlying.updaterFor(self._strip(key))

    def l1For(self, key):
        return self.underlying.l1For(self._strip(key))

    def l2For(self, key):
        return self.underlying.l2For(self._strip(key))

    def is_bias(self, key):
        return self.underlying.is_bias(self._strip(key))


class LastTimeStep(BaseWrapperLayer):
    RUNTIME = "deeplearning4j_amd.nn.layers.recurrent:LastTimeStepImpl"

    def __init__(self, underlying=None, **kw):
        super().__init__(underlying=underlying, **kw)

    def getOutputType(self, layerIndex, inputType):
        t = self.underlying.getOutputType(layerIndex, inputType)
        return InputType.feedForward(t.size)


class FrozenLayer(BaseWrapperLayer):
    """Wraps a layer and blocks all updates to its params (reference FrozenLayer.java:77)."""
    RUNTIME = "deeplearning4j_amd.nn.layers.misc:FrozenLayerImpl"
    _ALIASES = dict(Layer._ALIASES, layer="underlying")     # FrozenLayer.Builder().layer(l)

    def __init__(self, layer=None, **kw):
        if layer is not None:
            kw["underlying"] = layer
        super().__init__(**kw)

    def getLayer(self):
        return self.underlying

    def updaterFor(self, key):
        from .updaters import NoOp
        return NoOp()

    def l1For(self, key):
        return 0.0

    def l2For(self, key):
        return 0.0


class FrozenLayerWithBackprop(FrozenLayer):
    """FrozenLayer variant whose backprop still produces the input epsilon (later DL4J releases'
    FrozenLayerWithBackprop; this reference snapshot only has FrozenLayer.java)."""
    RUNTIME = "deeplearning4j_amd.nn.layers.misc:FrozenLayerWithBackpropImpl"


class MaskLayer(NoParamLayer):
    RUNTIME = "deeplearning4j_amd.nn.layers.misc:MaskLayerImpl"


class MaskZeroLayer(BaseWrapperLayer):
    FIELDS = {"maskingValue": 0.0}
    RUNTIME = "deeplearning4j_amd.nn.layers.misc:MaskZeroLayerImpl"

    def __init__(self, underlying=None, maskingValue=0.0, **kw):
        super().__init__(underlying=underlying, maskingValue=maskingValue, **kw)


# ------------------------------------------------------------------------------- pretrain / misc
class AutoEncoder(FeedForwardLayer):
    FIELDS = {"corruptionLevel": 3e-1, "sparsity": 0.0, "lossFunction": None}
    _CONVERTERS = dict(FeedForwardLayer._CONVERTERS, lossFunction=to_loss)
    RUNTIME = "deeplearning4j_amd.nn.layers.pretrain:AutoEncoderImpl"

    def param_specs(self):
        return [ParamSpec("W", [self.nIn, self.nOut], "f", "weight", self.nIn, self.nOut),
                ParamSpec("b", [1, self.nOut], "c", "bias"),
                ParamSpec("vb", [1, self.nIn], "c", "bias")]

    def isPretrainParam(self, key):
        return key == "vb"


class VariationalAutoencoder(FeedForwardLayer):
    """VAE layer (Kingma & Welling), reference nn/layers/variational/VariationalAutoencoder.java:51."""
    FIELDS = {"encoderLayerSizes": [100], "decoderLayerSizes": [100], "outputDistribution": None,
              "pzxActivationFn": None, "numSamples": 1, "lossFunction": None}
    _CONVERTERS = dict(FeedForwardLayer._CONVERTERS, pzxActivationFn=to_activation)
    RUNTIME = "deeplearning4j_amd.nn.layers.variational:VariationalAutoencoderImpl"

    @staticmethod
    def _builder_hook_lossFunction(kw, v):
        """lossFunction(activation, loss): an ordinary loss as the reconstruction distribution (reference
        VariationalAutoencoder.Builder.lossFunction -> LossFunctionWrapper); lossFunction(loss): the pretrain-layer
        loss field inherited from BasePretrainNetwork.Builder (not used by the VAE's own objective)."""
        if isinstance(v, list) and len(v) == 2:
            from .variational import LossFunctionWrapper
            kw["outputDistribution"] = LossFunctionWrapper(v[0], v[1])
        else:
            kw["lossFunction"] = v

    def _dist_size(self):
        d = self.outputDistribution
        return d.distributionInputSize(self.nIn) if d is not None else 2 * self.nIn

    def param_specs(self):
        specs = []
        prev = self.nIn
        for i, s in enumerate(self.encoderLayerSizes):
            specs += [ParamSpec(f"e{i}W", [prev, s], "f", "weight", prev, s), ParamSpec(f"e{i}b", [1, s], "c", "bias")]
            prev = s
        n = self.nOut
        specs += [ParamSpec("pZXMeanW", [prev, n], "f", "weight", prev, n), ParamSpec("pZXMeanb", [1, n], "c", "bias"),
                  ParamSpec("pZXLogStd2W", [prev, n], "f", "weight", prev, n),
                  ParamSpec("pZXLogStd2b", [1, n], "c", "bias")]
        prev = n
        for i, s in enumerate(self.decoderLayerSizes):
            specs += [ParamSpec(f"d{i}W", [prev, s], "f", "weight", prev, s), ParamSpec(f"d{i}b", [1, s], "c", "bias")]
            prev = s
        ds = self._dist_size()
        specs += [ParamSpec("pXZW", [prev, ds], "f", "weight", prev, ds), ParamSpec("pXZb", [1, ds], "c", "bias")]
        return specs

    def is_bias(self, key):
        return key.endswith("b")

    def isPretrainParam(self, key):
        return key.startswith("d") or key.startswith("pXZ") or key.startswith("pZXLogStd2")


class Yolo2OutputLayer(Layer):
    """YOLOv2 loss layer, reference nn/conf/layers/objdetect/Yolo2OutputLayer.java:70."""
    FIELDS = {"lambdaCoord": 5.0, "lambdaNoObj": 0.5, "boundingBoxes": None, "lossPositionScale": None,
              "lossClassPredictions": None}
    _CONVERTERS = dict(Layer._CONVERTERS, lossPositionScale=to_loss, lossClassPredictions=to_loss)
    RUNTIME = "deeplearning4j_amd.nn.layers.objdetect:Yolo2OutputLayerImpl"

    def getOutputType(self, layerIndex, inputType):
        return inputType

    def setNIn(self, inputType, override=False):
        pass

    def getPreProcessorForInputType(self, inputType):
        return None


class SameDiffLayerConf(Layer):
    """Base for user layers defined as a SameDiff-lite graph (reference BaseSameDiffLayer.java:43).
    Subclasses implement ``defineParameters(params)`` and ``defineLayer(sd, input, paramTable)``."""
    FIELDS = {"nIn": 0, "nOut": 0, "weightInit": None, "dist": None, "biasInit": 0.0, "updater": None,
              "biasUpdater": None, "l1": None, "l2": None, "l1Bias": None, "l2Bias": None, "activation": None}
    _CONVERTERS = dict(Layer._CONVERTERS, weightInit=to_weight_init, updater=to_updater, biasUpdater=to_updater,
                       activation=to_activation)
    RUNTIME = "deeplearning4j_amd.samediff.layer:SameDiffLayerImpl"

    def defineParameters(self, params):
        raise NotImplementedError

    def defineLayer(self, sd, layerInput, paramTable):
        raise NotImplementedError

    def initializeParameters(self, params):
        pass

    def param_specs(self):
        from ...samediff.layer import SDLayerParams
        p = SDLayerParams()
        self.defineParameters(p)
        specs = []
        for k, shape in p.weights.items():
            fan_in = shape[0] if len(shape) > 1 else 1
            specs.append(ParamSpec(k, shape, "c", "weight", fan_in, shape[-1]))
        for k, shape in p.biases.items():
            specs.append(ParamSpec(k, shape, "c", "bias"))
        return specs

    def is_bias(self, key):
        from ...samediff.layer import SDLayerParams
        p = SDLayerParams()
        self.defineParameters(p)
        return key in p.biases

    def finalize_defaults(self):
        from .updaters import Sgd
        from .weights import WeightInit
        if self.weightInit is None:
            self.weightInit = WeightInit.XAVIER
        if self.updater is None:
            self.updater = Sgd(1e-3)
        for k in ("l1", "l2", "l1Bias", "l2Bias"):
            if getattr(self, k) is None:
                setattr(self, k, 0.0)

    def applyGlobal(self, g):
        for k in ("weightInit", "dist", "updater", "biasUpdater", "l1", "l2", "l1Bias", "l2Bias", "activation"):
            if getattr(self, k) is None and g.get(k) is not None:
                conv = self._CONVERTERS.get(k)
                setattr(self, k, conv(g[k]) if conv else g[k])

    def getOutputType(self, layerIndex, inputType):
        return InputType.feedForward(self.nOut)

    def setNIn(self, inputType, override=False):
        if not self.nIn or override:
            self.nIn = inputType.size if hasattr(inputType, "size") else inputType.arrayElementsPerExample()


class SelfAttentionLayer(FeedForwardLayer):
    """Multi-head self attention over RNN-format input [mb, nIn, T] (new: BERT config)."""
    FIELDS = {"nHeads": 1, "headSize": 0, "projectInput": True, "causal": False}
    RUNTIME = "deeplearning4j_amd.nn.layers.attention:SelfAttentionLayerImpl"

    def getOutputType(self, layerIndex, inputType):
        T = inputType.timeSeriesLength if isinstance(inputType, InputTypeRecurrent) else -1
        return InputType.recurrent(self.nOut, T)

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        self.nIn = inputType.size
        if not self.nOut:
            self.nOut = self.nIn

    def getPreProcessorForInputType(self, inputType):
        return None

    def param_specs(self):
        hs = self.headSize or (self.nOut // self.nHeads)
        d = self.nHeads * hs
        return [ParamSpec("Wq", [self.nIn, d], "c", "weight", self.nIn, d),
                ParamSpec("Wk", [self.nIn, d], "c", "weight", self.nIn, d),
                ParamSpec("Wv", [self.nIn, d], "c", "weight", self.nIn, d),
                ParamSpec("Wo", [d, self.nOut], "c", "weight", d, self.nOut),
                ParamSpec("bq", [1, d], "c", "bias"), ParamSpec("bk", [1, d], "c", "bias"),
                ParamSpec("bv", [1, d], "c", "bias"), ParamSpec("bo", [1, self.nOut], "c", "bias")]

    def is_bias(self, key):
        return key.startswith("b")


# ------------------------------------------------------------------------------------------------ transformer
class TransformerEncoderLayer(FeedForwardLayer):
    """One post-LN transformer encoder block (BERT): fused QKV projection -> multi-head attention (flash-style HIP
    kernel) -> output projection -> LayerNorm(+residual) -> FFN (GELU) -> LayerNorm(+residual). RNN-format
    input/output [mb, nIn, T] (new: BERT-base config of BASELINE.json; not in the reference)."""
    FIELDS = {"nHeads": 12, "ffnSize": 3072, "layerNormEps": 1e-12, "causal": False, "hiddenDropout": 0.0}
    RUNTIME = "deeplearning4j_amd.nn.layers.transformer:TransformerEncoderLayerImpl"

    def getOutputType(self, layerIndex, inputType):
        T = inputType.timeSeriesLength if isinstance(inputType, InputTypeRecurrent) else -1
        return InputType.recurrent(self.nOut, T)

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        self.nIn = inputType.size
        self.nOut = self.nIn

    def getPreProcessorForInputType(self, inputType):
        return None

    def param_specs(self):
        E, F = self.nIn, self.ffnSize
        return [ParamSpec("Wqkv", [E, 3 * E], "c", "weight", E, E), ParamSpec("bqkv", [1, 3 * E], "c", "bias"),
                ParamSpec("Wo", [E, E], "c", "weight", E, E), ParamSpec("bo", [1, E], "c", "bias"),
                ParamSpec("ln1g", [1, E], "c", "const", value=1.0), ParamSpec("ln1b", [1, E], "c", "const", value=0.0),
                ParamSpec("W1", [E, F], "c", "weight", E, F), ParamSpec("b1", [1, F], "c", "bias"),
                ParamSpec("W2", [F, E], "c", "weight", F, E), ParamSpec("b2", [1, E], "c", "bias"),
                ParamSpec("ln2g", [1, E], "c", "const", value=1.0), ParamSpec("ln2b", [1, E], "c", "const", value=0.0)]

    def is_bias(self, key):
        return key.startswith("b") or key in ("ln1b", "ln2b")


class BertEmbeddingLayer(FeedForwardLayer):
    """Token ids [mb, T] -> LayerNorm(word + position + token-type(0) embeddings) as [mb, nOut, T]
    (nIn = vocabulary size)."""
    FIELDS = {"maxPositions": 512, "typeVocabSize": 2, "layerNormEps": 1e-12, "inputLength": -1}
    RUNTIME = "deeplearning4j_amd.nn.layers.transformer:BertEmbeddingLayerImpl"

    def getOutputType(self, layerIndex, inputType):
        return InputType.recurrent(self.nOut, self.inputLength)

    def setNIn(self, inputType, override=False):
        return

    def getPreProcessorForInputType(self, inputType):
        return None

    def param_specs(self):
        E = self.nOut
        return [ParamSpec("Wword", [self.nIn, E], "c", "weight", self.nIn, E),
                ParamSpec("Wpos", [self.maxPositions, E], "c", "weight", self.maxPositions, E),
                ParamSpec("Wtype", [self.typeVocabSize, E], "c", "weight", self.typeVocabSize, E),
                ParamSpec("lng", [1, E], "c", "const", value=1.0), ParamSpec("lnb", [1, E], "c", "const", value=0.0)]

    def is_bias(self, key):
        return key == "lnb"


class BertPoolerLayer(FeedForwardLayer):
    """First ([CLS]) time step of [mb, nIn, T] -> tanh(x W + b) as [mb, nOut]."""
    RUNTIME = "deeplearning4j_amd.nn.layers.transformer:BertPoolerLayerImpl"

    def setNIn(self, inputType, override=False):
        if self.nIn and not override:
            return
        self.nIn = inputType.size

    def getPreProcessorForInputType(self, inputType):
        return None

    def param_specs(self):
        return [ParamSpec("W", [self.nIn, self.nOut], "c", "weight", self.nIn, self.nOut),
                ParamSpec("b", [1, self.nOut], "c", "bias")]
