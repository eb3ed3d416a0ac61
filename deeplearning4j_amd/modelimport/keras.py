"""Keras (1.x and 2.x, TensorFlow or Theano dim ordering) model import from HDF5 / JSON.

Reference: deeplearning4j-modelimport (KER:KerasModelImport.java:50-190, KerasModel.java:360-376,
KerasSequentialModel.java, layers/**, utils/KerasModelUtils.java:60,170). Files are read with the in-repo HDF5
reader (modelimport/hdf5.py); nothing in the file is ever executed (Lambda layers need a registered mapper,
exactly like the reference's KerasLayer.registerCustomLayer).

Output: Sequential -> MultiLayerNetwork, functional Model -> ComputationGraph, with the Keras weights copied into
the DL4J flat parameter layout:
  * Dense kernel [nIn, nOut] -> W; conv kernels: TF [kh, kw, in, out] -> [out, in, kh, kw]; Theano ordering kept
    and each filter rotated by 180 degrees (KerasConvolution.java:101-141)
  * LSTM: Keras gate blocks (i, f, c, o) -> DL4J (c, f, o, i); Keras 1 separate W_*/U_*/b_* matrices concatenated
  * BatchNormalization: moving variance + epsilon -> DL4J's global variance (DL4J stores var+eps and uses it
    unchanged at inference), gamma/beta/mean as-is
  * Flatten/Reshape after channels-last tensors insert preprocessors that reproduce TensorFlow's (h, w, c)
    flatten order, so the following Dense weights apply unchanged (TensorFlowCnnToFeedForwardPreProcessor)
DL4J-side inputs are NCHW for images and [mb, features, T] for sequences (the reference's convention).
"""
import copy
import json

import numpy as np
import torch

from ..nn.conf import preprocessors as PP
from ..nn.conf.activations import Activation
from ..nn.conf.base import Config
from ..nn.conf.enums import ConvolutionMode, PoolingType
from ..nn.conf.inputs import InputType, InputTypeConvolutional, InputTypeRecurrent
from ..nn.conf import layers as L
from ..nn.conf import graph as G
from . import hdf5


class InvalidKerasConfigurationException(Exception):
    pass


class UnsupportedKerasConfigurationException(Exception):
    pass


# --------------------------------------------------------------------------------------- preprocessors
class TensorFlowCnnToFeedForwardPreProcessor(PP.InputPreProcessor):
    """NCHW activations flattened in TensorFlow's NHWC (h, w, c) order."""
    FIELDS = {"inputHeight": 0, "inputWidth": 0, "numChannels": 0}

    def preProcess(self, x, miniBatchSize, training=False):
        if x.dim() == 2:
            return x
        self._shape = x.shape
        return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)

    def backprop(self, eps, miniBatchSize):
        n, c, h, w = getattr(self, "_shape", (eps.shape[0], self.numChannels, self.inputHeight, self.inputWidth))
        return eps.reshape(n, h, w, c).permute(0, 3, 1, 2)

    def getOutputType(self, inputType):
        if isinstance(inputType, InputTypeConvolutional):
            return InputType.feedForward(inputType.channels * inputType.height * inputType.width)
        return inputType


class KerasReshapePreprocessor(PP.InputPreProcessor):
    """Keras Reshape: the flat (TF-ordered) vector reshaped to ``targetShape`` given in Keras order, delivered
    in DL4J layout (NCHW for 3-d targets in channels_last, [mb, f, T] for 2-d targets)."""
    FIELDS = {"targetShape": [], "channelsLast": True, "inputShape": []}

    def _flat(self, x):
        if x.dim() == 4:
            return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1) if self.channelsLast else x.reshape(x.shape[0], -1)
        if x.dim() == 3:
            return x.permute(0, 2, 1).reshape(x.shape[0], -1)       # [mb, f, T] -> Keras [mb, T, f] flat
        return x

    def preProcess(self, x, miniBatchSize, training=False):
        self._in = x.shape
        t = list(self.targetShape)
        f = self._flat(x)
        if len(t) == 3:
            if self.channelsLast:
                return f.reshape(x.shape[0], t[0], t[1], t[2]).permute(0, 3, 1, 2).contiguous()
            return f.reshape(x.shape[0], *t)
        if len(t) == 2:
            return f.reshape(x.shape[0], t[0], t[1]).permute(0, 2, 1).contiguous()
        return f.reshape(x.shape[0], *t)

    def backprop(self, eps, miniBatchSize):
        shp = self._in
        n = eps.shape[0]
        if eps.dim() == 4 and self.channelsLast:
            flat = eps.permute(0, 2, 3, 1).reshape(n, -1)
        elif eps.dim() == 3:
            flat = eps.permute(0, 2, 1).reshape(n, -1)
        else:
            flat = eps.reshape(n, -1)
        if len(shp) == 4:
            if self.channelsLast:
                return flat.reshape(n, shp[2], shp[3], shp[1]).permute(0, 3, 1, 2)
            return flat.reshape(shp)
        if len(shp) == 3:
            return flat.reshape(n, shp[2], shp[1]).permute(0, 2, 1)
        return flat.reshape(shp)

    def getOutputType(self, inputType):
        t = list(self.targetShape)
        if len(t) == 3:
            h, w, c = t if self.channelsLast else (t[1], t[2], t[0])
            return InputType.convolutional(h, w, c)
        if len(t) == 2:
            return InputType.recurrent(t[1], t[0])
        return InputType.feedForward(int(np.prod(t)))


# --------------------------------------------------------------------------------------- helpers
_ACT = {"linear": "IDENTITY", "relu": "RELU", "tanh": "TANH", "sigmoid": "SIGMOID", "softmax": "SOFTMAX",
        "hard_sigmoid": "HARDSIGMOID", "softplus": "SOFTPLUS", "softsign": "SOFTSIGN", "elu": "ELU", "selu": "SELU",
        "relu6": "RELU6", "swish": "SWISH", "gelu": "GELU", "exponential": None}

_LOSS = {"categorical_crossentropy": "MCXENT", "sparse_categorical_crossentropy": "SPARSE_MCXENT",
         "binary_crossentropy": "XENT", "mse": "MSE", "mean_squared_error": "MSE", "mae": "MEAN_ABSOLUTE_ERROR",
         "mean_absolute_error": "MEAN_ABSOLUTE_ERROR", "mape": "MEAN_ABSOLUTE_PERCENTAGE_ERROR",
         "msle": "MEAN_SQUARED_LOGARITHMIC_ERROR", "hinge": "HINGE", "squared_hinge": "SQUARED_HINGE",
         "kld": "KL_DIVERGENCE", "kullback_leibler_divergence": "KL_DIVERGENCE", "poisson": "POISSON",
         "cosine_proximity": "COSINE_PROXIMITY", "logcosh": "MSE"}


def _act(name):
    if name is None:
        return Activation.IDENTITY
    if isinstance(name, dict):
        name = name.get("class_name", "linear").lower()
    a = _ACT.get(str(name).lower())
    if a is None:
        raise UnsupportedKerasConfigurationException(f"Unsupported Keras activation {name!r}")
    return Activation[a]


def _pair(v, default=1):
    if v is None:
        return [default, default]
    if isinstance(v, int):
        return [v, v]
    return [int(x) for x in v]


def _mode(border):
    b = (border or "valid").lower()
    if b == "same":
        return ConvolutionMode.Same
    if b in ("valid", "causal"):
        return ConvolutionMode.Truncate
    raise UnsupportedKerasConfigurationException(f"padding {border!r}")


def _channels_last(cfg, default=True):
    if "data_format" in cfg and cfg["data_format"] is not None:
        return cfg["data_format"] == "channels_last"
    if "dim_ordering" in cfg and cfg["dim_ordering"] not in (None, "default"):
        return cfg["dim_ordering"] == "tf"
    return default


class _KLayer:
    """Translation of one Keras layer."""

    def __init__(self, name, kind, obj=None, inbound=None, setter=None, keras_class=None, cfg=None):
        self.name, self.kind, self.obj = name, kind, obj
        self.inbound = inbound or []
        self.setter = setter            # fn(dl4j_param_dict, keras_weight_dict)
        self.keras_class, self.cfg = keras_class, cfg


_CUSTOM = {}


class KerasLayer:
    @staticmethod
    def registerCustomLayer(name, mapper):
        """Register a mapper for a custom/Lambda layer class name: ``mapper(cfg, ctx) -> (kind, obj, setter)``
        (kind: "layer" | "vertex" | "preprocessor" | "skip"). Lambda bodies in Keras files are never run."""
        _CUSTOM[name] = mapper

    @staticmethod
    def clearCustomLayers():
        _CUSTOM.clear()

    @staticmethod
    def fromConfig(layerConfig, previousLayer=None, kerasMajorVersion=None):
        """One Keras layer config map ({class_name, config[, keras_version]}) -> the DL4J layer configuration (or
        graph vertex), as the reference's per-class Keras layer objects (KerasDense(layerConfig).getDenseLayer(),
        ...). ``previousLayer``: the config map of the layer feeding it (a mask_zero Embedding wraps a recurrent
        layer in MaskZeroLayer)."""
        v = kerasMajorVersion or int(layerConfig.get("keras_version", 2))
        ctx = _Ctx(v, False)
        m = _map_layer(layerConfig, ctx)
        if previousLayer is not None and _masks_zero(_map_layer(previousLayer, ctx)):
            _mask_zero_wrap(m)
        return m.obj

    @staticmethod
    def getInputPreprocessor(layerConfig, inputType, kerasMajorVersion=None):
        """The preprocessor a shape-only Keras layer (Reshape) puts in front of its consumer, for the given input
        type (reference KerasReshape.getInputPreprocessor(InputType...)): None for layers that carry a DL4J layer."""
        v = kerasMajorVersion or int(layerConfig.get("keras_version", 2))
        m = _map_layer(layerConfig, _Ctx(v, False))
        if m.kind != "reshape":
            return None
        cl = _channels_last(m.cfg)
        pp = KerasReshapePreprocessor(targetShape=list(m.cfg["target_shape"]), channelsLast=cl)
        if inputType is not None:
            pp.getOutputType(inputType)
        return pp


def space_to_depth_mapper(block_size=2):
    """Mapper for the reference's KerasSpaceToDepth custom Lambda (space_to_depth with block 2)."""
    def m(cfg, ctx):
        return "layer", L.SpaceToDepthLayer(blockSize=block_size), None
    return m


# --------------------------------------------------------------------------------------- weight setters
def _w(kw, *names):
    for n in names:
        if n in kw:
            return kw[n]
    raise InvalidKerasConfigurationException(f"missing Keras weight among {names}; have {sorted(kw)}")


def _set(params, key, arr):
    t = params[key]
    src = torch.as_tensor(np.ascontiguousarray(arr), dtype=t.dtype).reshape(t.shape)
    with torch.no_grad():
        t.copy_(src.to(t.device))


def _dense_setter(has_bias):
    def s(p, kw):
        _set(p, "W", _w(kw, "kernel", "W"))
        if has_bias:
            _set(p, "b", _w(kw, "bias", "b").reshape(1, -1))
    return s


def _conv_setter(has_bias, kernel_last, flip, conv1d=False):
    """kernel_last: kernel stored [kh, kw, in, out] (all Keras 2 files; Keras 1 'tf' ordering), otherwise
    [out, in, kh, kw] (Keras 1 'th'). flip: the file was trained on Theano, whose conv2d is a true convolution,
    so every filter is rotated by 180 degrees to get DL4J's cross-correlation (KerasConvolution.java:101-141)."""
    def s(p, kw):
        k = np.asarray(_w(kw, "kernel", "W"))
        if conv1d:
            if k.ndim == 4:                  # keras 1 conv1d kernel [k, 1, in, out]
                k = k[:, 0]
            w = np.transpose(k, (2, 1, 0))[..., None]   # [out, in, k, 1]
            if flip:
                w = w[:, :, ::-1, :]
        else:
            w = np.transpose(k, (3, 2, 0, 1)) if kernel_last else k
            if flip:
                w = w[:, :, ::-1, ::-1]
        _set(p, "W", np.ascontiguousarray(w))
        if has_bias:
            _set(p, "b", _w(kw, "bias", "b").reshape(1, -1))
    return s


def _bn_setter(eps, center, scale):
    def s(p, kw):
        if scale and "gamma" in p:
            _set(p, "gamma", _w(kw, "gamma"))
        if center and "beta" in p:
            _set(p, "beta", _w(kw, "beta"))
        _set(p, "mean", _w(kw, "moving_mean", "running_mean"))
        var = np.asarray(_w(kw, "moving_variance", "running_std"))
        _set(p, "var", var + eps)
    return s


def _lstm_arrays(kw, prefix=""):
    g = lambda *n: _w(kw, *[prefix + x for x in n])  # noqa: E731
    if prefix + "kernel" in kw:
        W, U, b = np.asarray(g("kernel")), np.asarray(g("recurrent_kernel")), np.asarray(g("bias"))
        H = U.shape[0]
        blk = lambda a, i: a[..., i * H:(i + 1) * H]  # noqa: E731
        Wi, Wf, Wc, Wo = (blk(W, i) for i in range(4))
        Ui, Uf, Uc, Uo = (blk(U, i) for i in range(4))
        bi, bf, bc, bo = (blk(b, i) for i in range(4))
    else:                                          # keras 1: separate matrices
        Wi, Wf, Wc, Wo = (np.asarray(g("W_" + x)) for x in "ifco")
        Ui, Uf, Uc, Uo = (np.asarray(g("U_" + x)) for x in "ifco")
        bi, bf, bc, bo = (np.asarray(g("b_" + x)) for x in "ifco")
    # DL4J column blocks: [cell candidate (layer activation), forget, output, input gate] (KerasLstm.java:400)
    W = np.concatenate([Wc, Wf, Wo, Wi], axis=-1)
    U = np.concatenate([Uc, Uf, Uo, Ui], axis=-1)
    b = np.concatenate([bc, bf, bo, bi], axis=-1)
    return W, U, b


def _lstm_setter(prefix_keys=("",), dl4j_prefix=("",)):
    def s(p, kw):
        for kp, dp in zip(prefix_keys, dl4j_prefix):
            W, U, b = _lstm_arrays(kw, kp)
            _set(p, dp + "W", W)
            _set(p, dp + "RW", U)
            _set(p, dp + "b", b.reshape(1, -1))
    return s


def _simple_rnn_setter(p, kw):
    _set(p, "W", _w(kw, "kernel", "W"))
    _set(p, "RW", _w(kw, "recurrent_kernel", "U"))
    _set(p, "b", np.asarray(_w(kw, "bias", "b")).reshape(1, -1))


def _embedding_setter(p, kw):
    _set(p, "W", _w(kw, "embeddings", "W"))


# --------------------------------------------------------------------------------------- layer mappers
class _Ctx:
    def __init__(self, keras_major, training, backend=None):
        self.major = keras_major
        self.training = training
        self.backend = backend
        self.theano = backend == "theano"


# --------------------------------------------------------------------------------------- common layer fields
# Keras initializer names -> DL4J WeightInit (KER:utils/KerasInitilizationUtils.java:56-175); distributions below
_INIT = {"glorot_normal": "XAVIER", "glorot_uniform": "XAVIER_UNIFORM", "lecun_normal": "LECUN_NORMAL",
         "lecun_uniform": "LECUN_UNIFORM", "he_normal": "RELU", "he_uniform": "RELU_UNIFORM", "one": "ONES",
         "ones": "ONES", "zero": "ZERO", "zeros": "ZERO", "identity": "IDENTITY"}


def _init(spec, layer_cfg=None):
    """(WeightInit, Distribution or None) of a Keras 1 initializer name or a Keras 2 {class_name, config}; None when
    the layer config has none. Keras 1 keeps the initializer parameters (mean / stddev / scale / minval / maxval /
    value / gain) in the layer config itself (KER:utils/KerasInitilizationUtils.java getWeightInitFromConfig)."""
    from ..nn.conf import weights as Wt
    if spec is None:
        return None
    if isinstance(spec, dict):
        name, icfg = spec.get("class_name"), spec.get("config") or {}
    else:
        name, icfg = spec, dict(layer_cfg or {})
    key = {"RandomUniform": "random_uniform", "RandomNormal": "random_normal", "Ones": "ones", "Zeros": "zeros",
           "Constant": "constant", "Orthogonal": "orthogonal", "TruncatedNormal": "truncated_normal",
           "Identity": "identity", "GlorotNormal": "glorot_normal", "GlorotUniform": "glorot_uniform",
           "HeNormal": "he_normal", "HeUniform": "he_uniform", "LecunNormal": "lecun_normal",
           "LecunUniform": "lecun_uniform"}.get(name, name)
    if key in _INIT:
        return Wt.WeightInit[_INIT[key]], None
    if key in ("uniform", "random_uniform"):
        if "minval" in icfg:
            return Wt.WeightInit.DISTRIBUTION, Wt.UniformDistribution(float(icfg["minval"]), float(icfg["maxval"]))
        sc = float(icfg.get("scale", 0.05))
        return Wt.WeightInit.DISTRIBUTION, Wt.UniformDistribution(-sc, sc)
    if key in ("normal", "random_normal"):
        if "stddev" in icfg:
            return Wt.WeightInit.DISTRIBUTION, Wt.NormalDistribution(float(icfg.get("mean", 0.0)),
                                                                     float(icfg["stddev"]))
        return Wt.WeightInit.DISTRIBUTION, Wt.NormalDistribution(0.0, float(icfg.get("scale", 0.05)))
    if key == "constant":
        return Wt.WeightInit.DISTRIBUTION, Wt.ConstantDistribution(float(icfg.get("value", 0.0)))
    if key == "orthogonal":
        return Wt.WeightInit.DISTRIBUTION, Wt.OrthogonalDistribution(float(icfg.get("gain", icfg.get("scale", 1.0))))
    if key == "truncated_normal":
        return Wt.WeightInit.DISTRIBUTION, Wt.TruncatedNormalDistribution(float(icfg.get("mean", 0.0)),
                                                                          float(icfg.get("stddev", 0.05)))
    if key == "VarianceScaling":
        mode = {"fan_in": "FAN_IN", "fan_out": "FAN_OUT", "fan_avg": "FAN_AVG"}.get(icfg.get("mode"))
        if mode is None:
            raise InvalidKerasConfigurationException("VarianceScaling 'mode' must be fan_in, fan_out or fan_avg")
        dist = "NORMAL" if icfg.get("distribution", "normal") in ("normal", "truncated_normal") else "UNIFORM"
        return Wt.WeightInit[f"VAR_SCALING_{dist}_{mode}"], None
    raise UnsupportedKerasConfigurationException(f"Unsupported Keras weight initializer {name!r}")


def _reg(cfg, *fields):
    """(l1, l2) of the first present regularizer field: {l1, l2} or {class_name: L1L2, config: {l1, l2}}
    (KER:utils/KerasRegularizerUtils.java:20-60)."""
    for f in fields:
        r = cfg.get(f)
        if isinstance(r, dict):
            inner = r.get("config") if r.get("class_name") == "L1L2" else r
            inner = inner or {}
            return float(inner.get("l1", 0.0) or 0.0), float(inner.get("l2", 0.0) or 0.0)
    return 0.0, 0.0


def _apply_common(k, ctx):
    """The fields every DL4J layer built from Keras gets (KER:KerasLayer.java, KerasLayerUtils): the layer name,
    weight initialisation, L1 / L2 weight and bias regularisation, the generic ``dropout`` fraction (retain
    probability 1 - p), and for LSTMs the recurrent initialisation and the forget-gate bias."""
    cfg, obj = k.cfg or {}, k.obj
    if k.kind not in ("layer", "timedistributed") or not isinstance(obj, L.Layer):
        return k
    from ..nn.conf.regularization import Dropout
    target = obj
    while isinstance(target, (L.LastTimeStep,)) and getattr(target, "underlying", None) is not None:
        target = target.underlying
    for o in {id(obj): obj, id(target): target}.values():
        if k.name is not None and "layerName" in o._all_fields():
            o.layerName = k.name
    fields = target._all_fields()
    emb = k.keras_class == "Embedding"
    init = _init(cfg.get("embeddings_initializer") if emb and "embeddings_initializer" in cfg else
                 cfg.get("kernel_initializer", cfg.get("init", cfg.get("depthwise_initializer"))), cfg)
    if init is not None and "weightInit" in fields:
        target.weightInit, dist = init
        if dist is not None:
            target.dist = dist
    if "weightInitRecurrent" in fields:
        rinit = _init(cfg.get("recurrent_initializer", cfg.get("inner_init")))
        if rinit is not None:
            target.weightInitRecurrent = rinit[0]
            if rinit[1] is not None:
                target.distRecurrent = rinit[1]
    if "l1" in fields:
        l1, l2 = _reg(cfg, "embeddings_regularizer", "kernel_regularizer", "W_regularizer") if emb else \
            _reg(cfg, "kernel_regularizer", "W_regularizer", "depthwise_regularizer")
        if l1:
            target.l1 = l1
        if l2:
            target.l2 = l2
        b1, b2 = _reg(cfg, "bias_regularizer", "b_regularizer")
        if b1:
            target.l1Bias = b1
        if b2:
            target.l2Bias = b2
    p = cfg.get("dropout", cfg.get("dropout_W"))
    if isinstance(p, (int, float)) and not isinstance(p, bool) and p > 0 and "idropout" in fields and \
            k.keras_class not in ("Dropout", "SpatialDropout1D", "SpatialDropout2D", "AlphaDropout",
                                  "GaussianDropout", "GaussianNoise"):
        target.idropout = Dropout(1.0 - float(p))
    if "forgetGateBiasInit" in fields:
        if "unit_forget_bias" in cfg:
            target.forgetGateBiasInit = 1.0 if cfg["unit_forget_bias"] else 0.0
        elif "forget_bias_init" in cfg:
            fb = cfg["forget_bias_init"]
            if isinstance(fb, str):
                if fb not in ("one", "ones", "zero", "zeros"):
                    raise UnsupportedKerasConfigurationException(f"LSTM forget_bias_init {fb!r}")
                target.forgetGateBiasInit = 1.0 if fb.startswith("one") else 0.0
            else:
                target.forgetGateBiasInit = float(fb)
    return k


def _map_layer(kl, ctx):
    return _apply_common(_map_layer_core(kl, ctx), ctx)


def _masks_zero(k):
    return k is not None and k.keras_class == "Embedding" and bool((k.cfg or {}).get("mask_zero", False))


def _mask_zero_wrap(m):
    """A recurrent layer fed by a mask_zero Embedding: MaskZeroLayer(layer) (inside the LastTimeStep wrapper when
    return_sequences is false), as KER:layers/recurrent/KerasLstm.java / KerasSimpleRnn.java."""
    if m.keras_class not in ("LSTM", "SimpleRNN", "Bidirectional"):
        return m
    if isinstance(m.obj, L.LastTimeStep):
        m.obj.underlying = L.MaskZeroLayer(underlying=m.obj.underlying, maskingValue=0.0)
    else:
        m.obj = L.MaskZeroLayer(underlying=m.obj, maskingValue=0.0)
    return m


def _map_layer_core(kl, ctx):
    cls = kl["class_name"]
    cfg = kl.get("config", {}) or {}
    name = cfg.get("name") or kl.get("name")
    if cls in _CUSTOM:
        kind, obj, setter = _CUSTOM[cls](cfg, ctx)
        return _KLayer(name, kind, obj, setter=setter, keras_class=cls, cfg=cfg)
    k1 = ctx.major == 1
    act = lambda: _act(cfg.get("activation", "linear"))  # noqa: E731
    if cls == "InputLayer":
        return _KLayer(name, "input", keras_class=cls, cfg=cfg)
    if cls in ("Dense", "TimeDistributedDense"):
        # Keras 1's TimeDistributedDense maps to the same DL4J DenseLayer (KER:utils/KerasLayerUtils.java:199-201);
        # on a recurrent input the layer gets the usual RnnToFeedForward preprocessor
        units = cfg.get("units", cfg.get("output_dim"))
        hb = cfg.get("use_bias", cfg.get("bias", True))
        lay = L.DenseLayer(nOut=int(units), activation=act(), hasBias=bool(hb)) if "hasBias" in \
            L.DenseLayer._all_fields() else L.DenseLayer(nOut=int(units), activation=act())
        return _KLayer(name, "layer", lay, setter=_dense_setter(hb), keras_class=cls, cfg=cfg)
    if cls == "Activation":
        return _KLayer(name, "layer", L.ActivationLayer(activation=act()), keras_class=cls, cfg=cfg)
    if cls == "LeakyReLU":
        from ..nn.conf.activations import ActivationLReLU
        return _KLayer(name, "layer", L.ActivationLayer(activation=ActivationLReLU(alpha=float(cfg.get("alpha", 0.3)))),
                       keras_class=cls, cfg=cfg)
    if cls in ("Dropout", "SpatialDropout1D", "SpatialDropout2D"):
        rate = float(cfg.get("rate", cfg.get("p", 0.0)))
        from ..nn.conf.regularization import Dropout
        return _KLayer(name, "layer", L.DropoutLayer(idropout=Dropout(1.0 - rate)), keras_class=cls, cfg=cfg)
    if cls in ("AlphaDropout", "GaussianDropout", "GaussianNoise"):
        from ..nn.conf import regularization as R
        if cls == "AlphaDropout":
            d = R.AlphaDropout(1.0 - float(cfg.get("rate", cfg.get("p", 0.0))))
        elif cls == "GaussianDropout":
            d = R.GaussianDropout(float(cfg.get("rate", cfg.get("p", 0.0))))
        else:
            d = R.GaussianNoise(float(cfg.get("stddev", cfg.get("sigma", 0.0))))
        return _KLayer(name, "layer", L.DropoutLayer(idropout=d), keras_class=cls, cfg=cfg)
    if cls == "Flatten":
        return _KLayer(name, "flatten", keras_class=cls, cfg=cfg)
    if cls == "Reshape":
        return _KLayer(name, "reshape", keras_class=cls, cfg=cfg)
    if cls in ("Conv2D", "Convolution2D", "AtrousConvolution2D", "Conv2DTranspose", "Deconvolution2D",
               "SeparableConv2D", "SeparableConvolution2D"):
        filt = int(cfg.get("filters", cfg.get("nb_filter")))
        ks = cfg.get("kernel_size") or [cfg.get("nb_row"), cfg.get("nb_col")]
        st = cfg.get("strides", cfg.get("subsample", [1, 1]))
        dil = cfg.get("dilation_rate", cfg.get("atrous_rate", [1, 1]))
        hb = cfg.get("use_bias", cfg.get("bias", True))
        cl = _channels_last(cfg)
        common = dict(nOut=filt, kernelSize=_pair(ks), stride=_pair(st), dilation=_pair(dil),
                      convolutionMode=_mode(cfg.get("padding", cfg.get("border_mode"))), activation=act(),
                      hasBias=bool(hb))
        if cls in ("Conv2DTranspose", "Deconvolution2D"):
            lay = L.Deconvolution2D(**common)

            def setter(p, kw, hb=hb, cl=cl):
                k = np.asarray(_w(kw, "kernel", "W"))          # TF [kh, kw, out, in]
                w = np.transpose(k, (3, 2, 0, 1)) if cl else k
                _set(p, "W", w)
                if hb:
                    _set(p, "b", _w(kw, "bias", "b").reshape(1, -1))
            return _KLayer(name, "layer", lay, setter=setter, keras_class=cls, cfg=cfg)
        if cls in ("SeparableConv2D", "SeparableConvolution2D"):
            dm = int(cfg.get("depth_multiplier", 1))
            lay = L.SeparableConvolution2D(depthMultiplier=dm, **common)

            def setter(p, kw, hb=hb):
                dk = np.asarray(_w(kw, "depthwise_kernel"))    # [kh, kw, in, dm]
                pk = np.asarray(_w(kw, "pointwise_kernel"))    # [1, 1, in*dm, out]
                _set(p, "W", np.transpose(dk, (3, 2, 0, 1)))
                _set(p, "pW", np.transpose(pk, (3, 2, 0, 1)))
                if hb:
                    _set(p, "b", _w(kw, "bias", "b").reshape(1, -1))
            return _KLayer(name, "layer", lay, setter=setter, keras_class=cls, cfg=cfg)
        lay = L.ConvolutionLayer(**common)
        return _KLayer(name, "layer", lay, setter=_conv_setter(hb, ctx.major >= 2 or cl, ctx.theano),
                       keras_class=cls, cfg=cfg)
    if cls in ("Conv1D", "Convolution1D", "AtrousConvolution1D"):
        filt = int(cfg.get("filters", cfg.get("nb_filter")))
        ks = cfg.get("kernel_size", cfg.get("filter_length"))
        ks = ks[0] if isinstance(ks, (list, tuple)) else ks
        st = cfg.get("strides", cfg.get("subsample_length", 1))
        st = st[0] if isinstance(st, (list, tuple)) else st
        dil = cfg.get("dilation_rate", cfg.get("atrous_rate", 1))
        dil = dil[0] if isinstance(dil, (list, tuple)) else dil
        hb = cfg.get("use_bias", cfg.get("bias", True))
        lay = L.Convolution1DLayer(nOut=filt, kernelSize=[int(ks), 1], stride=[int(st), 1], dilation=[int(dil), 1],
                                   convolutionMode=_mode(cfg.get("padding", cfg.get("border_mode"))),
                                   activation=act(), hasBias=bool(hb))
        return _KLayer(name, "layer", lay, setter=_conv_setter(hb, True, ctx.theano, conv1d=True), keras_class=cls, cfg=cfg)
    if cls in ("MaxPooling2D", "AveragePooling2D", "MaxPooling1D", "AveragePooling1D"):
        one_d = cls.endswith("1D")
        pt = PoolingType.MAX if cls.startswith("Max") else PoolingType.AVG
        if one_d:
            ps = cfg.get("pool_size", cfg.get("pool_length", 2))
            ps = ps[0] if isinstance(ps, (list, tuple)) else ps
            st = cfg.get("strides", cfg.get("stride", None)) or ps
            st = st[0] if isinstance(st, (list, tuple)) else st
            lay = L.Subsampling1DLayer(poolingType=pt, kernelSize=[int(ps), 1], stride=[int(st), 1],
                                       convolutionMode=_mode(cfg.get("padding", cfg.get("border_mode"))))
        else:
            ps = _pair(cfg.get("pool_size", [2, 2]))
            st = _pair(cfg.get("strides") or ps)
            lay = L.SubsamplingLayer(poolingType=pt, kernelSize=ps, stride=st,
                                     convolutionMode=_mode(cfg.get("padding", cfg.get("border_mode"))))
        return _KLayer(name, "layer", lay, keras_class=cls, cfg=cfg)
    if cls in ("GlobalMaxPooling1D", "GlobalAveragePooling1D", "GlobalMaxPooling2D", "GlobalAveragePooling2D"):
        pt = PoolingType.MAX if "Max" in cls else PoolingType.AVG
        return _KLayer(name, "layer", L.GlobalPoolingLayer(poolingType=pt), keras_class=cls, cfg=cfg)
    if cls == "BatchNormalization":
        eps = float(cfg.get("epsilon", 1e-3))
        if cfg.get("mode", 0) not in (0, None):
            raise UnsupportedKerasConfigurationException("BatchNormalization mode != 0")
        center, scale = cfg.get("center", True), cfg.get("scale", True)
        lay = L.BatchNormalization(eps=eps, decay=float(cfg.get("momentum", 0.99)),
                                   lockGammaBeta=not (center and scale))
        return _KLayer(name, "layer", lay, setter=_bn_setter(eps, center, scale), keras_class=cls, cfg=cfg)
    if cls in ("LSTM", "SimpleRNN"):
        units = int(cfg.get("units", cfg.get("output_dim")))
        gate = _act(cfg.get("recurrent_activation", cfg.get("inner_activation", "hard_sigmoid")))
        if cls == "LSTM":
            lay = L.LSTM(nOut=units, activation=act() if "activation" in cfg else Activation.TANH,
                         gateActivationFn=gate.getActivationFunction())
            setter = _lstm_setter()
        else:
            lay = L.SimpleRnn(nOut=units, activation=act() if "activation" in cfg else Activation.TANH)
            setter = _simple_rnn_setter
        if not cfg.get("return_sequences", False):
            lay = L.LastTimeStep(underlying=lay)
            inner = setter
            setter = inner
        if cfg.get("go_backwards", False):
            raise UnsupportedKerasConfigurationException("go_backwards recurrent layers")
        return _KLayer(name, "layer", lay, setter=setter, keras_class=cls, cfg=cfg)
    if cls == "Bidirectional":
        inner = cfg["layer"]
        icfg = inner["config"]
        sub = _map_layer(inner, ctx)
        base = sub.obj.underlying if isinstance(sub.obj, L.LastTimeStep) else sub.obj
        mode = {"concat": "CONCAT", "sum": "ADD", "mul": "MUL", "ave": "AVERAGE"}[cfg.get("merge_mode", "concat")]
        lay = L.Bidirectional(mode=mode, underlying=base)
        if not icfg.get("return_sequences", False):
            lay = L.LastTimeStep(underlying=lay)
        iname = icfg.get("name", "")

        def setter(p, kw, iname=iname, icls=inner["class_name"]):
            for d, direction in (("f", "forward"), ("b", "backward")):
                pre = f"{direction}_{iname}"
                sk = {k[len(pre) + 1:]: v for k, v in kw.items() if k.startswith(pre + "/") or
                      k.startswith(pre + "_")}
                if icls == "LSTM":
                    W, U, bb = _lstm_arrays(sk)
                else:
                    W, U = _w(sk, "kernel", "W"), _w(sk, "recurrent_kernel", "U")
                    bb = np.asarray(_w(sk, "bias", "b"))
                _set(p, d + "W", W)
                _set(p, d + "RW", U)
                _set(p, d + "b", np.asarray(bb).reshape(1, -1))
        return _KLayer(name, "layer", lay, setter=setter, keras_class=cls, cfg=cfg)
    if cls == "Embedding":
        # input_length null = variable-length sequences: recurrent output type with unknown length (-1)
        il = cfg.get("input_length")
        il = il[0] if isinstance(il, (list, tuple)) else il
        lay = L.EmbeddingSequenceLayer(nIn=int(cfg["input_dim"]), nOut=int(cfg["output_dim"]),
                                       inputLength=int(il) if il is not None else -1, hasBias=False,
                                       activation=Activation.IDENTITY)
        setter = _embedding_setter
        if cfg.get("mask_zero", False):
            # index 0 is Keras' padding token: its embedding row is zero, and the next recurrent layer masks the
            # all-zero time steps (KER:layers/embeddings/KerasEmbedding.java setWeights / hasZeroMasking)
            def setter(p, kw):
                _embedding_setter(p, kw)
                with torch.no_grad():
                    p["W"][0].zero_()
        return _KLayer(name, "layer", lay, setter=setter, keras_class=cls, cfg=cfg)
    if cls == "ZeroPadding2D":
        pd = cfg.get("padding", [1, 1])
        if isinstance(pd, int):
            pd = [pd, pd, pd, pd]
        elif len(pd) == 2 and not isinstance(pd[0], (list, tuple)):
            pd = [pd[0], pd[0], pd[1], pd[1]]
        else:
            pd = [pd[0][0], pd[0][1], pd[1][0], pd[1][1]]
        return _KLayer(name, "layer", L.ZeroPaddingLayer(padding=[int(v) for v in pd]), keras_class=cls, cfg=cfg)
    if cls == "ZeroPadding1D":
        pd = cfg.get("padding", 1)
        pd = [pd, pd] if isinstance(pd, int) else list(pd)
        return _KLayer(name, "layer", L.ZeroPadding1DLayer(padding=[int(v) for v in pd]), keras_class=cls, cfg=cfg)
    if cls == "Cropping2D":
        c = cfg.get("cropping", [[0, 0], [0, 0]])
        c = [c, c, c, c] if isinstance(c, int) else ([c[0], c[0], c[1], c[1]] if not isinstance(c[0], (list, tuple))
                                                     else [c[0][0], c[0][1], c[1][0], c[1][1]])
        return _KLayer(name, "layer", L.Cropping2D(cropping=[int(v) for v in c]), keras_class=cls, cfg=cfg)
    if cls in ("UpSampling2D", "UpSampling1D"):
        if cls.endswith("2D"):
            return _KLayer(name, "layer", L.Upsampling2D(size=_pair(cfg.get("size", [2, 2]))), keras_class=cls,
                           cfg=cfg)
        sz = cfg.get("size", cfg.get("length", 2))
        return _KLayer(name, "layer", L.Upsampling1D(size=[int(sz)]), keras_class=cls, cfg=cfg)
    if cls == "LRN":
        return _KLayer(name, "layer", L.LocalResponseNormalization(alpha=float(cfg.get("alpha", 1e-4)),
                                                                   beta=float(cfg.get("beta", 0.75)),
                                                                   k=float(cfg.get("k", 2.0)),
                                                                   n=float(cfg.get("n", 5))), keras_class=cls, cfg=cfg)
    if cls in ("Merge", "Add", "Subtract", "Multiply", "Average", "Maximum", "Concatenate"):
        mode = cfg.get("mode", cls.lower()) if cls == "Merge" else cls.lower()
        if mode in ("concat", "concatenate"):
            v = G.MergeVertex()
        else:
            op = {"sum": "Add", "add": "Add", "subtract": "Subtract", "mul": "Product", "multiply": "Product",
                  "ave": "Average", "average": "Average", "max": "Max", "maximum": "Max"}.get(mode)
            if op is None:
                raise UnsupportedKerasConfigurationException(f"Merge mode {mode!r}")
            v = G.ElementWiseVertex(op=op)
        return _KLayer(name, "vertex", v, keras_class=cls, cfg=cfg)
    if cls == "TimeDistributed":
        inner = _map_layer(cfg["layer"], ctx)
        if not isinstance(inner.obj, L.DenseLayer):
            raise UnsupportedKerasConfigurationException("TimeDistributed supports Dense only")
        inner.name = name
        inner.kind = "timedistributed"
        return inner
    if cls == "Lambda":
        raise UnsupportedKerasConfigurationException(
            f"Lambda layer {name!r}: register a mapper with KerasLayer.registerCustomLayer('Lambda', ...); "
            "the serialized Python function is never executed")
    raise UnsupportedKerasConfigurationException(f"Unsupported Keras layer type {cls!r}")


# --------------------------------------------------------------------------------------- input types
def _input_type(shape, channels_last=True):
    dims = [d for d in shape[1:]]
    if len(dims) == 1:
        if dims[0] is None:                  # [mb, null]: variable-length index sequence
            return InputType.recurrent(1, -1)
        return InputType.feedForward(int(dims[0]))
    if len(dims) == 2:
        T = dims[0] if dims[0] is not None else -1
        return InputType.recurrent(int(dims[1]), int(T))
    if len(dims) == 3:
        if channels_last:
            return InputType.convolutional(int(dims[0]), int(dims[1]), int(dims[2]))
        return InputType.convolutional(int(dims[1]), int(dims[2]), int(dims[0]))
    raise UnsupportedKerasConfigurationException(f"input shape {shape}")


def _flatten_pp(t, channels_last):
    if isinstance(t, InputTypeConvolutional):
        cls = TensorFlowCnnToFeedForwardPreProcessor if channels_last else PP.CnnToFeedForwardPreProcessor
        return cls(inputHeight=t.height, inputWidth=t.width, numChannels=t.channels)
    if isinstance(t, InputTypeRecurrent):
        return KerasReshapePreprocessor(targetShape=[t.size * max(t.timeSeriesLength, 1)], channelsLast=True)
    return None


# --------------------------------------------------------------------------------------- model
class KerasModel:
    def __init__(self, model_config, weights_root=None, training_config=None, keras_version="2", enforce=False,
                 backend=None):
        self.cfg = json.loads(model_config) if isinstance(model_config, str) else model_config
        self.weights_root = weights_root
        self.training_config = json.loads(training_config) if isinstance(training_config, str) else training_config
        self.major = int(str(keras_version or "2")[0]) if str(keras_version or "2")[0].isdigit() else 2
        self.enforce = enforce
        if backend is None:
            backend = self.cfg.get("backend") if isinstance(self.cfg, dict) else None
        self.ctx = _Ctx(self.major, enforce, backend)

    def isSequential(self):
        return self.cfg["class_name"] == "Sequential"

    def _layer_list(self):
        c = self.cfg["config"]
        return c["layers"] if isinstance(c, dict) else c

    # ------------------------------------------------------------------ weights
    def _weights_for(self, lname):
        """Keras weight arrays of one layer keyed by their parameter name ('kernel', 'W', 'W_i', ...).

        Weight names carry optional TensorFlow name scopes in front of the layer name and the layer name itself
        may contain '/' ('global/shared/dense_1/xxx/yyy_W:0' for layer 'dense_1/xxx/yyy'): the parameter name is
        what follows the LAST occurrence of '<layer>_' or '<layer>/' (KER:utils/KerasModelUtils.java:170-300)."""
        if self.weights_root is None:
            return None
        root = self.weights_root
        if "model_weights" in root:
            root = root["model_weights"]
        try:
            grp = root[lname]
        except (KeyError, Exception):
            return {}
        names = grp.attrs.get("weight_names")
        out = {}
        if names is None:
            names = []
            grp.visit(lambda p, n: names.append(p) if isinstance(n, hdf5.Dataset) else None)
        for full in list(names):
            full = full.decode() if isinstance(full, bytes) else str(full)
            ds = grp[full]
            stem = full.split(":")[0]
            key = None
            for sep in ("_", "/"):
                i = stem.rfind(lname + sep)
                if i >= 0 and (i == 0 or stem[i - 1] == "/"):
                    key = stem[i + len(lname) + 1:]
                    break
            if key is None:
                short = stem.split("/")
                key = short[-1]
                if len(short) >= 3:        # bidirectional: layer/forward_lstm_1/kernel:0
                    key = short[-2] + "/" + key
            out[key] = ds.read()
        return out

    # ------------------------------------------------------------------ sequential
    def getMultiLayerConfiguration(self):
        return self._sequential()[0]

    def _sequential(self):
        from ..nn.conf.network import NeuralNetConfiguration
        layers = self._layer_list()
        first = layers[0]["config"]
        shape = first.get("batch_input_shape")
        if shape is None and "input_dim" in first:
            shape = [None, first["input_dim"]]
        if shape is None:
            raise InvalidKerasConfigurationException("first layer has no batch_input_shape")
        cl = _channels_last(first, True)
        mapped = []
        for kl in layers:
            if kl["class_name"] == "InputLayer":
                shape = kl["config"]["batch_input_shape"]
                continue
            m = _map_layer(kl, self.ctx)
            mapped.append(_mask_zero_wrap(m) if mapped and _masks_zero(mapped[-1]) else m)
        if mapped and mapped[0].keras_class == "Embedding":
            # index input [mb, T]: T may be null (variable length)
            T = shape[1] if len(shape) > 1 else None
            t = InputType.recurrent(1, int(T) if T is not None else -1)
        else:
            t = _input_type(shape, cl)
        b = NeuralNetConfiguration.Builder().weightInit("XAVIER").list()
        idx = 0
        pending = None
        cur = t
        setters = []
        for m in mapped:
            if m.kind == "flatten":
                pending = _flatten_pp(cur, _channels_last(m.cfg, cl))
                if pending is not None:
                    cur = pending.getOutputType(cur)
                continue
            if m.kind == "reshape":
                pending = KerasReshapePreprocessor(targetShape=list(m.cfg["target_shape"]), channelsLast=cl)
                cur = pending.getOutputType(cur)
                continue
            if m.kind == "skip":
                continue
            if m.kind == "vertex":
                raise UnsupportedKerasConfigurationException(f"{m.keras_class} in a Sequential model")
            if m.kind == "timedistributed":
                m.obj = L.RnnOutputLayer(lossFn=None, nOut=m.obj.nOut, activation=m.obj.activation) \
                    if False else m.obj
            b.layer(idx, m.obj)
            if pending is not None:
                b.inputPreProcessor(idx, pending)
                pending = None
            lay = m.obj
            try:
                cur = lay.getOutputType(idx, cur if not hasattr(lay, "getPreProcessorForInputType") or
                                        lay.getPreProcessorForInputType(cur) is None
                                        else lay.getPreProcessorForInputType(cur).getOutputType(cur))
            except Exception:
                pass
            setters.append((idx, m))
            idx += 1
        loss = self._loss()
        if loss is not None and idx > 0:
            b.layer(idx, _loss_layer(loss, cur))
        b.setInputType(t)
        return b.build(), setters

    def getMultiLayerNetwork(self, importWeights=True, device=None):
        from ..nn.multilayer import MultiLayerNetwork
        conf, setters = self._sequential()
        net = MultiLayerNetwork(conf)
        net.init(device=device)
        if importWeights and self.weights_root is not None:
            for idx, m in setters:
                if m.setter is None:
                    continue
                kw = self._weights_for(m.name)
                if kw:
                    m.setter(net.layers[idx].params, kw)
            net._params_changed()
        return net

    def _loss(self):
        tc = self.training_config
        if not tc:
            return None
        loss = tc.get("loss")
        if isinstance(loss, dict):
            loss = list(loss.values())[0]
        if not isinstance(loss, str):
            return None
        from ..nn.conf.losses import LossFunction
        name = _LOSS.get(loss.lower())
        if name is None:
            if self.enforce:
                raise UnsupportedKerasConfigurationException(f"Keras loss {loss!r}")
            return None
        if name == "SPARSE_MCXENT":
            name = "MCXENT"
        return LossFunction[name]

    # ------------------------------------------------------------------ functional
    def getComputationGraphConfiguration(self):
        return self._functional()[0]

    def _functional(self):
        from ..nn.conf.network import NeuralNetConfiguration
        c = self.cfg["config"]
        if self.isSequential():
            layers = self._layer_list()
            # a Sequential model as a chain graph
            ins = [("input", layers[0]["config"].get("batch_input_shape"))]
            c = {"layers": [], "input_layers": [["input", 0, 0]], "output_layers": [[layers[-1]["config"]["name"],
                                                                                       0, 0]]}
            prev = "input"
            c["layers"].append({"name": "input", "class_name": "InputLayer",
                                "config": {"batch_input_shape": ins[0][1]}, "inbound_nodes": []})
            for kl in layers:
                nm = kl["config"]["name"]
                c["layers"].append({"name": nm, "class_name": kl["class_name"], "config": kl["config"],
                                    "inbound_nodes": [[[prev, 0, 0, {}]]]})
                prev = nm
        gb = NeuralNetConfiguration.Builder().weightInit("XAVIER").graphBuilder()
        types = {}
        inputs = [il[0] for il in c["input_layers"]]
        cl_of = {}
        for kl in c["layers"]:
            if kl["class_name"] == "InputLayer":
                cfg = kl["config"]
                cl = _channels_last(cfg, True)
                types[kl["name"]] = _input_type(cfg["batch_input_shape"], cl)
                cl_of[kl["name"]] = cl
        gb.addInputs(*inputs)
        gb.setInputTypes(*[types[n] for n in inputs])
        setters = []
        rename = {}
        by_name = {}
        for kl in c["layers"]:
            if kl["class_name"] == "InputLayer":
                continue
            name = kl.get("name") or kl["config"]["name"]
            nodes = kl.get("inbound_nodes") or []
            inb = [rename.get(x[0], x[0]) for x in (nodes[0] if nodes else [])]
            m = _map_layer(kl, self.ctx)
            by_name[name] = m
            if len(inb) == 1 and _masks_zero(by_name.get(inb[0])):
                _mask_zero_wrap(m)
            cl = cl_of.get(inb[0], True) if inb else True
            cl = _channels_last(kl.get("config", {}), cl)
            if m.kind == "skip":
                rename[name] = inb[0]
                continue
            if m.kind == "flatten":
                gb.addVertex(name, G.PreprocessorVertex(preProcessor=_flatten_pp(types.get(inb[0]), cl) or
                                                        PP.CnnToFeedForwardPreProcessor()), *inb)
            elif m.kind == "reshape":
                gb.addVertex(name, G.PreprocessorVertex(preProcessor=KerasReshapePreprocessor(
                    targetShape=list(m.cfg["target_shape"]), channelsLast=cl)), *inb)
            elif m.kind == "vertex":
                gb.addVertex(name, m.obj, *inb)
            else:
                gb.addLayer(name, m.obj, *inb)
                setters.append((name, m))
            cl_of[name] = cl
            try:
                v = gb._vertices[name]
                its = [types[i] for i in inb]
                types[name] = v.getOutputType(0, *its)
            except Exception:
                pass
        outs = [rename.get(o[0], o[0]) for o in c["output_layers"]]
        loss = self._loss()
        if loss is not None:
            new_outs = []
            for o in outs:
                ln = o + "_loss"
                gb.addLayer(ln, _loss_layer(loss, types.get(o)), o)
                new_outs.append(ln)
            outs = new_outs
        gb.setOutputs(*outs)
        return gb.build(), setters

    def getComputationGraph(self, importWeights=True, device=None):
        from ..nn.graph.computation_graph import ComputationGraph
        conf, setters = self._functional()
        net = ComputationGraph(conf)
        net.init(device=device)
        if importWeights and self.weights_root is not None:
            for name, m in setters:
                if m.setter is None:
                    continue
                kw = self._weights_for(name)
                if kw:
                    m.setter(net.layers_by_name[name].params, kw)
            net._params_changed()
        return net


def _loss_layer(loss, in_type):
    """Keras training loss -> DL4J loss layer matching the output's rank (the reference always uses a plain
    LossLayer, which would flatten conv/recurrent outputs; KerasLoss.java:70)."""
    if isinstance(in_type, InputTypeConvolutional):
        return L.CnnLossLayer(lossFn=loss, activation=Activation.IDENTITY)
    if isinstance(in_type, InputTypeRecurrent):
        return L.RnnLossLayer(lossFn=loss, activation=Activation.IDENTITY)
    return L.LossLayer(lossFn=loss, activation=Activation.IDENTITY)


def _read_h5(path):
    f = hdf5.File(path)
    a = f.attrs
    mc = a.get("model_config")
    if mc is None:
        raise InvalidKerasConfigurationException("HDF5 file has no model_config attribute")
    kv = a.get("keras_version", "1")
    if isinstance(kv, bytes):
        kv = kv.decode()
    return f, mc, a.get("training_config"), str(kv), a.get("backend")


class KerasModelImport:
    """Entry points mirroring KER:KerasModelImport.java."""

    @staticmethod
    def importKerasModelAndWeights(modelHdf5OrJson, weightsHdf5=None, enforceTrainingConfig=False, device=None):
        km = KerasModelImport._model(modelHdf5OrJson, weightsHdf5, enforceTrainingConfig)
        if km.isSequential():
            return km.getMultiLayerNetwork(True, device)
        return km.getComputationGraph(True, device)

    @staticmethod
    def importKerasSequentialModelAndWeights(modelHdf5OrJson, weightsHdf5=None, enforceTrainingConfig=False,
                                             device=None):
        km = KerasModelImport._model(modelHdf5OrJson, weightsHdf5, enforceTrainingConfig)
        if not km.isSequential():
            raise InvalidKerasConfigurationException("Model is not a Sequential model; use importKerasModelAndWeights")
        return km.getMultiLayerNetwork(True, device)

    @staticmethod
    def importKerasModelConfiguration(jsonOrPath, enforceTrainingConfig=False):
        cfg = _load_json(jsonOrPath)
        km = KerasModel(cfg, keras_version=cfg.get("keras_version", "2"), enforce=enforceTrainingConfig)
        return km.getComputationGraphConfiguration()

    @staticmethod
    def importKerasSequentialConfiguration(jsonOrPath, enforceTrainingConfig=False):
        cfg = _load_json(jsonOrPath)
        km = KerasModel(cfg, keras_version=cfg.get("keras_version", "2"), enforce=enforceTrainingConfig)
        return km.getMultiLayerConfiguration()

    @staticmethod
    def _model(modelHdf5OrJson, weightsHdf5, enforce):
        # JSON or HDF5 by content, not by extension ('model.json.with.tensorflow.scope' is JSON)
        if isinstance(modelHdf5OrJson, dict) or _is_json(modelHdf5OrJson):
            cfg = _load_json(modelHdf5OrJson)
            w = hdf5.File(weightsHdf5) if weightsHdf5 else None
            kv = cfg.get("keras_version", "2") if isinstance(cfg, dict) else "2"
            return KerasModel(cfg, w, None, kv, enforce)
        f, mc, tc, kv, backend = _read_h5(modelHdf5OrJson)
        w = hdf5.File(weightsHdf5) if weightsHdf5 else f
        return KerasModel(mc, w, tc, kv, enforce, backend)


def _is_json(x):
    s = str(x)
    if s.lstrip().startswith("{"):
        return True
    try:
        with open(s, "rb") as fh:
            head = fh.read(64).lstrip()
    except OSError:
        return s.endswith(".json")
    return head.startswith(b"{")


def _load_json(x):
    if isinstance(x, dict):
        return x
    s = str(x)
    if s.lstrip().startswith("{"):
        return json.loads(s)
    with open(s) as fh:
        return json.load(fh)


_ = (copy, Config)
