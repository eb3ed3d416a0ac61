"""DL4J's own JSON configuration format (Jackson), so ``configuration.json`` inside a ModelSerializer ZIP is read and
written exactly as the reference does.

Reference schema:
  * MultiLayerConfiguration (NN:nn/conf/MultiLayerConfiguration.java:120-200): ``{"confs": [NeuralNetConfiguration..],
    "inputPreProcessors": {"<index>": preprocessor}, "backprop", "backpropType", "tbpttFwdLength", ...}``.
  * NeuralNetConfiguration (NN:nn/conf/NeuralNetConfiguration.java:94): one per layer, the layer under ``"layer"``
    plus the network-wide fields (seed, optimizationAlgo, miniBatch, minimize, stepFunction, cacheMode, ...).
  * Layer (NN:nn/conf/layers/Layer.java:54-90): ``@JsonTypeInfo(use=NAME, include=WRAPPER_OBJECT)`` —
    ``{"dense": {...}}``, ``{"convolution": {...}}``, ``{"gravesLSTM": {...}}``; bean property names
    (``activationFn``, ``nin``, ``nout``, ``iupdater``, ``idropout``, ...).
  * IActivation / ILossFunction: wrapper objects named by the ND4J class minus its prefix (``{"ReLU": {}}``,
    ``{"MCXENT": {"softmaxClipEps": 1e-10}}``); IUpdater / ISchedule / IDropout / IWeightNoise / LayerConstraint:
    ``{"@class": "<fully qualified name>", ...}``; Distribution: ``{"type": "<fqn>", ...}``; GraphVertex and
    InputPreProcessor: wrapper objects (``{"LayerVertex": {"layerConf": ..}}``, ``{"cnnToFeedForward": {..}}``).
  * ComputationGraphConfiguration: ``{"vertices": {...}, "vertexInputs", "networkInputs", "networkOutputs",
    "defaultConfiguration", ...}``.
Reading also accepts the pre-1.0 layer fields (``updater`` enum + ``learningRate``/``momentum``/...,
``lossFunction`` enum, ``dropOut``) the reference's legacy deserializers handle
(NN:nn/conf/MultiLayerConfiguration.java:138-200, NN:nn/conf/serde/*Deserializer.java).
Fields of this framework's configs that DL4J does not have are written too (Jackson readers ignore unknown
properties), so a round trip through this format is lossless; the extension block ``"dl4jAmd"`` carries the input
types and global settings.
"""
import enum
import json
import math

from .base import Config, _REGISTRY, lookup

LAYER_NAMES = {
    "AutoEncoder": "autoEncoder", "ConvolutionLayer": "convolution", "Convolution1DLayer": "convolution1d",
    "GravesLSTM": "gravesLSTM", "LSTM": "LSTM", "GravesBidirectionalLSTM": "gravesBidirectionalLSTM",
    "OutputLayer": "output", "CenterLossOutputLayer": "CenterLossOutputLayer", "RnnOutputLayer": "rnnoutput",
    "LossLayer": "loss", "DenseLayer": "dense", "SubsamplingLayer": "subsampling",
    "Subsampling1DLayer": "subsampling1d", "BatchNormalization": "batchNormalization",
    "LocalResponseNormalization": "localResponseNormalization", "EmbeddingLayer": "embedding",
    "ActivationLayer": "activation", "VariationalAutoencoder": "VariationalAutoencoder", "DropoutLayer": "dropout",
    "GlobalPoolingLayer": "GlobalPooling", "ZeroPaddingLayer": "zeroPadding", "ZeroPadding1DLayer": "zeroPadding1d",
    "FrozenLayer": "FrozenLayer", "Upsampling2D": "Upsampling2D", "Yolo2OutputLayer": "Yolo2OutputLayer",
    "RnnLossLayer": "RnnLossLayer", "CnnLossLayer": "CnnLossLayer", "Bidirectional": "Bidirectional",
    "SimpleRnn": "SimpleRnn", "ElementWiseMultiplicationLayer": "ElementWiseMult", "MaskLayer": "MaskLayer",
    "MaskZeroLayer": "MaskZeroLayer", "Cropping2D": "Cropping2D",
}
PREPROC_NAMES = {
    "CnnToFeedForwardPreProcessor": "cnnToFeedForward", "CnnToRnnPreProcessor": "cnnToRnn",
    "ComposableInputPreProcessor": "composableInput", "FeedForwardToCnnPreProcessor": "feedForwardToCnn",
    "FeedForwardToRnnPreProcessor": "feedForwardToRnn", "RnnToFeedForwardPreProcessor": "rnnToFeedForward",
    "RnnToCnnPreProcessor": "rnnToCnn", "BinomialSamplingPreProcessor": "binomialSampling",
    "UnitVarianceProcessor": "unitVariance", "ZeroMeanAndUnitVariancePreProcessor": "zeroMeanAndUnitVariance",
    "ZeroMeanPrePreProcessor": "zeroMean",
}
RECON_NAMES = {"GaussianReconstructionDistribution": "Gaussian", "BernoulliReconstructionDistribution": "Bernoulli",
               "ExponentialReconstructionDistribution": "Exponential",
               "CompositeReconstructionDistribution": "Composite", "LossFunctionWrapper": "LossWrapper"}
FQN_PACKAGES = {
    "IUpdater": "org.nd4j.linalg.learning.config.", "ISchedule": "org.nd4j.linalg.schedule.",
    "IDropout": "org.deeplearning4j.nn.conf.dropout.", "IWeightNoise": "org.deeplearning4j.nn.conf.weightnoise.",
    "LayerConstraint": "org.deeplearning4j.nn.conf.constraint.",
}
# our field name -> DL4J bean property
FIELD_OUT = {"activation": "activationFn", "nIn": "nin", "nOut": "nout", "updater": "iupdater"}
FIELD_IN = {v: k for k, v in FIELD_OUT.items()}

_LAYER_IN = {v: k for k, v in LAYER_NAMES.items()}
_PREPROC_IN = {v: k for k, v in PREPROC_NAMES.items()}
_RECON_IN = {v: k for k, v in RECON_NAMES.items()}


def _base_of(obj):
    for klass in type(obj).__mro__:
        n = klass.__name__
        if n in ("IActivation", "ILossFunction", "IUpdater", "ISchedule", "IDropout", "IWeightNoise",
                 "LayerConstraint", "Distribution", "InputPreProcessor", "GraphVertex", "Layer",
                 "ReconstructionDistribution"):
            return n
    return None


# ------------------------------------------------------------------------------------------------ encode
def _enc(v):
    if isinstance(v, Config):
        return _enc_config(v)
    if isinstance(v, enum.Enum):
        return v.name
    if isinstance(v, float):
        if math.isnan(v):
            return "NaN"
        if math.isinf(v):
            return "Infinity" if v > 0 else "-Infinity"
        return v
    if isinstance(v, (list, tuple)):
        return [_enc(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _enc(x) for k, x in v.items()}
    if hasattr(v, "tolist"):                      # tensors / arrays (e.g. loss weights)
        return v.tolist()
    return v


def _fields(obj, rename=True):
    d = {}
    for k in sorted(obj._all_fields()):
        d[FIELD_OUT.get(k, k) if rename else k] = _enc(getattr(obj, k))
    return d


def _enc_config(obj):
    base = _base_of(obj)
    name = type(obj).__name__
    if base == "IActivation":
        return {name[len("Activation"):] if name.startswith("Activation") else name: _fields(obj, False)}
    if base == "ILossFunction":
        return {name[len("Loss"):] if name.startswith("Loss") else name: _fields(obj, False)}
    if base in FQN_PACKAGES:
        d = {"@class": FQN_PACKAGES[base] + name}
        d.update(_fields(obj, False))
        return d
    if base == "Distribution":
        d = {"type": "org.deeplearning4j.nn.conf.distribution." + name}
        d.update(_fields(obj, False))
        return d
    if base == "InputPreProcessor":
        return {PREPROC_NAMES.get(name, name): _fields(obj, False)}
    if base == "ReconstructionDistribution":
        return {RECON_NAMES.get(name, name): _fields(obj, False)}
    if base == "Layer":
        return {LAYER_NAMES.get(name, name): _fields(obj, True)}
    if base == "GraphVertex":
        if name == "LayerVertex":
            return {"LayerVertex": {"layerConf": None, "outputVertex": False, "preProcessor": _enc(obj.preProcessor)}}
        return {name: _fields(obj, False)}
    # any other config (input types, ...): this framework's own tagged form
    return obj.to_dict()


def _nnc(layer, g, iteration, epoch, variables=()):
    """NeuralNetConfiguration JSON object wrapping one layer (NN:nn/conf/NeuralNetConfiguration.java)."""
    return {
        "cacheMode": _enc(g.get("cacheMode", "NONE")) or "NONE",
        "epochCount": epoch,
        "iterationCount": iteration,
        "l1ByParam": {},
        "l2ByParam": {},
        "layer": _enc(layer) if layer is not None else None,
        "maxNumLineSearchIterations": g.get("maxNumLineSearchIterations", 5),
        "miniBatch": bool(g.get("miniBatch", True)),
        "minimize": bool(g.get("minimize", True)),
        "optimizationAlgo": _enc(g.get("optimizationAlgo", "STOCHASTIC_GRADIENT_DESCENT")),
        "pretrain": False,
        "seed": g.get("seed", 12345),
        "stepFunction": _enc(g.get("stepFunction")) if g.get("stepFunction") is not None else None,
        "variables": list(variables),
    }


def _variables(layer):
    try:
        return [s.key for s in layer.param_specs()]
    except Exception:       # noqa: BLE001 - layers whose nIn is not resolved yet
        return []


def _ext(conf, keys):
    return {k: _wrap_ours(getattr(conf, k)) for k in keys}


def _wrap_ours(v):
    from .base import _encode
    return _encode(v)


def mlc_to_dl4j(conf):
    g = conf.globalConf or {}
    confs = [_nnc(c, g, conf.iterationCount, conf.epochCount, _variables(c)) for c in conf.confs]
    return {
        "backprop": bool(conf.backprop),
        "backpropType": _enc(conf.backpropType),
        "cacheMode": _enc(g.get("cacheMode", "NONE")) or "NONE",
        "confs": confs,
        "dataType": _enc(g.get("dataType", "FLOAT")),
        "epochCount": conf.epochCount,
        "inferenceWorkspaceMode": _enc(g.get("inferenceWorkspaceMode", "ENABLED")) or "ENABLED",
        "inputPreProcessors": {str(k): _enc(v) for k, v in (conf.inputPreProcessors or {}).items()},
        "iterationCount": conf.iterationCount,
        "pretrain": bool(conf.pretrain),
        "tbpttBackLength": conf.tbpttBackLength,
        "tbpttFwdLength": conf.tbpttFwdLength,
        "trainingWorkspaceMode": _enc(g.get("trainingWorkspaceMode", "ENABLED")) or "ENABLED",
        "dl4jAmd": _ext(conf, ("globalConf", "inputType")),
    }


def cg_to_dl4j(conf):
    from .graph import LayerVertex
    g = conf.globalConf or {}
    verts = {}
    for name, v in conf.vertices.items():
        if isinstance(v, LayerVertex):
            verts[name] = {"LayerVertex": {
                "layerConf": _nnc(v.layerConf, g, conf.iterationCount, conf.epochCount, _variables(v.layerConf)),
                "outputVertex": name in conf.networkOutputs,
                "preProcessor": _enc(v.preProcessor)}}
        else:
            verts[name] = _enc(v)
    return {
        "backprop": bool(conf.backprop),
        "backpropType": _enc(conf.backpropType),
        "cacheMode": _enc(g.get("cacheMode", "NONE")) or "NONE",
        "dataType": _enc(g.get("dataType", "FLOAT")),
        "defaultConfiguration": _nnc(None, g, conf.iterationCount, conf.epochCount),
        "epochCount": conf.epochCount,
        "inferenceWorkspaceMode": _enc(g.get("inferenceWorkspaceMode", "ENABLED")) or "ENABLED",
        "iterationCount": conf.iterationCount,
        "networkInputs": list(conf.networkInputs),
        "networkOutputs": list(conf.networkOutputs),
        "pretrain": bool(conf.pretrain),
        "tbpttBackLength": conf.tbpttBackLength,
        "tbpttFwdLength": conf.tbpttFwdLength,
        "trainingWorkspaceMode": _enc(g.get("trainingWorkspaceMode", "ENABLED")) or "ENABLED",
        "vertexInputs": {k: list(v) for k, v in conf.vertexInputs.items()},
        "vertices": verts,
        "dl4jAmd": _ext(conf, ("globalConf", "inputTypes")),
    }


# ------------------------------------------------------------------------------------------------ decode
_SPECIAL = {"NaN": float("nan"), "Infinity": float("inf"), "-Infinity": float("-inf")}


def _cls_for(name, table=None):
    if table and name in table:
        name = table[name]
    return _REGISTRY.get(name)


def _dec(v):
    """Decode a DL4J JSON value into this framework's config objects (shape-driven)."""
    if isinstance(v, str) and v in _SPECIAL:
        return _SPECIAL[v]
    if isinstance(v, list):
        return [_dec(x) for x in v]
    if not isinstance(v, dict):
        return v
    if "@class" in v:
        cname = v["@class"]
        if cname.startswith("org."):
            cls = _REGISTRY.get(cname.rsplit(".", 1)[-1])
            if cls is None:
                raise KeyError(f"unsupported DL4J class {cname}")
            return _make(cls, {k: x for k, x in v.items() if k != "@class"})
        from .base import _decode
        return _decode(v)                         # this framework's own tagged form
    if "type" in v and isinstance(v["type"], str) and v["type"].startswith("org.deeplearning4j.nn.conf.distribution."):
        cls = _REGISTRY.get(v["type"].rsplit(".", 1)[-1])
        return _make(cls, {k: x for k, x in v.items() if k != "type"})
    if len(v) == 1:
        (name, body), = v.items()
        if isinstance(body, dict):
            cls = (_cls_for(name, _LAYER_IN) if name in _LAYER_IN else None) or \
                _cls_for(name, _PREPROC_IN) or _cls_for(name, _RECON_IN) or \
                _REGISTRY.get("Activation" + name) or _REGISTRY.get("Loss" + name)
            if cls is None and name in _REGISTRY and _base_of_cls(_REGISTRY[name]) in (
                    "Layer", "GraphVertex", "InputPreProcessor"):
                cls = _REGISTRY[name]
            if cls is None and name.upper() in ("TANH",):
                cls = _REGISTRY.get("ActivationTanH")
            if cls is not None:
                return _make(cls, body)
    return {k: _dec(x) for k, x in v.items()}


def _base_of_cls(cls):
    for klass in cls.__mro__:
        if klass.__name__ in ("Layer", "GraphVertex", "InputPreProcessor"):
            return klass.__name__
    return None


def _make(cls, body):
    fields = cls._all_fields()
    kw = {}
    for k, x in body.items():
        ours = FIELD_IN.get(k, k)
        if ours not in fields:
            continue
        val = _dec(x)
        default = fields[ours]
        if isinstance(val, str) and isinstance(default, enum.Enum):
            et = type(default)
            val = et[val] if val in et.__members__ else (et.of(val) if hasattr(et, "of") else val)
        kw[ours] = val
    if _base_of_cls(cls) == "Layer":
        _legacy_layer(cls, body, kw, fields)
    obj = cls.__new__(cls)
    for k, d in fields.items():
        setattr(obj, k, _copy(d))
    for k, val in kw.items():
        conv = cls._CONVERTERS.get(k)
        if conv is not None and val is not None and not isinstance(val, Config):
            try:
                val = conv(val)
            except Exception:       # noqa: BLE001 - keep the raw value if the converter does not take it
                pass
        setattr(obj, k, val)
    obj._post_init()
    return obj


def _copy(d):
    import copy
    return copy.deepcopy(d)


_LEGACY_UPDATERS = {"SGD": "Sgd", "NESTEROVS": "Nesterovs", "ADAM": "Adam", "RMSPROP": "RmsProp",
                    "ADAGRAD": "AdaGrad", "ADADELTA": "AdaDelta", "NONE": "NoOp", "ADAMAX": "AdaMax",
                    "NADAM": "Nadam"}
_LEGACY_LOSS = {"MSE": "LossMSE", "XENT": "LossBinaryXENT", "NEGATIVELOGLIKELIHOOD": "LossNegativeLogLikelihood",
                "MCXENT": "LossMCXENT", "SQUARED_LOSS": "LossL2", "L1": "LossL1", "L2": "LossL2",
                "MEAN_ABSOLUTE_ERROR": "LossMAE", "HINGE": "LossHinge", "KL_DIVERGENCE": "LossKLD",
                "POISSON": "LossPoisson", "COSINE_PROXIMITY": "LossCosineProximity"}


def _num(body, k):
    v = body.get(k)
    if v is None or (isinstance(v, str) and v in _SPECIAL) or (isinstance(v, float) and math.isnan(v)):
        return None
    return v


def _legacy_layer(cls, body, kw, fields):
    """Pre-1.0 layer fields (NN:nn/conf/serde/BaseNetConfigDeserializer.java): updater enum + hyperparameters,
    lossFunction enum, dropOut probability."""
    if "updater" in fields and (kw.get("updater") is None or isinstance(kw.get("updater"), str)) and \
            isinstance(body.get("updater"), str) and "iupdater" not in body:
        name = _LEGACY_UPDATERS.get(body["updater"].upper())
        if name is not None:
            ucls = lookup(name)
            args = {}
            lr = _num(body, "learningRate")
            if lr is not None and "learningRate" in ucls._all_fields():
                args["learningRate"] = lr
            for src, dst in (("momentum", "momentum"), ("adamMeanDecay", "beta1"), ("adamVarDecay", "beta2"),
                             ("epsilon", "epsilon"), ("rmsDecay", "rmsDecay"), ("rho", "rho")):
                val = _num(body, src)
                if val is not None and dst in ucls._all_fields():
                    args[dst] = val
            kw["updater"] = ucls(**args)
    if "lossFn" in fields and (kw.get("lossFn") is None or isinstance(kw.get("lossFn"), str)) and \
            isinstance(body.get("lossFunction"), str):
        name = _LEGACY_LOSS.get(body["lossFunction"].upper())
        if name is not None:
            kw["lossFn"] = lookup(name)()
    if "idropout" in fields and kw.get("idropout") is None:
        p = _num(body, "dropOut")
        if p:
            kw["idropout"] = lookup("Dropout")(p=p)


def _global(nnc, top):
    from .enums import OptimizationAlgorithm
    g = {}
    if nnc:
        for k in ("seed", "miniBatch", "minimize", "maxNumLineSearchIterations"):
            if k in nnc:
                g[k] = nnc[k]
        if nnc.get("optimizationAlgo"):
            try:
                g["optimizationAlgo"] = OptimizationAlgorithm[nnc["optimizationAlgo"]]
            except KeyError:
                pass
    return g


def _restore_ext(conf, top):
    from .base import _decode
    ext = top.get("dl4jAmd") or {}
    for k, v in ext.items():
        if k in conf._all_fields():
            setattr(conf, k, _decode(v))


def mlc_from_dl4j(d):
    from .enums import BackpropType
    from .network import MultiLayerConfiguration
    conf = MultiLayerConfiguration.__new__(MultiLayerConfiguration)
    for k, dflt in MultiLayerConfiguration._all_fields().items():
        setattr(conf, k, _copy(dflt))
    conf.confs = [_dec(c["layer"]) for c in d.get("confs", [])]
    conf.inputPreProcessors = {int(k): _dec(v) for k, v in (d.get("inputPreProcessors") or {}).items()
                               if v is not None}
    conf.backprop = d.get("backprop", True)
    conf.pretrain = d.get("pretrain", False)
    if d.get("backpropType"):
        conf.backpropType = BackpropType[d["backpropType"]]
    conf.tbpttFwdLength = d.get("tbpttFwdLength", 20)
    conf.tbpttBackLength = d.get("tbpttBackLength", 20)
    conf.iterationCount = d.get("iterationCount", 0)
    conf.epochCount = d.get("epochCount", 0)
    conf.globalConf = _global(d["confs"][0] if d.get("confs") else None, d)
    _restore_ext(conf, d)
    conf._post_init()
    return conf


def cg_from_dl4j(d):
    from .enums import BackpropType
    from .network import ComputationGraphConfiguration
    conf = ComputationGraphConfiguration.__new__(ComputationGraphConfiguration)
    for k, dflt in ComputationGraphConfiguration._all_fields().items():
        setattr(conf, k, _copy(dflt))
    from .graph import LayerVertex
    verts = {}
    first_nnc = d.get("defaultConfiguration")
    for name, v in d.get("vertices", {}).items():
        (vt, body), = v.items()
        if vt == "LayerVertex":
            lc = body.get("layerConf") or {}
            first_nnc = first_nnc or lc
            lv = LayerVertex.__new__(LayerVertex)
            for k, dflt in LayerVertex._all_fields().items():
                setattr(lv, k, _copy(dflt))
            lv.layerConf = _dec(lc.get("layer"))
            lv.preProcessor = _dec(body.get("preProcessor")) if body.get("preProcessor") else None
            lv._post_init()
            verts[name] = lv
        else:
            verts[name] = _dec(v)
    conf.vertices = verts
    conf.vertexInputs = {k: list(x) for k, x in d.get("vertexInputs", {}).items()}
    conf.networkInputs = list(d.get("networkInputs", []))
    conf.networkOutputs = list(d.get("networkOutputs", []))
    conf.backprop = d.get("backprop", True)
    conf.pretrain = d.get("pretrain", False)
    if d.get("backpropType"):
        conf.backpropType = BackpropType[d["backpropType"]]
    conf.tbpttFwdLength = d.get("tbpttFwdLength", 20)
    conf.tbpttBackLength = d.get("tbpttBackLength", 20)
    conf.iterationCount = d.get("iterationCount", 0)
    conf.epochCount = d.get("epochCount", 0)
    conf.globalConf = _global(first_nnc, d)
    _restore_ext(conf, d)
    conf._post_init()
    return conf


def is_dl4j_format(d):
    if not isinstance(d, dict) or "@class" in d:
        return False
    if "confs" in d:
        return all(isinstance(c, dict) and "layer" in c for c in d["confs"])
    return "vertices" in d and "networkInputs" in d


def from_json(s):
    d = json.loads(s) if isinstance(s, str) else s
    if "confs" in d:
        return mlc_from_dl4j(d)
    return cg_from_dl4j(d)


def to_json(conf):
    d = mlc_to_dl4j(conf) if type(conf).__name__ == "MultiLayerConfiguration" else cg_to_dl4j(conf)
    return json.dumps(d, indent=2)          # insertion order: vertex order fixes the flat parameter layout
