"""Memory reports: per-layer and per-network memory estimates by MemoryType as a function of minibatch size
(reference nn/conf/memory/{MemoryType,MemoryUseMode,LayerMemoryReport,NetworkMemoryReport}.java).

Totals follow NetworkMemoryReport.getTotalMemoryBytes: sum over layers of every non-working memory type +
the maximum over layers of the working memory (working memory is transient, reused layer to layer).
The per-layer numbers describe THIS framework's kernels: implicit-GEMM convolutions never materialise
im2col (the reference's dominant working memory), so conv working memory is the bf16 weight relayouts;
BN working memory is its per-block partial-sum buffers; the bf16 compute shadow of the parameters is
reported as fixed working memory of reduced-precision networks. ``fits(device_bytes)`` answers the
"does this minibatch fit in 288 GB of HBM3E" question the MI355X sizing needs.
"""
import enum

from .inputs import InputType


class MemoryType(enum.Enum):
    PARAMETERS = "PARAMETERS"
    PARAMATER_GRADIENTS = "PARAMATER_GRADIENTS"
    ACTIVATIONS = "ACTIVATIONS"
    ACTIVATION_GRADIENTS = "ACTIVATION_GRADIENTS"
    UPDATER_STATE = "UPDATER_STATE"
    WORKING_MEMORY_FIXED = "WORKING_MEMORY_FIXED"
    WORKING_MEMORY_VARIABLE = "WORKING_MEMORY_VARIABLE"
    CACHED_MEMORY_FIXED = "CACHED_MEMORY_FIXED"
    CACHED_MEMORY_VARIABLE = "CACHED_MEMORY_VARIABLE"

    def isInference(self):
        return self in (MemoryType.PARAMETERS, MemoryType.ACTIVATIONS, MemoryType.WORKING_MEMORY_FIXED,
                        MemoryType.WORKING_MEMORY_VARIABLE)


class MemoryUseMode(enum.Enum):
    TRAINING = "TRAINING"
    INFERENCE = "INFERENCE"


def bytes_per_element(dataType):
    name = str(getattr(dataType, "name", dataType)).upper()
    return {"DOUBLE": 8, "FLOAT": 4, "HALF": 2, "BFLOAT16": 2, "FLOAT16": 2}.get(name, 4)


class MemoryReport:
    def getTotalMemoryBytes(self, minibatchSize, memoryUseMode, cacheMode=None, dataType="FLOAT"):
        raise NotImplementedError

    def getMemoryBytes(self, memoryType, minibatchSize, memoryUseMode, cacheMode=None, dataType="FLOAT"):
        raise NotImplementedError

    # ---- JSON / YAML (reference MemoryReport.toJson / toYaml / fromJson / fromYaml)
    def to_dict(self):
        raise NotImplementedError

    def toJson(self):
        import json
        return json.dumps(self.to_dict(), indent=2)

    def toYaml(self):
        import yaml
        return yaml.safe_dump(self.to_dict(), sort_keys=False)

    @staticmethod
    def from_dict(d):
        cls = {"LayerMemoryReport": LayerMemoryReport, "NetworkMemoryReport": NetworkMemoryReport}[d["@class"]]
        return cls._from(d)

    @staticmethod
    def fromJson(s):
        import json
        return MemoryReport.from_dict(json.loads(s))

    @staticmethod
    def fromYaml(s):
        import yaml
        return MemoryReport.from_dict(yaml.safe_load(s))

    def __eq__(self, other):
        return isinstance(other, MemoryReport) and type(other) is type(self) and self.to_dict() == other.to_dict()

    def __hash__(self):
        return hash(self.toJson())


def _it_dict(t):
    return None if t is None else t.to_dict()


def _it_from(d):
    from .base import _decode
    return None if d is None else _decode(d)


class LayerMemoryReport(MemoryReport):
    def __init__(self, layerName, layerType, inputType, outputType, parameterSize=0, updaterStateSize=0,
                 workingMemoryFixedInference=0, workingMemoryVariableInference=0, workingMemoryFixedTrain=0,
                 workingMemoryVariableTrain=0, cacheModeMemFixed=0, cacheModeMemVariablePerEx=0):
        self.layerName, self.layerType = layerName, layerType
        self.inputType, self.outputType = inputType, outputType
        self.parameterSize, self.updaterStateSize = int(parameterSize), int(updaterStateSize)
        self.wFixInf, self.wVarInf = int(workingMemoryFixedInference), int(workingMemoryVariableInference)
        self.wFixTrain, self.wVarTrain = int(workingMemoryFixedTrain), int(workingMemoryVariableTrain)
        self.cacheFixed, self.cacheVarPerEx = int(cacheModeMemFixed), int(cacheModeMemVariablePerEx)

    def getReportClass(self):
        return self.layerType

    def getName(self):
        return self.layerName

    _KEYS = ("parameterSize", "updaterStateSize", "wFixInf", "wVarInf", "wFixTrain", "wVarTrain", "cacheFixed",
             "cacheVarPerEx")

    def to_dict(self):
        d = {"@class": "LayerMemoryReport", "layerName": self.layerName, "layerType": self.layerType,
             "inputType": _it_dict(self.inputType), "outputType": _it_dict(self.outputType)}
        d.update({k: getattr(self, k) for k in self._KEYS})
        return d

    @classmethod
    def _from(cls, d):
        r = cls(d["layerName"], d["layerType"], _it_from(d["inputType"]), _it_from(d["outputType"]))
        for k in cls._KEYS:
            setattr(r, k, int(d[k]))
        return r

    def getMemoryBytes(self, memoryType, minibatchSize, memoryUseMode, cacheMode=None, dataType="FLOAT"):
        b = bytes_per_element(dataType)
        train = memoryUseMode == MemoryUseMode.TRAINING
        mt = memoryType
        if mt == MemoryType.PARAMETERS:
            return self.parameterSize * b
        if mt == MemoryType.PARAMATER_GRADIENTS:
            return self.parameterSize * b if train else 0
        if mt == MemoryType.ACTIVATIONS:
            return minibatchSize * self.outputType.arrayElementsPerExample() * b
        if mt == MemoryType.ACTIVATION_GRADIENTS:
            return minibatchSize * self.inputType.arrayElementsPerExample() * b if train else 0
        if mt == MemoryType.UPDATER_STATE:
            return self.updaterStateSize * b if train else 0
        if mt == MemoryType.WORKING_MEMORY_FIXED:
            return (self.wFixTrain if train else self.wFixInf) * b
        if mt == MemoryType.WORKING_MEMORY_VARIABLE:
            return minibatchSize * (self.wVarTrain if train else self.wVarInf) * b
        mode = str(getattr(cacheMode, "name", cacheMode) or "NONE").upper()
        if mt == MemoryType.CACHED_MEMORY_FIXED:
            return self.cacheFixed * b if train and mode != "NONE" else 0
        if mt == MemoryType.CACHED_MEMORY_VARIABLE:
            return minibatchSize * self.cacheVarPerEx * b if train and mode != "NONE" else 0
        raise ValueError(memoryType)

    def getTotalMemoryBytes(self, minibatchSize, memoryUseMode, cacheMode=None, dataType="FLOAT"):
        return sum(self.getMemoryBytes(mt, minibatchSize, memoryUseMode, cacheMode, dataType) for mt in MemoryType)

    def __repr__(self):
        return (f"LayerMemoryReport(name={self.layerName}, type={self.layerType}, params={self.parameterSize}, "
                f"updaterState={self.updaterStateSize}, in={self.inputType}, out={self.outputType})")


class NetworkMemoryReport(MemoryReport):
    def __init__(self, layerAndVertexReports, modelClass, modelName, networkInputTypes):
        self.layerAndVertexReports = layerAndVertexReports      # ordered dict name -> LayerMemoryReport
        self.modelClass, self.modelName = modelClass, modelName
        self.networkInputTypes = networkInputTypes

    def getReportClass(self):
        return self.modelClass

    def getName(self):
        return self.modelName

    def to_dict(self):
        nit = self.networkInputTypes
        nit = [_it_dict(t) for t in nit] if isinstance(nit, (list, tuple)) else _it_dict(nit)
        return {"@class": "NetworkMemoryReport", "modelClass": self.modelClass, "modelName": self.modelName,
                "networkInputTypes": nit,
                "layerAndVertexReports": [[n, r.to_dict()] for n, r in self.layerAndVertexReports.items()]}

    @classmethod
    def _from(cls, d):
        nit = d["networkInputTypes"]
        nit = [_it_from(t) for t in nit] if isinstance(nit, list) else _it_from(nit)
        reps = {n: MemoryReport.from_dict(r) for n, r in d["layerAndVertexReports"]}
        return cls(reps, d["modelClass"], d["modelName"], nit)

    def getTotalMemoryBytes(self, minibatchSize, memoryUseMode, cacheMode=None, dataType="FLOAT"):
        total, best = 0, (0, 0)
        for r in self.layerAndVertexReports.values():
            for mt in MemoryType:
                if mt in (MemoryType.WORKING_MEMORY_FIXED, MemoryType.WORKING_MEMORY_VARIABLE):
                    continue
                total += r.getMemoryBytes(mt, minibatchSize, memoryUseMode, cacheMode, dataType)
            wf = r.getMemoryBytes(MemoryType.WORKING_MEMORY_FIXED, minibatchSize, memoryUseMode, cacheMode, dataType)
            wv = r.getMemoryBytes(MemoryType.WORKING_MEMORY_VARIABLE, minibatchSize, memoryUseMode, cacheMode,
                                  dataType)
            if wf + wv > sum(best):
                best = (wf, wv)
        return total + sum(best)

    def getMemoryBytes(self, memoryType, minibatchSize, memoryUseMode, cacheMode=None, dataType="FLOAT"):
        vals = [r.getMemoryBytes(memoryType, minibatchSize, memoryUseMode, cacheMode, dataType)
                for r in self.layerAndVertexReports.values()]
        if memoryType in (MemoryType.WORKING_MEMORY_FIXED, MemoryType.WORKING_MEMORY_VARIABLE):
            return max(vals) if vals else 0
        return sum(vals)

    def maxMinibatchFor(self, deviceBytes, memoryUseMode=MemoryUseMode.TRAINING, dataType="FLOAT", cacheMode=None):
        """Largest minibatch whose estimate fits in ``deviceBytes`` (e.g. 288e9 for one MI355X)."""
        fixed = self.getTotalMemoryBytes(0, memoryUseMode, cacheMode, dataType)
        per = self.getTotalMemoryBytes(1, memoryUseMode, cacheMode, dataType) - fixed
        return 0 if per <= 0 or deviceBytes <= fixed else int((deviceBytes - fixed) // per)

    def toString(self):
        fixedInf = self.getTotalMemoryBytes(0, MemoryUseMode.INFERENCE)
        perInf = self.getTotalMemoryBytes(1, MemoryUseMode.INFERENCE) - fixedInf
        fixedTr = self.getTotalMemoryBytes(0, MemoryUseMode.TRAINING)
        perTr = self.getTotalMemoryBytes(1, MemoryUseMode.TRAINING) - fixedTr
        counts = {}
        for r in self.layerAndVertexReports.values():
            counts[r.layerType] = counts.get(r.layerType, 0) + 1
        lines = ["----- Network Memory Report -----", f"  Model Class:                        {self.modelClass}",
                 f"  Model Name:                         {self.modelName}",
                 f"  Network Input:                      {self.networkInputTypes}",
                 f"  # Layers:                           {len(self.layerAndVertexReports)}",
                 f"  Layer Types:                        {counts}",
                 f"  Inference Memory (FP32)             {fixedInf:,} + {perInf:,} * minibatch bytes",
                 f"  Training Memory (FP32):             {fixedTr:,} + {perTr:,} * minibatch bytes",
                 "  Inference Memory Breakdown (FP32):"]
        for mt in MemoryType:
            if mt.isInference():
                f0 = self.getMemoryBytes(mt, 0, MemoryUseMode.INFERENCE)
                f1 = self.getMemoryBytes(mt, 1, MemoryUseMode.INFERENCE) - f0
                lines.append(f"  - {mt.value:<28} {f0:,} + {f1:,} * minibatch bytes")
        lines.append("  Training Memory Breakdown (FP32):")
        for mt in MemoryType:
            f0 = self.getMemoryBytes(mt, 0, MemoryUseMode.TRAINING)
            f1 = self.getMemoryBytes(mt, 1, MemoryUseMode.TRAINING) - f0
            lines.append(f"  - {mt.value:<28} {f0:,} + {f1:,} * minibatch bytes")
        return "\n".join(lines)

    __str__ = toString


# ----------------------------------------------------------------------------------------------- estimators
def _updater_state(lc):
    n = 0
    for spec in lc.param_specs():
        if not spec.trainable:
            continue
        u = lc.updaterFor(spec.key)
        if u is not None:
            n += u.stateSize(spec.numel)
    return n


def layer_memory_report(lc, inputType, outputType, name=None, compute_bytes=None):
    """Estimate one layer's memory. ``compute_bytes``: element size of a reduced-precision compute shadow."""
    t = type(lc).__name__
    base = lc.underlying if getattr(lc, "underlying", None) is not None and t in ("FrozenLayer",) else lc
    bt = type(base).__name__
    nparams = lc.numParams() if hasattr(lc, "numParams") else 0
    wfi = wvi = wft = wvt = 0
    cache_var = 0
    outE = outputType.arrayElementsPerExample() if outputType is not None else 0
    inE = inputType.arrayElementsPerExample() if inputType is not None else 0
    if bt in ("ConvolutionLayer", "Convolution2D", "Deconvolution2D", "SeparableConvolution2D",
              "DepthwiseConvolution2D", "Convolution1DLayer", "Convolution1D"):
        wfi = wft = 2 * nparams          # KRSC + flipped weight relayouts (counted in element units)
        cache_var = inE                  # the layer keeps its input for the weight gradient
    elif bt == "BatchNormalization":
        c = getattr(base, "nOut", 0) or 0
        wfi = wft = 4 * c + 2 * 1024 * c  # ctx + per-block partial sums
        cache_var = inE
    elif bt in ("LSTM", "GravesLSTM", "GravesBidirectionalLSTM", "SimpleRnn"):
        T = getattr(inputType, "timeSeriesLength", 1) or 1
        n = getattr(base, "nOut", 0) or 0
        gates = 4 if bt != "SimpleRnn" else 1
        wvi = gates * n * T
        wvt = 3 * gates * n * T           # gate pre-activations + activations + cell states kept for backprop
    elif bt in ("SubsamplingLayer", "Pooling2D"):
        wvt = outE // 2 if outE else 0    # 1-byte argmax per output element (units of 2-byte elements)
    elif bt == "SelfAttentionLayer":
        T = getattr(inputType, "timeSeriesLength", 1) or 1
        wvi = wvt = 3 * outE + getattr(base, "nHeads", 1) * T * T
    if compute_bytes:
        wfi += nparams * compute_bytes // 4
        wft += nparams * compute_bytes // 4
    return LayerMemoryReport(name or getattr(lc, "layerName", None) or t, t, inputType, outputType, nparams,
                             _updater_state(lc), wfi, wvi, wft, wvt, 0, cache_var)


def mln_memory_report(conf, inputType=None):
    from collections import OrderedDict
    t = inputType or conf.inputType
    if t is None:
        raise ValueError("A memory report needs the network's InputType (setInputType or pass inputType)")
    reps = OrderedDict()
    for i, lc in enumerate(conf.confs):
        pp = conf.inputPreProcessors.get(i)
        if pp is not None:
            t = pp.getOutputType(t)
        out = lc.getOutputType(i, t)
        reps[lc.layerName or f"layer{i}"] = layer_memory_report(lc, t, out)
        t = out
    return NetworkMemoryReport(reps, "MultiLayerNetwork", "MultiLayerNetwork", [inputType or conf.inputType])


def cg_memory_report(conf, inputTypes=None):
    from collections import OrderedDict
    from .graph import LayerVertex
    its = list(inputTypes or conf.inputTypes or [])
    if not its:
        raise ValueError("A memory report needs the graph's input types (setInputTypes or pass inputTypes)")
    types = dict(zip(conf.networkInputs, its))
    reps = OrderedDict()
    for i, name in enumerate(conf.topologicalOrder()):
        if name in conf.networkInputs:
            continue
        v = conf.vertices[name]
        ins = [types[x] for x in conf.vertexInputs[name]]
        out = v.getOutputType(i, *ins)
        types[name] = out
        if isinstance(v, LayerVertex):
            t = ins[0] if len(ins) == 1 else out
            if v.preProcessor is not None:
                t = v.preProcessor.getOutputType(t)
            reps[name] = layer_memory_report(v.layerConf, t, out, name)
        else:
            reps[name] = LayerMemoryReport(name, type(v).__name__, ins[0] if ins else None, out)
    return NetworkMemoryReport(reps, "ComputationGraph", "ComputationGraph", its)


def network_memory_report(net, minibatch=1):
    conf = net.conf
    if type(net).__name__ == "ComputationGraph":
        return cg_memory_report(conf)
    return mln_memory_report(conf)


_ = InputType
