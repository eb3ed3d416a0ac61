"""Transfer learning: fine-tune overrides, freezing (feature extractor), nOut replacement, removing/adding layers
or vertices, and featurize-then-train helpers.

Reference: nn/transferlearning/TransferLearning.java:32-261 (Builder for MultiLayerNetwork, GraphBuilder for
ComputationGraph), FineTuneConfiguration.java, TransferLearningHelper.java.
Parameters of every layer whose shape is unchanged are copied from the source network (device to device, no
host round trip); layers touched by nOutReplace (and the nIn side of the next layer) are re-initialised with
the requested WeightInit/distribution. Frozen layers are wrapped in FrozenLayer (NoOp updater, no l1/l2, no
epsilon past them).
"""
import copy

import torch

from .conf.layers import FeedForwardLayer, FrozenLayer, Layer
from .conf.weights import to_weight_init

_FT_LAYER_KEYS = ("activation", "weightInit", "biasInit", "dist", "l1", "l2", "l1Bias", "l2Bias", "updater",
                  "biasUpdater", "weightNoise", "gradientNormalization", "gradientNormalizationThreshold",
                  "convolutionMode", "idropout", "constraints")
_FT_GLOBAL_KEYS = ("seed", "optimizationAlgo", "miniBatch", "maxNumLineSearchIterations", "minimize",
                   "stepFunction", "trainingWorkspaceMode", "inferenceWorkspaceMode", "cacheMode")


class FineTuneConfiguration:
    """Hyperparameter overrides applied to every layer of the new network, frozen ones included (their parameters
    do not move, but their configuration reads as the reference's: TransferLearning.java:359-365, 474-487)."""

    def __init__(self, **kw):
        self.overrides = kw
        self.backpropType = kw.pop("backpropType", None)
        self.tbpttFwdLength = kw.pop("tbpttFwdLength", None)
        self.tbpttBackLength = kw.pop("tbpttBackLength", None)

    # ---- serde (reference FineTuneConfiguration.toJson / toYaml / fromJson / fromYaml) -------------------------
    def _as_dict(self):
        from .conf.base import _encode
        d = {"@class": "FineTuneConfiguration", "overrides": {k: _encode(v) for k, v in sorted(self.overrides.items())}}
        for k in ("backpropType", "tbpttFwdLength", "tbpttBackLength"):
            d[k] = _encode(getattr(self, k))
        return d

    @classmethod
    def _from_dict(cls, d):
        from .conf.base import _decode
        obj = cls()
        obj.overrides = {k: _decode(v) for k, v in d.get("overrides", {}).items()}
        for k in ("backpropType", "tbpttFwdLength", "tbpttBackLength"):
            setattr(obj, k, _decode(d.get(k)))
        return obj

    def toJson(self):
        import json
        return json.dumps(self._as_dict(), indent=2, sort_keys=True)

    @classmethod
    def fromJson(cls, s):
        import json
        return cls._from_dict(json.loads(s))

    def toYaml(self):
        import yaml
        return yaml.safe_dump(self._as_dict(), sort_keys=True)

    @classmethod
    def fromYaml(cls, s):
        import yaml
        return cls._from_dict(yaml.safe_load(s))

    def __eq__(self, other):
        return isinstance(other, FineTuneConfiguration) and self._as_dict() == other._as_dict()

    def __hash__(self):
        return hash(self.toJson())

    class Builder:
        def __init__(self):
            self._kw = {}

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)
            key = {"dropOut": "idropout", "activationFn": "activation", "iUpdater": "updater"}.get(name, name)

            def setter(*v):
                val = v[0] if len(v) == 1 else v
                if key == "idropout" and isinstance(val, (int, float)):
                    from .conf.regularization import Dropout
                    val = Dropout(float(val)) if val > 0 else None
                if key == "l1" or key == "l2":
                    val = float(val)
                self._kw[key] = val
                return self
            return setter

        def build(self):
            return FineTuneConfiguration(**self._kw)

    def applyToLayer(self, lc):
        fields = lc._all_fields() if hasattr(lc, "_all_fields") else {}
        for k, v in self.overrides.items():
            if k in _FT_LAYER_KEYS and k in fields:
                conv = getattr(lc, "_CONVERTERS", {}).get(k)
                setattr(lc, k, conv(copy.deepcopy(v)) if conv and v is not None else copy.deepcopy(v))
        if "weightInit" in self.overrides and "dist" not in self.overrides and "dist" in fields:
            pass

    def applyToGlobal(self, g):
        for k in _FT_GLOBAL_KEYS:
            if k in self.overrides:
                g[k] = self.overrides[k]


def _base(lc):
    while isinstance(lc, FrozenLayer) or (getattr(lc, "underlying", None) is not None and
                                           type(lc).__name__ == "FrozenLayer"):
        lc = lc.underlying
    return lc


def _shapes(impl):
    return {k: tuple(v.shape) for k, v in impl.params.items()} if impl is not None else {}


def _copy_params(dst_impl, src_impl):
    if dst_impl is None or src_impl is None:
        return
    for k, v in dst_impl.params.items():
        s = src_impl.params.get(k)
        if s is not None and tuple(s.shape) == tuple(v.shape):
            with torch.no_grad():
                v.copy_(s.to(v.device, v.dtype))


class TransferLearning:
    class Builder:
        """MultiLayerNetwork transfer learning (TransferLearning.Builder)."""

        def __init__(self, origModel):
            self.orig = origModel
            oc = origModel.conf
            self.confs = [copy.deepcopy(c) for c in oc.confs]
            self.src_index = list(range(len(self.confs)))      # new layer i <- original layer src_index[i]
            self.pps = copy.deepcopy(dict(oc.inputPreProcessors))
            self.globalConf = copy.deepcopy(dict(oc.globalConf))
            self.backpropType, self.fwd, self.back = oc.backpropType, oc.tbpttFwdLength, oc.tbpttBackLength
            self.inputType = oc.inputType
            self.frozenTill = -1
            self.reinit = set()
            self.ft = None

        def fineTuneConfiguration(self, ft):
            self.ft = ft
            return self

        def setFeatureExtractor(self, layerNum):
            self.frozenTill = int(layerNum)
            return self

        def nOutReplace(self, layerNum, nOut, weightInit=None, weightInitNext=None, dist=None, distNext=None):
            from .conf.weights import Distribution
            if isinstance(weightInit, Distribution):
                dist, weightInit = weightInit, "DISTRIBUTION"
            if isinstance(weightInitNext, Distribution):
                distNext, weightInitNext = weightInitNext, "DISTRIBUTION"
            lc = _base(self.confs[layerNum])
            lc.nOut = int(nOut)
            if weightInit is not None:
                lc.weightInit = to_weight_init(weightInit)
            if dist is not None:
                lc.dist = dist
            self.reinit.add(layerNum)
            for j in range(layerNum + 1, len(self.confs)):
                nx = _base(self.confs[j])
                if isinstance(nx, FeedForwardLayer) and nx.param_specs():
                    if type(nx).__name__ == "BatchNormalization":
                        nx.nIn = nx.nOut = int(nOut)
                        self.reinit.add(j)
                        continue
                    nx.nIn = int(nOut)
                    if weightInitNext is not None:
                        nx.weightInit = to_weight_init(weightInitNext)
                    if distNext is not None:
                        nx.dist = distNext
                    self.reinit.add(j)
                    break
            return self

        def removeOutputLayer(self):
            return self.removeLayersFromOutput(1)

        def removeLayersFromOutput(self, n):
            n = int(n)
            if n > len(self.confs):
                raise ValueError("Cannot remove more layers than the network has")
            self.confs = self.confs[:len(self.confs) - n]
            self.src_index = self.src_index[:len(self.src_index) - n]
            self.pps = {k: v for k, v in self.pps.items() if k < len(self.confs)}
            return self

        def addLayer(self, layer):
            if hasattr(layer, "build") and not isinstance(layer, Layer):
                layer = layer.build()
            layer = copy.deepcopy(layer)
            if isinstance(layer, FeedForwardLayer) and not getattr(layer, "nIn", 0) and self.confs:
                prev = next((_base(c) for c in reversed(self.confs) if getattr(_base(c), "nOut", 0)), None)
                if prev is not None:
                    layer.nIn = prev.nOut
            layer.applyGlobal(self.globalConf)
            if hasattr(layer, "finalize_defaults"):
                layer.finalize_defaults()
            self.confs.append(layer)
            self.src_index.append(None)
            return self

        def setInputPreProcessor(self, layer, pp):
            self.pps[int(layer)] = pp
            return self

        def build(self):
            from .conf.network import MultiLayerConfiguration
            from .multilayer import MultiLayerNetwork
            g = dict(self.globalConf)
            confs = []
            for i, c in enumerate(self.confs):
                c = _base(c)
                if self.ft is not None:
                    self.ft.applyToLayer(c)
                if c.layerName is None:
                    c.layerName = f"layer{i}"
                confs.append(FrozenLayer(layer=c, layerName=c.layerName) if i <= self.frozenTill else c)
            if self.ft is not None:
                self.ft.applyToGlobal(g)
            bp = self.ft.backpropType if self.ft is not None and self.ft.backpropType is not None else \
                self.backpropType
            conf = MultiLayerConfiguration(confs=confs, inputPreProcessors=self.pps, backpropType=bp,
                                           tbpttFwdLength=(self.ft.tbpttFwdLength if self.ft and
                                                           self.ft.tbpttFwdLength else self.fwd),
                                           tbpttBackLength=(self.ft.tbpttBackLength if self.ft and
                                                            self.ft.tbpttBackLength else self.back),
                                           globalConf=g, inputType=self.inputType)
            net = MultiLayerNetwork(conf)
            net.init(device=self.orig.device)
            for i, src in enumerate(self.src_index):
                if src is None or i in self.reinit:
                    continue
                _copy_params(net.layers[i], self.orig.layers[src])
            net._params_changed()
            return net

    class GraphBuilder:
        """ComputationGraph transfer learning (TransferLearning.GraphBuilder)."""

        def __init__(self, origGraph):
            self.orig = origGraph
            oc = origGraph.conf
            self.vertices = {k: copy.deepcopy(v) for k, v in oc.vertices.items()}
            self.vertexInputs = {k: list(v) for k, v in oc.vertexInputs.items()}
            self.inputs = list(oc.networkInputs)
            self.outputs = list(oc.networkOutputs)
            self.globalConf = copy.deepcopy(dict(oc.globalConf))
            self.oc = oc
            self.frozen = set()
            self.reinit = set()
            self.ft = None

        def fineTuneConfiguration(self, ft):
            self.ft = ft
            return self

        def setFeatureExtractor(self, *names):
            stack = list(names)
            while stack:
                n = stack.pop()
                if n in self.frozen or n in self.inputs:
                    continue
                self.frozen.add(n)
                stack += self.vertexInputs.get(n, [])
            return self

        def _lc(self, name):
            v = self.vertices[name]
            return _base(v.layerConf) if hasattr(v, "layerConf") else None

        def nOutReplace(self, name, nOut, weightInit=None, weightInitNext=None, dist=None, distNext=None):
            from .conf.weights import Distribution
            if isinstance(weightInit, Distribution):
                dist, weightInit = weightInit, "DISTRIBUTION"
            lc = self._lc(name)
            lc.nOut = int(nOut)
            if weightInit is not None:
                lc.weightInit = to_weight_init(weightInit)
            if dist is not None:
                lc.dist = dist
            self.reinit.add(name)
            for v, ins in self.vertexInputs.items():
                if name in ins and hasattr(self.vertices[v], "layerConf"):
                    nx = self._lc(v)
                    if isinstance(nx, FeedForwardLayer):
                        nx.nIn = int(nOut)
                        if weightInitNext is not None:
                            nx.weightInit = to_weight_init(weightInitNext)
                        if distNext is not None:
                            nx.dist = distNext
                        self.reinit.add(v)
            return self

        def removeVertexKeepConnections(self, name):
            self.vertices.pop(name)
            self.vertexInputs.pop(name)
            self.outputs = [o for o in self.outputs if o != name]
            return self

        def removeVertexAndConnections(self, name):
            self.removeVertexKeepConnections(name)
            for k in list(self.vertexInputs):
                self.vertexInputs[k] = [i for i in self.vertexInputs[k] if i != name]
            return self

        def addLayer(self, name, layer, *inputs):
            from .conf.graph import LayerVertex
            if hasattr(layer, "build") and not isinstance(layer, Layer):
                layer = layer.build()
            layer = copy.deepcopy(layer)
            if layer.layerName is None:
                layer.layerName = name
            layer.applyGlobal(self.globalConf)
            if hasattr(layer, "finalize_defaults"):
                layer.finalize_defaults()
            pp = None
            if inputs and not isinstance(inputs[0], str):
                pp, inputs = inputs[0], inputs[1:]
            self.vertices[name] = LayerVertex(layerConf=layer, preProcessor=pp)
            self.vertexInputs[name] = list(inputs)
            return self

        def addVertex(self, name, vertex, *inputs):
            self.vertices[name] = copy.deepcopy(vertex)
            self.vertexInputs[name] = list(inputs)
            return self

        def addInputs(self, *names):
            self.inputs += list(names)
            return self

        def setOutputs(self, *names):
            self.outputs = list(names)
            return self

        def build(self):
            from .conf.network import ComputationGraphConfiguration
            from .graph.computation_graph import ComputationGraph
            g = dict(self.globalConf)
            verts = {}
            for k, v in self.vertices.items():
                if hasattr(v, "layerConf"):
                    lc = _base(v.layerConf)
                    if self.ft is not None:
                        self.ft.applyToLayer(lc)
                    v.layerConf = FrozenLayer(layer=lc, layerName=lc.layerName) if k in self.frozen else lc
                verts[k] = v
            if self.ft is not None:
                self.ft.applyToGlobal(g)
            used = set(self.outputs)
            for ins in self.vertexInputs.values():
                used |= set(ins)
            conf = ComputationGraphConfiguration(
                vertices=verts, vertexInputs=self.vertexInputs, networkInputs=self.inputs,
                networkOutputs=self.outputs, backprop=self.oc.backprop, pretrain=self.oc.pretrain,
                backpropType=self.oc.backpropType, tbpttFwdLength=self.oc.tbpttFwdLength,
                tbpttBackLength=self.oc.tbpttBackLength, globalConf=g, inputTypes=self.oc.inputTypes)
            net = ComputationGraph(conf)
            net.init(device=self.orig.device)
            for name in verts:
                if name in self.reinit or not hasattr(verts[name], "layerConf"):
                    continue
                if name in self.orig.layers_by_name and name in net.layers_by_name:
                    _copy_params(net.layers_by_name[name], self.orig.layers_by_name[name])
            net._params_changed()
            return net


class TransferLearningHelper:
    """Featurize through the frozen front of a network once, then train only the unfrozen tail on the cached
    features (TransferLearningHelper.java). Works for MultiLayerNetwork whose first k layers are frozen (or
    given ``frozenTill``)."""

    def __init__(self, origModel, frozenTill=None):
        from .conf.network import MultiLayerConfiguration
        from .multilayer import MultiLayerNetwork
        self.orig = origModel
        if frozenTill is None:
            frozenTill = -1
            for i, c in enumerate(origModel.conf.confs):
                if isinstance(c, FrozenLayer):
                    frozenTill = i
        self.frozenTill = frozenTill
        oc = origModel.conf
        tail = [copy.deepcopy(_base(c)) for c in oc.confs[frozenTill + 1:]]
        pps = {k - frozenTill - 1: copy.deepcopy(v) for k, v in oc.inputPreProcessors.items() if k > frozenTill}
        conf = MultiLayerConfiguration(confs=tail, inputPreProcessors=pps, backpropType=oc.backpropType,
                                       tbpttFwdLength=oc.tbpttFwdLength, tbpttBackLength=oc.tbpttBackLength,
                                       globalConf=copy.deepcopy(dict(oc.globalConf)))
        self._tail = MultiLayerNetwork(conf)
        self._tail.init(device=origModel.device)
        for i in range(len(tail)):
            _copy_params(self._tail.layers[i], origModel.layers[frozenTill + 1 + i])
        self._tail._params_changed()

    def unfrozenMLN(self):
        return self._tail

    def featurize(self, ds):
        from ..datasets import DataSet
        with torch.no_grad():
            if self.frozenTill < 0:
                feats = ds.features
            else:
                acts = self.orig.feedForwardToLayer(self.frozenTill, ds.features, False)
                feats = acts[-1]
                pp = self.orig.conf.inputPreProcessors.get(self.frozenTill + 1)
                if pp is not None:
                    feats = pp.preProcess(feats, feats.shape[0])
        return DataSet(feats.float(), ds.labels, ds.featuresMask, ds.labelsMask)

    def fitFeaturized(self, data):
        self._tail.fit(data)
        for i in range(len(self._tail.layers)):
            _copy_params(self.orig.layers[self.frozenTill + 1 + i], self._tail.layers[i])
        self.orig._params_changed()

    def outputFromFeaturized(self, x):
        return self._tail.output(x)
