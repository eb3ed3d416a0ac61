"""Network-level configuration: NeuralNetConfiguration.Builder -> MultiLayerConfiguration /
ComputationGraphConfiguration (reference nn/conf/NeuralNetConfiguration.java:584-1262,
MultiLayerConfiguration.java:57-83,349-470, ComputationGraphConfiguration.java:59 (GraphBuilder)).

Global builder properties are inherited by every layer whose own value is unset. The JSON form
(``toJson``/``fromJson``) carries everything needed to rebuild the net, including iteration/epoch
counts so learning-rate schedules resume (MultiLayerConfiguration.java:80-83).
"""
import copy
import json

from ...exceptions import IllegalStateException
from .base import Config, _decode
from .enums import BackpropType, CacheMode, ConvolutionMode, DataType, OptimizationAlgorithm, WorkspaceMode
from .graph import GraphVertex, LayerVertex
from .inputs import InputType
from .layers import Layer
from .regularization import to_dropout
from .updaters import to_updater
from .weights import to_weight_init


_GLOBAL_DEFAULTS = {
    "seed": 12345, "optimizationAlgo": OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT, "miniBatch": True,
    "maxNumLineSearchIterations": 5, "minimize": True, "stepFunction": None,
    "trainingWorkspaceMode": WorkspaceMode.ENABLED, "inferenceWorkspaceMode": WorkspaceMode.ENABLED,
    "cacheMode": CacheMode.NONE, "dataType": DataType.FLOAT,
    # inheritable layer properties
    "activation": None, "weightInit": None, "biasInit": None, "dist": None, "l1": None, "l2": None,
    "l1Bias": None, "l2Bias": None, "updater": None, "biasUpdater": None, "weightNoise": None,
    "gradientNormalization": None, "gradientNormalizationThreshold": None, "idropout": None,
    "convolutionMode": None, "cudnnAlgoMode": None, "constraints": None,
}


class NeuralNetConfiguration:
    """Namespace holding the global ``Builder`` (reference class of the same name). ``Builder().layer(l).build()``
    gives the reference's single-layer configuration (``SingleLayerConfiguration``)."""

    @staticmethod
    def fromJson(s):
        return SingleLayerConfiguration.fromJson(s)

    @staticmethod
    def fromYaml(s):
        return SingleLayerConfiguration.fromYaml(s)

    class Builder:
        def __init__(self):
            self._g = dict(_GLOBAL_DEFAULTS)
            self._layer = None

        def layer(self, layer):
            """The single layer of a NeuralNetConfiguration (reference Builder.layer(Layer))."""
            if hasattr(layer, "build") and not isinstance(layer, Layer):
                layer = layer.build()
            self._layer = layer
            return self

        def _set(self, k, v):
            self._g[k] = v
            return self

        # hyperparameters ------------------------------------------------------------------
        def seed(self, s):
            return self._set("seed", int(s))

        def activation(self, a):
            from .activations import to_activation
            return self._set("activation", to_activation(a))

        def weightInit(self, w):
            from .weights import Distribution
            if isinstance(w, Distribution):
                self._set("dist", w)
                from .weights import WeightInit
                return self._set("weightInit", WeightInit.DISTRIBUTION)
            return self._set("weightInit", to_weight_init(w))

        def dist(self, d):
            return self._set("dist", d)

        def biasInit(self, b):
            return self._set("biasInit", float(b))

        def l1(self, v):
            return self._set("l1", float(v))

        def l2(self, v):
            return self._set("l2", float(v))

        def l1Bias(self, v):
            return self._set("l1Bias", float(v))

        def l2Bias(self, v):
            return self._set("l2Bias", float(v))

        def updater(self, u):
            return self._set("updater", to_updater(u))

        def biasUpdater(self, u):
            return self._set("biasUpdater", to_updater(u))

        def dropOut(self, d):
            return self._set("idropout", to_dropout(d))

        def weightNoise(self, w):
            return self._set("weightNoise", w)

        def gradientNormalization(self, g):
            from .enums import GradientNormalization
            return self._set("gradientNormalization", GradientNormalization.of(g))

        def gradientNormalizationThreshold(self, t):
            return self._set("gradientNormalizationThreshold", float(t))

        def convolutionMode(self, m):
            return self._set("convolutionMode", ConvolutionMode.of(m))

        def cudnnAlgoMode(self, m):
            from .enums import AlgoMode
            return self._set("cudnnAlgoMode", AlgoMode.of(m))

        def constrainWeights(self, *cs):
            out = []
            for c in cs:
                c = c.clone()
                c.params = ["W"]
                out.append(c)
            return self._set("constraints", (self._g.get("constraints") or []) + out)

        def constrainBias(self, *cs):
            out = []
            for c in cs:
                c = c.clone()
                c.params = ["b"]
                out.append(c)
            return self._set("constraints", (self._g.get("constraints") or []) + out)

        def constrainAllParameters(self, *cs):
            out = []
            for c in cs:
                c = c.clone()
                c.params = ["*"]
                out.append(c)
            return self._set("constraints", (self._g.get("constraints") or []) + out)

        def optimizationAlgo(self, a):
            return self._set("optimizationAlgo", OptimizationAlgorithm.of(a))

        def miniBatch(self, b):
            return self._set("miniBatch", bool(b))

        def maxNumLineSearchIterations(self, n):
            return self._set("maxNumLineSearchIterations", int(n))

        def minimize(self, b):
            return self._set("minimize", bool(b))

        def stepFunction(self, s):
            return self._set("stepFunction", s)

        def trainingWorkspaceMode(self, m):
            return self._set("trainingWorkspaceMode", WorkspaceMode.of(m))

        def inferenceWorkspaceMode(self, m):
            return self._set("inferenceWorkspaceMode", WorkspaceMode.of(m))

        def cacheMode(self, m):
            return self._set("cacheMode", CacheMode.of(m))

        def dataType(self, d):
            """Compute dtype policy (extension: FLOAT / BFLOAT16 / HALF / DOUBLE)."""
            return self._set("dataType", DataType.of(d))

        # deprecated reference knobs accepted for source compatibility
        def learningRate(self, lr):
            u = self._g.get("updater")
            if u is not None and hasattr(u, "learningRate"):
                u.learningRate = lr
            else:
                from .updaters import Sgd
                self._g["updater"] = Sgd(lr)
            return self

        def iterations(self, n):
            return self

        def regularization(self, b):
            return self

        def list(self, *layers):
            lb = ListBuilder(self._g)
            for i, l in enumerate(layers):
                lb.layer(i, l)
            return lb

        def graphBuilder(self):
            return GraphBuilder(self._g)

        def build(self):
            if self._layer is not None:
                return SingleLayerConfiguration.of(self._g, self._layer)
            return dict(self._g)


class SingleLayerConfiguration(Config):
    """The reference's single-layer NeuralNetConfiguration (nn/conf/NeuralNetConfiguration.java: one ``layer`` plus
    the settings that travel with it: seed, optimisation algorithm, minibatch / minimize flags, line-search
    iterations, step function, pretrain flag). The builder's inheritable properties are applied to the layer."""
    FIELDS = {"layer": None, "seed": 12345, "optimizationAlgo": OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT,
              "miniBatch": True, "minimize": True, "maxNumLineSearchIterations": 5, "stepFunction": None,
              "pretrain": False, "dataType": DataType.FLOAT}

    @classmethod
    def of(cls, g, layer):
        layer = copy.deepcopy(layer)
        if hasattr(layer, "applyGlobal"):
            layer.applyGlobal(g)
        if hasattr(layer, "finalize_defaults"):
            layer.finalize_defaults()
        return cls(layer=layer, **{k: g[k] for k in ("seed", "optimizationAlgo", "miniBatch", "minimize",
                                                      "maxNumLineSearchIterations", "stepFunction", "dataType")
                                   if k in g})

    def to_dict(self):
        d = super().to_dict()
        if self.stepFunction is not None and not isinstance(self.stepFunction, Config):
            d["stepFunction"] = {"@stepFunction": type(self.stepFunction).__name__}
        return d

    @classmethod
    def from_dict(cls, d):
        sf = d.get("stepFunction")
        if isinstance(sf, dict) and "@stepFunction" in sf:
            from ...optimize import solvers
            d = dict(d)
            d["stepFunction"] = None
            obj = super().from_dict(d)
            obj.stepFunction = getattr(solvers, sf["@stepFunction"])()
            return obj
        return super().from_dict(d)

    def __eq__(self, other):
        if type(self) is not type(other):
            return False
        a, b = self.to_dict(), other.to_dict()
        return a == b

    __hash__ = Config.__hash__

    def getLayer(self):
        return self.layer

    def setLayer(self, layer):
        self.layer = layer

    def isPretrain(self):
        return bool(self.pretrain)

    def setPretrain(self, b):
        self.pretrain = bool(b)

    def getStepFunction(self):
        return self.stepFunction

    def setStepFunction(self, f):
        self.stepFunction = f

    def getL1ByParam(self, key):
        return self.layer.l1For(key)

    def getL2ByParam(self, key):
        return self.layer.l2For(key)

    def getVariables(self):
        return [s.key for s in self.layer.param_specs()] if hasattr(self.layer, "param_specs") else []

    def toYaml(self):
        import yaml
        return yaml.safe_dump(json.loads(self.toJson()), sort_keys=True)

    @classmethod
    def fromYaml(cls, s):
        import yaml
        return _decode(yaml.safe_load(s))


class ListBuilder:
    def __init__(self, g):
        self._g = g
        self._layers = {}
        self._pp = {}
        self._inputType = None
        self._backprop = True
        self._pretrain = False
        self._bpType = BackpropType.Standard
        self._fwd = 20
        self._back = 20

    def layer(self, idx, layer=None):
        if layer is None:
            layer, idx = idx, len(self._layers)
        if hasattr(layer, "build") and not isinstance(layer, Layer):
            layer = layer.build()
        self._layers[int(idx)] = layer
        return self

    def inputPreProcessor(self, idx, pp):
        self._pp[int(idx)] = pp
        return self

    def setInputType(self, t):
        self._inputType = t
        return self

    def backprop(self, b):
        self._backprop = bool(b)
        return self

    def pretrain(self, b):
        self._pretrain = bool(b)
        return self

    def backpropType(self, t):
        self._bpType = BackpropType.of(t)
        return self

    def tBPTTLength(self, n):
        self._fwd = self._back = int(n)
        return self

    def tBPTTForwardLength(self, n):
        self._fwd = int(n)
        return self

    def tBPTTBackwardLength(self, n):
        self._back = int(n)
        return self

    def trainingWorkspaceMode(self, m):
        self._g["trainingWorkspaceMode"] = WorkspaceMode.of(m)
        return self

    def inferenceWorkspaceMode(self, m):
        self._g["inferenceWorkspaceMode"] = WorkspaceMode.of(m)
        return self

    def cacheMode(self, m):
        self._g["cacheMode"] = CacheMode.of(m)
        return self

    @staticmethod
    def _infer_input_type(confs, pps):
        """No setInputType: a first recurrent layer with nIn implies recurrent input, a first Dense / Embedding /
        Output layer with nIn implies feed-forward input (convolutional input cannot be guessed), so the FF<->RNN
        preprocessors still get added (reference MultiLayerConfiguration.Builder.build)."""
        from .layers import DenseLayer, EmbeddingLayer, OutputLayer
        if not confs or 0 in pps:
            return None
        first = confs[0]
        n_in = getattr(first, "nIn", 0) or 0
        if n_in <= 0:
            return None
        from .layers import Bidirectional, GravesBidirectionalLSTM, GravesLSTM, LSTM, SimpleRnn
        if isinstance(first, (LSTM, GravesLSTM, GravesBidirectionalLSTM, SimpleRnn)) and \
                not isinstance(first, Bidirectional):
            return InputType.recurrent(n_in)
        if type(first) in (DenseLayer, EmbeddingLayer, OutputLayer):
            return InputType.feedForward(n_in)
        return None

    def build(self):
        n = len(self._layers)
        if n == 0:
            raise IllegalStateException("Invalid configuration: no layers defined")
        if sorted(self._layers) != list(range(n)):
            raise IllegalStateException(f"Invalid configuration: layer indices must be contiguous from 0: got "
                                        f"{sorted(self._layers)}")
        confs = [copy.deepcopy(self._layers[i]) for i in range(n)]
        g = self._g
        for c in confs:
            c.applyGlobal(g)
        pps = dict(self._pp)
        t = self._inputType if self._inputType is not None else self._infer_input_type(confs, pps)
        if t is not None:
            for i, c in enumerate(confs):
                if i not in pps:
                    pp = c.getPreProcessorForInputType(t)
                    if pp is not None:
                        pps[i] = pp
                if i in pps:
                    t = pps[i].getOutputType(t)
                c.setNIn(t, False)
                t = c.getOutputType(i, t)
        for i, c in enumerate(confs):
            if hasattr(c, "finalize_defaults"):
                c.finalize_defaults()
            if c.layerName is None:
                c.layerName = f"layer{i}"
        return MultiLayerConfiguration(
            confs=confs, inputPreProcessors=pps, backprop=self._backprop, pretrain=self._pretrain,
            backpropType=self._bpType, tbpttFwdLength=self._fwd, tbpttBackLength=self._back,
            globalConf={k: v for k, v in g.items() if k in _NET_KEYS}, inputType=self._inputType)


_NET_KEYS = ("seed", "optimizationAlgo", "miniBatch", "maxNumLineSearchIterations", "minimize", "stepFunction",
             "trainingWorkspaceMode", "inferenceWorkspaceMode", "cacheMode", "dataType")


class _Counters:
    """Training-progress counters kept in the configuration (reference MultiLayerConfiguration /
    ComputationGraphConfiguration iterationCount / epochCount, serialised with it)."""

    def getIterationCount(self):
        return self.iterationCount

    def setIterationCount(self, n):
        self.iterationCount = int(n)

    def getEpochCount(self):
        return self.epochCount

    def setEpochCount(self, n):
        self.epochCount = int(n)


class LayerConfiguration:
    """The per-layer NeuralNetConfiguration view returned by ``MultiLayerConfiguration.getConf(i)``
    (reference NeuralNetConfiguration.getLayer / getVariables); attributes resolve on the wrapped layer config."""

    __slots__ = ("_layer",)

    def __init__(self, layer):
        object.__setattr__(self, "_layer", layer)

    def getLayer(self):
        return self._layer

    def setLayer(self, layer):
        object.__setattr__(self, "_layer", layer)

    def getVariables(self):
        return [s.key for s in self._layer.param_specs()] if hasattr(self._layer, "param_specs") else []

    def __getattr__(self, name):
        return getattr(self._layer, name)

    def __setattr__(self, name, value):
        setattr(self._layer, name, value)

    def __eq__(self, other):
        return self._layer == (other._layer if isinstance(other, LayerConfiguration) else other)

    def __repr__(self):
        return f"LayerConfiguration({self._layer!r})"


class MultiLayerConfiguration(_Counters, Config):
    FIELDS = {"confs": [], "inputPreProcessors": {}, "backprop": True, "pretrain": False,
              "backpropType": BackpropType.Standard, "tbpttFwdLength": 20, "tbpttBackLength": 20,
              "globalConf": {}, "iterationCount": 0, "epochCount": 0, "inputType": None}

    def __eq__(self, other):
        # the reference's @Data equality: the builder's input type is not part of the built configuration
        # (MultiLayerConfiguration.java:51 vs Builder.inputType :357), so a configuration completed by shape inference
        # equals the hand-written one (ConvolutionLayerSetupTest.testConvolutionLayerSetup)
        if type(self) is not type(other):
            return False
        a, b = self.to_dict(), other.to_dict()
        a.pop("inputType", None)
        b.pop("inputType", None)
        return a == b

    __hash__ = Config.__hash__

    def getConf(self, i):
        """Layer i's configuration as the reference's per-layer NeuralNetConfiguration: ``getLayer()`` is the layer
        config; every other attribute reads through to it (this framework keeps one object per layer)."""
        return LayerConfiguration(self.confs[i])

    def getMemoryReport(self, inputType=None):
        """Per-layer memory estimates (reference MultiLayerConfiguration.getMemoryReport)."""
        from .memory import mln_memory_report
        return mln_memory_report(self, inputType)

    def getInputPreProcess(self, i):
        return self.inputPreProcessors.get(i)

    def getInputPreProcessors(self):
        return self.inputPreProcessors

    @property
    def seed(self):
        return self.globalConf.get("seed", 12345)

    @property
    def dataType(self):
        return DataType.of(self.globalConf.get("dataType", DataType.FLOAT))

    def setDataType(self, d):
        self.globalConf["dataType"] = DataType.of(d)

    def toYaml(self):
        import yaml
        return yaml.safe_dump(json.loads(self.toJson()), sort_keys=True)

    @staticmethod
    def fromYaml(s):
        import yaml
        return MultiLayerConfiguration.fromJson(yaml.safe_load(s))

    def toJson(self):
        """DL4J's Jackson schema (see nn/conf/dl4j_json.py): readable by the reference's MultiLayerConfiguration."""
        from .dl4j_json import to_json
        return to_json(self)

    @staticmethod
    def fromJson(s):
        from .dl4j_json import from_json, is_dl4j_format
        d = json.loads(s) if isinstance(s, str) else s
        return from_json(d) if is_dl4j_format(d) else _decode(d)


class GraphBuilder:
    def __init__(self, g):
        self._g = g
        self._inputs = []
        self._outputs = []
        self._vertices = {}
        self._vertexInputs = {}
        self._inputTypes = None
        self._backprop = True
        self._pretrain = False
        self._bpType = BackpropType.Standard
        self._fwd = 20
        self._back = 20
        self._order = []
        self._allowDisconnected = False

    def allowDisconnected(self, b=True):
        """Permit inputs / vertices from which no network output is reachable (reference
        GraphBuilder.allowDisconnected); otherwise build() rejects them."""
        self._allowDisconnected = bool(b)
        return self

    def addInputs(self, *names):
        self._inputs += [n for ns in names for n in (ns if isinstance(ns, (list, tuple)) else [ns])]
        return self

    def setOutputs(self, *names):
        self._outputs = [n for ns in names for n in (ns if isinstance(ns, (list, tuple)) else [ns])]
        return self

    def addLayer(self, name, layer, *inputs):
        pp = None
        if inputs and not isinstance(inputs[0], str):
            pp, inputs = inputs[0], inputs[1:]
        if hasattr(layer, "build") and not isinstance(layer, Layer):
            layer = layer.build()
        layer = copy.deepcopy(layer)
        if layer.layerName is None:
            layer.layerName = name
        self._vertices[name] = LayerVertex(layerConf=layer, preProcessor=pp)
        self._vertexInputs[name] = list(inputs)
        self._order.append(name)
        return self

    def layer(self, name, layer, *inputs):
        return self.addLayer(name, layer, *inputs)

    def addVertex(self, name, vertex, *inputs):
        self._vertices[name] = copy.deepcopy(vertex)
        self._vertexInputs[name] = list(inputs)
        self._order.append(name)
        return self

    def removeVertex(self, name, removeConnections=True):
        self._vertices.pop(name, None)
        self._vertexInputs.pop(name, None)
        self._order = [n for n in self._order if n != name]
        if removeConnections:
            for k in self._vertexInputs:
                self._vertexInputs[k] = [i for i in self._vertexInputs[k] if i != name]
            self._outputs = [o for o in self._outputs if o != name]
        return self

    def setInputTypes(self, *types):
        self._inputTypes = list(types)
        return self

    def inputPreProcessor(self, name, pp):
        self._vertices[name].preProcessor = pp
        return self

    def backprop(self, b):
        self._backprop = bool(b)
        return self

    def pretrain(self, b):
        self._pretrain = bool(b)
        return self

    def backpropType(self, t):
        self._bpType = BackpropType.of(t)
        return self

    def tBPTTLength(self, n):
        self._fwd = self._back = int(n)
        return self

    def tBPTTForwardLength(self, n):
        self._fwd = int(n)
        return self

    def tBPTTBackwardLength(self, n):
        self._back = int(n)
        return self

    # vertices that consume exactly one activation: given several inputs they get a MergeVertex "<name>-merge" in
    # front of them (reference GraphBuilder.build, TestComputationGraphNetwork.testMergeVertexAddition)
    _SINGLE_INPUT = ("LayerVertex", "L2NormalizeVertex", "ScaleVertex", "ShiftVertex", "ReshapeVertex", "SubsetVertex",
                     "PreprocessorVertex", "PoolHelperVertex", "UnstackVertex", "DuplicateToTimeSeriesVertex",
                     "LastTimeStepVertex")

    def _add_merge_vertices(self):
        from .graph import MergeVertex
        for name in list(self._order):
            ins = self._vertexInputs.get(name, [])
            if len(ins) < 2 or type(self._vertices[name]).__name__ not in self._SINGLE_INPUT:
                continue
            mname = f"{name}-merge"
            self._vertices[mname] = MergeVertex()
            self._vertexInputs[mname] = list(ins)
            self._vertexInputs[name] = [mname]
            # right after its consumer, as the reference's builder adds it (vertex indices follow this order)
            self._order.insert(self._order.index(name) + 1, mname)

    def build(self):
        if not self._inputs:
            raise IllegalStateException("ComputationGraph must have at least one input (addInputs)")
        if not self._outputs:
            raise IllegalStateException("ComputationGraph must have at least one output (setOutputs)")
        names = set(self._vertices) | set(self._inputs)
        for v in self._vertices:
            if not self._vertexInputs.get(v):
                # reference ComputationGraphConfiguration.validate:299, checked before the disconnected vertices
                raise IllegalStateException(f"Invalid configuration: vertex {v!r} has no inputs")
        for v, ins in self._vertexInputs.items():
            for i in ins:
                if i not in names:
                    raise IllegalStateException(f"Vertex {v!r} has unknown input {i!r}")
        for o in self._outputs:
            if o not in self._vertices:
                raise IllegalStateException(f"Output {o!r} is not a vertex")
        if not self._allowDisconnected:
            # every input and vertex must lead to an output (reference ComputationGraphConfiguration.validate)
            reach, stack = set(self._outputs), list(self._outputs)
            while stack:
                for i in self._vertexInputs.get(stack.pop(), []):
                    if i not in reach:
                        reach.add(i)
                        stack.append(i)
            dis = [n for n in list(self._inputs) + list(self._order) if n not in reach]
            if dis:
                from ...exceptions import DL4JInvalidConfigException
                raise DL4JInvalidConfigException(
                    f"Invalid configuration: disconnected vertices found - {dis} are not connected to the network "
                    "output; use .allowDisconnected(True) to build it anyway")
        self._add_merge_vertices()
        conf = ComputationGraphConfiguration(
            vertices={k: self._vertices[k] for k in self._order}, vertexInputs=dict(self._vertexInputs),
            networkInputs=list(self._inputs), networkOutputs=list(self._outputs), backprop=self._backprop,
            pretrain=self._pretrain, backpropType=self._bpType, tbpttFwdLength=self._fwd,
            tbpttBackLength=self._back, globalConf={k: v for k, v in self._g.items() if k in _NET_KEYS},
            inputTypes=self._inputTypes)
        for v in conf.vertices.values():
            if isinstance(v, LayerVertex):
                v.layerConf.applyGlobal(self._g)
        if self._inputTypes is not None:
            conf.addPreProcessorsAndInferNIn()
        for v in conf.vertices.values():
            if isinstance(v, LayerVertex) and hasattr(v.layerConf, "finalize_defaults"):
                v.layerConf.finalize_defaults()
        return conf


class ComputationGraphConfiguration(_Counters, Config):
    FIELDS = {"vertices": {}, "vertexInputs": {}, "networkInputs": [], "networkOutputs": [], "backprop": True,
              "pretrain": False, "backpropType": BackpropType.Standard, "tbpttFwdLength": 20,
              "tbpttBackLength": 20, "globalConf": {}, "iterationCount": 0, "epochCount": 0, "inputTypes": None}

    @property
    def seed(self):
        return self.globalConf.get("seed", 12345)

    @property
    def dataType(self):
        return DataType.of(self.globalConf.get("dataType", DataType.FLOAT))

    def setDataType(self, d):
        self.globalConf["dataType"] = DataType.of(d)

    def getMemoryReport(self, *inputTypes):
        from .memory import cg_memory_report
        return cg_memory_report(self, list(inputTypes) or None)

    # reference ComputationGraphConfiguration getters
    def getVertices(self):
        return self.vertices

    def getVertexInputs(self):
        return self.vertexInputs

    def getNetworkInputs(self):
        return list(self.networkInputs)

    def getNetworkOutputs(self):
        return list(self.networkOutputs)

    def topologicalOrder(self):
        """Kahn's algorithm, ties broken by insertion order (reference ComputationGraph.java:1216-1318)."""
        all_names = list(self.networkInputs) + [k for k in self.vertices]
        indeg = {n: 0 for n in all_names}
        outs = {n: [] for n in all_names}
        for v, ins in self.vertexInputs.items():
            for i in ins:
                indeg[v] += 1
                outs[i].append(v)
        queue = [n for n in all_names if indeg[n] == 0]
        order = []
        while queue:
            n = queue.pop(0)
            order.append(n)
            for m in outs[n]:
                indeg[m] -= 1
                if indeg[m] == 0:
                    queue.append(m)
        if len(order) != len(all_names):
            raise IllegalStateException("Invalid ComputationGraph configuration: graph contains a cycle")
        return order

    def addPreProcessorsAndInferNIn(self):
        types = {}
        for name, t in zip(self.networkInputs, self.inputTypes):
            types[name] = t
        for i, name in enumerate(self.topologicalOrder()):
            if name in self.networkInputs:
                continue
            v = self.vertices[name]
            ins = [types[x] for x in self.vertexInputs[name]]
            if isinstance(v, LayerVertex):
                t = ins[0]
                if len(ins) > 1:
                    from .graph import MergeVertex
                    t = MergeVertex().getOutputType(i, *ins)
                if v.preProcessor is None:
                    v.preProcessor = v.layerConf.getPreProcessorForInputType(t)
                if v.preProcessor is not None:
                    t = v.preProcessor.getOutputType(t)
                v.layerConf.setNIn(t, False)
                types[name] = v.layerConf.getOutputType(i, t)
            else:
                types[name] = v.getOutputType(i, *ins)
        self._types = types
        return types

    def getLayerActivationTypes(self):
        return getattr(self, "_types", None) or self.addPreProcessorsAndInferNIn()

    def toJson(self):
        """DL4J's Jackson schema (see nn/conf/dl4j_json.py): readable by the reference's
        ComputationGraphConfiguration."""
        from .dl4j_json import to_json
        return to_json(self)

    @staticmethod
    def fromJson(s):
        from .dl4j_json import from_json, is_dl4j_format
        d = json.loads(s) if isinstance(s, str) else s
        return from_json(d) if is_dl4j_format(d) else _decode(d)

    def toYaml(self):
        import yaml
        return yaml.safe_dump(json.loads(self.toJson()), sort_keys=True)

    @staticmethod
    def fromYaml(s):
        import yaml
        return ComputationGraphConfiguration.fromJson(yaml.safe_load(s))


_ = (GraphVertex, InputType)
