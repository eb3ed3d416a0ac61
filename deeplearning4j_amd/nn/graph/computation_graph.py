"""ComputationGraph: DAG model (reference nn/graph/ComputationGraph.java, 3904 LoC).

* topological order by Kahn's algorithm (:1216-1318); flat params in topological order (:401-470)
* forward in topological order (:1577-1700); backward in reverse topological order with epsilon
  summation for fan-out (:1947-2107, sum at :2044-2063)
* multi-input / multi-output; score = sum of output-layer losses + L1/L2 once (:1360-1373)
* TBPTT (:2894), rnnTimeStep (:2720)
Planner: BatchNormalization -> ActivationLayer(ReLU) pairs where the BN output has a single consumer
are fused so the HIP BN kernel applies the ReLU (ResNet-50: 49 such pairs).
"""
import os

import torch

from ...datasets.dataset import DataSet, MultiDataSet
from ..conf.enums import BackpropType
from ..conf.graph import LayerVertex
from ..conf.layers import ActivationLayer, BatchNormalization
from ..conf.validation import check_layer_input, validate_network_conf
from ...exceptions import DL4JInvalidInputException
from ..layers.output import BaseOutputLayerImpl
from ..network_base import BaseNetwork
from ... import profiling as _prof


def _shares_storage(a, b):
    """True when the bytes addressed by tensors a and b overlap. Spans, not storages: arena tensors are carved from
    one shared storage (memory/arena.py) and must not count as aliases of each other."""
    if a is None or b is None or not torch.is_tensor(a) or not torch.is_tensor(b) or a.device != b.device:
        return False
    if a.numel() == 0 or b.numel() == 0:
        return False

    def span(t):
        n = 1 + sum((s - 1) * abs(st) for s, st in zip(t.shape, t.stride()))
        return t.data_ptr(), t.data_ptr() + n * t.element_size()
    a0, a1 = span(a)
    b0, b1 = span(b)
    return a0 < b1 and b0 < a1



def _out_dtype(t):
    """16-bit activations come back as fp32 (the reference's output dtype); fp32/fp64 graphs keep theirs."""
    return t.float() if t.dtype in (torch.bfloat16, torch.float16) else t

class ComputationGraph(BaseNetwork):
    _key_by_name = True

    def __init__(self, conf, params=None):
        super().__init__(conf)
        self._init_params = params
        self.inputs = None
        self.labels = None
        self.inputMaskArrays = None
        self.labelMaskArrays = None

    # ------------------------------------------------------------------------------ init
    def init(self, parameters=None, cloneParametersArray=False, device=None):
        if self.initCalled and parameters is None:
            return
        parameters = parameters if parameters is not None else self._init_params
        conf = self.conf
        if conf.inputTypes is not None and not hasattr(conf, "_types"):
            conf.addPreProcessorsAndInferNIn()
        self.topo = [n for n in conf.topologicalOrder() if n not in conf.networkInputs]
        validate_network_conf({n: conf.vertices[n].layerConf for n in self.topo
                               if isinstance(conf.vertices[n], LayerVertex)})
        self.vertex_inputs = conf.vertexInputs
        self.consumers = {n: [] for n in list(conf.networkInputs) + self.topo}
        for v in self.topo:
            for i in self.vertex_inputs[v]:
                self.consumers[i].append(v)
        self.layers_by_name = {}
        layer_list = []
        for idx, name in enumerate(self.topo):
            v = conf.vertices[name]
            if isinstance(v, LayerVertex):
                impl = v.layerConf.instantiate(index=idx, net=self)
                self.layers_by_name[name] = impl
                layer_list.append((idx, name, impl))
        self._setup_flat(layer_list, parameters, cloneParametersArray, device)
        self.outputs = list(conf.networkOutputs)
        self._plan_fusions()
        for l in self.layers_by_name.values():
            if hasattr(l, "bind"):
                l.bind()

    def _plan_fusions(self):
        """Graph-level fusion planner (MI355X: fewer HBM passes over the activations).

        * BN -> ActivationLayer(ReLU)                      => ReLU inside the BN apply kernel
        * BN -> ElementWiseVertex(Add, shortcut) -> ReLU   => y = relu(bn(x) + shortcut) in ONE kernel
          (every ResNet bottleneck block); backward emits d(shortcut) from the same pass.
        * BN -> ReLU -> SubsamplingLayer(MAX)             => BN + ReLU + max pool in one pass (ResNet stem); the
          backward takes the BN reductions over the pooled gradient and gathers dx in one more pass.
        Fused-away vertices become passthroughs: forward copies the producer's activation, backward routes
        epsilon to that single producer. Also computes which vertices need an input gradient at all
        (nothing trainable upstream => skip dL/dinput, e.g. the stem conv's backward-data)."""
        from ..conf.activations import ActivationReLU
        from ..conf.graph import ElementWiseVertex
        self._passthrough = {}
        self._residual_of = {}
        pos = {n: i for i, n in enumerate(self.topo)}
        for n in self.conf.networkInputs:
            pos[n] = -1

        def is_relu_layer(n):
            vv = self.conf.vertices.get(n)
            return isinstance(vv, LayerVertex) and isinstance(vv.layerConf, ActivationLayer) and \
                isinstance(vv.layerConf.activation, ActivationReLU) and vv.preProcessor is None and \
                vv.layerConf.idropout is None and len(self.vertex_inputs[n]) == 1

        def is_max_pool(n):
            from ..conf.layers import SubsamplingLayer
            vv = self.conf.vertices.get(n)
            if not (isinstance(vv, LayerVertex) and type(vv.layerConf) is SubsamplingLayer) or \
                    vv.preProcessor is not None or vv.layerConf.idropout is not None or \
                    len(self.vertex_inputs[n]) != 1:
                return False
            lc = vv.layerConf
            return lc.poolingType.value == "MAX" and tuple(lc.dilation) == (1, 1)

        for name in self.topo:
            v = self.conf.vertices[name]
            if not (isinstance(v, LayerVertex) and isinstance(v.layerConf, BatchNormalization)):
                continue
            if v.layerConf.idropout is not None:
                continue
            cons = self.consumers[name]
            if len(cons) != 1 or name in self.outputs:
                continue
            nxt_name = cons[0]
            nxt = self.conf.vertices[nxt_name]
            if isinstance(nxt, ElementWiseVertex) and nxt.op == "Add" and len(self.vertex_inputs[nxt_name]) == 2 \
                    and nxt_name not in self.outputs and len(self.consumers[nxt_name]) == 1 \
                    and is_relu_layer(self.consumers[nxt_name][0]) and os.environ.get("DL4J_AMD_FUSE_RES", "1") == "1":
                ins = self.vertex_inputs[nxt_name]
                other = ins[1] if ins[0] == name else ins[0]
                relu_name = self.consumers[nxt_name][0]
                if other != name and pos[other] < pos[name] and relu_name not in self.outputs:
                    self.layers_by_name[name].fuse_relu = True
                    self._residual_of[name] = other
                    self._passthrough[nxt_name] = name
                    self._passthrough[relu_name] = nxt_name
                    # the shortcut branch ends in its own BN (ResNet convBlock: conv -> BN -> add): in training that BN
                    # only folds its statistics and this layer applies both normalisations in one pass (forward) and
                    # runs both backwards from one partial-sum pass (csrc/batchnorm.hip RBN kernels)
                    ov = self.conf.vertices.get(other)
                    if isinstance(ov, LayerVertex) and isinstance(ov.layerConf, BatchNormalization) and \
                            ov.layerConf.idropout is None and ov.preProcessor is None and \
                            self.consumers.get(other) == [nxt_name] and other not in self.outputs and \
                            not getattr(ov.layerConf, "useLogStd", False) and \
                            os.environ.get("DL4J_AMD_FUSE_RES_BN", "1") == "1":
                        self.layers_by_name[name].residual_bn = self.layers_by_name[other]
                        self.layers_by_name[other].defer_apply = True
                    continue
            if is_relu_layer(nxt_name) and nxt_name not in self.outputs:
                self.layers_by_name[name].fuse_relu = True
                self._passthrough[nxt_name] = name
                # BN -> ReLU -> max SubsamplingLayer (ResNet stem): pool inside the BN pass as well
                pc = self.consumers[nxt_name]
                if len(pc) == 1 and pc[0] not in self.outputs and is_max_pool(pc[0]) and \
                        os.environ.get("DL4J_AMD_FUSE_POOL", "1") == "1":
                    self.layers_by_name[name].fuse_pool = self.layers_by_name[pc[0]]
                    self._passthrough[pc[0]] = nxt_name
        # ZeroPadding -> Convolution(Truncate): fold the zero padding into the convolution's own (possibly
        # asymmetric) padding, so the padded activation is never materialised (ResNet-50 stem: a 40M-element copy)
        from ..conf.layers import ConvolutionLayer, ZeroPaddingLayer
        from ..conf.enums import ConvolutionMode
        for name in self.topo:
            v = self.conf.vertices[name]
            if not (isinstance(v, LayerVertex) and isinstance(v.layerConf, ZeroPaddingLayer)) or \
                    name in self.outputs or len(self.consumers[name]) != 1 or \
                    os.environ.get("DL4J_AMD_FOLD_PAD", "1") != "1":
                continue
            cn = self.consumers[name][0]
            cv = self.conf.vertices[cn]
            if not (isinstance(cv, LayerVertex) and type(cv.layerConf) is ConvolutionLayer) or \
                    cv.preProcessor is not None or cv.layerConf.convolutionMode != ConvolutionMode.Truncate or \
                    len(self.vertex_inputs[cn]) != 1 or len(self.vertex_inputs[name]) != 1:
                continue
            p = list(v.layerConf.padding)
            self.layers_by_name[cn].extra_pad4 = (p[0], p[1], p[2], p[3])
            self._passthrough[name] = self.vertex_inputs[name][0]
        # Conv(+bias, identity activation) -> training-mode BatchNormalization: the bias cancels inside the batch
        # normalisation, so the conv skips the bias add while training and BN adds (1-decay)*bias to its running
        # mean instead (exact; saves a full read+write of the conv output when the library conv is used)
        for name in self.topo:
            v = self.conf.vertices[name]
            if not (isinstance(v, LayerVertex) and type(v.layerConf) is ConvolutionLayer) or name in self.outputs \
                    or len(self.consumers[name]) != 1 or os.environ.get("DL4J_AMD_DEFER_BIAS", "1") != "1":
                continue
            impl = self.layers_by_name[name]
            if "b" not in impl.params or type(v.layerConf.activation).__name__ != "ActivationIdentity":
                continue
            if v.layerConf.nIn % 8 == 0 and v.layerConf.nOut % 4 == 0 and \
                    os.environ.get("DL4J_AMD_DEFER_BIAS", "1") != "all":
                # the MFMA conv kernels fuse the bias into their epilogue for free; deferring would only add a
                # small running-mean launch per layer. Defer where the library conv runs (e.g. the C=3 stem).
                continue
            bn_name = self.consumers[name][0]
            bv = self.conf.vertices[bn_name]
            if not (isinstance(bv, LayerVertex) and isinstance(bv.layerConf, BatchNormalization)) or \
                    bv.preProcessor is not None or len(self.vertex_inputs[bn_name]) != 1:
                continue
            impl.defer_bias = True
            self.layers_by_name[bn_name].deferred_bias = impl
        # Conv (identity activation) -> training-mode BatchNormalization: the MFMA conv kernel emits per-tile BN
        # statistics from its epilogue, so BN skips its own full statistics pass over the conv output
        for name in self.topo:
            v = self.conf.vertices[name]
            if not (isinstance(v, LayerVertex) and type(v.layerConf) is ConvolutionLayer) or name in self.outputs \
                    or len(self.consumers[name]) != 1 or os.environ.get("DL4J_AMD_CONV_BN_STATS", "1") != "1":
                continue
            if type(v.layerConf.activation).__name__ != "ActivationIdentity" or v.layerConf.idropout is not None:
                continue
            bv = self.conf.vertices[self.consumers[name][0]]
            if isinstance(bv, LayerVertex) and isinstance(bv.layerConf, BatchNormalization) and \
                    bv.preProcessor is None and bv.layerConf.idropout is None and \
                    not getattr(bv.layerConf, "useLogStd", False):
                self.layers_by_name[name].emit_bn_stats = True
        # which vertices must produce an input gradient
        flows = {n: False for n in self.conf.networkInputs}
        self._need_input_grad = {}
        for name in self.topo:
            ins = self.vertex_inputs[name]
            need = any(flows.get(i, False) for i in ins)
            self._need_input_grad[name] = need
            layer = self.layers_by_name.get(name)
            own = layer is not None and layer.conf.numParams() > 0
            flows[name] = need or own
        for name, layer in self.layers_by_name.items():
            layer.need_input_grad = self._need_input_grad[name]

    def getLayers(self):
        return list(self.layers_by_name.values())

    def getLayer(self, name):
        if isinstance(name, int):
            return self.getLayers()[name]
        return self.layers_by_name[name]

    def getVertex(self, name):
        """The runtime vertex (reference nn/graph/vertex/GraphVertex): name / index / layer accessors and
        setLayerAsFrozen(); configuration attributes read through to the vertex configuration."""
        return _RuntimeVertex(self, name)

    def getVertices(self):
        """Runtime vertices in the index space of topologicalSortOrder(): network inputs first, then the vertices
        in the order they were added."""
        return [_RuntimeVertex(self, n) for n in list(self.conf.networkInputs) + list(self.conf.vertices)]

    def _replace_impl(self, idx, name, old, new):
        self.layers_by_name[name] = new

    def _summary_types(self, inputTypes):
        import copy
        c = copy.deepcopy(self.conf)
        c.inputTypes = list(inputTypes)
        types = c.addPreProcessorsAndInferNIn()
        out = {}
        for name in self.layers_by_name:
            ins = [types[i] for i in c.vertexInputs[name]]
            out[name] = (ins[0] if len(ins) == 1 else ins, types[name])
        return out

    def getNumLayers(self):
        return len(self.layers_by_name)

    def getOutputLayer(self, i):
        return self.layers_by_name[self.outputs[i]]

    def getConfiguration(self):
        return self.conf

    # ------------------------------------------------------------------------------ forward
    def _prep_inputs(self, inputs):
        if torch.is_tensor(inputs) or not isinstance(inputs, (list, tuple)):
            inputs = [inputs]
        out = []
        for x in inputs:
            if not torch.is_tensor(x):
                import numpy as np
                x = torch.from_numpy(np.asarray(x))
            x = x.toTensor() if hasattr(x, "toTensor") else x
            out.append(self._to_dev(x, self._feat_dtype()) if x.is_floating_point() else self._to_dev(x))
        return out

    def feedForward(self, inputs=None, train=False, masks=None, stored_state=False, store_last_for_tbptt=False,
                    layerTillIndex=None):
        if isinstance(inputs, bool):            # reference feedForward(boolean train) on the set inputs
            inputs, train = None, inputs
        inputs = self._prep_inputs(self.inputs if inputs is None else inputs)
        if len(inputs) != len(self.conf.networkInputs):
            raise DL4JInvalidInputException(f"ComputationGraph has {len(self.conf.networkInputs)} inputs "
                                            f"{list(self.conf.networkInputs)}, got {len(inputs)} arrays")
        chk = self._input_check(inputs)
        idx = self._index_checked()
        if masks is None:
            masks = self.inputMaskArrays
        acts = {}
        amask = {}
        active = {}                 # feature-mask state per vertex: False once an LSTM passed the mask through
        mb = inputs[0].shape[0]
        self._prep_mb = mb
        for i, n in enumerate(self.conf.networkInputs):
            acts[n] = inputs[i]
            amask[n] = masks[i] if masks is not None and i < len(masks) else None
            active[n] = True
        self._ctx = {}
        for name in self.topo:
            v = self.conf.vertices[name]
            ins = [acts[i] for i in self.vertex_inputs[name]]
            ms = [amask.get(i) for i in self.vertex_inputs[name]]
            active[name] = any(active.get(i, True) for i in self.vertex_inputs[name])
            if isinstance(v, LayerVertex):
                x = ins[0] if len(ins) == 1 else torch.cat(ins, dim=1)
                if len(ins) > 1:
                    self._ctx[name] = ("merge", [t.shape[1] for t in ins])
                mask = ms[0] if ms else None
                if v.preProcessor is not None:
                    x = v.preProcessor.preProcess(x, mb, train)
                    if mask is not None:
                        mask, _ = v.preProcessor.feedForwardMaskArray(mask, None, mb)
                if chk is not None or name in idx:
                    check_layer_input(v.layerConf, x, name)
                if name in self._passthrough:
                    acts[name] = acts[self._passthrough[name]]
                    amask[name] = mask
                    continue
                layer = self.layers_by_name[name]
                layer.iteration, layer.epoch = self.conf.iterationCount, self.conf.epochCount
                if name in self._residual_of:
                    layer.residual = acts[self._residual_of[name]]
                tok = _prof.layer_begin("fwd", name, layer) if _prof.ACTIVE else None
                if not active[name] and hasattr(layer, "setLabels"):
                    mask = None             # a passed-through feature mask does not mask an output layer
                if stored_state and hasattr(layer, "tBpttStateMap"):
                    out = layer.activate(x, train, mask, stored_state=True, store_last_for_tbptt=store_last_for_tbptt)
                else:
                    out = layer.activate(x, train, mask)
                if tok is not None:
                    _prof.layer_end(tok, "fwd", name, layer, out)
                acts[name] = out
                amask[name], _ = layer.feedForwardMaskArray(mask, None, mb)
                if getattr(layer, "MASK_PASSTHROUGH", False):
                    active[name] = False
            elif name in self._passthrough:
                acts[name] = acts[self._passthrough[name]]
                amask[name] = ms[0] if ms else None
            else:
                from ..conf.graph import DuplicateToTimeSeriesVertex
                if isinstance(v, DuplicateToTimeSeriesVertex):
                    v._T = acts[v.inputName].shape[2]
                out, ctx = v.forward(ins, train, ms)
                self._ctx[name] = ("vertex", ctx)
                acts[name] = out
                amask[name] = v.feedForwardMask(ms)
        if chk is not None:
            self._validated = chk
        self._acts_masks = amask
        return acts

    def setLayerMaskArrays(self, featureMaskArrays, labelMaskArrays):
        """Masks used by later output/feedForward calls that pass none (reference ComputationGraph.setLayerMaskArrays)."""
        self.inputMaskArrays = list(featureMaskArrays) if featureMaskArrays is not None else None
        self.labelMaskArrays = list(labelMaskArrays) if labelMaskArrays is not None else None

    def clearLayerMaskArrays(self):
        self.inputMaskArrays = self.labelMaskArrays = None

    def output(self, *inputs, train=False, masks=None):
        """output(x...), output([x...]) or, as the reference, output(train, x...)."""
        if inputs and isinstance(inputs[0], bool):
            train, inputs = inputs[0], inputs[1:]
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = inputs[0]
        with torch.no_grad():
            acts = self.feedForward(list(inputs), train, masks)
        outs = [_out_dtype(acts[o]) for o in self.outputs]
        lm = self.labelMaskArrays
        if lm is not None:                      # label masks set with setLayerMaskArrays zero those outputs
            from ..network_base import _apply_output_mask
            outs = [_apply_output_mask(t, lm[i]) if i < len(lm) and hasattr(self.layers_by_name.get(o), "setLabels")
                    else t for i, (o, t) in enumerate(zip(self.outputs, outs))]
        return outs

    def outputSingle(self, *inputs, train=False):
        """outputSingle(x...) or, as the reference, outputSingle(train, x...)."""
        if inputs and isinstance(inputs[0], bool):
            train, inputs = inputs[0], inputs[1:]
        return self.output(*inputs, train=train)[0]

    # ------------------------------------------------------------------------------ backward
    def _backprop(self, tbptt_back=None):
        eps_acc = {}

        def add(name, e):
            if e is None:
                return
            if name in eps_acc:
                if eps_acc[name] is e:                 # already summed in place by the producing kernel
                    return
                eps_acc[name] = eps_acc[name] + e
            else:
                eps_acc[name] = e

        self._begin_backward()
        for name in reversed(self.topo):
            v = self.conf.vertices[name]
            if name in self._passthrough:
                add(self._passthrough[name], eps_acc.pop(name, None))
                continue
            if isinstance(v, LayerVertex):
                layer = self.layers_by_name.get(name)
                if name in self.outputs and (isinstance(layer, BaseOutputLayerImpl) or hasattr(layer, "computeScore")):
                    tok = _prof.layer_begin("bwd", name, layer) if _prof.ACTIVE else None
                    _, e = layer.backpropGradient(None)
                    if tok is not None:
                        _prof.layer_end(tok, "bwd", name, layer, e)
                    self._grad_ready(name)
                else:
                    e_in = eps_acc.pop(name, None)
                    if e_in is None:
                        continue
                    if not self._need_input_grad[name] and layer.conf.numParams() == 0:
                        continue
                    tok = _prof.layer_begin("bwd", name, layer) if _prof.ACTIVE else None
                    ins0 = self.vertex_inputs[name]
                    if len(ins0) == 1 and v.preProcessor is None and ins0[0] in eps_acc and \
                            hasattr(layer, "dx_accum") and \
                            not any(_shares_storage(eps_acc[ins0[0]], t) for t in
                                    [e_in] + [t for k, t in eps_acc.items() if k != ins0[0]]):
                        # fan-out: let the conv kernel sum dX in place. Never when the running sum is also this
                        # layer's own incoming gradient or another vertex's pending one (x + conv(x) with an
                        # identity activation hands one tensor to both branches): the kernel would overwrite a
                        # gradient that is still to be read.
                        layer.dx_accum = eps_acc[ins0[0]]
                    if tbptt_back is not None and hasattr(layer, "tBpttStateMap"):
                        _, e = layer.backpropGradient(e_in, tbptt_back=tbptt_back)
                    else:
                        _, e = layer.backpropGradient(e_in)
                    if tok is not None:
                        _prof.layer_end(tok, "bwd", name, layer, e)
                    self._grad_ready(name)
                    if name in self._residual_of:
                        add(self._residual_of[name], layer.dresidual)
                        layer.dresidual = None
                if e is None or not self._need_input_grad[name]:
                    continue
                if v.preProcessor is not None:
                    e = v.preProcessor.backprop(e, self._mb)
                ins = self.vertex_inputs[name]
                if len(ins) > 1:
                    parts = torch.split(e, self._ctx[name][1], dim=1)
                    for i, p in zip(ins, parts):
                        add(i, p)
                else:
                    add(ins[0], e)
            else:
                e_in = eps_acc.pop(name, None)
                if e_in is None or not self._need_input_grad[name]:
                    continue
                es = v.backward(e_in, self._ctx[name][1])
                for i, ei in zip(self.vertex_inputs[name], es):
                    add(i, ei)
        self._end_backward()
        for l in self.listeners:
            if hasattr(l, "onBackwardPass"):
                l.onBackwardPass(self)
        self._input_eps = [eps_acc.get(n) for n in self.conf.networkInputs]
        return self._input_eps

    def computeGradientAndScore(self, inputs=None, labels=None, fmasks=None, lmasks=None, stored_state=False,
                                store_last_for_tbptt=False, tbptt_back=None, defer_reg=False):
        if inputs is None:
            # the setInputs / setLabels / setLayerMaskArrays path (reference computeGradientAndScore())
            fmasks = getattr(self, "inputMaskArrays", None) if fmasks is None else fmasks
            lmasks = getattr(self, "labelMaskArrays", None) if lmasks is None else lmasks
        inputs = self._prep_inputs(self.inputs if inputs is None else inputs)
        labels = self.labels if labels is None else labels
        if torch.is_tensor(labels):
            labels = [labels]
        self._mb = inputs[0].shape[0]
        self._prepare_conv_weights()
        fm = [self._to_dev(m) for m in fmasks] if fmasks else None
        # the output activation of a training forward is not read (the fused loss recomputes the softmax from the
        # pre-activation) unless a listener asks for the activations or another vertex consumes that output
        skip = not any(hasattr(l, "onForwardPass") for l in self.listeners)
        outs = [self.layers_by_name.get(o) for o in self.outputs]
        for o, l in zip(self.outputs, outs):
            if l is not None and skip and not self.consumers.get(o):
                l._skip_train_output = True
        try:
            acts = self.feedForward(inputs, True, fm, stored_state, store_last_for_tbptt)
        finally:
            for l in outs:
                if l is not None:
                    l._skip_train_output = False
        for l in self.listeners:
            if hasattr(l, "onForwardPass"):
                l.onForwardPass(self, acts)
        mb_in = self._prep_mb if getattr(self, "_prep_mb", None) else None
        for i, o in enumerate(self.outputs):
            layer = self.layers_by_name.get(o)
            if layer is None or not hasattr(layer, "setLabels"):
                from ...exceptions import DL4JException
                kind = type(layer.conf).__name__ if layer is not None else type(self.conf.vertices[o]).__name__
                raise DL4JException(f"Cannot calculate gradient and score: network output \"{o}\" is not an output "
                                    f"layer ({kind}); end the graph in an OutputLayer / RnnOutputLayer / LossLayer")
            layer.setLabels(self._to_dev(labels[i], self.master_dtype))
            layer.inputMiniBatchSize = mb_in
            lm = lmasks[i] if lmasks is not None and i < len(lmasks) else None
            if lm is not None:
                layer.maskArray = self._to_dev(lm)
        self._backprop(tbptt_back)
        l1, l2 = (0.0, 0.0) if defer_reg else self._regularization_terms()
        score = None
        for i, o in enumerate(self.outputs):
            layer = self.layers_by_name[o]
            s = layer.computeScore(l1 if i == 0 else 0.0, l2 if i == 0 else 0.0, True)
            score = s if score is None else score + s
        self._loss_part = score
        self._score_t = score
        self._score_val = None
        return score

    def _fit_batch_sgd(self, inputs, labels, fmasks=None, lmasks=None):
        x0 = inputs[0] if isinstance(inputs, (list, tuple)) else inputs
        if self.conf.backpropType == BackpropType.TruncatedBPTT and x0.dim() == 3:
            return self._fit_tbptt(inputs, labels, fmasks, lmasks)
        self.computeGradientAndScore(inputs, labels, fmasks, lmasks, defer_reg=True)
        self._apply_update(x0.shape[0])
        self._iteration_done()

    def _fit_tbptt(self, inputs, labels, fmasks, lmasks):
        inputs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
        labels = labels if isinstance(labels, (list, tuple)) else [labels]
        T = inputs[0].shape[2]
        fwd, back = self.conf.tbpttFwdLength, self.conf.tbpttBackLength
        self.rnnClearPreviousState()
        for s in range((T + fwd - 1) // fwd):
            t0, t1 = s * fwd, min(T, (s + 1) * fwd)
            xs = [x[:, :, t0:t1] if x.dim() == 3 else x for x in inputs]
            ys = [y[:, :, t0:t1] if y.dim() == 3 else y for y in labels]
            fm = [m[:, t0:t1] if m is not None else None for m in fmasks] if fmasks else None
            lm = [m[:, t0:t1] if m is not None else None for m in lmasks] if lmasks else None
            if self._try_graph_step(xs, ys, fm, lm, tbptt_back=back):
                continue                           # this window replayed as a HIP graph (nn/hipgraph.py)
            from ...memory.arena import tbptt_scope
            with tbptt_scope(self):                  # LOOP_TBPTT arena for this window
                self.computeGradientAndScore(xs, ys, fm, lm, stored_state=True, store_last_for_tbptt=True,
                                             tbptt_back=back, defer_reg=True)
                self._apply_update(inputs[0].shape[0])
            self._iteration_done()
        self.rnnClearPreviousState()

    def fit(self, data, labels=None, numEpochs=None, featureMaskArrays=None, labelMaskArrays=None):
        if not self.initCalled:
            self.init()
        if labels is not None and not isinstance(labels, int):
            self._fit_batch(data, labels, featureMaskArrays, labelMaskArrays)
            return self
        if isinstance(labels, int):
            numEpochs = labels
        if numEpochs is not None:
            for _ in range(numEpochs):
                self.fit(data)
            return self
        if isinstance(data, DataSet):
            self._fit_batch([data.features], [data.labels],
                            None if data.featuresMask is None else [data.featuresMask],
                            None if data.labelsMask is None else [data.labelsMask])
            return self
        if isinstance(data, MultiDataSet):
            self._fit_batch(data.features, data.labels, data.featuresMasks, data.labelsMasks)
            return self
        self._fit_iterator(data)
        return self

    def _fit_iterator(self, it):
        from ...datasets.iterators import AsyncDataSetIterator
        wrap = it
        if getattr(it, "asyncSupported", lambda: False)() and not isinstance(it, AsyncDataSetIterator) and \
                type(it).__name__ not in ("BenchmarkDataSetIterator", "BenchmarkMultiDataSetIterator",
                                          "ListDataSetIterator"):
            wrap = AsyncDataSetIterator(it, 2, self.device)
        for l in self.listeners:
            if hasattr(l, "onEpochStart"):
                l.onEpochStart(self)
        wrap.reset()
        t0 = self._timer()
        while wrap.hasNext():
            ds = wrap.next()
            self.lastEtlTime = (self._timer() - t0) * 1000.0
            if isinstance(ds, MultiDataSet):
                self._fit_batch(ds.features, ds.labels, ds.featuresMasks, ds.labelsMasks)
            else:
                self._fit_batch([ds.features], [ds.labels], None if ds.featuresMask is None else [ds.featuresMask],
                                None if ds.labelsMask is None else [ds.labelsMask])
            t0 = self._timer()
        if wrap is not it and hasattr(wrap, "shutdown"):
            wrap.shutdown()
        for l in self.listeners:
            if hasattr(l, "onEpochEnd"):
                l.onEpochEnd(self)
        self.incrementEpochCount()

    # ------------------------------------------------------------------------------ scoring / eval
    def _score_dataset(self, ds, training=False):
        if isinstance(ds, DataSet):
            ds = MultiDataSet.fromDataSet(ds)
        with torch.no_grad():
            self._mb = ds.features[0].shape[0]
            self.feedForward(ds.features, training)
            l1, l2 = self._regularization_terms()
            score = 0.0
            for i, o in enumerate(self.outputs):
                layer = self.layers_by_name[o]
                layer.setLabels(self._to_dev(ds.labels[i], self.master_dtype))
                layer.inputMiniBatchSize = self._mb
                score += float(layer.computeScore(l1 if i == 0 else 0.0, l2 if i == 0 else 0.0, training))
            return score

    def scoreExamples(self, data, addRegularizationTerms=True):
        """Per-example score, summed over the output layers (reference ComputationGraph.scoreExamples,
        NN:nn/graph/ComputationGraph.java:2386-2403); regularisation terms added to every example when asked."""
        ds = data if isinstance(data, (DataSet, MultiDataSet)) else data.next()
        if isinstance(ds, DataSet):
            ds = MultiDataSet.fromDataSet(ds)
        with torch.no_grad():
            self.feedForward(ds.features, False, ds.featuresMasks)
            l1, l2 = self._regularization_terms() if addRegularizationTerms else (0.0, 0.0)
            total = None
            for i, o in enumerate(self.outputs):
                layer = self.layers_by_name[o]
                layer.setLabels(self._to_dev(ds.labels[i], self.master_dtype))
                if ds.labelsMasks and i < len(ds.labelsMasks) and ds.labelsMasks[i] is not None:
                    layer.maskArray = self._to_dev(ds.labelsMasks[i])
                s = layer.computeScoreForExamples(l1 if i == 0 else 0.0, l2 if i == 0 else 0.0)
                total = s if total is None else total + s
            return total

    def evaluate(self, it, labelsList=None, topN=1):
        from ...eval.evaluation import Evaluation
        return self.doEvaluation(it, Evaluation(labelsList, topN=topN))[0]

    def evaluateRegression(self, it):
        from ...eval.regression import RegressionEvaluation
        return self.doEvaluation(it, RegressionEvaluation())[0]

    def evaluateROC(self, it, steps=0):
        from ...eval.roc import ROC
        return self.doEvaluation(it, ROC(steps))[0]

    def doEvaluation(self, it, *evals):
        items = [it] if isinstance(it, (DataSet, MultiDataSet)) else it
        if not isinstance(it, (DataSet, MultiDataSet)):
            it.reset()
        for ds in items:
            if isinstance(ds, MultiDataSet):
                out = self.output(ds.features)[0]
                lab = ds.labels[0]
                lm = ds.labelsMasks[0] if ds.labelsMasks else None
            else:
                out = self.output(ds.features)[0]
                lab, lm = ds.labels, ds.labelsMask
            for e in evals:
                e.eval(lab, out, lm)
        return list(evals)

    # ------------------------------------------------------------------------------ rnn
    def rnnTimeStep(self, *inputs):
        inputs = self._prep_inputs(list(inputs))
        mb = inputs[0].shape[0]          # a FF->RNN preprocessor reshapes [mb*T, n] rows back by the INPUT minibatch
        acts = {n: inputs[i] for i, n in enumerate(self.conf.networkInputs)}
        with torch.no_grad():
            for name in self.topo:
                v = self.conf.vertices[name]
                if name in self._passthrough:
                    acts[name] = acts[self._passthrough[name]]
                    continue
                ins = [acts[i] for i in self.vertex_inputs[name]]
                if isinstance(v, LayerVertex):
                    x = ins[0] if len(ins) == 1 else torch.cat(ins, 1)
                    if v.preProcessor is not None:
                        x = v.preProcessor.preProcess(x, mb, False)
                    layer = self.layers_by_name[name]
                    if name in self._residual_of:
                        layer.residual = acts[self._residual_of[name]]
                    if hasattr(layer, "rnnTimeStep"):
                        acts[name] = layer.rnnTimeStep(x)
                    else:
                        acts[name] = layer.activate(x, False)
                else:
                    acts[name], _ = v.forward(ins, False, None)
        return [_out_dtype(acts[o]) for o in self.outputs]

    def rnnClearPreviousState(self):
        for l in self.layers_by_name.values():
            if hasattr(l, "rnnClearPreviousState"):
                l.rnnClearPreviousState()

    def rnnGetPreviousState(self, layerName):
        """Stored rnnTimeStep state of one recurrent layer (reference ComputationGraph.rnnGetPreviousState,
        NN:nn/graph/ComputationGraph.java:2805-2855)."""
        layer = self.layers_by_name[layerName] if isinstance(layerName, str) else self.getLayers()[layerName]
        return layer.rnnGetPreviousState() if hasattr(layer, "rnnGetPreviousState") else None

    def rnnSetPreviousState(self, layerName, state):
        layer = self.layers_by_name[layerName] if isinstance(layerName, str) else self.getLayers()[layerName]
        if not hasattr(layer, "rnnSetPreviousState"):
            raise ValueError(f"layer {layerName} is not a recurrent layer")
        layer.rnnSetPreviousState(state)

    def rnnGetPreviousStates(self):
        return {n: l.rnnGetPreviousState() for n, l in self.layers_by_name.items() if hasattr(l, "rnnGetPreviousState")}

    def rnnSetPreviousStates(self, states):
        for n, st in states.items():
            self.rnnSetPreviousState(n, st)

    # ------------------------------------------------------------------------------ pretraining
    def pretrainLayer(self, layerName, data, numEpochs=1):
        """Unsupervised pretraining of one AutoEncoder / VAE vertex (reference ComputationGraph.pretrainLayer,
        NN:nn/graph/ComputationGraph.java:669-722): its input is the inference-mode activation of its input vertices."""
        if not self.initCalled:
            self.init()
        impl = self.layers_by_name[layerName]
        if not hasattr(impl, "computePretrainGradientAndScore"):
            return self
        v = self.conf.vertices[layerName]
        for _ in range(int(numEpochs)):
            items = [data] if isinstance(data, (DataSet, MultiDataSet)) else data
            if not isinstance(items, list):
                items.reset()
            for ds in items:
                feats = [ds.features] if isinstance(ds, DataSet) else ds.features
                with torch.no_grad():
                    acts = self.feedForward(feats, False)
                    ins = [acts[i] for i in self.vertex_inputs[layerName]]
                    x = ins[0] if len(ins) == 1 else torch.cat(ins, dim=1)
                    if v.preProcessor is not None:
                        x = v.preProcessor.preProcess(x, x.shape[0], False)
                self._pretrain_step(impl, x)
        return self

    def pretrain(self, data, numEpochs=1):
        """Layer-wise pretraining of every pretrainable vertex in topological order (reference
        ComputationGraph.pretrain)."""
        for name in self.topo:
            l = self.layers_by_name.get(name)
            if l is not None and hasattr(l, "computePretrainGradientAndScore"):
                self.pretrainLayer(name, data, numEpochs)
        return self

    # ------------------------------------------------------------------------------ misc
    def clone(self):
        import copy
        net = ComputationGraph(copy.deepcopy(self.conf))
        net.init(self.params().clone(), device=self.device)
        net.updater.setStateViewArray(self.updater.getStateViewArray().clone())
        return net

    def setInputs(self, *x):
        self.inputs = list(x)

    def setLabels(self, *y):
        self.labels = list(y)

    def setInput(self, i, x):
        """Set network input i (reference ComputationGraph.setInput(int, INDArray))."""
        n = len(self.conf.networkInputs)
        cur = list(self.inputs) if self.inputs is not None else []
        cur += [None] * (n - len(cur))
        cur[i] = x
        self.inputs = cur

    def setLabel(self, i, y):
        """Set the labels of output i (reference ComputationGraph.setLabel(int, INDArray))."""
        cur = list(self.labels) if self.labels is not None else []
        cur += [None] * (len(self.outputs) - len(cur))
        cur[i] = y
        self.labels = cur

    def getInput(self, i):
        return self.inputs[i]

    def layerSize(self, name):
        """nOut of layer ``name`` (0 for layers without one) (reference ComputationGraph.layerSize)."""
        if name not in self.layers_by_name:
            raise ValueError(f"No layer named {name!r}")
        return int(getattr(self.layers_by_name[name].conf, "nOut", 0) or 0)

    def getNumInputArrays(self):
        return len(self.conf.networkInputs)

    def getNumOutputArrays(self):
        return len(self.conf.networkOutputs)

    def topologicalSortOrder(self):
        """Topological order as vertex indices: inputs first, then vertices in the order they were added
        (reference ComputationGraph.topologicalSortOrder / calcTopologicalSortOrder :1216-1318)."""
        idx = {n: i for i, n in enumerate(list(self.conf.networkInputs) + list(self.conf.vertices))}
        return [idx[n] for n in self.conf.topologicalOrder()]

    def gradientAndScore(self):
        """(gradient, score) of the last computeGradientAndScore (reference Model.gradientAndScore)."""
        return self.gradient(), self.score()

    def setLearningRate(self, lr, layerName=None):
        """setLearningRate(newLr), or setLearningRate(layerName, newLr) as in the reference."""
        if isinstance(lr, str):
            lr, layerName = layerName, lr
        self.updater.setLearningRate(lr, layerName)

    def save(self, path, saveUpdater=True):
        from ...utils.model_serializer import ModelSerializer
        ModelSerializer.writeModel(self, path, saveUpdater)

    @staticmethod
    def load(path, loadUpdater=True):
        from ...utils.model_serializer import ModelSerializer
        return ModelSerializer.restoreComputationGraph(path, loadUpdater)

    def clear(self):
        for l in self.layers_by_name.values():
            l.clear()


class _RuntimeVertex:
    """A live graph vertex (reference GraphVertex): getVertexName / getVertexIndex / hasLayer / getLayer /
    getInputVertices / setLayerAsFrozen; any other attribute is the vertex configuration's."""

    def __init__(self, graph, name):
        object.__setattr__(self, "_g", graph)
        object.__setattr__(self, "_name", name)

    def getVertexName(self):
        return self._name

    def getVertexIndex(self):
        return (list(self._g.conf.networkInputs) + list(self._g.conf.vertices)).index(self._name)

    def isInputVertex(self):
        return self._name in self._g.conf.networkInputs

    def hasLayer(self):
        return self._name in self._g.layers_by_name

    def getLayer(self):
        return self._g.layers_by_name.get(self._name)

    def getInputVertices(self):
        return list(self._g.conf.vertexInputs.get(self._name, []))

    def setLayerAsFrozen(self):
        if not self.hasLayer():
            raise ValueError(f"vertex {self._name!r} has no layer to freeze")
        self._g._freeze_layer_in_place(self._name)

    def __getattr__(self, item):
        return getattr(self._g.conf.vertices[self._name], item)

    def __repr__(self):
        return f"GraphVertex({self._name!r})"
