"""MultiLayerNetwork: sequential model (reference nn/multilayer/MultiLayerNetwork.java, 3545 LoC).

init (:549-663) -> flat params/gradients + per-layer views, updater blocks;
fit (:1268-1360) -> per minibatch: forward (feedForwardToLayer :955-1041), backward
(calcBackpropGradients :1378-1519), score, fused update; TBPTT (doTruncatedBPTT :1521-1593);
output (:2031), rnnTimeStep (:2806), evaluate (:2985-3057).
"""
import torch

from ..datasets.dataset import DataSet, DataSetIterator
from .conf.enums import BackpropType
from .conf.layers import ActivationLayer, BatchNormalization
from .conf.validation import check_layer_input, validate_network_conf
from .layers.output import BaseOutputLayerImpl
from .network_base import BaseNetwork
from .. import profiling as _prof


class MultiLayerNetwork(BaseNetwork):
    _key_by_name = False

    def __init__(self, conf, params=None):
        super().__init__(conf)
        self.layers = []
        self._init_params = params
        self.input = None
        self.labels = None
        self.mask = None
        self.labelsMask = None

    # ------------------------------------------------------------------------------ init
    def init(self, parameters=None, cloneParametersArray=False, device=None):
        if self.initCalled and parameters is None:
            return
        parameters = parameters if parameters is not None else self._init_params
        validate_network_conf(self.conf.confs)
        self.layers = [c.instantiate(index=i, net=self) for i, c in enumerate(self.conf.confs)]
        self._setup_flat([(i, self.conf.confs[i].layerName, l) for i, l in enumerate(self.layers)], parameters,
                         cloneParametersArray, device)
        self._plan_fusions()
        for l in self.layers:
            if hasattr(l, "bind"):
                l.bind()

    def _plan_fusions(self):
        """BN -> ActivationLayer(ReLU): run the ReLU inside the BN kernel (forward and backward)."""
        from .conf.activations import ActivationReLU
        self._fused_passthrough = set()
        for i in range(len(self.layers) - 1):
            a, b = self.conf.confs[i], self.conf.confs[i + 1]
            if isinstance(a, BatchNormalization) and isinstance(b, ActivationLayer) and \
                    isinstance(b.activation, ActivationReLU) and (i + 1) not in self.conf.inputPreProcessors \
                    and b.idropout is None:
                if a.idropout is None:
                    self.layers[i].fuse_relu = True
                    self._fused_passthrough.add(i + 1)
        seen_params = False
        for l in self.layers:
            l.need_input_grad = seen_params       # nothing trainable upstream => skip dL/dinput
            seen_params = seen_params or l.conf.numParams() > 0
        self._plan_lstm_stacks()

    def _plan_lstm_stacks(self):
        """Consecutive LSTM / GravesLSTM layers of the same kind, with nothing between them (no preprocessor, input
        dropout or weight noise), run as ONE pipelined two-layer launch (nn/layers/recurrent.py _stack_forward /
        _stack_backward; the kernels decide at run time whether the shape fits)."""
        from .conf.activations import ActivationSigmoid, ActivationTanH
        from .layers.recurrent import LSTMImpl
        for l in self.layers:
            l._stack_next = l._stack_prev = None
        i = 0
        while i < len(self.layers) - 1:
            a, b = self.layers[i], self.layers[i + 1]
            ca, cb = a.conf, b.conf
            ok = (type(a) is type(b) and isinstance(a, LSTMImpl) and type(ca) is type(cb)
                  and ca.nOut == cb.nOut and cb.nIn == ca.nOut and (i + 1) not in self.conf.inputPreProcessors
                  and getattr(cb, "idropout", None) is None and getattr(ca, "weightNoise", None) is None
                  and getattr(cb, "weightNoise", None) is None
                  and all(isinstance(c.activation, ActivationTanH) and isinstance(c.gateActivationFn,
                                                                                  ActivationSigmoid)
                          for c in (ca, cb)))
            if ok:
                a._stack_next, b._stack_prev = b, a
                i += 2
            else:
                i += 1

    def getLayers(self):
        return self.layers

    def getLayer(self, i):
        if isinstance(i, str):
            for l in self.layers:
                if l.conf.layerName == i:
                    return l
            raise KeyError(i)
        return self.layers[i]

    def getnLayers(self):
        return len(self.layers)

    def getOutputLayer(self):
        return self.layers[-1]

    def getLayerWiseConfigurations(self):
        return self.conf

    # ------------------------------------------------------------------------------ forward
    def _pp(self, i, x, mb, training):
        pp = self.conf.inputPreProcessors.get(i)
        return pp.preProcess(x, mb, training) if pp is not None else x

    def _mask_for(self, i, mask, mb):
        pp = self.conf.inputPreProcessors.get(i)
        if pp is not None and mask is not None:
            mask, _ = pp.feedForwardMaskArray(mask, None, mb)
        return mask

    def feedForwardToLayer(self, layerNum, x, train=False, fmask=None, stored_state=False,
                           store_last_for_tbptt=False):
        """Activations of layers 0..layerNum (inclusive); index 0 of the returned list is the input."""
        x = x.toTensor() if hasattr(x, "toTensor") else x
        x = self._to_dev(x, self._feat_dtype()) if x.is_floating_point() else self._to_dev(x)
        mb = x.shape[0]
        acts = [x]
        mask = fmask
        active = True                     # feature-mask state: False once an LSTM has passed it through
        chk = self._input_check([x])
        idx = self._index_checked()
        for i in range(layerNum + 1):
            layer = self.layers[i]
            x = self._pp(i, x, mb, train)
            mask = self._mask_for(i, mask, mb)
            if chk is not None or i in idx:
                check_layer_input(self.conf.confs[i], x, i)
            if i in self._fused_passthrough:
                acts.append(x)
                continue
            layer.iteration, layer.epoch = self.conf.iterationCount, self.conf.epochCount
            tok = _prof.layer_begin("fwd", i, layer) if _prof.ACTIVE else None
            lmask = mask if active or not hasattr(layer, "setLabels") else None
            if stored_state and hasattr(layer, "tBpttStateMap"):
                x = layer.activate(x, train, lmask, stored_state=True, store_last_for_tbptt=store_last_for_tbptt)
            else:
                x = layer.activate(x, train, lmask)
            if tok is not None:
                _prof.layer_end(tok, "fwd", i, layer, x)
            mask, _ = layer.feedForwardMaskArray(lmask, None, mb)
            active = active and not getattr(layer, "MASK_PASSTHROUGH", False)
            acts.append(x)
        self._fmask_active = active
        if chk is not None and layerNum == len(self.layers) - 1:
            self._validated = chk
        return acts

    def rnnActivateUsingStoredState(self, x, training=False, storeLastForTBPTT=False):
        """Forward pass whose recurrent layers start from their stored rnnTimeStep state (zeros when none) without
        changing it; with ``storeLastForTBPTT`` each layer's final state is kept as its TBPTT state
        (rnnGetTBPTTState). Reference MultiLayerNetwork.rnnActivateUsingStoredState."""
        rec = [l for l in self.layers if hasattr(l, "tBpttStateMap") and hasattr(l, "stateMap")]
        saved = [dict(l.tBpttStateMap) for l in rec]
        for l in rec:
            l.tBpttStateMap = dict(l.stateMap)
        try:
            with torch.no_grad():
                return self.feedForwardToLayer(len(self.layers) - 1, x, training, None, True, storeLastForTBPTT)
        finally:
            if not storeLastForTBPTT:
                for l, s in zip(rec, saved):
                    l.tBpttStateMap = s

    def feedForward(self, x=None, train=False, fmask=None):
        x = self.input if x is None else x
        acts = self.feedForwardToLayer(len(self.layers) - 1, x, train, fmask)
        for l in self.listeners:
            if hasattr(l, "onForwardPass"):
                l.onForwardPass(self, acts)
        return acts

    def output(self, x, train=False, featuresMask=None, labelsMask=None):
        if isinstance(x, DataSetIterator):
            return [self.output(ds.features, train, ds.featuresMask) for ds in x]
        if featuresMask is None:
            featuresMask = self.mask            # masks set with setLayerMaskArrays apply (reference output(INDArray))
        if labelsMask is None:
            labelsMask = self.labelsMask
        with torch.no_grad():
            acts = self.feedForwardToLayer(len(self.layers) - 1, x, train, self._to_dev(featuresMask))
        out = acts[-1]
        if labelsMask is not None and hasattr(self.layers[-1], "setLabels"):
            from .network_base import _apply_output_mask
            out = _apply_output_mask(out, labelsMask)
        # 16-bit activations come back as fp32 (the reference's output dtype); fp32/fp64 networks keep theirs
        return out.float() if out.dtype in (torch.bfloat16, torch.float16) else out

    def activate(self, x, train=False):
        return self.output(x, train)

    def layerSize(self, layer):
        """nOut of layer ``layer`` (0 for layers without one, e.g. pooling) (reference MultiLayerNetwork.layerSize)."""
        if not 0 <= layer < len(self.layers):
            raise ValueError(f"Invalid layer index {layer}: the network has {len(self.layers)} layers")
        return int(getattr(self.layers[layer].conf, "nOut", 0) or 0)

    def computeZ(self, x, training=False):
        """[input, z_0, z_1, ...]: every layer's pre-activation on the way forward (reference
        MultiLayerNetwork.computeZ); layers without one (pooling, activation) contribute their output."""
        x = x.toTensor() if hasattr(x, "toTensor") else x
        x = self._to_dev(x, self._feat_dtype()) if x.is_floating_point() else self._to_dev(x)
        mb = x.shape[0]
        out = [x]
        with torch.no_grad():
            for i, layer in enumerate(self.layers):
                x = self._pp(i, x, mb, training)
                if hasattr(layer, "preOutput2d"):
                    z = layer._out_from2d(layer.preOutput2d(layer._in2d(x)))
                else:
                    try:
                        z = layer.preOutput(x, training)
                    except NotImplementedError:
                        z = None
                x = layer.activate(x, training)
                out.append(x if z is None else z)
        return out

    def preOutput(self, x, train=False):
        """The output layer's pre-activation (z = x W + b) for input x, in the layout of its output (reference
        MultiLayerNetwork.preOutput)."""
        out = self.layers[-1]
        with torch.no_grad():
            self.feedForwardToLayer(len(self.layers) - 1, x, train)
        if getattr(out, "_z", None) is None:
            raise NotImplementedError(f"preOutput: {type(out).__name__} is not an output layer")
        return out._out_from2d(out._z)

    def predict(self, x):
        return torch.argmax(self.output(x), dim=1)

    def labelProbabilities(self, x):
        return self.output(x)

    # ------------------------------------------------------------------------------ backward
    def _backprop(self, tbptt_back=None):
        """Reverse pass from the output layer; gradients land in the flat gradient views."""
        n = len(self.layers)
        out_layer = self.layers[-1]
        if not (isinstance(out_layer, BaseOutputLayerImpl) or hasattr(out_layer, "computeScore")):
            raise ValueError("Cannot calculate gradient and score with respect to labels: final layer is not an "
                             "IOutputLayer")
        self._begin_backward()
        tok = _prof.layer_begin("bwd", n - 1, out_layer) if _prof.ACTIVE else None
        _, eps = out_layer.backpropGradient(None)
        if tok is not None:
            _prof.layer_end(tok, "bwd", n - 1, out_layer, eps)
        self._grad_ready(n - 1)
        mb = self._mb
        for i in range(n - 2, -1, -1):
            pp = self.conf.inputPreProcessors.get(i + 1)
            if pp is not None:
                eps = pp.backprop(eps, mb)
            if i in self._fused_passthrough:
                continue
            layer = self.layers[i]
            tok = _prof.layer_begin("bwd", i, layer) if _prof.ACTIVE else None
            if tbptt_back is not None and hasattr(layer, "tBpttStateMap"):
                _, eps = layer.backpropGradient(eps, tbptt_back=tbptt_back)
            else:
                _, eps = layer.backpropGradient(eps)
            if tok is not None:
                _prof.layer_end(tok, "bwd", i, layer, eps)
            self._grad_ready(i)
            if eps is None:
                break
        self._end_backward()
        for l in self.listeners:
            if hasattr(l, "onBackwardPass"):
                l.onBackwardPass(self)
        return eps

    def computeGradientAndScore(self, x=None, y=None, fmask=None, lmask=None, stored_state=False,
                                store_last_for_tbptt=False, tbptt_back=None, defer_reg=False):
        x = self.input if x is None else x
        y = self.labels if y is None else y
        fmask = self.mask if fmask is None else fmask
        lmask = self.labelsMask if lmask is None else lmask
        self._mb = x.shape[0]
        self._prepare_conv_weights()
        out_l = self.layers[-1]
        if not hasattr(out_l, "setLabels"):
            from ..exceptions import DL4JException
            raise DL4JException(f"Cannot calculate gradient and score: the last layer ({type(out_l.conf).__name__}) "
                                f"is not an output layer; end the network in an OutputLayer / RnnOutputLayer / "
                                f"LossLayer (reference MultiLayerNetwork.computeGradientAndScore)")
        # nobody reads the output activation of a training forward unless a listener asks for the activations
        out_l._skip_train_output = not any(hasattr(l, "onForwardPass") for l in self.listeners)
        try:
            acts = self.feedForwardToLayer(len(self.layers) - 1, x, True, self._to_dev(fmask), stored_state,
                                           store_last_for_tbptt)
        finally:
            out_l._skip_train_output = False
        for l in self.listeners:
            if hasattr(l, "onForwardPass"):
                l.onForwardPass(self, acts)
        out = self.layers[-1]
        out.setLabels(self._to_dev(y, self.master_dtype))
        out.inputMiniBatchSize = self._mb
        if lmask is not None:
            out.maskArray = self._to_dev(lmask)
        elif (fmask is not None and out.maskArray is None and out.input is not None and out.input.dim() == 3
              and getattr(self, "_fmask_active", True)):
            # the feature mask doubles as the label mask of a time-series output; a layer that consumed the mask
            # on the way (LastTimeStep, global pooling) left a 2-D output that has none
            out.maskArray = self._to_dev(fmask)
        self._backprop(tbptt_back)
        if defer_reg:      # regularisation term comes out of the fused updater kernel (see _apply_update)
            self._loss_part = out.computeScore(0.0, 0.0, True)
            self._score_t = self._loss_part
        else:
            l1, l2 = self._regularization_terms()
            self._score_t = out.computeScore(l1, l2, True)
        self._score_val = None
        return self._score_t

    def _fit_batch_sgd(self, x, y, fmask=None, lmask=None):
        if self.conf.backpropType == BackpropType.TruncatedBPTT and x.dim() == 3:
            return self._fit_tbptt(x, y, fmask, lmask)
        self.computeGradientAndScore(x, y, fmask, lmask, defer_reg=True)
        self._apply_update(x.shape[0])
        self._iteration_done()

    def _fit_tbptt(self, x, y, fmask, lmask):
        """Reference doTruncatedBPTT (MultiLayerNetwork.java:1521-1593)."""
        T = x.shape[2]
        fwd = self.conf.tbpttFwdLength
        back = self.conf.tbpttBackLength
        n_sub = (T + fwd - 1) // fwd
        self.rnnClearPreviousState()
        for s in range(n_sub):
            t0, t1 = s * fwd, min(T, (s + 1) * fwd)
            xs = x[:, :, t0:t1]
            ys = y[:, :, t0:t1] if y.dim() == 3 else y
            fm = fmask[:, t0:t1] if fmask is not None else None
            lm = lmask[:, t0:t1] if lmask is not None else None
            if self._try_graph_step([xs], [ys], fm, lm, tbptt_back=back):
                continue                           # this window replayed as a HIP graph (nn/hipgraph.py)
            from ..memory.arena import tbptt_scope
            with tbptt_scope(self):                  # LOOP_TBPTT arena for this window
                self.computeGradientAndScore(xs, ys, fm, lm, stored_state=True, store_last_for_tbptt=True,
                                             tbptt_back=back, defer_reg=True)
                self._apply_update(x.shape[0])
            self._iteration_done()
        self.rnnClearPreviousState()

    def fit(self, data, labels=None, numEpochs=None, featuresMask=None, labelsMask=None):
        """fit(DataSetIterator[, numEpochs]) | fit(DataSet) | fit(features, labels)."""
        if not self.initCalled:
            self.init()
        if isinstance(labels, int) and not torch.is_tensor(data):
            numEpochs, labels = labels, None
        if labels is not None:
            return self.fit(DataSet(data, labels, featuresMask, labelsMask))
        if isinstance(data, DataSet):
            self._fit_batch(data.features, data.labels, data.featuresMask, data.labelsMask)
            return self
        if isinstance(labels, int) or (numEpochs is not None):
            for _ in range(numEpochs or labels):
                self.fit(data)
            return self
        self._fit_iterator(data)
        return self

    def _fit_iterator(self, it):
        from ..datasets.iterators import AsyncDataSetIterator
        if getattr(self.conf, "pretrain", False):       # reference fit(): pretrain first when configured
            self.pretrain(it)
            if not getattr(self.conf, "backprop", True):
                return
        wrap = it
        if getattr(it, "asyncSupported", lambda: False)() and not isinstance(it, AsyncDataSetIterator) and \
                type(it).__name__ not in ("BenchmarkDataSetIterator", "ListDataSetIterator"):
            wrap = AsyncDataSetIterator(it, 2, self.device)
        for l in self.listeners:
            if hasattr(l, "onEpochStart"):
                l.onEpochStart(self)
        if hasattr(wrap, "reset"):
            wrap.reset()
        t0 = self._timer()
        while wrap.hasNext():
            ds = wrap.next()
            self.lastEtlTime = (self._timer() - t0) * 1000.0
            self._fit_batch(ds.features, ds.labels, ds.featuresMask, ds.labelsMask)
            t0 = self._timer()
        if wrap is not it and hasattr(wrap, "shutdown"):
            wrap.shutdown()
        for l in self.listeners:
            if hasattr(l, "onEpochEnd"):
                l.onEpochEnd(self)
        self.incrementEpochCount()

    # ------------------------------------------------------------------------------ scoring
    def _score_dataset(self, ds, training=False):
        with torch.no_grad():
            self._mb = ds.features.shape[0]
            self.feedForwardToLayer(len(self.layers) - 1, ds.features, training, self._to_dev(ds.featuresMask))
            out = self.layers[-1]
            out.setLabels(self._to_dev(ds.labels, self.master_dtype))
            out.inputMiniBatchSize = self._mb
            if ds.labelsMask is not None:
                out.maskArray = self._to_dev(ds.labelsMask)
            l1, l2 = self._regularization_terms()
            return float(out.computeScore(l1, l2, training))

    def scoreExamples(self, data, addRegularizationTerms=True):
        ds = data if isinstance(data, DataSet) else data.next()
        with torch.no_grad():
            self.feedForwardToLayer(len(self.layers) - 1, ds.features, False, self._to_dev(ds.featuresMask))
            out = self.layers[-1]
            out.setLabels(self._to_dev(ds.labels, self.master_dtype))
            l1, l2 = self._regularization_terms() if addRegularizationTerms else (0.0, 0.0)
            return out.computeScoreForExamples(l1, l2)

    def f1Score(self, ds):
        from ..eval.evaluation import Evaluation
        e = Evaluation()
        e.eval(ds.labels, self.output(ds.features))
        return e.f1()

    # ------------------------------------------------------------------------------ rnn
    def rnnTimeStep(self, x):
        x = self._to_dev(x, self._feat_dtype())
        mb = x.shape[0]
        with torch.no_grad():
            for i, layer in enumerate(self.layers):
                x = self._pp(i, x, mb, False)
                check_layer_input(self.conf.confs[i], x, i)
                if hasattr(layer, "rnnTimeStep"):
                    x = layer.rnnTimeStep(x)
                else:
                    x = layer.activate(x, False)
        return x.float() if x.dtype in (torch.bfloat16, torch.float16) else x

    def rnnClearPreviousState(self):
        for l in self.layers:
            if hasattr(l, "rnnClearPreviousState"):
                l.rnnClearPreviousState()

    def rnnGetPreviousState(self, layer):
        return self.layers[layer].rnnGetPreviousState()

    def rnnSetPreviousState(self, layer, state):
        self.layers[layer].rnnSetPreviousState(state)

    # ------------------------------------------------------------------------------ evaluation
    def evaluate(self, it, labelsList=None, topN=1):
        from ..eval.evaluation import Evaluation
        e = Evaluation(labelsList, topN=topN)
        return self.doEvaluation(it, e)[0]

    def evaluateRegression(self, it):
        from ..eval.regression import RegressionEvaluation
        return self.doEvaluation(it, RegressionEvaluation())[0]

    def evaluateROC(self, it, rocThresholdSteps=0):
        from ..eval.roc import ROC
        return self.doEvaluation(it, ROC(rocThresholdSteps))[0]

    def evaluateROCMultiClass(self, it, rocThresholdSteps=0):
        from ..eval.roc import ROCMultiClass
        return self.doEvaluation(it, ROCMultiClass(rocThresholdSteps))[0]

    def doEvaluation(self, it, *evals):
        if isinstance(it, DataSet):
            items = [it]
        else:
            it.reset()
            items = it
        for ds in items:
            out = self.output(ds.features, False, ds.featuresMask)
            for e in evals:
                e.eval(ds.labels, out, ds.labelsMask)
        return list(evals)

    # ------------------------------------------------------------------------------ misc
    def clone(self):
        import copy
        conf = copy.deepcopy(self.conf)
        net = MultiLayerNetwork(conf)
        net.init(self.params().clone(), device=self.device)
        net.updater.setStateViewArray(self.updater.getStateViewArray().clone())
        return net

    def setLearningRate(self, lr, layer=None):
        """setLearningRate(newLr) for every layer, or setLearningRate(layerNumber, newLr) as in the reference
        (MultiLayerNetwork.java setLearningRate(int, double)); ``layer=`` may also name the layer."""
        if layer is not None and isinstance(lr, int) and not isinstance(layer, (int, str)):
            lr, layer = layer, lr
        name = None
        if layer is not None:
            name = self.conf.confs[layer].layerName if isinstance(layer, int) else layer
        self.updater.setLearningRate(lr, name)

    def getLearningRate(self, layer):
        u = self.conf.confs[layer].updater
        return u.getLearningRate(self.conf.iterationCount, self.conf.epochCount) if u is not None else None

    def _replace_impl(self, idx, name, old, new):
        self.layers[idx] = new

    def _summary_types(self, inputTypes):
        t = inputTypes[0]
        out = {}
        for idx, name, impl, _ in self._layer_offsets:
            lc = impl.conf
            pp = self.conf.inputPreProcessors.get(idx) or lc.getPreProcessorForInputType(t)
            t_in = pp.getOutputType(t) if pp is not None else t
            t = lc.getOutputType(idx, t_in)
            out[name] = (t_in, t)
        return out

    def setInput(self, x):
        self.input = x

    def setLabels(self, y):
        self.labels = y

    def setLayerMaskArrays(self, fmask, lmask):
        self.mask, self.labelsMask = fmask, lmask

    def clearLayerMaskArrays(self):
        self.mask = self.labelsMask = None

    # ------------------------------------------------------------------------------ pretraining
    def pretrainLayer(self, layerIdx, data, numEpochs=1):
        """Unsupervised pretraining of one AutoEncoder / VAE layer (reference MultiLayerNetwork.pretrainLayer):
        inputs are the activations of layers [0, layerIdx) in inference mode."""
        if not self.initCalled:
            self.init()
        impl = self.layers[layerIdx]
        if not hasattr(impl, "computePretrainGradientAndScore"):
            return self
        for _ in range(numEpochs):
            items = [data] if isinstance(data, DataSet) or torch.is_tensor(data) else data
            if not isinstance(items, list):
                items.reset()
            for ds in items:
                f = ds if torch.is_tensor(ds) else ds.features
                x = self._to_dev(f, self._feat_dtype())
                with torch.no_grad():
                    if layerIdx > 0:
                        x = self.feedForwardToLayer(layerIdx - 1, x, False)[-1]
                    x = self._pp(layerIdx, x, x.shape[0], False)
                self._pretrain_step(impl, x)
        return self

    def pretrain(self, data, numEpochs=1):
        """Layer-wise pretraining of every pretrainable layer in order (reference MultiLayerNetwork.pretrain)."""
        for i, l in enumerate(self.layers):
            if hasattr(l, "computePretrainGradientAndScore"):
                self.pretrainLayer(i, data, numEpochs)
        return self

    def toComputationGraph(self):
        from ..utils.network_utils import to_computation_graph
        return to_computation_graph(self)

    def save(self, path, saveUpdater=True):
        from ..utils.model_serializer import ModelSerializer
        ModelSerializer.writeModel(self, path, saveUpdater)

    @staticmethod
    def load(path, loadUpdater=True):
        from ..utils.model_serializer import ModelSerializer
        return ModelSerializer.restoreMultiLayerNetwork(path, loadUpdater)

    def clear(self):
        for l in self.layers:
            l.clear()
