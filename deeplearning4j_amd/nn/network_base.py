"""Shared machinery of MultiLayerNetwork and ComputationGraph.

* ONE flat parameter vector [1, P] (master fp32, fp64 for gradient checks), ONE flat gradient vector,
  ONE flat updater-state vector; every layer holds views (reference MultiLayerNetwork.java:584-637,691-720).
* Reduced-precision compute (DataType.BFLOAT16/HALF): a flat bf16 shadow of the parameters that the
  fused updater kernel rewrites in the same pass that updates the master weights.
* Parameters are allocated once on the device in HBM; on MI355X (288 GB/GPU) the whole training state
  of every zoo model stays resident.
* Score is kept on device (no host sync per iteration); ``score()`` syncs lazily.
"""
import os
import time

import torch

from .conf.enums import DataType
from .conf.weights import WeightInit, init_weights_
from .updater import NetworkUpdater, build_entries
from .layers.base import ParamTable
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402
from .. import profiling as _prof


def default_device():
    d = os.environ.get("DL4J_AMD_DEVICE")
    if d:
        return torch.device(d)
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def make_view(flat, off, spec):
    n = spec.numel
    v = flat[off:off + n]
    if spec.order == "f" and len(spec.shape) == 2:
        return v.reshape(spec.shape[1], spec.shape[0]).t()
    if spec.order == "f":
        return v.reshape(list(reversed(spec.shape))).permute(*reversed(range(len(spec.shape))))
    return v.reshape(spec.shape)


def init_param_(view, spec, conf, gen):
    kind = spec.kind
    if kind in ("weight", "recurrent"):
        scheme = conf.weightInit
        dist = getattr(conf, "dist", None)
        if kind == "recurrent" and getattr(conf, "weightInitRecurrent", None) is not None:
            scheme = conf.weightInitRecurrent
            dist = getattr(conf, "distRecurrent", None) or dist
        if scheme is None:
            scheme = WeightInit.XAVIER
        shape = spec.shape
        init_weights_(view, spec.fan_in, spec.fan_out, shape, scheme, dist, gen)
    elif kind == "bias":
        view.fill_(float(getattr(conf, "biasInit", 0.0) or 0.0))
    elif kind == "const":
        view.fill_(float(spec.value))
    elif kind == "zero":
        view.zero_()
    elif kind == "lstm_bias":
        view.zero_()
        H = spec.numel // 4
        view.reshape(-1)[H:2 * H].fill_(float(spec.value))
    else:
        raise ValueError(kind)


def _apply_output_mask(out, m):
    """Zero the label-masked entries of an output layer's activations (reference RnnOutputLayer.output :131-155 and
    BaseOutputLayer.applyMask :427-435): [mb, T] per-step masks on [mb, n, T] outputs, per-output masks of the
    output's own shape, [mb] / [mb, 1] per-example masks on 2-D outputs."""
    if m is None:
        return out
    m = m.to(device=out.device, dtype=out.dtype)
    if m.shape == out.shape:
        return out * m
    if out.dim() == 3 and m.dim() == 2:
        return out * m.unsqueeze(1)
    if out.dim() == 2 and m.numel() == out.shape[0]:
        return out * m.reshape(-1, 1)
    raise ValueError(f"label mask of shape {tuple(m.shape)} does not fit output {tuple(out.shape)}")


class BaseNetwork:
    def __init__(self, conf):
        self.conf = conf
        self.listeners = []
        self.initCalled = False
        self._score_t = None
        self._score_val = None
        self.lastEtlTime = 0
        self.device = None

    # ------------------------------------------------------------------------------ setup
    @property
    def dataType(self):
        return self.conf.dataType

    def _setup_flat(self, layer_list, params=None, clone=False, device=None):
        """layer_list: [(idx, name, impl)] in flattening order."""
        self.device = torch.device(device) if device is not None else default_device()
        dt = self.conf.dataType
        self.master_dtype = dt.master_dtype()
        self.compute_dtype = dt.torch_dtype()
        if self.device.type == "cpu" and self.compute_dtype in (torch.bfloat16, torch.float16) and \
                os.environ.get("DL4J_AMD_CPU_LOWP", "0") != "1":
            # CPU reference path computes in fp32 (bf16 GEMMs on CPU are slow and not the target)
            self.compute_dtype = torch.float32
        total = sum(impl.conf.numParams() for _, _, impl in layer_list)
        self._numParams = total
        if params is not None:
            p = params.reshape(-1)
            if p.numel() != total:
                raise ValueError(f"Invalid parameters: expected {total} params, got {p.numel()}")
            flat = p.to(self.device, self.master_dtype)
            # cloneParametersArray=False adopts the caller's vector (the layers' parameters become views of it,
            # reference MultiLayerNetwork.init(INDArray, boolean)); a device / dtype change copies anyway
            flat = flat.clone() if clone else flat
            init = False
        else:
            flat = torch.zeros(total, dtype=self.master_dtype, device=self.device)
            init = True
        self.flattenedParams = flat
        self.flattenedGradients = torch.zeros(total, dtype=self.master_dtype, device=self.device)
        self.shadow = None
        if self.compute_dtype != self.master_dtype:
            self.shadow = torch.empty(total, dtype=self.compute_dtype, device=self.device)
        gen = torch.Generator().manual_seed(int(self.conf.seed))
        off = 0
        self._layer_offsets = []
        self._conv_ws = None
        self._offset_of = {}
        for idx, name, impl in layer_list:
            impl.net = self
            self._layer_offsets.append((idx, name, impl, off))
            self._offset_of[idx] = off
            self._offset_of[name] = off
            o = off
            impl.params, impl.grads, impl.cparams = ParamTable(), ParamTable(), ParamTable()
            for spec in impl.conf.param_specs():
                v = make_view(flat, o, spec)
                if init:
                    host = torch.empty(spec.numel, dtype=self.master_dtype)
                    hv = make_view(host, 0, spec)
                    iconf = impl.conf
                    while getattr(iconf, "underlying", None) is not None:   # wrappers (Bidirectional, Frozen...)
                        iconf = iconf.underlying
                    init_param_(hv, spec, iconf, gen)
                    with torch.no_grad():
                        flat[o:o + spec.numel].copy_(host.to(self.device))
                impl.params[spec.key] = v
                impl.grads[spec.key] = make_view(self.flattenedGradients, o, spec)
                if self.shadow is not None:
                    impl.cparams[spec.key] = make_view(self.shadow, o, spec)
                    v._dl4j_shadow = impl.cparams[spec.key]     # a library GEMM's bias epilogue takes the 16-bit copy
                else:
                    impl.cparams[spec.key] = v
                o += spec.numel
            impl.params.flat = flat[off:o]
            impl.grads.flat = self.flattenedGradients[off:o]
            off = o
        if self.shadow is not None:
            with torch.no_grad():
                self.shadow.copy_(flat)
        if self.device.type == "cuda":
            from ..ops import conv_native
            conv_native.register_managed(flat)          # every update of these bumps the weight version
            if self.shadow is not None:
                conv_native.register_managed(self.shadow)
        self.updater = NetworkUpdater(self, build_entries(self._layer_offsets))
        self.updater.init_state(self.device, self.master_dtype)
        self.initCalled = True

    def _freeze_layer_in_place(self, key):
        """Wrap a live layer in a FrozenLayer (reference GraphVertex.setLayerAsFrozen / FrozenLayer(layer)): the
        wrapper shares the layer's parameter and gradient views, so nothing moves in the flat vectors; the updater is
        rebuilt so the layer's segment gets the NoOp update (its previous updater state is dropped). The network
        configuration is left as it was, as in the reference (only the runtime layer changes)."""
        from .conf.layers import FrozenLayer
        from .updater import NetworkUpdater, build_entries
        for i, (idx, name, impl, off) in enumerate(self._layer_offsets):
            if key not in (idx, name):
                continue
            if isinstance(impl.conf, FrozenLayer):
                return impl
            conf = FrozenLayer(layer=impl.conf, layerName=getattr(impl.conf, "layerName", None))
            fz = conf.instantiate(index=impl.index, net=self)
            fz.inner = impl
            fz.params, fz.grads, fz.cparams = impl.params, impl.grads, impl.cparams
            fz.bind()
            self._layer_offsets[i] = (idx, name, fz, off)
            self._replace_impl(idx, name, impl, fz)
            self.updater = NetworkUpdater(self, build_entries(self._layer_offsets))
            self.updater.init_state(self.device, self.master_dtype)
            return fz
        raise ValueError(f"No layer {key!r}")

    def _replace_impl(self, idx, name, old, new):
        raise NotImplementedError

    def _params_changed(self):
        """Parameters were modified outside the fused updater (line search, setParams): refresh the bf16 compute
        shadow and invalidate weight relayout caches."""
        self.sync_shadow()

    def _fit_batch(self, x, y, fmask=None, lmask=None):
        """One optimizer iteration on a minibatch; afterwards no layer keeps the iteration's mask arrays
        (reference MultiLayerNetwork.fit -> clearLayerMaskArrays)."""
        try:
            return self._fit_batch_step(x, y, fmask, lmask)
        finally:
            if fmask is not None or lmask is not None:
                for _, _, impl, _ in self._layer_offsets:
                    impl.maskArray = None

    def _fit_batch_step(self, x, y, fmask=None, lmask=None):
        """The fused SGD-family step, or a line-search optimizer (LBFGS / CG / line GD) when the configuration
        asks for one (reference Solver.java:50-84)."""
        from .conf.enums import OptimizationAlgorithm as OA
        algo = self.conf.globalConf.get("optimizationAlgo") if hasattr(self.conf, "globalConf") else None
        if algo is None or OA.of(algo) == OA.STOCHASTIC_GRADIENT_DESCENT:
            if getattr(self, "_hipgraph_enabled", False):
                xs = list(x) if isinstance(x, (list, tuple)) else [x]
                ys = list(y) if isinstance(y, (list, tuple)) else [y]
                if self._try_graph_step(xs, ys, fmask, lmask):
                    return None
                from ..memory.arena import training_scope
                with training_scope(self):               # eager warmup: learns the iteration's workspace size
                    return self._fit_batch_sgd(x, y, fmask, lmask)
            from ..memory.arena import training_scope
            with training_scope(self):                   # LOOP_FF_BP workspace for this iteration's activations
                return self._fit_batch_sgd(x, y, fmask, lmask)
        if getattr(self, "_solver", None) is None:
            from ..optimize.solvers import Solver
            self._solver = Solver(self)
        self._solver.optimize(x, y, fmask, lmask)

    def _score_batch(self, x, y, fmask=None, lmask=None):
        from ..datasets import DataSet, MultiDataSet
        ds = MultiDataSet(x, y, fmask, lmask) if isinstance(x, (list, tuple)) else DataSet(x, y, fmask, lmask)
        return self._score_dataset(ds, training=True)

    # ------------------------------------------------------------------------------ layer-wise pretraining
    def _layer_range(self, impl):
        for _, _, li, off in self._layer_offsets:
            if li is impl:
                n = sum(s.numel for s in impl.conf.param_specs())
                return off, off + n
        raise KeyError("layer not part of this network")

    def _pretrain_step(self, impl, x):
        """One unsupervised step of a pretrain layer (AutoEncoder / VAE) on its own input activations
        (reference MultiLayerNetwork.pretrainLayer -> layer.fit): only that layer's params/state change."""
        self.flattenedGradients.zero_()
        score = impl.computePretrainGradientAndScore(x)
        lo, hi = self._layer_range(impl)
        self.updater.update_range(self.flattenedParams, self.flattenedGradients, self.conf.iterationCount,
                                  self.conf.epochCount, x.shape[0], lo, hi)
        self._params_changed()
        self._score_t, self._score_val = score, None
        self._iteration_done()
        return score

    def getLastEtlTime(self):
        return getattr(self, "lastEtlTime", 0.0)

    def sync_shadow(self):
        if self.shadow is not None:
            with torch.no_grad():
                self.shadow.copy_(self.flattenedParams)
        self._bump_weight_version()

    def _prepare_conv_weights(self):
        """Refresh the MFMA-kernel layouts of all conv weights in one batched launch before a training forward
        pass (instead of one relayout launch per conv per direction)."""
        if self.device is None or self.device.type != "cuda":
            return
        ws = getattr(self, "_conv_ws", None)
        if ws is None:
            # the compute-dtype views (bf16 shadow of fp32 masters) are what the conv kernels consume
            ws = [impl.cparams.get("W", impl.params["W"]) for _, _, impl, _ in self._layer_offsets
                  if type(impl.conf).__name__ == "ConvolutionLayer" and "W" in impl.params
                  and getattr(impl.conf, "weightNoise", None) is None]
            self._conv_ws = ws
        if ws:
            from ..ops import conv_native
            conv_native.relayout_all(ws)

    @staticmethod
    def _bump_weight_version():
        from ..ops import conv_native
        conv_native.bump_version()

    # ------------------------------------------------------------------------------ params API
    def numParams(self, backwards=False):
        return self._numParams

    def getFlattenedGradients(self):
        """The flat gradient vector (a view; reference getFlattenedGradients)."""
        return self.flattenedGradients

    def params(self):
        return self.flattenedParams.reshape(1, -1)

    def setParams(self, p):
        with torch.no_grad():
            self.flattenedParams.copy_(p.reshape(-1).to(self.flattenedParams))
        self.sync_shadow()

    def setParameters(self, p):
        self.setParams(p)

    def getGradientsViewArray(self):
        return self.flattenedGradients.reshape(1, -1)

    def getUpdater(self):
        return self.updater

    def setUpdater(self, u):
        self.updater = u

    def paramTable(self, backpropOnly=False):
        out = {}
        for idx, name, impl, _ in self._layer_offsets:
            for k, v in impl.params.items():
                out[f"{name if self._key_by_name else idx}_{k}"] = v
        return out

    def getParam(self, key):
        return self.paramTable()[key]

    def setParam(self, key, val):
        with torch.no_grad():
            self.paramTable()[key].copy_(val.reshape(self.paramTable()[key].shape))
        self.sync_shadow()

    def gradient(self):
        from .gradient import Gradient
        g = Gradient(self.flattenedGradients.reshape(1, -1))
        for idx, name, impl, _ in self._layer_offsets:
            for k, v in impl.grads.items():
                g.setGradientFor(f"{name if self._key_by_name else idx}_{k}", v)
        return g

    # ------------------------------------------------------------------------------ listeners
    def setListeners(self, *ls):
        self.listeners = [x for l in ls for x in (l if isinstance(l, (list, tuple)) else [l])]

    def addListeners(self, *ls):
        self.listeners += [x for l in ls for x in (l if isinstance(l, (list, tuple)) else [l])]

    def getListeners(self):
        return self.listeners

    # ------------------------------------------------------------------------------ score
    def score(self, dataset=None, training=False):
        if dataset is not None:
            return self._score_dataset(dataset, training)
        if self._score_val is None and self._score_t is not None:
            self._score_val = float(self._score_t)
        return self._score_val

    def setScore(self, s):
        self._score_t = None
        self._score_val = s

    def _regularization_terms(self):
        """(l1, l2) summed over the whole network, as device tensors (no host sync)."""
        l1 = None
        l2 = None
        for _, _, impl, _ in self._layer_offsets:
            for k, p in impl.params.items():
                c1 = impl.conf.l1For(k)
                c2 = impl.conf.l2For(k)
                if c1 > 0:
                    t = p.abs().sum() * c1
                    l1 = t if l1 is None else l1 + t
                if c2 > 0:
                    t = (_acc(p) * _acc(p)).sum() * (0.5 * c2)
                    l2 = t if l2 is None else l2 + t
        z = torch.zeros((), device=self.device)
        return (l1 if l1 is not None else z), (l2 if l2 is not None else z)

    def calcL1(self, backpropOnly=True):
        return float(self._regularization_terms()[0])

    def calcL2(self, backpropOnly=True):
        return float(self._regularization_terms()[1])

    # ------------------------------------------------------------------------------ iteration counters
    def getIterationCount(self):
        return self.conf.iterationCount

    def setIterationCount(self, n):
        self.conf.iterationCount = n

    def getEpochCount(self):
        return self.conf.epochCount

    def setEpochCount(self, n):
        self.conf.epochCount = n

    def incrementEpochCount(self):
        self.conf.epochCount += 1

    # ------------------------------------------------------------------------------ DP hooks
    def _begin_backward(self):
        # On the GPU, clear the whole flat gradient with ONE fill so layers whose kernels accumulate (conv
        # weight-gradient atomics, fused bias sums) need no per-layer memset launches.
        self._grads_zeroed = self.flattenedGradients is not None and self.flattenedGradients.is_cuda and \
            self._grad_zero_needed()
        if self._grads_zeroed:
            from ..ops.nd4j_kernels import zero_
            zero_(self.flattenedGradients)
        acc = getattr(self, "gradientsAccumulator", None)
        if acc is not None and hasattr(acc, "begin_backward"):
            acc.begin_backward(self)
        from ..ops import side_stream
        side_stream.begin(self.flattenedGradients)   # conv weight gradients overlap the rest of the reverse pass

    def _grad_zero_needed(self):
        """False when every layer of an MLN overwrites its whole gradient views (``GRADS_OVERWRITE``), so the
        per-step fill of the flat gradient is skipped (e.g. LSTM + RNN-output networks)."""
        v = getattr(self, "_grad_zero_cache", None)
        if v is None:
            layers = getattr(self, "layers", None)
            v = not (isinstance(layers, list) and layers and
                     all(getattr(l, "GRADS_OVERWRITE", False) or not getattr(l, "grads", None) for l in layers))
            self._grad_zero_cache = v
        return v

    def _end_backward(self):
        from ..ops import side_stream
        side_stream.end()

    def _grad_ready(self, key):
        acc = getattr(self, "gradientsAccumulator", None)
        if acc is not None and hasattr(acc, "grad_ready"):
            if not getattr(acc, "joins_side_stream", False):
                from ..ops import side_stream
                side_stream.join()                  # a bucket may read gradients the side stream still writes
            acc.grad_ready(self, self._offset_of.get(key, 0))

    def setGradientsAccumulator(self, acc):
        self.gradientsAccumulator = acc

    def _zero_contribution_step(self, batch_size):
        """A data-parallel replica with no batch in the trailing partial round of an epoch (reference
        PW:ParallelWrapper.java:514-578 trains such a round on the first ``locker`` workers only): it contributes a
        zero gradient to the round's all-reduce and applies the same update as the replicas that trained, so all
        replicas stay identical."""
        self.flattenedGradients.zero_()
        acc = getattr(self, "gradientsAccumulator", None)
        if acc is not None and hasattr(acc, "begin_backward"):
            acc.begin_backward(self)
        self._loss_part = None
        self._apply_update(batch_size)
        self._iteration_done()

    # ------------------------------------------------------------------------------ update step
    def _apply_update(self, batch_size):
        it, ep = self.conf.iterationCount, self.conf.epochCount
        for l in self.listeners:
            if hasattr(l, "onGradientCalculation"):
                l.onGradientCalculation(self)
        acc = getattr(self, "gradientsAccumulator", None)
        if acc is not None and getattr(acc, "handles_update", False):
            # encoded update sharing: the accumulator runs updater -> encode -> exchange -> apply itself
            acc.apply_update(self, batch_size, it, ep)
            self._loss_part = None
            self._score_val = None
            return
        if acc is not None:
            with _prof.range_("allreduce_gradients", "collective", self.device):
                acc.reduce_gradients(self)   # data-parallel all-reduce of the summed gradient (parallel/)
        with _prof.range_("updater", "update", self.device):
            self._apply_update_kernels(batch_size)
        self._bump_weight_version()

    def _apply_update_kernels(self, batch_size):
        """The device work of an update (fused updater + score's regularisation term + constraints); no host
        bookkeeping, so it can be captured into a HIP graph."""
        from ..ops import side_stream
        side_stream.end()                           # a pass that raised mid-way must not leave dW launches unjoined
        it, ep = self.conf.iterationCount, self.conf.epochCount
        acc = getattr(self, "gradientsAccumulator", None)
        mb_local = batch_size
        if acc is not None and not getattr(acc, "average", False):
            # summed gradients of every replica: divide by the global batch (an averaging accumulator already did
            # the 1/world part); user accumulators without a world_size count as one replica
            # (a partial data-parallel round divides by the replicas that really trained: ``participants``)
            batch_size = batch_size * (getattr(acc, "participants", None) or getattr(acc, "world_size", 1))
            if getattr(acc, "global_batch", None):
                batch_size = acc.global_batch       # the round's total example count, identical on every replica
        elif acc is not None and getattr(acc, "global_batch", None):
            # averaging accumulator: gradients were already divided by the replica count
            batch_size = acc.global_batch / (getattr(acc, "participants", None) or getattr(acc, "world_size", 1))
        reg = None
        if any(sg.l1 > 0 or sg.l2 > 0 for sg in self.updater.plan.segments):
            # the HIP updater writes (not accumulates) it; the host path expects zeros
            reg = torch.empty(1, dtype=self.master_dtype, device=self.device) if self.device.type == "cuda" and \
                self.master_dtype == torch.float32 else torch.zeros(1, dtype=self.master_dtype, device=self.device)
        self.updater.update(self.flattenedParams, self.flattenedGradients, it, ep, batch_size, self.shadow, reg)
        lp = getattr(self, "_loss_part", None)
        if lp is not None:
            from ..ops import native as _native
            if reg is not None and _native.score_reduce_ok(reg, lp if torch.is_tensor(lp) else None) and \
                    torch.is_tensor(lp) and lp.numel() == 1:
                # score = loss + reg / minibatch on one in-tree block (no library elementwise kernels)
                self._score_t = _native.score_reduce(reg, 0.0, 1.0 / mb_local, reg=lp.reshape(1), reg_scale=1.0)
            elif reg is None:
                self._score_t = lp                  # no regularisation term: the loss part is the score
            else:
                self._score_t = lp + reg[0] / mb_local
            self._loss_part = None
            self._score_val = None
        for _, _, impl, _ in self._layer_offsets:
            if getattr(impl.conf, "constraints", None):
                impl.applyConstraints(it, ep)

    # ------------------------------------------------------------------------------ helper fallbacks
    def helperCountFail(self):
        """Number of GPU op calls that could not run on an in-tree HIP kernel and took a library / torch path
        (reference ConvolutionLayer.helperCountFail, NN:nn/layers/convolution/ConvolutionLayer.java:58,173-200 —
        here counted process-wide per op; see ops/fallback.py, DL4J_AMD_STRICT_KERNELS=1 makes them errors)."""
        from ..ops import fallback
        return fallback.count()

    def fallbackSummary(self):
        from ..ops import fallback
        return fallback.summary()

    # ------------------------------------------------------------------------------ HIP graphs
    def enableHipGraphs(self, enabled=True, warmup=2):
        """Capture the training iteration into HIP graphs after ``warmup`` eager iterations of a fixed batch
        shape, then replay (see nn/hipgraph.py). Falls back to eager steps whenever a batch is not eligible."""
        self._hipgraph_enabled = bool(enabled)
        self._hipgraph_warmup = int(warmup)
        self._hipgraph = None
        self._hipgraph_seen = 0
        self._hipgraphs = {}
        self._hipgraph_seen_by = {}
        return self

    def _try_graph_step(self, inputs, labels, fmasks, lmasks, tbptt_back=None):
        """One training iteration (or, with ``tbptt_back``, one TBPTT window) as a HIP-graph replay when eligible;
        False = run it eagerly. One captured step per distinct shape signature (input / label / mask shapes and
        the window), each captured after ``warmup`` eager iterations of that signature."""
        if not getattr(self, "_hipgraph_enabled", False):
            return False
        from .hipgraph import CapturedTrainingStep, Sig, carries_state, graph_eligible
        fm = None if fmasks is None else [None if m is None else self._to_dev(m)
                                          for m in (fmasks if isinstance(fmasks, (list, tuple)) else [fmasks])]
        lm = None if lmasks is None else [None if m is None else self._to_dev(m)
                                          for m in (lmasks if isinstance(lmasks, (list, tuple)) else [lmasks])]
        # on the device, not yet cast: a replay's copy into the static buffers does the cast in the same kernel
        raw_in = [self._to_dev(t) for t in inputs]
        raw_lab = [self._to_dev(t) for t in labels]
        fdt, ldt = self._feat_dtype(), self.master_dtype

        def cast_sig(ts, dt):
            return [Sig(t.shape, dt if t.is_floating_point() else t.dtype) for t in ts]
        sig_in, sig_lab = cast_sig(raw_in, fdt), cast_sig(raw_lab, ldt)
        if not graph_eligible(self, raw_in, raw_lab, fm, lm, tbptt_window=tbptt_back is not None):
            return False
        key = CapturedTrainingStep.key(sig_in, sig_lab, fm, lm, tbptt_back)
        if tbptt_back is not None:
            key = key + (carries_state(self),)
        graphs = self.__dict__.setdefault("_hipgraphs", {})
        cs = graphs.get(key)
        if cs is not None and cs.ok:
            cs.step(raw_in, raw_lab, fm, lm)
            self._hipgraph = cs
            return True
        inputs = [t.to(fdt) if t.is_floating_point() else t for t in raw_in]
        labels = [t.to(ldt) if t.is_floating_point() else t for t in raw_lab]
        seen = self.__dict__.setdefault("_hipgraph_seen_by", {})
        seen[key] = seen.get(key, 0) + 1
        self._hipgraph_seen = seen[key]
        if seen[key] <= self._hipgraph_warmup:
            return False                           # eager warmup iterations populate every cache first
        cs = CapturedTrainingStep(self, inputs, labels, fm, lm, tbptt_back)
        self._bump_weight_version()
        cs.capture()                               # a failed capture leaves the stream unusable: let it raise
        graphs[key] = cs
        self._hipgraph = cs
        cs.step(inputs, labels, fm, lm)
        return True

    def _iteration_done(self):
        self.conf.iterationCount += 1
        for l in self.listeners:
            if hasattr(l, "iterationDone"):
                l.iterationDone(self, self.conf.iterationCount, self.conf.epochCount)

    def _to_dev(self, t, dtype=None):
        if t is None:
            return None
        if hasattr(t, "toTensor"):                       # nd4j.INDArray
            t = t.toTensor()
        if not torch.is_tensor(t):
            import numpy as np
            t = torch.from_numpy(np.asarray(t))
        t = t.to(self.device, non_blocking=True)
        if dtype is not None and t.is_floating_point() and t.dtype != dtype and t.is_cuda:
            # cast (and, for images, NCHW -> channels-last) in one in-tree strided-copy launch
            from ..ops import nd4j_kernels as NK
            src = t.permute(0, 2, 3, 1) if t.dim() == 4 else t
            c = NK.cast_pad_last(src, dtype, src.shape[-1]) if t.dim() > 0 and t.numel() else None
            if c is not None:
                t = c.permute(0, 3, 1, 2) if t.dim() == 4 else c
        if dtype is not None and t.is_floating_point():
            t = t.to(dtype)
        if t.dim() == 4 and t.is_cuda:
            t = t.contiguous(memory_format=torch.channels_last)
        return t

    def _feat_dtype(self):
        return self.compute_dtype

    def _input_check(self, inputs):
        """True when this forward must run the per-layer input checks (conf/validation.py): the first time each
        network-input shape signature is seen. Layer shapes downstream are a function of it, so repeated steps of
        the same shape skip the host checks; ``_validated`` is set by the caller once a full forward succeeded."""
        key = tuple(tuple(t.shape) for t in inputs)
        if getattr(self, "_validated", None) == key:
            return None
        return key

    def _index_checked(self):
        """Layers whose input VALUES are checked on every forward (embedding index range, host tensors only)."""
        if getattr(self, "_idx_layers", None) is None:
            from .conf.layers import EmbeddingLayer
            confs = self.conf.confs if hasattr(self.conf, "confs") else {
                n: v.layerConf for n, v in self.conf.vertices.items() if hasattr(v, "layerConf")}
            items = enumerate(confs) if isinstance(confs, list) else confs.items()
            self._idx_layers = {k for k, c in items if isinstance(c, EmbeddingLayer)}
        return self._idx_layers

    def summary(self, *inputTypes):
        """Per-layer table (index, name, type, parameter count); with the network's input type(s) — as the
        reference's summary(InputType...) — also each layer's input and output activation types."""
        io = self._summary_types(inputTypes) if inputTypes else {}
        head = f"{'idx':>4} {'name':<28} {'type':<32} {'nParams':>12}"
        if io:
            head += f"  {'input type':<40} {'output type'}"
        lines = [head]
        total = 0
        for idx, name, impl, _ in self._layer_offsets:
            n = impl.conf.numParams()
            total += n
            row = f"{idx:>4} {str(name):<28} {type(impl.conf).__name__:<32} {n:>12,}"
            if io and name in io:
                row += f"  {str(io[name][0]):<40} {io[name][1]}"
            lines.append(row)
        lines.append(f"Total Parameters: {total:,}")
        lines.append(f"Compute dtype: {self.compute_dtype}, device: {self.device}")
        return "\n".join(lines)

    def _summary_types(self, inputTypes):
        return {}

    def memoryReport(self, minibatch=1):
        from .conf.memory import network_memory_report
        return network_memory_report(self, minibatch)

    def _timer(self):
        return time.perf_counter()
