"""HIP-graph capture of a whole training iteration (forward + backward + fused update).

The MI355X answer to the reference's per-op executioner dispatch (and to a tracing compiler): once the batch
shape is fixed, one iteration is a fixed sequence of ~600 kernel launches (conv / BN / pool / softmax-xent /
updater). Capturing it once into a HIP graph and replaying it removes the host-side Python/ctypes work and the
inter-kernel launch gaps (measured ≈1.8 ms of a 15.7 ms ResNet-50 step).

Design:
  * Static input/label buffers; each step copies the new batch into them (stream-ordered) and replays.
  * Two graphs (A/B) captured from the same code, alternating replays. Iteration-dependent updater
    hyperparameters (Adam bias correction, learning-rate schedules) reach the fused-updater kernel through a
    per-graph pinned host buffer whose H2D copy is a graph node; the buffer of graph A is rewritten only after
    A's previous replay has finished (event), while B keeps the GPU busy — no host sync in steady state.
  * All memory allocated inside the captured region comes from one private pool shared by both graphs.
  * Host-side bookkeeping (iteration count, weight-version bump, listeners' iterationDone) runs outside the graph.
Data parallel: the AllReduceGradientsAccumulator's bucketed RCCL all-reduces are captured with the step (nccl
backend only); gloo and custom accumulators run eager.
Masks: feature / label masks are static buffers like the inputs (their presence is part of the captured shape).
Truncated BPTT (reference MultiLayerNetwork.doTruncatedBPTT, :1521-1593): every window shape gets its own captured
step (the last window of a sequence may be shorter). The recurrent state carried between windows (each recurrent
layer's tBpttStateMap: h, and c for LSTMs) lives in static buffers: the captured body reads them, and its last nodes
copy the window's final state back into them, so consecutive replays chain the state on the GPU with no host work.
Before a replay the buffers are refreshed from the layer's current map when an eager window (or a new sequence,
state zero) came in between.
Eligibility: plain SGD-family optimizer, a capturable (or no) gradient accumulator, no listeners with per-pass hooks
(onForwardPass/onBackwardPass/onGradientCalculation), CUDA device, fixed shapes. Anything else falls back to the
eager step transparently.
"""
import collections
import contextlib
import gc
import logging
import threading

import torch

log = logging.getLogger("deeplearning4j_amd")

# Python GC stays off while ANY thread captures (a collected cycle owning GPU resources, released inside a capture,
# would abort it); refcounted so that concurrent captures of the in-process ParallelWrapper's workers nest.
_gc_lock = threading.Lock()
_gc_state = {"n": 0, "was": False}

# Captures use thread-local mode: each worker thread of the in-process ParallelWrapper captures its own replica's
# step on its own device, and one thread's capture must not turn another thread's (legal) calls into errors.
CAPTURE_MODE = "thread_local"


_cap_streams = threading.local()


def capture(g, pool, fn, device=None):
    """Capture ``fn()`` into CUDAGraph ``g`` (memory from ``pool``) on a capture stream owned by THIS thread and
    device, in thread-local capture mode, and return fn's result.

    torch.cuda.graph's context manager is not used: it captures on ONE process-wide default capture stream and
    enters with a device-wide synchronize + empty_cache, which breaks concurrent captures by the in-process
    ParallelWrapper's worker threads (one per GPU)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    streams = _cap_streams.__dict__.setdefault("s", {})
    s = streams.get(dev.index)
    if s is None:
        s = streams[dev.index] = torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        g.capture_begin(pool=pool, capture_error_mode=CAPTURE_MODE)
        try:
            out = fn()
        finally:
            g.capture_end()
    cur.wait_stream(s)
    return out


@contextlib.contextmanager
def capture_gc_guard():
    with _gc_lock:
        if _gc_state["n"] == 0:
            gc.collect()
            _gc_state["was"] = gc.isenabled()
            gc.disable()
        _gc_state["n"] += 1
    try:
        yield
    finally:
        with _gc_lock:
            _gc_state["n"] -= 1
            if _gc_state["n"] == 0 and _gc_state["was"]:
                gc.enable()


class Sig(collections.namedtuple("Sig", "shape dtype")):
    """Shape + dtype of a tensor as the captured step will hold it (a replay key before any cast)."""


class CapturedTrainingStep:
    def __init__(self, net, inputs, labels, fmasks=None, lmasks=None, tbptt_back=None):
        self.net = net
        self.is_graph = type(net).__name__ == "ComputationGraph"
        self.static_x = [t.detach().clone() for t in inputs]
        self.static_y = [t.detach().clone() for t in labels]
        self.static_fm = [None if m is None else m.detach().clone() for m in (fmasks or [])]
        self.static_lm = [None if m is None else m.detach().clone() for m in (lmasks or [])]
        self.tbptt_back = tbptt_back
        self.state = []            # (layer, key, static tensor): carried recurrent state of a TBPTT window graph
        self.out_state = []        # per graph slot: (layer, key, tensor) the replayed window leaves as its state
        self.graphs = []
        self.pool = None
        self.score_t = [None, None]
        self.k = 0
        self.ok = False
        self.ws = None             # the step's own LOOP_FF_BP arena (memory/arena.py graph_workspace)

    @staticmethod
    def key(inputs, labels, fmasks, lmasks, tbptt_back):
        def sig(ts):
            return tuple(None if t is None else (tuple(t.shape), t.dtype) for t in (ts or []))
        return sig(inputs), sig(labels), sig(fmasks), sig(lmasks), tbptt_back

    def shapes_match(self, inputs, labels, fmasks=None, lmasks=None):
        return self.key(inputs, labels, fmasks, lmasks, self.tbptt_back) == \
            self.key(self.static_x, self.static_y, self.static_fm, self.static_lm, self.tbptt_back)

    def _recurrent_layers(self):
        return recurrent_layers(self.net)

    def _bind_state(self):
        """Static buffers for the recurrent state the previous (eager) window left in each layer's map."""
        self.state = []
        for l in self._recurrent_layers():
            for k, v in list(l.tBpttStateMap.items()):
                if torch.is_tensor(v):
                    buf = v.detach().clone()
                    self.state.append((l, k, buf))
                    l.tBpttStateMap[k] = buf

    def _body(self):
        n = self.net
        fm = self.static_fm or None
        lm = self.static_lm or None
        tb = self.tbptt_back is not None
        kw = dict(stored_state=True, store_last_for_tbptt=True, tbptt_back=self.tbptt_back) if tb else {}
        if self.is_graph:
            n.computeGradientAndScore(self.static_x, self.static_y, fm, lm, defer_reg=True, **kw)
        else:
            n.computeGradientAndScore(self.static_x[0], self.static_y[0], fm[0] if fm else None,
                                      lm[0] if lm else None, defer_reg=True, **kw)
        dst, src = [], []
        for l, k, buf in self.state:               # the window's final state becomes the next replay's input
            new = l.tBpttStateMap.get(k)
            if new is not None and new is not buf:
                dst.append(buf)
                src.append(new)
            l.tBpttStateMap[k] = buf
        if dst:                                    # one multi-tensor copy node instead of one per state tensor
            torch._foreach_copy_(dst, src)
        acc = getattr(n, "gradientsAccumulator", None)
        if acc is not None:
            acc.reduce_gradients(n)                # bucketed RCCL all-reduces become graph nodes
        n._apply_update_kernels(self.static_x[0].shape[0])
        return n._score_t

    def capture(self):
        from ..ops import native
        n = self.net
        plan = n.updater.plan
        self.pool = torch.cuda.graph_pool_handle()
        native.prepare_graph_slots(plan, n.device, n.conf.iterationCount, n.conf.epochCount)
        if self.tbptt_back is not None:
            self._bind_state()
        torch.cuda.current_stream(n.device).synchronize()
        from ..memory import arena
        self.ws = arena.graph_workspace(n, self.static_x[0].shape[0],
                                        self.key(self.static_x, self.static_y, self.static_fm, self.static_lm,
                                                 self.tbptt_back))
        # no Python GC while capturing: a collected cycle that owns GPU resources (events, other pools' blocks,
        # a previous network's buffers) would be released inside the capture and abort it
        guard = capture_gc_guard()
        guard.__enter__()
        # the recurrent state maps every slot's capture must start from (empty for a sequence's first window)
        start_maps = [(l, dict(l.tBpttStateMap)) for l in self._recurrent_layers()]
        try:
            for slot in (0, 1):
                for l, m in start_maps:            # not the outputs the previous slot's capture left behind
                    l.tBpttStateMap = dict(m)
                n._bump_weight_version()           # every graph must contain its own weight-relayout kernels
                g = torch.cuda.CUDAGraph()
                native.GRAPH_SLOT[0] = slot
                n._capturing = True
                with arena.graph_scope(n, self.ws):   # activations carved from the step's own arena
                    self.score_t[slot] = capture(g, self.pool, self._body, n.device)
                self.graphs.append(g)
                # the A and B graphs own different output tensors: remember which ones this slot writes
                self.out_state.append([(l, k, v) for l in self._recurrent_layers()
                                       for k, v in l.tBpttStateMap.items() if torch.is_tensor(v)]
                                      if self.tbptt_back is not None else [])
            self.ok = True
        finally:
            native.GRAPH_SLOT[0] = None
            n._capturing = False
            guard.__exit__(None, None, None)
        _ = plan
        return self.ok

    def step(self, inputs, labels, fmasks=None, lmasks=None):
        from ..ops import native
        n = self.net
        for d, s in zip(self.static_x, inputs):
            d.copy_(s, non_blocking=True)
        for d, s in zip(self.static_y, labels):
            d.copy_(s, non_blocking=True)
        for d, s in zip(self.static_fm, fmasks or []):
            if d is not None:
                d.copy_(s, non_blocking=True)
        for d, s in zip(self.static_lm, lmasks or []):
            if d is not None:
                d.copy_(s, non_blocking=True)
        for l, k, buf in self.state:               # state left by an eager window / a new sequence (none = zero)
            cur = l.tBpttStateMap.get(k)
            if cur is None:
                buf.zero_()
            elif cur is not buf:
                buf.copy_(cur)
            l.tBpttStateMap[k] = buf
        slot = self.k & 1
        plan = n.updater.plan
        native.refresh_graph_table(plan, slot, n.conf.iterationCount, n.conf.epochCount)
        self.graphs[slot].replay()
        native.mark_graph_replayed(plan, slot)
        from ..ops import rnn_native
        rnn_native.check_step_guard(n.device)
        for l, k, v in self.out_state[slot]:
            l.tBpttStateMap[k] = v
        self.k += 1
        n._score_t = self.score_t[slot]
        n._score_val = None
        n._loss_part = None
        n._bump_weight_version()
        n._mb = self.static_x[0].shape[0]
        n._iteration_done()


def recurrent_layers(net):
    by_name = getattr(net, "layers_by_name", None)
    layers = list(by_name.values()) if by_name else list(getattr(net, "layers", None) or [])
    return [l for l in layers if hasattr(l, "tBpttStateMap")]


def carries_state(net):
    """True when some recurrent layer holds TBPTT state from a previous window (the first window of a sequence
    starts from zero state and is captured as a graph of its own)."""
    return any(torch.is_tensor(v) for l in recurrent_layers(net) for v in l.tBpttStateMap.values())


def graph_eligible(net, inputs, labels, fmasks, lmasks, tbptt_window=False):
    from .conf.enums import BackpropType, OptimizationAlgorithm as OA
    if net.device is None or net.device.type != "cuda":
        return False
    acc = getattr(net, "gradientsAccumulator", None)
    if acc is not None and not (hasattr(acc, "capturable") and acc.capturable()):
        return False                               # gloo / custom accumulators: eager steps
    if acc is not None and getattr(acc, "participants", None):
        return False                               # partial data-parallel round: its divisor is not the captured one
    gb = getattr(acc, "global_batch", None) if acc is not None else None
    if gb and gb != inputs[0].shape[0] * getattr(acc, "world_size", 1):
        return False                               # unequal batches in the round: the divisor is not the captured one
    algo = net.conf.globalConf.get("optimizationAlgo")
    if algo is not None and OA.of(algo) != OA.STOCHASTIC_GRADIENT_DESCENT:
        return False
    if tbptt_window is False and net.conf.backpropType == BackpropType.TruncatedBPTT and inputs[0].dim() == 3:
        return False                               # whole sequences go through the window loop (graph per window)
    for l in net.listeners:
        for h in ("onForwardPass", "onBackwardPass", "onGradientCalculation"):
            f = getattr(type(l), h, None)
            if f is not None and f is not getattr(_NoHooks, h):
                return False
    ms = [m for m in list(fmasks or []) + list(lmasks or []) if m is not None]
    return all(t.is_cuda for t in list(inputs) + list(labels) + ms)


class _NoHooks:
    def onForwardPass(self, model, activations):
        pass

    def onBackwardPass(self, model):
        pass

    def onGradientCalculation(self, model):
        pass


# listeners deriving from the base class inherit no-op hooks: treat them as hook-free
def _base_hooks():
    from ..optimize.listeners import TrainingListener
    for h in ("onForwardPass", "onBackwardPass", "onGradientCalculation"):
        setattr(_NoHooks, h, getattr(TrainingListener, h))


_base_hooks()
