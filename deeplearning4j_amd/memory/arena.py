"""Per-iteration activation arena for training (reference MultiLayerNetwork.java:126-144 / ComputationGraph.java:
107-136: the LOOP_FF / LOOP_BP workspaces opened around each iteration).

``training_scope(net)`` opens this thread's ``LOOP_FF_BP`` MemoryWorkspace (csrc/runtime/workspace.cpp bump arena:
learning policy FIRST_LOOP, overallocation 0.2, reset every cycle) for one fit iteration; while it is open, op
outputs allocated through :func:`empty` — GEMM outputs (ops/gemm.py) and the conv forward / backward-data outputs
(ops/conv_native.py) — are carved from it instead of the caching allocator. Allocation order is identical every
iteration, so after the first (learning) cycle every activation gets the same address each step. Arrays carved
in an iteration are invalid after it: ``memory.workspace.check_scope`` raises (SCOPE_PANIC) on such a leaked
array, and anything handed back to the user is allocated outside the scope.
Recurrent networks: ``tbptt_scope`` gives every truncated-BPTT window its own LOOP_TBPTT arena (nested in the
iteration's), and the LSTM sequence kernels' per-call buffers (outputs, gate / cell caches: the reference's LOOP_LSTM
working memory) are carved from whichever arena is open; state carried past a scope is leveraged out of it.
"""
import logging
import threading

import torch

log = logging.getLogger("deeplearning4j_amd")

_tl = threading.local()


def current():
    return getattr(_tl, "ws", None)


def empty(shape, dtype, device, channels_last=False):
    """``torch.empty`` from the open training arena of this thread (same device), else from the caching allocator.
    ``channels_last``: a 4-D NCHW-logical tensor with NHWC storage."""
    ws = current()
    device = torch.device(device)
    if ws is None or ws.device.type != device.type or (device.index is not None and ws.device.index != device.index):
        if channels_last:
            return torch.empty(shape, dtype=dtype, device=device, memory_format=torch.channels_last)
        return torch.empty(shape, dtype=dtype, device=device)
    if channels_last and len(shape) == 4:
        N, C, H, W = shape
        return ws.create((N, H, W, C), dtype).permute(0, 3, 1, 2)
    return ws.create(tuple(shape), dtype)


def _eligible(net):
    """Training-workspace mode ENABLED and no layer whose pretraining / sampling keeps activations across calls
    (AutoEncoder / VAE). Recurrent networks are eligible: the state they carry (TBPTT windows, rnnTimeStep) is
    leveraged out of the arena when a scope closes (:func:`leverage_states`)."""
    from ..nn.conf.enums import WorkspaceMode
    g = getattr(net.conf, "globalConf", None) or {}
    mode = g.get("trainingWorkspaceMode", WorkspaceMode.ENABLED) if isinstance(g, dict) else WorkspaceMode.ENABLED
    if WorkspaceMode.of(mode) != WorkspaceMode.ENABLED:
        return False
    for _, _, impl, _ in getattr(net, "_layer_offsets", []):
        name = type(impl.conf).__name__
        if any(k in name for k in ("AutoEncoder", "Variational")):
            return False
    return True


def _owned(ws, t):
    """True when ``t``'s memory lies inside ``ws``'s arena buffer (views of carved arrays included)."""
    b = getattr(ws, "_buf", None)
    if b is None or not torch.is_tensor(t) or t.device != b.device or t.numel() == 0:
        return False
    p, s = t.data_ptr(), b.data_ptr()
    return s <= p < s + b.numel()


def _layer_impls(net):
    todo = [impl for _, _, impl, _ in getattr(net, "_layer_offsets", [])]
    while todo:
        impl = todo.pop()
        yield impl
        for attr in ("fwd", "bwd", "inner", "underlying"):
            sub = getattr(impl, attr, None)
            if sub is not None and hasattr(sub, "conf"):
                todo.append(sub)


def leverage_states(net, ws):
    """Recurrent state carried beyond a workspace cycle (``stateMap`` / ``tBpttStateMap``) that was carved from
    ``ws`` is copied out of it before the cycle ends (reference: the TBPTT state is leveraged to the outer workspace,
    MultiLayerNetwork.java:1556-1583). Returns the number of arrays moved."""
    moved = 0
    for impl in _layer_impls(net):
        for attr in ("stateMap", "tBpttStateMap"):
            m = getattr(impl, attr, None)
            if not m:
                continue
            for k, v in list(m.items()):
                if _owned(ws, v):
                    m[k] = v.detach().clone()
                    moved += 1
    return moved


def _loop_ws(net, attr, ws_id):
    ws = getattr(net, attr, None)
    if ws is None:
        from .workspace import (AllocationPolicy, LearningPolicy, ResetPolicy, SpillPolicy, WorkspaceConfiguration,
                                getWorkspaceManager)
        conf = WorkspaceConfiguration(initialSize=0, overallocationLimit=0.2,
                                      policyAllocation=AllocationPolicy.OVERALLOCATE,
                                      policyLearning=LearningPolicy.FIRST_LOOP, policyReset=ResetPolicy.BLOCK_LEFT,
                                      policySpill=SpillPolicy.REALLOCATE)
        ws = getWorkspaceManager().getWorkspaceForCurrentThread(conf, f"{ws_id}_{id(net)}", device=net.device)
        setattr(net, attr, ws)
    return ws


class tbptt_scope:
    """One truncated-BPTT window in its own LOOP_TBPTT arena (reference MultiLayerNetwork.doTruncatedBPTT opens the
    LOOP_TBPTT workspace per sub-sequence, :1556-1583): the window's activations, LSTM gate caches and gradients-in-
    flight are carved from it and released at window end; the carried h / c state is leveraged out first."""

    def __init__(self, net):
        self.net = net
        self.ws = None
        self.prev = None

    def __enter__(self):
        net = self.net
        ok = getattr(net, "_ws_ok", None)
        if ok is None:
            ok = net._ws_ok = _eligible(net)
        if not ok:
            return self
        from .workspace import LOOP_TBPTT
        ws = _loop_ws(net, "_tbptt_ws", LOOP_TBPTT)
        if ws.active:
            return self
        self.prev = current()
        ws.notifyScopeEntered()
        _tl.ws = self.ws = ws
        return self

    def __exit__(self, *a):
        if self.ws is not None:
            leverage_states(self.net, self.ws)
            _tl.ws = self.prev
            self.ws.notifyScopeLeft()
        return False


class training_scope:
    """Context manager around one training iteration of ``net`` (no-op when not eligible)."""

    def __init__(self, net):
        self.net = net
        self.ws = None

    def __enter__(self):
        net = self.net
        ok = getattr(net, "_ws_ok", None)
        if ok is None:
            ok = net._ws_ok = _eligible(net)
        if not ok or current() is not None:
            return self
        ws = _loop_ws(net, "_loop_ws", "LOOP_FF_BP")
        ws.notifyScopeEntered()
        _tl.ws = self.ws = ws
        return self

    def __exit__(self, *a):
        if self.ws is not None:
            leverage_states(self.net, self.ws)
            _tl.ws = None
            self.ws.notifyScopeLeft()
            mb = getattr(self.net, "_mb", None)      # the largest minibatch the eager arena has learned from
            if isinstance(mb, int) and mb > getattr(self.net, "_ws_learned_mb", 0):
                self.net._ws_learned_mb = mb
        return False


# ----------------------------------------------------------------------------------- HIP-graph training arenas
def _activation_estimate(net, minibatch):
    """Training-memory estimate of one iteration at ``minibatch`` from the network's memory report (reference
    NN:nn/conf/memory/NetworkMemoryReport.java:58-95), in the compute dtype; 0 when no report is available."""
    try:
        from ..nn.conf.memory import MemoryUseMode
        dt = {torch.bfloat16: "BFLOAT16", torch.float16: "HALF", torch.float64: "DOUBLE"}.get(
            getattr(net, "compute_dtype", torch.float32), "FLOAT")
        return int(net.memoryReport(minibatch).getTotalMemoryBytes(minibatch, MemoryUseMode.TRAINING, None, dt))
    except Exception:
        return 0


def graph_workspace(net, minibatch, key):
    """The LOOP_FF_BP arena a captured training step owns (nn/hipgraph.py): every activation, BN / pooling buffer
    and gradient-in-flight the captured iteration allocates is carved from it, so the graph's private memory IS the
    workspace. Sized per capture key from what the eager warmup iterations' LOOP_FF_BP arena learned (its peak, +5 %,
    scaled by this key's minibatch over the largest minibatch that arena saw, so a smaller tail-batch key gets a
    proportionally smaller arena), or from the memory report when that arena is not available. When the size
    exceeds the free HBM (hipMemGetInfo; the eager arena's buffer counts as free only when it is really released
    here) no arena is made and None is returned: the capture then allocates from the graph's private pool (or the
    step runs eagerly), with a warning naming the numbers. The arena is frozen: its buffer never moves while graphs
    hold its addresses, and an allocation beyond it falls back to the graph's own pool. Returns None for networks
    without a training arena."""
    ok = getattr(net, "_ws_ok", None)
    if ok is None:
        ok = net._ws_ok = _eligible(net)
    if not ok or net.device is None or net.device.type != "cuda":
        return None
    eager = getattr(net, "_loop_ws", None)
    learned = int(eager.stats()["maxPeak"]) if eager is not None else 0
    learned_mb = int(getattr(net, "_ws_learned_mb", 0) or 0)
    if learned > 0 and learned_mb > 0 and 0 < minibatch < learned_mb:
        learned = int(learned * minibatch / learned_mb)
    est = _activation_estimate(net, minibatch)
    need = int(learned * 1.05) + (1 << 20) if learned > 0 else int(est)
    if need <= (1 << 20):
        return None
    free, total = torch.cuda.mem_get_info(net.device)
    # the eager arena's buffer is released below (only when no eager step holds it open), so only then does it count
    # as free for the graph's arena
    releasable = eager is not None and eager._buf is not None and not eager.active
    reusable = eager._buf.numel() if releasable else 0
    if need > free + reusable:
        log.warning("training step of %s at minibatch %d: its workspace needs %.2f GiB (learned peak %.2f GiB, "
                    "memory-report estimate %.2f GiB) but only %.2f GiB of %.1f GiB HBM are free; capturing without "
                    "a frozen arena", type(net).__name__, minibatch, need / 2**30, learned / 2**30, est / 2**30,
                    (free + reusable) / 2**30, total / 2**30)
        return None
    if releasable:
        eager._buf = None                               # the eager arena re-learns if an eager step comes again
        eager._lib.rt_ws_set_capacity(eager._h, 0)
    from .workspace import (AllocationPolicy, LearningPolicy, MemoryWorkspace, ResetPolicy, SpillPolicy,
                            WorkspaceConfiguration)
    conf = WorkspaceConfiguration(initialSize=need, overallocationLimit=0.0, policyAllocation=AllocationPolicy.STRICT,
                                  policyLearning=LearningPolicy.NONE, policyReset=ResetPolicy.BLOCK_LEFT,
                                  policySpill=SpillPolicy.EXTERNAL)
    ws = MemoryWorkspace(conf, f"LOOP_FF_BP_GRAPH_{id(net)}_{abs(hash(key))}", device=net.device)
    ws.frozen = True
    ws.estimate_bytes = est
    return ws


class graph_scope:
    """Open ``ws`` (a graph_workspace) as this thread's training arena around one capture."""

    def __init__(self, net, ws):
        self.net, self.ws, self.prev = net, ws, None

    def __enter__(self):
        if self.ws is not None:
            self.prev = current()
            self.ws.notifyScopeEntered()
            _tl.ws = self.ws
        return self

    def __exit__(self, *a):
        if self.ws is not None:
            leverage_states(self.net, self.ws)
            _tl.ws = self.prev
            self.ws.notifyScopeLeft()
        return False
