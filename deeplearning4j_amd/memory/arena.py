"""Per-iteration activation arena for training (reference MultiLayerNetwork.java:126-144 / ComputationGraph.java:
107-136: the LOOP_FF / LOOP_BP workspaces opened around each iteration).

``training_scope(net)`` opens this thread's ``LOOP_FF_BP`` MemoryWorkspace (csrc/runtime/workspace.cpp bump arena:
learning policy FIRST_LOOP, overallocation 0.2, reset every cycle) for one fit iteration; while it is open, op
outputs allocated through :func:`empty` — GEMM outputs (ops/gemm.py) and the conv forward / backward-data outputs
(ops/conv_native.py) — are carved from it instead of the caching allocator. Allocation order is identical every
iteration, so after the first (learning) cycle every activation gets the same address each step. Arrays carved
in an iteration are invalid after it: ``memory.workspace.check_scope`` raises (SCOPE_PANIC) on such a leaked
array, and anything handed back to the user is allocated outside the scope.
"""
import threading

import torch

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
    """Networks whose iteration carries no activation into the next one (no recurrent state / TBPTT)."""
    from ..nn.conf.enums import WorkspaceMode
    g = getattr(net.conf, "globalConf", None) or {}
    mode = g.get("trainingWorkspaceMode", WorkspaceMode.ENABLED) if isinstance(g, dict) else WorkspaceMode.ENABLED
    if WorkspaceMode.of(mode) != WorkspaceMode.ENABLED:
        return False
    for _, _, impl, _ in getattr(net, "_layer_offsets", []):
        name = type(impl.conf).__name__
        if any(k in name for k in ("LSTM", "Rnn", "Recurrent", "Bidirectional", "LastTimeStep", "AutoEncoder",
                                   "Variational")):
            return False
    return True


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
        from .workspace import (AllocationPolicy, LearningPolicy, ResetPolicy, SpillPolicy, WorkspaceConfiguration,
                                getWorkspaceManager)
        ws = getattr(net, "_loop_ws", None)
        if ws is None:
            conf = WorkspaceConfiguration(initialSize=0, overallocationLimit=0.2,
                                          policyAllocation=AllocationPolicy.OVERALLOCATE,
                                          policyLearning=LearningPolicy.FIRST_LOOP, policyReset=ResetPolicy.BLOCK_LEFT,
                                          policySpill=SpillPolicy.REALLOCATE)
            ws = net._loop_ws = getWorkspaceManager().getWorkspaceForCurrentThread(
                conf, f"LOOP_FF_BP_{id(net)}", device=net.device)
        ws.notifyScopeEntered()
        _tl.ws = self.ws = ws
        return self

    def __exit__(self, *a):
        if self.ws is not None:
            _tl.ws = None
            self.ws.notifyScopeLeft()
        return False
