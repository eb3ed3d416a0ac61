"""Auxiliary subsystems: profiling modes / NaN panics / tracing, workspaces + SCOPE_PANIC,
failure detection (watchdog, NaN guard, fault injection, restart from checkpoint).

Reference tests mirrored: CORET:BaseDL4JTest.java:11-16 (profiling modes on in every test),
CORET:nn/misc/WorkspaceTests.java:36-41 (scope panics), PWT/EarlyStopping invalid-score termination."""
import json
import os
import time

import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd import profiling
from deeplearning4j_amd.memory import (LearningPolicy, ND4JWorkspaceException, ResetPolicy, SpillPolicy,
                                       WorkspaceConfiguration, check_scope, getWorkspaceManager, leverageTo)
from deeplearning4j_amd.optimize import CheckpointListener
from deeplearning4j_amd.parallel.watchdog import (FaultInjectionListener, InjectedFault, InvalidScoreException,
                                                  NaNGuardListener, StepWatchdog, fit_with_recovery)
from deeplearning4j_amd.utils.nd4j_io import Nd4j


def _net(seed=42):
    conf = (NeuralNetConfiguration.Builder().seed(seed).updater(Sgd(0.1)).list()
            .layer(0, DenseLayer.Builder().nIn(4).nOut(8).activation(Activation.TANH).build())
            .layer(1, OutputLayer.Builder(LossFunction.MCXENT).nIn(8).nOut(3).activation(Activation.SOFTMAX)
                   .build()).build())
    net = MultiLayerNetwork(conf)
    net.init(device="cpu")
    return net


def _xy(n=16):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(n, 4, generator=g)
    y = torch.zeros(n, 3)
    y[torch.arange(n), torch.randint(0, 3, (n,), generator=g)] = 1
    return x, y


@pytest.fixture(autouse=True)
def _reset_mode():
    yield
    ex = Nd4j.getExecutioner()
    ex.setProfilingMode("DISABLED")
    ex.tracing = False
    profiling._refresh_active()


# ------------------------------------------------------------------------------------------------ profiling
def test_profiling_mode_any_panic_names_layer():
    net = _net()
    x, y = _xy()
    Nd4j.getExecutioner().setProfilingMode(profiling.ProfilingMode.ANY_PANIC)
    net.fit(x, y)                                   # finite: no panic
    x_bad = x.clone()
    x_bad[3, 1] = float("nan")
    with pytest.raises(profiling.ND4JOpProfilerException, match="NaN.*layer 0"):
        net.fit(x_bad, y)


def test_inf_panic_only_counts_inf():
    Nd4j.getExecutioner().setProfilingMode("INF_PANIC")
    t = torch.tensor([1.0, float("nan")])
    Nd4j.getExecutioner().check("t", [t])          # NaN is not an INF_PANIC
    with pytest.raises(profiling.ND4JOpProfilerException, match="Inf"):
        Nd4j.getExecutioner().check("t", [torch.tensor([float("-inf")])])


def test_nonfinite_counts_torch_path():
    t = torch.tensor([0.0, float("nan"), float("inf"), -float("inf"), 2.0])
    assert profiling.nonfinite_counts([t, None]) == [(1, 2), (0, 0)]


def test_disabled_mode_hooks_off():
    assert not profiling.ACTIVE


def test_layer_timing_listener_and_chrome_trace(tmp_path):
    net = _net()
    x, y = _xy()
    lt = profiling.LayerTimingListener(frequency=1)
    net.setListeners(lt)
    for _ in range(3):
        net.fit(x, y)
    lt.close()
    st = lt.stats()
    cats = {k[0] for k in st}
    assert {"fwd", "bwd", "update"} <= cats
    p = lt.exportChromeTrace(str(tmp_path / "trace.json"))
    ev = json.load(open(p))["traceEvents"]
    assert len(ev) >= 3 * 5 and all(e["ph"] == "X" and e["dur"] >= 0 for e in ev)
    assert "0:" in lt.summary()


def test_roctx_range_is_safe_without_profiler():
    ex = Nd4j.getExecutioner()
    ex.enableRoctx(True)
    try:
        with profiling.range_("region"):
            pass
        net = _net()
        net.fit(*_xy())
    finally:
        ex.enableRoctx(False)


# ------------------------------------------------------------------------------------------------ workspaces
def test_workspace_learning_and_reuse():
    mgr = getWorkspaceManager()
    conf = WorkspaceConfiguration.builder().initialSize(0).policyLearning(LearningPolicy.FIRST_LOOP) \
        .overallocationLimit(0.5).build()
    ws = mgr.getWorkspaceForCurrentThread(conf, "WS_TEST_LEARN", "cpu")
    with ws:                                        # first cycle: nothing allocated yet, everything spills
        a = ws.create((100, 10))
        b = ws.create((50,), torch.float64)
        assert a.shape == (100, 10) and b.dtype == torch.float64
    st = ws.stats()
    assert st["capacity"] >= int((4000 + 512) * 1.5) - 512 and st["learned"] == 1
    with ws:                                        # second cycle: carved from the learned buffer
        a2 = ws.create((100, 10))
        assert ws.external_bytes == 0
        a2.fill_(3.0)
        assert float(a2.sum()) == 3000.0
    mgr.destroyAllWorkspacesForCurrentThread()


def test_scope_panic_on_leaked_array():
    mgr = getWorkspaceManager()
    conf = WorkspaceConfiguration(initialSize=1 << 16)
    ws = mgr.getWorkspaceForCurrentThread(conf, "WS_TEST_SCOPE", "cpu")
    with ws:
        a = ws.create((16,))
        check_scope(a)                              # fine while the cycle is open
        kept = leverageTo(a, "NOT_OPEN")            # leverage to a closed workspace = detached copy
    with pytest.raises(ND4JWorkspaceException, match="leaked workspace pointer"):
        check_scope(a)
    check_scope(kept)                               # detached copies are never scope-checked
    mgr.destroyAllWorkspacesForCurrentThread()


def test_workspace_spill_fail_policy_and_cyclic_reset():
    mgr = getWorkspaceManager()
    ws = mgr.getWorkspaceForCurrentThread(
        WorkspaceConfiguration(initialSize=4096, policySpill=SpillPolicy.FAIL, policyLearning=LearningPolicy.NONE),
        "WS_TEST_FAIL", "cpu")
    with ws:
        ws.create((512,))
        with pytest.raises(ND4JWorkspaceException, match="policySpill=FAIL"):
            ws.create((4096,))
    cyc = mgr.getWorkspaceForCurrentThread(
        WorkspaceConfiguration(initialSize=1024, policyReset=ResetPolicy.ENDOFBUFFER_REACHED,
                               policyLearning=LearningPolicy.NONE), "WS_TEST_CYC", "cpu")
    with cyc:
        g0 = cyc.getGeneration()
        first = cyc.create((128,))                  # 512 B
        cyc.create((128,))
        cyc.create((128,))                          # wraps: new generation, `first` is now invalid
        assert cyc.getGeneration() == g0 + 1
        with pytest.raises(ND4JWorkspaceException):
            check_scope(first)
    mgr.destroyAllWorkspacesForCurrentThread()


def test_scope_panic_mode_checks_layer_outputs():
    Nd4j.getExecutioner().setProfilingMode("SCOPE_PANIC")
    net = _net()
    net.fit(*_xy())                                 # ordinary (non-workspace) activations pass


# ------------------------------------------------------------------------------------------------ failures
def test_nan_guard_and_fault_injection():
    net = _net()
    x, y = _xy()
    net.setListeners(FaultInjectionListener(atIteration=2))
    net.fit(x, y)
    with pytest.raises(InjectedFault):
        net.fit(x, y)
    net2 = _net()
    net2.setListeners(NaNGuardListener())
    x_bad = x.clone()
    x_bad[0, 0] = float("nan")
    with pytest.raises(InvalidScoreException):
        net2.fit(x_bad, y)


def test_watchdog_raise_mode():
    wd = StepWatchdog(timeout_s=0.2, action="raise", poll_s=0.05)
    try:
        wd.heartbeat()
        time.sleep(0.5)
        assert wd.fired()
        with pytest.raises(TimeoutError):
            wd.heartbeat()
    finally:
        wd.close()


def test_watchdog_callback_not_fired_with_heartbeats():
    hits = []
    wd = StepWatchdog(timeout_s=0.5, action=lambda w: hits.append(1), poll_s=0.05)
    try:
        for _ in range(6):
            wd.heartbeat()
            time.sleep(0.05)
        assert not hits
    finally:
        wd.close()


def test_fit_with_recovery_restores_last_checkpoint(tmp_path):
    net = _net()
    x, y = _xy()
    ckpt = CheckpointListener.Builder(str(tmp_path)).saveEveryNIterations(2).keepLast(3).build()
    fault = FaultInjectionListener(atIteration=5)
    net.setListeners(ckpt, fault)
    seen = []

    def train(m):
        seen.append(m.getIterationCount())
        while m.getIterationCount() < 8:
            m.fit(x, y)

    model, restarts = fit_with_recovery(net, train, ckpt, maxRestarts=2)
    assert restarts == 1
    assert seen[0] == 0 and seen[1] == 4            # resumed from the iteration-4 checkpoint
    assert model.getIterationCount() == 8
    assert os.path.exists(tmp_path / "checkpointInfo.txt")
