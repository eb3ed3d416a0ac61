"""The device-wide step guard of the cooperative LSTM kernels (csrc/lstm_coop.hip): a timed-out
cross-workgroup hand-off sets the guard, the fused updater (csrc/updater.hip) then leaves parameters and updater
state untouched, and the host raises CoopTimeoutError at its next per-step check (ops/rnn_native.check_step_guard)
and clears the guard. A real timeout cannot be provoked on demand, so the test raises the guard word itself."""
import ctypes

import pytest
import torch

import _dist_workers as W

pytestmark = pytest.mark.gpu


def _set_guard(v):
    from deeplearning4j_amd.ops import native
    lib = native.load()
    native.register_sig("dl4j_lstm_step_guard", [])
    lib.dl4j_lstm_step_guard.restype = ctypes.c_void_p
    ptr = lib.dl4j_lstm_step_guard()
    assert ptr
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    buf = (ctypes.c_uint * 1)(v)
    torch.cuda.synchronize()
    assert hip.hipMemcpy(ctypes.c_void_p(ptr), ctypes.cast(buf, ctypes.c_void_p), 4, 1) == 0   # host -> device


def test_step_guard_skips_update_and_raises():
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.ops import rnn_native
    rnn_native.USED_COOP[0] = True
    proto = W.make_net(Adam(0.01))
    net = type(proto)(proto.conf)
    net.init(proto.params().clone(), device=torch.device("cuda", 0))
    b = W.make_batches(4, 8)
    net.fit(b[0])
    torch.cuda.synchronize()
    _set_guard(1)
    p0 = net.params().detach().clone()
    s0 = net.updater.getStateViewArray().detach().clone()
    net.fit(b[1])                                   # update skipped on the device
    torch.cuda.synchronize()
    assert torch.equal(net.params(), p0)
    assert torch.equal(net.updater.getStateViewArray(), s0)
    with pytest.raises(rnn_native.CoopTimeoutError):
        net.fit(b[2])                               # the host sees the guard and clears it
    torch.cuda.synchronize()
    net.fit(b[3])
    torch.cuda.synchronize()
    assert not torch.equal(net.params(), p0)


def test_step_guard_reported_without_host_sync():
    """with the host running ahead of the GPU (no synchronize between steps) the trip must still be
    reported within the snapshot FIFO's depth, not lost because only the newest snapshot was looked at."""
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.ops import rnn_native
    rnn_native.USED_COOP[0] = True
    rnn_native._guard.clear()
    proto = W.make_net(Adam(0.01))
    net = type(proto)(proto.conf)
    net.init(proto.params().clone(), device=torch.device("cuda", 0))
    b = W.make_batches(2, 8)
    net.fit(b[0])
    _set_guard(1)
    raised = False
    for i in range(rnn_native._GUARD_DEPTH + 3):
        try:
            net.fit(b[i % 2])                        # no torch.cuda.synchronize() between steps
        except rnn_native.CoopTimeoutError:
            raised = True
            break
    assert raised, "guard trip never reported"
    torch.cuda.synchronize()
    p0 = net.params().detach().clone()
    net.fit(b[0])
    torch.cuda.synchronize()
    assert not torch.equal(net.params(), p0)         # cleared: updates apply again
