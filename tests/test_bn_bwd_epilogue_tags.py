"""Host-side contract of the BN-backward epilogue tags (ops/native.py): which BN outputs request the sums, and when a
dX's planes are accepted by the BN backward. Pure Python on CPU tensors; the kernels are covered by
tests/test_gpu_bn_bwd_epilogue.py."""
import torch

from deeplearning4j_amd.ops import native


def _req(monkeypatch, mode, res, mask, training=True, dt=1):
    monkeypatch.setattr(native, "BNB_MODE", mode)
    monkeypatch.setattr(native, "BNB", mode > 0)
    y = torch.zeros(4, 8)
    xr = torch.zeros(4, 8)
    ctx = torch.zeros(32)
    native._bnb_request(y, xr, ctx, True, res, mask, training, dt)
    return getattr(y, "_bn_bwd_req", None)


def test_request_gating(monkeypatch):
    r = torch.zeros(4, 8)
    m = torch.zeros(4, dtype=torch.uint8)
    assert _req(monkeypatch, 0, None, None) is None                 # off by default
    assert _req(monkeypatch, 1, None, None) is not None             # plain BN layer
    assert _req(monkeypatch, 1, r, m) is None                       # residual layers only in mode 2
    req = _req(monkeypatch, 2, r, m)
    assert req is not None and req[3] is m and req[2] is True
    assert _req(monkeypatch, 2, r, None) is None                    # a residual layer without its bitmask
    assert _req(monkeypatch, 1, None, None, training=False) is None
    assert _req(monkeypatch, 1, None, None, dt=0) is None           # fp32: no 16-bit epilogue


def test_planes_accepted_only_for_the_same_forward_and_unmodified_dx():
    M, C = 130, 16
    P = (M + 63) // 64
    ctx = torch.zeros(4 * C)
    dx = torch.zeros(M, C)
    planes = torch.zeros(2, P, C)
    native.bnb_tag(dx, planes, (None, ctx, True, None))
    assert native._bnb_planes(dx, ctx, None, M, C) is planes
    assert native._bnb_planes(dx, torch.zeros(4 * C), None, M, C) is None      # another layer's forward context
    assert native._bnb_planes(dx, ctx, None, M + 64, C) is None                 # partial count mismatch
    assert native._bnb_planes(dx, ctx, torch.zeros(M, C), M, C) is None         # residual without a bitmask
    assert native._bnb_planes(dx, ctx, torch.zeros(M, C), M, C, torch.zeros(1, dtype=torch.uint8)) is planes
    dx.add_(1.0)                                                                 # in-place edit after the launch
    assert native._bnb_planes(dx, ctx, None, M, C) is None
    assert native._bnb_planes(dx.clone(), ctx, None, M, C) is None              # a copy carries no tag
