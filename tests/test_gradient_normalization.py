"""Gradient normalization / clipping modes (reference BaseMultiLayerUpdater.java:322-382,
TestGradientNormalization.java) applied inside the updater pass: the host path here; the GPU kernel path in
test_gpu_updaters_gn.py. Expected values are computed by hand from the raw gradient (tests/_gn_ref.py)."""
import pytest
import torch

import _gn_ref as R
from deeplearning4j_amd.nn.conf.enums import GradientNormalization as G

MODES = [(G.RenormalizeL2PerLayer, 1.0), (G.RenormalizeL2PerParamType, 1.0), (G.ClipElementWiseAbsoluteValue, 0.05),
         (G.ClipL2PerLayer, 0.3), (G.ClipL2PerParamType, 0.2), (G.ClipL2PerLayer, 1e6)]


@pytest.mark.parametrize("gn,thr", MODES)
def test_gradient_normalization_host_path(gn, thr):
    x, y = R.data()
    probe = R.make_net(gn, thr)
    want = R.expected_step(probe, x, y, gn, thr)
    net = R.make_net(gn, thr)
    net.fit(x, y)
    got = net.params().double().reshape(-1)
    assert torch.allclose(got, want, atol=1e-6), (got - want).abs().max()
    if thr < 1e6 and gn != G.ClipElementWiseAbsoluteValue:
        plain = R.make_net(G.None_, 1.0)
        plain.fit(x, y)
        assert not torch.allclose(plain.params(), net.params(), atol=1e-6)   # the mode really changed the step
