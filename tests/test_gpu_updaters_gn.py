"""Gradient normalization / clipping inside the fused HIP updater (csrc/updater.hip gn_sumsq_kernel +
fused_update_kernel) against the hand-computed reference semantics (tests/_gn_ref.py); the host pre-pass must not
run on the GPU path."""
import pytest
import torch

import _gn_ref as R
from deeplearning4j_amd.nn.conf.enums import GradientNormalization as G

pytestmark = pytest.mark.gpu

MODES = [(G.RenormalizeL2PerLayer, 1.0), (G.RenormalizeL2PerParamType, 1.0), (G.ClipElementWiseAbsoluteValue, 0.05),
         (G.ClipL2PerLayer, 0.3), (G.ClipL2PerParamType, 0.2), (G.ClipL2PerLayer, 1e6)]


@pytest.mark.parametrize("gn,thr", MODES)
def test_gradient_normalization_in_updater_kernel(gn, thr, monkeypatch):
    from deeplearning4j_amd.ops import update as U
    dev = torch.device("cuda", 0)
    x, y = R.data(dev)
    probe = R.make_net(gn, thr, dev)
    want = R.expected_step(probe, x, y, gn, thr)

    def boom(*a, **k):
        raise AssertionError("host pre_apply ran on the GPU path")
    monkeypatch.setattr(U, "pre_apply", boom)
    net = R.make_net(gn, thr, dev)
    net.fit(x, y)
    torch.cuda.synchronize()
    got = net.params().double().reshape(-1)
    assert torch.allclose(got, want, atol=2e-6), (got - want).abs().max()


def test_gradient_normalization_large_layer_many_blocks(monkeypatch):
    """A layer spanning many update blocks (2048 elements each): the per-layer norm sums every block's partial."""
    from deeplearning4j_amd import (Activation, DenseLayer, LossFunction, MultiLayerNetwork, NeuralNetConfiguration,
                                    OutputLayer, Sgd)
    dev = torch.device("cuda", 0)

    def make():
        conf = (NeuralNetConfiguration.Builder().seed(2).updater(Sgd(0.5))
                .gradientNormalization(G.RenormalizeL2PerLayer).list()
                .layer(0, DenseLayer.Builder().nIn(300).nOut(200).activation(Activation.TANH).build())
                .layer(1, OutputLayer.Builder(LossFunction.MCXENT).nIn(200).nOut(3).activation(Activation.SOFTMAX)
                       .build()).build())
        n = MultiLayerNetwork(conf)
        n.init(device=dev)
        return n
    g = torch.Generator().manual_seed(1)
    x = torch.randn(16, 300, generator=g).to(dev)
    yl = torch.zeros(16, 3)
    yl[:, 1] = 1
    yl = yl.to(dev)
    probe = make()
    want = R.expected_step(probe, x, yl, G.RenormalizeL2PerLayer, 1.0)
    net = make()
    net.fit(x, yl)
    torch.cuda.synchronize()
    got = net.params().double().reshape(-1)
    assert torch.allclose(got, want, atol=2e-6), (got - want).abs().max()
