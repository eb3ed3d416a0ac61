"""SelfAttentionLayer on the in-tree kernels (GEMM + flash attention fwd/bwd) with its hand-derived backward:
no fallback is counted, and every gradient matches the same network's fp32 explicit reference computed on the CPU
(same parameters and batch)."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403

pytestmark = pytest.mark.gpu


def _net(dt, device, causal):
    b = (NeuralNetConfiguration.Builder().seed(11).dataType(dt).updater(NoOp())
         .weightInit(NormalDistribution(0, 0.05)).list())
    b.layer(0, SelfAttentionLayer.Builder().nIn(128).nOut(128).nHeads(2).causal(causal)
            .activation(Activation.IDENTITY).build())
    b.layer(1, RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(128).nOut(5).activation(Activation.SOFTMAX).build())
    net = MultiLayerNetwork(b.build())
    net.init(device=device)
    return net


@pytest.mark.parametrize("causal,masked", [(False, False), (True, False), (False, True)])
def test_self_attention_native_matches_fp32_reference(causal, masked):
    from deeplearning4j_amd.ops import fallback
    gpu = _net(DataType.BFLOAT16, torch.device("cuda", 0), causal)
    cpu = _net(DataType.FLOAT, torch.device("cpu"), causal)
    with torch.no_grad():
        cpu.flattenedParams.copy_(gpu.flattenedParams.cpu())
    cpu._params_changed()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 128, 64, generator=g)
    y = torch.zeros(4, 5, 64)
    y[:, 2] = 1
    mask = None
    if masked:
        mask = torch.ones(4, 64)
        mask[1, 40:] = 0
        mask[3, 10:] = 0
    fallback.reset()
    gpu.computeGradientAndScore(x.cuda().to(torch.bfloat16), y.cuda(), None if mask is None else mask.cuda(),
                                None if mask is None else mask.cuda())
    torch.cuda.synchronize()
    assert gpu.helperCountFail() == 0, gpu.fallbackSummary()
    cpu.computeGradientAndScore(x, y, mask, mask)
    ga, gb = gpu.flattenedGradients.float().cpu(), cpu.flattenedGradients.float()
    rel = (ga - gb).norm() / gb.norm()
    assert rel < 3e-2, rel
