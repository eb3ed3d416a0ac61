"""GPU side of the aux subsystems: the native NaN/Inf panic-count kernel (csrc/checks.hip) vs torch, panic mode on a
GPU network, and device workspaces (arena views in HBM)."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd import profiling
from deeplearning4j_amd.memory import LearningPolicy, WorkspaceConfiguration, getWorkspaceManager
from deeplearning4j_amd.utils.nd4j_io import Nd4j

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1, 7, 4096, 1_000_003])
def test_nonfinite_kernel_matches_torch(cuda, dtype, n):
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g)
    k = max(1, n // 97)
    idx = torch.randperm(n, generator=g)[: 2 * k]
    x[idx[:k]] = float("nan")
    x[idx[k:2 * k:2]] = float("inf")
    x[idx[k + 1:2 * k:2]] = -float("inf")
    xd = x.to(dtype).to(cuda)
    sub = xd[1:] if n > 1 else xd                   # unaligned start exercises the scalar tail path
    got = profiling.nonfinite_counts([xd, sub])
    for t, (nan, inf) in zip([xd, sub], got):
        tc = t.float().cpu()
        assert nan == int(torch.isnan(tc).sum()) and inf == int(torch.isinf(tc).sum())


def test_nan_panic_on_gpu_network(cuda):
    conf = (NeuralNetConfiguration.Builder().seed(1).updater(Sgd(0.1)).list()
            .layer(0, DenseLayer.Builder().nIn(8).nOut(16).activation(Activation.RELU).build())
            .layer(1, OutputLayer.Builder(LossFunction.MCXENT).nIn(16).nOut(4).activation(Activation.SOFTMAX)
                   .build()).build())
    net = MultiLayerNetwork(conf)
    net.init(device=cuda)
    x = torch.randn(32, 8, device=cuda)
    y = torch.nn.functional.one_hot(torch.randint(0, 4, (32,), device=cuda), 4).float()
    ex = Nd4j.getExecutioner()
    try:
        ex.setProfilingMode("NAN_PANIC")
        net.fit(x, y)
        x[5, 2] = float("nan")
        with pytest.raises(profiling.ND4JOpProfilerException, match="layer 0"):
            net.fit(x, y)
    finally:
        ex.setProfilingMode("DISABLED")


def test_device_workspace_arena(cuda):
    mgr = getWorkspaceManager()
    ws = mgr.getWorkspaceForCurrentThread(WorkspaceConfiguration(policyLearning=LearningPolicy.FIRST_LOOP),
                                          "WS_GPU_TEST", cuda)
    for cycle in range(3):
        with ws:
            a = ws.create((1024, 256), torch.bfloat16)
            b = ws.create((4096,), torch.float32, zero=True)
            assert a.is_cuda and b.is_cuda and float(b.sum()) == 0.0
            a.fill_(1.0)
            assert float(a.float().sum()) == 1024 * 256
            if cycle > 0:
                assert ws.external_bytes == 0           # learned after the first cycle
    assert ws.stats()["capacity"] >= 1024 * 256 * 2 + 4096 * 4
    mgr.destroyAllWorkspacesForCurrentThread()


def test_indarray_lives_on_device_and_matches_cpu(cuda):
    from deeplearning4j_amd.nd4j import Nd4j as N, Transforms
    a = N.rand(64, 96, seed=1)
    b = N.rand(96, 32, seed=2)
    assert a.toTensor().is_cuda and N.getAffinityManager().getDeviceForArray(a) == 0
    c = a.mmul(b)
    ref = a.toTensor().cpu().double() @ b.toTensor().cpu().double()
    assert torch.allclose(c.toTensor().cpu().double(), ref, rtol=1e-2, atol=1e-2)
    s = Transforms.softmax(c)
    assert abs(s.sum(1).toTensor().cpu() - 1).max() < 1e-5
    f = a.dup("f")
    assert f.ordering() == "f" and f.toTensor().is_cuda and f.equals(a)
