"""dl4j_segment_stats (csrc/stats.hip) vs torch fp32 reductions, and the StatsListener on a GPU network."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_segment_stats_matches_torch(cuda, dtype):
    from deeplearning4j_amd.ops import native
    g = torch.Generator().manual_seed(0)
    sizes = [1, 7, 64, 1000, 250_003, 3]
    flat = (torch.randn(sum(sizes), generator=g) * 3 + 1).to(dtype).to(cuda)
    offs = [0]
    for s in sizes:
        offs.append(offs[-1] + s)
    stats, hist = native.segment_stats(flat, offs, 16)
    ref = flat.float().cpu()
    for i, (a, b) in enumerate(zip(offs[:-1], offs[1:])):
        x = ref[a:b]
        exp = torch.tensor([x.mean(), x.std(unbiased=False), x.abs().mean(), x.min(), x.max()])
        torch.testing.assert_close(stats[i].cpu(), exp, rtol=2e-4, atol=2e-4)
        assert int(hist[i].sum()) == b - a
        if x.max() > x.min():
            th = torch.histc(x, 16, float(x.min()), float(x.max()))
            assert (hist[i].cpu().float() - th).abs().max() <= 2      # edge-bin rounding only


def test_stats_listener_on_gpu(cuda):
    from deeplearning4j_amd.nn.conf import layers as L
    from deeplearning4j_amd.nn.conf.network import NeuralNetConfiguration
    from deeplearning4j_amd.nn.multilayer import MultiLayerNetwork
    from deeplearning4j_amd.ui import InMemoryStatsStorage, StatsListener
    conf = NeuralNetConfiguration.Builder().seed(1).list() \
        .layer(0, L.DenseLayer(nIn=4, nOut=8, activation="tanh")) \
        .layer(1, L.OutputLayer(nIn=8, nOut=3, activation="softmax", lossFn="MCXENT")).build()
    net = MultiLayerNetwork(conf)
    net.init(device=cuda)
    st = InMemoryStatsStorage()
    net.setListeners(StatsListener(st, 1))
    x = torch.randn(16, 4, device=cuda)
    y = torch.eye(3, device=cuda)[torch.randint(0, 3, (16,), device=cuda)]
    for _ in range(3):
        net.fit(x, y)
    sid = st.listSessionIDs()[0]
    w = st.listWorkerIDsForSession(sid)[0]
    d = st.getLatestUpdate(sid, "StatsListener", w).data
    w0 = net.getParam("0_W").float()
    assert abs(d["Parameters"]["0_W"]["meanMagnitude"] - float(w0.abs().mean())) < 1e-5
    assert d["memory"]["deviceMaxBytes"][0] > 0


@pytest.mark.parametrize("C", [8, 64, 256, 24])
def test_channel_sum_matches_torch(cuda, C):
    from deeplearning4j_amd.ops import native
    g = torch.Generator().manual_seed(C)
    x = torch.randn(100_003, C, generator=g).to(torch.bfloat16).to(cuda)
    got = native.channel_sum(x)
    torch.testing.assert_close(got.cpu(), x.float().sum(0).cpu(), rtol=1e-4, atol=1e-2)
