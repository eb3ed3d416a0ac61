"""HIP-graph capture of recurrent training (nn/hipgraph.py) on MI355X:

* truncated-BPTT windows (reference MultiLayerNetwork.doTruncatedBPTT, :1521-1593): one graph per window shape, the
  h/c state chained through static buffers; graph training == eager training (deterministic fp32 kernels);
* masked variable-length batches captured with static mask buffers;
* the cooperative-LSTM buffers a graph captured stay valid when inference at a LARGER batch runs between replays
  (round-2 ADVICE: capture -> output(bigger batch) -> replay must still equal eager).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _char_data(bs, T, V, seed):
    g = torch.Generator().manual_seed(seed)
    idx = torch.randint(0, V, (bs, T), generator=g)
    x = torch.nn.functional.one_hot(idx, V).permute(0, 2, 1).float()
    y = torch.nn.functional.one_hot(torch.roll(idx, -1, 1), V).permute(0, 2, 1).float()
    return x.cuda(), y.cuda()


def _textgen(hidden, tbptt, dtype=None):
    from deeplearning4j_amd.models import TextGenerationLSTM
    kw = {} if dtype is None else {"dataType": dtype}
    return TextGenerationLSTM(numLabels=24, inputShape=[1, 24], seed=3, hidden=hidden, tbptt=tbptt,
                              **kw).init(device=torch.device("cuda", 0))


@pytest.mark.parametrize("hidden,T,tbptt", [(64, 35, 10), (256, 40, 16)])
def test_tbptt_windows_replayed_as_graphs_match_eager(hidden, T, tbptt):
    eager = _textgen(hidden, tbptt)
    graph = _textgen(hidden, tbptt)
    graph.setParams(eager.params().clone())
    graph.enableHipGraphs(True, warmup=1)
    for i in range(4):
        x, y = _char_data(8, T, 24, i)
        eager.fit(x, y)
        graph.fit(x, y)
    torch.cuda.synchronize()
    caps = [k for k, cs in graph._hipgraphs.items() if cs.ok]
    assert len(caps) >= 2, "TBPTT windows were not captured"            # first window, carried-state windows, tail
    assert any(cs.state for cs in graph._hipgraphs.values()), "no graph carries the recurrent state"
    assert graph.getIterationCount() == eager.getIterationCount()
    err = (graph.params() - eager.params()).abs().max().item()
    assert err <= 1e-5, err
    assert abs(graph.score() - eager.score()) < 1e-4


def test_masked_variable_length_batch_in_graph():
    from deeplearning4j_amd import LossFunction, MultiLayerNetwork, NeuralNetConfiguration, Adam
    from deeplearning4j_amd.nn.conf.layers import LSTM, RnnOutputLayer

    def make():
        conf = (NeuralNetConfiguration.Builder().seed(4).updater(Adam(0.01)).list()
                .layer(0, LSTM.Builder().nIn(6).nOut(32).build())
                .layer(1, RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(32).nOut(5).build()).build())
        n = MultiLayerNetwork(conf)
        n.init(device=torch.device("cuda", 0))
        return n
    eager, graph = make(), make()
    graph.setParams(eager.params().clone())
    graph.enableHipGraphs(True, warmup=1)
    g = torch.Generator().manual_seed(1)
    for i in range(4):
        x = torch.randn(6, 6, 12, generator=g).cuda()
        y = torch.zeros(6, 5, 12)
        y[:, 0] = 1
        y = y.cuda()
        lens = torch.randint(4, 13, (6,), generator=g)
        m = (torch.arange(12)[None, :] < lens[:, None]).float().cuda()
        eager.fit(x, y, featuresMask=m, labelsMask=m)
        graph.fit(x, y, featuresMask=m, labelsMask=m)
    torch.cuda.synchronize()
    assert graph._hipgraph is not None and graph._hipgraph.ok and graph._hipgraph.static_fm
    err = (graph.params() - eager.params()).abs().max().item()
    assert err <= 1e-5, err


def test_graph_replay_after_larger_batch_inference():
    """H=256 runs the cooperative LSTM kernels (LDS-resident weight slices, exchange buffers sized by the batch)."""
    eager = _textgen(256, 20)
    graph = _textgen(256, 20)
    graph.setParams(eager.params().clone())
    graph.enableHipGraphs(True, warmup=1)
    for i in range(3):
        x, y = _char_data(8, 20, 24, 10 + i)
        eager.fit(x, y)
        graph.fit(x, y)
    assert graph._hipgraph is not None and graph._hipgraph.ok
    big, _ = _char_data(64, 30, 24, 99)
    oe = eager.output(big)
    og = graph.output(big)                          # larger batch, eager, between graph replays
    assert (oe - og).abs().max().item() <= 1e-5
    for i in range(3):
        x, y = _char_data(8, 20, 24, 20 + i)
        eager.fit(x, y)
        graph.fit(x, y)
    torch.cuda.synchronize()
    err = (graph.params() - eager.params()).abs().max().item()
    assert err <= 1e-5, err
