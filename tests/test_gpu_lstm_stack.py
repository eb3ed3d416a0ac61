"""Pipelined two-layer LSTM stack (csrc/lstm_coop.hip lstm_fwd_stack2 / lstm_bwd_stack2): both layers of a
GravesLSTM -> GravesLSTM stack in ONE launch per direction must give the same outputs, gradients and TBPTT training
as the two single-layer launches (whose numerics tests/test_gpu_lstm.py pins to the fp64 reference). Layer 2's input
projection runs inside the recurrence with fp32 accumulation instead of a bf16-rounded GEMM output, so the
comparison is within bf16 tolerance, not bitwise."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.nn.conf import DataType
from deeplearning4j_amd.ops import fallback, rnn_native

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _net(cuda, peep=True, tbptt=None, seed=5, H=256, nIn=24, nOut=10):
    L = GravesLSTM if peep else LSTM
    lb = (NeuralNetConfiguration.Builder().seed(seed).updater(Adam(2e-3)).dataType(DataType.BFLOAT16).list()
          .layer(L.Builder().nIn(nIn).nOut(H).activation(Activation.TANH).build())
          .layer(L.Builder().nIn(H).nOut(H).activation(Activation.TANH).build())
          .layer(RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(H).nOut(nOut).activation(Activation.SOFTMAX).build()))
    if tbptt:
        lb.backpropType(BackpropType.TruncatedBPTT).tBPTTLength(tbptt)
    net = MultiLayerNetwork(lb.build())
    net.init(device=cuda)
    return net


def _data(cuda, mb=37, nIn=24, nOut=10, T=20, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(mb, nIn, T, generator=g).to(cuda)
    y = torch.zeros(mb, nOut, T)
    y[torch.arange(mb), torch.randint(0, nOut, (mb,), generator=g)] = 1
    return x, y.to(cuda)


@pytest.mark.parametrize("peep", [True, False])
def test_stack_gradients_match_separate_layers(cuda, monkeypatch, peep):
    x, y = _data(cuda)
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DL4J_AMD_LSTM_STACK", flag)
        net = _net(cuda, peep)
        assert net.layers[0]._stack_next is net.layers[1]
        before = list(rnn_native.STACK_LAUNCHES)
        fallback.reset()
        net.computeGradientAndScore(x, y)
        torch.cuda.synchronize()
        assert fallback.count() == 0, fallback.summary()
        ran = [a - b for a, b in zip(rnn_native.STACK_LAUNCHES, before)]
        assert ran == ([1, 1] if flag == "1" else [0, 0]), ran
        rnn_native.check_coop_errors()                      # no hand-off wait timed out
        res[flag] = (net.score(), net.flattenedGradients.clone(), net.output(x).float())
    assert abs(res["1"][0] - res["0"][0]) < 1e-2 * abs(res["0"][0])
    assert _rel(res["1"][2], res["0"][2]) < 2e-2
    g1, g0 = res["1"][1], res["0"][1]
    assert _rel(g1, g0) < 3e-2, _rel(g1, g0)


def test_stack_tbptt_training_matches_separate_layers(cuda, monkeypatch):
    """TBPTT (windows of 8 over 24 steps, carried h/c of both layers, truncated backward) trains like the unstacked
    network, and the carried state lands in each layer's TBPTT map."""
    x, y = _data(cuda, T=24)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DL4J_AMD_LSTM_STACK", flag)
        net = _net(cuda, tbptt=8)
        scores = []
        for _ in range(3):
            net.fit(x, y)
            scores.append(net.score())
        torch.cuda.synchronize()
        # fit clears the carried state at the end of each sequence; one more window stores it again
        net.rnnClearPreviousState()
        net.feedForwardToLayer(2, x[:, :, :8], True, None, stored_state=True, store_last_for_tbptt=True)
        states = []
        for l in net.layers[:2]:
            assert l.tBpttStateMap["prevAct"].shape == (x.shape[0], 256)
            states += [l.tBpttStateMap["prevAct"].float(), l.tBpttStateMap["prevMem"].float()]
        net.rnnClearPreviousState()
        out[flag] = (scores, net.params().clone(), states)
    s1, s0 = out["1"][0], out["0"][0]
    assert all(abs(a - b) < 2e-2 * abs(b) for a, b in zip(s1, s0)), (s1, s0)
    assert _rel(out["1"][1], out["0"][1]) < 1e-2
    for a, b in zip(out["1"][2], out["0"][2]):
        assert _rel(a, b) < 3e-2, _rel(a, b)


def test_samediff_stacked_lstm_matches_pair(cuda, monkeypatch):
    """SameDiff's lstmLayer -> lstmLayer fusion (lstmStack2) on the stacked kernels == the two single-layer ops;
    training through TrainingConfig writes the gradients into the flat buffer (sinks)."""
    from deeplearning4j_amd.samediff import SameDiff, TrainingConfig
    g = torch.Generator().manual_seed(3)
    mb, V, T, H = 32, 40, 30, 256
    bf = torch.bfloat16
    vals = {}
    nin = V
    for i in range(2):
        vals[f"W{i}"] = torch.randn(nin, 4 * H, generator=g) * nin ** -0.5
        vals[f"RW{i}"] = torch.randn(H, 4 * H + 3, generator=g) * H ** -0.5
        vals[f"b{i}"] = torch.zeros(4 * H)
        nin = H
    vals["Wo"] = torch.randn(H, V, generator=g) * H ** -0.5
    idx = torch.randint(0, V, (mb, T + 1), generator=g)
    X = torch.nn.functional.one_hot(idx[:, :-1], V).permute(0, 2, 1).to(bf).to(cuda)
    Y = torch.nn.functional.one_hot(idx[:, 1:], V).to(bf).to(cuda)
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DL4J_AMD_LSTM_STACK", flag)
        sd = SameDiff.create()
        x = sd.placeHolder("x", X)
        y = sd.placeHolder("y", Y)
        h = x
        for i in range(2):
            h = sd.rnn().lstmLayer(f"l{i}", h, sd.var(f"W{i}", vals[f"W{i}"].to(bf).to(cuda)),
                                   sd.var(f"RW{i}", vals[f"RW{i}"].to(bf).to(cuda)),
                                   sd.var(f"b{i}", vals[f"b{i}"].to(bf).to(cuda)), peephole=True)
        logits = h.permute(0, 2, 1).mmul(sd.var("Wo", vals["Wo"].to(bf).to(cuda)))
        loss = sd.loss().softmaxCrossEntropy("loss", y, logits)
        before = list(rnn_native.STACK_LAUNCHES)
        gr = sd.execBackwards(loss)
        torch.cuda.synchronize()
        rnn_native.check_coop_errors()
        ran = [a - b for a, b in zip(rnn_native.STACK_LAUNCHES, before)]
        assert ran == ([1, 1] if flag == "1" else [0, 0]), ran
        res[flag] = (float(loss.value), {k: v.float().cpu() for k, v in gr.items() if v is not None})
    assert abs(res["1"][0] - res["0"][0]) < 1e-2 * abs(res["0"][0])
    for k, v in res["0"][1].items():
        assert _rel(res["1"][1][k], v) < 3e-2, (k, _rel(res["1"][1][k], v))
