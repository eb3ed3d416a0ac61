"""Variable-length time series through masks, after the reference's TestVariableLengthTS
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/multilayer/TestVariableLengthTS.java:37-594): a label-masked
trailing step leaves score and gradients unchanged (and its label value is irrelevant); masked MSE scores count only
unmasked steps; bidirectional LSTMs and masked global pooling give each example exactly the output (and per-example
score) of its unpadded prefix; time-series reversal with and without masks. fp64 networks, CPU."""
import pytest
import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.nn.util.time_series import reverse_time_series


def _lstm_mse(nIn, hidden, nOut, bidirectional=False, seed=12345, out_init=None, dist=False):
    lstm = D.GravesBidirectionalLSTM if bidirectional else D.GravesLSTM
    b = lstm.Builder().nIn(nIn).nOut(hidden).activation(D.Activation.TANH)
    if dist:
        b = b.weightInit(D.WeightInit.DISTRIBUTION).dist(D.NormalDistribution(0, 1))
    ob = D.RnnOutputLayer.Builder(D.LossFunction.MSE).nIn(hidden).nOut(nOut).activation(D.Activation.IDENTITY)
    if out_init is not None:
        ob = ob.weightInit(out_init)
    conf = (D.NeuralNetConfiguration.Builder().seed(seed).updater(D.Sgd(0.1)).dataType(D.DataType.DOUBLE).list()
            .layer(0, b.build()).layer(1, ob.build()).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    return net


def _grads(net):
    return {k: v.detach().clone() for k, v in net.gradient().gradientForVariable().items()}


@pytest.mark.parametrize("mb", [1, 2, 5])
def test_trailing_label_masked_step_changes_nothing(mb):
    """Length 4 vs length 5 with the fifth step's label masked: same score, same gradients; whatever label sits under
    the mask does not matter."""
    g = torch.Generator().manual_seed(12345)
    net = _lstm_mse(2, 2, 1)
    in1 = torch.rand(mb, 2, 4, generator=g, dtype=torch.float64)
    in2 = torch.rand(mb, 2, 5, generator=g, dtype=torch.float64)
    in2[:, :, :4] = in1
    lab1 = torch.rand(mb, 1, 4, generator=g, dtype=torch.float64)
    lab2 = torch.zeros(mb, 1, 5, dtype=torch.float64)
    lab2[:, :, :4] = lab1
    lmask = torch.ones(mb, 5, dtype=torch.float64)
    lmask[:, 4] = 0
    s1 = float(net.computeGradientAndScore(in1, lab1))
    g1 = _grads(net)
    s2 = float(net.computeGradientAndScore(in2, lab2, None, lmask))
    g2 = _grads(net)
    assert abs(s1 - s2) < 1e-10
    for k in g1:
        assert torch.allclose(g1[k], g2[k], atol=1e-12), k
    lab2[:, 0, 4] = torch.rand(mb, generator=g, dtype=torch.float64) * 10
    s3 = float(net.computeGradientAndScore(in2, lab2, None, lmask))
    assert abs(s2 - s3) < 1e-10
    for k, v in _grads(net).items():
        assert torch.allclose(g2[k], v, atol=1e-12), k


@pytest.mark.parametrize("ts_len", [3, 10])
@pytest.mark.parametrize("nOut", [1, 2, 5])
@pytest.mark.parametrize("mb", [1, 4])
def test_masked_mse_score_counts_unmasked_steps(ts_len, nOut, mb):
    """Zero-initialised identity output layer, all-ones labels: each unmasked step contributes MSE = 1, so the
    score (summed over steps, averaged over the minibatch) equals the number of unmasked steps per example."""
    g = torch.Generator().manual_seed(12345)
    net = _lstm_mse(3, 5, nOut, out_init=D.WeightInit.ZERO, dist=True)
    for n_mask in range(ts_len - 1):
        lmask = torch.ones(mb, ts_len, dtype=torch.float64)
        for i in range(mb):
            lmask[i, torch.randperm(ts_len, generator=g)[:n_mask]] = 0
        x = torch.rand(mb, 3, ts_len, generator=g, dtype=torch.float64)
        y = torch.ones(mb, nOut, ts_len, dtype=torch.float64)
        net.setLayerMaskArrays(None, lmask)
        net.setInput(x)
        net.setLabels(y)
        s = float(net.computeGradientAndScore())
        net.clearLayerMaskArrays()
        assert abs(s - (ts_len - n_mask)) < 0.1, (n_mask, s)


def test_bidirectional_masked_examples_match_their_prefixes():
    """Masks [11111], [11110], [11100] on two stacked bidirectional LSTMs: each example's output over its unmasked
    steps equals the output of feeding only that prefix, and scoreExamples gives each example its prefix's score."""
    g = torch.Generator().manual_seed(12345)
    conf = (D.NeuralNetConfiguration.Builder().seed(12345).weightInit(D.WeightInit.XAVIER).activation(D.Activation.TANH)
            .dataType(D.DataType.DOUBLE).list()
            .layer(0, D.GravesBidirectionalLSTM.Builder().nIn(4).nOut(3).build())
            .layer(1, D.GravesBidirectionalLSTM.Builder().nIn(3).nOut(3).build())
            .layer(2, D.RnnOutputLayer.Builder(D.LossFunction.MSE).nIn(3).nOut(3).build()).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    x = torch.rand(3, 4, 5, generator=g, dtype=torch.float64)
    y = torch.rand(3, 3, 5, generator=g, dtype=torch.float64)
    fmask = torch.tensor([[1, 1, 1, 1, 1], [1, 1, 1, 1, 0], [1, 1, 1, 0, 0]], dtype=torch.float64)
    net.setLayerMaskArrays(fmask, fmask.clone())
    out = net.output(x)
    net.clearLayerMaskArrays()
    for i in range(3):
        exp = net.output(x[i:i + 1, :, :5 - i])
        assert torch.allclose(out[i:i + 1, :, :5 - i], exp, atol=1e-10), i
    scores = net.scoreExamples(D.DataSet(x, y, fmask, fmask.clone()), False).reshape(-1)
    assert scores.numel() == 3
    for i in range(3):
        single = net.scoreExamples(D.DataSet(x[i:i + 1, :, :5 - i], y[i:i + 1, :, :5 - i]), False).reshape(-1)
        assert abs(float(single[0]) - float(scores[i])) < 1e-8, i


@pytest.mark.parametrize("bidirectional", [False, True])
@pytest.mark.parametrize("pooling", ["SUM", "AVG", "MAX"])
def test_masked_global_pooling_matches_prefixes(bidirectional, pooling):
    """LSTM (or bidirectional) x2 -> masked global pooling -> dense output: each example's pooled output and
    per-example score equal those of its unmasked prefix alone."""
    g = torch.Generator().manual_seed(12345)
    lstm = D.GravesBidirectionalLSTM if bidirectional else D.GravesLSTM
    conf = (D.NeuralNetConfiguration.Builder().seed(12345).weightInit(D.WeightInit.XAVIER).activation(D.Activation.TANH)
            .dataType(D.DataType.DOUBLE).list()
            .layer(0, lstm.Builder().nIn(2).nOut(4).build())
            .layer(1, lstm.Builder().nIn(4).nOut(4).build())
            .layer(2, D.GlobalPoolingLayer.Builder().poolingType(getattr(D.PoolingType, pooling)).build())
            .layer(3, D.OutputLayer.Builder(D.LossFunction.MSE).nIn(4).nOut(3).build()).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    x = torch.rand(3, 2, 5, generator=g, dtype=torch.float64)
    y = torch.rand(3, 3, generator=g, dtype=torch.float64)
    fmask = torch.tensor([[1, 1, 1, 1, 1], [1, 1, 1, 1, 0], [1, 1, 1, 0, 0]], dtype=torch.float64)
    net.setLayerMaskArrays(fmask, None)
    out = net.output(x)
    net.clearLayerMaskArrays()
    for i in range(3):
        exp = net.output(x[i:i + 1, :, :5 - i])
        assert torch.allclose(out[i:i + 1], exp, atol=1e-10), (i, pooling)
    scores = net.scoreExamples(D.DataSet(x, y, fmask, None), False).reshape(-1)
    for i in range(3):
        single = net.scoreExamples(D.DataSet(x[i:i + 1, :, :5 - i], y[i:i + 1]), False).reshape(-1)
        assert abs(float(single[0]) - float(scores[i])) < 1e-8, (i, pooling)


def test_reverse_time_series_and_mask():
    """TimeSeriesUtils.reverseTimeSeries / reverseTimeSeriesMask: full reversal along time; with a left-aligned mask
    each example's valid prefix is reversed and the padding stays in place."""
    x = torch.arange(1, 3 * 5 * 10 + 1, dtype=torch.float64).reshape(3, 5, 10)
    assert torch.equal(reverse_time_series(x), torch.flip(x, [2]))
    m = torch.arange(1, 31, dtype=torch.float64).reshape(3, 10)
    assert torch.equal(reverse_time_series(m), torch.flip(m, [1]))
    mask = torch.tensor([[1.0] * 10, [1.0] * 7 + [0.0] * 3, [1.0] * 4 + [0.0] * 6])
    r = reverse_time_series(x, mask)
    for i, n in enumerate((10, 7, 4)):
        assert torch.equal(r[i, :, :n], torch.flip(x[i, :, :n], [1]))
        assert torch.equal(r[i, :, n:], x[i, :, n:])
