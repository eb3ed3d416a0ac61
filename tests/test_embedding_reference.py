"""EmbeddingLayer equals a DenseLayer fed one-hot vectors, after the reference's EmbeddingLayerTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/feedforward/embedding/EmbeddingLayerTest.java:59-330):
with the same parameters, an embedding of class indices and a dense layer over the matching one-hot inputs give the
same activations, score and gradients -- feed-forward, inside an LSTM stack over time series (through
RnnToFeedForward / FeedForwardToRnn preprocessors), and with random per-step input masks. fp64, CPU."""
import random

import pytest
import torch

import deeplearning4j_amd as D


def _mln(first, rest, pre=False, sgd=False):
    b = D.NeuralNetConfiguration.Builder().activation(D.Activation.TANH).seed(12345).dataType(D.DataType.DOUBLE)
    if sgd:
        b = b.updater(D.Sgd(0.1))
    lb = b.list().layer(0, first)
    for i, l in enumerate(rest):
        lb = lb.layer(i + 1, l)
    if pre:
        lb = lb.inputPreProcessor(0, D.RnnToFeedForwardPreProcessor()) \
            .inputPreProcessor(len(rest) - 1, D.FeedForwardToRnnPreProcessor())
    net = D.MultiLayerNetwork(lb.build())
    net.init()
    return net


def _emb(n_in, n_out):
    return D.EmbeddingLayer.Builder().hasBias(True).nIn(n_in).nOut(n_out).build()


def _dense(n_in, n_out):
    return D.DenseLayer.Builder().nIn(n_in).nOut(n_out).build()


def _assert_same_grads(a, b, atol=1e-12):
    ga, gb = a.gradient().gradientForVariable(), b.gradient().gradientForVariable()
    assert set(ga) == set(gb)
    for k in ga:
        assert torch.allclose(ga[k], gb[k], atol=atol), k


@pytest.mark.parametrize("backward", [False, True])
def test_embedding_equals_dense_one_hot(backward):
    out = (D.OutputLayer.Builder(D.LossFunction.MCXENT).nIn(5).nOut(4).activation(D.Activation.SOFTMAX).build())
    net = _mln(_emb(10, 5), [out])
    net2 = _mln(_dense(10, 5), [D.OutputLayer.Builder(D.LossFunction.MCXENT).nIn(5).nOut(4)
                                .activation(D.Activation.SOFTMAX).build()])
    net2.setParams(net.params().clone())
    r = random.Random(12345)
    idx = torch.zeros(3, 1, dtype=torch.float64)
    oh = torch.zeros(3, 10, dtype=torch.float64)
    lab = torch.zeros(3, 4, dtype=torch.float64)
    for i in range(3):
        c = r.randrange(10)
        idx[i, 0] = c
        oh[i, c] = 1
        lab[i, r.randrange(4)] = 1
    a1, a2 = net.feedForward(idx, False), net2.feedForward(oh, False)
    for i in (1, 2):
        assert torch.allclose(a1[i], a2[i], atol=1e-12), i
    if backward:
        net.setInput(idx)
        net2.setInput(oh)
        net.setLabels(lab)
        net2.setLabels(lab)
        net.computeGradientAndScore()
        net2.computeGradientAndScore()
        assert abs(net.score() - net2.score()) < 1e-6
        _assert_same_grads(net, net2)


def _rnn_tail(n_in, n_hidden, act, loss=D.LossFunction.MCXENT, out_act=D.Activation.SOFTMAX):
    return [D.GravesLSTM.Builder().nIn(n_in).nOut(n_hidden).activation(act).build(),
            D.RnnOutputLayer.Builder(loss).nIn(n_hidden).nOut(4).activation(out_act).build()]


def _series(mb, T, n_classes, r):
    idx = torch.zeros(mb, 1, T, dtype=torch.float64)
    oh = torch.zeros(mb, n_classes, T, dtype=torch.float64)
    lab = torch.zeros(mb, 4, T, dtype=torch.float64)
    for i in range(mb):
        for t in range(T):
            c = r.randrange(n_classes)
            idx[i, 0, t] = c
            oh[i, c, t] = 1
            lab[i, r.randrange(4), t] = 1
    return idx, oh, lab


def test_embedding_in_rnn_equals_dense_one_hot():
    net = _mln(_emb(10, 5), _rnn_tail(5, 7, D.Activation.SOFTSIGN), pre=True)
    net2 = _mln(_dense(10, 5), _rnn_tail(5, 7, D.Activation.SOFTSIGN), pre=True)
    net2.setParams(net.params().clone())
    idx, oh, lab = _series(3, 8, 10, random.Random(12345))
    net.setInput(idx)
    net2.setInput(oh)
    net.setLabels(lab)
    net2.setLabels(lab)
    net.computeGradientAndScore()
    net2.computeGradientAndScore()
    assert abs(net.score() - net2.score()) < 1e-6
    _assert_same_grads(net, net2)


@pytest.mark.parametrize("mb", [1, 2, 5])
def test_embedding_with_masking_equals_dense_one_hot(mb):
    def tail():
        return [D.DenseLayer.Builder().activation(D.Activation.TANH).nIn(5).nOut(4).build(),
                D.GravesLSTM.Builder().activation(D.Activation.TANH).nIn(4).nOut(3).build(),
                D.RnnOutputLayer.Builder().lossFunction(D.LossFunction.MSE).nIn(3).nOut(4).build()]
    net = _mln(D.EmbeddingLayer.Builder().hasBias(True).activation(D.Activation.TANH).nIn(10).nOut(5).build(),
               tail(), sgd=True)
    net2 = _mln(D.DenseLayer.Builder().activation(D.Activation.TANH).nIn(10).nOut(5).build(), tail(), sgd=True)
    for n in (net, net2):          # RnnToFeedForward in front of layer 0, FeedForwardToRnn in front of the LSTM
        n.conf.inputPreProcessors[0] = D.RnnToFeedForwardPreProcessor()
        n.conf.inputPreProcessors[2] = D.FeedForwardToRnnPreProcessor()
    net2.setParams(net.params().clone())
    r = random.Random(12345)
    idx, oh, lab = _series(mb, 5, 10, r)
    mask = torch.tensor([[1.0 if r.random() < 0.5 else 0.0 for _ in range(5)] for _ in range(mb)],
                        dtype=torch.float64)
    net.setLayerMaskArrays(mask, None)
    net2.setLayerMaskArrays(mask, None)
    a1 = net.feedForward(idx, False)
    a2 = net2.feedForward(oh, False)
    for i in range(1, len(a1)):
        assert torch.allclose(a1[i], a2[i], atol=1e-12), i
    net.setInput(idx)
    net2.setInput(oh)
    net.setLabels(lab)
    net2.setLabels(lab)
    net.computeGradientAndScore()
    net2.computeGradientAndScore()
    assert abs(net.score() - net2.score()) < 1e-5
    _assert_same_grads(net, net2)
