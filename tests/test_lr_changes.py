"""Changing learning rates of a live network (reference nn/misc/TestLrChanges.java testChangeLrMLN): setting layer 0's
LR (and then every layer's LR) on a trained network gives exactly the same training as a network configured with
those LRs from the start, once parameters, updater state and iteration count are copied over."""
import torch

from deeplearning4j_amd import *  # noqa: F401,F403


def _conf(lr0, lr1):
    return (NeuralNetConfiguration.Builder().activation(Activation.TANH).seed(12345).dataType(DataType.DOUBLE).list()
            .layer(DenseLayer.Builder().nIn(10).nOut(10).updater(Adam(lr0)).build())
            .layer(DenseLayer.Builder().nIn(10).nOut(10).updater(RmsProp(lr1)).build())
            .layer(OutputLayer.Builder().nIn(10).nOut(10).updater(NoOp()).lossFunction(LossFunction.MSE).build())
            .build())


def _net(conf):
    n = MultiLayerNetwork(conf)
    n.init(device="cpu")
    return n


def _rand(g):
    return torch.rand(10, 10, generator=g, dtype=torch.float64)


def _sync(dst, src):
    dst.getUpdater().getStateViewArray().copy_(src.getUpdater().getStateViewArray())
    dst.conf.setIterationCount(src.conf.getIterationCount())
    dst.setParams(src.params().clone())


def test_change_lr_mln():
    g = torch.Generator().manual_seed(12345)
    net = _net(_conf(0.1, 0.01))
    for _ in range(10):
        net.fit(_rand(g), _rand(g))

    net2 = _net(_conf(0.5, 0.01))
    _sync(net2, net)
    net.setLearningRate(0, 0.5)                 # layer 0 only
    assert net.conf.toJson() == net2.conf.toJson()
    torch.testing.assert_close(net.getUpdater().getStateViewArray(), net2.getUpdater().getStateViewArray())
    for _ in range(3):
        x, y = _rand(g), _rand(g)
        net.fit(x, y)
        net2.fit(x, y)
    torch.testing.assert_close(net.params(), net2.params(), rtol=0, atol=1e-12)
    torch.testing.assert_close(net.getUpdater().getStateViewArray(), net2.getUpdater().getStateViewArray(),
                               rtol=0, atol=1e-12)
    x, y = _rand(g), _rand(g)
    net.setInput(x)
    net.setLabels(y)
    net.computeGradientAndScore()
    net2.setInput(x)
    net2.setLabels(y)
    net2.computeGradientAndScore()
    assert abs(net.score() - net2.score()) < 1e-8

    net3 = _net(_conf(0.3, 0.3))                # every layer's LR (the NoOp output layer has none)
    _sync(net3, net)
    net.setLearningRate(0.3)
    for _ in range(3):
        x, y = _rand(g), _rand(g)
        net.fit(x, y)
        net3.fit(x, y)
    torch.testing.assert_close(net.params(), net3.params(), rtol=0, atol=1e-12)
    torch.testing.assert_close(net.getUpdater().getStateViewArray(), net3.getUpdater().getStateViewArray(),
                               rtol=0, atol=1e-12)


def test_change_lr_computation_graph_layer():
    def conf(lr):
        return (NeuralNetConfiguration.Builder().activation(Activation.TANH).seed(12345).dataType(DataType.DOUBLE)
                .graphBuilder().addInputs("in")
                .addLayer("0", DenseLayer.Builder().nIn(10).nOut(10).updater(Adam(lr)).build(), "in")
                .addLayer("1", OutputLayer.Builder().nIn(10).nOut(10).updater(NoOp()).lossFunction(LossFunction.MSE)
                          .build(), "0")
                .setOutputs("1").build())
    g = torch.Generator().manual_seed(3)
    a = ComputationGraph(conf(0.1))
    a.init(device="cpu")
    for _ in range(3):
        a.fit([_rand(g)], [_rand(g)])
    b = ComputationGraph(conf(0.5))
    b.init(device="cpu")
    _sync(b, a)
    a.setLearningRate("0", 0.5)
    assert a.conf.toJson() == b.conf.toJson()
    for _ in range(3):
        x, y = _rand(g), _rand(g)
        a.fit([x], [y])
        b.fit([x], [y])
    torch.testing.assert_close(a.params(), b.params(), rtol=0, atol=1e-12)
