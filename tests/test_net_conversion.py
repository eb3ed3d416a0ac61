"""MultiLayerNetwork -> ComputationGraph conversion (reference nn/misc/TestNetConversion.java testMlnToCompGraph): the
converted graph carries the same parameters (fresh and after training), gives the same output, score and gradient,
and one fit step keeps both in lock-step — for a CNN and for a GravesLSTM -> LSTM -> RnnOutputLayer stack."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.nn.conf.enums import ConvolutionMode


def _fit_rand(net, fshape, lshape, g, n=3):
    for _ in range(n):
        net.fit(torch.rand(*fshape, generator=g, dtype=torch.float64), torch.rand(*lshape, generator=g,
                                                                                   dtype=torch.float64))


def _net1(train, g):
    conf = (NeuralNetConfiguration.Builder().convolutionMode(ConvolutionMode.Same).activation(Activation.TANH)
            .weightInit(WeightInit.XAVIER).updater(Sgd(0.1)).dataType(DataType.DOUBLE).seed(12345).list()
            .layer(ConvolutionLayer.Builder().nIn(3).nOut(5).kernelSize(2, 2).stride(1, 1).build())
            .layer(SubsamplingLayer.Builder().kernelSize(2, 2).stride(1, 1).build())
            .layer(DenseLayer.Builder().nOut(32).build())
            .layer(OutputLayer.Builder().nOut(10).lossFunction(LossFunction.MSE).build())
            .setInputType(InputType.convolutional(10, 10, 3)).build())
    net = MultiLayerNetwork(conf)
    net.init(device="cpu")
    if train:
        _fit_rand(net, (8, 3, 10, 10), (8, 10), g)
    return net


def _net2(g):
    conf = (NeuralNetConfiguration.Builder().activation(Activation.TANH).weightInit(WeightInit.XAVIER)
            .updater(Sgd(0.1)).dataType(DataType.DOUBLE).seed(12345).list()
            .layer(GravesLSTM.Builder().nOut(8).build())
            .layer(LSTM.Builder().nOut(8).build())
            .layer(RnnOutputLayer.Builder().nOut(10).lossFunction(LossFunction.MSE).build())
            .setInputType(InputType.recurrent(5)).build())
    net = MultiLayerNetwork(conf)
    net.init(device="cpu")
    _fit_rand(net, (8, 5, 10), (8, 10, 10), g)
    return net


@pytest.mark.parametrize("case", [0, 1, 2])
def test_mln_to_computation_graph(case):
    g = torch.Generator().manual_seed(12345)
    n = _net1(case == 1, g) if case <= 1 else _net2(g)
    fin = (8, 3, 10, 10) if case <= 1 else (8, 5, 10)
    lab = (8, 10) if case <= 1 else (8, 10, 10)
    x = torch.rand(*fin, generator=g, dtype=torch.float64)
    y = torch.rand(*lab, generator=g, dtype=torch.float64)
    cg = n.toComputationGraph()
    torch.testing.assert_close(n.output(x), cg.outputSingle(x))
    n.setInput(x)
    n.setLabels(y)
    cg.setInputs(x)
    cg.setLabels(y)
    n.computeGradientAndScore()
    cg.computeGradientAndScore()
    assert abs(n.score() - cg.score()) < 1e-6
    torch.testing.assert_close(n.gradient().gradient(), cg.gradient().gradient())
    n.fit(x, y)
    cg.fit([x], [y])
    torch.testing.assert_close(n.params(), cg.params())
