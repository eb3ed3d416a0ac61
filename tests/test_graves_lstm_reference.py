"""GravesLSTM layer behaviour, after the reference's GravesLSTMTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/recurrent/GravesLSTMTest.java:30-259): forward output
shapes for minibatch / length edge cases; backward gradient shapes (bias [1, 4H], input weights [nIn, 4H], recurrent
weights with the three peephole columns [H, 4H + 3]) and epsilon [mb, nIn, T]; the training-mode forward (which
keeps the per-step cache for backprop, the reference's forBackprop=true helper) equals the inference forward exactly;
a length-4 series and the same series extended to 5 steps give identical outputs on the first 4 steps; and both gate
activations (sigmoid, hardsigmoid) train. fp64, CPU."""
import pytest
import torch

import deeplearning4j_amd as D

LF = D.LossFunctions.LossFunction


def _lstm_layer(nIn, H, dist=False):
    b = D.GravesLSTM.Builder().nIn(nIn).nOut(H).activation(D.Activation.TANH)
    if dist:
        b = b.weightInit(D.WeightInit.DISTRIBUTION).dist(D.UniformDistribution(0, 1))
    conf = (D.NeuralNetConfiguration.Builder().seed(12345).dataType(D.DataType.DOUBLE).list().layer(b.build())
            .layer(D.RnnOutputLayer.Builder(LF.MSE).nIn(H).nOut(3).activation(D.Activation.IDENTITY).build())
            .build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    return net.getLayer(0)


def test_forward_basic():
    nIn, H = 13, 17
    layer = _lstm_layer(nIn, H)
    for mb, T in ((1, 1), (10, 1), (1, 12), (10, 15)):
        out = layer.activate(torch.ones(mb, nIn, T, dtype=torch.float64))
        assert tuple(out.shape) == (mb, H, T)


@pytest.mark.parametrize("mb,T", [(10, 7), (1, 7), (10, 1), (1, 1)])
def test_backward_basic(mb, T):
    nIn, H = 13, 17
    lstm = _lstm_layer(nIn, H, dist=True)
    lstm.activate(torch.ones(mb, nIn, T, dtype=torch.float64), True)
    assert lstm.input is not None
    grad, eps_in = lstm.backpropGradient(torch.ones(mb, H, T, dtype=torch.float64))
    b, w, rw = (grad.getGradientFor(k) for k in ("b", "W", "RW"))
    assert b is not None and w is not None and rw is not None
    assert tuple(b.reshape(1, -1).shape) == (1, 4 * H)
    assert tuple(w.shape) == (nIn, 4 * H)
    assert tuple(rw.shape) == (H, 4 * H + 3)
    assert tuple(eps_in.shape) == (mb, nIn, T)
    for k, g in grad.gradientForVariable().items():         # the reference's per-variable update call
        lstm.update(g, k)


def test_forward_for_backprop_equals_inference_forward():
    torch.manual_seed(12345)
    lstm = _lstm_layer(10, 15, dist=True)
    x = torch.rand(4, 10, 7, dtype=torch.float64)
    a_inf = lstm.activate(x, False).clone()
    a_train = lstm.activate(x, True)
    assert torch.equal(a_inf, a_train)


def test_single_example_prefix():
    conf = (D.NeuralNetConfiguration.Builder().optimizationAlgo(D.OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT)
            .updater(D.Sgd(0.1)).seed(12345).dataType(D.DataType.DOUBLE).list()
            .layer(0, D.GravesLSTM.Builder().activation(D.Activation.TANH).nIn(2).nOut(2).build())
            .layer(1, D.RnnOutputLayer.Builder().lossFunction(LF.MSE).nIn(2).nOut(1).activation(D.Activation.TANH)
                   .build()).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    g = torch.Generator().manual_seed(12345)
    in1 = torch.rand(1, 2, 4, generator=g, dtype=torch.float64)
    in2 = torch.rand(1, 2, 5, generator=g, dtype=torch.float64)
    in2[:, :, :4] = in1
    assert torch.equal(in1, in2[:, :, :4])
    out1, out2 = net.output(in1), net.output(in2)
    acts1, acts2 = net.feedForward(in1), net.feedForward(in2)
    assert len(acts1) == len(acts2) == 3
    for i in range(4):
        assert float(out1.reshape(-1)[i]) == float(out2.reshape(-1)[i])


@pytest.mark.parametrize("gate", ["sigmoid", "hardsigmoid"])
def test_gate_activation_fns(gate):
    conf = (D.NeuralNetConfiguration.Builder().optimizationAlgo(D.OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT)
            .seed(12345).list()
            .layer(0, D.GravesLSTM.Builder().gateActivationFunction(gate).activation(D.Activation.TANH).nIn(2).nOut(2)
                   .build())
            .layer(1, D.RnnOutputLayer.Builder().lossFunction(LF.MSE).nIn(2).nOut(2).activation(D.Activation.TANH)
                   .build()).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    assert str(net.getLayer(0).conf().getLayer().getGateActivationFn()) == gate
    g = torch.Generator().manual_seed(3)
    net.fit(torch.rand(3, 2, 5, generator=g), torch.rand(3, 2, 5, generator=g))
    assert torch.isfinite(torch.tensor(net.score()))
