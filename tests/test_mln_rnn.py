"""MultiLayerNetwork recurrent behaviour, after the reference's MultiLayerTestRNN
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/multilayer/MultiLayerTestRNN.java:37-700): GravesLSTM
parameter shapes and positive forget-gate biases; rnnTimeStep on 3-D, 2-D and length-1 inputs; forward passes from
stored state (rnnActivateUsingStoredState) that chain slice by slice into the full-sequence forward. fp64, CPU."""
import torch

import deeplearning4j_amd as D


def _lstm(nin, nout):
    return (D.GravesLSTM.Builder().nIn(nin).nOut(nout).activation(D.Activation.TANH)
            .weightInit(D.WeightInit.DISTRIBUTION).dist(D.NormalDistribution(0, 0.5)).build())


def _net():
    conf = (D.NeuralNetConfiguration.Builder().seed(12345).dataType(D.DataType.DOUBLE).list()
            .layer(0, _lstm(5, 7)).layer(1, _lstm(7, 8))
            .layer(2, D.RnnOutputLayer.Builder(D.LossFunction.MCXENT).nIn(8).nOut(4).activation(D.Activation.SOFTMAX)
                   .weightInit(D.WeightInit.DISTRIBUTION).dist(D.NormalDistribution(0, 0.5)).build())
            .build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    return net


def test_graves_lstm_parameter_shapes_and_forget_bias():
    nIn, n, nOut = 8, 17, 25
    conf = (D.NeuralNetConfiguration.Builder().list()
            .layer(0, D.GravesLSTM.Builder().nIn(nIn).nOut(n).weightInit(D.WeightInit.DISTRIBUTION)
                   .dist(D.NormalDistribution(0, 1)).activation(D.Activation.TANH).build())
            .layer(1, D.RnnOutputLayer.Builder(D.LossFunction.MSE).nIn(n).nOut(nOut)
                   .weightInit(D.WeightInit.DISTRIBUTION).dist(D.NormalDistribution(0, 1))
                   .activation(D.Activation.TANH).build())
            .build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    t = net.getLayer(0).paramTable()
    assert len(t) == 3
    assert tuple(t["RW"].shape) == (n, 4 * n + 3)       # recurrent weights + 3 peephole columns
    assert tuple(t["W"].shape) == (nIn, 4 * n)
    assert tuple(t["b"].shape) == (1, 4 * n)
    assert int((t["b"][0, n:2 * n] > 0).sum()) == n       # forget-gate biases start positive
    assert sum(v.numel() for v in t.values()) == net.getLayer(0).numParams()


def test_rnn_time_step_2d_and_length_one_inputs():
    net = _net()
    x = torch.rand(3, 5, 6, generator=torch.Generator().manual_seed(12345), dtype=torch.float64)
    out3d = net.rnnTimeStep(x)
    assert tuple(out3d.shape) == (3, 4, 6)
    net.rnnClearPreviousState()
    for i in range(6):
        o = net.rnnTimeStep(x[:, :, i])
        assert tuple(o.shape) == (3, 4)
        assert torch.allclose(o, out3d[:, :, i], atol=1e-12), i
    net.rnnClearPreviousState()
    for i in range(6):
        o = net.rnnTimeStep(x[:, :, i:i + 1])
        assert tuple(o.shape) == (3, 4, 1)
        assert torch.allclose(o[:, :, 0], out3d[:, :, i], atol=1e-12), i


def test_rnn_activate_using_stored_state_chains_slices():
    """From zero state the stored-state forward equals feedForward and is repeatable; slice by slice, with the TBPTT
    state of each slice handed over as the next slice's previous state, the activations are the full sequence's."""
    T, mb, slices = 12, 7, 5
    net = _net()
    xl = torch.rand(mb, 5, slices * T, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    x = xl[:, :, :T]
    std = net.feedForward(x, True)
    for _ in range(3):
        got = net.rnnActivateUsingStoredState(x, True, True)
        assert len(got) == len(std)
        for a, b in zip(std, got):
            assert torch.allclose(a, b, atol=1e-12)
    net.rnnClearPreviousState()
    full = net.feedForward(xl, True)
    l0, l1 = net.getLayer(0), net.getLayer(1)
    for i in range(slices):
        sl = slice(i * T, (i + 1) * T)
        for _ in range(2):                                   # repeatable: the previous state is not consumed
            got = net.rnnActivateUsingStoredState(xl[:, :, sl], True, True)
            for j, (a, b) in enumerate(zip(full, got)):
                assert torch.allclose(a[:, :, sl], b, atol=1e-10), (i, j)
        l0.rnnSetPreviousState(l0.rnnGetTBPTTState())
        l1.rnnSetPreviousState(l1.rnnGetTBPTTState())
