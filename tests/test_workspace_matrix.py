"""Workspace-mode matrix (reference CORET:nn/misc/WorkspaceTests.java: testWorkspaceIndependence,
testWithPreprocessorsCG/MLN, testRnnTimeStep, testTbpttFit, testScalarOutputCase, testClearing): every topology is
trained with the training workspace ENABLED (the LOOP_FF_BP / LOOP_TBPTT arenas, memory/arena.py) and with NONE, with
the executioner in SCOPE_PANIC mode (profiling.py: every layer output is checked against its arena generation), and
must give bitwise-identical parameters and scores."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.memory.workspace import check_scope
from deeplearning4j_amd.nn.conf import WorkspaceMode
from deeplearning4j_amd.profiling import ProfilingMode, getExecutioner


@pytest.fixture(autouse=True)
def _scope_panic():
    ex = getExecutioner()
    prev = ex.getProfilingMode()
    ex.setProfilingMode(ProfilingMode.SCOPE_PANIC)
    yield
    ex.setProfilingMode(prev)


def _b(mode, seed=3):
    return (NeuralNetConfiguration.Builder().seed(seed).updater(Adam(0.01)).weightInit(WeightInit.XAVIER)
            .trainingWorkspaceMode(mode).inferenceWorkspaceMode(mode))


def _cnn_mln(mode):
    conf = (_b(mode).list()
            .layer(ConvolutionLayer.Builder(3, 3).nIn(2).nOut(4).activation(Activation.RELU).build())
            .layer(SubsamplingLayer.Builder(PoolingType.MAX).kernelSize(2, 2).stride(2, 2).build())
            .layer(DenseLayer.Builder().nOut(8).activation(Activation.TANH).build())        # CnnToFeedForward
            .layer(OutputLayer.Builder(LossFunction.MCXENT).nOut(3).activation(Activation.SOFTMAX).build())
            .setInputType(InputType.convolutional(8, 8, 2)).build())
    net = MultiLayerNetwork(conf)
    net.init()
    return net


def _cnn_cg(mode):
    conf = (_b(mode).graphBuilder().addInputs("in")
            .addLayer("c", ConvolutionLayer.Builder(3, 3).nIn(2).nOut(4).activation(Activation.RELU).build(), "in")
            .addLayer("d", DenseLayer.Builder().nOut(8).activation(Activation.TANH).build(), "c")
            .addLayer("rnn_in", DenseLayer.Builder().nOut(8).activation(Activation.TANH).build(), "d")
            .addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).nOut(3).activation(Activation.SOFTMAX).build(),
                      "rnn_in")
            .setOutputs("out").setInputTypes(InputType.convolutional(8, 8, 2)).build())
    net = ComputationGraph(conf)
    net.init()
    return net


def _rnn_mln(mode, tbptt):
    lb = _b(mode).list()
    lb.layer(GravesLSTM.Builder().nIn(3).nOut(6).activation(Activation.TANH).build())
    lb.layer(LSTM.Builder().nIn(6).nOut(5).activation(Activation.TANH).build())
    lb.layer(RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(5).nOut(3).activation(Activation.SOFTMAX).build())
    if tbptt:
        lb.backpropType(BackpropType.TruncatedBPTT).tBPTTLength(4)
    net = MultiLayerNetwork(lb.build())
    net.init()
    return net


def _rnn_cg(mode, tbptt):
    g = (_b(mode).graphBuilder().addInputs("in")
         .addLayer("l0", GravesLSTM.Builder().nIn(3).nOut(6).activation(Activation.TANH).build(), "in")
         .addLayer("l1", LSTM.Builder().nIn(6).nOut(5).activation(Activation.TANH).build(), "l0")
         .addLayer("out", RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(5).nOut(3).activation(Activation.SOFTMAX)
                   .build(), "l1").setOutputs("out"))
    if tbptt:
        g = g.backpropType(BackpropType.TruncatedBPTT).tBPTTForwardLength(4).tBPTTBackwardLength(4)
    net = ComputationGraph(g.build())
    net.init()
    return net


def _img(n=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 2, 8, 8, generator=g)
    y = torch.nn.functional.one_hot(torch.randint(0, 3, (n,), generator=g), 3).float()
    return x, y


def _seq(n=4, T=10, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, T, generator=g)
    y = torch.zeros(n, 3, T)
    y[torch.arange(n), torch.randint(0, 3, (n,), generator=g)] = 1
    return x, y


def _fit(net, x, y, n=3):
    for _ in range(n):
        if isinstance(net, ComputationGraph):
            net.fit([x], [y])
        else:
            net.fit(x, y)
    return net


@pytest.mark.parametrize("make", ["mln", "cg"])
def test_with_preprocessors(make):
    mk = _cnn_mln if make == "mln" else _cnn_cg
    x, y = _img()
    a, b = _fit(mk(WorkspaceMode.ENABLED), x, y), _fit(mk(WorkspaceMode.NONE), x, y)
    assert torch.equal(a.params(), b.params())
    assert a.score() == b.score()
    assert a._loop_ws is not None and a._loop_ws.stats()["spilled"] == 0
    out = a.output(x) if make == "mln" else a.output(x)[0]
    check_scope(out, "output after fit")                                  # results never leak arena memory


@pytest.mark.parametrize("make", ["mln", "cg"])
@pytest.mark.parametrize("tbptt", [False, True])
def test_rnn_fit(make, tbptt):
    mk = _rnn_mln if make == "mln" else _rnn_cg
    x, y = _seq()
    a, b = _fit(mk(WorkspaceMode.ENABLED, tbptt), x, y), _fit(mk(WorkspaceMode.NONE, tbptt), x, y)
    assert torch.equal(a.params(), b.params())
    assert a.score() == b.score()


def test_rnn_time_step_matches_full_sequence():
    x, y = _seq()
    net = _fit(_rnn_mln(WorkspaceMode.ENABLED, False), x, y)
    full = net.output(x)
    net.rnnClearPreviousState()
    steps = [net.rnnTimeStep(x[:, :, t:t + 1]) for t in range(x.shape[2])]
    stepped = torch.cat([s.reshape(s.shape[0], s.shape[1], -1) for s in steps], dim=2)
    assert torch.allclose(stepped, full, atol=1e-5)
    for k, v in net.layers[0].stateMap.items():
        check_scope(v, f"rnnTimeStep state {k}")


def test_workspace_independence():
    """Two networks interleaving their fits (each with its own arena) equal the same networks fitted alone."""
    x, y = _img()
    a1, a2 = _cnn_mln(WorkspaceMode.ENABLED), _cnn_cg(WorkspaceMode.ENABLED)
    for _ in range(3):
        a1.fit(x, y)
        a2.fit([x], [y])
    b1, b2 = _fit(_cnn_mln(WorkspaceMode.NONE), x, y), _fit(_cnn_cg(WorkspaceMode.NONE), x, y)
    assert torch.equal(a1.params(), b1.params()) and torch.equal(a2.params(), b2.params())
    assert a1._loop_ws is not a2._loop_ws


def test_scalar_output_case():
    conf = (_b(WorkspaceMode.ENABLED).list()
            .layer(DenseLayer.Builder().nIn(4).nOut(3).activation(Activation.TANH).build())
            .layer(OutputLayer.Builder(LossFunction.MSE).nIn(3).nOut(1).activation(Activation.IDENTITY).build())
            .build())
    net = MultiLayerNetwork(conf)
    net.init()
    x = torch.randn(5, 4)
    net.fit(x, torch.randn(5, 1))
    out = net.output(x[:1])
    assert out.shape == (1, 1)
    check_scope(out, "scalar output")


def test_clearing():
    """After fit the layers hold no arena arrays a later output() could read by mistake (reference testClearing:
    the iteration's inputs / labels are cleared): the next output allocates plainly and is correct."""
    x, y = _img()
    a = _fit(_cnn_mln(WorkspaceMode.ENABLED), x, y)
    b = _fit(_cnn_mln(WorkspaceMode.NONE), x, y)
    assert torch.equal(a.output(x), b.output(x))
    assert torch.equal(a.output(x[:2]), b.output(x[:2]))
