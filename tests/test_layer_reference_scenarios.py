"""Layer-level scenarios with the reference's own inputs and expected numbers:
MaskZeroLayer over an LSTM (CORET: nn/layers/recurrent/MaskZeroLayerTest.java), Upsampling1D/2D forward and backprop
(nn/layers/convolution/Upsampling1DTest.java, Upsampling2DTest.java), SpaceToDepth forward/backward
(nn/layers/convolution/SpaceToDepthTest.java), recurrent weight init (nn/layers/recurrent/TestRecurrentWeightInit.java),
LastTimeStep with and without an input mask (nn/layers/recurrent/TestLastTimeStepLayer.java) and DropoutLayer
inference/training behaviour (nn/layers/DropoutLayerTest.java)."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403

DEV = torch.device("cpu")


def _mln(layers, inputType=None, weightInit=None, dtype=DataType.DOUBLE):
    b = NeuralNetConfiguration.Builder().seed(12345).dataType(dtype).updater(NoOp())
    if weightInit is not None:
        b = b.weightInit(weightInit)
    b = b.list()
    for i, l in enumerate(layers):
        b.layer(i, l)
    if inputType is not None:
        b.setInputType(inputType)
    net = MultiLayerNetwork(b.build())
    net.init(device=DEV)
    return net


def _eps_out(res):
    """backpropGradient returns (Gradient, epsilon) like the reference's Pair."""
    return res[1] if isinstance(res, tuple) else res


def test_mask_zero_layer_lstm():
    # LSTM(nIn=2, nOut=1), identity activations, all params 0 except the bias (indices 12..15) = 1: every unmasked step
    # adds 1 to the cell, masked steps (all-zero input columns) reset to 0
    lstm = LSTM.Builder().nIn(2).nOut(1).activation(Activation.IDENTITY).gateActivationFunction(
        Activation.IDENTITY).build()
    net = _mln([MaskZeroLayer(underlying=lstm, maskingValue=0.0)])
    p = torch.zeros(net.numParams(), dtype=torch.float64)
    p[12:16] = 1.0
    net.setParams(p)
    ex1 = [[0.0, 3.0, 5.0], [0.0, 0.0, 2.0]]
    ex2 = [[0.0, 0.0, 2.0], [0.0, 0.0, 2.0]]
    x = torch.tensor([ex1, ex2], dtype=torch.float64)          # [mb=2, nIn=2, T=3]
    out = net.output(x)
    assert tuple(out.shape) == (2, 1, 3)
    torch.testing.assert_close(out[0, 0], torch.tensor([0.0, 1.0, 2.0], dtype=torch.float64))
    torch.testing.assert_close(out[1, 0], torch.tensor([0.0, 0.0, 1.0], dtype=torch.float64))


def test_upsampling1d_forward_backward():
    net = _mln([Upsampling1D(size=2)])
    layer = net.layers[0]
    x = torch.tensor([1.0, 2.0, 3.0, 4.0], dtype=torch.float64).reshape(1, 1, 4)
    out = layer.activate(x, training=True)
    torch.testing.assert_close(out.reshape(-1), torch.tensor([1.0, 1, 2, 2, 3, 3, 4, 4], dtype=torch.float64))
    eps = torch.tensor([1.0, 3, 2, 6, 7, 2, 5, 5], dtype=torch.float64).reshape(1, 1, 8)
    dx = _eps_out(layer.backpropGradient(eps))
    torch.testing.assert_close(dx.reshape(-1), torch.tensor([4.0, 8, 9, 10], dtype=torch.float64))
    assert tuple(dx.shape) == (1, 1, 4)
    # a larger batch keeps rank and depth
    xb = torch.rand(5, 20, 28, dtype=torch.float64)
    ob = layer.activate(xb, training=True)
    assert tuple(ob.shape) == (5, 20, 56)
    assert tuple(_eps_out(layer.backpropGradient(torch.ones_like(ob))).shape) == (5, 20, 28)
    assert not net.layers[0].params


def test_upsampling2d_forward_backward():
    net = _mln([Upsampling2D(size=2)])
    layer = net.layers[0]
    x = torch.tensor([1.0, 2.0, 3.0, 4.0], dtype=torch.float64).reshape(1, 1, 2, 2)
    out = layer.activate(x, training=True)
    exp = torch.tensor([1.0, 1, 2, 2, 1, 1, 2, 2, 3, 3, 4, 4, 3, 3, 4, 4], dtype=torch.float64).reshape(1, 1, 4, 4)
    torch.testing.assert_close(out, exp)
    dx = _eps_out(layer.backpropGradient(torch.ones(1, 1, 4, 4, dtype=torch.float64)))
    torch.testing.assert_close(dx, torch.full((1, 1, 2, 2), 4.0, dtype=torch.float64))
    xb = torch.rand(5, 20, 28, 28, dtype=torch.float64)
    ob = layer.activate(xb, training=True)
    assert tuple(ob.shape) == (5, 20, 56, 56)
    assert tuple(_eps_out(layer.backpropGradient(torch.ones_like(ob))).shape) == (5, 20, 28, 28)


def test_space_to_depth_forward_backward():
    net = _mln([SpaceToDepthLayer.Builder(2).build()])
    layer = net.layers[0]
    data = torch.arange(1.0, 9.0, dtype=torch.float64).reshape(1, 2, 2, 2)
    expected = torch.tensor([1.0, 5, 2, 6, 3, 7, 4, 8], dtype=torch.float64).reshape(1, 8, 1, 1)
    out = layer.activate(data, training=True)
    assert tuple(out.shape) == (1, 8, 1, 1)
    torch.testing.assert_close(out, expected)
    # the backward pass is the inverse permutation: the expected output as epsilon gives back the input
    dx = _eps_out(layer.backpropGradient(expected))
    torch.testing.assert_close(dx, data)


@pytest.mark.parametrize("kind", ["LSTM", "GravesLSTM", "SimpleRnn"])
@pytest.mark.parametrize("rw_init", [False, True])
def test_recurrent_weight_init(kind, rw_init):
    cls = {"LSTM": LSTM, "GravesLSTM": GravesLSTM, "SimpleRnn": SimpleRnn}[kind]
    b = cls.Builder().nIn(10).nOut(10)
    if rw_init:
        b = b.weightInitRecurrent(UniformDistribution(2, 3))
    net = _mln([b.build()], weightInit=UniformDistribution(0, 1))
    W, RW = net.layers[0].params["W"], net.layers[0].params["RW"]
    assert 0.0 <= W.min().item() and W.max().item() <= 1.0
    if rw_init:
        assert RW.min().item() >= 2.0 and RW.max().item() <= 3.0
    else:
        assert 0.0 <= RW.min().item() and RW.max().item() <= 1.0


def test_last_time_step_with_and_without_mask():
    conf = (NeuralNetConfiguration.Builder().seed(12345).dataType(DataType.DOUBLE).graphBuilder().addInputs("in")
            .addLayer("lastTS", LastTimeStep(underlying=SimpleRnn.Builder().nIn(5).nOut(6).build()), "in")
            .setOutputs("lastTS").build())
    graph = ComputationGraph(conf)
    graph.init(device=DEV)
    g = torch.Generator().manual_seed(12345)
    x = torch.rand(3, 5, 6, generator=g, dtype=torch.float64)
    under = graph.getLayer("lastTS").getUnderlying()
    out_under = under.activate(x, training=False)
    torch.testing.assert_close(graph.outputSingle(x), out_under[:, :, 5])

    mask = torch.tensor([[1, 1, 1, 0, 0, 0], [1, 1, 1, 1, 0, 0], [1, 1, 1, 1, 1, 0]], dtype=torch.float64)
    graph.setLayerMaskArrays([mask], None)
    out = graph.outputSingle(x)
    exp = torch.stack([out_under[0, :, 2], out_under[1, :, 3], out_under[2, :, 4]])
    torch.testing.assert_close(out, exp)
    graph.clearLayerMaskArrays()


def test_dropout_layer_inference_identity_and_training_mask():
    net = _mln([DropoutLayer.Builder(0.5).nIn(20).nOut(20).build()])
    x = torch.rand(64, 20, dtype=torch.float64) + 0.5
    torch.testing.assert_close(net.output(x), x)                 # inference: identity
    layer = net.layers[0]
    y = layer.activate(x, training=True)
    kept = y != 0
    # inverted dropout with retain probability 0.5: survivors are scaled by 1/0.5, and roughly half survive
    torch.testing.assert_close(y[kept], x[kept] * 2.0)
    frac = kept.double().mean().item()
    assert 0.35 < frac < 0.65
    # the backward pass routes epsilon through the same mask
    dx = _eps_out(layer.backpropGradient(torch.ones_like(x)))
    torch.testing.assert_close(dx, kept.double() * 2.0)
