"""Layer gradient checks in double precision, one case per scenario of the reference's CORET:gradientcheck/ suites
not already in tests/test_gradient_checks.py: CNNGradientCheckTest (space-to-depth / -batch, upsampling, subsampling,
Same mode incl. strided, zero padding, deconvolution, separable and dilated convolution, cropping), BNGradientCheckTest
(fixed gamma / beta, CNN + subsampling, graph), GradientCheckTestsMasking (per-output masking MLP / RNN, output-layer
masking MLN / CG, bidirectional), NoBiasGradientCheckTests, RnnGradientChecks (Bidirectional wrapper modes,
SimpleRnn, LastTimeStep), OutputLayerGradientChecks (RnnLossLayer, CnnLossLayer), UtilLayerGradientChecks (MaskLayer),
CNN1DGradientCheckTest and LSTMGradientCheckTests (edge cases, CNN -> FF -> RNN). The networks are this framework's;
the reference's test topologies are the spec."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.gradientcheck import checkGradients
from deeplearning4j_amd.nn.conf.layers import (Bidirectional, Cropping2D, Deconvolution2D, LastTimeStep, MaskLayer,
                                               SeparableConvolution2D, SpaceToBatchLayer, SpaceToDepthLayer,
                                               Subsampling1DLayer, Upsampling2D, ZeroPadding1DLayer, ZeroPaddingLayer)

DEV = torch.device("cpu")


def mln(layers, inputType=None, l1=0.0, l2=0.0, seed=12345, **kw):
    b = (NeuralNetConfiguration.Builder().seed(seed).dataType(DataType.DOUBLE).updater(NoOp())
         .weightInit(NormalDistribution(0, 1)).l1(l1).l2(l2).list())
    for i, l in enumerate(layers):
        b.layer(i, l)
    if inputType is not None:
        b.setInputType(inputType)
    for k, v in kw.items():
        getattr(b, k)(v)
    net = MultiLayerNetwork(b.build())
    net.init(device=DEV)
    return net


def r(*shape, seed=1):
    return torch.randn(*shape, dtype=torch.float64, generator=torch.Generator().manual_seed(seed))


def onehot(n, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    y = torch.zeros(n, k, dtype=torch.float64)
    y[torch.arange(n), torch.randint(0, k, (n,), generator=g)] = 1
    return y


def rnn_onehot(n, k, T, seed=0):
    g = torch.Generator().manual_seed(seed)
    y = torch.zeros(n, k, T, dtype=torch.float64)
    idx = torch.randint(0, k, (n, T), generator=g)
    for i in range(n):
        y[i, idx[i], torch.arange(T)] = 1
    return y


def conv(nin, nout, k=2, s=1, act=Activation.TANH, **kw):
    b = ConvolutionLayer.Builder(k, k).stride(s, s).nIn(nin).nOut(nout).activation(act)
    for key, v in kw.items():
        getattr(b, key)(*v) if isinstance(v, tuple) else getattr(b, key)(v)
    return b.build()


def out(nout, nin=None, loss=LossFunction.MCXENT, act=Activation.SOFTMAX):
    b = OutputLayer.Builder(loss).nOut(nout).activation(act)
    if nin:
        b = b.nIn(nin)
    return b.build()


def check(net, x, y, **kw):
    assert checkGradients(net, input=x, labels=y, print_results=True, **kw)


# ------------------------------------------------------------------------------------------ CNNGradientCheckTest
@pytest.mark.parametrize("l1,l2", [(0.0, 0.0), (0.1, 0.2)])
def test_cnn_mln_l1_l2(l1, l2):
    net = mln([conv(1, 2), out(3)], InputType.convolutional(4, 4, 1), l1=l1, l2=l2)
    check(net, r(3, 1, 4, 4), onehot(3, 3))


def test_cnn_with_space_to_depth():
    net = mln([conv(2, 2, k=2), SpaceToDepthLayer.Builder(2).build(), out(3)], InputType.convolutional(5, 5, 2))
    check(net, r(2, 2, 5, 5), onehot(2, 3))


def test_cnn_with_space_to_batch():
    net = mln([conv(2, 3, k=2), SpaceToBatchLayer.Builder([2, 2]).build(),
               GlobalPoolingLayer.Builder(PoolingType.AVG).build(), out(3, 3)],
              InputType.convolutional(5, 5, 2))
    x = r(2, 2, 5, 5)
    y = onehot(8, 3)                 # space-to-batch multiplies the minibatch by the block count
    check(net, x, y)


@pytest.mark.parametrize("size", [1, 2, 3])
def test_cnn_with_upsampling(size):
    net = mln([conv(2, 2, k=2), Upsampling2D.Builder(size).build(), out(3)], InputType.convolutional(4, 4, 2))
    check(net, r(2, 2, 4, 4), onehot(2, 3))


@pytest.mark.parametrize("pt", [PoolingType.MAX, PoolingType.AVG, PoolingType.PNORM])
def test_cnn_with_subsampling(pt):
    b = SubsamplingLayer.Builder(pt).kernelSize(2, 2).stride(1, 1)
    if pt == PoolingType.PNORM:
        b = b.pnorm(2)
    net = mln([conv(2, 3, k=2), b.build(), out(2)], InputType.convolutional(5, 5, 2))
    check(net, r(3, 2, 5, 5), onehot(3, 2))


def test_cnn_with_subsampling_v2_and_multilayer():
    net = mln([conv(2, 3, k=2), SubsamplingLayer.Builder(PoolingType.MAX).kernelSize(2, 2).stride(2, 2).build(),
               conv(3, 2, k=2, act=Activation.SIGMOID), out(3)], InputType.convolutional(7, 7, 2))
    check(net, r(2, 2, 7, 7), onehot(2, 3))


@pytest.mark.parametrize("stride", [1, 2])
def test_cnn_same_padding_mode(stride):
    net = mln([ConvolutionLayer.Builder(3, 3).stride(stride, stride).nIn(2).nOut(2)
               .convolutionMode(ConvolutionMode.Same).activation(Activation.TANH).build(),
               SubsamplingLayer.Builder(PoolingType.MAX).kernelSize(2, 2).stride(stride, stride)
               .convolutionMode(ConvolutionMode.Same).build(),
               out(3)], InputType.convolutional(5, 5, 2))
    check(net, r(2, 2, 5, 5), onehot(2, 3))


def test_cnn_zero_padding_layer():
    net = mln([conv(2, 2, k=2), ZeroPaddingLayer.Builder(1, 2, 2, 1).build(), conv(2, 2, k=2), out(3)],
              InputType.convolutional(4, 4, 2))
    check(net, r(2, 2, 4, 4), onehot(2, 3))


@pytest.mark.parametrize("mode", [ConvolutionMode.Truncate, ConvolutionMode.Same])
def test_deconvolution_2d(mode):
    net = mln([Deconvolution2D.Builder(2, 2).stride(2, 2).nIn(2).nOut(3).convolutionMode(mode)
               .activation(Activation.TANH).build(), out(2)], InputType.convolutional(3, 3, 2))
    check(net, r(2, 2, 3, 3), onehot(2, 2))


def test_separable_conv_2d():
    net = mln([SeparableConvolution2D.Builder(2, 2).depthMultiplier(2).nIn(2).nOut(3)
               .activation(Activation.TANH).build(), out(2)], InputType.convolutional(4, 4, 2))
    check(net, r(2, 2, 4, 4), onehot(2, 2))


@pytest.mark.parametrize("dil", [1, 2])
def test_cnn_dilated(dil):
    net = mln([ConvolutionLayer.Builder(2, 2).dilation(dil, dil).nIn(2).nOut(2).activation(Activation.TANH).build(),
               SubsamplingLayer.Builder(PoolingType.MAX).kernelSize(2, 2).dilation(dil, dil).build(),
               out(3)], InputType.convolutional(7, 7, 2))
    check(net, r(2, 2, 7, 7), onehot(2, 3))


def test_cropping_2d_layer():
    net = mln([conv(2, 2, k=2), Cropping2D.Builder(1, 0, 2, 1).build(), out(3)], InputType.convolutional(6, 6, 2))
    check(net, r(2, 2, 6, 6), onehot(2, 3))


# ------------------------------------------------------------------------------------------ BNGradientCheckTest
def test_bn_2d_fixed_gamma_beta():
    net = mln([DenseLayer.Builder().nIn(4).nOut(3).activation(Activation.IDENTITY).build(),
               BatchNormalization.Builder().lockGammaBeta(True).gamma(2.0).beta(0.5).build(),
               ActivationLayer.Builder().activation(Activation.TANH).build(), out(3, 3)], InputType.feedForward(4))
    check(net, r(10, 4), onehot(10, 3))


def test_bn_cnn_fixed_gamma_beta():
    net = mln([conv(1, 2, k=2, act=Activation.IDENTITY),
               BatchNormalization.Builder().lockGammaBeta(True).gamma(2.0).beta(0.5).build(),
               ActivationLayer.Builder().activation(Activation.TANH).build(), out(3)],
              InputType.convolutional(4, 4, 1))
    check(net, r(5, 1, 4, 4), onehot(5, 3))


def test_bn_with_cnn_and_subsampling():
    net = mln([conv(2, 3, k=2, act=Activation.IDENTITY), BatchNormalization.Builder().build(),
               ActivationLayer.Builder().activation(Activation.TANH).build(),
               SubsamplingLayer.Builder(PoolingType.MAX).kernelSize(2, 2).stride(1, 1).build(),
               BatchNormalization.Builder().build(), out(2)], InputType.convolutional(5, 5, 2), l2=0.1)
    check(net, r(4, 2, 5, 5), onehot(4, 2))


def test_bn_comp_graph():
    g = (NeuralNetConfiguration.Builder().seed(1).dataType(DataType.DOUBLE).updater(NoOp())
         .weightInit(NormalDistribution(0, 1)).graphBuilder().addInputs("in")
         .addLayer("bn", BatchNormalization.Builder().build(), "in")
         .addLayer("out", out(3, 4), "bn").setOutputs("out").setInputTypes(InputType.feedForward(4)))
    net = ComputationGraph(g.build())
    net.init(device=DEV)
    check(net, [r(10, 4)], [onehot(10, 3)])


# ------------------------------------------------------------------------------------------ masking
def test_per_output_masking_mlp():
    net = mln([DenseLayer.Builder().nIn(4).nOut(5).activation(Activation.TANH).build(),
               out(3, 5, LossFunction.XENT, Activation.SIGMOID)])
    y = torch.bernoulli(torch.full((6, 3), 0.5, dtype=torch.float64), generator=torch.Generator().manual_seed(2))
    mask = torch.tensor([[1, 1, 0], [0, 1, 1], [1, 0, 1], [1, 1, 1], [0, 0, 1], [1, 0, 0]], dtype=torch.float64)
    check(net, r(6, 4), y, labelMask=mask)


def test_per_output_masking_rnn():
    net = mln([GravesLSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
               RnnOutputLayer.Builder(LossFunction.XENT).nIn(4).nOut(2).activation(Activation.SIGMOID).build()])
    y = torch.bernoulli(torch.full((2, 2, 4), 0.5, dtype=torch.float64), generator=torch.Generator().manual_seed(3))
    mask = torch.bernoulli(torch.full((2, 2, 4), 0.7, dtype=torch.float64),
                           generator=torch.Generator().manual_seed(4))
    check(net, r(2, 3, 4), y, labelMask=mask)


def test_output_layer_masking_cg():
    g = (NeuralNetConfiguration.Builder().seed(1).dataType(DataType.DOUBLE).updater(NoOp())
         .weightInit(NormalDistribution(0, 1)).graphBuilder().addInputs("in")
         .addLayer("lstm", LSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(), "in")
         .addLayer("out", RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(4).nOut(3).activation(Activation.SOFTMAX)
                   .build(), "lstm").setOutputs("out"))
    net = ComputationGraph(g.build())
    net.init(device=DEV)
    mask = torch.tensor([[1, 1, 1, 0], [1, 0, 0, 0]], dtype=torch.float64)
    check(net, [r(2, 3, 4)], [rnn_onehot(2, 3, 4)], inputMask=[mask], labelMask=[mask])


def test_bidirectional_lstm_masking():
    net = mln([GravesBidirectionalLSTM.Builder().nIn(3).nOut(3).activation(Activation.TANH).build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(3).nOut(2).activation(Activation.SOFTMAX).build()])
    mask = torch.tensor([[1, 1, 1, 1, 1], [1, 1, 1, 0, 0], [1, 0, 0, 0, 0]], dtype=torch.float64)
    check(net, r(3, 3, 5), rnn_onehot(3, 2, 5), inputMask=mask, labelMask=mask)


# ------------------------------------------------------------------------------------------ no bias
@pytest.mark.parametrize("bias", [True, False])
def test_no_bias_dense_and_output(bias):
    net = mln([DenseLayer.Builder().nIn(4).nOut(5).hasBias(bias).activation(Activation.TANH).build(),
               OutputLayer.Builder(LossFunction.MCXENT).nIn(5).nOut(3).hasBias(bias)
               .activation(Activation.SOFTMAX).build()])
    assert (len(net.params().reshape(-1)) == 4 * 5 + 5 * 3 + (8 if bias else 0))
    check(net, r(5, 4), onehot(5, 3))


def test_no_bias_rnn_output():
    net = mln([LSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(4).nOut(3).hasBias(False)
               .activation(Activation.SOFTMAX).build()])
    check(net, r(2, 3, 4), rnn_onehot(2, 3, 4))


def test_no_bias_embedding():
    net = mln([EmbeddingLayer.Builder().nIn(10).nOut(4).hasBias(False).build(), out(3, 4)])
    check(net, torch.tensor([[1], [7], [3]], dtype=torch.float64), onehot(3, 3))


def test_cnn_with_subsampling_no_bias():
    net = mln([ConvolutionLayer.Builder(2, 2).nIn(2).nOut(3).hasBias(False).activation(Activation.TANH).build(),
               SubsamplingLayer.Builder(PoolingType.MAX).kernelSize(2, 2).stride(1, 1).build(),
               out(2)], InputType.convolutional(5, 5, 2))
    check(net, r(2, 2, 5, 5), onehot(2, 2))


# ------------------------------------------------------------------------------------------ RNN
@pytest.mark.parametrize("mode", ["CONCAT", "ADD", "MUL", "AVERAGE"])
def test_bidirectional_wrapper(mode):
    nout = 4 if mode == "CONCAT" else 2
    net = mln([Bidirectional(LSTM.Builder().nIn(3).nOut(2).activation(Activation.TANH).build(), mode=mode),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(nout).nOut(3).activation(Activation.SOFTMAX).build()])
    check(net, r(2, 3, 4), rnn_onehot(2, 3, 4))


@pytest.mark.parametrize("masked", [False, True])
def test_simple_rnn(masked):
    net = mln([SimpleRnn.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(4).nOut(3).activation(Activation.SOFTMAX).build()])
    mask = torch.tensor([[1, 1, 1, 1], [1, 1, 0, 0]], dtype=torch.float64) if masked else None
    check(net, r(2, 3, 4), rnn_onehot(2, 3, 4), inputMask=mask, labelMask=mask)


@pytest.mark.parametrize("masked", [False, True])
def test_last_time_step_layer(masked):
    net = mln([LastTimeStep(SimpleRnn.Builder().nIn(3).nOut(4).activation(Activation.TANH).build()),
               out(3, 4)])
    mask = torch.tensor([[1, 1, 1, 1], [1, 1, 0, 0], [1, 0, 0, 0]], dtype=torch.float64) if masked else None
    check(net, r(3, 3, 4), onehot(3, 3), inputMask=mask)


# ------------------------------------------------------------------------------------------ output layers
@pytest.mark.parametrize("loss,act", [(LossFunction.MCXENT, Activation.SOFTMAX), (LossFunction.MSE, Activation.TANH),
                                      (LossFunction.XENT, Activation.SIGMOID)])
def test_rnn_loss_layer(loss, act):
    net = mln([LSTM.Builder().nIn(3).nOut(3).activation(Activation.TANH).build(),
               RnnLossLayer.Builder(loss).activation(act).build()])
    y = rnn_onehot(2, 3, 4) if loss != LossFunction.MSE else r(2, 3, 4, seed=5)
    mask = torch.tensor([[1, 1, 1, 1], [1, 1, 1, 0]], dtype=torch.float64)
    check(net, r(2, 3, 4), y, labelMask=mask)


@pytest.mark.parametrize("loss,act", [(LossFunction.MCXENT, Activation.SOFTMAX), (LossFunction.MSE, Activation.TANH)])
def test_cnn_loss_layer(loss, act):
    net = mln([ConvolutionLayer.Builder(2, 2).nIn(2).nOut(3).convolutionMode(ConvolutionMode.Same)
               .activation(Activation.TANH).build(), CnnLossLayer.Builder(loss).activation(act).build()],
              InputType.convolutional(4, 4, 2))
    if loss == LossFunction.MCXENT:
        y = torch.zeros(2, 3, 4, 4, dtype=torch.float64)
        y[:, 1] = 1
    else:
        y = r(2, 3, 4, 4, seed=6)
    check(net, r(2, 2, 4, 4), y)


# ------------------------------------------------------------------------------------------ utility layers
def test_mask_layer():
    net = mln([DenseLayer.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(), MaskLayer.Builder().build(),
               out(3, 4)])
    check(net, r(4, 3), onehot(4, 3))


def test_mask_layer_rnn():
    net = mln([SimpleRnn.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(), MaskLayer.Builder().build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(4).nOut(3).activation(Activation.SOFTMAX).build()])
    mask = torch.tensor([[1, 1, 1, 1], [1, 1, 0, 0]], dtype=torch.float64)
    check(net, r(2, 3, 4), rnn_onehot(2, 3, 4), inputMask=mask, labelMask=mask)


# ------------------------------------------------------------------------------------------ 1-D CNN
def test_cnn1d_with_zero_padding_1d():
    net = mln([Convolution1DLayer.Builder().kernelSize(2).nIn(3).nOut(4).activation(Activation.TANH).build(),
               ZeroPadding1DLayer.Builder(1, 2).build(),
               Convolution1DLayer.Builder().kernelSize(2).nIn(4).nOut(3).activation(Activation.TANH).build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nOut(3).activation(Activation.SOFTMAX).build()],
              InputType.recurrent(3, 6))
    T = 6 - 1 + 3 - 1
    check(net, r(2, 3, 6), rnn_onehot(2, 3, T))


@pytest.mark.parametrize("pt", [PoolingType.MAX, PoolingType.AVG])
def test_cnn1d_with_subsampling_1d(pt):
    net = mln([Convolution1DLayer.Builder().kernelSize(2).nIn(3).nOut(4).activation(Activation.TANH).build(),
               Subsampling1DLayer.Builder(pt).kernelSize(2).stride(1).build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nOut(3).activation(Activation.SOFTMAX).build()],
              InputType.recurrent(3, 6))
    check(net, r(2, 3, 6), rnn_onehot(2, 3, 4))


# ------------------------------------------------------------------------------------------ LSTM
@pytest.mark.parametrize("mb,T", [(1, 1), (1, 4), (3, 1)])
@pytest.mark.parametrize("kind", ["LSTM", "GravesLSTM", "GravesBidirectionalLSTM"])
def test_lstm_edge_cases(kind, mb, T):
    layer = getattr(__import__("deeplearning4j_amd", fromlist=[kind]), kind)
    net = mln([layer.Builder().nIn(3).nOut(2).activation(Activation.TANH).build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(2).nOut(2).activation(Activation.SOFTMAX).build()])
    check(net, r(mb, 3, T), rnn_onehot(mb, 2, T))


def test_lstm_basic_multi_layer_l1_l2():
    net = mln([LSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
               GravesLSTM.Builder().nIn(4).nOut(3).activation(Activation.SOFTSIGN).build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(3).nOut(2).activation(Activation.SOFTMAX).build()],
              l1=0.1, l2=0.2)
    check(net, r(2, 3, 4), rnn_onehot(2, 2, 4))


def test_cnn_ff_rnn():
    """CNN -> dense -> LSTM -> RNN output over time-distributed images (reference testGradientCnnFfRnn): the
    CnnToFeedForward / FeedForwardToRnn / RnnToCnn preprocessors are inferred from the input type."""
    from deeplearning4j_amd.nn.conf.preprocessors import (CnnToFeedForwardPreProcessor, FeedForwardToRnnPreProcessor,
                                                          RnnToCnnPreProcessor)
    b = (NeuralNetConfiguration.Builder().seed(12345).dataType(DataType.DOUBLE).updater(NoOp())
         .weightInit(NormalDistribution(0, 1)).list()
         .layer(0, ConvolutionLayer.Builder(2, 2).nIn(2).nOut(3).activation(Activation.TANH).build())
         .layer(1, DenseLayer.Builder().nIn(3 * 2 * 2).nOut(4).activation(Activation.TANH).build())
         .layer(2, GravesLSTM.Builder().nIn(4).nOut(3).activation(Activation.TANH).build())
         .layer(3, RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(3).nOut(2).activation(Activation.SOFTMAX).build())
         .inputPreProcessor(0, RnnToCnnPreProcessor(inputHeight=3, inputWidth=3, numChannels=2))
         .inputPreProcessor(1, CnnToFeedForwardPreProcessor(inputHeight=2, inputWidth=2, numChannels=3))
         .inputPreProcessor(2, FeedForwardToRnnPreProcessor()))
    net = MultiLayerNetwork(b.build())
    net.init(device=DEV)
    T = 3
    check(net, r(2, 2 * 3 * 3, T), rnn_onehot(2, 2, T))
