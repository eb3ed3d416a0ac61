"""Numerical gradient checks in double precision (reference CORET:gradientcheck/*.java:
GradientCheckTests, CNNGradientCheckTest, BNGradientCheckTest, LSTMGradientCheckTests,
GlobalPoolingGradientCheckTests, GradientCheckTestsComputationGraph, LossFunctionGradientCheck)."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.gradientcheck import checkGradients
from deeplearning4j_amd.nn.conf import losses as L

DEV = torch.device("cpu")


def onehot(n, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    y = torch.zeros(n, k, dtype=torch.float64)
    y[torch.arange(n), torch.randint(0, k, (n,), generator=g)] = 1
    return y


def mln(layers, inputType=None, updater=None, l1=0.0, l2=0.0, **kw):
    b = (NeuralNetConfiguration.Builder().seed(12345).dataType(DataType.DOUBLE).updater(updater or NoOp())
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


@pytest.mark.parametrize("act", [Activation.TANH, Activation.SIGMOID, Activation.SOFTPLUS, Activation.ELU,
                                 Activation.CUBE, Activation.SOFTSIGN, Activation.HARDTANH])
def test_dense_activations(act):
    net = mln([DenseLayer.Builder().nIn(4).nOut(5).activation(act).build(),
               OutputLayer.Builder(LossFunction.MCXENT).nIn(5).nOut(3).activation(Activation.SOFTMAX).build()])
    x = torch.randn(6, 4, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=onehot(6, 3), print_results=True)


def test_dense_l1_l2():
    net = mln([DenseLayer.Builder().nIn(4).nOut(5).activation(Activation.TANH).build(),
               OutputLayer.Builder(LossFunction.MSE).nIn(5).nOut(3).activation(Activation.IDENTITY).build()],
              l1=0.01, l2=0.02)
    x = torch.randn(5, 4, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=torch.randn(5, 3, dtype=torch.float64), print_results=True)


@pytest.mark.parametrize("loss,act,lab", [
    (LossFunction.MSE, Activation.IDENTITY, "real"), (LossFunction.L1, Activation.TANH, "real"),
    (LossFunction.XENT, Activation.SIGMOID, "binary"), (LossFunction.MCXENT, Activation.SOFTMAX, "onehot"),
    (LossFunction.NEGATIVELOGLIKELIHOOD, Activation.SOFTMAX, "onehot"), (LossFunction.HINGE, Activation.TANH, "pm1"),
    (LossFunction.SQUARED_HINGE, Activation.TANH, "pm1"), (LossFunction.KL_DIVERGENCE, Activation.SOFTMAX, "prob"),
    (LossFunction.POISSON, Activation.SOFTPLUS, "pos"), (LossFunction.COSINE_PROXIMITY, Activation.TANH, "real"),
    (LossFunction.MEAN_SQUARED_LOGARITHMIC_ERROR, Activation.SOFTPLUS, "pos"),
    (LossFunction.MEAN_ABSOLUTE_PERCENTAGE_ERROR, Activation.IDENTITY, "pos"),
    (LossFunction.L2, Activation.IDENTITY, "real"), (LossFunction.MEAN_ABSOLUTE_ERROR, Activation.IDENTITY, "real")])
def test_loss_functions(loss, act, lab):
    g = torch.Generator().manual_seed(3)
    n, k = 5, 4
    y = {"real": lambda: torch.randn(n, k, generator=g, dtype=torch.float64),
         "binary": lambda: (torch.rand(n, k, generator=g) > 0.5).double(),
         "onehot": lambda: onehot(n, k),
         "pm1": lambda: (torch.rand(n, k, generator=g) > 0.5).double() * 2 - 1,
         "prob": lambda: torch.softmax(torch.randn(n, k, generator=g, dtype=torch.float64), 1),
         "pos": lambda: torch.rand(n, k, generator=g, dtype=torch.float64) + 0.5}[lab]()
    net = mln([DenseLayer.Builder().nIn(3).nOut(6).activation(Activation.TANH).build(),
               OutputLayer.Builder(loss).nIn(6).nOut(k).activation(act).build()])
    assert checkGradients(net, input=torch.randn(n, 3, dtype=torch.float64), labels=y, print_results=True)


@pytest.mark.parametrize("mode", [ConvolutionMode.Truncate, ConvolutionMode.Same])
def test_cnn_pooling(mode):
    net = mln([ConvolutionLayer.Builder([3, 3], [2, 1]).nOut(3).activation(Activation.TANH).convolutionMode(mode)
               .build(),
               SubsamplingLayer.Builder(PoolingType.AVG, [2, 2], [1, 1]).convolutionMode(mode).build(),
               ConvolutionLayer.Builder([2, 2]).nOut(2).activation(Activation.SIGMOID).convolutionMode(mode).build(),
               OutputLayer.Builder(LossFunction.MCXENT).nOut(3).activation(Activation.SOFTMAX).build()],
              InputType.convolutional(7, 6, 2))
    x = torch.randn(3, 2, 7, 6, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=onehot(3, 3), print_results=True)


def test_cnn_maxpool_pnorm_zeropad():
    net = mln([ZeroPaddingLayer.Builder(1, 2).build(),
               ConvolutionLayer.Builder([2, 2]).nOut(3).activation(Activation.TANH).build(),
               SubsamplingLayer.Builder(PoolingType.MAX, [2, 2], [2, 2]).build(),
               SubsamplingLayer.Builder(PoolingType.PNORM, [2, 2], [1, 1]).pnorm(2).build(),
               OutputLayer.Builder(LossFunction.MCXENT).nOut(3).activation(Activation.SOFTMAX).build()],
              InputType.convolutional(6, 5, 2))
    x = torch.randn(2, 2, 6, 5, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=onehot(2, 3), print_results=True)


def test_batchnorm_cnn_and_dense():
    net = mln([ConvolutionLayer.Builder([2, 2]).nOut(4).activation(Activation.IDENTITY).build(),
               BatchNormalization.Builder().build(),
               ActivationLayer(Activation.TANH),
               DenseLayer.Builder().nOut(5).activation(Activation.IDENTITY).build(),
               BatchNormalization.Builder().build(),
               ActivationLayer(Activation.SIGMOID),
               OutputLayer.Builder(LossFunction.MCXENT).nOut(3).activation(Activation.SOFTMAX).build()],
              InputType.convolutional(5, 5, 2))
    x = torch.randn(6, 2, 5, 5, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=onehot(6, 3), print_results=True)


def test_batchnorm_fused_relu_path():
    """BN followed by ActivationLayer(ReLU) runs fused; gradients must still match (smooth region)."""
    net = mln([DenseLayer.Builder().nIn(4).nOut(6).activation(Activation.IDENTITY).build(),
               BatchNormalization.Builder().nOut(6).build(),
               ActivationLayer(Activation.RELU),
               OutputLayer.Builder(LossFunction.MSE).nOut(2).activation(Activation.IDENTITY).build()],
              InputType.feedForward(4))
    assert 2 in net._fused_passthrough
    x = torch.randn(8, 4, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=torch.randn(8, 2, dtype=torch.float64), print_results=True,
                          minAbsoluteError=1e-7)


@pytest.mark.parametrize("layer", ["LSTM", "GravesLSTM", "SimpleRnn", "GravesBidirectionalLSTM", "Bidirectional"])
def test_recurrent(layer):
    mk = {"LSTM": lambda: LSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
          "GravesLSTM": lambda: GravesLSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
          "SimpleRnn": lambda: SimpleRnn.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
          "GravesBidirectionalLSTM": lambda: GravesBidirectionalLSTM.Builder().nIn(3).nOut(4)
          .activation(Activation.TANH).build(),
          "Bidirectional": lambda: Bidirectional(LSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build())}
    net = mln([mk[layer](), RnnOutputLayer.Builder(LossFunction.MCXENT).nOut(3).activation(Activation.SOFTMAX).build()],
              InputType.recurrent(3))
    x = torch.randn(2, 3, 5, dtype=torch.float64)
    y = torch.zeros(2, 3, 5, dtype=torch.float64)
    y[:, 0, :] = 1
    y[1, 0, 2:] = 0
    y[1, 2, 2:] = 1
    assert checkGradients(net, input=x, labels=y, print_results=True)


def test_lstm_masking():
    net = mln([LSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
               RnnOutputLayer.Builder(LossFunction.MCXENT).nOut(2).activation(Activation.SOFTMAX).build()],
              InputType.recurrent(3))
    x = torch.randn(3, 3, 4, dtype=torch.float64)
    y = torch.zeros(3, 2, 4, dtype=torch.float64)
    y[:, 1] = 1
    mask = torch.tensor([[1, 1, 1, 1], [1, 1, 0, 0], [1, 0, 0, 0]], dtype=torch.float64)
    assert checkGradients(net, input=x, labels=y, inputMask=mask, labelMask=mask, print_results=True)


@pytest.mark.parametrize("pt", [PoolingType.AVG, PoolingType.MAX, PoolingType.SUM, PoolingType.PNORM])
def test_global_pooling_rnn_and_cnn(pt):
    net = mln([LSTM.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(),
               GlobalPoolingLayer.Builder(pt).build(),
               OutputLayer.Builder(LossFunction.MCXENT).nOut(2).activation(Activation.SOFTMAX).build()],
              InputType.recurrent(3))
    x = torch.randn(3, 3, 5, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=onehot(3, 2), print_results=True)
    net = mln([ConvolutionLayer.Builder([2, 2]).nOut(3).activation(Activation.TANH).build(),
               GlobalPoolingLayer.Builder(pt).build(),
               OutputLayer.Builder(LossFunction.MCXENT).nOut(2).activation(Activation.SOFTMAX).build()],
              InputType.convolutional(4, 4, 2))
    assert checkGradients(net, input=torch.randn(2, 2, 4, 4, dtype=torch.float64), labels=onehot(2, 2),
                          print_results=True)


def test_embedding_and_dropout_free_misc():
    net = mln([EmbeddingLayer.Builder().nIn(5).nOut(4).activation(Activation.TANH).build(),
               DenseLayer.Builder().nOut(3).activation(Activation.SIGMOID).build(),
               OutputLayer.Builder(LossFunction.MCXENT).nOut(2).activation(Activation.SOFTMAX).build()],
              InputType.feedForward(1))
    x = torch.tensor([[0], [3], [1], [4]], dtype=torch.float64)
    assert checkGradients(net, input=x, labels=onehot(4, 2), print_results=True)


def test_computation_graph_vertices():
    conf = (NeuralNetConfiguration.Builder().seed(1).dataType(DataType.DOUBLE).updater(NoOp())
            .weightInit(NormalDistribution(0, 1)).graphBuilder()
            .addInputs("in1", "in2")
            .addLayer("d1", DenseLayer.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(), "in1")
            .addLayer("d2", DenseLayer.Builder().nIn(2).nOut(4).activation(Activation.SIGMOID).build(), "in2")
            .addVertex("add", ElementWiseVertex(ElementWiseVertex.Op.Add), "d1", "d2")
            .addVertex("prod", ElementWiseVertex(ElementWiseVertex.Op.Product), "d1", "d2")
            .addVertex("sub", ElementWiseVertex(ElementWiseVertex.Op.Subtract), "add", "prod")
            .addVertex("merge", MergeVertex(), "sub", "d1")
            .addVertex("subset", SubsetVertex(1, 5), "merge")
            .addVertex("scale", ScaleVertex(0.5), "subset")
            .addVertex("l2n", L2NormalizeVertex(), "scale")
            .addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).nIn(5).nOut(3).activation(Activation.SOFTMAX)
                      .build(), "l2n")
            .addLayer("out2", OutputLayer.Builder(LossFunction.MSE).nIn(4).nOut(2).activation(Activation.TANH)
                      .build(), "d1")
            .setOutputs("out", "out2").build())
    net = ComputationGraph(conf)
    net.init(device=DEV)
    x1, x2 = torch.randn(4, 3, dtype=torch.float64), torch.randn(4, 2, dtype=torch.float64)
    assert checkGradients(net, input=[x1, x2], labels=[onehot(4, 3), torch.randn(4, 2, dtype=torch.float64)],
                          print_results=True)


def test_cg_l2_vertex_stack_unstack():
    conf = (NeuralNetConfiguration.Builder().seed(1).dataType(DataType.DOUBLE).updater(NoOp())
            .weightInit(NormalDistribution(0, 1)).graphBuilder()
            .addInputs("a", "b")
            .addVertex("stack", StackVertex(), "a", "b")
            .addLayer("d", DenseLayer.Builder().nIn(3).nOut(4).activation(Activation.TANH).build(), "stack")
            .addVertex("u0", UnstackVertex(0, 2), "d")
            .addVertex("u1", UnstackVertex(1, 2), "d")
            .addVertex("l2", L2Vertex(), "u0", "u1")
            .addLayer("out", OutputLayer.Builder(LossFunction.MSE).nIn(1).nOut(1).activation(Activation.IDENTITY)
                      .build(), "l2")
            .setOutputs("out").build())
    net = ComputationGraph(conf)
    net.init(device=DEV)
    a, b = torch.randn(3, 3, dtype=torch.float64), torch.randn(3, 3, dtype=torch.float64)
    assert checkGradients(net, input=[a, b], labels=[torch.randn(3, 1, dtype=torch.float64)], print_results=True)


def test_fused_bn_add_relu_residual():
    """ResNet bottleneck tail: BN -> Add(shortcut) -> ReLU is planned into ONE fused BN kernel."""
    conf = (NeuralNetConfiguration.Builder().seed(3).dataType(DataType.DOUBLE).updater(NoOp())
            .weightInit(NormalDistribution(0, 0.5)).activation(Activation.IDENTITY)
            .convolutionMode(ConvolutionMode.Same).graphBuilder()
            .addInputs("in").setInputTypes(InputType.convolutional(4, 4, 3))
            .addLayer("c0", ConvolutionLayer.Builder([1, 1]).nOut(4).build(), "in")
            .addLayer("c1", ConvolutionLayer.Builder([3, 3]).nOut(4).build(), "c0")
            .addLayer("bn1", BatchNormalization(), "c1")
            .addVertex("add", ElementWiseVertex(ElementWiseVertex.Op.Add), "bn1", "c0")
            .addLayer("relu", ActivationLayer(Activation.RELU), "add")
            .addLayer("out", OutputLayer.Builder(LossFunction.MSE).nOut(2).activation(Activation.IDENTITY).build(),
                      "relu")
            .setOutputs("out").build())
    net = ComputationGraph(conf)
    net.init(device=DEV)
    assert net._residual_of == {"bn1": "c0"}
    assert net._passthrough == {"add": "bn1", "relu": "add"}
    x = torch.randn(3, 3, 4, 4, dtype=torch.float64)
    y = torch.randn(3, 2, dtype=torch.float64)
    assert checkGradients(net, input=[x], labels=[y], print_results=True, minAbsoluteError=1e-7)


def test_fused_bn_relu_maxpool_stem():
    """ResNet stem tail: BN -> ReLU -> MaxPool(3x3/2) is planned into the BN layer (pool + relu passthroughs)."""
    conf = (NeuralNetConfiguration.Builder().seed(3).dataType(DataType.DOUBLE).updater(NoOp())
            .weightInit(NormalDistribution(0, 0.5)).activation(Activation.IDENTITY).graphBuilder()
            .addInputs("in").setInputTypes(InputType.convolutional(9, 9, 3))
            .addLayer("c1", ConvolutionLayer.Builder([3, 3]).nOut(4).build(), "in")
            .addLayer("bn1", BatchNormalization(), "c1")
            .addLayer("relu", ActivationLayer(Activation.RELU), "bn1")
            .addLayer("pool", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).build(), "relu")
            .addLayer("out", OutputLayer.Builder(LossFunction.MSE).nOut(2).activation(Activation.IDENTITY).build(),
                      "pool")
            .setOutputs("out").build())
    net = ComputationGraph(conf)
    net.init(device=DEV)
    assert net._passthrough == {"relu": "bn1", "pool": "relu"}
    assert net.layers_by_name["bn1"].fuse_pool is net.layers_by_name["pool"]
    x = torch.randn(3, 3, 9, 9, dtype=torch.float64)
    y = torch.randn(3, 2, dtype=torch.float64)
    assert checkGradients(net, input=[x], labels=[y], print_results=True, minAbsoluteError=1e-7)


def test_resnet_style_residual_graph():
    conf = (NeuralNetConfiguration.Builder().seed(1).dataType(DataType.DOUBLE).updater(NoOp())
            .weightInit(NormalDistribution(0, 0.5)).activation(Activation.IDENTITY)
            .convolutionMode(ConvolutionMode.Same).graphBuilder()
            .addInputs("in").setInputTypes(InputType.convolutional(4, 4, 3))
            .addLayer("c1", ConvolutionLayer.Builder([3, 3]).nOut(3).build(), "in")
            .addLayer("bn1", BatchNormalization(), "c1")
            .addLayer("a1", ActivationLayer(Activation.TANH), "bn1")
            .addVertex("add", ElementWiseVertex(ElementWiseVertex.Op.Add), "a1", "in")
            .addLayer("pool", SubsamplingLayer.Builder(PoolingType.MAX, [2, 2], [2, 2]).build(), "add")
            .addLayer("out", OutputLayer.Builder(LossFunction.NEGATIVELOGLIKELIHOOD).nOut(2)
                      .activation(Activation.SOFTMAX).build(), "pool")
            .setOutputs("out").build())
    net = ComputationGraph(conf)
    net.init(device=DEV)
    x = torch.randn(4, 3, 4, 4, dtype=torch.float64)
    assert checkGradients(net, input=[x], labels=[onehot(4, 2)], print_results=True)


_ = L
