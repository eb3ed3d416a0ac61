"""Layer builders, after the reference's LayerBuilderTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/layers/LayerBuilderTest.java): every builder sets the
fields it names (activation, weight init, distribution, dropout, updater, gradient normalization, nIn / nOut, kernel /
stride / padding, pooling type, autoencoder corruption / sparsity, LSTM forget-gate bias, batch-norm gamma / beta /
decay / lockGammaBeta), and each layer survives the single-layer NeuralNetConfiguration round trips: in-process object
serialisation (pickle of the framework's own object, the reference's Java serialisation), JSON and YAML; a changed
dropout makes layers unequal (equality covers the base-class fields). CPU."""
import pickle
import random

import pytest

import deeplearning4j_amd as D
from deeplearning4j_amd.nn.conf.activations import ActivationSoftmax, ActivationTanH

NUM_IN, NUM_OUT = 10, 5
KERNEL, STRIDE, PADDING = [2, 2], [2, 2], [1, 1]


def check_serialization(layer):
    expected = D.NeuralNetConfiguration.Builder().layer(layer).build()
    actual = pickle.loads(pickle.dumps(expected))
    assert expected.getLayer() == actual.getLayer(), "unequal object serialisation"
    actual = D.NeuralNetConfiguration.fromJson(expected.toJson())
    assert expected.getLayer() == actual.getLayer(), "unequal JSON serialisation"
    actual = D.NeuralNetConfiguration.fromYaml(expected.toYaml())
    assert expected.getLayer() == actual.getLayer(), "unequal YAML serialisation"
    actual.getLayer().setIDropout(D.Dropout(random.uniform(0.01, 0.99)))
    assert expected.getLayer() != actual.getLayer(), "equality ignores the base-layer fields"


def test_layer():
    act, dist, upd = ActivationSoftmax(), D.NormalDistribution(1.0, 0.1), D.AdaGrad()
    layer = (D.DenseLayer.Builder().activation(act).weightInit(D.WeightInit.XAVIER).dist(dist).dropOut(0.1)
             .updater(upd).gradientNormalization(D.GradientNormalization.ClipL2PerParamType)
             .gradientNormalizationThreshold(8).build())
    check_serialization(layer)
    assert layer.getActivationFn() == act
    assert layer.getWeightInit() == D.WeightInit.XAVIER
    assert layer.getDist() == dist
    assert layer.getIDropout() == D.Dropout(0.1)
    assert layer.getIUpdater() == upd
    assert layer.getGradientNormalization() == D.GradientNormalization.ClipL2PerParamType
    assert layer.getGradientNormalizationThreshold() == 8


def test_feed_forward_layer():
    ff = D.DenseLayer.Builder().nIn(NUM_IN).nOut(NUM_OUT).build()
    check_serialization(ff)
    assert (ff.getNIn(), ff.getNOut()) == (NUM_IN, NUM_OUT)


def test_convolution_layer():
    conv = D.ConvolutionLayer.Builder(KERNEL, STRIDE, PADDING).build()
    check_serialization(conv)
    assert list(conv.getKernelSize()) == KERNEL
    assert list(conv.getStride()) == STRIDE
    assert list(conv.getPadding()) == PADDING


def test_subsampling_layer():
    s = D.SubsamplingLayer.Builder(D.PoolingType.MAX, STRIDE).kernelSize(KERNEL).padding(PADDING).build()
    check_serialization(s)
    assert list(s.getPadding()) == PADDING
    assert list(s.getKernelSize()) == KERNEL
    assert s.getPoolingType() == D.PoolingType.MAX
    assert list(s.getStride()) == STRIDE


@pytest.mark.parametrize("cls", ["OutputLayer", "RnnOutputLayer"])
def test_output_layers(cls):
    check_serialization(getattr(D, cls).Builder(D.LossFunction.MCXENT).build())


def test_auto_encoder():
    enc = D.AutoEncoder.Builder().corruptionLevel(0.5).sparsity(0.3).build()
    check_serialization(enc)
    assert enc.getCorruptionLevel() == 0.5
    assert enc.getSparsity() == 0.3


@pytest.mark.parametrize("cls", ["GravesLSTM", "GravesBidirectionalLSTM"])
def test_graves_lstm(cls):
    g = getattr(D, cls).Builder().forgetGateBiasInit(1.5).activation(D.Activation.TANH).nIn(NUM_IN) \
        .nOut(NUM_OUT).build()
    check_serialization(g)
    assert g.getForgetGateBiasInit() == 1.5
    assert (g.nIn, g.nOut) == (NUM_IN, NUM_OUT)
    assert isinstance(g.getActivationFn(), ActivationTanH)


def test_embedding_layer():
    el = D.EmbeddingLayer.Builder().nIn(10).nOut(5).build()
    check_serialization(el)
    assert (el.getNIn(), el.getNOut()) == (10, 5)


def test_batch_norm_layer():
    bn = D.BatchNormalization.Builder().nIn(NUM_IN).nOut(NUM_OUT).gamma(2).beta(1).decay(0.5).lockGammaBeta(True) \
        .build()
    check_serialization(bn)
    assert (bn.nIn, bn.nOut) == (NUM_IN, NUM_OUT)
    assert bn.isLockGammaBeta() is True
    assert abs(bn.decay - 0.5) < 1e-4 and abs(bn.gamma - 2) < 1e-4 and abs(bn.beta - 1) < 1e-4


def test_activation_layer():
    act = ActivationSoftmax()
    al = D.ActivationLayer.Builder().activation(act).build()
    check_serialization(al)
    assert al.activation == act
