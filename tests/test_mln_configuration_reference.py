"""MultiLayerConfiguration JSON / YAML / clone / validation, after the reference's
MultiLayerNeuralNetConfigurationTest (deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/
MultiLayerNeuralNetConfigurationTest.java:52-394): JSON and YAML round trips (also through a properties file),
convnet / upsampling / global-pooling configurations equal after fromJson, clones are equal but share no layer or
preprocessor objects, seeded initialisation is reproducible, listeners reach every layer whether set before or after
init, empty / gapped layer lists are rejected with IllegalStateException, list(layers...) equals the indexed form,
pretrain / backprop flags, and a global bias updater reaches every layer's "b" parameter. CPU."""
import pytest
import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.exceptions import IllegalStateException
from deeplearning4j_amd.optimize.listeners import ScoreIterationListener


def _dense_pp_conf():
    return (D.NeuralNetConfiguration.Builder().list()
            .layer(0, D.DenseLayer.Builder().dist(D.NormalDistribution(1, 1e-1)).build())
            .inputPreProcessor(0, D.CnnToFeedForwardPreProcessor()).build())


def _through_properties(text, tmp_path):
    """Store the string under key "json" in a java.util.Properties-style file (backslash escapes for \\, newline,
    tab, carriage return, '=' and ':') and read it back."""
    esc = {"\\": "\\\\", "\n": "\\n", "\t": "\\t", "\r": "\\r", "=": "\\=", ":": "\\:"}
    f = tmp_path / "props"
    f.write_text("#\njson=" + "".join(esc.get(ch, ch) for ch in text) + "\n")
    line = next(ln for ln in f.read_text().split("\n") if ln.startswith("json="))[5:]
    out, i = [], 0
    unesc = {"n": "\n", "t": "\t", "r": "\r"}
    while i < len(line):
        if line[i] == "\\" and i + 1 < len(line):
            out.append(unesc.get(line[i + 1], line[i + 1]))
            i += 2
        else:
            out.append(line[i])
            i += 1
    return "".join(out)


def test_json(tmp_path):
    conf = _dense_pp_conf()
    js = conf.toJson()
    assert D.MultiLayerConfiguration.fromJson(js).getConf(0) == conf.getConf(0)
    js2 = _through_properties(js, tmp_path)
    assert js2 == js
    assert D.MultiLayerConfiguration.fromJson(js2).getConf(0) == conf.getConf(0)


def test_yaml(tmp_path):
    conf = _dense_pp_conf()
    y = conf.toYaml()
    assert D.MultiLayerConfiguration.fromYaml(y).getConf(0) == conf.getConf(0)
    y2 = _through_properties(y, tmp_path)
    assert y2 == y
    assert D.MultiLayerConfiguration.fromYaml(y2).getConf(0) == conf.getConf(0)


def test_convnet_json():
    conf = (D.NeuralNetConfiguration.Builder().seed(123).l1(1e-1).l2(2e-4).weightNoise(D.DropConnect(0.5))
            .miniBatch(True).optimizationAlgo(D.OptimizationAlgorithm.CONJUGATE_GRADIENT).list()
            .layer(0, D.ConvolutionLayer.Builder(5, 5).nOut(5).dropOut(0.5).weightInit(D.WeightInit.XAVIER)
                   .activation(D.Activation.RELU).build())
            .layer(1, D.SubsamplingLayer.Builder(D.SubsamplingLayer.PoolingType.MAX, [2, 2]).build())
            .layer(2, D.ConvolutionLayer.Builder(3, 3).nOut(10).dropOut(0.5).weightInit(D.WeightInit.XAVIER)
                   .activation(D.Activation.RELU).build())
            .layer(3, D.SubsamplingLayer.Builder(D.SubsamplingLayer.PoolingType.MAX, [2, 2]).build())
            .layer(4, D.DenseLayer.Builder().nOut(100).activation(D.Activation.RELU).build())
            .layer(5, D.OutputLayer.Builder(D.LossFunction.NEGATIVELOGLIKELIHOOD).nOut(6)
                   .weightInit(D.WeightInit.XAVIER).activation(D.Activation.SOFTMAX).build())
            .backprop(True).pretrain(False).setInputType(D.InputType.convolutional(76, 76, 3)).build())
    assert D.MultiLayerConfiguration.fromJson(conf.toJson()) == conf


def test_upsampling_convnet_json():
    conf = (D.NeuralNetConfiguration.Builder().seed(123).l1(1e-1).l2(2e-4).dropOut(0.5).miniBatch(True)
            .optimizationAlgo(D.OptimizationAlgorithm.CONJUGATE_GRADIENT).list()
            .layer(D.ConvolutionLayer.Builder(5, 5).nOut(5).dropOut(0.5).weightInit(D.WeightInit.XAVIER)
                   .activation(D.Activation.RELU).build())
            .layer(D.Upsampling2D.Builder().size(2).build())
            .layer(2, D.ConvolutionLayer.Builder(3, 3).nOut(10).dropOut(0.5).weightInit(D.WeightInit.XAVIER)
                   .activation(D.Activation.RELU).build())
            .layer(D.Upsampling2D.Builder().size(2).build())
            .layer(4, D.DenseLayer.Builder().nOut(100).activation(D.Activation.RELU).build())
            .layer(5, D.OutputLayer.Builder(D.LossFunction.NEGATIVELOGLIKELIHOOD).nOut(6)
                   .weightInit(D.WeightInit.XAVIER).activation(D.Activation.SOFTMAX).build())
            .backprop(True).pretrain(False).setInputType(D.InputType.convolutional(76, 76, 3)).build())
    assert D.MultiLayerConfiguration.fromJson(conf.toJson()) == conf


def test_global_pooling_json():
    conf = (D.NeuralNetConfiguration.Builder().updater(D.NoOp()).weightInit(D.WeightInit.DISTRIBUTION)
            .dist(D.NormalDistribution(0, 1.0)).seed(12345).list()
            .layer(0, D.ConvolutionLayer.Builder().kernelSize(2, 2).stride(1, 1).nOut(5).build())
            .layer(1, D.GlobalPoolingLayer.Builder().poolingType(D.PoolingType.PNORM).pnorm(3).build())
            .layer(2, D.OutputLayer.Builder(D.LossFunction.MCXENT).activation(D.Activation.SOFTMAX).nOut(3).build())
            .pretrain(False).backprop(True).setInputType(D.InputType.convolutional(32, 32, 1)).build())
    assert conf.fromJson(conf.toJson()) == conf


def test_clone():
    conf = (D.NeuralNetConfiguration.Builder().list().layer(0, D.DenseLayer.Builder().build())
            .layer(1, D.OutputLayer.Builder().build()).inputPreProcessor(1, D.CnnToFeedForwardPreProcessor()).build())
    conf2 = conf.clone()
    assert conf == conf2 and conf is not conf2
    assert conf.getConfs() is not conf2.getConfs()
    for i in range(len(conf.getConfs())):
        assert conf.getConf(i) is not conf2.getConf(i)
    assert conf.getInputPreProcessors() is not conf2.getInputPreProcessors()
    for layer in conf.getInputPreProcessors():
        assert conf.getInputPreProcess(layer) is not conf2.getInputPreProcess(layer)


def _get_conf():
    return (D.NeuralNetConfiguration.Builder().seed(12345).list()
            .layer(0, D.DenseLayer.Builder().nIn(2).nOut(2).weightInit(D.WeightInit.DISTRIBUTION)
                   .dist(D.NormalDistribution(0, 1)).build())
            .layer(1, D.OutputLayer.Builder().nIn(2).nOut(1).weightInit(D.WeightInit.DISTRIBUTION)
                   .dist(D.NormalDistribution(0, 1)).build()).build())


def test_random_weight_init():
    m1 = D.MultiLayerNetwork(_get_conf())
    m1.init()
    torch.manual_seed(12345)
    m2 = D.MultiLayerNetwork(_get_conf())
    m2.init()
    assert torch.equal(m1.params(), m2.params())


def test_iteration_listener():
    m1 = D.MultiLayerNetwork(_get_conf())
    m1.init()
    m1.setListeners([ScoreIterationListener(1)])
    m2 = D.MultiLayerNetwork(_get_conf())
    m2.setListeners([ScoreIterationListener(1)])
    m2.init()
    for m in (m1, m2):
        for layer in m.getLayers():
            assert layer.getListeners() is not None and len(layer.getListeners()) == 1


@pytest.mark.parametrize("case", ["no layers", "missing layer 0", "gap at layer 1"])
def test_invalid_config(case):
    b = D.NeuralNetConfiguration.Builder().seed(12345).list()
    if case == "missing layer 0":
        b = b.layer(1, D.DenseLayer.Builder().nIn(3).nOut(4).build()).layer(2, D.OutputLayer.Builder().nIn(4).nOut(5)
                                                                             .build())
    elif case == "gap at layer 1":
        b = b.layer(0, D.DenseLayer.Builder().nIn(3).nOut(4).build()).layer(2, D.OutputLayer.Builder().nIn(4).nOut(5)
                                                                             .build())
    with pytest.raises(IllegalStateException):
        conf = b.pretrain(False).backprop(True).build()
        net = D.MultiLayerNetwork(conf)
        net.init()


def test_list_overloads():
    def indexed():
        return (D.NeuralNetConfiguration.Builder().seed(12345).list()
                .layer(0, D.DenseLayer.Builder().nIn(3).nOut(4).build())
                .layer(1, D.OutputLayer.Builder().nIn(4).nOut(5).build()).pretrain(False).backprop(True).build())
    conf, conf2 = indexed(), indexed()
    for c in (conf, conf2):
        D.MultiLayerNetwork(c).init()
    dl, ol = conf.getConf(0).getLayer(), conf.getConf(1).getLayer()
    assert (dl.getNIn(), dl.getNOut(), ol.getNIn(), ol.getNOut()) == (3, 4, 4, 5)
    conf3 = (D.NeuralNetConfiguration.Builder().seed(12345)
             .list(D.DenseLayer.Builder().nIn(3).nOut(4).build(), D.OutputLayer.Builder().nIn(4).nOut(5).build())
             .pretrain(False).backprop(True).build())
    D.MultiLayerNetwork(conf3).init()
    assert conf == conf2 and conf == conf3


def test_pretrain_backprop_flags():
    conf = (D.NeuralNetConfiguration.Builder().list().layer(0, D.DenseLayer.Builder().nIn(2).nOut(2).build())
            .layer(1, D.DenseLayer.Builder().nIn(2).nOut(2).build()).build())
    assert not conf.isPretrain() and conf.isBackprop()
    conf = (D.NeuralNetConfiguration.Builder().list().layer(0, D.DenseLayer.Builder().nIn(2).nOut(2).build())
            .layer(1, D.DenseLayer.Builder().nIn(2).nOut(2).build()).pretrain(True).backprop(False).build())
    assert conf.isPretrain() and not conf.isBackprop()


def test_bias_lr():
    conf = (D.NeuralNetConfiguration.Builder().seed(12345).updater(D.Adam(1e-2)).biasUpdater(D.Adam(0.5)).list()
            .layer(0, D.ConvolutionLayer.Builder(5, 5).nOut(5).weightInit(D.WeightInit.XAVIER)
                   .activation(D.Activation.RELU).build())
            .layer(1, D.DenseLayer.Builder().nOut(100).activation(D.Activation.RELU).build())
            .layer(2, D.DenseLayer.Builder().nOut(100).activation(D.Activation.RELU).build())
            .layer(3, D.OutputLayer.Builder(D.LossFunction.NEGATIVELOGLIKELIHOOD).nOut(10)
                   .weightInit(D.WeightInit.XAVIER).activation(D.Activation.SOFTMAX).build())
            .setInputType(D.InputType.convolutional(28, 28, 1)).build())
    for i in range(4):
        layer = conf.getConf(i).getLayer()
        assert abs(layer.getUpdaterByParam("b").getLearningRate() - 0.5) < 1e-6
        assert abs(layer.getUpdaterByParam("W").getLearningRate() - 1e-2) < 1e-6
