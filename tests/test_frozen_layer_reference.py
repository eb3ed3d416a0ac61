"""Frozen layers, after the reference's FrozenLayerTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/FrozenLayerTest.java:37-360): a network whose first
two layers are frozen by TransferLearning.setFeatureExtractor trains exactly like a fresh network made of the unfrozen
tail fed the frozen features (MultiLayerNetwork and ComputationGraph, and their clones); FrozenLayer-wrapped layers
initialise to the same parameters as the unwrapped ones and survive a JSON round trip. fp64, CPU."""
import torch

import deeplearning4j_amd as D


def _data():
    g = torch.Generator().manual_seed(12345)
    return D.DataSet(torch.rand(10, 4, generator=g, dtype=torch.float64),
                     torch.rand(10, 3, generator=g, dtype=torch.float64))


def _overall():
    return (D.NeuralNetConfiguration.Builder().updater(D.Sgd(0.1)).activation(D.Activation.IDENTITY)
            .dataType(D.DataType.DOUBLE))


def _softmax_out(nIn):
    return D.OutputLayer.Builder(D.LossFunction.MCXENT).activation(D.Activation.SOFTMAX).nIn(nIn).nOut(3).build()


def _mln_to_tune():
    net = D.MultiLayerNetwork(_overall().list()
                              .layer(0, D.DenseLayer.Builder().nIn(4).nOut(3).build())
                              .layer(1, D.DenseLayer.Builder().nIn(3).nOut(2).build())
                              .layer(2, D.DenseLayer.Builder().nIn(2).nOut(3).build())
                              .layer(3, _softmax_out(3)).build())
    net.init()
    return net


def _mln_tail(params):
    net = D.MultiLayerNetwork(_overall().list().layer(0, D.DenseLayer.Builder().nIn(2).nOut(3).build())
                              .layer(1, _softmax_out(3)).build())
    net.init(params.clone())
    return net


def _split(net, n_head):
    """(flat params of the first n_head layers, flat params of the rest), cut from the network's flat vector."""
    layers = net.getLayers()
    k = sum(l.numParams() for l in layers[:n_head])
    p = net.params().reshape(-1)
    return p[:k].clone(), p[k:].clone()


def test_frozen_mln_and_clone_match_unfrozen_tail():
    ds = _data()
    base = _mln_to_tune()
    frozen_feats = base.feedForwardToLayer(2, ds.getFeatures(), False)[2]
    now = (D.TransferLearning.Builder(base).fineTuneConfiguration(D.FineTuneConfiguration.Builder()
                                                                  .updater(D.Sgd(0.1)).build())
           .setFeatureExtractor(1).build())
    cloned = now.clone()
    assert torch.equal(now.params(), cloned.params())
    head, rest = _split(base, 2)
    tail = _mln_tail(rest)
    assert torch.allclose(now.output(ds.getFeatures()), tail.output(frozen_feats), atol=1e-14)
    for _ in range(5):
        tail.fit(D.DataSet(frozen_feats, ds.getLabels()))
        now.fit(ds)
        cloned.fit(ds)
    expected = torch.cat([head, tail.params().reshape(-1)])
    assert torch.allclose(now.params().reshape(-1), expected, atol=1e-14)
    assert torch.allclose(cloned.params().reshape(-1), expected, atol=1e-14)


def _cg_to_tune():
    g = D.ComputationGraph(_overall().graphBuilder().addInputs("layer0In")
                           .addLayer("layer0", D.DenseLayer.Builder().nIn(4).nOut(3).build(), "layer0In")
                           .addLayer("layer1", D.DenseLayer.Builder().nIn(3).nOut(2).build(), "layer0")
                           .addLayer("layer2", D.DenseLayer.Builder().nIn(2).nOut(3).build(), "layer1")
                           .addLayer("layer3", _softmax_out(3), "layer2").setOutputs("layer3").build())
    g.init()
    return g


def test_frozen_cg_and_clone_match_unfrozen_tail():
    ds = _data()
    base = _cg_to_tune()
    frozen_feats = base.feedForward([ds.getFeatures()], False)["layer1"]
    now = D.TransferLearning.GraphBuilder(base).setFeatureExtractor("layer1").build()
    cloned = now.clone()
    assert torch.equal(now.params(), cloned.params())
    tail = D.ComputationGraph(_overall().graphBuilder().addInputs("layer0In")
                              .addLayer("layer0", D.DenseLayer.Builder().nIn(2).nOut(3).build(), "layer0In")
                              .addLayer("layer1", _softmax_out(3), "layer0").setOutputs("layer1").build())
    tail.init()
    head, rest = _split(base, 2)
    tail.setParams(rest)
    for _ in range(5):
        tail.fit(D.DataSet(frozen_feats, ds.getLabels()))
        now.fit(ds)
        cloned.fit(ds)
    expected = torch.cat([head, tail.params().reshape(-1)])
    assert torch.allclose(now.params().reshape(-1), expected, atol=1e-14)
    assert torch.allclose(cloned.params().reshape(-1), expected, atol=1e-14)


def _dense10():
    return D.DenseLayer.Builder().nIn(10).nOut(10).activation(D.Activation.TANH).weightInit(D.WeightInit.XAVIER).build()


def _out10():
    return D.OutputLayer.Builder(D.LossFunction.MCXENT).activation(D.Activation.SOFTMAX).nIn(10).nOut(10).build()


def test_frozen_layer_instantiation_mln():
    c1 = D.NeuralNetConfiguration.Builder().seed(12345).list().layer(0, _dense10()).layer(1, _dense10()) \
        .layer(2, _out10()).build()
    c2 = D.NeuralNetConfiguration.Builder().seed(12345).list().layer(0, D.FrozenLayer(_dense10())) \
        .layer(1, D.FrozenLayer(_dense10())).layer(2, _out10()).build()
    n1, n2 = D.MultiLayerNetwork(c1), D.MultiLayerNetwork(c2)
    n1.init()
    n2.init()
    assert torch.equal(n1.params(), n2.params())
    c3 = D.MultiLayerConfiguration.fromJson(c2.toJson())
    assert c3.toJson() == c2.toJson()
    n3 = D.MultiLayerNetwork(c3)
    n3.init()
    x = torch.rand(10, 10, generator=torch.Generator().manual_seed(1))
    assert torch.equal(n2.output(x), n3.output(x))


def test_frozen_layer_instantiation_cg():
    c1 = (D.NeuralNetConfiguration.Builder().seed(12345).graphBuilder().addInputs("in")
          .addLayer("0", _dense10(), "in").addLayer("1", _dense10(), "0").addLayer("2", _out10(), "1")
          .setOutputs("2").build())
    c2 = (D.NeuralNetConfiguration.Builder().seed(12345).graphBuilder().addInputs("in")
          .addLayer("0", D.FrozenLayer.Builder().layer(_dense10()).build(), "in")
          .addLayer("1", D.FrozenLayer.Builder().layer(_dense10()).build(), "0")
          .addLayer("2", _out10(), "1").setOutputs("2").build())
    n1, n2 = D.ComputationGraph(c1), D.ComputationGraph(c2)
    n1.init()
    n2.init()
    assert torch.equal(n1.params(), n2.params())
    c3 = D.ComputationGraphConfiguration.fromJson(c2.toJson())
    assert c3.toJson() == c2.toJson()
    n3 = D.ComputationGraph(c3)
    n3.init()
    x = torch.rand(10, 10, generator=torch.Generator().manual_seed(1))
    assert torch.equal(n2.outputSingle(x), n3.outputSingle(x))
