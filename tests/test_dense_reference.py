"""Dense layers, after the reference's DenseTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/feedforward/dense/DenseTest.java:35-130): a dense
layer's bias has one row of nOut values set by biasInit; two identically seeded Iris MLPs (Sgd, L1 0.3 + L2 1e-3)
trained over the same iterator end with identical parameters and F1, with backprop and with pretrain-only (which
leaves a network of dense layers untouched). CPU."""
import os

import pytest
import torch

import deeplearning4j_amd as D
from _ref_fixtures import path as _ref_path

IRIS = _ref_path("deeplearning4j-core/src/main/resources/iris.dat")


def test_dense_bias_init():
    net = D.MultiLayerNetwork(D.NeuralNetConfiguration.Builder().list()
                              .layer(0, D.DenseLayer.Builder().nIn(1).nOut(3).biasInit(1).build())
                              .layer(1, D.OutputLayer.Builder().nIn(3).nOut(2).build()).build())
    net.init()
    b = net.getLayer(0).getParam("b")
    assert b.reshape(-1).numel() == 3 and torch.allclose(b, torch.ones_like(b))


def _mln(backprop, pretrain):
    conf = (D.NeuralNetConfiguration.Builder().seed(6).updater(D.Sgd(1e-3)).l1(0.3).l2(1e-3).list()
            .layer(0, D.DenseLayer.Builder().nIn(4).nOut(3).activation(D.Activation.TANH)
                   .weightInit(D.WeightInit.XAVIER).build())
            .layer(1, D.DenseLayer.Builder().nIn(3).nOut(2).activation(D.Activation.TANH)
                   .weightInit(D.WeightInit.XAVIER).build())
            .layer(2, D.OutputLayer.Builder(D.LossFunction.MCXENT).weightInit(D.WeightInit.XAVIER).nIn(2).nOut(3)
                   .build())
            .backprop(backprop).pretrain(pretrain).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    return net


@pytest.mark.skipif(not os.path.exists(IRIS), reason="reference iris.dat not present")
@pytest.mark.parametrize("backprop,pretrain", [(True, False), (False, True)])
def test_identically_seeded_mlps_train_identically(backprop, pretrain):
    it = D.IrisDataSetIterator(150, 150, path=IRIS)
    m1, m2 = _mln(backprop, pretrain), _mln(backprop, pretrain)
    p0 = m1.params().clone()
    m1.fit(it)
    it.reset()
    m2.fit(it)
    it.reset()
    test = it.next()
    assert torch.equal(m1.params(), m2.params())
    if not backprop:
        assert torch.equal(m1.params(), p0)       # dense layers have nothing to pretrain
    e1, e2 = D.Evaluation(), D.Evaluation()
    e1.eval(test.getLabels(), m1.output(test.getFeatures()))
    e2.eval(test.getLabels(), m2.output(test.getFeatures()))
    assert abs(e1.f1() - e2.f1()) < 1e-4
