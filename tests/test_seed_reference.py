"""Seeded AutoEncoder pretraining, after the reference's SeedTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/SeedTest.java:22-50): after one unsupervised pass
over the Iris features, reading the parameters and setting them back leaves the parameters and the pretrain score
unchanged. The reference instantiates the AutoEncoder over a bare params view; here it is the only layer of a
seeded network (MultiLayerNetwork.pretrainLayer is the reference's layer.fit). CPU."""
import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.datasets.fetchers import IrisDataSetIterator

from _ref_fixtures import path as _ref_path

IRIS = _ref_path("deeplearning4j-core/src/main/resources/iris.dat")


def test_auto_encoder_seed():
    data = IrisDataSetIterator(50, 50, path=IRIS).next()
    conf = (D.NeuralNetConfiguration.Builder().seed(123).list()
            .layer(0, D.AutoEncoder.Builder().nIn(4).nOut(3).corruptionLevel(0.0).activation(D.Activation.SIGMOID)
                   .build()).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    net.pretrainLayer(0, data.getFeatures())
    layer = net.getLayers()[0]
    x = data.getFeatures().to(net.params().dtype)
    score = layer.computePretrainGradientAndScore(x)
    params = net.params().clone()
    net.setParams(params)
    score2 = layer.computePretrainGradientAndScore(x)
    assert torch.equal(params, net.params())
    assert abs(score - score2) < 1e-4
