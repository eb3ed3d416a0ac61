"""CenterLossOutputLayer's lambda, after the reference's CenterLossOutputLayerTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/CenterLossOutputLayerTest.java:40-110): the same
graph with lambda 0.1 and 0.01 gives different scores; with the class centers still at zero the difference is exactly
(0.1 - 0.01) / 2 * mean ||h||^2 over the minibatch, h being the dense layer's activations. fp64, CPU."""
import random

import torch

import deeplearning4j_amd as D


def _graph(n_labels, lam):
    conf = (D.NeuralNetConfiguration.Builder().seed(12345).weightInit(D.WeightInit.DISTRIBUTION)
            .dist(D.NormalDistribution(0, 1)).updater(D.NoOp()).dataType(D.DataType.DOUBLE)
            .graphBuilder().addInputs("input1")
            .addLayer("l1", D.DenseLayer.Builder().nIn(4).nOut(5).activation(D.Activation.RELU).build(), "input1")
            .addLayer("lossLayer", D.CenterLossOutputLayer.Builder().lossFunction(D.LossFunction.MCXENT).nIn(5)
                      .nOut(n_labels).lambda_(lam).activation(D.Activation.SOFTMAX).build(), "l1")
            .setOutputs("lossLayer").build())
    g = D.ComputationGraph(conf)
    g.init()
    return g


def test_lambda_changes_score_by_the_center_term():
    x = torch.rand(150, 4, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    y = torch.zeros(150, 2, dtype=torch.float64)
    r = random.Random(12345)
    for i in range(150):
        y[i, r.randrange(2)] = 1
    scores, hs = [], []
    for lam in (0.1, 0.01):
        g = _graph(2, lam)
        g.setInput(0, x)
        g.setLabel(0, y)
        g.computeGradientAndScore()
        scores.append(float(g.score()))
        hs.append(g.feedForward([x], False)["l1"])
    assert scores[0] != scores[1]
    assert torch.equal(hs[0], hs[1])                   # same seed -> same dense layer
    term = float((hs[0] ** 2).sum(1).mean())
    assert abs((scores[0] - scores[1]) - (0.1 - 0.01) / 2 * term) < 1e-9
