"""Backtracking line search, after the reference's BackTrackLineSearchTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/optimize/solver/BackTrackLineSearchTest.java:35-255): on a
softmax output layer over 5 normalised Iris examples, a minimising search along the gradient (default and
NegativeDefaultStepFunction) accepts the full step 1.0 and stepping by it lowers the score; a maximising search
(DefaultStepFunction, adds the direction) raises it; line gradient descent, conjugate gradient and L-BFGS networks
lower their score over a few fits; HESSIAN_FREE is refused. The single output layer is a one-layer
MultiLayerNetwork here (the reference drives the bare layer object). fp64, CPU."""
import pytest
import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.optimize.solvers import (BackTrackLineSearch, DefaultStepFunction,
                                                 NegativeDefaultStepFunction)

from _ref_fixtures import path as _ref_path

IRIS = _ref_path("deeplearning4j-core/src/main/resources/iris.dat")

LF = D.LossFunctions.LossFunction
OA = D.OptimizationAlgorithm


def _iris(n):
    ds = D.IrisDataSetIterator(n, n, path=IRIS).next()
    ds.normalizeZeroMeanZeroUnitVariance()
    return ds


def _layer(loss, act=D.Activation.SOFTMAX, max_iter=100):
    conf = (D.NeuralNetConfiguration.Builder().seed(12345).miniBatch(True).maxNumLineSearchIterations(max_iter)
            .dataType(D.DataType.DOUBLE).list()
            .layer(D.OutputLayer.Builder(loss).nIn(4).nOut(3).activation(act).weightInit(D.WeightInit.XAVIER).build())
            .build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    return net


def _prepared(loss):
    data = _iris(5)
    net = _layer(loss)
    net.setInput(data.getFeatures().double())
    net.setLabels(data.getLabels().double())
    net.computeGradientAndScore()
    return net


def _grad(net):
    return net.gradient().gradient().reshape(-1)


@pytest.mark.parametrize("sf", [None, NegativeDefaultStepFunction()])
def test_single_min_line_search(sf):
    net = _prepared(LF.NEGATIVELOGLIKELIHOOD)
    ls = BackTrackLineSearch(net, sf) if sf is not None else BackTrackLineSearch(net)
    g = _grad(net).clone()
    step = ls.optimize(net.params().reshape(-1), g, g)
    assert abs(step - 1.0) < 1e-3


def test_mult_min_line_search():
    net = _prepared(LF.NEGATIVELOGLIKELIHOOD)
    s1 = net.score()
    g = _grad(net).clone()
    sf = NegativeDefaultStepFunction()
    step = BackTrackLineSearch(net, sf).optimize(net.params().reshape(-1), g, g)
    p = net.params().reshape(-1).clone()
    sf.step(p, g, step)
    net.setParams(p)
    net.computeGradientAndScore()
    assert s1 > net.score()


def test_mult_max_line_search():
    net = _prepared(LF.MCXENT)
    s1 = net.score()
    g = _grad(net).clone()
    sf = DefaultStepFunction()
    step = BackTrackLineSearch(net, sf).optimize(net.params().reshape(-1).clone(), g.clone(), g.clone())
    assert step > 0
    p = net.params().reshape(-1).clone()
    sf.step(p, g, step)
    net.setParams(p)
    net.computeGradientAndScore()
    assert s1 < net.score()


def _iris_net(act, algo):
    conf = (D.NeuralNetConfiguration.Builder().optimizationAlgo(algo).miniBatch(False).updater(D.Nesterovs(0.9))
            .seed(12345).dataType(D.DataType.DOUBLE).list()
            .layer(0, D.DenseLayer.Builder().nIn(4).nOut(100).weightInit(D.WeightInit.XAVIER).activation(act).build())
            .layer(1, D.OutputLayer.Builder(LF.MCXENT).nIn(100).nOut(3).weightInit(D.WeightInit.XAVIER)
                   .activation(D.Activation.SOFTMAX).build())
            .backprop(True).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    from deeplearning4j_amd.optimize.listeners import ScoreIterationListener
    net.setListeners(ScoreIterationListener(1))
    return net


@pytest.mark.parametrize("algo,act,n,fits", [(OA.LINE_GRADIENT_DESCENT, D.Activation.SIGMOID, 1, 100),
                                             (OA.CONJUGATE_GRADIENT, D.Activation.RELU, 5, 5),
                                             (OA.LBFGS, D.Activation.RELU, 5, 5)])
def test_backtrack_line_optimizers(algo, act, n, fits):
    data = _iris(n) if n > 1 else D.IrisDataSetIterator(1, 1, path=IRIS).next()
    x, y = data.getFeatures().double(), data.getLabels().double()
    net = _iris_net(act, algo)
    old = net.score(D.DataSet(x, y))
    for _ in range(fits):
        net.fit(x, y)
    assert net.score() < old


def test_hessian_free_refused():
    data = D.IrisDataSetIterator(5, 5, path=IRIS).next()
    from deeplearning4j_amd.exceptions import UnsupportedOperationException
    with pytest.raises(UnsupportedOperationException):
        net = _iris_net(D.Activation.RELU, OA.HESSIAN_FREE)
        for _ in range(3):
            net.fit(data.getFeatures().double(), data.getLabels().double())
