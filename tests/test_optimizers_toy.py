"""Optimizers on non-network cost functions, after the reference's TestOptimizers
(deeplearning4j-core/src/test/java/org/deeplearning4j/optimize/solver/TestOptimizers.java:134-700): the sphere
function (convex, minimum 0 at x = 0), the Rastrigin function (many local minima, +inf outside [-5.12, 5.12]) and
the Rosenbrock valley (minimum 0 at x = 1, +inf outside [-5, 5]), each driven through optimize/solvers.py exactly as
a network is: ``computeGradientAndScore`` -> the configured updater turns the raw gradient into the search direction
-> backtracking line search -> step. Plus the reference's Iris MLP check that every algorithm's score never rises
over 30 x 10 full-batch fits.

The reference's SimpleOptimizableModel is replaced by ``FunctionModel``, which implements the slice of the network
interface the solvers use (flattened params / gradients, updater, score, iteration hooks)."""
import math
import os
from types import SimpleNamespace

import pytest
import torch

from deeplearning4j_amd.optimize.solvers import (ConjugateGradient, LBFGS, LineGradientDescent,
                                                 NegativeDefaultStepFunction, StochasticGradientDescent)
from _ref_fixtures import path as _ref_path

ALGOS = {"sgd": StochasticGradientDescent, "line": LineGradientDescent, "cg": ConjugateGradient, "lbfgs": LBFGS}


class _Updater:
    """Sgd(lr): g <- lr*g; AdaGrad(lr): h += g^2, g <- lr*g/(sqrt(h)+eps) (the update direction, params untouched)."""

    def __init__(self, kind, lr, n):
        self.kind, self.lr = kind, lr
        self.h = torch.zeros(n, dtype=torch.float64)

    def update(self, params, grad, iteration, epoch, batch, _):
        if self.kind == "adagrad":
            self.h.add_(grad * grad)
            grad.mul_(self.lr / (self.h.sqrt() + 1e-6))
        else:
            grad.mul_(self.lr)


class FunctionModel:
    def __init__(self, x0, updater="sgd", lr=1e-2, max_ls=5):
        self.flattenedParams = x0.clone().double()
        self.flattenedGradients = torch.zeros_like(self.flattenedParams)
        self.conf = SimpleNamespace(globalConf={"maxNumLineSearchIterations": max_ls}, iterationCount=0,
                                    epochCount=0)
        self.listeners = []
        self.updater = _Updater(updater, lr, self.flattenedParams.numel())
        self._score = float("nan")

    # cost and gradient of the function at x
    def f(self, x):
        raise NotImplementedError

    def grad(self, x):
        raise NotImplementedError

    def computeGradientAndScore(self, x=None, y=None, fm=None, lm=None):
        p = self.flattenedParams
        self._score = float(self.f(p))
        self.flattenedGradients.copy_(self.grad(p))

    def score(self):
        return self._score

    def _score_batch(self, x, y, fm, lm):
        return float(self.f(self.flattenedParams))

    def _params_changed(self):
        pass

    def _iteration_done(self):
        self.conf.iterationCount += 1

    def _fit_batch_sgd(self, x, y, fm, lm):
        self.computeGradientAndScore()
        g = self.flattenedGradients
        self.updater.update(self.flattenedParams, g, self.conf.iterationCount, 0, 1, None)
        NegativeDefaultStepFunction().step(self.flattenedParams, g)
        self._iteration_done()


class Sphere(FunctionModel):
    def f(self, x):
        return float((x * x).sum())

    def grad(self, x):
        return 2 * x


class Rastrigin(FunctionModel):
    def f(self, x):
        if bool((x.abs() > 5.12).any()):
            return math.inf
        return float(10 * x.numel() + (x * x).sum() - 10 * torch.cos(2 * math.pi * x).sum())

    def grad(self, x):
        return 2 * x + 20 * math.pi * torch.sin(2 * math.pi * x)


class Rosenbrock(FunctionModel):
    def f(self, x):
        if bool((x.abs() > 5.0).any()):
            return math.inf
        return float((100 * (x[1:] - x[:-1] ** 2) ** 2 + (x[:-1] - 1) ** 2).sum())

    def grad(self, x):
        g = torch.zeros_like(x)
        t = x[1:] - x[:-1] ** 2
        g[:-1] += -400 * x[:-1] * t + 2 * (x[:-1] - 1)
        g[1:] += 200 * t
        return g


def _uniform(n, lo, hi, seed=12345):
    gen = torch.Generator().manual_seed(seed)
    return torch.rand(n, generator=gen, dtype=torch.float64) * (hi - lo) + lo


def _run(model, algo, calls):
    opt = ALGOS[algo](model)
    for _ in range(calls):
        opt.optimize(None, None)
    model.computeGradientAndScore()
    return model.score()


@pytest.mark.parametrize("algo", ["sgd", "line", "cg", "lbfgs"])
@pytest.mark.parametrize("n_ls", [1, 5])
@pytest.mark.parametrize("dims", [2, 10, 100])
def test_sphere_improves(algo, n_ls, dims):
    """testSphereFnOpt*: 100 optimizer calls from U(-10, 10) with Sgd(1e-2) lower the score."""
    m = Sphere(_uniform(dims, -10, 10), "sgd", 1e-2, n_ls)
    m.computeGradientAndScore()
    before = m.score()
    assert math.isfinite(before)
    after = _run(m, algo, 100)
    assert math.isfinite(after) and after < before, (algo, n_ls, dims, before, after)


@pytest.mark.parametrize("algo", ["sgd", "line", "cg", "lbfgs"])
def test_sphere_multiple_steps_reaches_minimum(algo):
    """testSphereFn*MultipleSteps: 100-dimensional sphere, Sgd(0.1), 5 line-search iterations, 100 calls — the score
    ends near the minimum (< 1) and identical repeated runs give identical scores (deterministic solvers)."""
    scores = []
    for _ in range(3):
        m = Sphere(_uniform(100, -10, 10), "sgd", 0.1, 5)
        scores.append(_run(m, algo, 100))
    assert scores[0] == scores[1] == scores[2]
    assert scores[-1] < 1.0, (algo, scores)


@pytest.mark.parametrize("algo,calls,n_ls", [("sgd", 5, 20), ("line", 10, 20), ("cg", 10, 20), ("lbfgs", 10, 20)])
def test_rastrigin_never_worsens(algo, calls, n_ls):
    """testRastriginFn*MultipleSteps: AdaGrad(1e-2), 10 dimensions in U(-5.12, 5.12); one optimizer call per fresh
    model, repeated — the score after is never above the score before, and stays finite (the line search rejects
    steps that leave the box, where the cost is +inf)."""
    m0 = Rastrigin(_uniform(10, -5.12, 5.12), "adagrad", 1e-2, n_ls)
    m0.computeGradientAndScore()
    prev = m0.score()
    m = Rastrigin(_uniform(10, -5.12, 5.12), "adagrad", 1e-2, n_ls)
    opt = ALGOS[algo](m)
    for _ in range(calls):
        opt.optimize(None, None)
        m.computeGradientAndScore()
        s = m.score()
        assert math.isfinite(s)
        assert s <= prev + 1e-9, (algo, prev, s)
        prev = s


@pytest.mark.parametrize("algo", ["line", "cg", "lbfgs"])
def test_rosenbrock_descends(algo):
    """testRosenbrockFn*MultipleSteps: 100 dimensions in U(-4, 4), Sgd(0.1), 20 line-search iterations: the first
    call strictly improves and no later call makes the score worse."""
    m = Rosenbrock(_uniform(100, -4.0, 4.0), "sgd", 0.1, 20)
    m.computeGradientAndScore()
    prev = m.score()
    opt = ALGOS[algo](m)
    for i in range(20):
        opt.optimize(None, None)
        m.computeGradientAndScore()
        s = m.score()
        assert math.isfinite(s), (algo, i, s)
        if i == 0:
            assert s < prev, (algo, prev, s)
        else:
            assert s <= prev, (algo, i, prev, s)
        prev = s


def test_rosenbrock_gradient_is_exact():
    """The analytic Rosenbrock / Rastrigin gradients used above agree with autograd (guards the fixtures)."""
    x = _uniform(7, -2, 2).requires_grad_(True)
    f = (100 * (x[1:] - x[:-1] ** 2) ** 2 + (x[:-1] - 1) ** 2).sum()
    f.backward()
    assert torch.allclose(Rosenbrock(x.detach()).grad(x.detach()), x.grad)
    x2 = _uniform(7, -5, 5).requires_grad_(True)
    f2 = 10 * 7 + (x2 * x2).sum() - 10 * torch.cos(2 * math.pi * x2).sum()
    f2.backward()
    assert torch.allclose(Rastrigin(x2.detach()).grad(x2.detach()), x2.grad)


IRIS = _ref_path("deeplearning4j-core/src/main/resources/iris.dat")


@pytest.mark.skipif(not os.path.exists(IRIS), reason="reference iris.dat not present")
@pytest.mark.parametrize("algo_name", ["STOCHASTIC_GRADIENT_DESCENT", "LINE_GRADIENT_DESCENT", "CONJUGATE_GRADIENT",
                                       "LBFGS"])
def test_iris_mlp_score_never_rises(algo_name):
    """testOptimizersMLP: Iris (150, normalised), 4-3-3 ReLU/softmax MLP with AdaGrad(0.1) and XAVIER init; 30 rounds
    of 10 full-batch fits — the score never goes up between rounds."""
    import deeplearning4j_amd as D
    ds = D.IrisDataSetIterator(150, 150, path=IRIS).next()
    ds.normalizeZeroMeanZeroUnitVariance()
    conf = (D.NeuralNetConfiguration.Builder().optimizationAlgo(getattr(D.OptimizationAlgorithm, algo_name))
            .updater(D.AdaGrad(0.1)).seed(12345).list()
            .layer(0, D.DenseLayer.Builder().nIn(4).nOut(3).weightInit(D.WeightInit.XAVIER)
                   .activation(D.Activation.RELU).build())
            .layer(1, D.OutputLayer.Builder(D.LossFunction.MCXENT).nIn(3).nOut(3).weightInit(D.WeightInit.XAVIER)
                   .activation(D.Activation.SOFTMAX).build())
            .build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    score = net.score(ds)
    assert score != 0.0 and math.isfinite(score)
    for _ in range(30):
        for _ in range(10):
            net.fit(ds)
        after = net.score(ds)
        assert math.isfinite(after)
        assert after <= score + 1e-6, (algo_name, score, after)
        score = after
