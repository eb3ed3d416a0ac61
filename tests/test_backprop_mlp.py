"""Hand-derived backpropagation vs the network, after the reference's BackPropMLPTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/multilayer/BackPropMLPTest.java:77-330): for sigmoid / tanh
MLPs with a softmax + MCXENT output on Iris minibatches, the forward pass, the deltas (out - labels, then
W^T delta * sigma'(z)) and the resulting dL/dW = a_prev^T delta, dL/db = sum(delta) are computed by hand in fp64 and
compared with the network's (raw, not yet minibatch-divided) gradient; and one SGD step on a single example moves
every parameter by -lr * dL/dparam."""
import os

import pytest
import torch

import deeplearning4j_amd as D
from _ref_fixtures import path as _ref_path

IRIS = _ref_path("deeplearning4j-core/src/main/resources/iris.dat")
pytestmark = pytest.mark.skipif(not os.path.exists(IRIS), reason="reference iris.dat not present")


def _net(hidden, act, lr=0.1):
    lb = D.NeuralNetConfiguration.Builder().updater(D.Sgd(lr)).seed(12345).dataType(D.DataType.DOUBLE).list()
    for i, n in enumerate(hidden):
        lb = lb.layer(i, D.DenseLayer.Builder().nIn(4 if i == 0 else hidden[i - 1]).nOut(n)
                      .weightInit(D.WeightInit.XAVIER).activation(act).build())
    lb = lb.layer(len(hidden), D.OutputLayer.Builder(D.LossFunction.MCXENT).nIn(hidden[-1]).nOut(3)
                  .weightInit(D.WeightInit.XAVIER).activation(D.Activation.SOFTMAX).build())
    net = D.MultiLayerNetwork(lb.build())
    net.init()
    return net


def _hand_gradients(net, x, y, act):
    L = len(net.getLayers())
    Ws = [net.getLayer(i).paramTable()["W"].detach().double() for i in range(L)]
    bs = [net.getLayer(i).paramTable()["b"].detach().double().reshape(1, -1) for i in range(L)]
    f = torch.sigmoid if act == D.Activation.SIGMOID else torch.tanh

    def fprime(z):
        return torch.sigmoid(z) * (1 - torch.sigmoid(z)) if act == D.Activation.SIGMOID else 1 - torch.tanh(z) ** 2
    zs, acts = [], []
    for i in range(L):
        a_in = x if i == 0 else acts[-1]
        z = a_in @ Ws[i] + bs[i]
        zs.append(z)
        acts.append(torch.softmax(z, 1) if i == L - 1 else f(z))
    deltas = [None] * L
    deltas[-1] = acts[-1] - y
    for i in range(L - 2, -1, -1):
        deltas[i] = (deltas[i + 1] @ Ws[i + 1].t()) * fprime(zs[i])
    dW = [(x if i == 0 else acts[i - 1]).t() @ deltas[i] for i in range(L)]
    db = [deltas[i].sum(0, keepdim=True) for i in range(L)]
    return dW, db


@pytest.mark.parametrize("mb,hidden,act", [(1, [1], D.Activation.SIGMOID), (1, [5], D.Activation.SIGMOID),
                                           (12, [15, 25, 10], D.Activation.SIGMOID),
                                           (50, [10, 50, 200, 50, 10], D.Activation.TANH),
                                           (150, [30, 50, 20], D.Activation.TANH)])
def test_network_gradient_matches_hand_backprop(mb, hidden, act):
    total = min(10 * mb, mb * (150 // mb))
    it = D.IrisDataSetIterator(mb, total, path=IRIS)
    net = _net(hidden, act)
    while it.hasNext():
        ds = it.next()
        x, y = ds.getFeatures().double(), ds.getLabels().double()
        dW, db = _hand_gradients(net, x, y, act)
        net.setInput(x)
        net.setLabels(y)
        net.computeGradientAndScore()
        g = net.gradient()
        for i in range(len(hidden) + 1):
            gw = g.getGradientFor(f"{i}_W").double()
            gb = g.getGradientFor(f"{i}_b").double().reshape(1, -1)
            # raw sums over the minibatch, as in the reference (the division happens in the updater)
            assert torch.allclose(gw, dW[i], atol=1e-8), (mb, hidden, i)
            assert torch.allclose(gb, db[i], atol=1e-8), (mb, hidden, i)


def test_single_example_sgd_step():
    """testSingleExampleWeightUpdates: 4-1-3 sigmoid MLP, one Iris example, Sgd(0.1): every parameter moves by
    -0.1 * dL/dparam of the hand-derived backward pass."""
    it = D.IrisDataSetIterator(1, 10, path=IRIS)
    net = _net([1], D.Activation.SIGMOID)
    while it.hasNext():
        ds = it.next()
        x, y = ds.getFeatures().double(), ds.getLabels().double()
        before = {k: v.detach().clone() for k, v in net.paramTable().items()}
        dW, db = _hand_gradients(net, x, y, D.Activation.SIGMOID)
        net.fit(ds)
        after = net.paramTable()
        for i in range(2):
            assert torch.allclose(after[f"{i}_W"].double(), before[f"{i}_W"].double() - 0.1 * dW[i], atol=1e-10)
            assert torch.allclose(after[f"{i}_b"].double().reshape(1, -1),
                                  before[f"{i}_b"].double().reshape(1, -1) - 0.1 * db[i], atol=1e-10)
