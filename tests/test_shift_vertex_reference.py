"""ShiftVertex, after the reference's ShiftVertexTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/graph/ShiftVertexTest.java:33-229): the vertex has no
parameters; it adds its shift factor to its input (first primes / 10 through identity activation layers); and in
tanh dense -> shift -> sigmoid MSE output the score and every parameter gradient equal the reference's hand-written
chain rule (MSE divided by nOut, raw per-minibatch gradient sums). fp64, CPU."""
import torch

import deeplearning4j_amd as D

INPUT = [[0.2, 0.3, 0.5], [0.7, 1.1, 1.3], [1.7, 1.9, 2.3], [2.9, 3.1, 3.7]]
TARGET = [[0.05, 0.10, 0.15, 0.20, 0.25], [0.30, 0.35, 0.40, 0.45, 0.50], [0.55, 0.60, 0.65, 0.70, 0.75],
          [0.80, 0.85, 0.90, 0.95, 0.99]]
EPS = 1e-10


def test_shift_vertex_num_params():
    sv = D.ShiftVertex(0.7)
    assert sv.numParams(True) == 0
    assert sv.numParams(False) == 0


def test_shift_vertex_get():
    assert abs(D.ShiftVertex(0.7).getShiftFactor() - 0.7) < EPS


def test_shift_vertex_simple():
    x = torch.tensor(INPUT, dtype=torch.float64)
    sf = 4.1
    cgc = (D.NeuralNetConfiguration.Builder().dataType(D.DataType.DOUBLE).graphBuilder().addInputs("input")
           .addLayer("denselayer", D.DenseLayer.Builder().nIn(3).nOut(1).activation(D.Activation.IDENTITY).build(),
                     "input")
           .addLayer("identityinputactivation", D.ActivationLayer.Builder().activation(D.Activation.IDENTITY).build(),
                     "input")
           .addVertex("shiftvertex", D.ShiftVertex(sf), "identityinputactivation")
           .addLayer("identityshiftvertex", D.ActivationLayer.Builder().activation(D.Activation.IDENTITY).build(),
                     "shiftvertex")
           .setOutputs("identityshiftvertex", "denselayer").build())
    cg = D.ComputationGraph(cgc)
    cg.init()
    out = cg.output(True, x)[0]
    assert float(((out.double() - (x + sf)) ** 2).sum()) < EPS


def test_shift_vertex_comprehensive():
    x = torch.tensor(INPUT, dtype=torch.float64)
    t = torch.tensor(TARGET, dtype=torch.float64)
    sf = 4.1
    cgc = (D.NeuralNetConfiguration.Builder().dataType(D.DataType.DOUBLE).weightInit(D.WeightInit.XAVIER)
           .updater(D.Sgd(0.01)).optimizationAlgo(D.OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT)
           .graphBuilder().addInputs("input")
           .addLayer("denselayer", D.DenseLayer.Builder().nIn(3).nOut(3).activation(D.Activation.TANH).build(),
                     "input")
           .addVertex("shiftvertex", D.ShiftVertex(sf), "denselayer")
           .addLayer("output", D.OutputLayer.Builder().nIn(3).nOut(5).activation(D.Activation.SIGMOID)
                     .lossFunction(D.LossFunction.MSE).build(), "shiftvertex")
           .setOutputs("output").build())
    cg = D.ComputationGraph(cgc)
    cg.init()
    cg.setInput(0, x)
    cg.setLabel(0, t)
    cg.computeGradientAndScore()
    score_dl4j = cg.score()
    w = cg.paramTable()
    W, b = w["denselayer_W"].double(), w["denselayer_b"].double().reshape(1, -1)
    V, c = w["output_W"].double(), w["output_b"].double().reshape(1, -1)
    # the reference's manual chain rule
    z = x @ W + b
    a = torch.tanh(z) + sf
    q = a @ V + c
    o = torch.sigmoid(q)
    score_manual = float(((o - t) ** 2).sum()) / (o.shape[0] * o.shape[1])
    dEdo = 2 * (o - t) / t.shape[1]
    dEdq = dEdo * o * (1 - o)
    manual = {"output_b": dEdq.sum(0, keepdim=True), "output_W": a.t() @ dEdq}
    dEdz = (dEdq @ V.t()) * (1 - torch.tanh(z) ** 2)
    manual["denselayer_b"] = dEdz.sum(0, keepdim=True)
    manual["denselayer_W"] = x.t() @ dEdz
    grads = cg.gradient().gradientForVariable()
    summse = (score_manual - score_dl4j) ** 2
    denom = 1
    for name, g in grads.items():
        m = manual[name]
        g = g.double().reshape(m.shape)
        summse += float(((g - m) ** 2).sum())
        denom += m.numel()
    assert summse / denom < EPS
