"""Evaluation scenarios of the reference's CORET:eval/EvalTest.java (testEval, testEval2, testStringListLabels,
testStringHashLabels, testEvalMasking, testFalsePerfectRecall, testEvaluationMerging, testSingleClassBinary-
Classification, testEvalInvalid, testEvalMethods, testTopNAccuracy(+Merging), testBinaryCase,
testF1FBeta_MicroMacroAveraging, testConfusionMatrixStats) with the reference's own numbers."""
import math
import random

import pytest
import torch

from deeplearning4j_amd.eval import Evaluation
from deeplearning4j_amd.eval.base import EvaluationAveraging


def _oh(i, n):
    v = torch.zeros(1, n)
    v[0, i] = 1
    return v


def test_eval_edge_cases():
    e = Evaluation(5)
    e.eval(_oh(0, 5), _oh(0, 5))
    assert e.classCount(0) == 1 and abs(e.f1() - 1.0) < 1e-1
    e.eval(_oh(1, 5), _oh(0, 5))
    assert abs(e.f1() - 0.6) < 1e-1                                  # sklearn classification_report (reference)
    assert e.classCount(0) == 1 and e.classCount(1) == 1
    assert e.positive()[0] == 1 and e.negative()[0] == 1
    assert e.truePositives()[0] == 1 and e.falsePositives()[0] == 1
    assert e.trueNegatives()[0] == 0 and e.falseNegatives()[0] == 0
    assert e.accuracy() == 0.5


def test_eval_confusion_counts():
    ev = Evaluation(["class0", "class1"])
    p0, p1 = torch.tensor([[1.0, 0]]), torch.tensor([[0.0, 1]])
    for lab, pred, n in ((p0, p0, 20), (p0, p1, 3), (p1, p0, 10), (p1, p1, 5)):
        for _ in range(n):
            ev.eval(lab, pred)
    assert (ev.truePositives()[0], ev.falseNegatives()[0], ev.falsePositives()[0], ev.trueNegatives()[0]) == \
        (20, 3, 10, 5)
    assert abs(ev.accuracy() - 25 / 38) < 1e-6
    assert "class0" in ev.confusionToString()


@pytest.mark.parametrize("labels", [["hobbs", "cal"], {0: "hobbs", 1: "cal"}])
def test_string_labels(labels):
    e = Evaluation(labels)
    e.eval(_oh(0, 2), _oh(0, 2))
    assert e.classCount(0) == 1 and e.getClassLabel(0) == "hobbs"


def test_eval_masking_time_series():
    mb, n, T = 5, 3, 6
    g = torch.Generator().manual_seed(12345)
    r = random.Random(12345)
    labels, pred = torch.zeros(mb, n, T), torch.zeros(mb, n, T)
    for i in range(mb):
        for j in range(T):
            p = torch.rand(n, generator=g)
            pred[i, :, j] = p / p.sum()
            labels[i, r.randrange(n), j] = 1
    labels2, pred2 = torch.zeros(mb, n, T + 2), torch.zeros(mb, n, T + 2)
    labels2[:, :, 1:T + 1], pred2[:, :, 1:T + 1] = labels, pred
    mask = torch.ones(mb, T + 2)
    mask[:, 0] = mask[:, T + 1] = 0
    a, b = Evaluation(), Evaluation()
    a.evalTimeSeries(labels, pred)
    b.evalTimeSeries(labels2, pred2, mask)
    assert a.accuracy() == b.accuracy() and a.f1() == b.f1()
    for f in ("falsePositives", "falseNegatives", "truePositives", "trueNegatives"):
        assert dict(getattr(a, f)()) == dict(getattr(b, f)())
    assert all(a.classCount(i) == b.classCount(i) for i in range(n))


def test_false_perfect_recall():
    g = torch.Generator().manual_seed(241)
    r = random.Random(241)
    labels, pred = torch.zeros(100, 5), torch.zeros(100, 5)
    for i in range(100):
        p = torch.rand(5, generator=g)
        p[1] = p.sum()
        pred[i] = p / p.sum()
        labels[i, r.randrange(5)] = 1
    e = Evaluation(5)
    e.eval(labels, pred)
    assert e.recall() != 1.0


def _same(a, b):
    assert abs(a.accuracy() - b.accuracy()) < 1e-3 and abs(a.f1() - b.f1()) < 1e-3
    assert a.getNumRowCounter() == b.getNumRowCounter()
    for f in ("falseNegatives", "falsePositives", "trueNegatives", "truePositives"):
        assert dict(getattr(a, f)()) == dict(getattr(b, f)())
    for f in ("precision", "recall", "falsePositiveRate", "falseNegativeRate", "falseAlarmRate"):
        assert abs(getattr(a, f)() - getattr(b, f)()) < 1e-3, f
    assert a.getConfusionMatrix() == b.getConfusionMatrix()


def test_evaluation_merging():
    r = random.Random(12345)
    act, pred = torch.zeros(20, 3), torch.zeros(20, 3)
    for i in range(20):
        act[i, r.randrange(3)] = 1
        pred[i, r.randrange(3)] = 1
    exp = Evaluation()
    exp.eval(act, pred)
    parts = []
    for lo, hi in ((0, 5), (5, 10), (10, 20)):
        e = Evaluation()
        e.eval(act[lo:hi], pred[lo:hi])
        parts.append(e)
    m = Evaluation()
    for p in parts:
        m.merge(p)
    _same(exp, m)
    e1 = Evaluation()
    e1.eval(act[:5], pred[:5])
    for p in (Evaluation(), parts[1], Evaluation(), parts[2]):       # empty evaluations merge as no-ops
        e1.merge(p)
    _same(exp, e1)


def test_single_class_binary():
    e = Evaluation(1)
    for _ in range(3):
        zero, one = torch.zeros(1, 1), torch.ones(1, 1)
        e.eval(one, zero)
        e.eval(one, one)
        e.eval(one, one)
        e.eval(zero, zero)
        assert abs(e.accuracy() - 0.75) < 1e-6 and e.getNumRowCounter() == 4
        assert e.truePositives()[0] == 1 and e.truePositives()[1] == 2 and e.falseNegatives()[1] == 1
        e.reset()


def test_eval_invalid_and_int_methods():
    e = Evaluation(5)
    e.evalSingle(0, 1)
    e.evalSingle(1, 0)
    e.evalSingle(1, 1)
    assert "�" not in e.stats()
    e1, e2 = Evaluation(4), Evaluation(4)
    oh = [_oh(i, 4) for i in range(4)]
    for actual, predicted in ((0, 0), (0, 2), (0, 2), (1, 2), (3, 3), (3, 0), (3, 0)):
        e1.eval(oh[actual], oh[predicted])
        e2.evalSingle(predicted, actual)                           # (predicted, actual), as the reference's eval(int, int)
    _same(e1, e2)


_P0 = [[0.8, 0.05, 0.05, 0.05, 0.05], [0.4, 0.45, 0.05, 0.05, 0.05], [0.1, 0.45, 0.35, 0.05, 0.05],
       [0.1, 0.40, 0.30, 0.15, 0.05]]
_P1 = [[0.05, 0.80, 0.05, 0.05, 0.05], [0.45, 0.40, 0.05, 0.05, 0.05], [0.35, 0.10, 0.45, 0.05, 0.05],
       [0.40, 0.10, 0.30, 0.15, 0.05]]


def test_top_n_accuracy():
    e = Evaluation(None, 3)
    exp = [(1, 1, 1), (1, 2, 2), (1, 3, 3), (1, 3, 4), (2, 4, 5), (2, 5, 6), (2, 6, 7), (2, 6, 8)]
    for k, (cls, p) in enumerate([(0, q) for q in _P0] + [(1, q) for q in _P1]):
        e.eval(_oh(cls, 5), torch.tensor([p]))
        c, tn, tot = exp[k]
        assert abs(e.accuracy() - c / tot) < 1e-6 and abs(e.topNAccuracy() - tn / tot) < 1e-6
    assert e.getTopNCorrectCount() == 6 and e.getTopNTotalCount() == 8


def test_top_n_accuracy_merging():
    e1, e2 = Evaluation(None, 3), Evaluation(None, 3)
    for p in _P0:
        e1.eval(_oh(0, 5), torch.tensor([p]))
    for p in _P1:
        e2.eval(_oh(1, 5), torch.tensor([p]))
    assert (e1.getTopNCorrectCount(), e1.getTopNTotalCount()) == (3, 4)
    assert abs(e2.topNAccuracy() - 0.75) < 1e-6
    e1.merge(e2)
    assert e1.getNumRowCounter() == 8 and e1.getTopNTotalCount() == 8 and e1.getTopNCorrectCount() == 6
    assert abs(e1.accuracy() - 0.25) < 1e-6 and abs(e1.topNAccuracy() - 0.75) < 1e-6


def test_binary_single_column_case():
    e = Evaluation()
    for lab, pred, n in ((1, 1, 10), (1, 0, 3), (0, 1, 4), (0, 0, 2)):
        e.eval(torch.full((n, 1), float(lab)), torch.full((n, 1), float(pred)))
    assert abs(e.accuracy() - 12 / 19) < 1e-6
    assert (e.truePositives()[1], e.falseNegatives()[1], e.falsePositives()[1], e.trueNegatives()[1]) == (10, 3, 4, 2)
    assert (e.trueNegatives()[0], e.falsePositives()[0], e.falseNegatives()[0], e.truePositives()[0]) == (10, 3, 4, 2)


def test_f1_fbeta_micro_macro_averaging():
    z, o, t = (torch.tensor([v]) for v in ([1.0, 0, 0], [0.0, 1, 0], [0.0, 0, 1]))
    e = Evaluation()
    for n, pred, lab in ((3, z, z), (1, o, z), (2, z, o), (2, o, o), (1, t, o), (3, o, t), (4, t, t)):
        for _ in range(n):                                          # (count, predicted, actual) as the reference
            e.eval(lab, pred)
    cm = e.getConfusionMatrix()
    assert [[cm.getCount(a, p) for p in range(3)] for a in range(3)] == [[3, 1, 0], [2, 2, 1], [0, 3, 4]]
    tp, fp, fn, tn = (dict(getattr(e, f)()) for f in ("truePositives", "falsePositives", "falseNegatives",
                                                        "trueNegatives"))
    assert [(tp[i], fn[i], fp[i], tn[i]) for i in range(3)] == [(3, 1, 2, 10), (2, 3, 4, 7), (4, 3, 1, 8)]
    beta = 3.5
    prec = [tp[i] / (tp[i] + fp[i]) for i in range(3)]
    rec = [tp[i] / (tp[i] + fn[i]) for i in range(3)]
    fb = [(1 + beta ** 2) * prec[i] * rec[i] / (beta ** 2 * prec[i] + rec[i]) for i in range(3)]
    f1 = [2 * prec[i] * rec[i] / (prec[i] + rec[i]) for i in range(3)]
    mcc = [(tp[i] * tn[i] - fp[i] * fn[i]) / math.sqrt((tp[i] + fp[i]) * (tp[i] + fn[i]) * (tn[i] + fp[i]) *
                                                       (tn[i] + fn[i])) for i in range(3)]
    for i in range(3):
        assert abs(e.fBeta(beta, i) - fb[i]) < 1e-6 and abs(e.f1(i) - f1[i]) < 1e-6
        assert abs(e.gMeasure(i) - math.sqrt(prec[i] * rec[i])) < 1e-6
        assert abs(e.matthewsCorrelation(i) - mcc[i]) < 1e-6
    T, FN, FP, TN = (sum(d.values()) for d in (tp, fn, fp, tn))
    mp, mr = T / (T + FP), T / (T + FN)
    assert abs(e.precision(EvaluationAveraging.Macro) - sum(prec) / 3) < 1e-6
    assert abs(e.recall(EvaluationAveraging.Macro) - sum(rec) / 3) < 1e-6
    assert abs(e.f1(EvaluationAveraging.Macro) - sum(f1) / 3) < 1e-6
    assert abs(e.fBeta(beta, EvaluationAveraging.Macro) - sum(fb) / 3) < 1e-6
    assert abs(e.matthewsCorrelation(EvaluationAveraging.Macro) - sum(mcc) / 3) < 1e-6
    assert abs(e.precision(EvaluationAveraging.Micro) - mp) < 1e-6
    assert abs(e.recall(EvaluationAveraging.Micro) - mr) < 1e-6
    assert abs(e.f1(EvaluationAveraging.Micro) - 2 * mp * mr / (mp + mr)) < 1e-6
    assert abs(e.fBeta(beta, EvaluationAveraging.Micro) -
               (1 + beta ** 2) * mp * mr / (beta ** 2 * mp + mr)) < 1e-6
    assert abs(e.matthewsCorrelation(EvaluationAveraging.Micro) -
               (T * TN - FP * FN) / math.sqrt((T + FP) * (T + FN) * (TN + FP) * (TN + FN))) < 1e-6


def test_confusion_matrix_stats_text():
    e = Evaluation()
    c = [torch.tensor([v]) for v in ([1.0, 0, 0], [0.0, 1, 0], [0.0, 0, 1])]
    for _ in range(3):
        e.eval(c[0], c[2])                                         # predicted 2 when actually 0
    for _ in range(2):
        e.eval(c[1], c[0])
    st = e.stats()
    assert "Predictions labeled as 0 classified by model as 2: 3 times" in st
    assert "Predictions labeled as 1 classified by model as 0: 2 times" in st


# ---- CORET:eval/EvalCustomThreshold.java
def _probs(n, c, seed=12345):
    g = torch.Generator().manual_seed(seed)
    p = torch.rand(n, c, generator=g)
    return p / p.sum(1, keepdim=True)


def _cm(e):
    return e.getConfusionMatrix()


def test_custom_binary_threshold():
    probs = _probs(20, 2)
    r = random.Random(12345)
    labels = torch.zeros(20, 2)
    for i in range(20):
        labels[i, r.randrange(2)] = 1
    e, e05, e05v2 = Evaluation(), Evaluation(0.5), Evaluation(0.5)
    e.eval(labels, probs)
    e05.eval(labels, probs)
    e05v2.eval(labels[:, 1:2], probs[:, 1:2])                      # single-output binary
    for e2 in (e05, e05v2):
        for f in ("accuracy", "f1", "precision", "recall"):
            assert abs(getattr(e, f)() - getattr(e2, f)()) < 1e-6
        assert _cm(e) == _cm(e2)
    # threshold 0.25 == doubling the positive probability (capped at 1) with the default argmax
    p2 = probs.clone()
    p2[:, 1] = (p2[:, 1] * 2).clamp(max=1.0)
    p2[:, 0] = 1 - p2[:, 1]
    ex2, e025, e025v2 = Evaluation(), Evaluation(0.25), Evaluation(0.25)
    ex2.eval(labels, p2)
    e025.eval(labels, probs)
    e025v2.eval(labels[:, 1:2], probs[:, 1:2])
    for e2 in (e025, e025v2):
        for f in ("accuracy", "f1", "precision", "recall"):
            assert abs(getattr(ex2, f)() - getattr(e2, f)()) < 1e-6
        assert _cm(ex2) == _cm(e2)


def test_cost_array():
    probs = _probs(20, 3)
    r = random.Random(12345)
    labels = torch.zeros(20, 3)
    for j in range(20):
        labels[j, r.randrange(2)] = 1
    e = Evaluation()
    e.eval(labels, probs)
    for i in (1, 2, 3):                                            # a uniform cost array changes nothing
        e2 = Evaluation(torch.full((1, 3), float(i)))
        e2.eval(labels, probs)
        assert abs(e.accuracy() - e2.accuracy()) < 1e-6 and _cm(e) == _cm(e2)
    labels = torch.eye(3)
    probs = torch.tensor([[0.2, 0.3, 0.5], [0.1, 0.4, 0.5], [0.1, 0.1, 0.8]])
    e = Evaluation()
    e.eval(labels, probs)
    assert abs(e.accuracy() - 1 / 3) < 1e-6
    e2 = Evaluation(torch.tensor([5.0, 2, 1]))
    e2.eval(labels, probs)
    assert abs(e2.accuracy() - 1.0) < 1e-6


def test_evaluation_binary_custom_threshold():
    from deeplearning4j_amd.eval import EvaluationBinary
    g = torch.Generator().manual_seed(7)
    probs = torch.rand(20, 2, generator=g)
    labels = (torch.rand(20, 2, generator=g) < 0.5).float()
    std = EvaluationBinary()
    std.eval(labels, probs)
    b05, b05v2 = EvaluationBinary(torch.tensor([0.5, 0.5])), EvaluationBinary(torch.tensor([0.5, 0.5]))
    b05.eval(labels, probs)
    for i in range(20):
        b05v2.eval(labels[i:i + 1], probs[i:i + 1])
    for b in (b05, b05v2):
        for j in range(2):
            assert (b.truePositives(j), b.falsePositives(j), b.trueNegatives(j), b.falseNegatives(j)) == \
                (std.truePositives(j), std.falsePositives(j), std.trueNegatives(j), std.falseNegatives(j))
            assert abs(b.accuracy(j) - std.accuracy(j)) < 1e-6 and abs(b.f1(j) - std.f1(j)) < 1e-6
    thr = EvaluationBinary(torch.tensor([0.25, 0.125]))
    thr.eval(labels, probs)
    s2, s4 = EvaluationBinary(), EvaluationBinary()
    s2.eval(labels, (probs * 2).clamp(max=1.0))
    s4.eval(labels, (probs * 4).clamp(max=1.0))
    for j, ref in ((0, s2), (1, s4)):
        assert (thr.truePositives(j), thr.trueNegatives(j), thr.falsePositives(j), thr.falseNegatives(j)) == \
            (ref.truePositives(j), ref.trueNegatives(j), ref.falsePositives(j), ref.falseNegatives(j))


# ---- CORET:eval/RegressionEvalTest.java
def test_regression_perfect_and_known_values():
    from deeplearning4j_amd.eval import RegressionEvaluation
    ev = RegressionEvaluation(5)
    g = torch.Generator().manual_seed(0)
    for _ in range(100):
        r = torch.rand(3, 5, generator=g)
        ev.eval(r, r)
    for i in range(5):
        assert abs(ev.meanSquaredError(i)) < 1e-6 and abs(ev.meanAbsoluteError(i)) < 1e-6
        assert abs(ev.rootMeanSquaredError(i)) < 1e-6 and abs(ev.relativeSquaredError(i)) < 1e-6
        assert abs(ev.correlationR2(i) - 1) < 1e-6 and abs(ev.pearsonCorrelation(i) - 1) < 1e-6
        assert abs(ev.rSquared(i) - 1) < 1e-6
    labels = torch.tensor([[1, 2, 3], [0.1, 0.2, 0.3], [6, 5, 4]], dtype=torch.float64)
    pred = torch.tensor([[2.5, 3.2, 3.8], [2.15, 1.3, -1.2], [7, 4.5, 3]], dtype=torch.float64)
    exp = {"meanSquaredError": [2.484166667, 0.966666667, 1.296666667],
           "meanAbsoluteError": [1.516666667, 0.933333333, 1.1],
           "relativeSquaredError": [0.368813923, 0.246598639, 0.530937216],
           "pearsonCorrelation": [0.997013483, 0.968619605, 0.915603032],
           "rSquared": [0.63118608, 0.75340136, 0.46906278]}
    ev = RegressionEvaluation(3)
    for _ in range(2):
        ev.eval(labels, pred)
        for col in range(3):
            for f, v in exp.items():
                assert abs(getattr(ev, f)(col) - v[col]) < 1e-5, (f, col)
            assert abs(ev.rootMeanSquaredError(col) - math.sqrt(exp["meanSquaredError"][col])) < 1e-5
        ev.reset()


def test_regression_merging_masking_and_splitting():
    from deeplearning4j_amd.eval import RegressionEvaluation
    g = torch.Generator().manual_seed(12345)
    single, parts = RegressionEvaluation(3), [RegressionEvaluation(3) for _ in range(4)]
    for p in parts:
        for _ in range(5):
            pr, act = torch.rand(20, 3, generator=g), torch.rand(20, 3, generator=g)
            single.eval(act, pr)
            p.eval(act, pr)
    merged = parts[0]
    for p in parts[1:]:
        merged.merge(p)
    for i in range(3):
        for f in ("correlationR2", "meanAbsoluteError", "meanSquaredError", "relativeSquaredError",
                  "rootMeanSquaredError"):
            assert abs(getattr(single, f)(i) - getattr(merged, f)(i)) < 1e-5, f
    # per-output mask
    lab = torch.tensor([[1.0, 2, 3], [10, 20, 30], [-5, -10, -20]])
    mask = torch.tensor([[0.0, 1, 1], [1, 1, 0], [0, 1, 0]])
    re = RegressionEvaluation()
    re.eval(lab, torch.zeros_like(lab), mask)
    mse = [100.0, (4 + 400 + 100) / 3, 9.0]
    mae = [10.0, 32 / 3, 3.0]
    for i in range(3):
        assert abs(re.meanSquaredError(i) - mse[i]) < 1e-5 and abs(re.meanAbsoluteError(i) - mae[i]) < 1e-5
        assert abs(re.rootMeanSquaredError(i) - math.sqrt(mse[i])) < 1e-5
    # time series evaluated whole == in two halves
    out, lab = torch.rand(3, 5, 20, generator=g), torch.rand(3, 5, 20, generator=g)
    e1, e2 = RegressionEvaluation(), RegressionEvaluation()
    e1.eval(lab, out)
    e2.eval(lab[:, :, :10], out[:, :, :10])
    e2.eval(lab[:, :, 10:], out[:, :, 10:])
    for i in range(5):
        assert abs(e1.meanSquaredError(i) - e2.meanSquaredError(i)) < 1e-6
        assert abs(e1.pearsonCorrelation(i) - e2.pearsonCorrelation(i)) < 1e-5


def test_regression_eval_methods_on_networks():
    from deeplearning4j_amd import (Activation, ComputationGraph, DataSet, MultiLayerNetwork, NeuralNetConfiguration,
                                    OutputLayer, WeightInit)
    from deeplearning4j_amd.datasets.dataset import ExistingDataSetIterator
    ds = DataSet(torch.zeros(4, 10), torch.ones(4, 5))
    net = MultiLayerNetwork(NeuralNetConfiguration.Builder().weightInit(WeightInit.ZERO).list()
                            .layer(0, OutputLayer.Builder().activation(Activation.TANH).nIn(10).nOut(5).build())
                            .build())
    net.init()
    cg = ComputationGraph(NeuralNetConfiguration.Builder().weightInit(WeightInit.ZERO).graphBuilder().addInputs("in")
                          .addLayer("0", OutputLayer.Builder().activation(Activation.TANH).nIn(10).nOut(5).build(),
                                    "in").setOutputs("0").build())
    cg.init()
    for m in (net, cg):
        re = m.evaluateRegression(ExistingDataSetIterator([ds]))
        for i in range(5):
            assert abs(re.meanSquaredError(i) - 1) < 1e-6 and abs(re.meanAbsoluteError(i) - 1) < 1e-6


# ---- CORET:eval/ROCTest.java
_EXP_TPR = {0: 1, 1: 1, 2: 1, 3: 1, 4: 1, 5: 1, 6: .8, 7: .6, 8: .4, 9: .2, 10: 0}
_EXP_FPR = {0: 1, 1: .8, 2: .6, 3: .4, 4: .2, 5: 0, 6: 0, 7: 0, 8: 0, 9: 0, 10: 0}


@pytest.mark.parametrize("single", [False, True])
def test_roc_basic(single):
    from deeplearning4j_amd.eval import ROC
    p1 = torch.tensor([0.001, 0.101, 0.201, 0.301, 0.401, 0.501, 0.601, 0.701, 0.801, 0.901], dtype=torch.float64)
    y1 = torch.tensor([0.0] * 5 + [1.0] * 5, dtype=torch.float64)
    pred = p1.reshape(-1, 1) if single else torch.stack([1 - p1, p1], 1)
    act = y1.reshape(-1, 1) if single else torch.stack([1 - y1, y1], 1)
    roc = ROC(10)
    for _ in range(2):
        roc.eval(act, pred)
        c = roc.getRocCurve()
        assert c.numPoints() == 11
        for i in range(11):
            assert abs(c.getThreshold(i) - i / 10) < 1e-5
            assert abs(c.getFalsePositiveRate(i) - _EXP_FPR[i]) < 1e-5
            assert abs(c.getTruePositiveRate(i) - _EXP_TPR[i]) < 1e-5
        assert abs(roc.calculateAUC() - 1.0) < 1e-6
        roc.reset()


def test_roc_known_values_and_pr_confusion():
    from deeplearning4j_amd.eval import ROC
    labels = torch.tensor([[0.0, 1], [0, 1], [1, 0], [1, 0], [1, 0]])
    pred = torch.tensor([[0.199, 0.801], [0.499, 0.501], [0.399, 0.601], [0.799, 0.201], [0.899, 0.101]])
    tpr = [1, 1, 1, 1, 1, 1, .5, .5, .5, 0, 0]
    fpr = [1, 1, 2 / 3, 1 / 3, 1 / 3, 1 / 3, 1 / 3, 0, 0, 0, 0]
    tps = [2, 2, 2, 2, 2, 2, 1, 1, 1, 0, 0]
    fps = [3, 3, 2, 1, 1, 1, 1, 0, 0, 0, 0]
    roc = ROC(10)
    roc.eval(labels, pred)
    c = roc.getRocCurve()
    for i in range(11):
        assert abs(c.getFalsePositiveRate(i) - fpr[i]) < 1e-5 and abs(c.getTruePositiveRate(i) - tpr[i]) < 1e-5
    assert abs(roc.calculateAUC() - (0.5 / 3 + 2 / 3)) < 1e-6
    prc = roc.getPrecisionRecallCurve()
    for i in range(11):
        cf = prc.getConfusionMatrixAtThreshold(i * 0.1)
        assert (cf.getTpCount(), cf.getFpCount(), cf.getFnCount()) == (tps[i], fps[i], 2 - tps[i])
        assert cf.getTnCount() == 5 - tps[i] - fps[i] - (2 - tps[i])


def test_precision_recall_curve_point_methods():
    from deeplearning4j_amd.eval.curves import PrecisionRecallCurve
    thr = [i / 100 for i in range(101)]
    prc = PrecisionRecallCurve(thr, thr, [1 - t for t in thr], None, None, None, -1)
    for p in (prc.getPointAtThreshold(0.05), prc.getPointAtPrecision(0.05), prc.getPointAtRecall(1 - 0.05),
              prc.getPointAtThreshold(0.0495), prc.getPointAtPrecision(0.0495), prc.getPointAtRecall(1 - 0.0505)):
        assert p.getIdx() == 5 and abs(p.getThreshold() - 0.05) < 1e-6
        assert abs(p.getPrecision() - 0.05) < 1e-6 and abs(p.getRecall() - 0.95) < 1e-6


@pytest.mark.parametrize("remove", [True, False])
def test_precision_recall_curve_confusion_consistent(remove):
    from deeplearning4j_amd.eval import ROC
    g = torch.Generator().manual_seed(11)
    labels = (torch.rand(100, 1, generator=g) < 0.5).double()
    probs = torch.rand(100, 1, generator=g, dtype=torch.float64)
    r = ROC(0, remove)
    r.eval(labels, probs)
    prc = r.getPrecisionRecallCurve()
    for i in range(prc.numPoints()):
        cf = prc.getConfusionMatrixAtPoint(i)
        p = cf.getPoint()
        tp, fp, fn = cf.getTpCount(), cf.getFpCount(), cf.getFnCount()
        prec = 1.0 if tp == 0 and fp == 0 else tp / (tp + fp)
        assert abs(p.getPrecision() - prec) < 1e-8 and abs(p.getRecall() - tp / (tp + fn)) < 1e-8


# ---- CORET:eval/EvaluationBinaryTest.java
def _bern(shape, g):
    return (torch.rand(*shape, generator=g) < 0.5).double()


def test_evaluation_binary_vs_evaluation_per_column():
    from deeplearning4j_amd.eval import EvaluationBinary
    g = torch.Generator().manual_seed(12345)
    labels, pred = _bern((50, 4), g), torch.rand(50, 4, generator=g, dtype=torch.float64)
    eb = EvaluationBinary()
    eb.eval(labels, pred)
    for i in range(4):
        lc, pc = labels[:, i:i + 1], pred[:, i:i + 1]
        bp = (pc > 0.5).double()
        correct = (lc == bp)
        e = Evaluation()
        e.eval(lc, pc)
        assert abs(eb.accuracy(i) - correct.double().mean().item()) < 1e-6
        assert abs(e.accuracy() - eb.accuracy(i)) < 1e-6
        assert abs(e.precision(1) - eb.precision(i)) < 1e-6 and abs(e.recall(1) - eb.recall(i)) < 1e-6
        assert abs(e.f1(1) - eb.f1(i)) < 1e-6
        assert eb.truePositives(i) == int((correct & (lc == 1)).sum()) == e.truePositives()[1]
        assert eb.trueNegatives(i) == int((correct & (lc == 0)).sum()) == e.trueNegatives()[1]
        assert eb.falsePositives(i) == e.falsePositives()[1] and eb.falseNegatives(i) == e.falseNegatives()[1]
        assert eb.totalCount(i) == 50


def test_evaluation_binary_merging_masking_time_series_roc():
    from deeplearning4j_amd.eval import EvaluationBinary
    g = torch.Generator().manual_seed(12345)
    l1, l2 = _bern((30, 4), g), _bern((50, 4), g)
    p1, p2 = torch.rand(30, 4, generator=g, dtype=torch.float64), torch.rand(50, 4, generator=g, dtype=torch.float64)
    eb, eb1, eb2 = EvaluationBinary(), EvaluationBinary(), EvaluationBinary()
    eb.eval(l1, p1)
    eb.eval(l2, p2)
    eb1.eval(l1, p1)
    eb2.eval(l2, p2)
    eb1.merge(eb2)
    assert eb.stats() == eb1.stats()
    # per-output mask
    mask = torch.tensor([[1.0, 1, 0], [1, 0, 0], [1, 1, 0], [1, 0, 0], [1, 1, 1]])
    labels = torch.tensor([[1.0, 1, 1], [0, 0, 0], [1, 1, 1], [0, 1, 1], [1, 0, 1]])
    pred = torch.tensor([[0.9] * 3, [0.7] * 3, [0.6] * 3, [0.4] * 3, [0.1] * 3])
    m = EvaluationBinary()
    m.eval(labels, pred, mask)
    assert [m.accuracy(i) for i in range(3)] == pytest.approx([0.6, 1.0, 0.0])
    assert [m.truePositives(i) for i in range(3)] == [2, 2, 0]
    assert [m.trueNegatives(i) for i in range(3)] == [1, 1, 0]
    assert [m.falsePositives(i) for i in range(3)] == [1, 0, 0]
    assert [m.falseNegatives(i) for i in range(3)] == [1, 0, 1]
    # time series == step by step
    lab, prd, msk = _bern((2, 4, 3), g), torch.rand(2, 4, 3, generator=g, dtype=torch.float64), _bern((2, 4, 3), g)
    a, b = EvaluationBinary(), EvaluationBinary()
    a.eval(lab, prd, msk)
    for t in range(3):
        b.eval(lab[:, :, t], prd[:, :, t], msk[:, :, t])
    assert a.stats() == b.stats()
    # with ROC attached
    r = EvaluationBinary(4, 30)
    r.eval(l1, p1)
    assert r.getROCBinary() is not None and r.getROCBinary().numLabels() == 4
