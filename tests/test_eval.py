"""Evaluation metrics vs independent implementations (scikit-learn) and the reference's own expectations
(deeplearning4j-core/src/test/java/org/deeplearning4j/eval/EvalTest.java, ROCTest.java, RegressionEvalTest.java,
EvaluationBinaryTest.java, EvaluationCalibrationTest.java)."""
import numpy as np
import pytest
import torch
from sklearn import metrics as skm

from deeplearning4j_amd.eval import (ROC, Evaluation, EvaluationAveraging, EvaluationBinary, EvaluationCalibration,
                                     RegressionEvaluation, ROCBinary, ROCMultiClass)


def _onehot(idx, n):
    y = torch.zeros(len(idx), n)
    y[torch.arange(len(idx)), torch.as_tensor(idx)] = 1
    return y


def test_evaluation_matches_sklearn():
    g = torch.Generator().manual_seed(0)
    n, C = 500, 5
    actual = torch.randint(0, C, (n,), generator=g)
    probs = torch.softmax(torch.randn(n, C, generator=g) + 2 * _onehot(actual, C), 1)
    e = Evaluation()
    for i in range(0, n, 64):     # minibatched accumulation
        e.eval(_onehot(actual[i:i + 64], C), probs[i:i + 64])
    pred = probs.argmax(1).numpy()
    a = actual.numpy()
    assert e.accuracy() == pytest.approx(skm.accuracy_score(a, pred))
    assert e.precision() == pytest.approx(skm.precision_score(a, pred, average="macro"))
    assert e.recall() == pytest.approx(skm.recall_score(a, pred, average="macro"))
    assert e.f1() == pytest.approx(skm.f1_score(a, pred, average="macro"))
    assert e.precision(EvaluationAveraging.Micro) == pytest.approx(skm.precision_score(a, pred, average="micro"))
    for c in range(C):
        assert e.precision(c) == pytest.approx(skm.precision_score(a, pred, labels=[c], average="macro"))
        assert e.recall(c) == pytest.approx(skm.recall_score(a, pred, labels=[c], average="macro"))
    cm = skm.confusion_matrix(a, pred)
    assert np.array_equal(e.getConfusionMatrix().m, cm)
    tn = e.trueNegatives()
    assert all(tn[c] + e.truePositives()[c] + e.falsePositives()[c] + e.falseNegatives()[c] == n for c in range(C))
    s = e.stats()
    assert "Accuracy" in s and "Confusion" in s
    e2 = Evaluation.fromJson(e.toJson())
    assert e2.accuracy() == e.accuracy() and np.array_equal(e2.table, e.table)


def test_evaluation_topn_and_merge():
    probs = torch.tensor([[0.1, 0.3, 0.6], [0.5, 0.3, 0.2], [0.2, 0.5, 0.3]])
    labels = _onehot([1, 2, 0], 3)
    e = Evaluation(None, topN=2)
    e.eval(labels, probs)
    # example 0: class 1 is 2nd -> top2 hit; example 1: class 2 is 3rd -> miss; example 2: class 0 is 3rd -> miss
    assert e.topNAccuracy() == pytest.approx(1 / 3)
    a, b = Evaluation(), Evaluation()
    a.eval(labels[:2], probs[:2])
    b.eval(labels[2:], probs[2:])
    a.merge(b)
    full = Evaluation()
    full.eval(labels, probs)
    assert np.array_equal(a.table, full.table)


def test_evaluation_binary_single_column_and_timeseries_mask():
    # EvalTest: single-output binary case uses threshold 0.5
    y = torch.tensor([[1.0], [0.0], [1.0], [0.0]])
    p = torch.tensor([[0.9], [0.6], [0.4], [0.1]])
    e = Evaluation()
    e.eval(y, p)
    assert e.truePositives()[1] == 1 and e.falsePositives()[1] == 1 and e.falseNegatives()[1] == 1
    assert e.accuracy() == 0.5
    # time series [mb, C, T] with mask [mb, T]: masked steps ignored
    lab = torch.zeros(2, 3, 4)
    lab[:, 0, :] = 1
    out = torch.zeros(2, 3, 4)
    out[:, 0, :2] = 1
    out[:, 2, 2:] = 1          # wrong predictions only in masked-out steps
    mask = torch.tensor([[1, 1, 0, 0], [1, 1, 0, 0]])
    e = Evaluation()
    e.eval(lab, out, mask)
    assert e.getNumRowCounter() == 4 and e.accuracy() == 1.0


@pytest.mark.parametrize("steps", [0, 100])
def test_roc_vs_sklearn(steps):
    g = torch.Generator().manual_seed(1)
    n = 2000
    y = (torch.rand(n, generator=g) < 0.4).float()
    p = torch.clamp(0.3 * y + 0.7 * torch.rand(n, generator=g), 0, 1)
    r = ROC(steps)
    for i in range(0, n, 256):
        r.eval(y[i:i + 256, None], p[i:i + 256, None])
    auc = skm.roc_auc_score(y.numpy(), p.numpy())
    tol = 1e-9 if steps == 0 else 5e-3
    assert r.calculateAUC() == pytest.approx(auc, abs=tol)
    ap = skm.auc(*skm.precision_recall_curve(y.numpy(), p.numpy())[1::-1])
    assert r.calculateAUCPR() == pytest.approx(ap, abs=1e-2 if steps else 5e-3)
    # two-column form (softmax output) gives the same result
    r2 = ROC(steps)
    r2.eval(torch.stack([1 - y, y], 1), torch.stack([1 - p, p], 1))
    assert r2.calculateAUC() == pytest.approx(r.calculateAUC())
    r3 = ROC.fromJson(r.toJson())
    assert r3.calculateAUC() == pytest.approx(r.calculateAUC())


def test_roc_multiclass_and_binary():
    g = torch.Generator().manual_seed(2)
    n, C = 600, 4
    a = torch.randint(0, C, (n,), generator=g)
    p = torch.softmax(torch.randn(n, C, generator=g) + _onehot(a, C), 1)
    r = ROCMultiClass()
    r.eval(_onehot(a, C), p)
    for c in range(C):
        assert r.calculateAUC(c) == pytest.approx(skm.roc_auc_score((a == c).numpy(), p[:, c].numpy()))
    rb = ROCBinary()
    yb = (torch.rand(n, 3, generator=g) < 0.5).float()
    pb = torch.clamp(yb * 0.3 + torch.rand(n, 3, generator=g) * 0.7, 0, 1)
    rb.eval(yb, pb)
    for c in range(3):
        assert rb.calculateAUC(c) == pytest.approx(skm.roc_auc_score(yb[:, c].numpy(), pb[:, c].numpy()))


def test_regression_eval_vs_sklearn():
    g = torch.Generator().manual_seed(3)
    y = torch.randn(300, 3, generator=g)
    p = y + 0.3 * torch.randn(300, 3, generator=g)
    r = RegressionEvaluation(3)
    r.eval(y[:100], p[:100])
    r.eval(y[100:], p[100:])
    for c in range(3):
        assert r.meanSquaredError(c) == pytest.approx(skm.mean_squared_error(y[:, c], p[:, c]), rel=1e-6)
        assert r.meanAbsoluteError(c) == pytest.approx(skm.mean_absolute_error(y[:, c], p[:, c]), rel=1e-6)
        assert r.rSquared(c) == pytest.approx(skm.r2_score(y[:, c], p[:, c]), rel=1e-5)
        assert r.pearsonCorrelation(c) == pytest.approx(np.corrcoef(y[:, c], p[:, c])[0, 1], rel=1e-5)
        rse = ((p[:, c] - y[:, c]) ** 2).sum() / ((y[:, c] - y[:, c].mean()) ** 2).sum()
        assert r.relativeSquaredError(c) == pytest.approx(rse.item(), rel=1e-4)
    assert "MSE" in r.stats()


def test_evaluation_binary_and_calibration():
    y = torch.tensor([[1, 0], [0, 1], [1, 1], [0, 0]], dtype=torch.float32)
    p = torch.tensor([[0.8, 0.4], [0.3, 0.7], [0.4, 0.9], [0.6, 0.2]])
    e = EvaluationBinary()
    e.eval(y, p)
    assert [e.truePositives(0), e.falsePositives(0), e.trueNegatives(0), e.falseNegatives(0)] == [1, 1, 1, 1]
    assert [e.truePositives(1), e.falsePositives(1), e.trueNegatives(1), e.falseNegatives(1)] == [2, 0, 2, 0]
    assert e.accuracy(1) == 1.0
    m = torch.tensor([[1, 1], [1, 1], [1, 1], [0, 1]])
    e2 = EvaluationBinary()
    e2.eval(y, p, m)
    assert e2.totalCount(0) == 3 and e2.totalCount(1) == 4
    cal = EvaluationCalibration(5, 10)
    g = torch.Generator().manual_seed(4)
    a = torch.randint(0, 3, (200,), generator=g)
    pr = torch.softmax(torch.randn(200, 3, generator=g), 1)
    cal.eval(_onehot(a, 3), pr)
    assert cal.getLabelCountsEachClass().sum() == 200
    assert cal.getPredictionCountsEachClass().sum() == 200
    assert cal.getProbabilityHistogramAllClasses().binCounts.sum() == 600
    rd = cal.getReliabilityDiagram(0)
    assert len(rd.meanPredictedValueX) == len(rd.fractionPositivesY) <= 5
