"""Per-output binary classification metrics for multi-label outputs (reference eval/EvaluationBinary.java:62-560):
each column thresholded at 0.5 (or a per-column decision threshold), optional per-element masks, optional
ROCBinary tracked alongside."""
import numpy as np
import torch

from .base import BaseEvaluation, EvaluationUtils, to_2d
from .roc import ROCBinary


class EvaluationBinary(BaseEvaluation):
    def __init__(self, decisionThreshold=None, rocBinarySteps=None, size=None):
        if isinstance(decisionThreshold, int) and not isinstance(decisionThreshold, bool):
            size, decisionThreshold = decisionThreshold, None
        self.decisionThreshold = None if decisionThreshold is None else \
            np.asarray(torch.as_tensor(decisionThreshold).float().reshape(-1).cpu())
        self.rocBinarySteps = rocBinarySteps
        self.labels = None
        self.tp = self.fp = self.tn = self.fn = None
        if size is not None:
            self._zero(size)
        self._roc = ROCBinary(rocBinarySteps) if rocBinarySteps is not None else None

    def _zero(self, n):
        self.tp, self.fp, self.tn, self.fn = (np.zeros(n, dtype=np.int64) for _ in range(4))

    def _after_load(self):
        for k in ("tp", "fp", "tn", "fn"):
            if getattr(self, k) is not None:
                setattr(self, k, np.asarray(getattr(self, k), dtype=np.int64))
        self._roc = None

    def reset(self):
        if self.tp is not None:
            self._zero(len(self.tp))
        if self._roc is not None:
            self._roc.reset()

    def setLabelNames(self, labels):
        self.labels = list(labels)

    def eval(self, labels, predictions, mask=None):
        labels, preds, m2 = to_2d(labels, predictions, mask)
        if self.tp is not None and len(self.tp) != labels.shape[1]:
            raise ValueError(f"Labels array does not match stored state size. Expected labels array with size "
                             f"{len(self.tp)}, got labels array with size {labels.shape[1]}")
        preds = preds.to(labels.device).float()
        y = labels.float() != 0
        thr = 0.5 if self.decisionThreshold is None else torch.as_tensor(self.decisionThreshold, device=preds.device)
        p = preds > thr
        m = torch.ones_like(y) if m2 is None else (m2.to(y.device) != 0).expand_as(y)
        stats = torch.stack([(p & y & m).sum(0), (p & ~y & m).sum(0), (~p & ~y & m).sum(0),
                             (~p & y & m).sum(0)]).cpu().numpy().astype(np.int64)
        if self.tp is None:
            self._zero(labels.shape[1])
        self.tp += stats[0]
        self.fp += stats[1]
        self.tn += stats[2]
        self.fn += stats[3]
        if self._roc is not None:
            self._roc.eval(labels, preds, m2)

    def merge(self, other):
        if other.tp is None:
            return
        if self.tp is None:
            self._zero(len(other.tp))
        self.tp += other.tp
        self.fp += other.fp
        self.tn += other.tn
        self.fn += other.fn
        if self._roc is not None and other._roc is not None:
            self._roc.merge(other._roc)

    def numLabels(self):
        return 0 if self.tp is None else len(self.tp)

    def totalCount(self, i):
        return int(self.tp[i] + self.fp[i] + self.tn[i] + self.fn[i])

    def truePositives(self, i):
        return int(self.tp[i])

    def trueNegatives(self, i):
        return int(self.tn[i])

    def falsePositives(self, i):
        return int(self.fp[i])

    def falseNegatives(self, i):
        return int(self.fn[i])

    def accuracy(self, i):
        return (self.tp[i] + self.tn[i]) / float(self.totalCount(i))

    def precision(self, i):
        return EvaluationUtils.precision(int(self.tp[i]), int(self.fp[i]))

    def recall(self, i):
        return EvaluationUtils.recall(int(self.tp[i]), int(self.fn[i]))

    def fBeta(self, beta, i):
        return EvaluationUtils.fBeta(beta, int(self.tp[i]), int(self.fp[i]), int(self.fn[i]))

    def f1(self, i):
        return self.fBeta(1.0, i)

    def matthewsCorrelation(self, i):
        return EvaluationUtils.matthewsCorrelation(int(self.tp[i]), int(self.fp[i]), int(self.fn[i]), int(self.tn[i]))

    def gMeasure(self, i):
        return EvaluationUtils.gMeasure(self.precision(i), self.recall(i))

    def falsePositiveRate(self, i, edgeCase=0.0):
        return EvaluationUtils.falsePositiveRate(int(self.fp[i]), int(self.tn[i]), edgeCase)

    def falseNegativeRate(self, i, edgeCase=0.0):
        return EvaluationUtils.falseNegativeRate(int(self.fn[i]), int(self.tp[i]), edgeCase)

    def _avg(self, f):
        n = self.numLabels()
        return sum(f(i) for i in range(n)) / n

    def averageAccuracy(self):
        return self._avg(self.accuracy)

    def averagePrecision(self):
        return self._avg(self.precision)

    def averageRecall(self):
        return self._avg(self.recall)

    def averageF1(self):
        return self._avg(self.f1)

    def getROCBinary(self):
        return self._roc

    def stats(self, printPrecision=4):
        if self.tp is None:
            return "EvaluationBinary: No data"
        p = printPrecision
        rows = [f"{'Label':<15}{'Accuracy':<12}{'F1':<12}{'Precision':<12}{'Recall':<12}{'Total':<8}"
                f"{'TP':<8}{'TN':<8}{'FP':<8}{'FN':<8}" + ("AUC" if self._roc is not None else "")]
        for i in range(self.numLabels()):
            name = self.labels[i] if self.labels else str(i)
            r = (f"{name:<15}{self.accuracy(i):<12.{p}f}{self.f1(i):<12.{p}f}{self.precision(i):<12.{p}f}"
                 f"{self.recall(i):<12.{p}f}{self.totalCount(i):<8d}{int(self.tp[i]):<8d}{int(self.tn[i]):<8d}"
                 f"{int(self.fp[i]):<8d}{int(self.fn[i]):<8d}")
            if self._roc is not None:
                r += f"{self._roc.calculateAUC(i):.{p}f}"
            rows.append(r)
        return "\n".join(rows)
