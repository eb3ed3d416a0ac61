"""ROC / AUC / AUPRC for binary, per-output binary and one-vs-all multi-class problems
(reference eval/ROC.java, ROCBinary.java, ROCMultiClass.java).

thresholdSteps == 0 -> exact mode: (probability, label) pairs are kept and the curve is computed from a sort
(ROC.java:475-520). thresholdSteps > 0 -> fixed thresholds i/steps; per minibatch the TP/FP counts at ALL
thresholds come from one vectorised comparison on the device (predicted positive iff p >= t and t < 1,
matching the CompareAndSet pair at ROC.java:264-300).
"""
import numpy as np
import torch

from .base import BaseEvaluation, to_2d
from .curves import PrecisionRecallCurve, RocCurve


def _remove_redundant(t, x, y, ints=None):
    keep = [0]
    n = len(t)
    for i in range(1, n - 1):
        same_x = x[i - 1] == x[i] == x[i + 1]
        same_y = y[i - 1] == y[i] == y[i + 1]
        if not (same_x or same_y):
            keep.append(i)
    if n > 1:
        keep.append(n - 1)
    k = np.asarray(keep)
    out = [np.asarray(t)[k], np.asarray(x)[k], np.asarray(y)[k]]
    if ints is not None:
        out += [np.asarray(a)[k] for a in ints]
    return out


class _BinaryROCState:
    """Accumulator for one binary output column."""

    def __init__(self, steps):
        self.steps = int(steps)
        self.pos = 0
        self.neg = 0
        self.n = 0
        self.probs, self.labels = [], []
        self.tp = np.zeros(self.steps + 1, dtype=np.int64) if self.steps > 0 else None
        self.fp = np.zeros(self.steps + 1, dtype=np.int64) if self.steps > 0 else None

    def add(self, p, y):
        """p, y: 1-d tensors (probability of class 1, label in {0,1})."""
        y = y.to(torch.float64)
        npos = int(y.sum().item())
        self.pos += npos
        self.neg += y.numel() - npos
        self.n += y.numel()
        if self.steps == 0:
            self.probs.append(p.detach().to(torch.float64).cpu().numpy())
            self.labels.append(y.cpu().numpy())
        else:
            t = torch.arange(self.steps + 1, device=p.device, dtype=torch.float64) / self.steps
            pred = (p.to(torch.float64).unsqueeze(0) >= t.unsqueeze(1)) & (t.unsqueeze(1) < 1.0)
            yy = y.to(p.device).unsqueeze(0)
            self.tp += (pred * yy).sum(1).long().cpu().numpy()
            self.fp += (pred * (1 - yy)).sum(1).long().cpu().numpy()

    def merge(self, o):
        self.pos += o.pos
        self.neg += o.neg
        self.n += o.n
        if self.steps == 0:
            self.probs += o.probs
            self.labels += o.labels
        else:
            self.tp += o.tp
            self.fp += o.fp

    def _sorted(self):
        p = np.concatenate(self.probs) if self.probs else np.zeros(0)
        y = np.concatenate(self.labels) if self.labels else np.zeros(0)
        order = np.argsort(-p, kind="stable")
        return p[order], y[order]

    def roc(self, remove=True):
        if self.steps == 0:
            p, y = self._sorted()
            L = len(p)
            cpos, cneg = np.cumsum(y), np.cumsum(1 - y)
            t = np.concatenate([[1.0], p, [0.0]])
            fpr = np.concatenate([[0.0], cneg / max(self.neg, 1) if self.neg else np.zeros(L), [1.0]])
            tpr = np.concatenate([[0.0], cpos / max(self.pos, 1) if self.pos else np.zeros(L), [1.0]])
            if remove:
                t, fpr, tpr = _remove_redundant(t, fpr, tpr)
            return RocCurve(t, fpr, tpr)
        t = np.arange(self.steps + 1) / self.steps
        return RocCurve(t, self.fp / float(self.neg) if self.neg else np.zeros_like(t),
                        self.tp / float(self.pos) if self.pos else np.zeros_like(t))

    def pr(self, remove=True):
        if self.steps == 0:
            p, y = self._sorted()
            L = len(p)
            cpos = np.cumsum(y)
            t = np.concatenate([[1.0], p, [0.0]])
            prec = np.concatenate([[1.0], cpos / np.arange(1, L + 1), [cpos[-1] / L if L else 1.0]])
            rec = np.concatenate([[0.0], cpos / self.pos if self.pos else np.zeros(L), [1.0]])
            tp = np.concatenate([[0], cpos.astype(np.int64), [self.pos]])
            fp = np.concatenate([[0], (np.arange(1, L + 1) - cpos).astype(np.int64), [self.n - self.pos]])
            fn = self.pos - tp
            t, prec, rec, tp, fp, fn = [a[::-1] for a in (t, prec, rec, tp, fp, fn)]
            if remove:
                t, prec, rec, tp, fp, fn = _remove_redundant(t, prec, rec, [tp, fp, fn])
            return PrecisionRecallCurve(t, prec, rec, tp, fp, fn, self.n)
        t = np.arange(self.steps + 1) / self.steps
        with np.errstate(invalid="ignore", divide="ignore"):
            prec = np.where(self.tp + self.fp == 0, 1.0, self.tp / np.maximum(self.tp + self.fp, 1))
        rec = self.tp / float(self.pos) if self.pos else np.ones_like(t)
        return PrecisionRecallCurve(t, prec, rec, self.tp, self.fp, self.pos - self.tp, self.n)

    def to_state(self):
        p, y = self._sorted() if self.steps == 0 else (None, None)
        return {"steps": self.steps, "pos": self.pos, "neg": self.neg, "n": self.n,
                "p": None if p is None else p.tolist(), "y": None if y is None else y.tolist(),
                "tp": None if self.tp is None else self.tp.tolist(), "fp": None if self.fp is None else self.fp.tolist()}

    @staticmethod
    def from_state(d):
        s = _BinaryROCState(d["steps"])
        s.pos, s.neg, s.n = d["pos"], d["neg"], d["n"]
        if s.steps == 0:
            s.probs, s.labels = [np.asarray(d["p"], dtype=np.float64)], [np.asarray(d["y"], dtype=np.float64)]
        else:
            s.tp, s.fp = np.asarray(d["tp"], dtype=np.int64), np.asarray(d["fp"], dtype=np.int64)
        return s


class ROC(BaseEvaluation):
    """Binary ROC: labels/predictions [N,1] (probability of class 1) or [N,2] (column 1 used)."""

    def __init__(self, thresholdSteps=0, rocRemoveRedundantPts=True, exactAllocBlockSize=2048):
        self.thresholdSteps = int(thresholdSteps)
        self.rocRemoveRedundantPts = rocRemoveRedundantPts
        self._s = _BinaryROCState(self.thresholdSteps)

    def reset(self):
        self._s = _BinaryROCState(self.thresholdSteps)

    def isExact(self):
        return self.thresholdSteps == 0

    def eval(self, labels, predictions, mask=None):
        labels, preds, _ = to_2d(labels, predictions, mask)
        if labels.dim() != 2 or labels.shape[1] != preds.shape[1] or labels.shape[1] > 2:
            raise ValueError(f"Invalid input data shape: labels shape = {list(labels.shape)}, predictions shape = "
                             f"{list(preds.shape)}; require rank 2 array with size(1) == 1 or 2")
        col = 0 if labels.shape[1] == 1 else 1
        self._s.add(preds[:, col].to(labels.device), labels[:, col])

    def merge(self, other):
        if self.thresholdSteps != other.thresholdSteps:
            raise ValueError("Cannot merge ROC instances with different numbers of threshold steps ("
                             f"{self.thresholdSteps} vs. {other.thresholdSteps})")
        self._s.merge(other._s)

    def getRocCurve(self):
        return self._s.roc(self.rocRemoveRedundantPts)

    def getPrecisionRecallCurve(self):
        return self._s.pr(self.rocRemoveRedundantPts)

    def calculateAUC(self):
        return self.getRocCurve().calculateAUC() if self._s.n else float("nan")

    def calculateAUCPR(self):
        return self.getPrecisionRecallCurve().calculateAUPRC() if self._s.n else float("nan")

    def getCountActualPositive(self):
        return self._s.pos

    def getCountActualNegative(self):
        return self._s.neg

    def stats(self):
        return f"AUC: [{self.calculateAUC()}]"

    def toJson(self):
        import json
        return json.dumps({"@class": "ROC", "thresholdSteps": self.thresholdSteps,
                           "rocRemoveRedundantPts": self.rocRemoveRedundantPts, "state": self._s.to_state()})

    @classmethod
    def fromJson(cls, s):
        import json
        d = json.loads(s)
        if d.get("@class") == "ROC":
            r = ROC(d["thresholdSteps"], d["rocRemoveRedundantPts"])
            r._s = _BinaryROCState.from_state(d["state"])
            return r
        return BaseEvaluation.fromJson(s)


class ROCBinary(BaseEvaluation):
    """Independent ROC per output column (multi-label binary outputs, e.g. sigmoid layers); per-output masks
    supported (ROCBinary.java)."""

    def __init__(self, thresholdSteps=0, rocRemoveRedundantPts=True):
        self.thresholdSteps = int(thresholdSteps)
        self.rocRemoveRedundantPts = rocRemoveRedundantPts
        self._u = None
        self.labels = None

    def reset(self):
        self._u = None

    def setLabelNames(self, names):
        self.labels = list(names)

    def eval(self, labels, predictions, mask=None):
        labels, preds, m2 = to_2d(labels, predictions, mask)
        n = labels.shape[1]
        if self._u is None:
            self._u = [_BinaryROCState(self.thresholdSteps) for _ in range(n)]
        preds = preds.to(labels.device)
        for i in range(n):
            y, p = labels[:, i], preds[:, i]
            if m2 is not None:
                keep = m2[:, i].to(labels.device) != 0
                y, p = y[keep], p[keep]
            self._u[i].add(p, y)

    def merge(self, other):
        if other._u is None:
            return
        if self._u is None:
            self._u = [_BinaryROCState(self.thresholdSteps) for _ in other._u]
        for a, b in zip(self._u, other._u):
            a.merge(b)

    def numLabels(self):
        return 0 if self._u is None else len(self._u)

    def calculateAUC(self, i):
        return self._u[i].roc(self.rocRemoveRedundantPts).calculateAUC()

    def calculateAUCPR(self, i):
        return self._u[i].pr(self.rocRemoveRedundantPts).calculateAUPRC()

    def getRocCurve(self, i):
        return self._u[i].roc(self.rocRemoveRedundantPts)

    def getPrecisionRecallCurve(self, i):
        return self._u[i].pr(self.rocRemoveRedundantPts)

    def calculateAverageAuc(self):
        return sum(self.calculateAUC(i) for i in range(self.numLabels())) / self.numLabels()

    def calculateAverageAUCPR(self):
        return sum(self.calculateAUCPR(i) for i in range(self.numLabels())) / self.numLabels()

    def getCountActualPositive(self, i):
        return self._u[i].pos

    def getCountActualNegative(self, i):
        return self._u[i].neg

    def stats(self):
        if self._u is None:
            return "ROCBinary: No data"
        rows = ["Label          AUC       # Pos     # Neg"]
        for i in range(self.numLabels()):
            name = self.labels[i] if self.labels else str(i)
            rows.append(f"{name:<15}{self.calculateAUC(i):<10.4f}{self._u[i].pos:<10d}{self._u[i].neg:<10d}")
        rows.append(f"Average AUC: {self.calculateAverageAuc():.4f}")
        return "\n".join(rows)


class ROCMultiClass(BaseEvaluation):
    """One-vs-all ROC per class for softmax outputs [N, C] (ROCMultiClass.java)."""

    def __init__(self, thresholdSteps=0, rocRemoveRedundantPts=True):
        self.thresholdSteps = int(thresholdSteps)
        self.rocRemoveRedundantPts = rocRemoveRedundantPts
        self._u = None
        self.labels = None

    def reset(self):
        self._u = None

    def setLabelNames(self, names):
        self.labels = list(names)

    def eval(self, labels, predictions, mask=None):
        labels, preds, _ = to_2d(labels, predictions, mask)
        n = labels.shape[1]
        if n == 1:
            raise ValueError("ROCMultiClass requires at least 2 output classes; use ROC for a single output")
        if self._u is None:
            self._u = [_BinaryROCState(self.thresholdSteps) for _ in range(n)]
        preds = preds.to(labels.device)
        for i in range(n):
            self._u[i].add(preds[:, i], labels[:, i])

    def merge(self, other):
        if other._u is None:
            return
        if self._u is None:
            self._u = [_BinaryROCState(self.thresholdSteps) for _ in other._u]
        for a, b in zip(self._u, other._u):
            a.merge(b)

    def getNumClasses(self):
        return 0 if self._u is None else len(self._u)

    def calculateAUC(self, c):
        return self._u[c].roc(self.rocRemoveRedundantPts).calculateAUC()

    def calculateAUCPR(self, c):
        return self._u[c].pr(self.rocRemoveRedundantPts).calculateAUPRC()

    def getRocCurve(self, c):
        return self._u[c].roc(self.rocRemoveRedundantPts)

    def getPrecisionRecallCurve(self, c):
        return self._u[c].pr(self.rocRemoveRedundantPts)

    def calculateAverageAUC(self):
        return sum(self.calculateAUC(i) for i in range(self.getNumClasses())) / self.getNumClasses()

    def calculateAverageAUCPR(self):
        return sum(self.calculateAUCPR(i) for i in range(self.getNumClasses())) / self.getNumClasses()

    def stats(self):
        if self._u is None:
            return "ROCMultiClass: No data"
        rows = [f"{'Class':<15}AUC"]
        for i in range(self.getNumClasses()):
            name = self.labels[i] if self.labels else str(i)
            rows.append(f"{name:<15}{self.calculateAUC(i):.4f}")
        rows.append(f"Average AUC: {self.calculateAverageAUC():.4f}")
        return "\n".join(rows)
