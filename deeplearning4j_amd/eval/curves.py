"""ROC / precision-recall curves, histograms and reliability diagrams (reference eval/curves/*)."""
import json

import numpy as np


def _area(x, y):
    """Trapezoid area in threshold order (reference curves/BaseCurve.java:45-63)."""
    x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
    if len(x) < 2:
        return 0.0
    return float(np.sum(np.abs(np.diff(x)) * (y[1:] + y[:-1]) / 2.0))


class BaseCurve:
    def numPoints(self):
        return len(self.threshold)

    def getThreshold(self, i):
        return float(self.threshold[i])

    def toJson(self):
        return json.dumps({"@class": type(self).__name__,
                           **{k: (np.asarray(v).tolist() if isinstance(v, (np.ndarray, list)) else v)
                              for k, v in self.__dict__.items()}})

    @staticmethod
    def fromJson(s):
        d = json.loads(s)
        cls = {"RocCurve": RocCurve, "PrecisionRecallCurve": PrecisionRecallCurve}[d.pop("@class")]
        obj = cls.__new__(cls)
        obj.__dict__.update({k: (np.asarray(v) if isinstance(v, list) else v) for k, v in d.items()})
        return obj


class RocCurve(BaseCurve):
    def __init__(self, threshold, fpr, tpr):
        self.threshold, self.fpr, self.tpr = np.asarray(threshold), np.asarray(fpr), np.asarray(tpr)

    def getX(self):
        return self.fpr

    def getY(self):
        return self.tpr

    def getFalsePositiveRate(self, i):
        return float(self.fpr[i])

    def getTruePositiveRate(self, i):
        return float(self.tpr[i])

    def calculateAUC(self):
        return _area(self.fpr, self.tpr)

    def getTitle(self):
        return f"ROC (Area={self.calculateAUC():.4f})"


class PrecisionRecallCurve(BaseCurve):
    def __init__(self, threshold, precision, recall, tpCount=None, fpCount=None, fnCount=None, totalCount=None):
        self.threshold, self.precision, self.recall = np.asarray(threshold), np.asarray(precision), np.asarray(recall)
        self.tpCount = None if tpCount is None else np.asarray(tpCount)
        self.fpCount = None if fpCount is None else np.asarray(fpCount)
        self.fnCount = None if fnCount is None else np.asarray(fnCount)
        self.totalCount = totalCount

    def getX(self):
        return self.recall

    def getY(self):
        return self.precision

    def getPrecision(self, i):
        return float(self.precision[i])

    def getRecall(self, i):
        return float(self.recall[i])

    def calculateAUPRC(self):
        return _area(self.recall, self.precision)

    class Point:
        def __init__(self, idx, threshold, precision, recall):
            self.idx, self.threshold, self.precision, self.recall = int(idx), float(threshold), float(precision), \
                float(recall)

        def getIdx(self):
            return self.idx

        def getThreshold(self):
            return self.threshold

        def getPrecision(self):
            return self.precision

        def getRecall(self):
            return self.recall

    class Confusion:
        def __init__(self, point, tp, fp, fn, tn):
            self.point, self.tp, self.fp, self.fn, self.tn = point, int(tp), int(fp), int(fn), int(tn)

        def getPoint(self):
            return self.point

        def getTpCount(self):
            return self.tp

        def getFpCount(self):
            return self.fp

        def getFnCount(self):
            return self.fn

        def getTnCount(self):
            return self.tn

    def _pt(self, i):
        return PrecisionRecallCurve.Point(i, self.threshold[i], self.precision[i], self.recall[i])

    def getPointAtThreshold(self, t):
        """First point whose threshold is >= t (thresholds ascend), the last one when t is above all of them."""
        # thresholds within 1e-9 count as equal (i * 0.1 vs i / 10 step arithmetic)
        i = int(np.searchsorted(self.threshold, t - 1e-9, side="left"))
        return self._pt(min(i, len(self.threshold) - 1))

    def getPointAtPrecision(self, p):
        """First point (lowest threshold) reaching precision p, else the last point."""
        hit = np.nonzero(self.precision >= p)[0]
        return self._pt(int(hit[0]) if hit.size else len(self.threshold) - 1)

    def getPointAtRecall(self, r):
        """Among the points with recall >= r: the highest-threshold one, preferring higher precision at equal
        recall; the first point when none reaches r."""
        found = None
        for i in range(len(self.recall) - 1, -1, -1):
            if self.recall[i] >= r and (found is None or (self.recall[i] == found.recall and
                                                          self.precision[i] >= found.precision)):
                found = self._pt(i)
        return found if found is not None else self._pt(0)

    def getConfusionMatrixAtThreshold(self, t):
        if self.tpCount is None:
            raise ValueError("this curve was built without confusion counts")
        p = self.getPointAtThreshold(t)
        i = p.idx
        tn = self.totalCount - (self.tpCount[i] + self.fpCount[i] + self.fnCount[i])
        return PrecisionRecallCurve.Confusion(p, self.tpCount[i], self.fpCount[i], self.fnCount[i], tn)

    def getConfusionMatrixAtPoint(self, i):
        return self.getConfusionMatrixAtThreshold(self.threshold[i])

    def getTitle(self):
        return f"Precision-Recall Curve (Area={self.calculateAUPRC():.4f})"


class Histogram:
    def __init__(self, title, lower, upper, binCounts):
        self.title, self.lower, self.upper = title, float(lower), float(upper)
        self.binCounts = np.asarray(binCounts, dtype=np.int64)

    def numPoints(self):
        return len(self.binCounts)

    def getBinLowerBounds(self):
        n = len(self.binCounts)
        return np.linspace(self.lower, self.upper, n + 1)[:-1]

    def getBinUpperBounds(self):
        n = len(self.binCounts)
        return np.linspace(self.lower, self.upper, n + 1)[1:]

    def getBinMidValues(self):
        return (self.getBinLowerBounds() + self.getBinUpperBounds()) / 2

    def getTitle(self):
        return self.title


class ReliabilityDiagram:
    def __init__(self, title, meanPredictedValueX, fractionPositivesY):
        self.title = title
        self.meanPredictedValueX = np.asarray(meanPredictedValueX)
        self.fractionPositivesY = np.asarray(fractionPositivesY)

    def getTitle(self):
        return self.title
