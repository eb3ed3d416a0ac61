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

    def getPointAtThreshold(self, t):
        i = int(np.argmin(np.abs(self.threshold - t)))
        return i, float(self.threshold[i]), float(self.precision[i]), float(self.recall[i])

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
