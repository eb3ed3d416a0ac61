"""Classification evaluation (reference eval/Evaluation.java:88-1774).

Per minibatch the confusion table is built on the predictions' device with one ``bincount`` over
``actual * C + predicted`` (no per-example host loop), then accumulated on the host. TP/FP/FN/TN follow from
the table exactly as the reference's per-example increments do (Evaluation.java:366-527): for class i,
TP = C[i,i], FP = colsum - TP, FN = rowsum - TP, TN = N - TP - FP - FN.
"""
import numpy as np
import torch

from .base import BaseEvaluation, EvaluationAveraging, EvaluationUtils, to_2d
from .confusion import ConfusionMatrix

DEFAULT_EDGE_VALUE = 0.0


class Prediction:
    def __init__(self, actualClass, predictedClass, recordMetaData=None):
        self.actualClass, self.predictedClass, self.recordMetaData = actualClass, predictedClass, recordMetaData

    def getActualClass(self):
        return self.actualClass

    def getPredictedClass(self):
        return self.predictedClass

    def getRecordMetaData(self):
        return self.recordMetaData

    def __repr__(self):
        return f"Prediction(actualClass={self.actualClass},predictedClass={self.predictedClass},RecordMetaData=" \
               f"{self.recordMetaData})"


class Evaluation(BaseEvaluation):
    class Metric:
        ACCURACY, F1, PRECISION, RECALL, GMEASURE, MCC = "ACCURACY", "F1", "PRECISION", "RECALL", "GMEASURE", "MCC"

    _TRANSIENT = ("confusion", "meta")

    def __init__(self, labels=None, topN=1, binaryDecisionThreshold=None, costArray=None, binaryPositiveClass=1,
                 numClasses=None):
        if isinstance(labels, int):
            numClasses, labels = labels, None
        elif isinstance(labels, float):
            binaryDecisionThreshold, labels = labels, None
        elif torch.is_tensor(labels) or isinstance(labels, np.ndarray):
            costArray, labels = labels, None
        if isinstance(labels, dict):
            labels = [labels[i] for i in sorted(labels)]
        self.labelsList = list(labels) if labels is not None else None
        self.topN = int(topN)
        self.binaryDecisionThreshold = binaryDecisionThreshold
        self.costArray = None if costArray is None else np.asarray(torch.as_tensor(costArray).float().cpu().reshape(-1))
        self.binaryPositiveClass = binaryPositiveClass
        self.numRowCounter = 0
        self.topNCorrectCount = 0
        self.topNTotalCount = 0
        n = numClasses if numClasses is not None else (len(self.labelsList) if self.labelsList else None)
        self.table = np.zeros((n, n), dtype=np.int64) if n else None
        self.meta = {}

    def _after_load(self):
        self.table = np.asarray(self.table, dtype=np.int64) if self.table is not None else None
        if self.costArray is not None:
            self.costArray = np.asarray(self.costArray)
        self.meta = {}

    def reset(self):
        n = None if self.table is None else self.table.shape[0]
        self.numRowCounter = self.topNCorrectCount = self.topNTotalCount = 0
        self.table = np.zeros((n, n), dtype=np.int64) if n else None
        self.meta = {}

    # ------------------------------------------------------------------ accumulation
    def eval(self, trueLabels, predictions, mask=None, recordMetaData=None, network=None):
        if network is not None:           # eval(labels, input, network) form
            predictions = network.output(predictions)
        if isinstance(trueLabels, int) and isinstance(predictions, int):
            return self.evalSingle(trueLabels, predictions)
        labels, preds, _ = to_2d(trueLabels, predictions, mask)
        preds = preds.to(labels.device).float()
        labels = labels.float()
        n_rows, n_cols = labels.shape
        self.numRowCounter += n_rows
        C = 2 if n_cols == 1 else n_cols
        if self.table is None:
            self.table = np.zeros((C, C), dtype=np.int64)
            if self.labelsList is None:
                self.labelsList = [str(i) for i in range(C)]
        elif self.table.shape[0] < C:
            # e.g. Evaluation(1) fed single-column binary data: two classes (reference EvalTest
            # .testSingleClassBinaryClassification)
            grown = np.zeros((C, C), dtype=np.int64)
            n = self.table.shape[0]
            grown[:n, :n] = self.table
            self.table = grown
            if self.labelsList is not None and len(self.labelsList) < C:
                self.labelsList = list(self.labelsList) + [str(i) for i in range(len(self.labelsList), C)]
        if n_cols == 1:
            thr = 0.5 if self.binaryDecisionThreshold is None else self.binaryDecisionThreshold
            guess = (preds.reshape(-1) > thr).long()
            actual = (labels.reshape(-1) != 0).long()
        else:
            if self.binaryDecisionThreshold is not None:
                if n_cols != 2:
                    raise ValueError("Binary decision threshold is set, but number of columns for predictions is "
                                     f"{n_cols}. Binary decision threshold can only be used for binary prediction cases")
                guess = (preds[:, 1] > self.binaryDecisionThreshold).long()
            elif self.costArray is not None:
                guess = torch.argmax(preds * torch.as_tensor(self.costArray, device=preds.device), dim=1)
            else:
                guess = torch.argmax(preds, dim=1)
            actual = torch.argmax(labels, dim=1)
        counts = torch.bincount(actual * C + guess, minlength=C * C).reshape(C, C).cpu().numpy()
        self.table[:C, :C] += counts
        if recordMetaData is not None:
            a, g = actual.cpu().tolist(), guess.cpu().tolist()
            for i, m in enumerate(recordMetaData[:len(a)]):
                self.meta.setdefault((a[i], g[i]), []).append(m)
        if n_cols > 1 and self.topN > 1:
            p_true = preds.gather(1, actual.unsqueeze(1))
            greater = (preds > p_true).sum(dim=1)
            self.topNCorrectCount += int((greater < self.topN).sum().item())
            self.topNTotalCount += n_rows

    def evalSingle(self, predictedIdx, actualIdx):
        """Single prediction (reference eval(int predictedIdx, int actualIdx))."""
        if self.table is None:
            raise ValueError("Cannot evaluate single example without initializing confusion matrix first")
        self.numRowCounter += 1
        self.table[actualIdx, predictedIdx] += 1

    def merge(self, other):
        if other.table is None:
            return
        if self.table is None:
            self.table = other.table.copy()
            self.labelsList = other.labelsList
        else:
            self.table += other.table
        self.numRowCounter += other.numRowCounter
        self.topNCorrectCount += other.topNCorrectCount
        self.topNTotalCount += other.topNTotalCount
        for k, v in other.meta.items():
            self.meta.setdefault(k, []).extend(v)

    # ------------------------------------------------------------------ counts
    def numClasses(self):
        return 0 if self.table is None else self.table.shape[0]

    def _tp(self):
        return np.diag(self.table)

    def _fp(self):
        return self.table.sum(0) - self._tp()

    def _fn(self):
        return self.table.sum(1) - self._tp()

    def _tn(self):
        return self.table.sum() - self._tp() - self._fp() - self._fn()

    def truePositives(self):
        return {i: int(v) for i, v in enumerate(self._tp())}

    def falsePositives(self):
        return {i: int(v) for i, v in enumerate(self._fp())}

    def falseNegatives(self):
        return {i: int(v) for i, v in enumerate(self._fn())}

    def trueNegatives(self):
        return {i: int(v) for i, v in enumerate(self._tn())}

    def positive(self):
        return {i: int(v) for i, v in enumerate(self.table.sum(1))}

    def negative(self):
        s = self.table.sum()
        return {i: int(s - v) for i, v in enumerate(self.table.sum(1))}

    def classCount(self, c):
        return int(self.table[c].sum())

    def getNumRowCounter(self):
        return self.numRowCounter

    def getTopNCorrectCount(self):
        return self.topNCorrectCount if self.topN > 1 else int(self._tp().sum())

    def getTopNTotalCount(self):
        return self.topNTotalCount if self.topN > 1 else self.numRowCounter

    def getClassLabel(self, c):
        return self.labelsList[c] if self.labelsList and c < len(self.labelsList) else str(c)

    def getConfusionMatrix(self):
        cm = ConfusionMatrix(self.numClasses())
        cm.add_table(self.table)
        return cm

    confusion = getConfusionMatrix

    # ------------------------------------------------------------------ per-class metrics
    def _bin(self):
        return self.binaryPositiveClass is not None and self.numClasses() == 2

    def precision(self, classLabel=None, edgeCase=DEFAULT_EDGE_VALUE):
        if isinstance(classLabel, EvaluationAveraging):
            return self._avg("precision", classLabel)
        if classLabel is None:
            return self.precision(self.binaryPositiveClass) if self._bin() else self._avg("precision",
                                                                                          EvaluationAveraging.Macro)
        return EvaluationUtils.precision(int(self._tp()[classLabel]), int(self._fp()[classLabel]), edgeCase)

    def recall(self, classLabel=None, edgeCase=DEFAULT_EDGE_VALUE):
        if isinstance(classLabel, EvaluationAveraging):
            return self._avg("recall", classLabel)
        if classLabel is None:
            return self.recall(self.binaryPositiveClass) if self._bin() else self._avg("recall",
                                                                                       EvaluationAveraging.Macro)
        return EvaluationUtils.recall(int(self._tp()[classLabel]), int(self._fn()[classLabel]), edgeCase)

    def falsePositiveRate(self, classLabel=None, edgeCase=DEFAULT_EDGE_VALUE):
        if isinstance(classLabel, EvaluationAveraging):
            return self._avg("fpr", classLabel)
        if classLabel is None:
            return self.falsePositiveRate(self.binaryPositiveClass) if self._bin() else \
                self._avg("fpr", EvaluationAveraging.Macro)
        return EvaluationUtils.falsePositiveRate(int(self._fp()[classLabel]), int(self._tn()[classLabel]), edgeCase)

    def falseNegativeRate(self, classLabel=None, edgeCase=DEFAULT_EDGE_VALUE):
        if isinstance(classLabel, EvaluationAveraging):
            return self._avg("fnr", classLabel)
        if classLabel is None:
            return self.falseNegativeRate(self.binaryPositiveClass) if self._bin() else \
                self._avg("fnr", EvaluationAveraging.Macro)
        return EvaluationUtils.falseNegativeRate(int(self._fn()[classLabel]), int(self._tp()[classLabel]), edgeCase)

    def falseAlarmRate(self):
        return (self.falsePositiveRate() + self.falseNegativeRate()) / 2.0

    def fBeta(self, beta, classLabel=None, defaultValue=0.0):
        if isinstance(classLabel, EvaluationAveraging):
            return self._avg_fbeta(beta, classLabel)
        if classLabel is None:
            return self._avg_fbeta(beta, EvaluationAveraging.Macro)
        p, r = self.precision(classLabel, -1), self.recall(classLabel, -1)
        if p == -1 or r == -1:
            return defaultValue
        return EvaluationUtils.fBeta(beta, p, r)

    def f1(self, classLabel=None):
        if classLabel is None and self._bin():
            return self.fBeta(1.0, self.binaryPositiveClass)
        return self.fBeta(1.0, classLabel)

    def gMeasure(self, x=EvaluationAveraging.Macro):
        if isinstance(x, EvaluationAveraging):
            n = self.numClasses()
            if x == EvaluationAveraging.Macro:
                return sum(self.gMeasure(i) for i in range(n)) / n
            tp, fp, fn = int(self._tp().sum()), int(self._fp().sum()), int(self._fn().sum())
            return EvaluationUtils.gMeasure(EvaluationUtils.precision(tp, fp), EvaluationUtils.recall(tp, fn))
        return EvaluationUtils.gMeasure(self.precision(x), self.recall(x))

    def matthewsCorrelation(self, x=EvaluationAveraging.Macro):
        if isinstance(x, EvaluationAveraging):
            n = self.numClasses()
            if x == EvaluationAveraging.Macro:
                return sum(self.matthewsCorrelation(i) for i in range(n)) / n
            return EvaluationUtils.matthewsCorrelation(int(self._tp().sum()), int(self._fp().sum()),
                                                       int(self._fn().sum()), int(self._tn().sum()))
        return EvaluationUtils.matthewsCorrelation(int(self._tp()[x]), int(self._fp()[x]), int(self._fn()[x]),
                                                   int(self._tn()[x]))

    def accuracy(self):
        if self.numRowCounter == 0:
            return 0.0
        return float(np.trace(self.table)) / self.numRowCounter

    def topNAccuracy(self):
        if self.topN <= 1:
            return self.accuracy()
        return 0.0 if self.topNTotalCount == 0 else self.topNCorrectCount / float(self.topNTotalCount)

    def _avg(self, what, averaging):
        if self.numRowCounter == 0:
            return 0.0
        n = self.numClasses()
        fn = {"precision": self.precision, "recall": self.recall, "fpr": self.falsePositiveRate,
              "fnr": self.falseNegativeRate}[what]
        if averaging == EvaluationAveraging.Macro:
            vals = [fn(i, -1) for i in range(n)]
            vals = [v for v in vals if v != -1]
            return sum(vals) / len(vals) if vals else 0.0
        tp, fp, fnn, tn = int(self._tp().sum()), int(self._fp().sum()), int(self._fn().sum()), int(self._tn().sum())
        if what == "precision":
            return EvaluationUtils.precision(tp, fp)
        if what == "recall":
            return EvaluationUtils.recall(tp, fnn)
        if what == "fpr":
            return EvaluationUtils.falsePositiveRate(fp, tn)
        return EvaluationUtils.falseNegativeRate(fnn, tp)

    def _avg_fbeta(self, beta, averaging):
        if self.numRowCounter == 0:
            return float("nan")
        n = self.numClasses()
        if n == 2:
            return EvaluationUtils.fBeta(beta, int(self._tp()[1]), int(self._fp()[1]), int(self._fn()[1]))
        if averaging == EvaluationAveraging.Macro:
            vals = [self.fBeta(beta, i, -1) for i in range(n)]
            vals = [v for v in vals if v != -1]
            return sum(vals) / len(vals) if vals else 0.0
        return EvaluationUtils.fBeta(beta, int(self._tp().sum()), int(self._fp().sum()), int(self._fn().sum()))

    def _excluded(self, what):
        n = self.numClasses()
        if what == "precision":
            return sum(1 for i in range(n) if self.precision(i, -1) == -1)
        if what == "recall":
            return sum(1 for i in range(n) if self.recall(i, -1) == -1)
        return sum(1 for i in range(n) if self.fBeta(1.0, i, -1) == -1)

    def averagePrecisionNumClassesExcluded(self):
        return self._excluded("precision")

    def averageRecallNumClassesExcluded(self):
        return self._excluded("recall")

    def averageF1NumClassesExcluded(self):
        return self._excluded("f1")

    averageFBetaNumClassesExcluded = averageF1NumClassesExcluded

    def scoreForMetric(self, metric):
        m = metric if isinstance(metric, str) else getattr(metric, "name", str(metric))
        return {"ACCURACY": self.accuracy, "F1": self.f1, "PRECISION": self.precision, "RECALL": self.recall,
                "GMEASURE": self.gMeasure, "MCC": self.matthewsCorrelation}[m]()

    # ------------------------------------------------------------------ predictions / metadata
    def getPredictionErrors(self):
        out = []
        for (a, p), ms in sorted(self.meta.items()):
            if a != p:
                out += [Prediction(a, p, m) for m in ms]
        return out

    def getPredictionsByActualClass(self, actual):
        return [Prediction(a, p, m) for (a, p), ms in sorted(self.meta.items()) if a == actual for m in ms]

    def getPredictionByPredictedClass(self, predicted):
        return [Prediction(a, p, m) for (a, p), ms in sorted(self.meta.items()) if p == predicted for m in ms]

    def getPredictions(self, actual, predicted):
        return [Prediction(actual, predicted, m) for m in self.meta.get((actual, predicted), [])]

    # ------------------------------------------------------------------ reporting
    def confusionToString(self):
        n = self.numClasses()
        w = max([len(self.getClassLabel(i)) for i in range(n)] + [5])
        head = " " * (w + 3) + " ".join(f"{i:>6d}" for i in range(n))
        rows = [head]
        for i in range(n):
            rows.append(f"{i:>3d} {self.getClassLabel(i):<{w}} " + " ".join(f"{int(v):>6d}" for v in self.table[i]))
        return "\n".join(rows)

    def stats(self, suppressWarnings=False):
        if self.table is None or self.numRowCounter == 0:
            return "Evaluation: No data available (no evaluation has been performed)"
        n = self.numClasses()
        lines = []
        for a in range(n):
            for p in range(n):
                c = int(self.table[a, p])
                if c:
                    lines.append(f"Predictions labeled as {self.getClassLabel(a)} classified by model as "
                                 f"{self.getClassLabel(p)}: {c} times")
        warn = []
        if not suppressWarnings:
            never = [i for i in range(n) if int(self.table[:, i].sum()) == 0]
            if never:
                warn.append(f"Warning: {len(never)} class{'es were' if len(never) > 1 else ' was'} never predicted "
                            "by the model and w" + ("ere" if len(never) > 1 else "as") +
                            " excluded from average precision")
                warn.append("Classes excluded from average precision: " + str(never))
        out = ["", *lines, "", *warn, "", "==========================Scores========================================",
               f" # of classes:    {n}", f" Accuracy:        {self.accuracy():.4f}"]
        if self.topN > 1:
            out.append(f" Top {self.topN} Accuracy:  {self.topNAccuracy():.4f}")
        out += [f" Precision:       {self.precision():.4f}", f" Recall:          {self.recall():.4f}",
                f" F1 Score:        {self.f1():.4f}"]
        if self._bin():
            out.append(f"Precision, recall & F1: reported for positive class (class {self.binaryPositiveClass}"
                       f" - \"{self.getClassLabel(self.binaryPositiveClass)}\") only")
        else:
            out.append("Precision, recall & F1: macro-averaged (equally weighted avg. of " + str(n) + " classes)")
        out += ["", "", "=========================Confusion Matrix=========================", self.confusionToString(),
                "", "Confusion matrix format: Actual (rowClass) predicted as (columnClass) N times",
                "=================================================================="]
        return "\n".join(out)
