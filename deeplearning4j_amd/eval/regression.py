"""Regression evaluation (reference eval/RegressionEvaluation.java: per-column running sums -> MSE, MAE, RMSE,
RSE, Pearson correlation, R^2; formulas at :328-410). Sums are float64 and reduced on the device."""
import numpy as np
import torch

from .base import BaseEvaluation, to_2d

EPS_THRESHOLD = 1e-5


class RegressionEvaluation(BaseEvaluation):
    class Metric:
        MSE, MAE, RMSE, RSE, PC, R2 = "MSE", "MAE", "RMSE", "RSE", "PC", "R2"

    def __init__(self, columnNames=None, precision=5):
        if isinstance(columnNames, int):
            columnNames = [f"col_{i}" for i in range(columnNames)]
        self.columnNames = list(columnNames) if columnNames is not None else None
        self.precision = precision
        self._zero(None if columnNames is None else len(self.columnNames))

    def _zero(self, n):
        z = (lambda: np.zeros(n, dtype=np.float64)) if n else (lambda: None)
        self.sumSquaredErrors, self.sumAbsErrors, self.sumLabels, self.sumPredicted = z(), z(), z(), z()
        self.sumSquaredLabels, self.sumSquaredPredicted, self.sumOfProducts, self.count = z(), z(), z(), z()

    def _after_load(self):
        for k in ("sumSquaredErrors", "sumAbsErrors", "sumLabels", "sumPredicted", "sumSquaredLabels",
                  "sumSquaredPredicted", "sumOfProducts", "count"):
            v = getattr(self, k)
            if v is not None:
                setattr(self, k, np.asarray(v, dtype=np.float64))

    def reset(self):
        self._zero(None if self.count is None else len(self.count))

    def eval(self, labels, predictions, mask=None):
        labels, preds, m2 = to_2d(labels, predictions, mask)
        y = labels.to(torch.float64)
        p = preds.to(y.device, torch.float64)
        m = torch.ones_like(y) if m2 is None else m2.to(y.device, torch.float64).expand_as(y)
        n = y.shape[1]
        if self.count is None:
            self._zero(n)
            if self.columnNames is None:
                self.columnNames = [f"col_{i}" for i in range(n)]
        d = (p - y) * m
        stats = torch.stack([(d * d).sum(0), d.abs().sum(0), (y * m).sum(0), (p * m).sum(0), (y * y * m).sum(0),
                             (p * p * m).sum(0), (y * p * m).sum(0), m.sum(0)]).cpu().numpy()
        self.sumSquaredErrors += stats[0]
        self.sumAbsErrors += stats[1]
        self.sumLabels += stats[2]
        self.sumPredicted += stats[3]
        self.sumSquaredLabels += stats[4]
        self.sumSquaredPredicted += stats[5]
        self.sumOfProducts += stats[6]
        self.count += stats[7]

    def merge(self, other):
        if other.count is None:
            return
        if self.count is None:
            self.__dict__.update({k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in other.__dict__.items()})
            return
        for k in ("sumSquaredErrors", "sumAbsErrors", "sumLabels", "sumPredicted", "sumSquaredLabels",
                  "sumSquaredPredicted", "sumOfProducts", "count"):
            setattr(self, k, getattr(self, k) + getattr(other, k))

    def numColumns(self):
        return 0 if self.count is None else len(self.count)

    def meanSquaredError(self, c):
        return self.sumSquaredErrors[c] / self.count[c]

    def meanAbsoluteError(self, c):
        return self.sumAbsErrors[c] / self.count[c]

    def rootMeanSquaredError(self, c):
        return float(np.sqrt(self.meanSquaredError(c)))

    def _means(self, c):
        return self.sumLabels[c] / self.count[c], self.sumPredicted[c] / self.count[c]

    def pearsonCorrelation(self, c):
        lm, pm = self._means(c)
        n = self.count[c]
        r = self.sumOfProducts[c] - n * pm * lm
        r /= np.sqrt(self.sumSquaredLabels[c] - n * lm * lm) * np.sqrt(self.sumSquaredPredicted[c] - n * pm * pm)
        return float(r)

    correlationR2 = pearsonCorrelation

    def rSquared(self, c):
        lm, _ = self._means(c)
        n = self.count[c]
        sstot = self.sumSquaredLabels[c] + lm * (n * lm - 2 * self.sumLabels[c])
        return float((sstot - self.sumSquaredErrors[c]) / sstot)

    def relativeSquaredError(self, c):
        lm, _ = self._means(c)
        num = self.sumSquaredPredicted[c] - 2 * self.sumOfProducts[c] + self.sumSquaredLabels[c]
        den = self.sumSquaredLabels[c] - self.count[c] * lm * lm
        return float(num / den) if abs(den) > EPS_THRESHOLD else float("inf")

    def _avg(self, f):
        n = self.numColumns()
        return sum(f(i) for i in range(n)) / n

    def averageMeanSquaredError(self):
        return self._avg(self.meanSquaredError)

    def averageMeanAbsoluteError(self):
        return self._avg(self.meanAbsoluteError)

    def averagerootMeanSquaredError(self):
        return self._avg(self.rootMeanSquaredError)

    def averagerelativeSquaredError(self):
        return self._avg(self.relativeSquaredError)

    def averagePearsonCorrelation(self):
        return self._avg(self.pearsonCorrelation)

    averagecorrelationR2 = averagePearsonCorrelation

    def averageRSquared(self):
        return self._avg(self.rSquared)

    def scoreForMetric(self, metric):
        m = metric if isinstance(metric, str) else getattr(metric, "name", str(metric))
        return {"MSE": self.averageMeanSquaredError, "MAE": self.averageMeanAbsoluteError,
                "RMSE": self.averagerootMeanSquaredError, "RSE": self.averagerelativeSquaredError,
                "PC": self.averagePearsonCorrelation, "R2": self.averageRSquared}[m]()

    def stats(self):
        if self.count is None:
            return "RegressionEvaluation: No Data"
        w = max([len(c) for c in self.columnNames] + [6]) + 4
        p = self.precision
        head = f"{'Column':<{w}}" + "".join(f"{h:<{p + 8}}" for h in
                                             ["MSE", "MAE", "RMSE", "RSE", "PC", "R^2"])
        rows = [head]
        for i, c in enumerate(self.columnNames):
            vals = [self.meanSquaredError(i), self.meanAbsoluteError(i), self.rootMeanSquaredError(i),
                    self.relativeSquaredError(i), self.pearsonCorrelation(i), self.rSquared(i)]
            rows.append(f"{c:<{w}}" + "".join(f"{v:<{p + 8}.{p}e}" for v in vals))
        return "\n".join(rows)
