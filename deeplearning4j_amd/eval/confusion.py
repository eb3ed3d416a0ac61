"""ConfusionMatrix (reference eval/ConfusionMatrix.java) backed by a dense int64 count table."""
import numpy as np


class ConfusionMatrix:
    def __init__(self, classes=None):
        if isinstance(classes, int):
            classes = list(range(classes))
        self.classes = list(classes or [])
        self.m = np.zeros((len(self.classes), len(self.classes)), dtype=np.int64)

    def _grow(self, n):
        if n > len(self.classes):
            m = np.zeros((n, n), dtype=np.int64)
            k = len(self.classes)
            m[:k, :k] = self.m
            self.m = m
            self.classes = list(range(n))

    def add(self, actual, predicted, count=1):
        if isinstance(actual, ConfusionMatrix):
            other = actual
            self._grow(len(other.classes))
            self.m[:other.m.shape[0], :other.m.shape[1]] += other.m
            return
        self._grow(max(actual, predicted) + 1)
        self.m[actual, predicted] += count

    def add_table(self, table):
        self._grow(table.shape[0])
        self.m[:table.shape[0], :table.shape[1]] += table

    def getCount(self, actual, predicted):
        return int(self.m[actual, predicted])

    def getPredictedTotal(self, predicted):
        return int(self.m[:, predicted].sum())

    def getActualTotal(self, actual):
        return int(self.m[actual, :].sum())

    def getClasses(self):
        return list(self.classes)

    def toCSV(self):
        n = len(self.classes)
        lines = [",," + "Predicted:", "," + ",".join(str(c) for c in self.classes) + ",Total"]
        for i in range(n):
            lines.append(("Actual:" if i == 0 else "") + f",{self.classes[i]}," +
                         ",".join(str(int(x)) for x in self.m[i]) + f",{int(self.m[i].sum())}")
        lines.append(",Total," + ",".join(str(int(x)) for x in self.m.sum(0)))
        return "\n".join(lines)

    def __str__(self):
        return self.toCSV()

    def __eq__(self, other):
        return isinstance(other, ConfusionMatrix) and np.array_equal(self.m, other.m)
