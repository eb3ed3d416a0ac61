"""Ranked classification results (reference deeplearning4j-nn/src/main/java/org/deeplearning4j/nn/simple/multiclass/
RankClassificationResult.java): per row of a [rows, classes] outcome matrix, the class indices sorted by descending
score and the label of the best one ("0", "1", ... unless labels are given)."""
import torch

from ..exceptions import IllegalStateException


class RankClassificationResult:
    def __init__(self, outcome, labels=None):
        t = torch.as_tensor(getattr(outcome, "tensor", outcome)).detach().to("cpu", torch.float32)
        if t.dim() > 2:
            raise IllegalStateException("Only works with vectors and matrices right now")
        if t.dim() < 2:
            t = t.reshape(1, -1)
        self.labels = [str(i) for i in range(t.shape[1])] if labels is None else list(labels)
        # stable descending sort: ties keep the lower class index first
        self.rankedIndices = torch.sort(t, dim=1, descending=True, stable=True).indices.tolist()
        self.probabilities = t.tolist()
        self.maxLabels = None
        self.maxOutcomes()

    def getLabels(self):
        return self.labels

    def getRankedIndices(self):
        return self.rankedIndices

    def getProbabilities(self):
        return self.probabilities

    def maxOutcomeForRow(self, r):
        return self.labels[self.rankedIndices[r][0]]

    def maxOutcomes(self):
        if self.maxLabels is None:
            self.maxLabels = [self.maxOutcomeForRow(i) for i in range(len(self.rankedIndices))]
        return self.maxLabels
