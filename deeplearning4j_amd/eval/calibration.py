"""Calibration evaluation: reliability diagrams, residual and probability histograms
(reference eval/EvaluationCalibration.java:43-410). Bin counts for all bins come from one ``bucketize`` +
scatter-add per minibatch on the device instead of the reference's per-bin mask loop."""
import numpy as np
import torch

from .base import BaseEvaluation, to_2d
from .curves import Histogram, ReliabilityDiagram

DEFAULT_RELIABILITY_DIAG_NUM_BINS = 10
DEFAULT_HISTOGRAM_NUM_BINS = 50


def _bins(v, n):
    # bin j = [j/n, (j+1)/n), last bin closed at 1.0 (EvaluationCalibration.java:162-168)
    return torch.clamp((v * n).floor().long(), 0, n - 1)


class EvaluationCalibration(BaseEvaluation):
    def __init__(self, reliabilityDiagNumBins=DEFAULT_RELIABILITY_DIAG_NUM_BINS,
                 histogramNumBins=DEFAULT_HISTOGRAM_NUM_BINS, excludeEmptyBins=True):
        self.reliabilityDiagNumBins = int(reliabilityDiagNumBins)
        self.histogramNumBins = int(histogramNumBins)
        self.excludeEmptyBins = excludeEmptyBins
        self.rPos = self.rTot = self.rSum = None

    def _init(self, C):
        R, H = self.reliabilityDiagNumBins, self.histogramNumBins
        self.rPos, self.rTot, self.rSum = np.zeros((R, C)), np.zeros((R, C)), np.zeros((R, C))
        self.labelCounts, self.predCounts = np.zeros(C, dtype=np.int64), np.zeros(C, dtype=np.int64)
        self.residAll, self.residByClass = np.zeros(H, dtype=np.int64), np.zeros((H, C))
        self.probAll, self.probByClass = np.zeros(H, dtype=np.int64), np.zeros((H, C))

    def _after_load(self):
        for k in ("rPos", "rTot", "rSum", "labelCounts", "predCounts", "residAll", "residByClass", "probAll",
                  "probByClass"):
            if getattr(self, k, None) is not None:
                setattr(self, k, np.asarray(getattr(self, k)))

    def reset(self):
        self.rPos = None

    def eval(self, labels, predictions, mask=None):
        labels, preds, m2 = to_2d(labels, predictions, mask)
        y = labels.to(torch.float64)
        p = preds.to(y.device, torch.float64)
        N, C = y.shape
        if self.rPos is None:
            self._init(C)
        m = torch.ones_like(y) if m2 is None else m2.to(y.device, torch.float64).expand_as(y)
        R, H = self.reliabilityDiagNumBins, self.histogramNumBins
        col = torch.arange(C, device=y.device).expand(N, C)

        def scat(nb, bins, w):
            out = torch.zeros(nb * C, dtype=torch.float64, device=y.device)
            out.index_add_(0, (bins * C + col).reshape(-1), w.reshape(-1))
            return out.reshape(nb, C)

        rb = _bins(p, R)
        rpos, rtot, rsum = scat(R, rb, y * m), scat(R, rb, m), scat(R, rb, p * m)
        pred_idx = torch.argmax(p, dim=1)
        is_pred = torch.zeros_like(y).scatter_(1, pred_idx.unsqueeze(1), 1.0) * m
        resid = (y - p).abs()
        hb_r, hb_p = _bins(resid, H), _bins(p, H)
        res = [rpos, rtot, rsum, (y * m).sum(0), is_pred.sum(0), scat(H, hb_r, m), scat(H, hb_r, y * m),
               scat(H, hb_p, m), scat(H, hb_p, y * m)]
        res = [r.cpu().numpy() for r in res]
        self.rPos += res[0]
        self.rTot += res[1]
        self.rSum += res[2]
        self.labelCounts += res[3].astype(np.int64)
        self.predCounts += res[4].astype(np.int64)
        self.residAll += res[5].sum(1).astype(np.int64)
        self.residByClass += res[6]
        self.probAll += res[7].sum(1).astype(np.int64)
        self.probByClass += res[8]

    def merge(self, other):
        if other.rPos is None:
            return
        if self.rPos is None:
            self._init(other.rPos.shape[1])
        for k in ("rPos", "rTot", "rSum", "labelCounts", "predCounts", "residAll", "residByClass", "probAll",
                  "probByClass"):
            setattr(self, k, getattr(self, k) + getattr(other, k))

    def numClasses(self):
        return -1 if self.rPos is None else self.rPos.shape[1]

    def getReliabilityDiagram(self, classIdx):
        tot = self.rTot[:, classIdx]
        keep = tot > 0 if self.excludeEmptyBins else np.ones_like(tot, dtype=bool)
        with np.errstate(invalid="ignore", divide="ignore"):
            mean_pred = np.where(tot > 0, self.rSum[:, classIdx] / tot, 0.0)
            frac_pos = np.where(tot > 0, self.rPos[:, classIdx] / tot, 0.0)
        return ReliabilityDiagram(f"Reliability Diagram: Class {classIdx}", mean_pred[keep], frac_pos[keep])

    def getLabelCountsEachClass(self):
        return self.labelCounts.copy()

    def getPredictionCountsEachClass(self):
        return self.predCounts.copy()

    def getResidualPlotAllClasses(self):
        return Histogram("Residual Plot - All Predictions and Classes", 0.0, 1.0, self.residAll)

    def getResidualPlot(self, labelClassIdx):
        return Histogram(f"Residual Plot - Predictions for Label Class {labelClassIdx}", 0.0, 1.0,
                         self.residByClass[:, labelClassIdx].astype(np.int64))

    def getProbabilityHistogramAllClasses(self):
        return Histogram("Network Probabilities Histogram - All Predictions and Classes", 0.0, 1.0, self.probAll)

    def getProbabilityHistogram(self, labelClassIdx):
        return Histogram(f"Network Probabilities Histogram - P(class {labelClassIdx}) - Data Labelled Class "
                         f"{labelClassIdx} Only", 0.0, 1.0, self.probByClass[:, labelClassIdx].astype(np.int64))

    def stats(self):
        return "EvaluationCalibration(nClasses=" + str(self.numClasses()) + ")"
