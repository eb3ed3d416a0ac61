"""Fixed-count value histogram for the weights UI (reference deeplearning4j-ui/src/main/java/org/deeplearning4j/ui/
weights/HistogramBin.java): numberOfBins bins between the array's min and max, bin width (max - min) / (bins - 1),
bin keys = the bin's lower edge rounded UP to ``rounds`` decimals; out-of-range positions clamp to the end bins."""
import decimal

import torch


class HistogramBin:
    def __init__(self):
        self.numberOfBins, self.rounds = 0, 2
        self.min = self.max = 0.0
        self.bins = None
        self.data = {}

    def _calc(self, source):
        t = torch.as_tensor(getattr(source, "tensor", source)).detach().reshape(-1).double().cpu()
        f32max, f32min = 3.4028234663852886e38, 1.401298464324817e-45
        mx, mn = float(t.max()), float(t.min())
        fix = lambda v, inf_v, nan_v: inf_v if v in (float("inf"), float("-inf")) else (nan_v if v != v else v)  # noqa
        self.max, self.min = fix(mx, f32max, f32min), fix(mn, f32max, f32min)
        n = self.numberOfBins
        size = (self.max - self.min) / (n - 1)
        q = decimal.Decimal(1).scaleb(-self.rounds)
        keys = [decimal.Decimal(self.min + x * size).quantize(q, rounding=decimal.ROUND_CEILING) for x in range(n)]
        self.data = {k: 0 for k in keys}
        counts = [0] * n
        for d in t.tolist():
            b = int((d - self.min) / size) if size != 0 else 0
            b = 0 if b < 0 else (n - 1 if b >= n else b)
            counts[b] += 1
            self.data[keys[b]] += 1
        self.bins = torch.tensor(counts, dtype=torch.float64)

    def getMin(self):
        return self.min

    def getMax(self):
        return self.max

    def getBins(self):
        return self.bins

    def getData(self):
        return self.data

    class Builder:
        def __init__(self, array):
            self.source, self.binCount, self.rounds = array, 0, 2

        def setRounding(self, rounds):
            self.rounds = int(rounds)
            return self

        def setBinCount(self, bins):
            self.binCount = int(bins)
            return self

        def build(self):
            h = HistogramBin()
            h.numberOfBins, h.rounds = self.binCount, self.rounds
            h._calc(self.source)
            return h
