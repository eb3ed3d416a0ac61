"""Data normalizers (DataSetPreProcessor + fit/transform/revert), as used by iterators and stored in model zips.

The reference takes these from ND4J (`org.nd4j.linalg.dataset.api.preprocessor.*`), e.g. used in
`NN:util/ModelSerializer.java:690` (addNormalizerToModel) and the iterator tests. Semantics kept:
  * NormalizerStandardize: per-feature mean/std over all examples (and time steps / spatial positions for
    3d/4d data); x' = (x - mean) / std, std clamped at 1e-8 (ND4J Nd4j.EPS_THRESHOLD). Optional label fit.
  * NormalizerMinMaxScaler: x' = (x - min)/(max - min) * (hi - lo) + lo.
  * ImagePreProcessingScaler: pixels in [0, 2^bits - 1] -> [lo, hi].
  * VGG16ImagePreProcessor: subtract the ImageNet channel means (103.939, 116.779, 123.68) in BGR order.
Statistics are accumulated in float64 in one streaming pass (sum / sum of squares per batch), so fitting on
an iterator never materialises the whole dataset.
Serialization: a small self-describing binary ("DL4JAMD-NORM" + JSON header + raw little-endian float64).
"""
import json
import struct

import torch

_MAGIC = b"DL4JAMD-NORM\x01"
EPS = 1e-8


def _reduce_dims(x):
    # features [N, F] -> dim 0; [N, F, T] -> (0, 2); [N, C, H, W] -> (0, 2, 3)
    return (0,) if x.dim() == 2 else tuple([0] + list(range(2, x.dim())))


def _bshape(x, v):
    shape = [1, v.numel()] + [1] * (x.dim() - 2)
    return v.reshape(shape).to(device=x.device, dtype=torch.float64)


class _Stats:
    """Streaming per-feature count/sum/sumsq/min/max."""

    def __init__(self):
        self.n = 0
        self.s = self.ss = self.mn = self.mx = None

    def add(self, x, mask=None):
        x = x.detach().to(torch.float64)
        dims = _reduce_dims(x)
        if mask is not None and x.dim() == 3:
            m = mask.detach().to(torch.float64).unsqueeze(1)
            cnt = m.sum().item()
            s = (x * m).sum(dim=dims)
            ss = (x * x * m).sum(dim=dims)
            big = torch.finfo(torch.float64).max
            mn = torch.where(m > 0, x, torch.full_like(x, big)).amin(dim=dims)
            mx = torch.where(m > 0, x, torch.full_like(x, -big)).amax(dim=dims)
        else:
            cnt = x.numel() // x.shape[1]
            s, ss = x.sum(dim=dims), (x * x).sum(dim=dims)
            mn, mx = x.amin(dim=dims), x.amax(dim=dims)
        s, ss, mn, mx = s.cpu(), ss.cpu(), mn.cpu(), mx.cpu()
        if self.s is None:
            self.s, self.ss, self.mn, self.mx = s, ss, mn, mx
        else:
            self.s, self.ss = self.s + s, self.ss + ss
            self.mn, self.mx = torch.minimum(self.mn, mn), torch.maximum(self.mx, mx)
        self.n += cnt

    def mean(self):
        return self.s / max(self.n, 1)

    def std(self):
        m = self.mean()
        var = (self.ss / max(self.n, 1) - m * m).clamp_min(0)
        return var.sqrt()


def _iter_datasets(data):
    from .dataset import DataSet
    if isinstance(data, DataSet):
        yield data
        return
    if hasattr(data, "reset") and getattr(data, "resetSupported", lambda: True)():
        data.reset()
    while data.hasNext():
        yield data.next()
    if hasattr(data, "reset") and getattr(data, "resetSupported", lambda: True)():
        data.reset()


class DataNormalization:
    """Base: fit(DataSet | DataSetIterator), preProcess(ds) in place, transform(features), revert*."""
    TYPE = None
    _REG = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        if cls.TYPE:
            DataNormalization._REG[cls.TYPE] = cls

    fitLabels = False

    def fitLabel(self, b):
        self.fitLabels = bool(b)
        return self

    def isFitLabel(self):
        return self.fitLabels

    # -- subclass hooks
    def _fit_stats(self, fs, ls):
        raise NotImplementedError

    def _tf(self, x, which):
        raise NotImplementedError

    def _rev(self, x, which):
        raise NotImplementedError

    def fit(self, data):
        fs, ls = _Stats(), _Stats()
        for ds in _iter_datasets(data):
            fs.add(ds.getFeatures(), ds.getFeaturesMaskArray())
            if self.fitLabels and ds.getLabels() is not None:
                ls.add(ds.getLabels(), ds.getLabelsMaskArray())
        self._fit_stats(fs, ls if self.fitLabels else None)
        return self

    def preProcess(self, ds):
        ds.features = self.transform(ds.getFeatures())
        if self.fitLabels and ds.getLabels() is not None:
            ds.labels = self.transformLabel(ds.getLabels())

    __call__ = preProcess

    def transform(self, x):
        if hasattr(x, "getFeatures"):
            self.preProcess(x)
            return x
        return self._tf(x, "f")

    def transformLabel(self, y):
        return self._tf(y, "l")

    def revert(self, ds):
        ds.features = self.revertFeatures(ds.getFeatures())
        if self.fitLabels and ds.getLabels() is not None:
            ds.labels = self.revertLabels(ds.getLabels())

    def revertFeatures(self, x):
        return self._rev(x, "f")

    def revertLabels(self, y):
        return self._rev(y, "l")

    # -- serialization
    def _state(self):
        return {}, {}

    def _load(self, meta, arrays):
        pass

    def to_bytes(self):
        meta, arrays = self._state()
        names = sorted(k for k, v in arrays.items() if v is not None)
        header = {"type": self.TYPE, "fitLabels": self.fitLabels, "meta": meta,
                  "arrays": [[k, int(arrays[k].numel())] for k in names]}
        hb = json.dumps(header).encode()
        out = [_MAGIC, struct.pack("<I", len(hb)), hb]
        for k in names:
            out.append(arrays[k].detach().to(torch.float64).cpu().contiguous().numpy().astype("<f8").tobytes())
        return b"".join(out)

    @staticmethod
    def from_bytes(b):
        import numpy as np
        if not b.startswith(_MAGIC):
            raise ValueError("not a deeplearning4j_amd normalizer blob")
        off = len(_MAGIC)
        (hl,) = struct.unpack_from("<I", b, off)
        off += 4
        header = json.loads(b[off:off + hl].decode())
        off += hl
        arrays = {}
        for k, n in header["arrays"]:
            arrays[k] = torch.from_numpy(np.frombuffer(b, dtype="<f8", count=n, offset=off).copy())
            off += 8 * n
        cls = DataNormalization._REG[header["type"]]
        obj = cls.__new__(cls)
        DataNormalization.__init__(obj)
        obj.fitLabels = header["fitLabels"]
        obj._load(header["meta"], arrays)
        return obj

    def __eq__(self, other):
        if type(self) is not type(other):
            return False
        return self.to_bytes() == other.to_bytes()


class NormalizerStandardize(DataNormalization):
    TYPE = "STANDARDIZE"

    def __init__(self, featureMean=None, featureStd=None, labelMean=None, labelStd=None):
        self.fMean, self.fStd, self.lMean, self.lStd = featureMean, featureStd, labelMean, labelStd
        if labelMean is not None:
            self.fitLabels = True

    def _fit_stats(self, fs, ls):
        self.fMean, self.fStd = fs.mean(), fs.std().clamp_min(EPS)
        if ls is not None and ls.s is not None:
            self.lMean, self.lStd = ls.mean(), ls.std().clamp_min(EPS)

    def _ms(self, which):
        return (self.fMean, self.fStd) if which == "f" else (self.lMean, self.lStd)

    def _tf(self, x, which):
        m, s = self._ms(which)
        return ((x.to(torch.float64) - _bshape(x, m)) / _bshape(x, s)).to(x.dtype)

    def _rev(self, x, which):
        m, s = self._ms(which)
        return (x.to(torch.float64) * _bshape(x, s) + _bshape(x, m)).to(x.dtype)

    def getMean(self):
        return self.fMean

    def getStd(self):
        return self.fStd

    def getLabelMean(self):
        return self.lMean

    def getLabelStd(self):
        return self.lStd

    def _state(self):
        return {}, {"fMean": self.fMean, "fStd": self.fStd, "lMean": self.lMean, "lStd": self.lStd}

    def _load(self, meta, a):
        self.fMean, self.fStd, self.lMean, self.lStd = a.get("fMean"), a.get("fStd"), a.get("lMean"), a.get("lStd")


class NormalizerMinMaxScaler(DataNormalization):
    TYPE = "MIN_MAX"

    def __init__(self, minRange=0.0, maxRange=1.0):
        self.lo, self.hi = float(minRange), float(maxRange)
        self.fMin = self.fMax = self.lMin = self.lMax = None

    def _fit_stats(self, fs, ls):
        self.fMin, self.fMax = fs.mn, fs.mx
        if ls is not None and ls.s is not None:
            self.lMin, self.lMax = ls.mn, ls.mx

    def _mm(self, which):
        return (self.fMin, self.fMax) if which == "f" else (self.lMin, self.lMax)

    def _tf(self, x, which):
        mn, mx = self._mm(which)
        rng = (mx - mn).clamp_min(EPS)
        y = (x.to(torch.float64) - _bshape(x, mn)) / _bshape(x, rng)
        return (y * (self.hi - self.lo) + self.lo).to(x.dtype)

    def _rev(self, x, which):
        mn, mx = self._mm(which)
        rng = (mx - mn).clamp_min(EPS)
        y = (x.to(torch.float64) - self.lo) / (self.hi - self.lo)
        return (y * _bshape(x, rng) + _bshape(x, mn)).to(x.dtype)

    def getMin(self):
        return self.fMin

    def getMax(self):
        return self.fMax

    def getTargetMin(self):
        return self.lo

    def getTargetMax(self):
        return self.hi

    def _state(self):
        return {"lo": self.lo, "hi": self.hi}, {"fMin": self.fMin, "fMax": self.fMax, "lMin": self.lMin,
                                                "lMax": self.lMax}

    def _load(self, meta, a):
        self.lo, self.hi = meta["lo"], meta["hi"]
        self.fMin, self.fMax, self.lMin, self.lMax = a.get("fMin"), a.get("fMax"), a.get("lMin"), a.get("lMax")


class ImagePreProcessingScaler(DataNormalization):
    """Stateless pixel scaler: [0, 2^bits-1] -> [a, b] (fit is a no-op)."""
    TYPE = "IMAGE_MIN_MAX"

    def __init__(self, a=0.0, b=1.0, maxBits=8):
        self.lo, self.hi, self.maxBits = float(a), float(b), int(maxBits)
        self.maxPixelVal = float(2 ** self.maxBits - 1)

    def fit(self, data):
        return self

    def _tf(self, x, which):
        if which == "l":
            return x
        return (x / self.maxPixelVal * (self.hi - self.lo) + self.lo).to(x.dtype) if x.is_floating_point() else \
            (x.float() / self.maxPixelVal * (self.hi - self.lo) + self.lo)

    def _rev(self, x, which):
        if which == "l":
            return x
        return ((x - self.lo) / (self.hi - self.lo) * self.maxPixelVal).to(x.dtype)

    def _state(self):
        return {"lo": self.lo, "hi": self.hi, "maxBits": self.maxBits}, {}

    def _load(self, meta, a):
        self.__init__(meta["lo"], meta["hi"], meta["maxBits"])


class VGG16ImagePreProcessor(DataNormalization):
    TYPE = "IMAGE_VGG16"
    VGG_MEAN_OFFSET_BGR = (103.939, 116.779, 123.68)

    def fit(self, data):
        return self

    def _off(self, x):
        return torch.tensor(self.VGG_MEAN_OFFSET_BGR, dtype=x.dtype, device=x.device).reshape(1, 3, 1, 1)

    def _tf(self, x, which):
        return x if which == "l" else x - self._off(x)

    def _rev(self, x, which):
        return x if which == "l" else x + self._off(x)


class _MultiNormalizer:
    """Per-input / per-output normalization of MultiDataSets (ND4J MultiNormalizerStandardize /
    MultiNormalizerMinMaxScaler): one single-array normalizer per feature (and, with fitLabel, label) array."""

    def __init__(self):
        self.fitLabels = False
        self.f, self.l = [], []

    def fitLabel(self, b):
        self.fitLabels = bool(b)
        return self

    def isFitLabel(self):
        return self.fitLabels

    def _make(self, stats):
        raise NotImplementedError

    def fit(self, data):
        from .dataset import MultiDataSet
        items = [data] if isinstance(data, MultiDataSet) else list(_iter_datasets(data))
        nf = items[0].numFeatureArrays()
        nl = items[0].numLabelsArrays() if items[0].labels is not None else 0
        fs, ls = [_Stats() for _ in range(nf)], [_Stats() for _ in range(nl)]
        for mds in items:
            for i in range(nf):
                fs[i].add(mds.getFeatures(i))
            if self.fitLabels:
                for i in range(nl):
                    ls[i].add(mds.getLabels(i))
        self.f = [self._make(s) for s in fs]
        self.l = [self._make(s) for s in ls] if self.fitLabels else []
        return self

    def preProcess(self, mds):
        for i, n in enumerate(self.f):
            mds.features[i] = n.transform(mds.features[i])
        for i, n in enumerate(self.l):
            mds.labels[i] = n.transform(mds.labels[i])

    __call__ = preProcess

    def revert(self, mds):
        for i, n in enumerate(self.f):
            mds.features[i] = n.revertFeatures(mds.features[i])
        for i, n in enumerate(self.l):
            mds.labels[i] = n.revertFeatures(mds.labels[i])

    def revertFeatures(self, features):
        return [n.revertFeatures(x) for n, x in zip(self.f, features)]

    def revertLabels(self, labels):
        return [n.revertFeatures(y) for n, y in zip(self.l, labels)]


class MultiNormalizerStandardize(_MultiNormalizer):
    def _make(self, st):
        return NormalizerStandardize(st.mean(), st.std().clamp_min(EPS))

    def getFeatureMean(self, i):
        return self.f[i].getMean()

    def getFeatureStd(self, i):
        return self.f[i].getStd()


class MultiNormalizerMinMaxScaler(_MultiNormalizer):
    def __init__(self, minRange=0.0, maxRange=1.0):
        super().__init__()
        self.lo, self.hi = float(minRange), float(maxRange)

    def _make(self, st):
        n = NormalizerMinMaxScaler(self.lo, self.hi)
        n.fMin, n.fMax = st.mn, st.mx
        return n

    def getMin(self, i):
        return self.f[i].getMin()

    def getMax(self, i):
        return self.f[i].getMax()
