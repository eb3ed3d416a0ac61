"""DataSet / MultiDataSet containers and the iterator protocol (ND4J DataSet, DataSetIterator,
MultiDataSetIterator equivalents)."""
import numpy as np
import torch


def as_tensor(x, dtype=None):
    if x is None:
        return None
    if hasattr(x, "toTensor"):                           # nd4j.INDArray
        x = x.toTensor()
    if torch.is_tensor(x):
        return x if dtype is None else x.to(dtype)
    t = torch.from_numpy(np.ascontiguousarray(x))
    return t if dtype is None else t.to(dtype)


class DataSet:
    def __init__(self, features=None, labels=None, featuresMask=None, labelsMask=None):
        self.features = as_tensor(features)
        self.labels = as_tensor(labels)
        self.featuresMask = as_tensor(featuresMask)
        self.labelsMask = as_tensor(labelsMask)
        self.exampleMetaData = None

    # reference accessors
    def getFeatures(self):
        return self.features

    def getLabels(self):
        return self.labels

    def getFeaturesMaskArray(self):
        return self.featuresMask

    def getLabelsMaskArray(self):
        return self.labelsMask

    def setFeatures(self, f):
        self.features = as_tensor(f)

    def setLabels(self, l):
        self.labels = as_tensor(l)

    def hasMaskArrays(self):
        return self.featuresMask is not None or self.labelsMask is not None

    def numExamples(self):
        return 0 if self.features is None else self.features.shape[0]

    def numInputs(self):
        return self.features.shape[1]

    def numOutcomes(self):
        return self.labels.shape[1]

    def to(self, device, non_blocking=False):
        mv = lambda t: None if t is None else t.to(device, non_blocking=non_blocking)  # noqa: E731
        return DataSet(mv(self.features), mv(self.labels), mv(self.featuresMask), mv(self.labelsMask))

    def splitTestAndTrain(self, n_or_frac, rng=None):
        n = self.numExamples()
        k = int(n * n_or_frac) if isinstance(n_or_frac, float) and n_or_frac < 1 else int(n_or_frac)
        idx = torch.arange(n)
        a, b = idx[:k], idx[k:]
        return SplitTestAndTrain(self._sub(a), self._sub(b))

    def _sub(self, idx):
        pick = lambda t: None if t is None else t[idx]  # noqa: E731
        return DataSet(pick(self.features), pick(self.labels), pick(self.featuresMask), pick(self.labelsMask))

    def shuffle(self, seed=None):
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        p = torch.randperm(self.numExamples(), generator=g)
        d = self._sub(p)
        self.features, self.labels, self.featuresMask, self.labelsMask = d.features, d.labels, d.featuresMask, \
            d.labelsMask

    def batchBy(self, n):
        return [self._sub(torch.arange(i, min(i + n, self.numExamples()))) for i in range(0, self.numExamples(), n)]

    # ND4J DataSet feature transforms (in place), used by the reference's tests on Iris / MNIST batches
    def normalizeZeroMeanZeroUnitVariance(self):
        """Per-column (per-feature) standardisation over the examples: (x - mean) / std, std of a constant column
        treated as 1 so it stays 0."""
        f = self.features.double()
        mu = f.mean(0, keepdim=True)
        sd = f.std(0, unbiased=True, keepdim=True)
        sd = torch.where(sd > 0, sd, torch.ones_like(sd))
        self.features = ((f - mu) / sd).to(self.features.dtype)

    def scaleMinAndMax(self, lo, hi):
        """Per-column linear rescale of the features to [lo, hi]."""
        f = self.features.double()
        mn, mx = f.amin(0, keepdim=True), f.amax(0, keepdim=True)
        rng = torch.where(mx > mn, mx - mn, torch.ones_like(mx))
        self.features = (lo + (f - mn) / rng * (hi - lo)).to(self.features.dtype)

    def binarize(self, cutoff=0.0):
        """Features > cutoff -> 1, else 0."""
        self.features = (self.features > cutoff).to(self.features.dtype)

    def labelCounts(self):
        """{class index: number of examples} of a one-hot / probability label matrix."""
        idx = self.labels.reshape(self.labels.shape[0], -1).argmax(1)
        u, c = torch.unique(idx, return_counts=True)
        return {int(a): int(b) for a, b in zip(u, c)}

    def get(self, i):
        """Example(s) ``i`` (an int or an index list) as a new DataSet."""
        idx = torch.as_tensor([i] if isinstance(i, int) else list(i), dtype=torch.long)
        return self._sub(idx)

    def asList(self):
        return self.batchBy(1)

    @staticmethod
    def merge(dss):
        cat = lambda xs: None if xs[0] is None else torch.cat(xs, 0)  # noqa: E731
        return DataSet(cat([d.features for d in dss]), cat([d.labels for d in dss]),
                       cat([d.featuresMask for d in dss]), cat([d.labelsMask for d in dss]))

    def copy(self):
        c = lambda t: None if t is None else t.clone()  # noqa: E731
        return DataSet(c(self.features), c(self.labels), c(self.featuresMask), c(self.labelsMask))

    def __len__(self):
        return self.numExamples()

    def __iter__(self):
        yield self.features
        yield self.labels

    def save(self, path):
        """Write features / labels / masks (each optional) as a sequence of ND4J-binary arrays behind a presence
        bitmask byte (DataSet.save(File) layout idea: flags, then arrays)."""
        from ..utils import nd4j_io
        parts = [self.features, self.labels, self.featuresMask, self.labelsMask]

        def _w(fh):
            fh.write(bytes([sum(1 << i for i, t in enumerate(parts) if t is not None)]))
            for t in parts:
                if t is not None:
                    nd4j_io.write(t.detach().cpu(), fh)
        if hasattr(path, "write"):
            _w(path)
        else:
            with open(path, "wb") as fh:
                _w(fh)

    @staticmethod
    def load(path):
        """From a path or a binary stream."""
        from ..utils import nd4j_io

        def _r(fh):
            flags = fh.read(1)[0]
            return DataSet(*[nd4j_io.read(fh) if flags & (1 << i) else None for i in range(4)])
        if hasattr(path, "read"):
            return _r(path)
        with open(path, "rb") as fh:
            return _r(fh)


class SplitTestAndTrain:
    def __init__(self, train, test):
        self._train, self._test = train, test

    def getTrain(self):
        return self._train

    def getTest(self):
        return self._test


class MultiDataSet:
    def __init__(self, features=None, labels=None, featuresMasks=None, labelsMasks=None):
        wrap = lambda x: None if x is None else [as_tensor(t) for t in (x if isinstance(x, (list, tuple)) else [x])]  # noqa
        self.features = wrap(features)
        self.labels = wrap(labels)
        self.featuresMasks = wrap(featuresMasks)
        self.labelsMasks = wrap(labelsMasks)

    def getFeatures(self, i=None):
        return self.features if i is None else self.features[i]

    def getLabels(self, i=None):
        return self.labels if i is None else self.labels[i]

    def getFeaturesMaskArrays(self):
        return self.featuresMasks

    def getLabelsMaskArrays(self):
        return self.labelsMasks

    def numFeatureArrays(self):
        return len(self.features)

    def numLabelsArrays(self):
        return len(self.labels)

    def numExamples(self):
        return self.features[0].shape[0]

    @staticmethod
    def fromDataSet(ds):
        return MultiDataSet([ds.features], [ds.labels], None if ds.featuresMask is None else [ds.featuresMask],
                            None if ds.labelsMask is None else [ds.labelsMask])


class DataSetIterator:
    """Iterator protocol of the reference (hasNext/next/reset/batch/...) plus Python iteration."""

    def hasNext(self):
        raise NotImplementedError

    def next(self, num=None):
        raise NotImplementedError

    def reset(self):
        pass

    def resetSupported(self):
        return True

    def asyncSupported(self):
        return True

    def batch(self):
        return None

    def inputColumns(self):
        return None

    def totalOutcomes(self):
        return None

    def getLabels(self):
        return None

    def setPreProcessor(self, p):
        self.preProcessor = p

    def getPreProcessor(self):
        return getattr(self, "preProcessor", None)

    def _pp(self, ds):
        p = getattr(self, "preProcessor", None)
        if p is not None:
            p.preProcess(ds)
        return ds

    def __iter__(self):
        self.reset()
        while self.hasNext():
            yield self.next()

    def __next__(self):
        if not self.hasNext():
            raise StopIteration
        return self.next()


MultiDataSetIterator = DataSetIterator


class ListDataSetIterator(DataSetIterator):
    def __init__(self, data, batch=None):
        if isinstance(data, DataSet):
            data = data.batchBy(batch) if batch else [data]
        elif batch and data and isinstance(data[0], DataSet) and data[0].numExamples() == 1:
            data = [DataSet.merge(data[i:i + batch]) for i in range(0, len(data), batch)]
        self.data = list(data)
        self.i = 0
        self._batch = batch

    def hasNext(self):
        return self.i < len(self.data)

    def next(self, num=None):
        d = self.data[self.i]
        self.i += 1
        return self._pp(d)

    def reset(self):
        self.i = 0

    def batch(self):
        return self._batch or (self.data[0].numExamples() if self.data else 0)

    def inputColumns(self):
        return self.data[0].features.shape[1] if self.data else 0

    def totalOutcomes(self):
        return self.data[0].labels.shape[1] if self.data else 0


class IteratorDataSetIterator(ListDataSetIterator):
    pass


class ExistingDataSetIterator(ListDataSetIterator):
    def __init__(self, iterable):
        super().__init__(list(iterable))


class IteratorMultiDataSetIterator(ListDataSetIterator):
    pass
