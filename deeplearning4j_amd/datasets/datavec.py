"""Record readers and the record-reader -> DataSet bridges.

Reference: DataVec record readers used throughout DL4J (CSVRecordReader, CSVSequenceRecordReader, ImageRecordReader
with ParentPathLabelGenerator, CollectionRecordReader, FileSplit / NumberedFileInputSplit) and
deeplearning4j-data/deeplearning4j-datavec-iterators RecordReaderDataSetIterator.java (classification: one-hot of
the label column; regression: label columns as-is), SequenceRecordReaderDataSetIterator.java (one or two readers,
AlignmentMode EQUAL_LENGTH / ALIGN_START / ALIGN_END with masks), RecordReaderMultiDataSetIterator.java
(Builder: addReader / addSequenceReader / addInput / addOutput / addOutputOneHot).
Records are lists of Python scalars/strings; sequences are lists of records.
"""
import csv
import glob
import os

import numpy as np
import torch

from .dataset import DataSet, DataSetIterator, MultiDataSet


# ------------------------------------------------------------------------------------------------ input splits

def _check_classes(classes, n):
    """A class index outside [0, numPossibleLabels) is a data error, reported as the reference does (its message
    says the value could not be converted "to one-hot")."""
    for c in classes:
        if not 0 <= c < n:
            raise ValueError(f"Invalid classification data: can't convert class index {c} to one-hot "
                             f"representation with {n} possible labels (valid indices 0..{n - 1})")

class FileSplit:
    def __init__(self, path, allowFormat=None, recursive=True):
        if os.path.isdir(path):
            files = sorted(glob.glob(os.path.join(path, "**", "*"), recursive=True)) if recursive else \
                sorted(os.path.join(path, f) for f in os.listdir(path))
            files = [f for f in files if os.path.isfile(f)]
        else:
            files = [path]
        if allowFormat:
            ext = tuple("." + e.lstrip(".").lower() for e in allowFormat)
            files = [f for f in files if f.lower().endswith(ext)]
        self.files = files

    def locations(self):
        return list(self.files)


class NumberedFileInputSplit(FileSplit):
    """``base_%d.csv`` for indices [minIdx, maxIdx] inclusive."""

    def __init__(self, baseString, minIdx, maxIdx):
        self.files = [baseString % i for i in range(minIdx, maxIdx + 1)]


class CollectionInputSplit(FileSplit):
    def __init__(self, files):
        self.files = list(files)


def _num(v):
    try:
        return float(v)
    except (TypeError, ValueError):
        return v


# ------------------------------------------------------------------------------------------------ readers
class RecordReader:
    def initialize(self, split):
        self.split = split
        self.reset()
        return self

    def hasNext(self):
        raise NotImplementedError

    def next(self):
        raise NotImplementedError

    def reset(self):
        pass

    def getLabels(self):
        return None

    def __iter__(self):
        self.reset()
        while self.hasNext():
            yield self.next()


class CollectionRecordReader(RecordReader):
    def __init__(self, records):
        self.records = [list(r) for r in records]
        self.i = 0

    def hasNext(self):
        return self.i < len(self.records)

    def next(self):
        r = self.records[self.i]
        self.i += 1
        return r

    def reset(self):
        self.i = 0


class CSVRecordReader(RecordReader):
    def __init__(self, skipNumLines=0, delimiter=",", quote='"'):
        self.skip, self.delim, self.quote = int(skipNumLines), delimiter, quote
        self.rows = []
        self.i = 0

    def reset(self):
        self.rows = []
        for f in self.split.locations():
            with open(f, newline="", encoding="utf-8") as fh:
                rd = csv.reader(fh, delimiter=self.delim, quotechar=self.quote)
                for k, row in enumerate(rd):
                    if k < self.skip or not row:
                        continue
                    self.rows.append([_num(v) for v in row])
        self.i = 0

    def hasNext(self):
        return self.i < len(self.rows)

    def next(self):
        r = self.rows[self.i]
        self.i += 1
        return r


class LineRecordReader(CSVRecordReader):
    def reset(self):
        self.rows = []
        for f in self.split.locations():
            with open(f, encoding="utf-8") as fh:
                self.rows.extend([[l.rstrip("\n")] for l in fh])
        self.i = 0


class SequenceRecordReader(RecordReader):
    def nextSequence(self):
        return self.next()


class CSVSequenceRecordReader(SequenceRecordReader):
    """One sequence per file; one time step per line."""

    def __init__(self, skipNumLines=0, delimiter=","):
        self.skip, self.delim = int(skipNumLines), delimiter
        self.i = 0

    def reset(self):
        self.files = self.split.locations()
        self.i = 0

    def hasNext(self):
        return self.i < len(self.files)

    def next(self):
        f = self.files[self.i]
        self.i += 1
        with open(f, newline="", encoding="utf-8") as fh:
            rows = [r for k, r in enumerate(csv.reader(fh, delimiter=self.delim)) if k >= self.skip and r]
        return [[_num(v) for v in r] for r in rows]


class CollectionSequenceRecordReader(SequenceRecordReader):
    def __init__(self, sequences):
        self.seqs = [[list(s) for s in seq] for seq in sequences]
        self.i = 0

    def hasNext(self):
        return self.i < len(self.seqs)

    def next(self):
        s = self.seqs[self.i]
        self.i += 1
        return s

    def reset(self):
        self.i = 0


class ParentPathLabelGenerator:
    def getLabelForPath(self, path):
        return os.path.basename(os.path.dirname(path))


class ImageRecordReader(RecordReader):
    """Images -> records [CHW float array (0..255), label index]; labels from the parent folder name."""

    def __init__(self, height, width, channels=3, labelGenerator=None):
        self.h, self.w, self.c = height, width, channels
        self.labelGen = labelGenerator
        self.labels = []
        self.i = 0

    def reset(self):
        self.files = [f for f in self.split.locations()
                      if f.lower().endswith((".png", ".jpg", ".jpeg", ".bmp", ".gif"))]
        if self.labelGen is not None:
            self.labels = sorted({self.labelGen.getLabelForPath(f) for f in self.files})
        self.i = 0

    def getLabels(self):
        return list(self.labels)

    def hasNext(self):
        return self.i < len(self.files)

    def next(self):
        from .fetchers import _load_image
        f = self.files[self.i]
        self.i += 1
        img = _load_image(f, self.h, self.w, self.c)
        rec = [img]
        if self.labelGen is not None:
            rec.append(float(self.labels.index(self.labelGen.getLabelForPath(f))))
        return rec


# ------------------------------------------------------------------------------------------------ iterators
def _flatten_record(rec):
    out = []
    for v in rec:
        if isinstance(v, np.ndarray):
            out.extend(v.reshape(-1).tolist())
        else:
            out.append(v)
    return out


class RecordReaderDataSetIterator(DataSetIterator):
    """Classification (labelIndex + numPossibleLabels -> one-hot), regression (labelIndex..labelIndexTo as-is), or
    unsupervised (labelIndex < 0). ImageRecordReader records keep their [C,H,W] image shape."""

    class Builder:
        def __init__(self, recordReader, batchSize):
            self.rr, self.bs = recordReader, batchSize
            self.li, self.lt, self.n, self.reg = -1, -1, -1, False
            self.pp = None

        def classification(self, labelIndex, numClasses):
            self.li, self.n, self.reg = labelIndex, numClasses, False
            return self

        def regression(self, labelIndexFrom, labelIndexTo=None):
            self.li, self.lt, self.reg = labelIndexFrom, labelIndexFrom if labelIndexTo is None else labelIndexTo, \
                True
            return self

        def preProcessor(self, p):
            self.pp = p
            return self

        def build(self):
            it = RecordReaderDataSetIterator(self.rr, self.bs, self.li, self.n, self.reg, self.lt)
            it.preProcessor = self.pp
            return it

    def __init__(self, recordReader, batchSize, labelIndex=-1, numPossibleLabels=-1, regression=False,
                 labelIndexTo=None):
        self.rr, self.bs = recordReader, int(batchSize)
        self.li, self.n, self.reg = labelIndex, numPossibleLabels, regression
        self.lt = labelIndex if labelIndexTo is None or labelIndexTo < 0 else labelIndexTo
        self.preProcessor = None
        self._buf = None

    def _split(self, rec):
        if len(rec) == 2 and isinstance(rec[0], np.ndarray) and self.li == 1:        # image record
            return rec[0], [rec[1]]
        if self.li < 0:
            return np.array(_flatten_record(rec), dtype=np.float32), None
        lab = rec[self.li:self.lt + 1]
        feat = rec[:self.li] + rec[self.lt + 1:]
        return np.array(_flatten_record(feat), dtype=np.float32), lab

    def hasNext(self):
        return self.rr.hasNext()

    def next(self, num=None):
        n = num or self.bs
        feats, labs = [], []
        while len(feats) < n and self.rr.hasNext():
            f, l = self._split(self.rr.next())
            feats.append(f)
            labs.append(l)
        x = torch.from_numpy(np.stack(feats).astype(np.float32))
        if labs[0] is None:
            y = x.clone()
        elif self.reg:
            y = torch.tensor([[float(v) for v in l] for l in labs], dtype=torch.float32)
        else:
            cls = [int(float(l[0])) for l in labs]
            _check_classes(cls, self.n)
            y = torch.zeros(len(labs), self.n)
            y[torch.arange(len(labs)), torch.tensor(cls)] = 1.0
        return self._pp(DataSet(x, y))

    def reset(self):
        self.rr.reset()

    def batch(self):
        return self.bs

    def totalOutcomes(self):
        return self.n

    def getLabels(self):
        return self.rr.getLabels()


class AlignmentMode:
    EQUAL_LENGTH, ALIGN_START, ALIGN_END = "EQUAL_LENGTH", "ALIGN_START", "ALIGN_END"


def _seq_tensor(seqs, T, align, dtype=torch.float32):
    """list of [t_i, f] arrays -> ([n, f, T], mask [n, T] or None)."""
    n, f = len(seqs), seqs[0].shape[1]
    out = torch.zeros(n, f, T, dtype=dtype)
    mask = torch.zeros(n, T)
    for i, s in enumerate(seqs):
        t = s.shape[0]
        st = T - t if align == AlignmentMode.ALIGN_END else 0
        out[i, :, st:st + t] = torch.from_numpy(s.T.astype(np.float32))
        mask[i, st:st + t] = 1.0
    return out, (None if bool((mask == 1).all()) else mask)


class SequenceRecordReaderDataSetIterator(DataSetIterator):
    """Features [mb, nIn, T] and labels [mb, nOut, T] (one-hot per step for classification); either one reader with
    a label column, or separate feature/label readers with an alignment mode for different lengths."""

    def __init__(self, featuresReader, labels_or_batch, miniBatchSize=None, numPossibleLabels=-1, regression=False,
                 alignmentMode=AlignmentMode.EQUAL_LENGTH, labelIndex=-1):
        if isinstance(labels_or_batch, int):            # single reader: (reader, batch, numLabels, labelIndex, reg)
            self.fr, self.lr = featuresReader, None
            self.bs = labels_or_batch
            self.n = miniBatchSize if miniBatchSize is not None else numPossibleLabels
            self.li = numPossibleLabels if miniBatchSize is not None else labelIndex
            self.reg = regression
        else:
            self.fr, self.lr, self.bs = featuresReader, labels_or_batch, int(miniBatchSize)
            self.n, self.reg, self.li = numPossibleLabels, regression, -1
        self.align = alignmentMode
        self.preProcessor = None

    def hasNext(self):
        return self.fr.hasNext()

    def _labels(self, s):
        if self.reg:
            return s
        oh = np.zeros((s.shape[0], self.n), np.float32)
        _check_classes(s[:, 0].astype(np.int64).tolist(), self.n)
        oh[np.arange(s.shape[0]), s[:, 0].astype(np.int64)] = 1.0
        return oh

    def next(self, num=None):
        n = num or self.bs
        fs, ls = [], []
        while len(fs) < n and self.fr.hasNext():
            f = np.array(self.fr.next(), dtype=np.float32)
            if self.lr is not None:
                l = np.array(self.lr.next(), dtype=np.float32)
            else:
                li = self.li if self.li >= 0 else f.shape[1] - 1
                l = f[:, li:li + 1]
                f = np.delete(f, li, axis=1)
            fs.append(f)
            ls.append(self._labels(l))
        tf = max(s.shape[0] for s in fs)
        tl = max(s.shape[0] for s in ls)
        if self.align == AlignmentMode.EQUAL_LENGTH and (tf != tl or any(a.shape[0] != b.shape[0]
                                                                           for a, b in zip(fs, ls))):
            raise ValueError("EQUAL_LENGTH alignment with sequences of different lengths: use ALIGN_START/ALIGN_END")
        T = max(tf, tl)
        x, fm = _seq_tensor(fs, T, self.align)
        y, lm = _seq_tensor(ls, T, self.align)
        return self._pp(DataSet(x, y, fm, lm))

    def reset(self):
        self.fr.reset()
        if self.lr is not None:
            self.lr.reset()

    def batch(self):
        return self.bs

    def totalOutcomes(self):
        return self.n


class RecordReaderMultiDataSetIterator(DataSetIterator):
    class Builder:
        def __init__(self, batchSize):
            self.bs = batchSize
            self.readers, self.seq_readers = {}, {}
            self.inputs, self.outputs = [], []
            self.align = AlignmentMode.EQUAL_LENGTH

        def addReader(self, name, rr):
            self.readers[name] = rr
            return self

        def addSequenceReader(self, name, rr):
            self.seq_readers[name] = rr
            return self

        def addInput(self, name, colFirst=None, colLast=None):
            self.inputs.append((name, colFirst, colLast, None))
            return self

        def addInputOneHot(self, name, column, numClasses):
            self.inputs.append((name, column, column, numClasses))
            return self

        def addOutput(self, name, colFirst=None, colLast=None):
            self.outputs.append((name, colFirst, colLast, None))
            return self

        def addOutputOneHot(self, name, column, numClasses):
            self.outputs.append((name, column, column, numClasses))
            return self

        def sequenceAlignmentMode(self, m):
            self.align = m
            return self

        def build(self):
            return RecordReaderMultiDataSetIterator(self)

    def __init__(self, b):
        self.b = b
        self.preProcessor = None

    def hasNext(self):
        rs = list(self.b.readers.values()) + list(self.b.seq_readers.values())
        return all(r.hasNext() for r in rs)

    @staticmethod
    def _cols(arr, a, z, nc):
        a = 0 if a is None else a
        z = arr.shape[-1] - 1 if z is None else z
        sub = arr[..., a:z + 1]
        if nc is None:
            return sub
        oh = np.zeros(sub.shape[:-1] + (nc,), np.float32)
        idx = sub[..., 0].astype(np.int64)
        np.put_along_axis(oh, idx[..., None], 1.0, axis=-1)
        return oh

    def next(self, num=None):
        n = num or self.b.bs
        recs = {k: [] for k in list(self.b.readers) + list(self.b.seq_readers)}
        while len(next(iter(recs.values()))) < n and self.hasNext():
            for k, r in self.b.readers.items():
                recs[k].append(np.array(_flatten_record(r.next()), dtype=np.float32))
            for k, r in self.b.seq_readers.items():
                recs[k].append(np.array(r.next(), dtype=np.float32))

        def build(spec):
            arrs, masks = [], []
            for name, a, z, nc in spec:
                if name in self.b.readers:
                    arrs.append(torch.from_numpy(self._cols(np.stack(recs[name]), a, z, nc)))
                    masks.append(None)
                else:
                    seqs = [self._cols(s, a, z, nc) for s in recs[name]]
                    T = max(s.shape[0] for s in seqs)
                    t, m = _seq_tensor(seqs, T, self.b.align)
                    arrs.append(t)
                    masks.append(m)
            return arrs, (masks if any(m is not None for m in masks) else None)
        f, fm = build(self.b.inputs)
        l, lm = build(self.b.outputs)
        return self._pp(MultiDataSet(f, l, fm, lm))

    def reset(self):
        for r in list(self.b.readers.values()) + list(self.b.seq_readers.values()):
            r.reset()

    def batch(self):
        return self.b.bs
