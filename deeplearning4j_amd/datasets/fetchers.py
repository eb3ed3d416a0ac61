"""Dataset fetchers and their iterators (MNIST, EMNIST, Iris, CIFAR-10, SVHN, LFW, TinyImageNet, UCI sequences).

Reference: deeplearning4j-data/deeplearning4j-datasets — fetchers/{MnistDataFetcher, EmnistDataFetcher,
IrisDataFetcher, TinyImageNetFetcher, SvhnDataFetcher, UciSequenceDataFetcher}.java, iterator/impl/*DataSetIterator.java,
mnist/{MnistManager, MnistImageFile, MnistLabelFile}.java (IDX format), base/IrisUtils.java.

There is no network here: every fetcher reads the standard on-disk format from a local directory —
``$DL4J_AMD_DATA_DIR/<DATASET>`` (default ``~/.deeplearning4j/data/<DATASET>``, the reference's cache layout) or an
explicit ``dataDir`` — and raises a clear error naming the expected files when they are absent (the reference would
download them). Parsing is vectorised numpy (IDX, CIFAR binary batches); image folders decode through PIL.
"""
import gzip
import os

import numpy as np
import torch

from .dataset import DataSet, DataSetIterator


def data_root(name, dataDir=None):
    if dataDir:
        return dataDir
    base = os.environ.get("DL4J_AMD_DATA_DIR", os.path.join(os.path.expanduser("~"), ".deeplearning4j", "data"))
    return os.path.join(base, name)


def _open(path):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(f"dataset file not found: {path}[.gz] (no network access: place the files there or "
                            f"set DL4J_AMD_DATA_DIR)")


# ------------------------------------------------------------------------------------------------ IDX (MNIST)
class MnistImageFile:
    """IDX3 image file: magic 2051, count, rows, cols, then uint8 pixels."""

    def __init__(self, path):
        with _open(path) as fh:
            hdr = np.frombuffer(fh.read(16), dtype=">i4")
            if hdr[0] != 2051:
                raise ValueError(f"{path}: not an IDX3 image file (magic {hdr[0]})")
            self.count, self.rows, self.cols = int(hdr[1]), int(hdr[2]), int(hdr[3])
            self.data = np.frombuffer(fh.read(), dtype=np.uint8).reshape(self.count, self.rows * self.cols)

    def readImage(self, i):
        return self.data[i].reshape(self.rows, self.cols)


class MnistLabelFile:
    """IDX1 label file: magic 2049, count, then uint8 labels."""

    def __init__(self, path):
        with _open(path) as fh:
            hdr = np.frombuffer(fh.read(8), dtype=">i4")
            if hdr[0] != 2049:
                raise ValueError(f"{path}: not an IDX1 label file (magic {hdr[0]})")
            self.count = int(hdr[1])
            self.labels = np.frombuffer(fh.read(), dtype=np.uint8)[:self.count]


def write_idx(images, labels, img_path, lbl_path):
    """Write uint8 images [n, rows, cols] / labels [n] in IDX format (tests, conversions)."""
    images = np.asarray(images, dtype=np.uint8)
    n, r, c = images.shape
    with open(img_path, "wb") as fh:
        fh.write(np.array([2051, n, r, c], dtype=">i4").tobytes())
        fh.write(images.tobytes())
    with open(lbl_path, "wb") as fh:
        fh.write(np.array([2049, n], dtype=">i4").tobytes())
        fh.write(np.asarray(labels, dtype=np.uint8).tobytes())


class MnistManager:
    def __init__(self, imagesFile, labelsFile):
        self.images = MnistImageFile(imagesFile)
        self.labels = MnistLabelFile(labelsFile) if labelsFile else None
        self.cur = 0

    def readImage(self):
        img = self.images.readImage(self.cur)
        self.cur += 1
        return img

    def readLabel(self):
        return int(self.labels.labels[self.cur - 1])


# ------------------------------------------------------------------------------------------------ base
class DataSetFetcher:
    """Holds the whole (small) dataset as tensors; ``fetch(n)`` serves the next n examples."""

    def __init__(self):
        self.features = None
        self.labels = None
        self.cursor = 0
        self.curr = None

    def totalExamples(self):
        return int(self.features.shape[0])

    def inputColumns(self):
        return int(np.prod(self.features.shape[1:]))

    def totalOutcomes(self):
        return int(self.labels.shape[1])

    def hasMore(self):
        return self.cursor < self.totalExamples()

    def fetch(self, n):
        a, b = self.cursor, min(self.cursor + n, self.totalExamples())
        self.curr = DataSet(self.features[a:b], self.labels[a:b])
        self.cursor = b
        return self.curr

    def next(self):
        return self.curr

    def reset(self):
        self.cursor = 0

    def shuffle(self, seed):
        g = torch.Generator().manual_seed(int(seed))
        p = torch.randperm(self.totalExamples(), generator=g)
        self.features, self.labels = self.features[p], self.labels[p]


def _one_hot(idx, n):
    out = torch.zeros(len(idx), n)
    out[torch.arange(len(idx)), torch.as_tensor(np.asarray(idx, dtype=np.int64))] = 1.0
    return out


class BaseDatasetIterator(DataSetIterator):
    def __init__(self, batch, numExamples, fetcher):
        self._batch = int(batch)
        self.fetcher = fetcher
        self.numExamples = fetcher.totalExamples() if numExamples is None or numExamples < 0 else \
            min(int(numExamples), fetcher.totalExamples())
        self.preProcessor = None

    def hasNext(self):
        return self.fetcher.cursor < self.numExamples

    def next(self, num=None):
        n = min(num or self._batch, self.numExamples - self.fetcher.cursor)
        return self._pp(self.fetcher.fetch(n))

    def reset(self):
        self.fetcher.reset()

    def batch(self):
        return self._batch

    def inputColumns(self):
        return self.fetcher.inputColumns()

    def totalOutcomes(self):
        return self.fetcher.totalOutcomes()

    def totalExamples(self):
        return self.numExamples


# ------------------------------------------------------------------------------------------------ MNIST / EMNIST
class MnistDataFetcher(DataSetFetcher):
    FILES = {True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
             False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}
    NUM_LABELS = 10
    NAME = "MNIST"

    def __init__(self, binarize=True, train=True, shuffle=True, rngSeed=123, numExamples=None, dataDir=None):
        super().__init__()
        root = data_root(self.NAME, dataDir)
        fi, fl = self._files(train)
        imgs = MnistImageFile(os.path.join(root, fi))
        lbls = MnistLabelFile(os.path.join(root, fl))
        x = imgs.data.astype(np.float32)
        x = (x > 30).astype(np.float32) if binarize else x / 255.0      # MnistDataFetcher: binarize threshold 30
        n = imgs.count if numExamples is None else min(numExamples, imgs.count)
        self.features = torch.from_numpy(x[:n].copy())
        self.labels = _one_hot(self._map_labels(lbls.labels[:n]), self.NUM_LABELS)
        if shuffle:
            self.shuffle(rngSeed)

    def _files(self, train):
        return self.FILES[bool(train)]

    def _map_labels(self, l):
        return l


class MnistDataSetIterator(BaseDatasetIterator):
    """MnistDataSetIterator(batch, train, seed) or (batch, numExamples, binarize, train, shuffle, seed)."""

    def __init__(self, batch, train_or_num=True, seed=123, binarize=False, train=True, shuffle=True, dataDir=None):
        if isinstance(train_or_num, bool):
            numExamples, train = None, train_or_num
        else:
            numExamples = int(train_or_num)
        super().__init__(batch, numExamples, MnistDataFetcher(binarize, train, shuffle, seed, numExamples, dataDir))


class EmnistDataSetIterator(BaseDatasetIterator):
    class Set:
        COMPLETE = "byclass"
        BYCLASS = "byclass"
        MERGE = "bymerge"
        BYMERGE = "bymerge"
        BALANCED = "balanced"
        LETTERS = "letters"
        DIGITS = "digits"
        MNIST = "mnist"

    NUM_LABELS = {"byclass": 62, "bymerge": 47, "balanced": 47, "letters": 26, "digits": 10, "mnist": 10}

    class _Fetcher(MnistDataFetcher):
        NAME = "EMNIST"

        def __init__(self, dataSet, *a, **k):
            self.set = dataSet
            self.NUM_LABELS = EmnistDataSetIterator.NUM_LABELS[dataSet]
            super().__init__(*a, **k)

        def _files(self, train):
            t = "train" if train else "test"
            return f"emnist-{self.set}-{t}-images-idx3-ubyte", f"emnist-{self.set}-{t}-labels-idx1-ubyte"

        def _map_labels(self, l):
            return l - 1 if self.set == "letters" else l     # EMNIST letters are labelled 1..26

    def __init__(self, dataSet, batch, train=True, seed=123, binarize=False, dataDir=None):
        super().__init__(batch, None, EmnistDataSetIterator._Fetcher(dataSet, binarize, train, True, seed, None,
                                                                     dataDir))

    @staticmethod
    def numLabels(dataSet):
        return EmnistDataSetIterator.NUM_LABELS[dataSet]


# ------------------------------------------------------------------------------------------------ Iris
class IrisDataFetcher(DataSetFetcher):
    """150 examples x 4 features, 3 classes. Reads ``iris.dat`` (CSV ``f1,f2,f3,f4,label``)."""

    def __init__(self, path=None, dataDir=None):
        super().__init__()
        p = path or os.path.join(data_root("IRIS", dataDir), "iris.dat")
        if not os.path.exists(p):
            raise FileNotFoundError(f"iris data not found at {p} (set DL4J_AMD_DATA_DIR or pass path)")
        a = np.loadtxt(p, delimiter=",", dtype=np.float64)
        self.features = torch.from_numpy(a[:, :4].astype(np.float32))
        self.labels = _one_hot(a[:, 4].astype(np.int64), 3)


class IrisDataSetIterator(BaseDatasetIterator):
    def __init__(self, batch=150, numExamples=150, path=None, dataDir=None):
        super().__init__(batch, numExamples, IrisDataFetcher(path, dataDir))


# ------------------------------------------------------------------------------------------------ CIFAR-10
class CifarDataSetIterator(BaseDatasetIterator):
    """CIFAR-10 binary batches (data_batch_1..5.bin / test_batch.bin: 1 label byte + 3072 CHW bytes), NCHW float in
    [0, 1] (or raw 0..255 with ``normalize=False``)."""
    LABELS = ["airplane", "automobile", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck"]

    class _Fetcher(DataSetFetcher):
        def __init__(self, train, numExamples, normalize, dataDir):
            super().__init__()
            root = data_root("CIFAR10", dataDir)
            sub = os.path.join(root, "cifar-10-batches-bin")
            root = sub if os.path.isdir(sub) else root
            files = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
            recs = []
            for f in files:
                with _open(os.path.join(root, f)) as fh:
                    recs.append(np.frombuffer(fh.read(), dtype=np.uint8).reshape(-1, 3073))
            r = np.concatenate(recs)
            if numExamples:
                r = r[:numExamples]
            x = r[:, 1:].reshape(-1, 3, 32, 32).astype(np.float32)
            self.features = torch.from_numpy(x / 255.0 if normalize else x)
            self.labels = _one_hot(r[:, 0].astype(np.int64), 10)

        def inputColumns(self):
            return 3 * 32 * 32

    def __init__(self, batch, numExamples=None, train=True, normalize=True, dataDir=None):
        super().__init__(batch, numExamples, CifarDataSetIterator._Fetcher(train, numExamples, normalize, dataDir))

    def getLabels(self):
        return list(self.LABELS)


# ------------------------------------------------------------------------------------------------ image folders
def _load_image(path, h, w, c):
    from PIL import Image
    im = Image.open(path)
    im = im.convert("L" if c == 1 else "RGB")
    if (h, w) != (im.height, im.width):
        im = im.resize((w, h))
    a = np.asarray(im, dtype=np.float32)
    return a[None] if c == 1 else a.transpose(2, 0, 1)


class ImageFolderFetcher(DataSetFetcher):
    """Images under ``root/<label>/*``; labels in sorted folder order; NCHW float in [0, 1]."""

    EXT = (".png", ".jpg", ".jpeg", ".bmp", ".gif")

    def __init__(self, root, height, width, channels=3, numExamples=None, shuffle=True, seed=123):
        super().__init__()
        if not os.path.isdir(root):
            raise FileNotFoundError(f"image folder dataset not found at {root}")
        self.labelNames = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
        items = [(os.path.join(root, l, f), i) for i, l in enumerate(self.labelNames)
                 for f in sorted(os.listdir(os.path.join(root, l))) if f.lower().endswith(self.EXT)]
        if shuffle:
            np.random.RandomState(seed).shuffle(items)
        if numExamples:
            items = items[:numExamples]
        x = np.stack([_load_image(p, height, width, channels) for p, _ in items]) / 255.0
        self.features = torch.from_numpy(x.astype(np.float32))
        self.labels = _one_hot([l for _, l in items], len(self.labelNames))


class LFWDataSetIterator(BaseDatasetIterator):
    """Labeled Faces in the Wild: ``LFW/lfw/<person>/*.jpg`` (or a root passed as dataDir)."""

    def __init__(self, batch, numExamples=None, imgDim=(250, 250, 3), seed=123, dataDir=None):
        root = data_root("LFW", dataDir)
        sub = os.path.join(root, "lfw")
        root = sub if os.path.isdir(sub) else root
        f = ImageFolderFetcher(root, imgDim[0], imgDim[1], imgDim[2], numExamples, True, seed)
        super().__init__(batch, numExamples, f)
        self.labels = f.labelNames

    def getLabels(self):
        return self.labels


class TinyImageNetDataSetIterator(BaseDatasetIterator):
    """Tiny ImageNet 200: ``TINYIMAGENET_200/train/<wnid>/images/*.JPEG`` (64x64x3, 200 classes)."""

    def __init__(self, batch, train=True, numExamples=None, seed=123, dataDir=None):
        root = data_root("TINYIMAGENET_200", dataDir)
        split = os.path.join(root, "train" if train else "val")
        items = []
        wnids = sorted(d for d in os.listdir(split) if os.path.isdir(os.path.join(split, d))) \
            if os.path.isdir(split) else []
        if not wnids:
            raise FileNotFoundError(f"Tiny ImageNet not found at {split}")
        for i, w in enumerate(wnids):
            d = os.path.join(split, w, "images")
            d = d if os.path.isdir(d) else os.path.join(split, w)
            items += [(os.path.join(d, f), i) for f in sorted(os.listdir(d)) if f.lower().endswith(".jpeg")]
        np.random.RandomState(seed).shuffle(items)
        if numExamples:
            items = items[:numExamples]
        f = DataSetFetcher()
        f.features = torch.from_numpy((np.stack([_load_image(p, 64, 64, 3) for p, _ in items]) / 255.0)
                                      .astype(np.float32))
        f.labels = _one_hot([l for _, l in items], 200)
        super().__init__(batch, numExamples, f)
        self.labels = wnids


class SvhnDataFetcher(DataSetFetcher):
    """SVHN cropped digits from ``SVHN/{train,test}/<label>/*.png`` folders (pre-extracted)."""

    def __init__(self, train=True, numExamples=None, dataDir=None):
        root = os.path.join(data_root("SVHN", dataDir), "train" if train else "test")
        f = ImageFolderFetcher(root, 32, 32, 3, numExamples)
        super().__init__()
        self.features, self.labels = f.features, f.labels


# ------------------------------------------------------------------------------------------------ UCI sequences
class UciSequenceDataSetIterator(DataSetIterator):
    """UCI synthetic control chart time series: 600 series x 60 steps, 6 classes (100 each, in order). Reads
    ``synthetic_control.data`` (whitespace separated); features [mb, 1, 60], per-step labels [mb, 6, 60] with a
    labels mask on the last step only (UciSequenceDataFetcher: classification at the final time step)."""

    def __init__(self, batch, train=True, seed=123, dataDir=None):
        p = os.path.join(data_root("UCI", dataDir), "synthetic_control.data")
        if not os.path.exists(p):
            raise FileNotFoundError(f"UCI synthetic control data not found at {p}")
        a = np.loadtxt(p, dtype=np.float32)
        labels = np.repeat(np.arange(6), 100)
        idx = np.random.RandomState(seed).permutation(600)
        idx = idx[:450] if train else idx[450:]
        x = a[idx]
        x = (x - x.mean()) / x.std()
        self.x = torch.from_numpy(x).reshape(-1, 1, 60)
        self.y = labels[idx]
        self._batch = batch
        self.cursor = 0

    def hasNext(self):
        return self.cursor < self.x.shape[0]

    def next(self, num=None):
        n = min(num or self._batch, self.x.shape[0] - self.cursor)
        sl = slice(self.cursor, self.cursor + n)
        self.cursor += n
        lab = torch.zeros(n, 6, 60)
        lab[torch.arange(n), torch.as_tensor(self.y[sl]), 59] = 1.0
        mask = torch.zeros(n, 60)
        mask[:, 59] = 1.0
        return self._pp(DataSet(self.x[sl], lab, None, mask))

    def reset(self):
        self.cursor = 0

    def batch(self):
        return self._batch

    def totalOutcomes(self):
        return 6

    def inputColumns(self):
        return 1
