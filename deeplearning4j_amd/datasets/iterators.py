"""Utility iterators (reference deeplearning4j-data/deeplearning4j-utility-iterators):
BenchmarkDataSetIterator (synthetic, BenchmarkDataSetIterator.java:26-47), AsyncDataSetIterator
(background prefetch, ITER:AsyncDataSetIterator.java:29-108,383-397), MultipleEpochsIterator,
EarlyTerminationDataSetIterator, SamplingDataSetIterator, KFoldIterator, ... .

AsyncDataSetIterator on a GPU stages each batch into pinned host memory and copies it to the device
on a dedicated HIP copy stream from the prefetch thread, recording an event the consumer waits on,
so H2D overlaps the previous step's compute.
"""
import queue
import threading

import torch

from .dataset import DataSet, DataSetIterator, MultiDataSet


class BenchmarkDataSetIterator(DataSetIterator):
    """Returns the same random [mb, ...] features and one-hot labels ``totalIterations`` times."""

    def __init__(self, featuresShape, numLabels, totalIterations, gridWidth=-1, gridHeight=-1, device=None,
                 dtype=torch.float32, seed=12345):
        g = torch.Generator().manual_seed(seed)
        mb = featuresShape[0]
        f = torch.rand(*featuresShape, generator=g, dtype=torch.float32)
        if gridWidth > 0 and gridHeight > 0:
            lab = torch.zeros(mb, numLabels, gridHeight, gridWidth)
            cls = torch.randint(0, numLabels, (mb, gridHeight, gridWidth), generator=g)
            lab.scatter_(1, cls.unsqueeze(1), 1.0)
        else:
            lab = torch.zeros(mb, numLabels)
            lab[torch.arange(mb), torch.randint(0, numLabels, (mb,), generator=g)] = 1.0
        if device is not None:
            f, lab = f.to(device), lab.to(device)
            if f.dim() == 4 and f.is_cuda:
                f = f.contiguous(memory_format=torch.channels_last)
        self.ds = DataSet(f.to(dtype), lab)
        self.total = totalIterations
        self.i = 0

    def hasNext(self):
        return self.total < 0 or self.i < self.total

    def next(self, num=None):
        self.i += 1
        return self.ds

    def reset(self):
        self.i = 0

    def batch(self):
        return self.ds.features.shape[0]

    def inputColumns(self):
        return self.ds.features[0].numel()

    def totalOutcomes(self):
        return self.ds.labels.shape[1]


class BenchmarkMultiDataSetIterator(BenchmarkDataSetIterator):
    def next(self, num=None):
        self.i += 1
        return MultiDataSet.fromDataSet(self.ds)


_END = object()


class AsyncDataSetIterator(DataSetIterator):
    def __init__(self, base, queueSize=2, device=None, useWorkspace=True):
        self.base = base
        self.qsize = max(1, queueSize)
        self.device = device
        self._thread = None
        self._q = None
        self._next = None
        self._err = None
        self._stop = threading.Event()

    def _worker(self):
        stream = torch.cuda.Stream(device=self.device) if (self.device is not None and
                                                           torch.device(self.device).type == "cuda") else None
        try:
            while not self._stop.is_set() and self.base.hasNext():
                ds = self.base.next()
                ev = None
                if stream is not None:
                    with torch.cuda.stream(stream):
                        ds = _to_device(ds, self.device, pin=True)
                        ev = torch.cuda.Event()
                        ev.record(stream)
                while not self._stop.is_set():
                    try:
                        self._q.put((ds, ev), timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except BaseException as e:  # propagate to consumer
            self._err = e
        finally:
            while True:
                try:
                    self._q.put((_END, None), timeout=0.1)
                    break
                except queue.Full:
                    if self._stop.is_set():
                        break

    def _start(self):
        self._stop.clear()
        self._q = queue.Queue(self.qsize)
        self._next = None
        self._thread = threading.Thread(target=self._worker, name="ADSI prefetch thread", daemon=True)
        self._thread.start()

    def _peek(self):
        if self._thread is None:
            self._start()
        if self._next is None:
            self._next = self._q.get()
            if self._err is not None:
                raise self._err
        return self._next

    def hasNext(self):
        return self._peek()[0] is not _END

    def next(self, num=None):
        ds, ev = self._peek()
        if ds is _END:
            raise StopIteration
        self._next = None
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        return ds

    def shutdown(self):
        if self._thread is not None:
            self._stop.set()
            try:
                while True:
                    self._q.get_nowait()
            except queue.Empty:
                pass
            self._thread.join(timeout=5)
            self._thread = None

    def reset(self):
        self.shutdown()
        self.base.reset()

    def batch(self):
        return self.base.batch()

    def inputColumns(self):
        return self.base.inputColumns()

    def totalOutcomes(self):
        return self.base.totalOutcomes()

    def __del__(self):
        try:
            self.shutdown()
        except Exception:
            pass


AsyncMultiDataSetIterator = AsyncDataSetIterator


def _to_device(ds, device, pin=False):
    def mv(t):
        if t is None:
            return None
        if pin and not t.is_cuda and not t.is_pinned():
            t = t.pin_memory()
        return t.to(device, non_blocking=True)
    if isinstance(ds, MultiDataSet):
        m = lambda xs: None if xs is None else [mv(x) for x in xs]  # noqa: E731
        return MultiDataSet(m(ds.features), m(ds.labels), m(ds.featuresMasks), m(ds.labelsMasks))
    return DataSet(mv(ds.features), mv(ds.labels), mv(ds.featuresMask), mv(ds.labelsMask))


class _DataSetSource:
    """A single in-memory DataSet seen as an iterator: next(num) hands out the next num examples (all remaining when
    num is None)."""

    def __init__(self, ds):
        self.ds = ds
        self.pos = 0

    def hasNext(self):
        return self.pos < self.ds.numExamples()

    def next(self, num=None):
        n = self.ds.numExamples()
        end = n if num is None else min(n, self.pos + num)
        out = self.ds if (self.pos == 0 and end == n) else self.ds.get(list(range(self.pos, end)))
        self.pos = end
        return out

    def reset(self):
        self.pos = 0

    def batch(self):
        return self.ds.numExamples()


class MultipleEpochsIterator(DataSetIterator):
    """Replays an iterator (or one DataSet) for ``numEpochs`` epochs, or for ``totalIterations`` minibatches
    (reference datasets/iterator/MultipleEpochsIterator.java). Constructors as in the reference:
    (numEpochs, iterator[, queueSize]), (iterator, queueSize, totalIterations), (numEpochs, DataSet). ``epochs``
    counts completed passes."""

    def __init__(self, *args):
        from .dataset import DataSet
        self.numEpochs, self.totalIterations = 1, None
        if isinstance(args[0], int):
            self.numEpochs = args[0]
            src = args[1]
        else:
            src = args[0]
            if len(args) >= 3:
                self.totalIterations = int(args[2])
                self.numEpochs = 2 ** 62
        self.base = _DataSetSource(src) if isinstance(src, DataSet) else src
        self.epochs = 0
        self.iterations = 0
        self._counted = False

    @property
    def n(self):
        return self.numEpochs

    @property
    def epoch(self):
        return self.epochs

    def hasNext(self):
        if self.totalIterations is not None:
            if self.iterations >= self.totalIterations:
                return False
            if not self.base.hasNext():
                self.epochs += 1
                self.base.reset()
            return self.base.hasNext()
        if self.base.hasNext():
            return True
        if not self._counted:                  # the underlying pass just ended
            self.epochs += 1
            self._counted = True
        if self.epochs < self.numEpochs:
            self.base.reset()
            self._counted = False
            return self.base.hasNext()
        return False

    def next(self, num=None):
        if not self.hasNext():
            raise StopIteration("MultipleEpochsIterator: no more minibatches")
        self.iterations += 1
        return self.base.next(num) if num is not None else self.base.next()

    def reset(self):
        self.epochs = 0
        self.iterations = 0
        self._counted = False
        self.base.reset()

    def batch(self):
        return self.base.batch()


class EarlyTerminationDataSetIterator(DataSetIterator):
    """At most ``terminationPoint`` minibatches per pass; asking for more is an error (reference
    datasets/iterator/EarlyTerminationDataSetIterator.java)."""

    def __init__(self, base, terminationPoint):
        if terminationPoint <= 0:
            raise ValueError("Termination point (the number of calls to .next() or .fit()) must be > 0")
        self.base = base
        self.limit = terminationPoint
        self.i = 0

    def hasNext(self):
        return self.i < self.limit and self.base.hasNext()

    def next(self, num=None):
        if self.i >= self.limit:
            raise RuntimeError("Calls to next have exceeded the allotted number of minibatches.")
        self.i += 1
        return self.base.next(num) if num is not None else self.base.next()

    def reset(self):
        self.i = 0
        self.base.reset()

    def batch(self):
        return self.base.batch()


class EarlyTerminationMultiDataSetIterator(EarlyTerminationDataSetIterator):
    """EarlyTerminationDataSetIterator over a MultiDataSetIterator (reference
    datasets/iterator/EarlyTerminationMultiDataSetIterator.java): at most ``terminationPoint`` MultiDataSets per pass,
    the same ones again after reset, and a further next() is an error."""


class MultiDataSetIteratorAdapter:
    """Presents a DataSetIterator as a MultiDataSetIterator (reference
    datasets/iterator/impl/MultiDataSetIteratorAdapter.java:13-61): each DataSet becomes a single-input,
    single-output MultiDataSet, so ComputationGraph APIs that take MultiDataSets accept plain iterators."""

    def __init__(self, iter):
        self.iter = iter
        self.preProcessor = None

    def hasNext(self):
        return self.iter.hasNext()

    def next(self, num=None):
        from .dataset import MultiDataSet
        ds = self.iter.next() if num is None else self.iter.next(num)
        m = MultiDataSet.fromDataSet(ds)
        if self.preProcessor is not None:
            self.preProcessor.preProcess(m)
        return m

    def __iter__(self):
        self.reset()
        while self.hasNext():
            yield self.next()

    def reset(self):
        self.iter.reset()

    def resetSupported(self):
        return getattr(self.iter, "resetSupported", lambda: True)()

    def asyncSupported(self):
        return getattr(self.iter, "asyncSupported", lambda: True)()

    def setPreProcessor(self, p):
        self.preProcessor = p

    def getPreProcessor(self):
        return self.preProcessor


class SamplingDataSetIterator(DataSetIterator):
    def __init__(self, sampleFrom, batchSize, totalNumberSamples, seed=None):
        self.ds = sampleFrom
        self.bs = batchSize
        self.total = totalNumberSamples
        self.n = 0
        self.g = torch.Generator().manual_seed(seed if seed is not None else 12345)

    def hasNext(self):
        return self.n < self.total

    def next(self, num=None):
        idx = torch.randint(0, self.ds.numExamples(), (self.bs,), generator=self.g)
        self.n += self.bs
        return self.ds._sub(idx)

    def reset(self):
        self.n = 0

    def batch(self):
        return self.bs


class KFoldIterator(DataSetIterator):
    def __init__(self, k, ds):
        self.k = k
        self.ds = ds
        self.i = 0
        n = ds.numExamples()
        self.bounds = [(j * n // k, (j + 1) * n // k) for j in range(k)]

    def hasNext(self):
        return self.i < self.k

    def next(self, num=None):
        a, b = self.bounds[self.i]
        n = self.ds.numExamples()
        idx = torch.cat([torch.arange(0, a), torch.arange(b, n)])
        self._test = self.ds._sub(torch.arange(a, b))
        self.i += 1
        return self.ds._sub(idx)

    def testFold(self):
        return self._test

    def reset(self):
        self.i = 0


class DoublesDataSetIterator(DataSetIterator):
    """Iterates (features, labels) pairs of python lists/arrays in minibatches."""

    def __init__(self, pairs, batchSize):
        self.pairs = list(pairs)
        self.bs = batchSize
        self.i = 0

    def hasNext(self):
        return self.i < len(self.pairs)

    def next(self, num=None):
        chunk = self.pairs[self.i:self.i + self.bs]
        self.i += self.bs
        f = torch.tensor([list(p[0]) for p in chunk], dtype=torch.float32)
        l = torch.tensor([list(p[1]) for p in chunk], dtype=torch.float32)
        return DataSet(f, l)

    def reset(self):
        self.i = 0

    def batch(self):
        return self.bs


class FloatsDataSetIterator(DoublesDataSetIterator):
    """(float[] features, float[] labels) pairs in float32 minibatches (reference
    datasets/iterator/FloatsDataSetIterator.java over AbstractDataSetIterator): the iterable is drained lazily, one
    minibatch at a time, and re-iterated on reset, so a generator-backed iterable need not fit in memory."""

    def __init__(self, iterable, batchSize):
        self.source = iterable
        self.bs = batchSize
        self._it = iter(iterable)
        self._peek = None

    def _fill(self):
        if self._peek is None:
            self._peek = next(self._it, None)
        return self._peek

    def hasNext(self):
        return self._fill() is not None

    def next(self, num=None):
        n = num or self.bs
        chunk = []
        while len(chunk) < n and self._fill() is not None:
            chunk.append(self._peek)
            self._peek = None
        if not chunk:
            raise StopIteration("FloatsDataSetIterator: no more pairs (reset first)")
        f = torch.tensor([list(p[0]) for p in chunk], dtype=torch.float32)
        l = torch.tensor([list(p[1]) for p in chunk], dtype=torch.float32)
        return self._pp(DataSet(f, l))

    def reset(self):
        self._it = iter(self.source)
        self._peek = None


class INDArrayDataSetIterator(FloatsDataSetIterator):
    """(INDArray features, INDArray labels) pairs (reference datasets/iterator/INDArrayDataSetIterator.java): rows
    are stacked into minibatches as given (any float dtype is kept as float32)."""

    def next(self, num=None):
        n = num or self.bs
        chunk = []
        while len(chunk) < n and self._fill() is not None:
            chunk.append(self._peek)
            self._peek = None
        if not chunk:
            raise StopIteration("INDArrayDataSetIterator: no more pairs (reset first)")
        t = lambda a: torch.as_tensor(getattr(a, "tensor", a)).reshape(-1).float()  # noqa: E731
        return self._pp(DataSet(torch.stack([t(p[0]) for p in chunk]), torch.stack([t(p[1]) for p in chunk])))


class DataSetIteratorSplitter:
    """Splits one iterator into train / test views by batch count (DataSetIteratorSplitter.java): the first
    ``ratio * totalBatches`` batches of each pass feed getTrainIterator(), the following ones getTestIterator().
    Streaming: nothing is cached, the views share the underlying iterator's position. A test pass that starts before
    the train part of the current pass was consumed skips it; resetting either view restarts the underlying pass.

    Cost: the test view of a fresh pass replays (reads and discards) the ``ntrain`` train batches of that pass first,
    so a test-only evaluation after ``reset()`` costs a full pass of the underlying iterator.
    As in the reference (DataSetIteratorSplitter.java:158-166), the first train batch of the first pass is kept and
    compared with the first train batch of every later pass: a shuffling underlying iterator would silently move
    examples between the train and test parts, so that raises instead. ``next(num)`` is unsupported (the reference
    throws UnsupportedOperationException)."""

    def __init__(self, base, totalBatches, ratio):
        if not 0.0 < ratio < 1.0:
            raise ValueError("ratio must be in (0, 1)")
        if int(totalBatches) <= 0:
            raise ValueError("totalBatches should be a positive value")
        self.base, self.total = base, int(totalBatches)
        self.ntrain = int(self.total * ratio)
        self.pos = 0                          # batches of the current underlying pass handed out (or skipped)
        self.first_train = None               # features of the first train batch of the first pass

    def _check_first(self, ds):
        f = ds.getFeatures() if hasattr(ds, "getFeatures") else getattr(ds, "features", None)
        if f is None:
            return
        if isinstance(f, (list, tuple)):            # MultiDataSet: every feature array, flattened in order
            f = torch.cat([a.detach().reshape(-1).to("cpu", torch.float32) for a in f])
        f = f.detach().to("cpu", torch.float32)
        if self.first_train is None:
            self.first_train = f.clone()
        elif f.shape != self.first_train.shape or not torch.allclose(f, self.first_train, atol=1e-5, rtol=0):
            raise RuntimeError("DataSetIteratorSplitter: first examples do not match. Randomization was used?")

    def _restart(self):
        self.base.reset()
        self.pos = 0

    def getTrainIterator(self):
        return _SplitView(self, 0, self.ntrain)

    def getTestIterator(self):
        return _SplitView(self, self.ntrain, self.total)


class _SplitView(DataSetIterator):
    def __init__(self, sp, lo, hi):
        self.sp, self.lo, self.hi = sp, lo, hi

    def hasNext(self):
        sp = self.sp
        if sp.pos > self.hi or (self.lo == 0 and sp.pos >= self.hi):
            return False
        while sp.pos < self.lo and sp.base.hasNext():      # test view: skip the train part of this pass
            sp.base.next()
            sp.pos += 1
        return sp.pos < self.hi and sp.base.hasNext()

    def next(self, num=None):
        if num is not None:
            raise NotImplementedError("DataSetIteratorSplitter views do not support next(num)")
        if not self.hasNext():
            raise StopIteration("DataSetIteratorSplitter: this part of the pass is exhausted (reset first)")
        first = self.sp.pos == 0
        self.sp.pos += 1
        ds = self.sp.base.next()
        if first:
            self.sp._check_first(ds)
        return self._pp(ds)

    def reset(self):
        self.sp._restart()

    def batch(self):
        return self.sp.base.batch()


MultiDataSetIteratorSplitter = DataSetIteratorSplitter


class FileDataSetIterator(DataSetIterator):
    """Iterates DataSet files written by DataSet.save (one minibatch per file, sorted by name)."""

    def __init__(self, rootDir, pattern=".bin"):
        import os
        self.files = sorted(os.path.join(dp, f) for dp, _, fs in os.walk(rootDir) for f in fs if f.endswith(pattern))
        self.i = 0

    def hasNext(self):
        return self.i < len(self.files)

    def next(self, num=None):
        from .dataset import DataSet
        d = DataSet.load(self.files[self.i])
        self.i += 1
        return self._pp(d)

    def reset(self):
        self.i = 0


class ReconstructionDataSetIterator(DataSetIterator):
    """Wraps an iterator so labels = features (autoencoder training)."""

    def __init__(self, base):
        self.base = base

    def hasNext(self):
        return self.base.hasNext()

    def next(self, num=None):
        from .dataset import DataSet
        d = self.base.next()
        return self._pp(DataSet(d.features, d.features.clone(), d.featuresMask, d.featuresMask))

    def reset(self):
        self.base.reset()

    def batch(self):
        return self.base.batch()


# ------------------------------------------------------------------------------------------------ combinators
class InequalityHandling:
    """What JointParallelDataSetIterator does once one source runs dry (reference enums/InequalityHandling.java)."""
    STOP_EVERYONE = "STOP_EVERYONE"      # stop as soon as the source whose turn it is has nothing left
    PASS_NULL = "PASS_NULL"              # an exhausted source's turns yield None; rounds run while any source has data
    RELOCATE = "RELOCATE"                # an exhausted source's turns go to the next source that still has data
    RESET = "RESET"                      # an exhausted source restarts, until every source has run dry once


class JointParallelDataSetIterator(DataSetIterator):
    """Round-robin over several source iterators, one batch per source per turn (reference
    datasets/iterator/parallel/JointParallelDataSetIterator.java: feeds ParallelWrapper workers from several
    sources, e.g. one per device), with the inequality policy above for sources of different lengths."""

    class Builder:
        def __init__(self, inequalityHandling=InequalityHandling.STOP_EVERYONE):
            self._h = inequalityHandling
            self._src = []
            self._pp = None

        def addSourceIterator(self, it):
            self._src.append(it)
            return self

        def setPreProcessor(self, pp):
            self._pp = pp
            return self

        def build(self):
            j = JointParallelDataSetIterator(self._src, self._h)
            j.preProcessor = self._pp
            return j

    def __init__(self, sources, inequalityHandling=InequalityHandling.STOP_EVERYONE):
        if not sources:
            raise ValueError("JointParallelDataSetIterator needs at least one source iterator")
        self.sources = list(sources)
        self.handling = inequalityHandling
        self.turn = 0
        self.dried = [False] * len(self.sources)      # ran dry at least once (RESET)

    def _live(self):
        return [i for i, s in enumerate(self.sources) if s.hasNext()]

    def hasNext(self):
        h, i = self.handling, self.turn
        if h == InequalityHandling.STOP_EVERYONE:
            return self.sources[i].hasNext()
        if h == InequalityHandling.RESET:
            if self.sources[i].hasNext():
                return True
            self.dried[i] = True
            return not all(self.dried)
        if h == InequalityHandling.PASS_NULL and i != 0:
            return True                            # a started round is completed (with None for dry sources)
        return bool(self._live())

    def next(self, num=None):
        if not self.hasNext():
            raise StopIteration
        i = self.turn
        self.turn = (i + 1) % len(self.sources)
        s, h = self.sources[i], self.handling
        if s.hasNext():
            return self._pp(s.next())
        if h == InequalityHandling.PASS_NULL:
            return None
        if h == InequalityHandling.RESET:
            self.dried[i] = True
            s.reset()
            return self._pp(s.next())
        # RELOCATE: the next source (in turn order) that still has data
        for k in range(1, len(self.sources)):
            j = (i + k) % len(self.sources)
            if self.sources[j].hasNext():
                return self._pp(self.sources[j].next())
        raise StopIteration

    def reset(self):
        for s in self.sources:
            s.reset()
        self.turn = 0
        self.dried = [False] * len(self.sources)

    def batch(self):
        return self.sources[0].batch()


class FileSplitDataSetIterator(DataSetIterator):
    """DataSets from an explicit list of files through a callback (reference iterator/FileSplitDataSetIterator.java +
    callbacks/FileCallback): ``callback(path) -> DataSet``; the default callback is ``DataSet.load``."""

    def __init__(self, files, callback=None):
        from .dataset import DataSet
        self.files = list(files)
        self.callback = callback or DataSet.load
        self.i = 0

    def hasNext(self):
        return self.i < len(self.files)

    def next(self, num=None):
        if num is not None:
            raise NotImplementedError("FileSplitDataSetIterator does not support next(num)")
        f = self.files[self.i]
        self.i += 1
        cb = self.callback
        return self._pp(cb.call(f) if hasattr(cb, "call") else cb(f))

    def reset(self):
        self.i = 0


class BaseParallelDataSetIterator(DataSetIterator):
    """One iterator over N producers (reference iterator/parallel/BaseParallelDataSetIterator.java:20-126): ``next()``
    takes the producers round-robin with the InequalityHandling policy once one runs dry, and a ParallelWrapper
    worker thread bound to producer k (``attachThread(k)``) pulls only its own producer with ``hasNextFor()`` /
    ``nextFor()`` — the per-device feeding of ParallelWrapper. Subclasses implement ``hasNextFor(k)``,
    ``nextFor(k)`` and ``resetProducer(k)``."""

    def __init__(self, numProducers, inequalityHandling=InequalityHandling.STOP_EVERYONE):
        self.numProducers = int(numProducers)
        self.inequalityHandling = inequalityHandling
        self.counter = 0
        self.states = [True] * self.numProducers          # producer still has data
        self.resetTracker = [False] * self.numProducers   # producer ran dry at least once (RESET)
        self.allDepleted = False
        self._affinity = threading.local()

    # ---- per-producer API
    def hasNextFor(self, consumer=None):
        raise NotImplementedError

    def nextFor(self, consumer=None):
        raise NotImplementedError

    def resetProducer(self, consumer):
        raise NotImplementedError

    def attachThread(self, producer):
        if not 0 <= int(producer) < self.numProducers:
            raise ValueError(f"Non-existent producer {producer}")
        self._affinity.producer = int(producer)

    def _attached(self):
        k = getattr(self._affinity, "producer", None)
        if k is None:
            raise RuntimeError("attachThread(int) should be called prior to this call")
        return k

    # ---- round-robin view
    def _cur(self):
        return self.counter % self.numProducers

    def hasNext(self):
        if self.allDepleted or not any(self.states):
            return False
        cur = self._cur()
        if self.hasNextFor(cur):
            return True
        self.states[cur] = False
        if not any(self.states):
            return False
        h = self.inequalityHandling
        if h == InequalityHandling.RESET:
            self.resetTracker[cur] = True
            if all(self.resetTracker):
                self.allDepleted = True
                return False
            self.resetProducer(cur)
            self.states[cur] = True
            return True
        if h == InequalityHandling.RELOCATE:
            while True:
                self.counter += 1
                k = self._cur()
                self.states[k] = bool(self.hasNextFor(k))
                if self.states[k]:
                    return True
                if not any(self.states):
                    return False
        if h == InequalityHandling.PASS_NULL:
            return True
        return all(self.states)                            # STOP_EVERYONE

    def next(self, num=None):
        if num is not None:
            raise NotImplementedError("parallel iterators do not support next(num)")
        cur = self._cur()
        ds = self.nextFor(cur) if self.hasNextFor(cur) else None   # PASS_NULL: a dry producer's turn yields None
        self.counter += 1
        return None if ds is None else self._pp(ds)

    def reset(self):
        for k in range(self.numProducers):
            self.resetProducer(k)
            self.states[k] = True
            self.resetTracker[k] = False
        self.allDepleted = False
        self.counter = 0

    def resetSupported(self):
        return True

    def asyncSupported(self):
        return False


class FileSplitParallelDataSetIterator(BaseParallelDataSetIterator):
    """Per-device producers over a folder of DataSet files (reference iterator/parallel/
    FileSplitParallelDataSetIterator.java): the files matching ``pattern`` (``%d`` = any index, default
    "dataset-%d.bin") are split into ``numThreads`` contiguous parts, each read by its own AsyncDataSetIterator
    (``bufferPerThread`` batches prefetched; on a GPU build each part is staged onto device ``k % numDevices``).
    Unlike the reference's Lists.partition split, which drops the last ``files % numThreads`` files, the parts here
    differ in size by at most one file."""
    DEFAULT_PATTERN = "dataset-%d.bin"

    def __init__(self, rootFolder, pattern=DEFAULT_PATTERN, callback=None, numThreads=None, bufferPerThread=2,
                 inequalityHandling=InequalityHandling.STOP_EVERYONE, devices=None):
        import os
        import re
        if not os.path.isdir(rootFolder):
            raise ValueError("Root folder should point to existing folder")
        if numThreads is None:
            numThreads = max(1, torch.cuda.device_count())
        super().__init__(numThreads, inequalityHandling)
        rx = re.compile("^" + ".*".join(re.escape(x) for x in pattern.split("%d")) + "$")
        key = lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f)]      # noqa: E731
        files = sorted((f for f in os.listdir(rootFolder) if rx.match(f)), key=key)
        if not files:
            raise ValueError("No suitable files were found")
        if devices is None:
            devices = [torch.device("cuda", k) for k in range(torch.cuda.device_count())] or [None]
        n, T = len(files), self.numProducers
        bounds = [(k * n) // T for k in range(T + 1)]
        self.parts = [[os.path.join(rootFolder, f) for f in files[bounds[k]:bounds[k + 1]]] for k in range(T)]
        self.asyncIterators = [AsyncDataSetIterator(FileSplitDataSetIterator(part, callback), bufferPerThread,
                                                    devices[k % len(devices)])
                               for k, part in enumerate(self.parts)]

    def _check(self, k):
        if not 0 <= k < self.numProducers:
            raise ValueError("Non-existent consumer was requested")
        return self.asyncIterators[k]

    def hasNextFor(self, consumer=None):
        return self._check(self._attached() if consumer is None else consumer).hasNext()

    def nextFor(self, consumer=None):
        return self._check(self._attached() if consumer is None else consumer).next()

    def resetProducer(self, consumer):
        self._check(consumer).reset()

    def shutdown(self):
        for it in self.asyncIterators:
            if hasattr(it, "shutdown"):
                it.shutdown()


class CombinedPreProcessor:
    """Applies several DataSet pre-processors in order (reference nd4j CombinedPreProcessor; Builder.addPreProcessor
    appends, addPreProcessor(index, p) inserts)."""

    class Builder:
        def __init__(self):
            self._pps = []

        def addPreProcessor(self, a, b=None):
            if b is None:
                self._pps.append(a)
            else:
                self._pps.insert(int(a), b)
            return self

        def build(self):
            return CombinedPreProcessor(self._pps)

    def __init__(self, preProcessors):
        self.preProcessors = list(preProcessors)

    def preProcess(self, ds):
        for p in self.preProcessors:
            p.preProcess(ds)

    __call__ = preProcess


class CombinedMultiDataSetPreProcessor(CombinedPreProcessor):
    """The MultiDataSet variant (reference CombinedMultiDataSetPreProcessor)."""

    class Builder(CombinedPreProcessor.Builder):
        def build(self):
            return CombinedMultiDataSetPreProcessor(self._pps)
