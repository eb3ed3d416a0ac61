"""Per-producer parallel dataset iterators (reference deeplearning4j-utility-iterators iterator/parallel/
BaseParallelDataSetIterator.java, FileSplitParallelDataSetIterator.java; test strategy after
FileSplitParallelDataSetIteratorTest / JointParallelDataSetIteratorTest): round-robin order over the producers, the
four InequalityHandling policies, thread-affine hasNextFor/nextFor for ParallelWrapper workers, reset, and the file
split (every file read exactly once, parts balanced). CPU."""
import threading

import pytest
import torch

from deeplearning4j_amd.datasets import (BaseParallelDataSetIterator, DataSet, FileSplitParallelDataSetIterator,
                                         InequalityHandling)


class _Lists(BaseParallelDataSetIterator):
    def __init__(self, lens, h):
        super().__init__(len(lens), h)
        self.lens, self.pos = list(lens), [0] * len(lens)

    def hasNextFor(self, consumer=None):
        k = self._attached() if consumer is None else consumer
        return self.pos[k] < self.lens[k]

    def nextFor(self, consumer=None):
        k = self._attached() if consumer is None else consumer
        self.pos[k] += 1
        return DataSet(torch.tensor([[float(k), float(self.pos[k] - 1)]]), torch.zeros(1, 1))

    def resetProducer(self, consumer):
        self.pos[consumer] = 0


def _drain(it, cap=100):
    out = []
    while it.hasNext() and len(out) < cap:
        d = it.next()
        out.append(None if d is None else tuple(int(v) for v in d.getFeatures()[0].tolist()))
    return out


def test_round_robin_and_policies():
    assert _drain(_Lists([2, 2], InequalityHandling.STOP_EVERYONE)) == [(0, 0), (1, 0), (0, 1), (1, 1)]
    assert _drain(_Lists([3, 1], InequalityHandling.STOP_EVERYONE)) == [(0, 0), (1, 0), (0, 1)]
    assert _drain(_Lists([3, 1], InequalityHandling.RELOCATE)) == [(0, 0), (1, 0), (0, 1), (0, 2)]
    got = _drain(_Lists([3, 1], InequalityHandling.PASS_NULL))
    assert got == [(0, 0), (1, 0), (0, 1), None, (0, 2), None]     # a dry turn is only noticed at that turn
    got = _drain(_Lists([3, 1], InequalityHandling.RESET))
    assert got[:5] == [(0, 0), (1, 0), (0, 1), (1, 0), (0, 2)]          # the short producer restarts
    it = _Lists([2, 2], InequalityHandling.STOP_EVERYONE)
    _drain(it)
    it.reset()
    assert _drain(it) == [(0, 0), (1, 0), (0, 1), (1, 1)]


def test_thread_affinity():
    it = _Lists([5, 5, 5], InequalityHandling.STOP_EVERYONE)
    with pytest.raises(RuntimeError, match="attachThread"):
        it.hasNextFor()
    seen = {}

    def worker(k):
        it.attachThread(k)
        xs = []
        while it.hasNextFor():
            xs.append(tuple(int(v) for v in it.nextFor().getFeatures()[0].tolist()))
        seen[k] = xs

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert all(seen[k] == [(k, i) for i in range(5)] for k in range(3))


def test_file_split_parallel(tmp_path):
    for i in range(11):
        DataSet(torch.full((2, 3), float(i)), torch.zeros(2, 1)).save(str(tmp_path / f"dataset-{i}.bin"))
    (tmp_path / "other.bin").write_bytes(b"x")
    it = FileSplitParallelDataSetIterator(str(tmp_path), "dataset-%d.bin", numThreads=3, bufferPerThread=2,
                                          inequalityHandling=InequalityHandling.RELOCATE, devices=[None])
    assert [len(p) for p in it.parts] == [3, 4, 4]
    vals = sorted(int(d.getFeatures()[0, 0]) for d in iter(lambda: it.next() if it.hasNext() else None, None))
    assert vals == list(range(11))
    it.reset()
    it.attachThread(1)
    mine = []
    while it.hasNextFor():
        mine.append(int(it.nextFor().getFeatures()[0, 0]))
    assert mine == [3, 4, 5, 6]
    it.shutdown()
    with pytest.raises(ValueError):
        FileSplitParallelDataSetIterator(str(tmp_path), "missing-%d.bin", numThreads=2, devices=[None])
