"""DataSetIteratorSplitter, after the reference's DataSetSplitterTests
(deeplearning4j-core/src/test/java/org/deeplearning4j/datasets/iterator/DataSetSplitterTests.java:13-90): over a
generator of 1000 numbered batches split 0.7 / 0.3, each epoch's train view yields batches 0..699 and the test view
700..999 (also when the test view is only read every second epoch), in order; nothing is cached. CPU."""
import torch

import deeplearning4j_amd as D


class _Numbered(D.ListDataSetIterator):
    """Batch i has features filled with i (the reference's DataSetGenerator); counts how often it is reset."""

    def __init__(self, n):
        super().__init__([])
        self.n, self.i, self.resets = n, 0, 0

    def hasNext(self):
        return self.i < self.n

    def next(self, num=None):
        d = D.DataSet(torch.full((4, 3), float(self.i)), torch.zeros(4, 2))
        self.i += 1
        return d

    def reset(self):
        self.i = 0
        self.resets += 1


def test_train_then_test_every_epoch():
    back = _Numbered(1000)
    sp = D.DataSetIteratorSplitter(back, 1000, 0.7)
    train, test = sp.getTrainIterator(), sp.getTestIterator()
    total = 0
    for _ in range(3):
        cnt = 0
        while train.hasNext():
            assert float(train.next().getFeatures()[0, 0]) == cnt
            cnt += 1
            total += 1
        assert cnt == 700
        train.reset()
        while test.hasNext():
            assert float(test.next().getFeatures()[0, 0]) == cnt
            cnt += 1
            total += 1
        assert cnt == 1000
        test.reset()
    assert total == 3000


def test_test_view_every_second_epoch():
    sp = D.DataSetIteratorSplitter(_Numbered(1000), 1000, 0.7)
    train, test = sp.getTrainIterator(), sp.getTestIterator()
    total = 0
    for e in range(4):
        cnt = 0
        while train.hasNext():
            assert float(train.next().getFeatures()[0, 0]) == cnt
            cnt += 1
            total += 1
        if e % 2 == 0:
            while test.hasNext():
                assert float(test.next().getFeatures()[0, 0]) == cnt
                cnt += 1
                total += 1
        train.reset()
    assert total == 700 * 4 + 300 * 2


def test_shuffled_base_raises_and_next_num_refused():
    """Reference DataSetIteratorSplitter.java:158-166: the first train batch of later passes must equal the first
    pass's, or the split moved examples between train and test; next(num) is unsupported."""
    import pytest

    class Shuffling(_Numbered):
        def next(self, num=None):
            d = D.DataSet(torch.full((4, 3), float((self.i + self.resets) % self.n)), torch.zeros(4, 2))
            self.i += 1
            return d

    sp = D.DataSetIteratorSplitter(Shuffling(10), 10, 0.7)
    tr = sp.getTrainIterator()
    with pytest.raises(NotImplementedError):
        tr.next(4)
    while tr.hasNext():
        tr.next()
    tr.reset()
    with pytest.raises(RuntimeError, match="Randomization"):
        tr.next()
