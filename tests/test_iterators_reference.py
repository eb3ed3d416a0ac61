"""Epoch and early-termination iterator wrappers, after the reference's MultipleEpochsIteratorTest and
EarlyTerminationDataSetIteratorTest (deeplearning4j-core/src/test/java/org/deeplearning4j/datasets/iterator/
MultipleEpochsIteratorTest.java:36-160, EarlyTerminationDataSetIteratorTest.java:28-85): MultipleEpochsIterator
replays an iterator for N epochs and counts them, replays a single DataSet (whole, or in next(num) slices), restarts
on reset, and stops after totalIterations minibatches in that mode; EarlyTerminationDataSetIterator yields at most
the termination point's number of minibatches, repeats the same data after reset and refuses further next() calls.
The reference reads Iris / MNIST; a fixed synthetic set of the same shape stands in where MNIST is needed. CPU."""
import pytest
import torch

import deeplearning4j_amd as D


def _examples(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, 4, generator=g)
    y = torch.eye(3)[torch.randint(3, (n,), generator=g)]
    return D.DataSet(x, y)


def _list_iter(n, batch):
    return D.ListDataSetIterator(_examples(n), batch)


def test_multiple_epochs_over_iterator():
    it = D.MultipleEpochsIterator(3, _list_iter(150, 150))
    assert it.hasNext()
    count = 0
    while it.hasNext():
        assert it.next() is not None
        count += 1
    assert count == 3 and it.epochs == 3


def test_multiple_epochs_over_one_dataset():
    ds = _examples(50)
    it = D.MultipleEpochsIterator(3, ds)
    count = 0
    while it.hasNext():
        assert it.next().numExamples() == 50
        count += 1
    assert count == 3 and it.epochs == 3

    it = D.MultipleEpochsIterator(2, _examples(20))
    n = 0
    while it.hasNext():
        assert it.next(10).numExamples() == 10
        n += 1
    assert n == 4 and it.epochs == 2


def test_multiple_epochs_reset_and_total_iterations():
    it = D.MultipleEpochsIterator(10, _list_iter(100, 1))
    first = sum(1 for _ in range(150) if it.next() is not None)
    it.reset()
    rest = 0
    while it.hasNext():
        it.next()
        rest += 1
    assert first + rest == 10 * 100 + 150
    it = D.MultipleEpochsIterator(_list_iter(10000, 1), 24, 136)
    n = 0
    while it.hasNext():
        it.next()
        n += 1
    assert n == 136


def test_early_termination_next_and_reset():
    it = D.EarlyTerminationDataSetIterator(_list_iter(105, 10), 2)
    assert it.hasNext()
    seen = []
    while it.hasNext():
        seen.append(it.next())
    assert len(seen) == 2
    it.reset()
    i = 0
    while it.hasNext():
        ds = it.next()
        assert torch.equal(ds.getFeatures(), seen[i].getFeatures())
        assert torch.equal(ds.getLabels(), seen[i].getLabels())
        i += 1
    assert i == 2


def test_early_termination_limits_next_calls():
    base = _list_iter(105, 10)
    it = D.EarlyTerminationDataSetIterator(base, 1)
    it.next(10)
    assert not it.hasNext()
    it.reset()
    assert it.hasNext()
    it.next(10)
    base.reset()
    with pytest.raises(RuntimeError):
        it.next(10)
    with pytest.raises(ValueError):
        D.EarlyTerminationDataSetIterator(base, 0)
