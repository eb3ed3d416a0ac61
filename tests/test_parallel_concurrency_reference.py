"""Concurrency helpers, after the reference's MultiBooleanTest and AsyncIteratorTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/parallelism/MultiBooleanTest.java:12-75,
AsyncIteratorTest.java:15-35): flag-set all-true / all-false queries, initial values, one-time freezing; the
prefetching iterator yields every element of its source in order and re-raises a producer error. CPU."""
import pytest

from deeplearning4j_amd.parallel import AsyncIterator, MultiBoolean


def test_boolean_1_2():
    b = MultiBoolean(5)
    assert b.allFalse() and not b.allTrue()
    b.set(True, 2)
    assert not b.allFalse() and not b.allTrue()


def test_boolean_3():
    b = MultiBoolean(5)
    for i in range(4):
        b.set(True, i)
    assert not b.allTrue()
    b.set(True, 4)
    assert not b.allFalse() and b.allTrue()
    b.set(False, 2)
    assert not b.allTrue()
    b.set(True, 2)
    assert b.allTrue()


def test_boolean_4_5():
    b = MultiBoolean(5, True)
    assert b.get(1)
    b.set(False, 1)
    assert not b.get(1)
    b = MultiBoolean(5, True, True)
    for i in range(5):
        b.set(False, i)
    for i in range(5):
        b.set(True, i)                   # one-time: frozen once every flag left its initial value
    assert b.allFalse()


def test_async_iterator():
    src = list(range(100000))
    it = AsyncIterator(iter(src), 512)
    cnt = 0
    while it.hasNext():
        assert it.next() == cnt
        cnt += 1
    assert cnt == len(src)


def test_async_iterator_propagates_errors():
    def gen():
        yield 1
        raise RuntimeError("source failed")
    it = AsyncIterator(gen(), 4)
    assert it.next() == 1
    with pytest.raises(RuntimeError, match="source failed"):
        it.hasNext()
