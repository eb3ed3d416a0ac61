"""Iterator / pre-processor scenarios with the reference's numbers: JointParallelDataSetIterator under every
InequalityHandling (CORET: datasets/iterator/JointParallelDataSetIteratorTest.java with its SimpleVariableGenerator),
CombinedMultiDataSetPreProcessor over a MultiNormalizerMinMaxScaler (CombinedPreProcessorTests.java)."""
import torch

from deeplearning4j_amd.datasets import (CombinedMultiDataSetPreProcessor, CombinedPreProcessor, DataSet,
                                         DataSetIterator, InequalityHandling, JointParallelDataSetIterator,
                                         MultiDataSet, MultiNormalizerMinMaxScaler)


class SimpleVariableGenerator(DataSetIterator):
    """Batch i: features all i, labels all i + 0.5 (the reference's tools/SimpleVariableGenerator)."""

    def __init__(self, seed, numBatches, batchSize, numFeatures, numLabels):
        self.n, self.bs, self.nf = numBatches, batchSize, numFeatures
        self.counter = 0

    def hasNext(self):
        return self.counter < self.n

    def next(self, num=None):
        c = self.counter
        self.counter += 1
        return DataSet(torch.full((self.bs, self.nf), float(c)), torch.full((self.bs, self.nf), c + 0.5))

    def reset(self):
        self.counter = 0

    def batch(self):
        return self.bs


def _joint(h, na, nb):
    return (JointParallelDataSetIterator.Builder(h).addSourceIterator(SimpleVariableGenerator(119, na, 32, 100, 10))
            .addSourceIterator(SimpleVariableGenerator(119, nb, 32, 100, 10)).build())


def _mean(t):
    return t.mean().item()


def test_joint_stop_everyone():
    it = _joint(InequalityHandling.STOP_EVERYONE, 100, 100)
    cnt = example = 0
    while it.hasNext():
        ds = it.next()
        assert ds is not None
        assert abs(_mean(ds.getFeatures()) - example) < 1e-3
        assert abs(_mean(ds.getLabels()) - (example + 0.5)) < 1e-3
        cnt += 1
        if cnt % 2 == 0:
            example += 1
    assert (example, cnt) == (100, 200)


def test_joint_pass_null():
    it = _joint(InequalityHandling.PASS_NULL, 200, 100)
    cnt = example = nulls = 0
    while it.hasNext():
        ds = it.next()
        if cnt < 200:
            assert ds is not None
        if ds is None:
            nulls += 1
        cnt += 1
        if cnt % 2 == 0:
            example += 1
    assert (nulls, example, cnt) == (100, 200, 400)


def test_joint_relocate():
    it = _joint(InequalityHandling.RELOCATE, 200, 100)
    cnt = example = 0
    while it.hasNext():
        ds = it.next()
        assert ds is not None
        assert abs(_mean(ds.getFeatures()) - example) < 1e-3
        assert abs(_mean(ds.getLabels()) - (example + 0.5)) < 1e-3
        cnt += 1
        if cnt < 200:
            if cnt % 2 == 0:
                example += 1
        else:
            example += 1
    assert (cnt, example) == (300, 200)


def test_joint_reset():
    it = _joint(InequalityHandling.RESET, 200, 100)
    cnt = cnt_sec = example_sec = example = 0
    while it.hasNext():
        ds = it.next()
        assert ds is not None
        if cnt % 2 == 0 or cnt <= 200:
            want = example
        else:
            want = example_sec
        assert abs(_mean(ds.getFeatures()) - want) < 1e-3, (cnt, want)
        assert abs(_mean(ds.getLabels()) - (want + 0.5)) < 1e-3
        cnt += 1
        if cnt % 2 == 0:
            example += 1
        if cnt > 201 and cnt % 2 == 1:
            cnt_sec += 1
            example_sec += 1
    assert (cnt, example) == (400, 200)


def test_combined_multidataset_preprocessor():
    features = [torch.linspace(100, 200, 20, dtype=torch.float64).reshape(10, 2)]
    mds = MultiDataSet(features, None, None, None)
    scaler = MultiNormalizerMinMaxScaler()
    scaler.fit(mds)

    class AddFive:
        def preProcess(self, m):
            m.getFeatures(0).add_(5)

    pp = CombinedMultiDataSetPreProcessor.Builder().addPreProcessor(scaler).addPreProcessor(1, AddFive()).build()
    pp.preProcess(mds)
    expect = torch.zeros(10, 2, dtype=torch.float64) + torch.linspace(0, 1, 10, dtype=torch.float64).reshape(10, 1) + 5
    torch.testing.assert_close(mds.getFeatures(0), expect)
    # insertion order: addPreProcessor(0, p) runs p first
    order = []

    class Tag:
        def __init__(self, t):
            self.t = t

        def preProcess(self, ds):
            order.append(self.t)
    CombinedPreProcessor.Builder().addPreProcessor(Tag("b")).addPreProcessor(0, Tag("a")).build().preProcess(None)
    assert order == ["a", "b"]
