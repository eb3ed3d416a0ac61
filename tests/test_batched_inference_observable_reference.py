"""The BATCHED-mode request batcher, after the reference's BatchedInferenceObservableTest
(deeplearning4j-scaleout/deeplearning4j-scaleout-parallelwrapper/src/test/java/org/deeplearning4j/parallelism/
inference/observers/BatchedInferenceObservableTest.java:20-127): 32 single requests stack into one batch along
dimension 0 (rank-1 rows -> [32, 100]; [1, 3, 72, 72] -> [32, 3, 72, 72]); multi-input requests of 3 examples each
stack per input ([96, 72, 72] and [96, 100]) with example i*3+j from request i; and batched outputs split back into
one array list per request. Plus: incompatible shapes or the example limit start a new batch. CPU."""
import torch

from deeplearning4j_amd.parallel.inference import BatchedInferenceObservable


def test_vertical_batch1():
    ob = BatchedInferenceObservable()
    for i in range(32):
        ob.addInput([torch.full((100,), float(i))], None)
    batches = ob.getInputBatches()
    assert len(batches) == 1
    a = batches[0].getFirst()[0]
    assert a.dim() == 2
    for i in range(32):
        assert abs(float(a[i].mean()) - i) < 1e-3


def test_vertical_batch2():
    ob = BatchedInferenceObservable()
    for i in range(32):
        ob.addInput([torch.full((1, 3, 72, 72), float(i))], None)
    batches = ob.getInputBatches()
    assert len(batches) == 1
    a = batches[0].getFirst()[0]
    assert a.dim() == 4 and a.shape[0] == 32
    for i in range(32):
        assert abs(float(a[i].mean()) - i) < 1e-3


def test_horizontal_batch1():
    ob = BatchedInferenceObservable()
    for i in range(32):
        ob.addInput([torch.full((3, 72, 72), float(i)), torch.full((3, 100), 100.0 + i)], None)
    batches = ob.getInputBatches()
    assert len(batches) == 1
    f0, f1 = batches[0].getFirst()
    assert tuple(f0.shape) == (96, 72, 72) and tuple(f1.shape) == (96, 100)
    for i in range(32):
        for j in range(3):
            assert abs(float(f0[3 * i + j].mean()) - i) < 1e-3
            assert abs(float(f1[3 * i + j].mean()) - (100 + i)) < 1e-3


def test_tears_batch1():
    ob = BatchedInferenceObservable()
    out0, out1 = torch.zeros(32, 10), torch.zeros(32, 15)
    for i in range(32):
        out0[i] = i
        out1[i] = i
        ob.addInput([out0[i:i + 1], out1[i:i + 1]], None)
    ob.outputBatchInputArrays = [[0, 31]]
    ob.setCounter(32)
    ob.setOutputBatches([[out0, out1]])
    outputs = ob.getOutputs()
    for i in range(32):
        assert len(outputs[i]) == 2
        assert abs(float(outputs[i][0].mean()) - i) < 1e-3
        assert abs(float(outputs[i][1].mean()) - i) < 1e-3


def test_incompatible_shapes_and_limit_split_batches():
    ob = BatchedInferenceObservable(batchLimit=4)
    for i in range(6):
        ob.addInput([torch.full((1, 5), float(i))], None)
    ob.addInput([torch.full((1, 7), 9.0)], None)
    batches = ob.getInputBatches()
    assert [tuple(b.getFirst()[0].shape) for b in batches] == [(4, 5), (2, 5), (1, 7)]
    assert ob.outputBatchInputArrays == [[0, 3], [4, 5], [6, 6]]
    ob.setOutputBatches([[b.getFirst()[0] * 2] for b in batches])
    outs = ob.getOutputs()
    assert len(outs) == 7 and float(outs[5][0].mean()) == 10.0 and tuple(outs[6][0].shape) == (1, 7)
