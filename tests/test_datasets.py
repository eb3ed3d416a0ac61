"""Dataset fetchers and record-reader bridges (reference deeplearning4j-data tests: MnistFetcherTest, IrisUtils,
RecordReaderDataSetiteratorTest, RecordReaderMultiDataSetIteratorTest). No downloads: files are written locally in
the standard formats (IDX, CIFAR binary, image folders); Iris uses the reference's own iris.dat."""
import os

import numpy as np
import pytest
import torch

from deeplearning4j_amd.datasets.datavec import (AlignmentMode, CollectionRecordReader, CollectionSequenceRecordReader,
                                                 CSVRecordReader, CSVSequenceRecordReader, FileSplit,
                                                 ImageRecordReader, NumberedFileInputSplit, ParentPathLabelGenerator,
                                                 RecordReaderDataSetIterator, RecordReaderMultiDataSetIterator,
                                                 SequenceRecordReaderDataSetIterator)
from deeplearning4j_amd.datasets.fetchers import (CifarDataSetIterator, EmnistDataSetIterator, IrisDataSetIterator,
                                                  LFWDataSetIterator, MnistDataSetIterator, UciSequenceDataSetIterator,
                                                  write_idx)
from _ref_fixtures import path as _ref_path

IRIS = _ref_path("deeplearning4j-core/src/main/resources/iris.dat")


def test_mnist_idx(tmp_path):
    rng = np.random.RandomState(0)
    imgs = rng.randint(0, 256, (50, 28, 28))
    lbls = rng.randint(0, 10, 50)
    write_idx(imgs, lbls, str(tmp_path / "train-images-idx3-ubyte"), str(tmp_path / "train-labels-idx1-ubyte"))
    it = MnistDataSetIterator(16, True, 1, dataDir=str(tmp_path), shuffle=False)
    ds = it.next()
    assert ds.features.shape == (16, 784) and ds.labels.shape == (16, 10)
    np.testing.assert_allclose(ds.features[0].numpy(), imgs[0].reshape(-1) / 255.0, atol=1e-6)
    assert int(ds.labels[3].argmax()) == lbls[3]
    n = 16
    while it.hasNext():
        n += it.next().numExamples()
    assert n == 50
    it.reset()
    assert it.next().numExamples() == 16
    b = MnistDataSetIterator(10, 20, 1, binarize=True, train=True, dataDir=str(tmp_path))
    assert set(b.next().features.unique().tolist()) <= {0.0, 1.0}


def test_emnist_letters_labels(tmp_path):
    write_idx(np.zeros((5, 28, 28)), [1, 2, 3, 26, 1], str(tmp_path / "emnist-letters-train-images-idx3-ubyte"),
              str(tmp_path / "emnist-letters-train-labels-idx1-ubyte"))
    it = EmnistDataSetIterator(EmnistDataSetIterator.Set.LETTERS, 5, True, dataDir=str(tmp_path))
    ds = it.next()
    assert ds.labels.shape == (5, 26)
    assert sorted(ds.labels.argmax(1).tolist()) == [0, 0, 1, 2, 25]


@pytest.mark.skipif(not os.path.exists(IRIS), reason="reference iris.dat not present")
def test_iris():
    it = IrisDataSetIterator(150, 150, path=IRIS)
    ds = it.next()
    assert ds.features.shape == (150, 4) and ds.labels.sum(0).tolist() == [50.0, 50.0, 50.0]


def test_cifar_binary(tmp_path):
    rng = np.random.RandomState(1)
    recs = np.concatenate([rng.randint(0, 10, (20, 1)), rng.randint(0, 256, (20, 3072))], 1).astype(np.uint8)
    (tmp_path / "test_batch.bin").write_bytes(recs.tobytes())
    it = CifarDataSetIterator(8, None, train=False, dataDir=str(tmp_path))
    ds = it.next()
    assert ds.features.shape == (8, 3, 32, 32)
    np.testing.assert_allclose(ds.features[2].numpy().reshape(-1), recs[2, 1:] / 255.0, atol=1e-6)
    assert int(ds.labels[2].argmax()) == recs[2, 0]


def test_image_folders(tmp_path):
    from PIL import Image
    for lab in ("alice", "bob"):
        os.makedirs(tmp_path / "lfw" / lab)
        for k in range(3):
            Image.fromarray(np.full((20, 20, 3), 40 * k, np.uint8)).save(tmp_path / "lfw" / lab / f"{k}.png")
    it = LFWDataSetIterator(4, None, (10, 10, 3), dataDir=str(tmp_path))
    ds = it.next()
    assert ds.features.shape == (4, 3, 10, 10) and ds.labels.shape == (4, 2)
    assert it.getLabels() == ["alice", "bob"]
    rr = ImageRecordReader(10, 10, 1, ParentPathLabelGenerator()).initialize(FileSplit(str(tmp_path / "lfw")))
    rit = RecordReaderDataSetIterator(rr, 6, 1, 2)
    d = rit.next()
    assert d.features.shape == (6, 1, 10, 10) and d.labels.sum().item() == 6


def test_uci_sequences(tmp_path):
    os.makedirs(tmp_path / "uci")
    np.savetxt(tmp_path / "uci" / "synthetic_control.data", np.random.RandomState(0).randn(600, 60))
    it = UciSequenceDataSetIterator(32, True, dataDir=str(tmp_path / "uci"))
    ds = it.next()
    assert ds.features.shape == (32, 1, 60) and ds.labels.shape == (32, 6, 60)
    assert ds.labelsMask[:, -1].sum() == 32 and ds.labelsMask[:, :-1].sum() == 0


def test_csv_record_reader_classification_and_regression(tmp_path):
    p = tmp_path / "d.csv"
    p.write_text("a,b,c,label\n1,2,3,0\n4,5,6,2\n7,8,9,1\n")
    rr = CSVRecordReader(1, ",").initialize(FileSplit(str(p)))
    it = RecordReaderDataSetIterator(rr, 2, 3, 3)
    ds = it.next()
    assert ds.features.tolist() == [[1, 2, 3], [4, 5, 6]]
    assert ds.labels.tolist() == [[1, 0, 0], [0, 0, 1]]
    assert it.next().numExamples() == 1 and not it.hasNext()
    it.reset()
    reg = RecordReaderDataSetIterator.Builder(rr, 3).regression(1, 2).build()
    d = reg.next()
    assert d.features.tolist() == [[1, 0], [4, 2], [7, 1]] and d.labels.tolist() == [[2, 3], [5, 6], [8, 9]]


def test_sequence_record_reader(tmp_path):
    for i, T in enumerate((4, 2)):
        (tmp_path / f"f_{i}.csv").write_text("\n".join(f"{t},{t * 10}" for t in range(T)))
        (tmp_path / f"l_{i}.csv").write_text("\n".join(str(t % 3) for t in range(T)))
    fr = CSVSequenceRecordReader().initialize(NumberedFileInputSplit(str(tmp_path / "f_%d.csv"), 0, 1))
    lr = CSVSequenceRecordReader().initialize(NumberedFileInputSplit(str(tmp_path / "l_%d.csv"), 0, 1))
    it = SequenceRecordReaderDataSetIterator(fr, lr, 2, 3, False, AlignmentMode.ALIGN_END)
    ds = it.next()
    assert ds.features.shape == (2, 2, 4) and ds.labels.shape == (2, 3, 4)
    assert ds.featuresMask.tolist() == [[1, 1, 1, 1], [0, 0, 1, 1]]
    assert ds.features[1, 1, 3].item() == 10.0
    # single reader with the label in the last column
    sr = CollectionSequenceRecordReader([[[0.5, 1], [0.25, 0]]])
    d = SequenceRecordReaderDataSetIterator(sr, 1, 2, 1).next()
    assert d.features.shape == (1, 1, 2) and d.labels[0, :, 0].tolist() == [0, 1]


def test_record_reader_multi_dataset():
    rr = CollectionRecordReader([[1, 2, 3, 0], [4, 5, 6, 1]])
    it = RecordReaderMultiDataSetIterator.Builder(2).addReader("r", rr).addInput("r", 0, 1).addInput("r", 2, 2) \
        .addOutputOneHot("r", 3, 2).build()
    m = it.next()
    assert m.features[0].tolist() == [[1, 2], [4, 5]] and m.features[1].tolist() == [[3], [6]]
    assert m.labels[0].tolist() == [[1, 0], [0, 1]]


def test_dataset_save_load_file_iterator_and_splitter(tmp_path):
    from deeplearning4j_amd.datasets import (DataSet, DataSetIteratorSplitter, FileDataSetIterator,
                                             ListDataSetIterator, ReconstructionDataSetIterator)
    d = DataSet(torch.randn(4, 3), torch.eye(4)[:, :2], None, torch.ones(4, 2))
    for i in range(3):
        d.save(str(tmp_path / f"b{i}.bin"))
    it = FileDataSetIterator(str(tmp_path))
    r = it.next()
    assert torch.equal(r.features, d.features) and r.featuresMask is None and torch.equal(r.labelsMask, d.labelsMask)
    base = ListDataSetIterator([DataSet(torch.full((2, 1), float(k)), torch.zeros(2, 1)) for k in range(10)])
    sp = DataSetIteratorSplitter(base, 10, 0.7)
    assert sum(1 for _ in sp.getTrainIterator()) == 7 and sum(1 for _ in sp.getTestIterator()) == 3
    rec = ReconstructionDataSetIterator(ListDataSetIterator([d]))
    x = rec.next()
    assert torch.equal(x.features, x.labels)


def test_dataset_feature_transforms():
    """ND4J DataSet transforms used by the reference tests: per-column standardisation (a constant column stays 0),
    min/max rescale, binarize, label counts and example selection."""
    from deeplearning4j_amd.datasets.dataset import DataSet
    g = torch.Generator().manual_seed(0)
    x = torch.rand(50, 4, generator=g) * 7 + 3
    x[:, 2] = 5.0
    y = torch.nn.functional.one_hot(torch.arange(50) % 3, 3).float()
    ds = DataSet(x.clone(), y)
    ds.normalizeZeroMeanZeroUnitVariance()
    f = ds.getFeatures()
    assert torch.allclose(f.mean(0), torch.zeros(4), atol=1e-5)
    assert torch.allclose(f[:, [0, 1, 3]].std(0), torch.ones(3), atol=1e-5)
    assert torch.all(f[:, 2] == 0)
    ds2 = DataSet(x.clone(), y)
    ds2.scaleMinAndMax(-1.0, 1.0)
    f2 = ds2.getFeatures()
    assert torch.allclose(f2[:, [0, 1, 3]].amin(0), -torch.ones(3)) and torch.allclose(f2[:, [0, 1, 3]].amax(0), torch.ones(3))
    ds3 = DataSet(x.clone(), y)
    ds3.binarize(6.5)
    assert set(ds3.getFeatures().unique().tolist()) <= {0.0, 1.0}
    assert ds.labelCounts() == {0: 17, 1: 17, 2: 16}
    one = ds.get(4)
    assert one.numExamples() == 1 and torch.equal(one.getLabels()[0], y[4])
    assert ds.get([1, 2, 3]).numExamples() == 3
