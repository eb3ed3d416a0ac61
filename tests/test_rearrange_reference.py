"""LocalUnstructuredDataFormatter, after the reference's LocalUnstructuredDataFormatterTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/datasets/rearrange/LocalUnstructuredDataFormatterTest.java:
20-60): a directory-labelled tree is split 0.8 / 0.2 into split/train and split/test, the file counts match the
formatter's totals. The reference downloads LFW; a generated 7-person tree of small files stands in. CPU."""
import os

from deeplearning4j_amd.datasets.rearrange import LocalUnstructuredDataFormatter


def _count(d):
    return sum(len(fs) for _, _, fs in os.walk(d))


def test_rearrange(tmp_path):
    src = tmp_path / "lfw"
    for p in range(7):
        (src / f"person_{p}").mkdir(parents=True)
        for i in range(p + 3):
            (src / f"person_{p}" / f"img_{i}.jpg").write_bytes(bytes([p, i]))
    dest = tmp_path / "rearrangedlfw"
    f = LocalUnstructuredDataFormatter(dest, src, LocalUnstructuredDataFormatter.LabelingType.DIRECTORY, 0.8)
    f.rearrange()
    split = dest / "split"
    assert len(os.listdir(split)) == 2
    assert f.getNumExamplesTotal() == _count(split) == _count(src)
    assert f.getNumExamplesToTrainOn() == _count(split / "train") == int(0.8 * _count(src))
    assert f.getNumTestExamples() == _count(split / "test")
    assert set(os.listdir(split / "train")) <= {f"person_{p}" for p in range(7)}
