"""Zoo utilities (reference deeplearning4j-zoo: util/BaseLabels.java, util/imagenet/ImageNetLabels.java,
util/darknet/*Labels.java, ClassPrediction.java, ModelSelector.java, ZooModel.java:51-93 checksum verification), after
the reference's TestImageNet / TestInstantiation. The pretrained weight files cannot be downloaded here, so the label
decoding is checked on one-hot probability rows at the class the reference's golden-retriever image decodes to, and
the Adler-32 verification on local files. CPU."""
import os
import zlib

import pytest
import torch

from deeplearning4j_amd.models import (COCOLabels, ClassPrediction, DarknetLabels, ImageNetLabels, LeNet, ModelSelector,
                                       PretrainedType, ResNet50, VOCLabels, ZooType, adler32_file)
from deeplearning4j_amd.models import zoo as Z


def test_imagenet_labels_top_k_and_string_form():
    lab = ImageNetLabels()
    assert lab.numLabels() == 1000 and lab.getLabel(207) == "golden_retriever" and lab.getLabel(0) == "tench"
    p = torch.full((2, 1000), 1e-4)
    p[0, 207], p[0, 208], p[1, 1] = 0.9, 0.05, 0.7
    dec = lab.decodePredictions(p, 3)
    assert [c.getNumber() for c in dec[0]] == [207, 208, 0]        # ties (1e-4) keep the lower index first
    assert dec[0][0] == ClassPrediction(207, "golden_retriever", float(torch.tensor(0.9, dtype=torch.float32)))
    assert dec[1][0].getLabel() == "goldfish"
    s = lab.decodePredictions(p[:1])                                 # the reference's string form (top five)
    assert s.startswith("Predictions for batch  :") and "golden_retriever" in s and s.count("\n\t") == 5
    assert "90.000000%, golden_retriever" in s


def test_darknet_voc_coco_labels():
    dn = DarknetLabels()
    i = dn.labels.index("golden retriever")
    row = torch.zeros(1, len(dn.labels))
    row[0, i] = 1.0
    assert dn.decodePredictions(row, 10)[0][0].getLabel() == "golden retriever"
    assert DarknetLabels(False).numLabels() == dn.numLabels()
    voc, coco = VOCLabels(), COCOLabels()
    assert voc.numLabels() == 20 and coco.numLabels() == 80
    v = torch.zeros(20)
    v[voc.labels.index("dog")] = 0.8
    assert voc.decodePredictions(v.reshape(-1, 1), 1)[0][0].getLabel() == "dog"   # a column vector is one row
    c = torch.zeros(1, 80)
    c[0, coco.labels.index("dog")] = 0.6
    assert coco.decodePredictions(c, 1)[0][0].getLabel() == "dog"
    with pytest.raises(ValueError):
        voc.decodePredictions(torch.zeros(1, 21), 1)


def test_model_selector_groups_and_types():
    cnn = ModelSelector.select(ZooType.CNN, numLabels=10)
    assert set(cnn) == {ZooType.SIMPLECNN, ZooType.ALEXNET, ZooType.LENET, ZooType.GOOGLENET, ZooType.RESNET50,
                        ZooType.VGG16, ZooType.VGG19, ZooType.DARKNET19, ZooType.TINYYOLO, ZooType.YOLO2}
    assert all(m.numLabels == 10 and m.seed == 123 for m in cnn.values())
    allm = ModelSelector.select(ZooType.ALL)
    assert ZooType.TEXTGENLSTM in allm and len(allm) == 11
    two = ModelSelector.select(ZooType.LENET, ZooType.RESNET50)
    assert set(two) == {ZooType.LENET, ZooType.RESNET50} and two[ZooType.LENET].numLabels == 0
    assert isinstance(ModelSelector.select(ZooType.RESNET50)[ZooType.RESNET50], ResNet50)
    assert ResNet50().zooType() == ZooType.RESNET50 and ResNet50().metaDataFull().getZooType() == ZooType.RESNET50


def test_pretrained_metadata_and_checksum(tmp_path, monkeypatch):
    assert ResNet50().pretrainedChecksum() == 1982516793
    assert ResNet50().pretrainedUrl().endswith("resnet50_dl4j_inference.zip")
    assert LeNet().pretrainedAvailable(PretrainedType.MNIST) and not LeNet().pretrainedAvailable()
    assert Z.Darknet19(inputShape=[3, 448, 448]).pretrainedChecksum() == 870575230
    assert Z.Darknet19().pretrainedChecksum() == 3952910425
    assert Z.VGG16().pretrainedChecksum(PretrainedType.CIFAR10) == 2192260131
    f = tmp_path / "blob.bin"
    data = os.urandom(3 << 20)
    f.write_bytes(data)
    assert adler32_file(str(f), chunk=1 << 16) == zlib.adler32(data) & 0xFFFFFFFF
    # a cached file with the wrong checksum is refused and removed (ZooModel.java:76-82)
    monkeypatch.setattr(Z, "ROOT_CACHE_DIR", str(tmp_path))
    cached = tmp_path / "resnet50_dl4j_inference.zip"
    cached.write_bytes(b"not the weights")
    with pytest.raises(RuntimeError, match="failed checksum"):
        ResNet50().initPretrained()
    assert not cached.exists()
    with pytest.raises(RuntimeError, match="cannot be downloaded"):
        ResNet50().initPretrained(PretrainedType.IMAGENET)
    with pytest.raises(NotImplementedError):
        Z.AlexNet().initPretrained()


def test_pretrained_restore_from_local_zip(tmp_path):
    """A local ModelSerializer zip given by path restores (no checksum: the file is the user's, not the zoo's)."""
    from deeplearning4j_amd.utils.model_serializer import ModelSerializer
    net = LeNet(numLabels=10).init()
    p = tmp_path / "lenet.zip"
    ModelSerializer.writeModel(net, str(p), True)
    back = LeNet(numLabels=10).initPretrained(str(p))
    assert torch.equal(back.params(), net.params())
