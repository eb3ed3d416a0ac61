"""Class-label decoding for zoo model outputs (reference deeplearning4j-zoo/src/main/java/org/deeplearning4j/zoo/util/:
Labels.java, BaseLabels.java:27-95, ClassPrediction.java, imagenet/ImageNetLabels.java:26-77,
darknet/{DarknetLabels,VOCLabels,COCOLabels}.java).

The label lists are the reference's own resource files, vendored under ``models/resources`` (ImageNet class index JSON,
darknet ImageNet short / long names, VOC and COCO names).

* ``getLabel(n)`` — the description of class ``n``.
* ``decodePredictions(predictions, n)`` — per row of a ``[batch, classes]`` probability matrix (a column vector is
  treated as one row, as the reference ravels it), the ``n`` most probable classes as ``ClassPrediction(number, label,
  probability)``, in descending probability. Ties keep the lower class index first (a stable sort; the reference sorts
  a [index; prob] matrix by its probability row).
* ``ImageNetLabels.decodePredictions(predictions)`` with no ``n`` keeps the reference's string form: per batch row a
  "Predictions for batch ..." header and the top five as ``"\\n\\t%3f%%, label"``.
"""
import json
import os

import torch

_RES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resources")


class ClassPrediction:
    """One decoded class: index, label text and probability (reference ClassPrediction.java)."""

    def __init__(self, number, label, probability):
        self.number = int(number)
        self.label = label
        self.probability = float(probability)

    def getNumber(self):
        return self.number

    def getLabel(self):
        return self.label

    def getProbability(self):
        return self.probability

    def __eq__(self, other):
        return isinstance(other, ClassPrediction) and (self.number, self.label, self.probability) == \
            (other.number, other.label, other.probability)

    def __repr__(self):
        return f"ClassPrediction(number={self.number},label={self.label},probability={self.probability})"

    __str__ = __repr__


def _as_matrix(predictions):
    if hasattr(predictions, "toTensor"):
        predictions = predictions.toTensor()
    elif hasattr(predictions, "tensor") and not isinstance(predictions, torch.Tensor):
        predictions = predictions.tensor
    p = torch.as_tensor(predictions).detach().to("cpu", torch.float64)
    if p.dim() == 1:
        p = p.reshape(1, -1)
    elif p.dim() == 2 and p.shape[1] == 1 and p.shape[0] > 1:
        p = p.reshape(1, -1)          # column vector: ravel to one row (BaseLabels.java:58-62)
    if p.dim() != 2:
        raise ValueError(f"predictions must be [batch, classes], got shape {tuple(p.shape)}")
    return p


class BaseLabels:
    """A label list read from a text resource, one label per line (BaseLabels.java:27-74)."""

    resource = None

    def __init__(self, textResource=None):
        self.labels = self.getLabels(textResource or self.resource)

    def getLabels(self, textResource=None):
        path = textResource if os.path.isabs(textResource) else os.path.join(_RES, textResource)
        with open(path, encoding="utf-8") as fh:
            return [ln.rstrip("\r\n") for ln in fh]

    def getLabel(self, n):
        return self.labels[n]

    def numLabels(self):
        return len(self.labels)

    def decodePredictions(self, predictions, n=5):
        p = _as_matrix(predictions)
        if p.shape[1] > len(self.labels):
            raise ValueError(f"{p.shape[1]} prediction columns but only {len(self.labels)} labels")
        n = min(int(n), p.shape[1])
        out = []
        for row in p:
            order = torch.sort(-row, stable=True).indices[:n]
            out.append([ClassPrediction(int(i), self.getLabel(int(i)), float(row[i])) for i in order])
        return out


class ImageNetLabels(BaseLabels):
    """The 1000 ImageNet classes from imagenet_class_index.json (ImageNetLabels.java:34-48: entry i's second field)."""

    resource = "imagenet_class_index.json"

    def getLabels(self, textResource=None):
        with open(os.path.join(_RES, "imagenet_class_index.json"), encoding="utf-8") as fh:
            m = json.load(fh)
        return [m[str(i)][1] for i in range(len(m))]

    def decodePredictions(self, predictions, n=None):
        if n is not None:
            return super().decodePredictions(predictions, n)
        # the reference's string form (ImageNetLabels.java:60-77), top five of every batch row
        p = _as_matrix(predictions)
        text = ""
        for b, row in enumerate(p):
            text += "Predictions for batch " + (str(b) if p.shape[0] > 1 else "") + " :"
            for cp in super().decodePredictions(row.reshape(1, -1), 5)[0]:
                pct = float(torch.tensor(cp.probability, dtype=torch.float32) * 100)   # Java float arithmetic
                text += "\n\t" + f"{pct:3f}" + "%, " + cp.label
        return text


class DarknetLabels(BaseLabels):
    """The darknet ImageNet label list (21,842 synsets): short names (default) or long labels (DarknetLabels.java:30-38)."""

    def __init__(self, shortnames=True):
        super().__init__("imagenet.shortnames.list" if shortnames else "imagenet.labels.list")


class VOCLabels(BaseLabels):
    """The 20 Pascal VOC classes (VOCLabels.java) — TinyYOLO's output classes."""

    resource = "voc.names"


class COCOLabels(BaseLabels):
    """The 80 COCO classes (COCOLabels.java) — YOLO2's output classes."""

    resource = "coco.names"


def adler32_file(path, chunk=1 << 20):
    """Adler-32 of a file, streamed (the reference's FileUtils.checksum(file, new Adler32()), ZooModel.java:71-74)."""
    import zlib
    v = 1
    with open(path, "rb") as fh:
        while True:
            b = fh.read(chunk)
            if not b:
                break
            v = zlib.adler32(b, v)
    return v & 0xFFFFFFFF
