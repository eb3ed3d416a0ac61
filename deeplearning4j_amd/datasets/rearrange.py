"""Train / test directory layout for unstructured (image, text, ...) files (reference deeplearning4j-core/src/main/
java/org/deeplearning4j/datasets/rearrange/LocalUnstructuredDataFormatter.java): every file under ``rootDir`` is
labelled by its parent directory (DIRECTORY) or by its file-name prefix before "_" / "-" (NAME), and copied to
``destinationRootDir/split/{train,test}/<label>/``; the first ``int(total * percentTrain)`` files of a seeded shuffle
go to train."""
import os
import random
import re
import shutil


class LocalUnstructuredDataFormatter:
    class LabelingType:
        DIRECTORY, NAME = "DIRECTORY", "NAME"

    def __init__(self, destinationRootDir, rootDir, labelingType="DIRECTORY", percentTrain=0.8, seed=123):
        self.dest, self.root = str(destinationRootDir), str(rootDir)
        self.labelingType, self.percentTrain, self.seed = labelingType, float(percentTrain), seed
        self.numExamplesTotal = self.numExamplesToTrainOn = self.numTestExamples = 0

    def _label(self, path):
        if self.labelingType == self.LabelingType.DIRECTORY:
            return os.path.basename(os.path.dirname(path))
        return re.split(r"[_\-]", os.path.basename(path), maxsplit=1)[0]

    def rearrange(self):
        files = sorted(os.path.join(d, f) for d, _, fs in os.walk(self.root) for f in fs)
        random.Random(self.seed).shuffle(files)
        self.numExamplesTotal = len(files)
        self.numExamplesToTrainOn = int(len(files) * self.percentTrain)
        self.numTestExamples = self.numExamplesTotal - self.numExamplesToTrainOn
        split = os.path.join(self.dest, "split")
        for i, f in enumerate(files):
            part = "train" if i < self.numExamplesToTrainOn else "test"
            out = os.path.join(split, part, self._label(f))
            os.makedirs(out, exist_ok=True)
            shutil.copy2(f, os.path.join(out, os.path.basename(f)))
        for part in ("train", "test"):
            os.makedirs(os.path.join(split, part), exist_ok=True)

    def getNumExamplesTotal(self):
        return self.numExamplesTotal

    def getNumExamplesToTrainOn(self):
        return self.numExamplesToTrainOn

    def getNumTestExamples(self):
        return self.numTestExamples
