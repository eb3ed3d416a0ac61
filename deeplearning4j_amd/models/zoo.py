"""Model zoo (reference deeplearning4j-zoo/src/main/java/org/deeplearning4j/zoo/model/*).

Every zoo model exposes ``conf()`` / ``graphBuilder()`` and ``init()`` like the reference. Pretrained
downloads are not available offline; ``initPretrained`` loads a local ModelSerializer zip if given.

ResNet50 here is the reference's zoo variant (ZOO:model/ResNet50.java:171-225): stride-2 stage 2
(convBlock(..., "2", "a", {2,2}) :194) and a MAX 3x3/2 "avgpool" head (:214-216) — ≈1.11 GMAC/img
forward at 224². ``ResNet50(variant="canonical")`` builds the standard ResNet-50 (stride-1 stage 2,
global average pool, ≈3.83 GMAC/img) for comparison.
"""
from ..nn.conf import (Activation, ActivationLayer, AdaDelta, BackpropType, BatchNormalization, ConvolutionLayer,
                       ConvolutionMode, DataType, DenseLayer, DropoutLayer, ElementWiseVertex, GlobalPoolingLayer,
                       GravesLSTM, InputType, LocalResponseNormalization, LossFunction, MergeVertex,
                       NeuralNetConfiguration, Nesterovs, NormalDistribution, OptimizationAlgorithm, OutputLayer,
                       PoolingType, RmsProp, RnnOutputLayer, ScaleVertex, SubsamplingLayer, WeightInit, ZeroPaddingLayer,
                       Adam)
from ..nn.conf.enums import WorkspaceMode
from ..nn.graph import ComputationGraph
from ..nn.multilayer import MultiLayerNetwork


class ZooModel:
    def __init__(self, numLabels=1000, seed=123, inputShape=None, dataType=DataType.FLOAT,
                 workspaceMode=WorkspaceMode.ENABLED, **kw):
        self.numLabels = numLabels
        self.seed = seed
        self.inputShape = inputShape or self.DEFAULT_SHAPE
        self.dataType = DataType.of(dataType)
        self.workspaceMode = workspaceMode
        for k, v in kw.items():
            setattr(self, k, v)

    DEFAULT_SHAPE = [3, 224, 224]

    @classmethod
    def builder(cls):
        return _ZooBuilder(cls)

    def metaData(self):
        return {"inputShape": [self.inputShape], "numOutputs": 1}

    def setInputShape(self, shape):
        self.inputShape = shape[0] if isinstance(shape[0], (list, tuple)) else shape

    # pretrained weight files of the reference zoo: {PretrainedType: (url, Adler-32)} per model class name
    # (ZOO:model/*.java pretrainedUrl / pretrainedChecksum); checked against any local copy before restoring
    def pretrainedUrl(self, pretrainedType=None):
        e = _PRETRAINED.get(self._pretrained_key(), {}).get(pretrainedType or PretrainedType.IMAGENET)
        return None if e is None else e[0]

    def pretrainedChecksum(self, pretrainedType=None):
        e = _PRETRAINED.get(self._pretrained_key(), {}).get(pretrainedType or PretrainedType.IMAGENET)
        return 0 if e is None else e[1]

    def _pretrained_key(self):
        return type(self).__name__

    def pretrainedAvailable(self, pretrainedType=None):
        return self.pretrainedUrl(pretrainedType) is not None

    def zooType(self):
        return ZooType.of_model(type(self).__name__)

    def modelType(self):
        return ComputationGraph if hasattr(self, "graphBuilder") else MultiLayerNetwork

    def metaDataFull(self):
        return ModelMetaData([list(self.inputShape)], 1, self.zooType())

    def initPretrained(self, pretrainedType=None, path=None, verify=True):
        """Restore pretrained weights (ZOO:ZooModel.java:51-93). No download is possible here: the weight file is
        ``path`` (a ModelSerializer zip) or the file the reference would have cached under
        ``~/.deeplearning4j/models/<name of the url>``. When the model has a known Adler-32 checksum for
        ``pretrainedType`` the file is verified first and a mismatch raises (a mismatching cached file is deleted,
        as the reference does; a file passed by path is left alone). ``initPretrained("<path>")`` also works."""
        import os
        if isinstance(pretrainedType, str) and not hasattr(PretrainedType, pretrainedType):
            pretrainedType, path = None, pretrainedType
        pretrainedType = PretrainedType.of(pretrainedType) if pretrainedType is not None else None
        url = self.pretrainedUrl(pretrainedType)
        cached = False
        if path is None:
            if url is None:
                raise NotImplementedError(f"Pretrained {pretrainedType or PretrainedType.IMAGENET} weights are not "
                                          f"available for this model.")
            path = os.path.join(ROOT_CACHE_DIR, os.path.basename(url))
            cached = True
            if not os.path.exists(path):
                raise RuntimeError(f"Pretrained weights cannot be downloaded in this environment: place {url} at "
                                   f"{path} or pass a local ModelSerializer zip path")
        expected = self.pretrainedChecksum(pretrainedType) if (url is not None and verify) else 0
        if expected:
            from .labels import adler32_file
            local = adler32_file(path)
            if local != expected:
                if cached:
                    os.remove(path)
                raise RuntimeError(f"Pretrained model file failed checksum (Adler-32 {local}, expecting {expected})")
        from ..utils.model_serializer import ModelSerializer
        return ModelSerializer.restoreModel(path)

    def _builder(self):
        return NeuralNetConfiguration.Builder().seed(self.seed).dataType(self.dataType) \
            .trainingWorkspaceMode(self.workspaceMode).inferenceWorkspaceMode(self.workspaceMode)


import enum as _enum
import os as _os

ROOT_CACHE_DIR = _os.path.join(_os.path.expanduser("~"), ".deeplearning4j", "models")


class PretrainedType(_enum.Enum):
    """Datasets pretrained weights exist for (ZOO:PretrainedType.java)."""
    IMAGENET = "IMAGENET"
    MNIST = "MNIST"
    CIFAR10 = "CIFAR10"
    VGGFACE = "VGGFACE"

    @classmethod
    def of(cls, v):
        return v if isinstance(v, cls) else cls[str(v).upper()]


class ZooType(_enum.Enum):
    """Model selectors (ZOO:ZooType.java): single models plus the ALL / CNN / RNN groups."""
    ALL = "ALL"
    CNN = "CNN"
    SIMPLECNN = "SIMPLECNN"
    ALEXNET = "ALEXNET"
    LENET = "LENET"
    GOOGLENET = "GOOGLENET"
    VGG16 = "VGG16"
    VGG19 = "VGG19"
    RESNET50 = "RESNET50"
    INCEPTIONRESNETV1 = "INCEPTIONRESNETV1"
    FACENETNN4SMALL2 = "FACENETNN4SMALL2"
    RNN = "RNN"
    TEXTGENLSTM = "TEXTGENLSTM"
    DARKNET19 = "DARKNET19"
    TINYYOLO = "TINYYOLO"
    YOLO2 = "YOLO2"

    @classmethod
    def of_model(cls, class_name):
        m = {"TextGenerationLSTM": "TEXTGENLSTM"}
        return cls[m.get(class_name, class_name.upper())] if m.get(class_name, class_name.upper()) in cls.__members__ \
            else None


class ModelMetaData:
    """Input shapes / output count / zoo type of a model (ZOO:ModelMetaData.java)."""

    def __init__(self, inputShape, numOutputs, zooType):
        self.inputShape, self.numOutputs, self.zooType = inputShape, numOutputs, zooType

    def getInputShape(self):
        return self.inputShape

    def getNumOutputs(self):
        return self.numOutputs

    def getZooType(self):
        return self.zooType

    def useMDS(self):
        return len(self.inputShape) > 1


_BLOB = "http://blob.deeplearning4j.org/models/"
_PRETRAINED = {
    "ResNet50": {PretrainedType.IMAGENET: (_BLOB + "resnet50_dl4j_inference.zip", 1982516793)},
    "LeNet": {PretrainedType.MNIST: (_BLOB + "lenet_dl4j_mnist_inference.zip", 1906861161)},
    "GoogLeNet": {PretrainedType.IMAGENET: (_BLOB + "googlenet_dl4j_inference.zip", 3337733202)},
    "VGG16": {PretrainedType.IMAGENET: (_BLOB + "vgg16_dl4j_inference.zip", 3501732770),
              PretrainedType.CIFAR10: (_BLOB + "vgg16_dl4j_cifar10_inference.v1.zip", 2192260131),
              PretrainedType.VGGFACE: (_BLOB + "vgg16_dl4j_vggface_inference.v1.zip", 2706403553)},
    "VGG19": {PretrainedType.IMAGENET: (_BLOB + "vgg19_dl4j_inference.zip", 2782932419)},
    "TinyYOLO": {PretrainedType.IMAGENET: (_BLOB + "tiny-yolo-voc_dl4j_inference.v1.zip", 2004171617)},
    "YOLO2": {PretrainedType.IMAGENET: (_BLOB + "yolo2_dl4j_inference.v1.zip", 1357637732)},
    "Darknet19": {PretrainedType.IMAGENET: (_BLOB + "darknet19_dl4j_inference.v1.zip", 3952910425)},
    "Darknet19@448": {PretrainedType.IMAGENET: (_BLOB + "darknet19_448_dl4j_inference.v1.zip", 870575230)},
}


class _ZooBuilder:
    def __init__(self, cls):
        self.cls = cls
        self.kw = {}

    def __getattr__(self, name):
        def setter(v):
            self.kw[name] = v
            return self
        return setter

    def build(self):
        return self.cls(**self.kw)


# ------------------------------------------------------------------------------------------ ResNet50
class ResNet50(ZooModel):
    """variant: "dl4j" (reference zoo graph, default) or "canonical"."""

    def __init__(self, numLabels=1000, seed=123, inputShape=None, variant="dl4j", updater=None, weightInit=None,
                 **kw):
        super().__init__(numLabels, seed, inputShape, **kw)
        self.variant = variant
        self.updater = updater
        # the reference zoo initialises from N(0, 0.5) (ZOO:model/ResNet50.java), which saturates the random-init
        # softmax; numerics checks pass e.g. WeightInit.RELU instead
        self.weightInit = weightInit

    def _identity(self, g, k, filters, stage, block, inp):
        conv, bn, act, sc = (f"res{stage}{block}_branch", f"bn{stage}{block}_branch", f"act{stage}{block}_branch",
                             f"short{stage}{block}_branch")
        g.addLayer(conv + "2a", ConvolutionLayer.Builder([1, 1]).nOut(filters[0]).build(), inp)
        g.addLayer(bn + "2a", BatchNormalization(), conv + "2a")
        g.addLayer(act + "2a", ActivationLayer.Builder().activation(Activation.RELU).build(), bn + "2a")
        g.addLayer(conv + "2b", ConvolutionLayer.Builder(k).nOut(filters[1]).convolutionMode(ConvolutionMode.Same)
                   .build(), act + "2a")
        g.addLayer(bn + "2b", BatchNormalization(), conv + "2b")
        g.addLayer(act + "2b", ActivationLayer.Builder().activation(Activation.RELU).build(), bn + "2b")
        g.addLayer(conv + "2c", ConvolutionLayer.Builder([1, 1]).nOut(filters[2]).build(), act + "2b")
        g.addLayer(bn + "2c", BatchNormalization(), conv + "2c")
        g.addVertex(sc, ElementWiseVertex(ElementWiseVertex.Op.Add), bn + "2c", inp)
        g.addLayer(conv, ActivationLayer.Builder().activation(Activation.RELU).build(), sc)

    def _conv_block(self, g, k, filters, stage, block, stride, inp):
        conv, bn, act, sc = (f"res{stage}{block}_branch", f"bn{stage}{block}_branch", f"act{stage}{block}_branch",
                             f"short{stage}{block}_branch")
        g.addLayer(conv + "2a", ConvolutionLayer.Builder([1, 1], stride).nOut(filters[0]).build(), inp)
        g.addLayer(bn + "2a", BatchNormalization(), conv + "2a")
        g.addLayer(act + "2a", ActivationLayer.Builder().activation(Activation.RELU).build(), bn + "2a")
        g.addLayer(conv + "2b", ConvolutionLayer.Builder(k).nOut(filters[1]).convolutionMode(ConvolutionMode.Same)
                   .build(), act + "2a")
        g.addLayer(bn + "2b", BatchNormalization(), conv + "2b")
        g.addLayer(act + "2b", ActivationLayer.Builder().activation(Activation.RELU).build(), bn + "2b")
        g.addLayer(conv + "2c", ConvolutionLayer.Builder([1, 1]).nOut(filters[2]).build(), act + "2b")
        g.addLayer(bn + "2c", BatchNormalization(), conv + "2c")
        g.addLayer(conv + "1", ConvolutionLayer.Builder([1, 1], stride).nOut(filters[2]).build(), inp)
        g.addLayer(bn + "1", BatchNormalization(), conv + "1")
        g.addVertex(sc, ElementWiseVertex(ElementWiseVertex.Op.Add), bn + "2c", bn + "1")
        g.addLayer(conv, ActivationLayer.Builder().activation(Activation.RELU).build(), sc)

    def graphBuilder(self):
        c, h, w = self.inputShape
        upd = self.updater if self.updater is not None else RmsProp(0.1, 0.96, 0.001)
        g = (self._builder().activation(Activation.IDENTITY)
             .optimizationAlgo(OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT)
             .updater(upd).weightInit(self.weightInit if self.weightInit is not None else NormalDistribution(0.0, 0.5))
             .l1(1e-7).l2(5e-5).miniBatch(True)
             .convolutionMode(ConvolutionMode.Truncate).graphBuilder())
        g.addInputs("input").setInputTypes(InputType.convolutional(h, w, c))
        g.addLayer("stem-zero", ZeroPaddingLayer.Builder(3, 3).build(), "input")
        g.addLayer("stem-cnn1", ConvolutionLayer.Builder([7, 7], [2, 2]).nOut(64).build(), "stem-zero")
        g.addLayer("stem-batch1", BatchNormalization(), "stem-cnn1")
        g.addLayer("stem-act1", ActivationLayer.Builder().activation(Activation.RELU).build(), "stem-batch1")
        g.addLayer("stem-maxpool1", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).build(), "stem-act1")
        s2 = [2, 2] if self.variant == "dl4j" else [1, 1]
        self._conv_block(g, [3, 3], [64, 64, 256], "2", "a", s2, "stem-maxpool1")
        self._identity(g, [3, 3], [64, 64, 256], "2", "b", "res2a_branch")
        self._identity(g, [3, 3], [64, 64, 256], "2", "c", "res2b_branch")
        self._conv_block(g, [3, 3], [128, 128, 512], "3", "a", [2, 2], "res2c_branch")
        for b, prev in zip("bcd", ["res3a_branch", "res3b_branch", "res3c_branch"]):
            self._identity(g, [3, 3], [128, 128, 512], "3", b, prev)
        self._conv_block(g, [3, 3], [256, 256, 1024], "4", "a", [2, 2], "res3d_branch")
        for b, prev in zip("bcdef", ["res4a_branch", "res4b_branch", "res4c_branch", "res4d_branch",
                                     "res4e_branch"]):
            self._identity(g, [3, 3], [256, 256, 1024], "4", b, prev)
        self._conv_block(g, [3, 3], [512, 512, 2048], "5", "a", [2, 2], "res4f_branch")
        self._identity(g, [3, 3], [512, 512, 2048], "5", "b", "res5a_branch")
        self._identity(g, [3, 3], [512, 512, 2048], "5", "c", "res5b_branch")
        if self.variant == "dl4j":
            g.addLayer("avgpool", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3]).build(), "res5c_branch")
        else:
            g.addLayer("avgpool", GlobalPoolingLayer.Builder(PoolingType.AVG).build(), "res5c_branch")
        g.addLayer("output", OutputLayer.Builder(LossFunction.NEGATIVELOGLIKELIHOOD).nOut(self.numLabels)
                   .activation(Activation.SOFTMAX).build(), "avgpool")
        g.setOutputs("output").backprop(True).pretrain(False)
        return g

    def conf(self):
        return self.graphBuilder().build()

    def init(self, device=None):
        net = ComputationGraph(self.conf())
        net.init(device=device)
        return net


# -------------------------------------------------------------------------------------------- LeNet
class LeNet(ZooModel):
    DEFAULT_SHAPE = [1, 28, 28]

    def __init__(self, numLabels=10, seed=123, inputShape=None, **kw):
        super().__init__(numLabels, seed, inputShape, **kw)

    def conf(self):
        c, h, w = self.inputShape
        return (self._builder().activation(Activation.IDENTITY).weightInit(WeightInit.XAVIER)
                .optimizationAlgo(OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT).updater(AdaDelta())
                .convolutionMode(ConvolutionMode.Same).list()
                .layer(0, ConvolutionLayer.Builder([5, 5], [1, 1]).name("cnn1").nIn(c).nOut(20)
                       .activation(Activation.RELU).build())
                .layer(1, SubsamplingLayer.Builder(PoolingType.MAX, [2, 2], [2, 2]).name("maxpool1").build())
                .layer(2, ConvolutionLayer.Builder([5, 5], [1, 1]).name("cnn2").nOut(50).activation(Activation.RELU)
                       .build())
                .layer(3, SubsamplingLayer.Builder(PoolingType.MAX, [2, 2], [2, 2]).name("maxpool2").build())
                .layer(4, DenseLayer.Builder().name("ffn1").activation(Activation.RELU).nOut(500).build())
                .layer(5, OutputLayer.Builder(LossFunction.MCXENT).name("output").nOut(self.numLabels)
                       .activation(Activation.SOFTMAX).build())
                .setInputType(InputType.convolutionalFlat(h, w, c)).backprop(True).pretrain(False).build())

    def init(self, device=None):
        net = MultiLayerNetwork(self.conf())
        net.init(device=device)
        return net


# ------------------------------------------------------------------------------------------ SimpleCNN
class SimpleCNN(ZooModel):
    DEFAULT_SHAPE = [3, 48, 48]

    def conf(self):
        c, h, w = self.inputShape
        b = (self._builder().activation(Activation.IDENTITY).weightInit(WeightInit.RELU).updater(Adam(1e-3))
             .convolutionMode(ConvolutionMode.Same).list())
        layers = []
        for n, k in ((16, 7), (16, 7)):
            layers += [ConvolutionLayer.Builder([k, k]).nOut(n).build(), BatchNormalization(),
                       ActivationLayer(activation=Activation.RELU)]
        layers += [SubsamplingLayer.Builder(PoolingType.AVG, [2, 2], [2, 2]).build(), DropoutLayer.Builder(0.5).build()]
        for n, k in ((32, 5), (32, 5)):
            layers += [ConvolutionLayer.Builder([k, k]).nOut(n).build(), BatchNormalization(),
                       ActivationLayer(activation=Activation.RELU)]
        layers += [SubsamplingLayer.Builder(PoolingType.AVG, [2, 2], [2, 2]).build(), DropoutLayer.Builder(0.5).build()]
        for n, k in ((64, 3), (64, 3)):
            layers += [ConvolutionLayer.Builder([k, k]).nOut(n).build(), BatchNormalization(),
                       ActivationLayer(activation=Activation.RELU)]
        layers += [SubsamplingLayer.Builder(PoolingType.AVG, [2, 2], [2, 2]).build(), DropoutLayer.Builder(0.5).build()]
        layers += [ConvolutionLayer.Builder([3, 3]).nOut(self.numLabels).build(),
                   GlobalPoolingLayer.Builder(PoolingType.AVG).build(),
                   OutputLayer.Builder(LossFunction.NEGATIVELOGLIKELIHOOD).nOut(self.numLabels)
                   .activation(Activation.SOFTMAX).build()]
        for i, l in enumerate(layers):
            b.layer(i, l)
        return b.setInputType(InputType.convolutional(h, w, c)).build()

    def init(self, device=None):
        net = MultiLayerNetwork(self.conf())
        net.init(device=device)
        return net


# ---------------------------------------------------------------------------------- TextGenerationLSTM
class TextGenerationLSTM(ZooModel):
    DEFAULT_SHAPE = [1, 77]   # [mb-agnostic, totalUniqueCharacters]

    def __init__(self, numLabels=77, seed=12345, inputShape=None, hidden=256, tbptt=50, **kw):
        super().__init__(numLabels, seed, inputShape, **kw)
        self.hidden = hidden
        self.tbptt = tbptt

    def conf(self):
        nchar = self.inputShape[1]
        return (self._builder().optimizationAlgo(OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT)
                .l2(0.001).weightInit(WeightInit.XAVIER).updater(RmsProp(0.01)).list()
                .layer(0, GravesLSTM.Builder().nIn(nchar).nOut(self.hidden).activation(Activation.TANH).build())
                .layer(1, GravesLSTM.Builder().nOut(self.hidden).activation(Activation.TANH).build())
                .layer(2, RnnOutputLayer.Builder(LossFunction.MCXENT).activation(Activation.SOFTMAX)
                       .nOut(self.numLabels).build())
                .setInputType(InputType.recurrent(nchar))
                .backpropType(BackpropType.TruncatedBPTT).tBPTTForwardLength(self.tbptt)
                .tBPTTBackwardLength(self.tbptt).pretrain(False).backprop(True).build())

    def init(self, device=None):
        net = MultiLayerNetwork(self.conf())
        net.init(device=device)
        return net


# --------------------------------------------------------------------------------------------- AlexNet
class AlexNet(ZooModel):
    def conf(self):
        c, h, w = self.inputShape
        return (self._builder().weightInit(NormalDistribution(0.0, 0.01)).activation(Activation.RELU)
                .updater(Nesterovs(1e-2, 0.9)).biasUpdater(Nesterovs(2e-2, 0.9))
                .convolutionMode(ConvolutionMode.Same).l2(5e-4).miniBatch(False).list()
                .layer(0, ConvolutionLayer.Builder([11, 11], [4, 4], [2, 2]).name("cnn1").nIn(c).nOut(96).build())
                .layer(1, LocalResponseNormalization.Builder().build())
                .layer(2, SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).name("maxpool1").build())
                .layer(3, ConvolutionLayer.Builder([5, 5], [1, 1], [2, 2]).name("cnn2").nOut(256).biasInit(0.1)
                       .build())
                .layer(4, SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).name("maxpool2").build())
                .layer(5, LocalResponseNormalization.Builder().build())
                .layer(6, ConvolutionLayer.Builder([3, 3], [1, 1]).name("cnn3").nOut(384).build())
                .layer(7, ConvolutionLayer.Builder([3, 3], [1, 1]).name("cnn4").nOut(384).biasInit(0.1).build())
                .layer(8, ConvolutionLayer.Builder([3, 3], [1, 1]).name("cnn5").nOut(256).biasInit(0.1).build())
                .layer(9, SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).name("maxpool3").build())
                .layer(10, DenseLayer.Builder().name("ffn1").nOut(4096).weightInit(NormalDistribution(0, 0.005))
                       .biasInit(0.1).dropOut(0.5).build())
                .layer(11, DenseLayer.Builder().name("ffn2").nOut(4096).weightInit(NormalDistribution(0, 0.005))
                       .biasInit(0.1).dropOut(0.5).build())
                .layer(12, OutputLayer.Builder(LossFunction.NEGATIVELOGLIKELIHOOD).name("output")
                       .nOut(self.numLabels).activation(Activation.SOFTMAX).build())
                .setInputType(InputType.convolutional(h, w, c)).build())

    def init(self, device=None):
        net = MultiLayerNetwork(self.conf())
        net.init(device=device)
        return net


# ----------------------------------------------------------------------------------------- VGG16 / 19
class VGG16(ZooModel):
    BLOCKS = [(2, 64), (2, 128), (3, 256), (3, 512), (3, 512)]

    def conf(self):
        c, h, w = self.inputShape
        b = (self._builder().activation(Activation.RELU).updater(Nesterovs(1e-2, 0.9)).weightInit(WeightInit.RELU)
             .convolutionMode(ConvolutionMode.Same).list())
        i = 0
        nin = c
        for reps, n in self.BLOCKS:
            for _ in range(reps):
                b.layer(i, ConvolutionLayer.Builder([3, 3], [1, 1], [1, 1]).nIn(nin).nOut(n).build())
                nin = n
                i += 1
            b.layer(i, SubsamplingLayer.Builder(PoolingType.MAX, [2, 2], [2, 2]).build())
            i += 1
        b.layer(i, DenseLayer.Builder().nOut(4096).dropOut(0.5).build())
        b.layer(i + 1, DenseLayer.Builder().nOut(4096).dropOut(0.5).build())
        b.layer(i + 2, OutputLayer.Builder(LossFunction.NEGATIVELOGLIKELIHOOD).nOut(self.numLabels)
                .activation(Activation.SOFTMAX).build())
        return b.setInputType(InputType.convolutional(h, w, c)).build()

    def init(self, device=None):
        net = MultiLayerNetwork(self.conf())
        net.init(device=device)
        return net


class VGG19(VGG16):
    BLOCKS = [(2, 64), (2, 128), (4, 256), (4, 512), (4, 512)]


# --------------------------------------------------------------------------------------------- Darknet19
class Darknet19(ZooModel):
    """Darknet-19 (reference ZOO:model/Darknet19.java): conv-BN-leakyReLU stacks + global avg pool."""

    def _pretrained_key(self):
        # the 448x448 ImageNet weights are a separate file (ZOO:model/Darknet19.java:62-81)
        return "Darknet19@448" if list(self.inputShape[1:]) == [448, 448] else "Darknet19"

    def _cbl(self, g, name, k, n, inp):
        g.addLayer(f"conv{name}", ConvolutionLayer.Builder([k, k]).nOut(n).hasBias(False)
                   .convolutionMode(ConvolutionMode.Same).build(), inp)
        g.addLayer(f"bn{name}", BatchNormalization(), f"conv{name}")
        g.addLayer(f"act{name}", ActivationLayer(activation=Activation.LEAKYRELU), f"bn{name}")
        return f"act{name}"

    def graphBuilder(self):
        c, h, w = self.inputShape
        g = (self._builder().updater(Adam(1e-3)).weightInit(WeightInit.RELU).activation(Activation.IDENTITY)
             .convolutionMode(ConvolutionMode.Same).graphBuilder())
        g.addInputs("input").setInputTypes(InputType.convolutional(h, w, c))
        x = "input"
        spec = [[(3, 32)], "M", [(3, 64)], "M", [(3, 128), (1, 64), (3, 128)], "M", [(3, 256), (1, 128), (3, 256)],
                "M", [(3, 512), (1, 256), (3, 512), (1, 256), (3, 512)], "M",
                [(3, 1024), (1, 512), (3, 1024), (1, 512), (3, 1024)]]
        li = 1
        for s in spec:
            if s == "M":
                g.addLayer(f"maxpool{li}", SubsamplingLayer.Builder(PoolingType.MAX, [2, 2], [2, 2]).build(), x)
                x = f"maxpool{li}"
                continue
            for k, n in s:
                x = self._cbl(g, str(li), k, n, x)
                li += 1
        g.addLayer("convout", ConvolutionLayer.Builder([1, 1]).nOut(self.numLabels).build(), x)
        g.addLayer("gap", GlobalPoolingLayer.Builder(PoolingType.AVG).build(), "convout")
        g.addLayer("output", OutputLayer.Builder(LossFunction.NEGATIVELOGLIKELIHOOD).nOut(self.numLabels)
                   .activation(Activation.SOFTMAX).build(), "gap")
        return g.setOutputs("output")

    def conf(self):
        return self.graphBuilder().build()

    def init(self, device=None):
        net = ComputationGraph(self.conf())
        net.init(device=device)
        return net


# ---------------------------------------------------------------------------------------------- GoogLeNet
class GoogLeNet(ZooModel):
    """Inception v1 (reference ZOO:model/GoogLeNet.java) built from inception modules with MergeVertex."""

    def _inception(self, g, name, inp, c1, c3r, c3, c5r, c5, pp):
        def cr(n, k, src, suffix):
            g.addLayer(f"{name}-{suffix}", ConvolutionLayer.Builder([k, k]).nOut(n)
                       .convolutionMode(ConvolutionMode.Same).activation(Activation.RELU).build(), src)
            return f"{name}-{suffix}"
        a = cr(c1, 1, inp, "cnn1")
        b = cr(c3, 3, cr(c3r, 1, inp, "cnn2"), "cnn3")
        c = cr(c5, 5, cr(c5r, 1, inp, "cnn4"), "cnn5")
        g.addLayer(f"{name}-max1", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [1, 1])
                   .convolutionMode(ConvolutionMode.Same).build(), inp)
        d = cr(pp, 1, f"{name}-max1", "cnn6")
        g.addVertex(f"{name}-depthconcat1", MergeVertex(), a, b, c, d)
        return f"{name}-depthconcat1"

    def graphBuilder(self):
        ch, h, w = self.inputShape
        g = (self._builder().activation(Activation.RELU).weightInit(WeightInit.XAVIER).updater(Nesterovs(1e-2, 0.9))
             .l2(2e-4).convolutionMode(ConvolutionMode.Same).graphBuilder())
        g.addInputs("input").setInputTypes(InputType.convolutional(h, w, ch))
        g.addLayer("cnn1", ConvolutionLayer.Builder([7, 7], [2, 2]).nOut(64).build(), "input")
        g.addLayer("max1", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2])
                   .convolutionMode(ConvolutionMode.Same).build(), "cnn1")
        g.addLayer("lrn1", LocalResponseNormalization.Builder().build(), "max1")
        g.addLayer("cnn2", ConvolutionLayer.Builder([1, 1]).nOut(64).build(), "lrn1")
        g.addLayer("cnn3", ConvolutionLayer.Builder([3, 3]).nOut(192).build(), "cnn2")
        g.addLayer("lrn2", LocalResponseNormalization.Builder().build(), "cnn3")
        g.addLayer("max2", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2])
                   .convolutionMode(ConvolutionMode.Same).build(), "lrn2")
        x = self._inception(g, "3a", "max2", 64, 96, 128, 16, 32, 32)
        x = self._inception(g, "3b", x, 128, 128, 192, 32, 96, 64)
        g.addLayer("max3", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2])
                   .convolutionMode(ConvolutionMode.Same).build(), x)
        x = "max3"
        for nm, cfg in (("4a", (192, 96, 208, 16, 48, 64)), ("4b", (160, 112, 224, 24, 64, 64)),
                        ("4c", (128, 128, 256, 24, 64, 64)), ("4d", (112, 144, 288, 32, 64, 64)),
                        ("4e", (256, 160, 320, 32, 128, 128))):
            x = self._inception(g, nm, x, *cfg)
        g.addLayer("max4", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2])
                   .convolutionMode(ConvolutionMode.Same).build(), x)
        x = self._inception(g, "5a", "max4", 256, 160, 320, 32, 128, 128)
        x = self._inception(g, "5b", x, 384, 192, 384, 48, 128, 128)
        g.addLayer("avg3", GlobalPoolingLayer.Builder(PoolingType.AVG).build(), x)
        g.addLayer("fc1", DenseLayer.Builder().nOut(1024).dropOut(0.4).build(), "avg3")
        g.addLayer("output", OutputLayer.Builder(LossFunction.NEGATIVELOGLIKELIHOOD).nOut(self.numLabels)
                   .activation(Activation.SOFTMAX).build(), "fc1")
        return g.setOutputs("output")

    def conf(self):
        return self.graphBuilder().build()

    def init(self, device=None):
        net = ComputationGraph(self.conf())
        net.init(device=device)
        return net




# ---------------------------------------------------------------------------------------- YOLO family
def _darknet_cbl(g, n, k, nout, inp, pool=0, pool_stride=None):
    """Darknet conv block (reference ZOO:model/helper/DarknetHelper.java): conv (Same, no bias) -> BN ->
    leaky ReLU(0.1) [-> max pool (Same)]. Returns the block's output vertex name."""
    from ..nn.conf.activations import ActivationLReLU
    g.addLayer(f"convolution2d_{n}", ConvolutionLayer.Builder([k, k]).nOut(nout).hasBias(False)
               .convolutionMode(ConvolutionMode.Same).weightInit(WeightInit.XAVIER)
               .activation(Activation.IDENTITY).build(), inp)
    g.addLayer(f"batchnormalization_{n}", BatchNormalization(), f"convolution2d_{n}")
    g.addLayer(f"activation_{n}", ActivationLayer(activation=ActivationLReLU(alpha=0.1)), f"batchnormalization_{n}")
    out = f"activation_{n}"
    if pool:
        s = pool_stride if pool_stride is not None else pool
        g.addLayer(f"maxpooling2d_{n}", SubsamplingLayer.Builder(PoolingType.MAX, [pool, pool], [s, s])
                   .convolutionMode(ConvolutionMode.Same).build(), out)
        out = f"maxpooling2d_{n}"
    return out


class _YoloBase(ZooModel):
    DEFAULT_SHAPE = [3, 416, 416]
    PRIORS = None

    def __init__(self, numLabels=20, seed=123, inputShape=None, **kw):
        super().__init__(numLabels, seed, inputShape, **kw)

    def _base(self):
        import torch
        c, h, w = self.inputShape
        g = (self._builder().optimizationAlgo(OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT)
             .gradientNormalization("RenormalizeL2PerLayer").gradientNormalizationThreshold(1.0)
             .updater(Adam(1e-3)).l2(1e-5).activation(Activation.IDENTITY).graphBuilder())
        g.addInputs("input").setInputTypes(InputType.convolutional(h, w, c))
        return g, torch.tensor(self.PRIORS, dtype=torch.float32)

    def _head(self, g, n, inp, priors):
        from ..nn.conf.layers import Yolo2OutputLayer
        nb = priors.shape[0]
        g.addLayer(f"convolution2d_{n}", ConvolutionLayer.Builder([1, 1]).nOut(nb * (5 + self.numLabels))
                   .convolutionMode(ConvolutionMode.Same).weightInit(WeightInit.RELU)
                   .activation(Activation.IDENTITY).build(), inp)
        g.addLayer("outputs", Yolo2OutputLayer(boundingBoxes=priors), f"convolution2d_{n}")
        return g.setOutputs("outputs")

    def gridWidth(self):
        return self.inputShape[2] // 32

    def gridHeight(self):
        return self.inputShape[1] // 32

    def conf(self):
        return self.graphBuilder().build()

    def init(self, device=None):
        net = ComputationGraph(self.conf())
        net.init(device=device)
        return net


class TinyYOLO(_YoloBase):
    """Tiny YOLOv2 (reference ZOO:model/TinyYOLO.java): 9 Darknet conv blocks with 6 max pools (the last with
    stride 1), a 1x1 conv to nBoxes*(5+classes) channels and a Yolo2OutputLayer with the VOC anchor priors."""
    PRIORS = [[1.08, 1.19], [3.42, 4.41], [6.63, 11.38], [9.42, 5.11], [16.62, 10.52]]

    def graphBuilder(self):
        g, priors = self._base()
        x = "input"
        spec = [(16, 2, 2), (32, 2, 2), (64, 2, 2), (128, 2, 2), (256, 2, 2), (512, 2, 1), (1024, 0, 0),
                (1024, 0, 0)]
        for i, (nout, pool, ps) in enumerate(spec, start=1):
            x = _darknet_cbl(g, i, 3, nout, x, pool, ps)
        return self._head(g, 9, x, priors)


class YOLO2(_YoloBase):
    """YOLOv2 (reference ZOO:model/YOLO2.java): Darknet-19 trunk, the 26x26 passthrough route reorganised by
    SpaceToDepth(2) and concatenated with the 13x13 features, then the detection head."""
    PRIORS = [[0.57273, 0.677385], [1.87446, 2.06253], [3.33843, 5.47434], [7.88282, 3.52778],
              [9.77052, 9.16828]]

    def graphBuilder(self):
        from ..nn.conf.layers import SpaceToDepthLayer
        g, priors = self._base()
        spec = [(3, 32, 2), (3, 64, 2), (3, 128, 0), (1, 64, 0), (3, 128, 2), (3, 256, 0), (1, 128, 0), (3, 256, 2),
                (3, 512, 0), (1, 256, 0), (3, 512, 0), (1, 256, 0), (3, 512, 2), (3, 1024, 0), (1, 512, 0),
                (3, 1024, 0), (1, 512, 0), (3, 1024, 0), (3, 1024, 0), (3, 1024, 0)]
        x = "input"
        for i, (k, nout, pool) in enumerate(spec, start=1):
            x = _darknet_cbl(g, i, k, nout, x, pool)
        route = _darknet_cbl(g, 21, 1, 64, "activation_13")           # passthrough from the 26x26 stage
        g.addLayer("rearrange_21", SpaceToDepthLayer(blockSize=2), route)
        g.addVertex("concatenate_21", MergeVertex(), "rearrange_21", x)
        x = _darknet_cbl(g, 22, 3, 1024, "concatenate_21")
        return self._head(g, 23, x, priors)


# --------------------------------------------------------------------------------------- face models
class FaceNetNN4Small2(ZooModel):
    """FaceNet NN4.small2 (reference ZOO:model/FaceNetNN4Small2.java + helper/FaceNetHelper.java): conv stem with
    LRN, inception modules 3a/3b/3c/4a/4e/5a/5b (1x1-reduce -> NxN branches, pooled 1x1 branch, MergeVertex),
    3x3 average pool, 128-d bottleneck, L2-normalised embeddings, center-loss softmax output."""
    DEFAULT_SHAPE = [3, 96, 96]

    def __init__(self, numLabels=5749, seed=123, inputShape=None, embeddingSize=128, **kw):
        super().__init__(numLabels, seed, inputShape, **kw)
        self.embeddingSize = embeddingSize

    @staticmethod
    def _cbr(g, name, inp, k, nout, stride=1, bias_init=None):
        b = ConvolutionLayer.Builder([k, k], [stride, stride]).nOut(nout)
        if bias_init is not None:
            b = b.biasInit(bias_init)
        g.addLayer(name, b.build(), inp)
        g.addLayer(name + "-norm", BatchNormalization.Builder().build(), name)
        g.addLayer(name + "-act", ActivationLayer(activation=Activation.RELU), name + "-norm")
        return name + "-act"

    def _inception(self, g, mod, inp, branches, pool):
        """branches: list of (kernel, stride, reduce, out); pool: (ptype, size, stride, pool_proj or None);
        plus optional plain 1x1 branch via kernel 1 entries."""
        outs = []
        for i, (k, s, red, out) in enumerate(branches):
            if k == 1:
                outs.append(self._cbr(g, f"{mod}-1x1-{i}", inp, 1, out, s, 0.2))
                continue
            r = self._cbr(g, f"{mod}-{k}x{k}-reduce-{i}", inp, 1, red, 1, 0.2)
            outs.append(self._cbr(g, f"{mod}-{k}x{k}-{i}", r, k, out, s, 0.2))
        ptype, size, stride, proj = pool
        pb = SubsamplingLayer.Builder(ptype, [size, size], [stride, stride])
        if ptype == PoolingType.PNORM:
            pb = pb.pnorm(2)
        g.addLayer(f"{mod}-pool", pb.build(), inp)
        outs.append(self._cbr(g, f"{mod}-pool-proj", f"{mod}-pool", 1, proj, 1, 0.2) if proj else f"{mod}-pool")
        g.addVertex(f"inception-{mod}", MergeVertex(), *outs)
        return f"inception-{mod}"

    def graphBuilder(self):
        from ..nn.conf.graph import L2NormalizeVertex
        from ..nn.conf.layers import CenterLossOutputLayer
        c, h, w = self.inputShape
        g = (self._builder().activation(Activation.IDENTITY)
             .optimizationAlgo(OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT)
             .updater(Adam(0.1, 0.9, 0.999, 0.01)).weightInit(WeightInit.RELU).l2(5e-5).miniBatch(True)
             .convolutionMode(ConvolutionMode.Same).graphBuilder())
        g.addInputs("input1").setInputTypes(InputType.convolutional(h, w, c))
        x = self._cbr(g, "stem-cnn1", "input1", 7, 64, 2)
        g.addLayer("stem-pool1", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).build(), x)
        g.addLayer("stem-lrn1", LocalResponseNormalization.Builder(1, 5, 1e-4, 0.75).build(), "stem-pool1")
        x = self._cbr(g, "inception-2-cnn1", "stem-lrn1", 1, 64)
        x = self._cbr(g, "inception-2-cnn2", x, 3, 192)
        g.addLayer("inception-2-lrn1", LocalResponseNormalization.Builder(1, 5, 1e-4, 0.75).build(), x)
        g.addLayer("inception-2-pool1", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).build(),
                   "inception-2-lrn1")
        M, P = PoolingType.MAX, PoolingType.PNORM
        x = self._inception(g, "3a", "inception-2-pool1", [(3, 1, 96, 128), (5, 1, 16, 32), (1, 1, 0, 64)],
                            (M, 3, 1, 32))
        x = self._inception(g, "3b", x, [(3, 1, 96, 128), (5, 1, 32, 64), (1, 1, 0, 64)], (P, 3, 1, 64))
        x = self._inception(g, "3c", x, [(3, 2, 128, 256), (5, 2, 32, 64)], (M, 3, 2, None))
        x = self._inception(g, "4a", x, [(3, 1, 96, 192), (5, 1, 32, 64), (1, 1, 0, 256)], (P, 3, 1, 128))
        x = self._inception(g, "4e", x, [(3, 2, 160, 256), (5, 2, 64, 128)], (M, 3, 2, None))
        x = self._inception(g, "5a", x, [(3, 1, 96, 384), (1, 1, 0, 256)], (P, 3, 1, 96))
        x = self._inception(g, "5b", x, [(3, 1, 96, 384), (1, 1, 0, 256)], (M, 3, 1, 96))
        g.addLayer("avgpool", SubsamplingLayer.Builder(PoolingType.AVG, [3, 3], [3, 3]).build(), x)
        g.addLayer("bottleneck", DenseLayer.Builder().nOut(self.embeddingSize).activation(Activation.IDENTITY)
                   .build(), "avgpool")
        g.addVertex("embeddings", L2NormalizeVertex(dimension=[1], eps=1e-6), "bottleneck")
        g.addLayer("lossLayer", CenterLossOutputLayer.Builder().lossFunction(LossFunction.SQUARED_LOSS)
                   .activation(Activation.SOFTMAX).nOut(self.numLabels).alpha(0.9).lambda_(1e-4)
                   .gradientNormalization("RenormalizeL2PerLayer").build(), "embeddings")
        return g.setOutputs("lossLayer")

    def conf(self):
        return self.graphBuilder().build()

    def init(self, device=None):
        net = ComputationGraph(self.conf())
        net.init(device=device)
        return net


class InceptionResNetV1(ZooModel):
    """Inception-ResNet-v1 (reference ZOO:model/InceptionResNetV1.java + helper/InceptionResNetHelper.java):
    stem, 5x block35 (scale 0.17), reduction-A, 10x block17 (scale 0.10), reduction-B, 5x block8 (scale 0.20),
    average pool, 128-d bottleneck, L2-normalised embeddings and a center-loss softmax output. Residual branches are
    merged, projected by a linear 1x1 conv + BN, scaled (ScaleVertex) and added to the block input, then ReLU."""
    DEFAULT_SHAPE = [3, 160, 160]

    def __init__(self, numLabels=5749, seed=123, inputShape=None, embeddingSize=128, **kw):
        super().__init__(numLabels, seed, inputShape, **kw)
        self.embeddingSize = embeddingSize

    @staticmethod
    def _cb(g, name, inp, k, nout, stride=1, same=True, act=True):
        kk = k if isinstance(k, (list, tuple)) else [k, k]
        b = ConvolutionLayer.Builder(list(kk), [stride, stride]).nOut(nout)
        if same:
            b = b.convolutionMode(ConvolutionMode.Same)
        g.addLayer(name, b.activation(Activation.IDENTITY).build(), inp)
        g.addLayer(name + "-bn", BatchNormalization.Builder().decay(0.995).eps(1e-3).build(), name)
        if act:
            g.addLayer(name + "-relu", ActivationLayer(activation=Activation.RELU), name + "-bn")
            return name + "-relu"
        return name + "-bn"

    def _res_block(self, g, name, inp, branches, nout, scale):
        outs = []
        for bi, chain in enumerate(branches):
            x = inp
            for ci, (k, n) in enumerate(chain):
                x = self._cb(g, f"{name}-b{bi}-c{ci}", x, k, n)
            outs.append(x)
        g.addVertex(f"{name}-merge", MergeVertex(), *outs)
        g.addLayer(f"{name}-up", ConvolutionLayer.Builder([1, 1]).nOut(nout).activation(Activation.IDENTITY)
                   .convolutionMode(ConvolutionMode.Same).build(), f"{name}-merge")
        g.addLayer(f"{name}-up-bn", BatchNormalization.Builder().decay(0.995).eps(1e-3).build(), f"{name}-up")
        g.addVertex(f"{name}-scale", ScaleVertex(scale), f"{name}-up-bn")
        g.addVertex(f"{name}-add", ElementWiseVertex(ElementWiseVertex.Op.Add), inp, f"{name}-scale")
        g.addLayer(name, ActivationLayer(activation=Activation.RELU), f"{name}-add")
        return name

    def graphBuilder(self):
        from ..nn.conf.graph import L2NormalizeVertex
        from ..nn.conf.layers import CenterLossOutputLayer
        c, h, w = self.inputShape
        g = (self._builder().activation(Activation.RELU)
             .optimizationAlgo(OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT)
             .updater(RmsProp(0.1, 0.96, 0.001)).weightInit(NormalDistribution(0.0, 0.5)).l2(5e-5)
             .miniBatch(True).convolutionMode(ConvolutionMode.Truncate).graphBuilder())
        g.addInputs("input1").setInputTypes(InputType.convolutional(h, w, c))
        x = self._cb(g, "stem-cnn1", "input1", 3, 32, 2, same=False)
        x = self._cb(g, "stem-cnn2", x, 3, 32, 1, same=False)
        x = self._cb(g, "stem-cnn3", x, 3, 64, 1)
        g.addLayer("stem-pool4", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).build(), x)
        x = self._cb(g, "stem-cnn5", "stem-pool4", 1, 80)
        x = self._cb(g, "stem-cnn6", x, 3, 192, 1, same=False)
        x = self._cb(g, "stem-cnn7", x, 3, 256, 2, same=False)
        for i in range(5):                                                    # block35
            x = self._res_block(g, f"resnetA-{i}", x, [[(1, 32)], [(1, 32), (3, 32)],
                                                        [(1, 32), (3, 32), (3, 32)]], 256, 0.17)
        a = self._cb(g, "reduceA-b0", x, 3, 384, 2, same=False)             # reduction-A
        b = self._cb(g, "reduceA-b1-c0", x, 1, 192)
        b = self._cb(g, "reduceA-b1-c1", b, 3, 192)
        b = self._cb(g, "reduceA-b1-c2", b, 3, 256, 2, same=False)
        g.addLayer("reduceA-pool", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).build(), x)
        g.addVertex("reduceA", MergeVertex(), a, b, "reduceA-pool")
        x = "reduceA"
        for i in range(10):                                                   # block17
            x = self._res_block(g, f"resnetB-{i}", x, [[(1, 128)], [(1, 128), ([1, 7], 128), ([7, 1], 128)]],
                                896, 0.10)
        b0 = self._cb(g, "reduceB-b0-c0", x, 1, 256)                          # reduction-B
        b0 = self._cb(g, "reduceB-b0-c1", b0, 3, 384, 2, same=False)
        b1 = self._cb(g, "reduceB-b1-c0", x, 1, 256)
        b1 = self._cb(g, "reduceB-b1-c1", b1, 3, 256, 2, same=False)
        b2 = self._cb(g, "reduceB-b2-c0", x, 1, 256)
        b2 = self._cb(g, "reduceB-b2-c1", b2, 3, 256)
        b2 = self._cb(g, "reduceB-b2-c2", b2, 3, 256, 2, same=False)
        g.addLayer("reduceB-pool", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2]).build(), x)
        g.addVertex("reduceB", MergeVertex(), b0, b1, b2, "reduceB-pool")
        x = "reduceB"
        for i in range(5):                                                    # block8
            x = self._res_block(g, f"resnetC-{i}", x, [[(1, 192)], [(1, 192), ([1, 3], 192), ([3, 1], 192)]],
                                1792, 0.20)
        g.addLayer("avgpool", GlobalPoolingLayer.Builder(PoolingType.AVG).build(), x)
        g.addLayer("bottleneck", DenseLayer.Builder().nOut(self.embeddingSize).activation(Activation.IDENTITY)
                   .build(), "avgpool")
        g.addVertex("embeddings", L2NormalizeVertex(dimension=[1], eps=1e-10), "bottleneck")
        g.addLayer("outputLayer", CenterLossOutputLayer.Builder().lossFunction(LossFunction.NEGATIVELOGLIKELIHOOD)
                   .activation(Activation.SOFTMAX).nOut(self.numLabels).alpha(0.9).lambda_(1e-4).build(),
                   "embeddings")
        return g.setOutputs("outputLayer")

    def conf(self):
        return self.graphBuilder().build()

    def init(self, device=None):
        net = ComputationGraph(self.conf())
        net.init(device=device)
        return net


class ModelSelector:
    """Instantiate zoo models by ZooType (ZOO:ModelSelector.java:16-140): a single type, a group (CNN: SimpleCNN,
    AlexNet, LeNet, GoogLeNet, ResNet50, VGG16, VGG19, Darknet19, TinyYOLO, YOLO2; RNN: TextGenerationLSTM; ALL: both)
    or several types, as {ZooType: ZooModel}. Defaults as the reference: numLabels 1 for select(type), 0 for
    select(*types), seed 123. Unlike the reference's GOOGLENET case (which files GoogLeNet under LENET) every model is
    keyed by its own type."""
    _CNN = ("SIMPLECNN", "ALEXNET", "LENET", "GOOGLENET", "RESNET50", "VGG16", "VGG19", "DARKNET19", "TINYYOLO",
            "YOLO2")
    _SINGLE = {"TEXTGENLSTM": "TextGenerationLSTM", "SIMPLECNN": "SimpleCNN", "ALEXNET": "AlexNet", "LENET": "LeNet",
               "INCEPTIONRESNETV1": "InceptionResNetV1", "FACENETNN4SMALL2": "FaceNetNN4Small2",
               "GOOGLENET": "GoogLeNet", "RESNET50": "ResNet50", "VGG16": "VGG16", "VGG19": "VGG19",
               "DARKNET19": "Darknet19", "TINYYOLO": "TinyYOLO", "YOLO2": "YOLO2"}

    @classmethod
    def select(cls, *zooTypes, numLabels=None, seed=123, workspaceMode=WorkspaceMode.ENABLED):
        if not zooTypes:
            raise ValueError("no ZooType given")
        if numLabels is None:
            numLabels = 1 if len(zooTypes) == 1 else 0
        out = {}
        for t in zooTypes:
            cls._add(out, ZooType[t] if isinstance(t, str) else t, numLabels, seed, workspaceMode)
        if not out:
            raise ValueError("Zero models have been selected for benchmarking.")
        return out

    @classmethod
    def _add(cls, out, t, numLabels, seed, ws):
        if t == ZooType.ALL:
            cls._add(out, ZooType.CNN, numLabels, seed, ws)
            cls._add(out, ZooType.RNN, numLabels, seed, ws)
        elif t == ZooType.CNN:
            for n in cls._CNN:
                cls._add(out, ZooType[n], numLabels, seed, ws)
        elif t == ZooType.RNN:
            cls._add(out, ZooType.TEXTGENLSTM, numLabels, seed, ws)
        elif t.name in cls._SINGLE:
            out[t] = ZOO[cls._SINGLE[t.name]](numLabels=numLabels, seed=seed, workspaceMode=ws)


ZOO = {"ResNet50": ResNet50, "LeNet": LeNet, "SimpleCNN": SimpleCNN, "TextGenerationLSTM": TextGenerationLSTM,
       "AlexNet": AlexNet, "VGG16": VGG16, "VGG19": VGG19, "Darknet19": Darknet19, "GoogLeNet": GoogLeNet,
       "TinyYOLO": TinyYOLO, "YOLO2": YOLO2, "FaceNetNN4Small2": FaceNetNN4Small2,
       "InceptionResNetV1": InceptionResNetV1}


# ------------------------------------------------------------------------------------------------ BertBase
class BertBase(ZooModel):
    """BERT encoder + [CLS] pooler + softmax classifier (BASELINE.json's BERT-base config; new relative to the
    reference zoo). Defaults are BERT-base: 12 layers, hidden 768, 12 heads, FFN 3072, vocab 30522, 512 positions,
    N(0, 0.02) init, Adam(2e-5). ``inputShape = [seqLen]``; input = token ids [mb, seqLen] (featuresMask [mb, T]
    marks real tokens)."""
    DEFAULT_SHAPE = [128]

    def __init__(self, numLabels=2, seed=123, inputShape=None, vocabSize=30522, hidden=768, layers=12, heads=12,
                 ffn=3072, maxPositions=512, learningRate=2e-5, **kw):
        super().__init__(numLabels, seed, inputShape, **kw)
        self.vocabSize, self.hidden, self.layers, self.heads = vocabSize, hidden, layers, heads
        self.ffn, self.maxPositions, self.learningRate = ffn, maxPositions, learningRate

    def graphBuilder(self):
        from ..nn.conf import BertEmbeddingLayer, BertPoolerLayer, TransformerEncoderLayer
        T = self.inputShape[0]
        g = (self._builder().updater(Adam(self.learningRate)).weightInit(NormalDistribution(0.0, 0.02))
             .graphBuilder())
        g.addInputs("tokens")
        g.addLayer("embeddings", BertEmbeddingLayer.Builder().nIn(self.vocabSize).nOut(self.hidden)
                   .maxPositions(self.maxPositions).inputLength(T).build(), "tokens")
        prev = "embeddings"
        for i in range(self.layers):
            g.addLayer(f"encoder_{i}", TransformerEncoderLayer.Builder().nIn(self.hidden).nOut(self.hidden)
                       .nHeads(self.heads).ffnSize(self.ffn).build(), prev)
            prev = f"encoder_{i}"
        g.addLayer("pooler", BertPoolerLayer.Builder().nIn(self.hidden).nOut(self.hidden).build(), prev)
        g.addLayer("classifier", OutputLayer.Builder(LossFunction.MCXENT).activation(Activation.SOFTMAX)
                   .nIn(self.hidden).nOut(self.numLabels).build(), "pooler")
        g.setOutputs("classifier")
        return g

    def conf(self):
        return self.graphBuilder().build()

    def init(self, device=None):
        net = ComputationGraph(self.conf())
        net.init(device=device)
        return net
