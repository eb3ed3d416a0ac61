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
                       PoolingType, RmsProp, RnnOutputLayer, SubsamplingLayer, WeightInit, ZeroPaddingLayer, Adam)
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

    def pretrainedAvailable(self, t=None):
        return False

    def initPretrained(self, path=None):
        if path is None:
            raise RuntimeError("Pretrained weights cannot be downloaded in this environment; pass a local "
                               "ModelSerializer zip path")
        from ..utils.model_serializer import ModelSerializer
        return ModelSerializer.restoreModel(path)

    def _builder(self):
        return NeuralNetConfiguration.Builder().seed(self.seed).dataType(self.dataType) \
            .trainingWorkspaceMode(self.workspaceMode).inferenceWorkspaceMode(self.workspaceMode)


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

    def __init__(self, numLabels=1000, seed=123, inputShape=None, variant="dl4j", updater=None, **kw):
        super().__init__(numLabels, seed, inputShape, **kw)
        self.variant = variant
        self.updater = updater

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
             .updater(upd).weightInit(NormalDistribution(0.0, 0.5)).l1(1e-7).l2(5e-5).miniBatch(True)
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
                       ActivationLayer(Activation.RELU)]
        layers += [SubsamplingLayer.Builder(PoolingType.AVG, [2, 2], [2, 2]).build(), DropoutLayer.Builder(0.5).build()]
        for n, k in ((32, 5), (32, 5)):
            layers += [ConvolutionLayer.Builder([k, k]).nOut(n).build(), BatchNormalization(),
                       ActivationLayer(Activation.RELU)]
        layers += [SubsamplingLayer.Builder(PoolingType.AVG, [2, 2], [2, 2]).build(), DropoutLayer.Builder(0.5).build()]
        for n, k in ((64, 3), (64, 3)):
            layers += [ConvolutionLayer.Builder([k, k]).nOut(n).build(), BatchNormalization(),
                       ActivationLayer(Activation.RELU)]
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

    def _cbl(self, g, name, k, n, inp):
        g.addLayer(f"conv{name}", ConvolutionLayer.Builder([k, k]).nOut(n).hasBias(False)
                   .convolutionMode(ConvolutionMode.Same).build(), inp)
        g.addLayer(f"bn{name}", BatchNormalization(), f"conv{name}")
        g.addLayer(f"act{name}", ActivationLayer(Activation.LEAKYRELU), f"bn{name}")
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


ZOO = {"ResNet50": ResNet50, "LeNet": LeNet, "SimpleCNN": SimpleCNN, "TextGenerationLSTM": TextGenerationLSTM,
       "AlexNet": AlexNet, "VGG16": VGG16, "VGG19": VGG19, "Darknet19": Darknet19, "GoogLeNet": GoogLeNet}
