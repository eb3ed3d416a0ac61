"""Helper-fallback accounting on the flagship configurations (reference ConvolutionLayer.helperCountFail,
NN:nn/layers/convolution/ConvolutionLayer.java:58,173-200): one training step of each must run every GPU op on an
in-tree HIP kernel — ops/fallback.py counts any call that took a library / torch path instead."""
import pytest
import torch

from deeplearning4j_amd.ops import fallback

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _assert_clean(net, what):
    torch.cuda.synchronize()
    assert net.helperCountFail() == 0, f"{what}: fallbacks {fallback.summary()}"


def test_resnet50_bf16_step_has_no_fallbacks():
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    net = ResNet50(numLabels=10, dataType=DataType.BFLOAT16).init(device=DEV)
    x = torch.rand(4, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last).bfloat16()
    y = torch.zeros(4, 10, device=DEV)
    y[:, 3] = 1
    fallback.reset()
    net.fit([x], [y])
    _assert_clean(net, "ResNet-50 bf16")


def test_bert_bf16_step_has_no_fallbacks():
    from deeplearning4j_amd.models import BertBase
    from deeplearning4j_amd.nn.conf import DataType
    net = BertBase(numLabels=2, inputShape=[64], layers=2, dataType=DataType.BFLOAT16).init(device=DEV)
    x = torch.randint(0, 30522, (4, 64), device=DEV)
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (4,)), 2).float().to(DEV)
    fallback.reset()
    net.fit([x], [y])
    _assert_clean(net, "BERT bf16")


def test_textgen_lstm_bf16_step_has_no_fallbacks():
    from deeplearning4j_amd.models import TextGenerationLSTM
    from deeplearning4j_amd.nn.conf import DataType
    net = TextGenerationLSTM(numLabels=77, inputShape=[1, 77], dataType=DataType.BFLOAT16).init(device=DEV)
    idx = torch.randint(0, 77, (8, 100))
    x = torch.nn.functional.one_hot(idx, 77).permute(0, 2, 1).float().to(DEV)
    y = torch.nn.functional.one_hot(torch.roll(idx, -1, 1), 77).permute(0, 2, 1).float().to(DEV)
    fallback.reset()
    net.fit(x, y)
    _assert_clean(net, "TextGenerationLSTM bf16")


def test_lenet_fp32_gpu_no_fallbacks_and_matches_cpu():
    """fp32 on the GPU never reaches the library conv: im2col + the exact-fp32 MFMA GEMM (ops/conv.py), fp32 pooling /
    dense / softmax-xent kernels; a few SGD steps match the CPU run of the same network."""
    from deeplearning4j_amd.models import LeNet
    from deeplearning4j_amd.nn.conf import DataType
    g = torch.Generator().manual_seed(0)
    x = torch.rand(16, 1, 28, 28, generator=g)
    y = torch.nn.functional.one_hot(torch.randint(0, 10, (16,), generator=g), 10).float()
    nets = {}
    for dev in ("cpu", "cuda"):
        net = LeNet(numLabels=10, inputShape=[1, 28, 28], dataType=DataType.FLOAT).init(device=dev)
        fallback.reset()
        for _ in range(3):
            net.fit(x.to(dev), y.to(dev))
        if dev == "cuda":
            _assert_clean(net, "LeNet fp32")
        nets[dev] = net
    pc, pg = nets["cpu"].params().cpu(), nets["cuda"].params().cpu()
    assert torch.allclose(pc, pg, rtol=1e-3, atol=1e-4), (pc - pg).abs().max()


def test_resnet50_fp16_step_has_no_fallbacks():
    """fp16 conv / BN / pool on the round-3 engines (v3 tile engine, halo weight gradient, fp16 BN / pool kernels;
    the 3-channel stem is zero-padded to 64 channels): no library path, finite loss."""
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    net = ResNet50(numLabels=10, dataType=DataType.HALF).init(device=DEV)
    x = torch.rand(4, 3, 224, 224, device=DEV).contiguous(memory_format=torch.channels_last).half()
    y = torch.zeros(4, 10, device=DEV)
    y[:, 3] = 1
    fallback.reset()
    p0 = net.params().clone()
    net.fit([x], [y])
    _assert_clean(net, "ResNet-50 fp16")
    assert torch.isfinite(torch.tensor(net.score()))
    assert not torch.equal(p0, net.params())


def test_textgen_lstm_fp16_step_has_no_fallbacks():
    from deeplearning4j_amd.models import TextGenerationLSTM
    from deeplearning4j_amd.nn.conf import DataType
    net = TextGenerationLSTM(numLabels=77, inputShape=[1, 77], dataType=DataType.HALF).init(device=DEV)
    idx = torch.randint(0, 77, (8, 100))
    x = torch.nn.functional.one_hot(idx, 77).permute(0, 2, 1).float().to(DEV)
    y = torch.nn.functional.one_hot(torch.roll(idx, -1, 1), 77).permute(0, 2, 1).float().to(DEV)
    fallback.reset()
    net.fit(x, y)
    _assert_clean(net, "TextGenerationLSTM fp16")
    assert torch.isfinite(torch.tensor(net.score()))


def test_small_cnn_fp16_matches_fp32_cpu():
    """fp16 GPU forward / gradients of a conv -> BN -> ReLU -> max-pool -> 1x1 conv -> BN -> global pool net against
    the same network in fp32 on the CPU (parameters copied)."""
    from deeplearning4j_amd import (Activation, LossFunction, MultiLayerNetwork, NeuralNetConfiguration, OutputLayer,
                                    Sgd)
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.nn.conf.inputs import InputType
    from deeplearning4j_amd.nn.conf.layers import (BatchNormalization, ConvolutionLayer, GlobalPoolingLayer,
                                                   SubsamplingLayer)

    def build(dt, dev):
        conf = (NeuralNetConfiguration.Builder().seed(11).dataType(dt).updater(Sgd(0.0)).list()
                .layer(0, ConvolutionLayer.Builder([3, 3]).nOut(64).padding(1, 1).activation(Activation.IDENTITY).build())
                .layer(1, BatchNormalization.Builder().activation(Activation.RELU).build())
                .layer(2, SubsamplingLayer.Builder([2, 2], [2, 2]).build())
                .layer(3, ConvolutionLayer.Builder([1, 1]).nOut(64).activation(Activation.IDENTITY).build())
                .layer(4, BatchNormalization.Builder().activation(Activation.RELU).build())
                .layer(5, GlobalPoolingLayer.Builder("AVG").build())
                .layer(6, OutputLayer.Builder(LossFunction.MCXENT).nOut(5).activation(Activation.SOFTMAX).build())
                .setInputType(InputType.convolutional(16, 16, 64)).build())
        n = MultiLayerNetwork(conf)
        n.init(device=dev)
        return n
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 64, 16, 16, generator=g)
    y = torch.nn.functional.one_hot(torch.randint(0, 5, (8,), generator=g), 5).float()
    ref = build(DataType.FLOAT, "cpu")
    net = build(DataType.HALF, DEV)
    net.setParams(ref.params().to(DEV))
    fallback.reset()
    oh = net.output(x.to(DEV).half()).float().cpu()
    of = ref.output(x)
    assert (oh - of).abs().max() <= 2e-2, (oh - of).abs().max()
    net.computeGradientAndScore(x.to(DEV).half(), y.to(DEV))
    ref.computeGradientAndScore(x, y)
    gh, gf = net.gradient().gradient().float().cpu(), ref.gradient().gradient()
    rel = (gh - gf).norm() / gf.norm()
    assert rel <= 3e-2, rel
    _assert_clean(net, "small CNN fp16")
