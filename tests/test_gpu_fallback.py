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
