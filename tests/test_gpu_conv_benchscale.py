"""Bench-scale conv parity: every distinct conv shape of the headline ResNet-50 (DL4J zoo graph)
at batch 256 - spatial 112/56/28/14/7, where split-K weight-gradient reductions, 32-bit index decomposition and
grid caps actually apply - forward, backward-data and weight gradient against a plain fp32 torch reference (library
convolution with cuDNN/MIOpen disabled, i.e. torch's own direct implementation) on the same bf16-rounded inputs."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

N = 256


def _resnet_conv_shapes():
    """(C, H, W, K, R, S, stride, pad4) of every conv in the zoo ResNet-50, from a batch-1 CPU forward."""
    from deeplearning4j_amd import ops
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.layers import convolution as convmod
    seen = []
    orig = ops.conv2d_forward

    def spy(x, w, b, stride, pad4, dilation=(1, 1), groups=1, want_stats=False):
        key = (x.shape[1], x.shape[2], x.shape[3], w.shape[0], w.shape[2], w.shape[3], tuple(stride), tuple(pad4))
        if key not in seen:
            seen.append(key)
        return orig(x, w, b, stride, pad4, dilation, groups, want_stats)
    convmod.ops.conv2d_forward = spy
    try:
        net = ResNet50(numLabels=10).init()
        net.output(torch.rand(1, 3, 224, 224))
    finally:
        convmod.ops.conv2d_forward = orig
    return seen


_SHAPES = None


def _shapes():
    global _SHAPES
    if _SHAPES is None:
        _SHAPES = _resnet_conv_shapes()
    return _SHAPES


def _err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


@pytest.mark.parametrize("idx", range(21))
def test_resnet50_conv_shape_at_batch_256(cuda, idx):
    shapes = _shapes()
    if idx >= len(shapes):
        pytest.skip("fewer distinct conv shapes")
    C, H, W, K, R, S, stride, pad4 = shapes[idx]
    from deeplearning4j_amd.ops import conv2d_backward, conv2d_forward, fallback
    g = torch.Generator(device=cuda).manual_seed(idx)
    bf = torch.bfloat16
    x = torch.randn(N, C, H, W, device=cuda, generator=g).to(bf).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, S, device=cuda, generator=g) * (C * R * S) ** -0.5).to(bf)
    fallback.reset()
    y = conv2d_forward(x, w, None, stride, pad4)
    dy = torch.randn(y.shape, device=cuda, generator=g).to(bf).contiguous(memory_format=torch.channels_last)
    gW = torch.zeros(K, C, R, S, device=cuda)
    dx, dW, _ = conv2d_backward(x, w, dy, stride, pad4, (1, 1), True, True, False, gW=gW)
    dW = gW if dW is None else dW
    torch.cuda.synchronize()
    assert fallback.count() == 0, fallback.summary()
    pt, pb, pl, pr = pad4
    xf = F.pad(x.float(), (pl, pr, pt, pb)).contiguous()
    with torch.backends.cudnn.flags(enabled=False):
        yr = F.conv2d(xf, w.float(), None, stride)
        dxr, dWr, _ = torch.ops.aten.convolution_backward(dy.float().contiguous(), xf, w.float(), None, list(stride),
                                                          [0, 0], [1, 1], False, [0, 0], 1, [True, True, False])
    dxr = dxr[:, :, pt:pt + H, pl:pl + W]
    shape = f"C{C} {H}x{W} K{K} {R}x{S} s{stride} p{pad4}"
    assert y.shape == yr.shape, shape
    assert _err(y, yr) < 2e-2, ("fwd", shape, _err(y, yr))
    assert _err(dx, dxr) < 2e-2, ("bwd-data", shape, _err(dx, dxr))
    assert _err(dW, dWr) < 2e-2, ("wrw", shape, _err(dW, dWr))
