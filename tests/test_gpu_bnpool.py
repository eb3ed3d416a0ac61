"""Fused BatchNorm -> ReLU -> max pool HIP kernels (csrc/batchnorm.hip bnpool_*) vs a plain PyTorch fp32
reference of the same three ops, and the ResNet-stem fusion inside a network vs the unfused layers."""
import pytest
import torch
import torch.nn.functional as F

from deeplearning4j_amd.ops import native

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    a, b = a.double().cpu(), b.double().cpu()
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert err <= tol * scale, f"max abs err {err} (scale {scale})"


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize("shape,k,s,pad", [((4, 64, 28, 28), 3, 2, (1, 1, 1, 1)), ((3, 16, 13, 11), 3, 2, (0, 0, 0, 0)),
                                           ((2, 8, 10, 10), 2, 2, (0, 0, 0, 0))])
def test_bn_pool_kernels_match_reference(cuda, dtype, tol, shape, k, s, pad):
    g = torch.Generator().manual_seed(shape[1] + k)
    N, C, H, W = shape
    x = (torch.randn(shape, generator=g) * 1.5 + 0.3).to(dtype).to(cuda).contiguous(memory_format=torch.channels_last)
    gamma = (torch.rand(C, generator=g) + 0.5).to(cuda)
    beta = (torch.randn(C, generator=g) * 0.3).to(cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    r = native.bn_pool_fwd(x, gamma, beta, rm, rv, True, 0.9, 1e-5, (k, k), (s, s), pad)
    assert r is not None, "fused kernel refused the shape"
    y, ctx = r
    dy = torch.randn(y.shape, generator=g).to(dtype).to(cuda).contiguous(memory_format=torch.channels_last)
    dgamma = torch.empty(C, device=cuda)
    dbeta = torch.empty(C, device=cuda)
    dx, _, _ = native.bn_pool_bwd(dy, ctx, dgamma, dbeta)
    # reference in fp32 from the same (rounded) input
    xr = x.float().detach().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    mean = xr.mean((0, 2, 3))
    var = xr.var((0, 2, 3), unbiased=False)
    xh = (xr - mean.view(1, -1, 1, 1)) * torch.rsqrt(var + 1e-5).view(1, -1, 1, 1)
    a = torch.relu(xh * gr.view(1, -1, 1, 1) + br.view(1, -1, 1, 1))
    pt, pb, pl, pr = pad
    ap = F.pad(a, (pl, pr, pt, pb), value=float("-inf")) if any(pad) else a
    yr = F.max_pool2d(ap, k, s)
    yr.backward(dy.float())
    _close(y, yr, tol)
    _close(dx, xr.grad, tol * 4)
    _close(dgamma, gr.grad, tol * 4)
    _close(dbeta, br.grad, tol * 4)
    _close(rm, 0.1 * mean.detach(), 1e-4)                       # running stats updated like the unfused BN
    _close(rv, 0.9 + 0.1 * (var.detach() + 1e-5), 1e-4)


def test_resnet_stem_fusion_in_network_matches_unfused(cuda, monkeypatch):
    from deeplearning4j_amd import (Activation, ActivationLayer, BatchNormalization, ComputationGraph, ConvolutionLayer,
                                    DataType, InputType, LossFunction, NeuralNetConfiguration, OutputLayer,
                                    PoolingType, Sgd, SubsamplingLayer)
    from deeplearning4j_amd.nn.conf.enums import ConvolutionMode

    def build():
        gb = (NeuralNetConfiguration.Builder().seed(7).dataType(DataType.BFLOAT16).updater(Sgd(0.05)).graphBuilder()
              .addInputs("in").setInputTypes(InputType.convolutional(32, 32, 3)))
        gb.addLayer("c1", ConvolutionLayer.Builder([7, 7]).stride([2, 2]).padding([3, 3]).nOut(64)
                    .activation(Activation.IDENTITY).build(), "in")
        gb.addLayer("bn1", BatchNormalization.Builder().build(), "c1")
        gb.addLayer("r1", ActivationLayer.Builder().activation(Activation.RELU).build(), "bn1")
        gb.addLayer("p1", SubsamplingLayer.Builder(PoolingType.MAX, [3, 3], [2, 2])
                    .convolutionMode(ConvolutionMode.Same).build(), "r1")
        gb.addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).activation(Activation.SOFTMAX).nOut(5).build(),
                    "p1")
        gb.setOutputs("out")
        n = ComputationGraph(gb.build())
        n.init(device=cuda)
        return n

    gen = torch.Generator().manual_seed(2)
    x = torch.randn(8, 3, 32, 32, generator=gen).to(cuda)
    y = F.one_hot(torch.randint(0, 5, (8,), generator=gen), 5).float().to(cuda)
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DL4J_AMD_FUSE_POOL", flag)
        net = build()
        assert (getattr(net.layers_by_name["bn1"], "fuse_pool", None) is not None) == (flag == "1")
        out0 = net.outputSingle(x)
        net.fit([x], [y])
        torch.cuda.synchronize()
        if flag == "1":
            assert net.layers_by_name["bn1"]._ctx[0] == "NATIVE_POOL", "fused HIP kernel did not run"
        res.append((out0, net.params().clone()))
    _close(res[0][0], res[1][0], 2e-2)
    _close(res[0][1], res[1][1], 1e-2)                         # one bf16 ulp at |p| ~ 1 is 7.8e-3


@pytest.mark.parametrize("N,H", [(2, 224), (3, 64), (1, 32)])
def test_stem_conv_kernel_matches_reference(cuda, N, H):
    """csrc/conv_stem.hip (7x7/2, pad 3, 3->64) vs fp32 F.conv2d, and its epilogue BN tile statistics vs the
    batch statistics of the output."""
    from deeplearning4j_amd.ops import conv_native, conv_stem
    conv_native.bump_version()                                   # packed-weight cache is keyed by buffer + version
    g = torch.Generator().manual_seed(N * H)
    x = torch.randn(N, 3, H, H, generator=g).to(torch.bfloat16).to(cuda).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    assert conv_stem.supported(x, w, None, (2, 2), (3, 3, 3, 3), (1, 1))
    y = conv_stem.forward(x, w, want_stats=True)
    assert y is not None
    ref = F.conv2d(x.float(), w.float(), None, 2, 3)
    _close(y, ref, 1e-2)
    ts, P, rpp = y._bn_tile_stats
    M = N * y.shape[2] * y.shape[3]
    assert P * rpp == M
    rows = y.permute(0, 2, 3, 1).reshape(-1, 64).float()
    sh = ts[2]                                                   # [P, 64] per-tile shifts
    n = float(rpp)
    mean_t = sh + ts[0] / n                                      # per-tile means
    mean = mean_t.mean(0)
    _close(mean, rows.mean(0), 1e-4)
    var = ((ts[1] + 2 * (sh - mean) * ts[0] + n * (sh - mean) ** 2).sum(0)) / M
    _close(var, rows.var(0, unbiased=False), 1e-3)


@pytest.mark.parametrize("N,H", [(2, 224), (3, 64)])
def test_stem_conv_weight_gradient_matches_reference(cuda, N, H):
    """Stem weight/bias gradient kernel (csrc/conv_stem.hip stem_conv_wrw + fixed-order reduce) vs fp32 autograd."""
    from deeplearning4j_amd.ops import conv_stem
    g = torch.Generator().manual_seed(N + H)
    x = torch.randn(N, 3, H, H, generator=g).to(torch.bfloat16).to(cuda).contiguous(memory_format=torch.channels_last)
    OH = (H - 1) // 2 + 1
    dy = torch.randn(N, 64, OH, OH, generator=g).to(torch.bfloat16).to(cuda).contiguous(
        memory_format=torch.channels_last)
    gW = torch.zeros(64, 3, 7, 7, device=cuda)
    gb = torch.zeros(64, device=cuda)
    r = conv_stem.backward_weight(x, dy, gW, gb, True)
    assert r == (None, None), "gradients were not written in place"
    w = torch.zeros(64, 3, 7, 7, device=cuda, requires_grad=True)
    b = torch.zeros(64, device=cuda, requires_grad=True)
    F.conv2d(x.float(), w, b, 2, 3).backward(dy.float())
    _close(gW, w.grad, 2e-3)
    _close(gb, b.grad, 2e-3)
