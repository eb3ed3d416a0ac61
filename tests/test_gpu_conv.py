"""MFMA implicit-GEMM conv kernels vs a plain fp32 torch reference (run on MI355X)."""
import pytest
import torch
import torch.nn.functional as F

from deeplearning4j_amd.ops import conv_native

pytestmark = pytest.mark.gpu

CASES = [
    # N, C, H, W, K, R, S, stride, pad4(t,b,l,r)
    (2, 64, 9, 9, 64, 1, 1, (1, 1), (0, 0, 0, 0)),
    (3, 64, 8, 7, 256, 1, 1, (1, 1), (0, 0, 0, 0)),
    (2, 128, 11, 11, 64, 1, 1, (2, 2), (0, 0, 0, 0)),
    (2, 64, 10, 9, 64, 3, 3, (1, 1), (1, 1, 1, 1)),
    (2, 32, 7, 7, 136, 3, 3, (1, 1), (0, 1, 0, 1)),
    (2, 8, 23, 23, 64, 7, 7, (2, 2), (3, 3, 3, 3)),
    (1, 256, 5, 5, 512, 3, 3, (1, 1), (1, 1, 1, 1)),
    (4, 512, 4, 4, 2048, 1, 1, (1, 1), (0, 0, 0, 0)),
    (2, 48, 6, 6, 64, 3, 3, (1, 1), (1, 1, 1, 1)),
    (3, 96, 9, 9, 64, 3, 3, (2, 2), (1, 1, 1, 1)),
]


def _ref(x, w, b, stride, pad4):
    xp = F.pad(x, (pad4[2], pad4[3], pad4[0], pad4[1]))
    return F.conv2d(xp, w, b, stride)


def _close(a, b, tol):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err <= tol * scale, f"max abs err {err} vs scale {scale}"


@pytest.mark.parametrize("case", CASES)
def test_conv_fwd_bwd(cuda, case):
    N, C, H, W, K, R, S, stride, pad4 = case
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, C, H, W, generator=g).to(cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, S, generator=g) * 0.1).to(cuda).bfloat16()
    b = torch.randn(K, generator=g).to(cuda)
    conv_native.bump_version()
    y = conv_native.conv2d_fwd(x, w, b, stride, pad4, (1, 1))
    assert y is not None
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = _ref(xr, wr, br, stride, pad4)
    _close(y, yr.detach(), 2e-2)
    dy = torch.randn(yr.shape, generator=g).to(cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    gW = torch.empty(K, C, R, S, device=cuda)
    gb = torch.empty(K, device=cuda)
    dx, dW, db = conv_native.conv2d_bwd(x, w, dy, stride, pad4, (1, 1), True, True, True, gW, gb)
    assert dW is None and db is None          # written in place into the fp32 views
    _close(gW, wr.grad, 2e-2)
    _close(gb, br.grad, 2e-2)
    _close(dx, xr.grad, 2e-2)


def test_conv_layer_uses_native_kernels(cuda):
    """A bf16 ConvolutionLayer routes through the HIP kernels (no MIOpen) for supported shapes."""
    from deeplearning4j_amd import ops
    x = torch.randn(2, 64, 8, 8, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 64, 3, 3, device=cuda).bfloat16()
    assert ops.use_native(x, "conv")
    y = ops.conv2d_forward(x, w, None, (1, 1), (1, 1, 1, 1))
    assert y.is_contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("case", CASES)
def test_conv_kernel_variants_agree(cuda, case):
    """LDS-DMA pipelined kernel (variant 1) == register-staged kernel (variant 0), bit for bit."""
    N, C, H, W, K, R, S, stride, pad4 = case
    if C % 8 != 0:
        pytest.skip("native path needs C % 8 == 0")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, C, H, W, generator=g).to(cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, S, generator=g) * 0.1).to(cuda).bfloat16()
    outs = []
    for v in (0, 1):
        conv_native.set_kernel_variant(v)
        conv_native.set_wrw_variant(v)
        conv_native.bump_version()
        y = conv_native.conv2d_fwd(x, w, None, stride, pad4, (1, 1))
        dy = torch.ones_like(y) * 0.01 + y * 0.1
        dx, _, _ = conv_native.conv2d_bwd(x, w, dy, stride, pad4, (1, 1), True, False, False)
        gW = torch.zeros(K, C, R, S, device=cuda)
        gb = torch.zeros(K, device=cuda)
        conv_native.conv2d_bwd(x, w, dy, stride, pad4, (1, 1), False, True, True, gW, gb)
        outs.append((y, dx, gW, gb))
    conv_native.set_kernel_variant(1)
    conv_native.set_wrw_variant(0)
    assert torch.equal(outs[0][0], outs[1][0])
    if outs[0][1] is not None:
        assert torch.equal(outs[0][1], outs[1][1])
    # weight/bias gradients accumulate with atomics in a different order: equal up to fp32 rounding
    _close(outs[1][2], outs[0][2], 1e-5)
    _close(outs[1][3], outs[0][3], 1e-5)


@pytest.mark.parametrize("tiled", [True, False])
def test_batched_relayout_matches_per_weight(tiled):
    """One launch refreshes every weight's kernel layouts: the LDS-tiled kernel (<= 16 taps; edge tiles in K and C,
    K % 8 != 0 without a flipped copy, 1x1 KRSC as a view) and the element-gather kernel (a 7x7 weight in the set)
    both equal the permuted / rotated weight exactly."""
    from deeplearning4j_amd.ops import conv_native as cn
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    shapes = [(64, 64, 3, 3), (256, 64, 1, 1), (128, 256, 1, 1), (12, 16, 3, 3), (200, 40, 3, 3), (72, 24, 1, 3)]
    if not tiled:
        shapes.append((64, 8, 7, 7))
    ws = [torch.randn(s, generator=g).to(torch.bfloat16).to(dev) for s in shapes]
    cn.bump_version()
    assert cn.relayout_all(ws) == len(ws)
    got = [(cn._ent(w).krsc.clone(), None if cn._ent(w).flip is None else cn._ent(w).flip.clone()) for w in ws]
    for w, (k, f) in zip(ws, got):
        K, C, R, S = w.shape
        torch.testing.assert_close(k.cpu(), w.permute(0, 2, 3, 1).contiguous().cpu(), rtol=0, atol=0)
        if K % 8 == 0:
            ref = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()
            torch.testing.assert_close(f.cpu(), ref.cpu(), rtol=0, atol=0)


def test_network_uses_batched_relayout():
    """A bf16 ResNet-50 training step refreshes every conv weight through the single batched relayout (the
    per-weight kernel is then never needed)."""
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.ops import conv_native as cn
    dev = torch.device("cuda", 0)
    net = ResNet50(numLabels=10, dataType=DataType.BFLOAT16).init(device=dev)
    calls = {"single": 0}
    orig = cn.native.load().dl4j_conv_w_relayout

    class Spy:
        def __call__(self, *a):
            calls["single"] += 1
            return orig(*a)
    lib = cn.native.load()
    lib.dl4j_conv_w_relayout = Spy()
    try:
        x = torch.rand(2, 3, 224, 224, device=dev)
        y = torch.zeros(2, 10, device=dev)
        y[:, 1] = 1
        net.fit([x], [y])
        net.fit([x], [y])
    finally:
        lib.dl4j_conv_w_relayout = orig
    assert len(net._conv_ws) == 53
    assert calls["single"] <= 2          # only weights outside the batched criteria (the C=3 stem goes to MIOpen)


@pytest.mark.parametrize("case", [c for c in CASES if c[5] == c[6] and (c[7] == (1, 1) or c[5] == 1)])
def test_conv_bwd_data_accumulates_in_place(cuda, case):
    """dx_accum: the bwd-data kernel adds its result into an existing gradient of x (graph fan-out) in the epilogue."""
    N, C, H, W, K, R, S, stride, pad4 = case
    if R == 1 and any(pad4):
        pytest.skip("padded 1x1 is not a native bwd-data path")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, C, H, W, generator=g).to(cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, S, generator=g) * 0.1).to(cuda).bfloat16()
    conv_native.bump_version()
    y = conv_native.conv2d_fwd(x, w, None, stride, pad4, (1, 1))
    dy = torch.randn(y.shape, generator=g).to(cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    other = torch.randn(x.shape, generator=g).to(cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    dx_ref, _, _ = conv_native.conv2d_bwd(x, w, dy, stride, pad4, (1, 1), True, False, False)
    acc = other.clone()
    dx, _, _ = conv_native.conv2d_bwd(x, w, dy, stride, pad4, (1, 1), True, False, False, dx_accum=acc)
    assert dx is acc
    _close(dx, other.float() + dx_ref.float(), 2e-2)


@pytest.mark.parametrize("batch", [16, 400])
def test_conv_epilogue_bn_stats_match_separate_pass(cuda, monkeypatch, batch):
    """Conv -> BN (training): statistics from the conv kernel epilogue give the same BN forward / running stats /
    update as the separate statistics pass (DL4J_AMD_CONV_BN_STATS=0). batch 16: <= 64 folded tile rows (one fused
    fold+finalize launch); batch 400: 2500 tile partials (tile re-centring pass, then the ticketed fold)."""
    from deeplearning4j_amd import (Activation, ActivationLayer, BatchNormalization, ComputationGraph, ConvolutionLayer,
                                    DataType, GlobalPoolingLayer, InputType, LossFunction, NeuralNetConfiguration,
                                    OutputLayer, PoolingType, Sgd)

    def build():
        g = (NeuralNetConfiguration.Builder().seed(3).dataType(DataType.BFLOAT16).updater(Sgd(0.1)).graphBuilder()
             .addInputs("in").setInputTypes(InputType.convolutional(20, 20, 64)))
        g.addLayer("c1", ConvolutionLayer.Builder([3, 3]).padding([1, 1]).nOut(128)
                   .activation(Activation.IDENTITY).build(), "in")
        g.addLayer("bn1", BatchNormalization.Builder().build(), "c1")
        g.addLayer("r1", ActivationLayer.Builder().activation(Activation.RELU).build(), "bn1")
        g.addLayer("p", GlobalPoolingLayer.Builder(PoolingType.AVG).build(), "r1")
        g.addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).activation(Activation.SOFTMAX).nOut(5).build(), "p")
        g.setOutputs("out")
        n = ComputationGraph(g.build())
        n.init(device=cuda)
        return n

    gen = torch.Generator().manual_seed(1)
    x = (torch.randn(batch, 64, 20, 20, generator=gen) + 0.7).to(cuda)
    y = torch.nn.functional.one_hot(torch.randint(0, 5, (batch,), generator=gen), 5).float().to(cuda)
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DL4J_AMD_CONV_BN_STATS", flag)
        net = build()
        assert net.layers_by_name["c1"].emit_bn_stats == (flag == "1")
        net.fit([x], [y])
        torch.cuda.synchronize()
        res.append((net.params().clone(), net.getParam("bn1_mean").clone(), net.getParam("bn1_var").clone()))
    (p1, m1, v1), (p0, m0, v0) = res
    _close(m1, m0, 1e-4)
    _close(v1, v0, 1e-4)
    _close(p1, p0, 1e-3)


PHASE_CASES = [
    # N, C, H, W, K, R, S, stride, pad4 — strided bwd-data through the phase-split path (canonical ResNet-50's 3x3/2,
    # odd sizes, 5x5/2, a 2x2/2 deconv-style kernel and a 7x7/2 stem-like conv)
    (2, 64, 56, 56, 64, 3, 3, (2, 2), (1, 1, 1, 1)),
    (2, 128, 15, 13, 64, 3, 3, (2, 2), (1, 1, 1, 1)),
    (2, 64, 17, 17, 128, 5, 5, (2, 2), (2, 2, 2, 2)),
    (2, 64, 16, 16, 64, 2, 2, (2, 2), (0, 0, 0, 0)),
    (2, 64, 29, 29, 64, 3, 3, (2, 2), (0, 0, 0, 0)),
    (2, 64, 30, 30, 64, 7, 7, (2, 2), (3, 3, 3, 3)),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", PHASE_CASES)
def test_strided_bwd_data_phase_split(cuda, case, dtype, monkeypatch):
    """Phase-split strided bwd-data (one stride-1 sub-conv per phase) == fp32 torch, == the zero-interleave path, and
    accumulates into dx_accum."""
    N, C, H, W, K, R, S, stride, pad4 = case
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, C, H, W, generator=g).to(cuda).to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, S, generator=g) * 0.1).to(cuda).to(dtype)
    xr = x.float().requires_grad_(True)
    yr = _ref(xr, w.float(), None, stride, pad4)
    dy = torch.randn(yr.shape, generator=g).to(cuda).to(dtype).contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    conv_native.bump_version()
    plan = conv_native._phase_plan(H, W, dy.shape[2], dy.shape[3], R, S, stride, pad4, (1, 1))
    assert plan is not None
    calls = {"n": 0}
    orig = conv_native._bwd_data_phases

    def spy(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)
    monkeypatch.setattr(conv_native, "_bwd_data_phases", spy)
    dx, _, _ = conv_native.conv2d_bwd(x, w, dy, stride, pad4, (1, 1), True, False, False)
    if dtype == torch.float16 and calls["n"] == 0:
        pytest.skip("fp16 sub-kernel outside the round-3 engine")
    assert calls["n"] == 1
    _close(dx, xr.grad, 2e-2)
    other = torch.randn(x.shape, generator=g).to(cuda).to(dtype).contiguous(memory_format=torch.channels_last)
    acc = other.clone()
    dx2, _, _ = conv_native.conv2d_bwd(x, w, dy, stride, pad4, (1, 1), True, False, False, dx_accum=acc)
    _close(dx2, other.float() + xr.grad, 2e-2)
    if dtype == torch.bfloat16:
        monkeypatch.setattr(conv_native, "_PHASE", False)
        dxz, _, _ = conv_native.conv2d_bwd(x, w, dy, stride, pad4, (1, 1), True, False, False)
        _close(dx, dxz.float(), 1e-2)
