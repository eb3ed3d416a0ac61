"""Halo-staged 3x3 convolution (csrc/conv_halo.hip, conv variant 101): 64 -> 64 channels, stride 1, pad 1, NHWC bf16
— forward against fp32 torch conv2d (with bias), its per-chunk BatchNorm statistics against sums of the stored output,
a BatchNorm layer consuming those statistics (rows-per-partial = pixels per chunk) against torch batch statistics, and
the stride-1 backward-data path (the same kernel on the flipped weights) against torch autograd. Shapes cover one-row
bands (28 x 28: 4 rows per chunk, 56 x 56: 2 rows, 3-slot and 2-slot rings) and multi-image chunks (8 x 8: 2 images)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _data(N, H, W, seed=3):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.randn(N, 64, H, W, generator=g) * 0.5).to(DEV).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.1).to(DEV).to(torch.bfloat16)
    b = torch.randn(64, generator=g).to(DEV)
    return x, w, b


@pytest.mark.parametrize("N,H", [(4, 28), (3, 28), (2, 56), (8, 8), (16, 14)])
@pytest.mark.parametrize("stats", [False, True])
def test_conv_halo_forward(N, H, stats):
    from deeplearning4j_amd.ops import conv_native as CN
    x, w, b = _data(N, H, H)
    geom = (N, H, H, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, H, H)
    nch, pc = CN._halo_plan(geom)
    assert nch > 0 and 0 < pc <= 128 and nch * pc == N * H * H
    wk = w.permute(0, 2, 3, 1).contiguous()
    y = torch.full((N, 64, H, H), float("nan"), device=DEV, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ts = CN._stats_buf(CN.HALO_VAR, N * H * H, 64, x.device, geom) if stats else None
    if stats:
        ts.fill_(float("nan"))
    rc = CN._fwd_launch(CN.HALO_VAR, x, wk, b, y, geom, 0.0, ts)
    assert rc == (1 if stats else 0), rc
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv2d(x.float(), w.float(), b, padding=1)
    err = (y.float() - ref).abs().max().item()
    assert err <= 8e-3 * ref.abs().max().item() + 1e-2 * (9 * 64 / 64) ** 0.5, err
    if stats:
        yr = y.permute(0, 2, 3, 1).reshape(nch, pc, 64).float()
        sh = yr[:, 0]
        assert torch.equal(ts[2], sh)
        d = yr - sh[:, None]
        assert torch.allclose(ts[0], d.sum(1), atol=2e-2, rtol=1e-4)
        assert torch.allclose(ts[1], (d * d).sum(1), atol=2e-2, rtol=1e-4)


def test_conv_halo_refuses_other_shapes():
    from deeplearning4j_amd.ops import conv_native as CN
    x = torch.zeros(2, 128, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wk = torch.zeros(128, 3, 3, 128, device=DEV, dtype=torch.bfloat16)
    y = torch.empty_like(x)
    assert CN._fwd_launch(CN.HALO_VAR, x, wk, None, y, (2, 14, 14, 128, 128, 3, 3, 1, 1, 1, 1, 1, 1, 14, 14), 0.0,
                          None) == -1
    x64 = torch.zeros(2, 64, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wk64 = torch.zeros(64, 3, 3, 64, device=DEV, dtype=torch.bfloat16)
    assert CN._fwd_launch(CN.HALO_VAR, x64, wk64, None, torch.empty_like(x64),
                          (2, 14, 14, 64, 64, 3, 3, 2, 2, 1, 1, 1, 1, 7, 7), 0.0, None) == -1          # stride 2
    assert CN._fwd_launch(CN.HALO_VAR, x64, wk64, None, torch.empty_like(x64),
                          (2, 14, 14, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, 14, 14), 1.0, None) == -1        # beta


@pytest.mark.parametrize("N,H", [(8, 28), (16, 8)])
def test_batchnorm_consumes_halo_chunk_statistics(N, H):
    """conv (halo kernel, statistics epilogue) -> training BN: the BN statistics come from the chunk partials."""
    from deeplearning4j_amd.ops import conv_native as CN
    from deeplearning4j_amd.ops.norm import bn_forward
    x, w, b = _data(N, H, H, seed=5)
    geom = (N, H, H, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, H, H)
    key = ("fwd", geom, False, True, torch.bfloat16)
    CN._V3_CHOICE[key] = CN.HALO_VAR
    try:
        y = CN._conv2d_fwd(x, w, None, (1, 1), (1, 1, 1, 1), (1, 1), want_stats=True)
    finally:
        CN._V3_CHOICE.pop(key, None)
    assert len(y._bn_tile_stats) == 3 and y._bn_tile_stats[2] == CN._halo_plan(geom)[1]
    gamma = torch.rand(64, device=DEV) + 0.5
    beta = torch.randn(64, device=DEV)
    rm, rv = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    out, ctx = bn_forward(y, gamma, beta, rm, rv, True, 0.9, 1e-5, relu=True)
    torch.cuda.synchronize()
    yf = y.float()
    mean = yf.mean(dim=(0, 2, 3))
    var = yf.var(dim=(0, 2, 3), unbiased=False)
    assert torch.allclose(rm, 0.1 * mean, atol=1e-4, rtol=1e-3)
    assert torch.allclose(rv, 0.9 + 0.1 * (var + 1e-5), atol=1e-4, rtol=1e-3)
    ref = torch.relu((yf - mean[None, :, None, None]) * torch.rsqrt(var + 1e-5)[None, :, None, None] *
                     gamma[None, :, None, None] + beta[None, :, None, None])
    assert (out.float() - ref).abs().max().item() < 3e-2


@pytest.mark.parametrize("N,H", [(4, 28), (8, 8)])
def test_conv_halo_backward_data(N, H):
    """Stride-1 backward-data on the halo kernel (flipped, transposed weights) vs torch autograd."""
    from deeplearning4j_amd.ops import conv_native as CN
    x, w, _ = _data(N, H, H, seed=9)
    g = torch.Generator(device="cpu").manual_seed(10)
    dy = (torch.randn(N, 64, H, H, generator=g) * 0.5).to(DEV).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    geo_b = (N, H, H, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, H, H)
    key = ("bwd", geo_b, torch.bfloat16, False)
    CN._V3_CHOICE[key] = CN.HALO_VAR
    try:
        r = CN._conv2d_bwd(x, w, dy, (1, 1), (1, 1, 1, 1), (1, 1), True, False, False)
    finally:
        CN._V3_CHOICE.pop(key, None)
    dx = r[0]
    torch.cuda.synchronize()
    xr = x.float().requires_grad_()
    torch.nn.functional.conv2d(xr, w.float(), None, padding=1).backward(dy.float())
    err = (dx.float() - xr.grad).abs().max().item()
    assert err <= 8e-3 * xr.grad.abs().max().item() + 3e-2, err
