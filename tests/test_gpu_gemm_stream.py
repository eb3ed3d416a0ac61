"""GPU numerics of the persistent streaming GEMM (csrc/gemm_stream.hip, dl4j_gemm configuration 10) against an fp32
torch reference: every (BN, K/64, slots) variant, bf16 and fp16, bias / ReLU epilogues, the BatchNorm tile-statistics
epilogue, grids with idle blocks (fewer m-tiles than blocks) and many tiles per block, the zoo ResNet-50 bench shapes,
and refusal (-4) of shapes outside its contract. Asymmetric random operands."""
import pytest
import torch

from deeplearning4j_amd.ops import gemm

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(M, N, K, dt=torch.bfloat16, bias=False, act=None, stats=False, seed=0):
    torch.manual_seed(seed)
    a = (torch.randn(M, K, device=DEV) * 0.5).to(dt)
    w = (torch.randn(N, K, device=DEV) * 0.5).to(dt)              # [out, in]: B = w.t() is K-contiguous
    bv = torch.randn(N, device=DEV) if bias else None
    ts = torch.full((3, M // 64, N), float("nan"), device=DEV) if stats else None
    old = gemm._FORCE_CFG
    gemm._FORCE_CFG = gemm.STREAM_CFG
    try:
        out = gemm.mmul(a, w.t(), bias=bv, act=act, stats=ts) if stats else gemm.mmul(a, w.t(), bias=bv, act=act,
                                                                                        out_dtype=dt)
    finally:
        gemm._FORCE_CFG = old
    torch.cuda.synchronize()
    ref = a.float() @ w.float().t()
    if bias:
        ref = ref + bv.reshape(1, -1)
    if act == "relu":
        ref = ref.clamp_min(0)
    tol = (3e-2 if dt == torch.bfloat16 else 6e-3) * max(1.0, (K / 64) ** 0.5) * max(1.0, ref.abs().max().item() / 8)
    err = (out.float() - ref).abs().max().item()
    assert err <= tol, f"M={M} N={N} K={K} {dt}: max err {err:.4g} > {tol:.4g}"
    return out, ts


@pytest.mark.parametrize("N,K", [(256, 64), (512, 64), (128, 64), (256, 128), (512, 256), (64, 64), (64, 128),
                                 (64, 256), (128, 512), (192, 64)])
def test_variants(N, K):
    _run(128 * 40, N, K)                   # 40 m-tiles: most blocks idle
    _run(128 * 1000, N, K, seed=1)         # ~4-16 tiles per block


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_dtypes_bias_relu(dt):
    _run(128 * 300, 256, 64, dt=dt, bias=True, act="relu")
    _run(128 * 300, 1024, 256, dt=dt, bias=True)


@pytest.mark.parametrize("N,K", [(256, 64), (512, 128), (1024, 256), (64, 256)])
def test_bn_tile_statistics(N, K):
    M = 128 * 333
    out, ts = _run(M, N, K, stats=True, seed=3)
    y = out.float()
    P = M // 64
    blk = y.reshape(P, 64, N)
    sh = blk[:, 0]
    assert torch.equal(ts[2], sh)
    d = blk - sh[:, None]
    assert torch.allclose(ts[0], d.sum(1), atol=2e-2, rtol=1e-4)
    assert torch.allclose(ts[1], (d * d).sum(1), atol=2e-1, rtol=1e-4)


def test_bench_shapes_and_determinism():
    """The zoo ResNet-50 batch-1024 1x1 shapes; two launches give bitwise equal outputs."""
    for M, N, K in [(802816, 256, 64), (802816, 64, 256), (200704, 512, 128), (50176, 1024, 256)]:
        o1, _ = _run(M, N, K, seed=7)
        o2, _ = _run(M, N, K, seed=7)
        assert torch.equal(o1, o2)


def test_refuses_outside_contract():
    a = torch.randn(1000, 64, device=DEV).bfloat16()       # M % 128 != 0
    w = torch.randn(256, 64, device=DEV).bfloat16()
    old = gemm._FORCE_CFG
    gemm._FORCE_CFG = gemm.STREAM_CFG
    try:
        with pytest.raises(RuntimeError):
            gemm.mmul(a, w.t(), out_dtype=torch.bfloat16)
    finally:
        gemm._FORCE_CFG = old


@pytest.mark.parametrize("case", [
    # N, H, W, C, K, R, S, stride, pad
    (16, 28, 28, 64, 64, 3, 3, 1, 1),
    (32, 14, 14, 128, 128, 3, 3, 1, 1),
    (8, 28, 28, 64, 256, 1, 1, 1, 0),
    (128, 14, 14, 256, 128, 3, 3, 2, 1),     # strided, ragged taps at the border
    (128, 7, 7, 512, 512, 3, 3, 1, 1),
])
@pytest.mark.parametrize("stats", [False, True])
def test_conv_stream(case, stats):
    """Persistent implicit-GEMM conv (conv_stream, conv variant 100) vs fp32 torch conv2d, with bias and the BN
    tile-statistics epilogue."""
    from deeplearning4j_amd.ops import conv_native
    N, H, W, C, K, R, S, st, pd = case
    torch.manual_seed(11)
    x = (torch.randn(N, C, H, W, device=DEV) * 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, S, device=DEV) * 0.1).to(torch.bfloat16)
    b = torch.randn(K, device=DEV)
    OH, OW = (H + 2 * pd - R) // st + 1, (W + 2 * pd - S) // st + 1
    M = N * OH * OW
    if M % 128:
        pytest.skip("conv_stream needs N*OH*OW % 128 == 0")
    wk = w.permute(0, 2, 3, 1).contiguous()                       # [K][R][S][C]
    y = torch.empty(N, K, OH, OW, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ts = torch.full((3, M // 64, K), float("nan"), device=DEV) if stats else None
    geom = (N, H, W, C, K, R, S, st, st, pd, pd, 1, 1, OH, OW)
    rc = conv_native._fwd_launch(conv_native.STREAM_VAR, x, wk, b, y, geom, 0.0, ts)
    assert rc == (1 if stats else 0), rc
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv2d(x.float(), w.float(), b, stride=st, padding=pd)
    err = (y.float() - ref).abs().max().item()
    # bf16 output rounding (2^-8 relative) + accumulation of bf16 products over R*S*C terms
    assert err <= 8e-3 * ref.abs().max().item() + 1e-2 * (R * S * C / 64) ** 0.5, err
    if stats:
        yr = y.permute(0, 2, 3, 1).reshape(M, K).float().reshape(M // 64, 64, K)
        sh = yr[:, 0]
        assert torch.equal(ts[2], sh)
        d = yr - sh[:, None]
        assert torch.allclose(ts[0], d.sum(1), atol=2e-2, rtol=1e-4)
