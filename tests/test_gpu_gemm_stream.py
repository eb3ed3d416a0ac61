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
