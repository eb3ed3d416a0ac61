"""BatchNorm backward sums from the epilogue of the consuming conv's backward-data launch (csrc/mfma_tile.h
epi_bnbwd_wave, csrc/batchnorm.hip dl4j_bn_bwd_planes) against the full BN backward (bn_bwd_partial re-reading dy
and x) and the fp32 torch reference of the same op (reference NN:nn/layers/normalization/BatchNormalization.java:
131-210)."""
import pytest
import torch

from deeplearning4j_amd import ops
from deeplearning4j_amd.ops import native

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert err <= tol * scale, f"max abs err {err} (scale {scale})"


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("R,shape,K", [(1, (8, 64, 14, 14), 128), (3, (8, 64, 14, 14), 64),
                                       (1, (4, 128, 7, 9), 256), (3, (3, 64, 11, 13), 128),
                                       (3, (2, 192, 5, 6), 64)])
def test_bn_bwd_epilogue_matches_full(cuda, monkeypatch, dtype, relu, R, shape, K):
    monkeypatch.setenv("DL4J_AMD_CONV_TUNE", "0")       # default tiles: the round-3 engine, which has the epilogue
    monkeypatch.setattr(native, "BNB", True)
    monkeypatch.setattr(native, "BNB_MODE", 2)
    g = torch.Generator().manual_seed(1)
    N, C, H, W = shape
    x = _cl((torch.randn(*shape, generator=g) * 2 + 0.5).to(dtype).to(cuda))
    gamma = (torch.rand(C, generator=g) + 0.5).to(cuda)
    beta = torch.randn(C, generator=g).to(cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, ctx = ops.bn_forward(x, gamma, beta, rm, rv, True, 0.9, 1e-5, relu)
    assert ctx[0] == "NATIVE" and hasattr(y, "_bn_bwd_req")
    w = (torch.randn(K, C, R, R, generator=g) * 0.1).to(dtype).to(cuda)
    dz = _cl(torch.randn(N, K, H, W, generator=g).to(dtype).to(cuda))
    p = R // 2
    dx, _, _ = ops.conv2d_backward(y, w, dz, (1, 1), (p, p, p, p), need_dx=True, need_dw=False, need_db=False)
    assert hasattr(dx, "_bn_bwd_stats"), "bwd-data launch did not produce the BN-backward planes"
    plain = dx.clone()                                   # same values, no planes: the full backward
    assert not hasattr(plain, "_bn_bwd_stats")
    got = ops.bn_backward(dx, ctx)
    ref = ops.bn_backward(plain, ctx)
    _close(got[0], ref[0], 2e-2)
    _close(got[1], ref[1], 2e-3)
    _close(got[2], ref[2], 2e-3)
    # fp32 torch reference of the BN backward on the stored dy
    rm_c, rv_c = torch.zeros(C), torch.ones(C)
    _, c_ref = ops.bn_forward(x.float().cpu(), gamma.cpu(), beta.cpu(), rm_c, rv_c, True, 0.9, 1e-5, relu)
    dx_r, dg_r, db_r, _ = ops.bn_backward(dx.float().cpu(), c_ref)
    _close(got[0], dx_r, 4e-2)
    _close(got[1], dg_r, 3e-2)
    _close(got[2], db_r, 3e-2)


@pytest.mark.parametrize("residual", [False, True])
def test_bn_bwd_epilogue_of_accumulated_gradient(cuda, monkeypatch, residual):
    """Fan-out: the 1x1 bwd-data GEMM sums dX into another consumer's gradient (beta = 1) and its epilogue sums are
    those of the stored SUM; a BN layer with a fused residual takes its ReLU from the forward's bitmask. Both match
    the full backward (dx, dgamma, dbeta, dresidual); an in-place edit afterwards invalidates the planes."""
    monkeypatch.setenv("DL4J_AMD_CONV_TUNE", "0")
    monkeypatch.setattr(native, "BNB", True)
    monkeypatch.setattr(native, "BNB_MODE", 2)
    g = torch.Generator().manual_seed(2)
    C, K = 128, 64
    x = _cl((torch.randn(4, C, 9, 8, generator=g) + 0.3).to(torch.bfloat16).to(cuda))
    res = _cl(torch.randn(4, C, 9, 8, generator=g).to(torch.bfloat16).to(cuda)) if residual else None
    gamma = (torch.rand(C, generator=g) + 0.5).to(cuda)
    beta = torch.randn(C, generator=g).to(cuda)
    y, ctx = ops.bn_forward(x, gamma, beta, torch.zeros(C, device=cuda), torch.ones(C, device=cuda), True, 0.9, 1e-5,
                            True, residual=res)
    assert hasattr(y, "_bn_bwd_req") and (y._bn_bwd_req[3] is not None) == residual
    w = (torch.randn(K, C, 1, 1, generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    dz = _cl(torch.randn(4, K, 9, 8, generator=g).to(torch.bfloat16).to(cuda))
    other = _cl(torch.randn(4, C, 9, 8, generator=g).to(torch.bfloat16).to(cuda))   # another consumer's gradient
    acc = other.clone()
    d, _, _ = ops.conv2d_backward(y, w, dz, (1, 1), (0, 0, 0, 0), need_dx=True, need_dw=False, need_db=False,
                                  dx_accum=acc)
    assert d is acc and hasattr(d, "_bn_bwd_stats")
    plain, _, _ = ops.conv2d_backward(y, w, dz, (1, 1), (0, 0, 0, 0), need_dx=True, need_dw=False, need_db=False)
    _close(d, plain.float() + other.float(), 2e-2)
    got = ops.bn_backward(d, ctx)
    ref = ops.bn_backward(d.clone(), ctx)
    _close(got[0], ref[0], 2e-2)
    _close(got[1], ref[1], 2e-3)
    _close(got[2], ref[2], 2e-3)
    if residual:
        _close(got[3], ref[3], 1e-6)
    d.mul_(1.0)                                          # an in-place edit after the launch: planes are stale
    assert native._bnb_planes(d, ctx[2], ctx[6], ctx[4], ctx[5], ctx[7]) is None


def test_resnet_gradients_with_bn_bwd_epilogue_match_full(cuda, monkeypatch):
    """Whole-network gradient of the zoo ResNet-50 (bf16) with and without the epilogue sums: the flat gradients agree
    to bf16 summation-order noise (relative L2 distance), and the epilogue path really ran."""
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    monkeypatch.setenv("DL4J_AMD_CONV_TUNE", "0")
    monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
    g = torch.Generator().manual_seed(3)
    x = torch.rand(4, 3, 224, 224, generator=g).to(cuda)
    y = torch.zeros(4, 10, device=cuda)
    y[torch.arange(4), torch.tensor([1, 2, 3, 4])] = 1
    calls = {"planes": 0}
    orig = native._bnb_planes

    def spy(*a):
        r = orig(*a)
        calls["planes"] += r is not None
        return r
    monkeypatch.setattr(native, "_bnb_planes", spy)
    grads = []
    for flag in (False, True):
        monkeypatch.setattr(native, "BNB", flag)
        monkeypatch.setattr(native, "BNB_MODE", 2 if flag else 0)
        net = ResNet50(numLabels=10, seed=11, dataType=DataType.BFLOAT16).init(device=cuda)
        net.computeGradientAndScore([x], [y])
        grads.append(net.flattenedGradients.float().clone())
        if not flag:
            assert calls["planes"] == 0
    assert calls["planes"] >= 32, calls                 # >= 2 non-residual BNs per bottleneck x 16 blocks
    g0, g1 = grads
    rel = ((g1 - g0).norm() / g0.norm()).item()
    assert rel < 2e-2, rel
