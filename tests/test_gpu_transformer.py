"""Transformer HIP kernels vs plain-torch fp32 references: flash-style attention forward/backward
(csrc/attention.hip) and LayerNorm (+ fused residual) forward/backward (csrc/layernorm.hip)."""
import pytest
import torch

from deeplearning4j_amd.ops import transformer_native as TN

pytestmark = pytest.mark.gpu


def _err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return (a - b).abs().max().item() / max(1.0, b.abs().max().item())


@pytest.mark.parametrize("B,T,H,D", [(2, 64, 2, 64), (3, 77, 4, 64), (2, 200, 2, 128), (1, 512, 12, 64)])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_attention_fwd_bwd_matches_reference(cuda, B, T, H, D, masked, causal, dt):
    g = torch.Generator().manual_seed(B * 1000 + T + D)
    qkv = (torch.randn(B, T, 3 * H * D, generator=g) * 0.8).to(dt)
    mask = None
    if masked:
        lens = torch.randint(T // 2, T + 1, (B,), generator=g)
        mask = (torch.arange(T).reshape(1, T) < lens.reshape(B, 1)).float()
    dout = torch.randn(B, T, H * D, generator=g).to(dt)
    # reference (fp32 autograd on the bf16-rounded inputs)
    qr = qkv.float().requires_grad_(True)
    o_ref = TN.attention_reference(qr, H, mask, causal)
    o_ref.backward(dout.float())
    qd = qkv.to(cuda)
    md = mask.to(cuda) if mask is not None else None
    out, lse = TN.attn_fwd(qd, H, md, causal)
    assert out.dtype == dt
    keep = torch.ones(B, T, 1)
    assert _err(out.cpu() * keep, o_ref.detach() * keep) < 2e-2
    dqkv = TN.attn_bwd(qd, out, lse, dout.to(cuda), H, md, causal)
    E = H * D
    for name, sl in (("dQ", slice(0, E)), ("dK", slice(E, 2 * E)), ("dV", slice(2 * E, 3 * E))):
        e = _err(dqkv[..., sl].cpu(), qr.grad[..., sl])
        assert e < 3e-2, (name, e)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2), (torch.float16, 4e-3)])
@pytest.mark.parametrize("M,N", [(5, 64), (1000, 768), (37, 1032), (64, 4096), (4096, 768), (5000, 768)])
@pytest.mark.parametrize("res", [False, True])
def test_layernorm_fwd_bwd_matches_reference(cuda, dtype, tol, M, N, res):
    g = torch.Generator().manual_seed(M + N)
    x = (torch.randn(M, N, generator=g) * 2 + 0.5).to(dtype)
    r = torch.randn(M, N, generator=g).to(dtype) if res else None
    gamma = torch.rand(N, generator=g) + 0.5
    beta = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g).to(dtype)
    xr = x.float().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    s = xr + rr if res else xr
    y_ref = torch.nn.functional.layer_norm(s, (N,), gr, br, 1e-12)
    y_ref.backward(dy.float())
    y, mean, rstd = TN.ln_fwd(x.to(cuda), gamma.to(cuda), beta.to(cuda), 1e-12, r.to(cuda) if res else None)
    assert _err(y, y_ref.detach()) < tol * 4
    dx, dg, db = TN.ln_bwd(dy.to(cuda), x.to(cuda), gamma.to(cuda), mean, rstd, r.to(cuda) if res else None)
    assert _err(dx, xr.grad) < tol * 8
    if res:
        assert _err(dx, rr.grad) < tol * 8
    assert _err(dg, gr.grad) < tol * 8 * (1 if dtype == torch.float32 else 4)
    assert _err(db, br.grad) < tol * 8 * (1 if dtype == torch.float32 else 4)
    # the dx column sums (the producing dense layer's bias gradient) from the same launch
    dsum = torch.full((N,), float("nan"), device=cuda)
    dx2, _, _ = TN.ln_bwd(dy.to(cuda), x.to(cuda), gamma.to(cuda), mean, rstd, r.to(cuda) if res else None,
                          dsum_out=dsum)
    assert _err(dx2, dx) < 1e-5   # the two template instances may contract FMAs differently
    assert _err(dsum, dx.float().sum(0)) < 1e-4


def test_bert_block_gpu_bf16_matches_cpu_fp32(cuda):
    """Encoder stack on the GPU (bf16 + flash-attention / LayerNorm kernels) vs the same weights on the CPU fp32
    reference path: outputs and parameter gradients."""
    from deeplearning4j_amd.models import BertBase
    from deeplearning4j_amd.nn.conf import DataType
    kw = dict(numLabels=3, inputShape=[40], vocabSize=97, hidden=128, layers=2, heads=2, ffn=256, maxPositions=64)
    ref = BertBase(**kw).init(device="cpu")
    gpu = BertBase(dataType=DataType.BFLOAT16, **kw).init(device=cuda)
    gpu.setParams(ref.params().to(cuda))
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 97, (6, 40), generator=g)
    y = torch.nn.functional.one_hot(torch.randint(0, 3, (6,), generator=g), 3).float()
    m = torch.ones(6, 40)
    m[2, 25:] = 0
    out_r = ref.output(x, masks=[m])[0]
    out_g = gpu.output(x.to(cuda), masks=[m.to(cuda)])[0]
    assert _err(out_g, out_r) < 3e-2
    ref.computeGradientAndScore([x], [y], [m])
    gpu.computeGradientAndScore([x.to(cuda)], [y.to(cuda)], [m.to(cuda)])
    gr, gg = ref.getGradientsViewArray().reshape(-1), gpu.getGradientsViewArray().reshape(-1).cpu()
    rel = (gg - gr).norm() / gr.norm()
    assert rel < 5e-2, rel


@pytest.mark.parametrize("dt,tol", [(torch.bfloat16, 2e-2), (torch.float16, 4e-3), (torch.float32, 1e-5)])
def test_gelu_and_softmax_xent_kernels_all_dtypes(cuda, dt, tol):
    from deeplearning4j_amd.ops import native
    g = torch.Generator().manual_seed(5)
    z = (torch.randn(4096, 24, generator=g) * 2).to(dt)
    dy = torch.randn(4096, 24, generator=g).to(dt)
    zr = z.float().requires_grad_(True)
    yr = torch.nn.functional.gelu(zr)
    yr.backward(dy.float())
    assert _err(TN.gelu(z.to(cuda)), yr.detach()) < tol
    assert _err(TN.gelu(z.to(cuda), dy.to(cuda)), zr.grad) < tol * 2
    logits = (torch.randn(64, 100, generator=g) * 3).to(dt)
    lab = torch.nn.functional.one_hot(torch.randint(0, 100, (64,), generator=g), 100).float()
    score, grad, _ = native.softmax_xent(logits.to(cuda), lab.to(cuda), 0.0)
    lr = logits.float().requires_grad_(True)
    ref = -(lab * torch.log_softmax(lr, 1)).sum(1)
    ref.sum().backward()
    assert _err(score, ref.detach()) < tol
    assert grad.dtype == dt and _err(grad, lr.grad) < tol * 2
    rows = torch.randn(1000, 64, generator=g).to(dt)
    assert _err(native.channel_sum(rows.to(cuda)), rows.float().sum(0)) < 1e-4


def test_bert_fp16_step_on_intree_kernels(cuda):
    """BASELINE config #5 precision: BERT (2 layers) trained in fp16 (fp32 masters, fp16 shadow written by the fused
    updater) runs every op on the in-tree kernels, and its loss decreases."""
    from deeplearning4j_amd.models import BertBase
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.ops import fallback
    net = BertBase(numLabels=2, inputShape=[64], layers=2, dataType=DataType.HALF).init(device=cuda)
    assert net.shadow is not None and net.shadow.dtype == torch.float16
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 30522, (8, 64), generator=g).to(cuda)
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (8,), generator=g), 2).float().to(cuda)
    fallback.reset()
    scores = []
    for _ in range(6):
        net.fit([x], [y])
        scores.append(net.score())
    torch.cuda.synchronize()
    assert net.helperCountFail() == 0, fallback.summary()
    assert all(s == s for s in scores) and scores[-1] < scores[0], scores
