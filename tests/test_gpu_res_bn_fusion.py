"""Shortcut-BatchNorm folding (csrc/batchnorm.hip RBN kernels, nn/graph planner): in a ResNet convBlock
(conv -> BN -> add <- BN <- conv -> ReLU) the shortcut BN only folds its statistics and the residual BN applies both
normalisations in one pass, and its backward computes both layers' gradients from one partial-sum pass. Checked
(1) in isolation against fp32 autograd of relu(bn(x) + bn_r(xr)) — outputs, both inputs' gradients, both layers'
gamma / beta gradients and running statistics — and (2) on the zoo ResNet-50 (bf16, one Sgd step): the fused network
is as close to an fp32 reference step as the unfused bf16 network (DL4J_AMD_FUSE_RES_BN=0) is, and the fusion really
ran (4 shortcut BN layers deferred)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net(fuse, monkeypatch, dtype="BFLOAT16"):
    from deeplearning4j_amd import Sgd, WeightInit
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    monkeypatch.setenv("DL4J_AMD_FUSE_RES_BN", "1" if fuse else "0")
    torch.manual_seed(3)
    return ResNet50(numLabels=100, dataType=getattr(DataType, dtype), updater=Sgd(0.01), weightInit=WeightInit.RELU,
                    inputShape=[3, 224, 224]).init(torch.device("cuda", 0))


@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (4, 256, 7, 7), (2, 512, 28, 28)])
def test_rbn_kernels_match_fp32(shape):
    """The RBN pair in isolation: stats-only shortcut BN + relu(bn(x) + bn_r(xr)) forward, and the one-pass backward
    (dx, d(xr), both layers' dgamma / dbeta), against fp32 autograd of the same composition on the bf16 inputs."""
    from deeplearning4j_amd.ops.norm import bn_backward, bn_forward
    N, C, H, W = shape
    g = torch.Generator(device="cpu").manual_seed(sum(shape))
    mk = lambda *s, sc=1.0, off=0.0: (torch.randn(*s, generator=g) * sc + off)  # noqa: E731
    x = mk(N, C, H, W, sc=2.0, off=0.5).cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = mk(N, C, H, W, sc=0.7, off=-0.3).cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = mk(N, C, H, W).cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g1, b1, g2, b2 = (mk(C, sc=0.3, off=o).cuda() for o in (1.0, 0.1, 0.8, -0.1))
    rm1, rv1, rm2, rv2 = (torch.full((C,), v, device="cuda") for v in (0.0, 1.0, 0.0, 1.0))
    decay, eps = 0.9, 1e-5
    r = bn_forward(xr, g2, b2, rm2, rv2, True, decay, eps, stats_only=True)
    assert r is not None and r[1][0] == "NATIVE_STATS"
    y, ctx = bn_forward(x, g1, b1, rm1, rv1, True, decay, eps, relu=True, residual=xr, rctx=r[1][2])
    dg2 = torch.empty(C, device="cuda")
    db2 = torch.empty(C, device="cuda")
    dx, dg1, db1, dxr = bn_backward(dy, ctx, rgrads=(dg2, db2))
    torch.cuda.synchronize()

    xf, xrf = x.float().requires_grad_(), xr.float().requires_grad_()
    pg1, pb1, pg2, pb2 = (t.clone().requires_grad_() for t in (g1, b1, g2, b2))

    def bn(t, gg, bb):
        m = t.mean(dim=(0, 2, 3), keepdim=True)
        v = t.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
        return (t - m) * torch.rsqrt(v + eps) * gg.reshape(1, -1, 1, 1) + bb.reshape(1, -1, 1, 1), m, v

    a, m1, v1 = bn(xf, pg1, pb1)
    b, m2, v2 = bn(xrf, pg2, pb2)
    yr = torch.relu(a + b)
    yr.backward(dy.float())
    close = lambda got, ref, tol: float((got.float() - ref).norm() / ref.norm().clamp_min(1e-12)) < tol  # noqa: E731
    assert close(y, yr.detach(), 8e-3)
    assert close(dx, xf.grad, 2e-2) and close(dxr, xrf.grad, 2e-2)
    for got, ref in ((dg1, pg1.grad), (db1, pb1.grad), (dg2, pg2.grad), (db2, pb2.grad)):
        assert close(got, ref, 5e-3), (got[:4], ref[:4])
    for rm, rv, m, v in ((rm1, rv1, m1, v1), (rm2, rv2, m2, v2)):
        assert torch.allclose(rm, (1 - decay) * m.detach().reshape(-1), rtol=1e-3, atol=1e-4)
        assert torch.allclose(rv, decay + (1 - decay) * (v.detach().reshape(-1) + eps), rtol=1e-3, atol=1e-4)


def test_shortcut_bn_folding_matches_unfused(monkeypatch):
    """Whole-network check against an fp32 reference of the same step: a random-init ResNet-50 amplifies bf16
    rounding (the fused pass rounds once where the unfused pair rounds the shortcut BN output first), so the fused
    network must be as close to fp32 as the unfused bf16 network is, not bitwise equal to it."""
    fused = _net(True, monkeypatch)
    plain = _net(False, monkeypatch)
    ref = _net(False, monkeypatch, "FLOAT")
    plain.setParams(fused.params().detach().clone())
    ref.setParams(fused.params().detach().clone())
    deferred = [n for n, l in fused.layers_by_name.items() if getattr(l, "defer_apply", False)]
    assert len(deferred) == 4, deferred
    assert not any(getattr(l, "defer_apply", False) for l in plain.layers_by_name.values())
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.rand(16, 3, 224, 224, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.zeros(16, 100, device="cuda")
    y[torch.arange(16), torch.randint(0, 100, (16,), generator=g).cuda()] = 1.0
    p0 = fused.params().detach().clone()
    fused.fit([x], [y])
    ran = [n for n in deferred if fused.layers_by_name[n]._ctx[0] == "NATIVE_STATS"]
    assert ran == deferred
    plain.fit([x], [y])
    ref.fit([x.float()], [y])
    torch.cuda.synchronize()
    s_f, s_p, s_r = fused.score(), plain.score(), ref.score()
    d_f, d_p, d_r = ((n.params() - p0).double().reshape(-1) for n in (fused, plain, ref))
    cos = lambda a, b: float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))  # noqa: E731
    print(f"score fused {s_f:.5f} plain {s_p:.5f} fp32 {s_r:.5f}; update cos vs fp32: fused {cos(d_f, d_r):.5f} "
          f"plain {cos(d_p, d_r):.5f}; fused vs plain {cos(d_f, d_p):.5f}")
    assert abs(s_f - s_r) <= max(2.0 * abs(s_p - s_r), 2e-3 * abs(s_r)), (s_f, s_p, s_r)
    assert cos(d_f, d_r) > min(0.995, cos(d_p, d_r) - 0.01), (cos(d_f, d_r), cos(d_p, d_r))
    for _, name, impl, off in fused._layer_offsets:
        n = sum(spec.numel for spec in impl.conf.param_specs())
        if n and name in deferred:
            sl = slice(off, off + n)                       # shortcut BN: gamma / beta gradients + running stats
            cf, cp = cos(d_f[sl], d_r[sl]), cos(d_p[sl], d_r[sl])
            print(f"  {name}: cos vs fp32 fused {cf:.5f} plain {cp:.5f}")
            assert cf > min(0.99, cp - 0.02), (name, cf, cp)
