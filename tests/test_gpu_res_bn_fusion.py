"""Shortcut-BatchNorm folding (csrc/batchnorm.hip RBN kernels, nn/graph planner): in a ResNet convBlock
(conv -> BN -> add <- BN <- conv -> ReLU) the shortcut BN only folds its statistics and the residual BN applies both
normalisations in one pass, and its backward computes both layers' gradients from one partial-sum pass. Checked
against the unfused network (DL4J_AMD_FUSE_RES_BN=0) on the zoo ResNet-50 (bf16, one Sgd step on a non-saturated
init): scores, parameter updates per layer (the shortcut BN's gamma / beta included) and running statistics agree to
bf16 noise, and the fusion really ran (4 shortcut BN layers deferred)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net(fuse, monkeypatch):
    from deeplearning4j_amd import Sgd, WeightInit
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    monkeypatch.setenv("DL4J_AMD_FUSE_RES_BN", "1" if fuse else "0")
    torch.manual_seed(3)
    return ResNet50(numLabels=100, dataType=DataType.BFLOAT16, updater=Sgd(0.01), weightInit=WeightInit.RELU,
                    inputShape=[3, 224, 224]).init(torch.device("cuda", 0))


def test_shortcut_bn_folding_matches_unfused(monkeypatch):
    fused = _net(True, monkeypatch)
    plain = _net(False, monkeypatch)
    plain.setParams(fused.params().detach().clone())
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
    torch.cuda.synchronize()
    s_f, s_p = fused.score(), plain.score()
    assert abs(s_f - s_p) / abs(s_p) < 2e-3, (s_f, s_p)
    d_f = (fused.params() - p0).double().reshape(-1)
    d_p = (plain.params() - p0).double().reshape(-1)
    cos = float(torch.dot(d_f, d_p) / (d_f.norm() * d_p.norm()))
    assert cos > 0.995, cos
    for _, name, impl, off in fused._layer_offsets:
        n = sum(spec.numel for spec in impl.conf.param_specs())
        if n and name in deferred:
            a, b = d_f[off:off + n], d_p[off:off + n]
            c = float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))
            assert c > 0.99, (name, c)                      # shortcut BN: gamma / beta gradients + running stats
