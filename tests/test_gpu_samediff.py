"""SameDiff on the GPU: graphs of transformer / CNN ops run their HIP kernels in both directions of SameDiff's own
reverse pass (GEMM, flash attention, LayerNorm, conv, pooling, softmax-xent) with no helper fallback; gradients in
bf16 match the fp64 CPU evaluation of the same recorded graph."""
import pytest
import torch

from deeplearning4j_amd.ops import fallback
from deeplearning4j_amd.samediff import SameDiff

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _transformer_block(dev, dt, base):
    sd = SameDiff.create()
    x = sd.placeHolder("x", base["x"].to(dev, dt))
    y = sd.placeHolder("y", base["y"].to(dev, dt))
    v = {k: sd.var(k, base[k].to(dev, dt)) for k in ("wqkv", "bqkv", "wo", "bo", "g", "b", "wf", "bf", "wc")}
    qkv = sd.nn().linear(x, v["wqkv"], v["bqkv"])
    a = sd.nn().fusedSelfAttention(qkv, 2)
    h = sd.nn().linear(a, v["wo"], v["bo"]).add(x)
    h = sd.nn().layerNorm(h, v["g"], v["b"])
    h = sd.nn().gelu(sd.nn().linear(h, v["wf"], v["bf"]))        # fused: GELU in the GEMM epilogue
    logits = h.get(slice(None), 0).mmul(v["wc"])
    loss = sd.loss().softmaxCrossEntropy("loss", y, logits)
    return sd, loss


def test_samediff_transformer_block_bf16_gpu_matches_fp64(cuda):
    g = torch.Generator().manual_seed(0)
    B, T, E, C = 4, 64, 128, 8
    base = {"x": torch.randn(B, T, E, generator=g), "wqkv": torch.randn(E, 3 * E, generator=g) * E ** -0.5,
            "bqkv": torch.randn(3 * E, generator=g) * 0.02, "wo": torch.randn(E, E, generator=g) * E ** -0.5,
            "bo": torch.zeros(E), "g": 1 + 0.1 * torch.randn(E, generator=g), "b": 0.1 * torch.randn(E, generator=g),
            "wc": torch.randn(E, C, generator=g) * E ** -0.5, "wf": torch.randn(E, E, generator=g) * E ** -0.5,
            "bf": 0.02 * torch.randn(E, generator=g),
            "y": torch.nn.functional.one_hot(torch.randint(0, C, (B,), generator=g), C).float()}
    fallback.reset()
    sd, loss = _transformer_block(cuda, torch.bfloat16, base)
    ops = [r[1] for r in sd._plan([loss.name])]
    assert "gelu" not in ops and "add" not in ops, ops
    gg = sd.execBackwards(loss)
    torch.cuda.synchronize()
    assert fallback.count() == 0, fallback.summary()
    sd64, loss64 = _transformer_block("cpu", torch.float64, base)
    g64 = sd64.execBackwards(loss64)
    assert abs(float(loss.value) - float(loss64.value)) < 2e-2 * abs(float(loss64.value))
    for k in g64:
        assert _rel(gg[k], g64[k]) < 6e-2, (k, _rel(gg[k], g64[k]))


def _cnn(dev, dt, base):
    sd = SameDiff.create()
    x = sd.placeHolder("x", base["x"].to(dev, dt).contiguous(memory_format=torch.channels_last))
    y = sd.placeHolder("y", base["y"].to(dev, dt))
    w = sd.var("w", base["w"].to(dev, dt))
    b = sd.var("b", base["b"].to(dev, dt))
    wd = sd.var("wd", base["wd"].to(dev, dt))
    h = sd.nn().relu(sd.cnn().conv2d(x, w, b, stride=(1, 1), padding=(1, 1)))
    h = sd.cnn().maxPooling2d(None, h, (2, 2), (2, 2))
    h = h.reshape(base["x"].shape[0], -1)
    loss = sd.loss().softmaxCrossEntropy("loss", y, h.mmul(wd))
    return sd, loss


def test_samediff_cnn_bf16_gpu_matches_fp64(cuda):
    g = torch.Generator().manual_seed(1)
    N, C, Hh, K, cls = 8, 16, 16, 32, 10
    base = {"x": torch.randn(N, C, Hh, Hh, generator=g), "w": torch.randn(K, C, 3, 3, generator=g) * (C * 9) ** -0.5,
            "b": 0.05 * torch.randn(K, generator=g),
            "wd": torch.randn(K * (Hh // 2) ** 2, cls, generator=g) * (K * (Hh // 2) ** 2) ** -0.5,
            "y": torch.nn.functional.one_hot(torch.randint(0, cls, (N,), generator=g), cls).float()}
    fallback.reset()
    sd, loss = _cnn(cuda, torch.bfloat16, base)
    gg = sd.execBackwards(loss)
    torch.cuda.synchronize()
    assert fallback.count() == 0, fallback.summary()
    sd64, loss64 = _cnn("cpu", torch.float64, base)
    g64 = sd64.execBackwards(loss64)
    for k in g64:
        assert _rel(gg[k], g64[k]) < 1e-1, (k, _rel(gg[k], g64[k]))


def test_samediff_fit_hip_graph_matches_eager(cuda):
    """sd.enableHipGraphs(): the captured step (every op's forward + explicit backward, gradient copy, fused Adam with
    its iteration-dependent bias correction through the A/B graph tables) gives the same parameters as eager fits."""
    from deeplearning4j_amd import Adam, DataSet
    from deeplearning4j_amd.samediff import TrainingConfig
    g = torch.Generator().manual_seed(0)
    B, T, E, C = 4, 64, 128, 8
    base = {"x": torch.randn(B, T, E, generator=g), "wqkv": torch.randn(E, 3 * E, generator=g) * E ** -0.5,
            "bqkv": torch.randn(3 * E, generator=g) * 0.02, "wo": torch.randn(E, E, generator=g) * E ** -0.5,
            "bo": torch.zeros(E), "g": 1 + 0.1 * torch.randn(E, generator=g), "b": 0.1 * torch.randn(E, generator=g),
            "wc": torch.randn(E, C, generator=g) * E ** -0.5, "wf": torch.randn(E, E, generator=g) * E ** -0.5,
            "bf": 0.02 * torch.randn(E, generator=g),
            "y": torch.nn.functional.one_hot(torch.randint(0, C, (B,), generator=g), C).float()}
    data = [DataSet(torch.randn(B, T, E, generator=g).to(cuda, torch.bfloat16),
                    torch.nn.functional.one_hot(torch.randint(0, C, (B,), generator=g), C).to(cuda, torch.bfloat16))
            for _ in range(6)]
    res = []
    for graphs in (False, True):
        sd, loss = _transformer_block(cuda, torch.bfloat16, base)
        sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(1e-3)).dataSetFeatureMapping("x")
                             .dataSetLabelMapping("y").build())
        if graphs:
            sd.enableHipGraphs(True, warmup=2)
        losses = [sd.fit(ds) for ds in data]
        torch.cuda.synchronize()
        if graphs:
            assert sd._graph is not None and sd._graph["ok"] and sd._graph["k"] == 4
        res.append((losses, torch.cat([sd._train_state["flat"]])))
    (l0, p0), (l1, p1) = res
    assert all(abs(a - b) < 1e-3 * max(1.0, abs(a)) for a, b in zip(l0, l1)), (l0, l1)
    assert torch.allclose(p0, p1, atol=1e-4), (p0 - p1).abs().max()


def test_samediff_gradient_sinks_and_master_views(cuda, monkeypatch):
    """Training writes single-reader gradients straight into the flat gradient buffer (GEMM fp32 epilogue,
    channel-sum, LayerNorm and embedding kernels) and reads GEMM biases / LayerNorm affine parameters from the fp32
    master copy: same parameters as the copy-through path."""
    from deeplearning4j_amd import Adam, DataSet
    from deeplearning4j_amd.samediff import TrainingConfig
    g = torch.Generator().manual_seed(2)
    B, T, E, C = 4, 64, 128, 8
    base = {"x": torch.randn(B, T, E, generator=g), "wqkv": torch.randn(E, 3 * E, generator=g) * E ** -0.5,
            "bqkv": torch.randn(3 * E, generator=g) * 0.02, "wo": torch.randn(E, E, generator=g) * E ** -0.5,
            "bo": torch.zeros(E), "g": 1 + 0.1 * torch.randn(E, generator=g), "b": 0.1 * torch.randn(E, generator=g),
            "wc": torch.randn(E, C, generator=g) * E ** -0.5, "wf": torch.randn(E, E, generator=g) * E ** -0.5,
            "bf": 0.02 * torch.randn(E, generator=g),
            "y": torch.nn.functional.one_hot(torch.randint(0, C, (B,), generator=g), C).float()}
    data = [DataSet(torch.randn(B, T, E, generator=g).to(cuda, torch.bfloat16),
                    torch.nn.functional.one_hot(torch.randint(0, C, (B,), generator=g), C).to(cuda, torch.bfloat16))
            for _ in range(3)]
    res = []
    for sinks in ("0", "1"):
        monkeypatch.setenv("DL4J_AMD_SD_SINKS", sinks)
        sd, loss = _transformer_block(cuda, torch.bfloat16, base)
        sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(1e-3)).dataSetFeatureMapping("x")
                             .dataSetLabelMapping("y").build())
        losses = [sd.fit(data[0])]
        torch.cuda.synchronize()
        st = sd._train_state
        g1 = st["grad"].clone()                       # first step: same parameters on both paths
        losses += [sd.fit(ds) for ds in data[1:]]
        torch.cuda.synchronize()
        inplace = {v.name for v, view in zip(sd.trainableVariables(), st["views"])
                   if sd._last_grads.get(v.name) is not None and sd._last_grads[v.name].data_ptr() == view.data_ptr()}
        if sinks == "1":
            assert {"wqkv", "bqkv", "wo", "bo", "g", "b", "wf", "bf"} <= inplace, inplace
            # "wo -> add -> layerNorm": the bias gradient of the out projection comes from the LayerNorm kernel
            assert sd._ln_bias_fusions(sd._plan([loss.name]), {"bo": None}), "LN dsum fusion not planned"
        else:
            assert not inplace
        assert sd.variables["bqkv"].value._dl4j_master.dtype == torch.float32
        res.append((losses, g1, st["flat"].clone()))
    (l0, g0, p0), (l1, g1, p1) = res
    assert all(abs(a - b) < 1e-2 * max(1.0, abs(a)) for a, b in zip(l0, l1)), (l0, l1)
    assert _rel(g1, g0) < 1e-2, _rel(g1, g0)          # bias sums from fp32 (LN kernel) vs bf16 (channel sum) rows
    assert torch.allclose(p0, p1, atol=5e-3), (p0 - p1).abs().max()


def test_samediff_residual_gradient_accumulated_in_gemm(cuda, monkeypatch):
    """A variable read by a linear op and by a residual add: with the reverse pass summing the linear's input gradient
    into the residual branch's partial gradient inside the GEMM (beta = 1), the gradients equal the unfused pass
    (separate add) and the fp64 CPU reference."""
    import deeplearning4j_amd.samediff as S
    g = torch.Generator().manual_seed(5)
    B, T, E = 2, 64, 128
    base = {"x": torch.randn(B, T, E, generator=g), "w0": torch.randn(E, E, generator=g) * E ** -0.5,
            "b0": 0.02 * torch.randn(E, generator=g), "wqkv": torch.randn(E, 3 * E, generator=g) * E ** -0.5,
            "bqkv": 0.02 * torch.randn(3 * E, generator=g), "wo": torch.randn(E, E, generator=g) * E ** -0.5,
            "bo": torch.zeros(E), "lg": 1 + 0.1 * torch.randn(E, generator=g), "lb": 0.1 * torch.randn(E, generator=g)}

    def run(dev, dt, fuse):
        monkeypatch.setattr(S, "_ACC_FUSE", fuse)
        sd = SameDiff.create()
        x = sd.placeHolder("x", base["x"].to(dev, dt))
        v = {k: sd.var(k, base[k].to(dev, dt)) for k in base if k != "x"}
        h0 = sd.nn().linear(x, v["w0"], v["b0"])
        qkv = sd.nn().linear(h0, v["wqkv"], v["bqkv"])
        a = sd.nn().fusedSelfAttention(qkv, 2)
        h = sd.nn().layerNorm(sd.nn().linear(a, v["wo"], v["bo"]).add(h0), v["lg"], v["lb"])
        sd.setLossVariables(h.mul(h).sum())
        names = [k for k in base if k != "x"]
        grads = sd.calculateGradients({}, *names)
        return {k: grads[k].float().cpu() for k in names}
    on = run(cuda, torch.float32, True)
    off = run(cuda, torch.float32, False)
    ref = run(torch.device("cpu"), torch.float64, True)
    for k in on:
        assert _rel(on[k], off[k]) < 1e-5, (k, _rel(on[k], off[k]))
        assert _rel(on[k], ref[k]) < 1e-3, (k, _rel(on[k], ref[k]))
