"""Whole-sequence LSTM/GravesLSTM HIP kernels (csrc/lstm.hip) vs the per-step torch reference in fp64 on the CPU.

Same strategy as the reference's cuDNN LSTM validation (CUDAT:lstm/ValidateCudnnLSTM.java:32-246): the helper's
activations and gradients must match the built-in implementation."""
import pytest
import torch

from deeplearning4j_amd.nn.conf.activations import ActivationSigmoid, ActivationTanH
from deeplearning4j_amd.nn.layers import recurrent as R
from deeplearning4j_amd.ops import native

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    a, b = a.double().cpu(), b.double().cpu()
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert err <= tol * scale, f"max abs err {err} (scale {scale})"


def _params(nIn, H, peep, g):
    W = torch.randn(nIn, 4 * H, generator=g, dtype=torch.float64) * 0.3
    RW = torch.randn(H, 4 * H + (3 if peep else 0), generator=g, dtype=torch.float64) * 0.3 / (H ** 0.5) * 4
    b = torch.randn(4 * H, generator=g, dtype=torch.float64) * 0.2
    return W, RW, b


def _run(x, W, RW, b, h0, c0, H, peep, mask, eps, tbptt):
    act, gate = ActivationTanH(), ActivationSigmoid()
    out, (hT, cT), cache = R._lstm_fwd(x, W, RW, b, h0, c0, H, peep, act, gate, mask, True)
    grads = {"W": torch.zeros_like(W), "RW": torch.zeros_like(RW), "b": torch.zeros_like(b)}
    dx, _, _ = R._lstm_bwd(eps, cache, W, RW, H, peep, act, gate, mask, tbptt, "", grads)
    return out, hT, cT, dx, grads, cache


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 4e-2)])
@pytest.mark.parametrize("H", [32, 64, 256, 512])
@pytest.mark.parametrize("peep", [False, True])
def test_lstm_seq_kernels_match_reference(cuda, dtype, tol, H, peep):
    if dtype == torch.float32 and H == 512:
        pytest.skip("covered by bf16")
    g = torch.Generator().manual_seed(H + peep)
    mb, nIn, T = 37, 24, 11                                      # mb not a multiple of 16: masked tail rows
    W, RW, b = _params(nIn, H, peep, g)
    x = torch.randn(mb, nIn, T, generator=g, dtype=torch.float64)
    h0 = torch.randn(mb, H, generator=g, dtype=torch.float64) * 0.5
    c0 = torch.randn(mb, H, generator=g, dtype=torch.float64) * 0.5
    mask = (torch.rand(mb, T, generator=g) > 0.2).double()
    eps = torch.randn(mb, H, T, generator=g, dtype=torch.float64)
    # reference: fp64 per-step path on the CPU, with weights rounded like the device copy
    Wd, RWd, bd = (t.to(dtype) for t in (W, RW, b))
    ref = _run(x, Wd.double(), RWd.double(), bd.double(), h0, c0, H, peep, mask, eps, 6)
    dev = [t.to(cuda) for t in (x.float(), Wd, RWd, bd, h0.float(), c0.float(), mask.float(), eps.float())]
    got = _run(dev[0], dev[1], dev[2], dev[3], dev[4], dev[5], H, peep, dev[6], dev[7], 6)
    assert got[5].get("native"), "the HIP sequence kernel did not run"
    _close(got[0], ref[0], tol)                                  # h for all t
    _close(got[1], ref[1], tol)
    _close(got[2], ref[2], tol)
    _close(got[3], ref[3], tol * 4)                              # dx
    for k in ("W", "RW", "b"):
        _close(got[4][k], ref[4][k], tol * 8)


def test_lstm_native_in_network_fit(cuda):
    """GravesLSTM char-model fit on the GPU goes through the sequence kernels and the score decreases."""
    from deeplearning4j_amd.models import TextGenerationLSTM
    net = TextGenerationLSTM(numLabels=32, inputShape=[1, 32], seed=3).init(device=cuda)
    g = torch.Generator().manual_seed(0)
    idx = torch.randint(0, 32, (8, 40), generator=g)
    x = torch.nn.functional.one_hot(idx, 32).permute(0, 2, 1).float()
    y = torch.nn.functional.one_hot(torch.roll(idx, -1, 1), 32).permute(0, 2, 1).float()
    lib = native.load()
    assert hasattr(lib, "dl4j_lstm_fwd")
    scores = []
    for _ in range(15):
        net.fit(x.to(cuda), y.to(cuda))
        scores.append(net.score())
    assert scores[-1] < scores[0]


@pytest.mark.parametrize("peep", [False, True])
def test_samediff_lstm_layer_gpu_matches_cpu(cuda, peep):
    """SameDiff lstmLayer: the GPU path (sequence kernels in both directions of SameDiff's own reverse pass) vs the
    CPU reference, values and grads."""
    from deeplearning4j_amd.samediff import SameDiff
    g = torch.Generator().manual_seed(5)
    mb, nIn, T, H = 19, 12, 9, 64
    base = {"x": torch.randn(mb, nIn, T, generator=g), "W": torch.randn(nIn, 4 * H, generator=g) * 0.3,
            "RW": torch.randn(H, 4 * H + (3 if peep else 0), generator=g) * 0.1, "b": torch.randn(4 * H, generator=g) * 0.1}
    res = {}
    for dev in ("cpu", cuda):
        sd = SameDiff.create()
        vs = {k: sd.var(k, v.clone().to(dev)) for k, v in base.items()}
        h = sd.rnn().lstmLayer("h", vs["x"], vs["W"], vs["RW"], vs["b"], peephole=peep)
        loss = (h * sd.constant("ramp", torch.linspace(-1, 1, T, device=h.value.device))).sum()
        grads = sd.execBackwards(loss, list(vs.values()))
        res[str(dev)] = (h.value.detach().cpu(), {k: v.cpu() for k, v in grads.items()})
    (hc, gc), (hg, gg) = res["cpu"], res[str(cuda)]
    _close(hg, hc, 1e-4)
    for k in base:
        _close(gg[k], gc[k], 1e-3)


@pytest.mark.parametrize("H,mb,peep", [(256, 32, True), (256, 37, False), (512, 20, True)])
def test_lstm_coop_kernel_matches_single_workgroup_kernel(cuda, monkeypatch, H, mb, peep):
    """Cooperative multi-workgroup forward (RW resident in LDS, granule hand-offs) == the single-workgroup kernel."""
    from deeplearning4j_amd.ops import rnn_native
    g = torch.Generator().manual_seed(H + mb)
    T = 23
    zx = (torch.randn(T, mb, 4 * H, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    RW = (torch.randn(H, 4 * H + (3 if peep else 0), generator=g) * (2.0 / H ** 0.5)).to(torch.bfloat16).to(cuda)
    h0 = torch.randn(mb, H, generator=g).to(cuda) * 0.3
    c0 = torch.randn(mb, H, generator=g).to(cuda) * 0.3
    mask = (torch.rand(mb, T, generator=g) > 0.1).float().to(cuda)
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DL4J_AMD_LSTM_COOP", flag)
        rnn_native.last_coop_err = None
        # cooperative run: weights packed by the one-launch pack kernel, bf16 copy of h written by the kernel
        packs = rnn_native.pack_rw(RW, H, peep) if flag == "1" else None
        res[flag] = rnn_native.lstm_seq_fwd(zx, RW, H, peep, h0, c0, mask, True, packs=packs, out16=flag == "1")
        if flag == "1":
            assert rnn_native.last_coop_err is not None, "cooperative kernel did not run"
            assert int(rnn_native.last_coop_err.item()) == 0, "hand-off wait timed out"
    for a, b in zip(res["1"][:5], res["0"][:5]):
        _close(a, b, 1e-5)
    assert res["0"][5] is None
    assert torch.equal(res["1"][5], res["1"][0].to(torch.bfloat16))


@pytest.mark.parametrize("H,mb,peep,t_end", [(256, 32, True, 0), (256, 37, False, 5), (512, 20, True, 0)])
def test_lstm_coop_bwd_matches_single_workgroup_kernel(cuda, monkeypatch, H, mb, peep, t_end):
    """Cooperative backward (K-split partial dh exchange) == the single-workgroup backward kernel, incl. TBPTT
    truncation (t_end), carried dh/dc and masks. Partial sums are fp32 (the single-WG kernel rounds nothing else
    differently), so only the summation order differs."""
    from deeplearning4j_amd.ops import rnn_native
    g = torch.Generator().manual_seed(H + mb + t_end)
    T = 19
    zx = (torch.randn(T, mb, 4 * H, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    RW = (torch.randn(H, 4 * H + (3 if peep else 0), generator=g) * (2.0 / H ** 0.5)).to(torch.bfloat16).to(cuda)
    c0 = torch.randn(mb, H, generator=g).to(cuda) * 0.3
    mask = (torch.rand(mb, T, generator=g) > 0.1).float().to(cuda)
    monkeypatch.setenv("DL4J_AMD_LSTM_COOP", "0")
    _, _, _, gates, call, _ = rnn_native.lstm_seq_fwd(zx, RW, H, peep, None, c0, mask, True)
    eps = torch.randn(T, mb, H, generator=g).to(cuda)
    dhl = torch.randn(mb, H, generator=g).to(cuda) * 0.2
    dcl = torch.randn(mb, H, generator=g).to(cuda) * 0.2
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DL4J_AMD_LSTM_COOP", flag)
        rnn_native.last_coop_bwd_err = None
        # cooperative run: packed weights from the pack kernel and bf16 eps read directly by the kernel
        packs = rnn_native.pack_rw(RW, H, peep) if flag == "1" else None
        e = eps.to(torch.bfloat16) if flag == "1" else eps.to(torch.bfloat16).float()
        res[flag] = rnn_native.lstm_seq_bwd(e, gates, call, c0, RW, H, peep, mask, dhl, dcl, t_end, packs=packs)
        if flag == "1":
            assert rnn_native.last_coop_bwd_err is not None, "cooperative backward did not run"
            assert int(rnn_native.last_coop_bwd_err.item()) == 0, "hand-off wait timed out"
    for a, b in zip(res["1"], res["0"]):
        _close(a, b, 2e-3)


def test_samediff_char_lm_trains_on_gpu(cuda):
    """The SameDiff char-LM of tools/bench_samediff_lstm.py: bf16 with fp32 masters, sequence kernels in both passes,
    loss decreases when fitting one window repeatedly."""
    import sys as _sys
    import os as _os
    _sys.path.insert(0, _os.path.join(_os.path.dirname(__file__), "..", "tools"))
    import bench_samediff_lstm as B
    from deeplearning4j_amd import DataSet
    sd = B.build(cuda, 8, 20, 77, 256)
    g = torch.Generator().manual_seed(3)
    idx = torch.randint(0, 77, (8, 21), generator=g)
    X = torch.nn.functional.one_hot(idx[:, :-1], 77).permute(0, 2, 1).to(torch.bfloat16).to(cuda)
    Y = torch.nn.functional.one_hot(idx[:, 1:], 77).to(torch.bfloat16).to(cuda)
    losses = [sd.fit(DataSet(X, Y)) for _ in range(40)]
    assert losses[-1] < 0.7 * losses[0], losses[::10]
    assert sd._train_state["shadow"] is not None            # mixed precision: bf16 compute copy of fp32 masters


@pytest.mark.parametrize("dtype,H", [(torch.bfloat16, 256), (torch.float16, 64), (torch.float32, 48)])
@pytest.mark.parametrize("forder", [False, True])
def test_lstm_pack_rw_matches_permute_pack(cuda, dtype, H, forder):
    """One-launch packing kernel == the permute/contiguous packing of rnn_native._pack_b (both images + peepholes),
    for row-major and DL4J 'f'-ordered weight views."""
    from deeplearning4j_amd.ops import rnn_native
    g = torch.Generator().manual_seed(H)
    RW = torch.randn(H, 4 * H + 3, generator=g).to(dtype).to(cuda)
    if forder:
        RW = RW.t().contiguous().t()
    p = rnn_native.pack_rw(RW, H, True)
    assert p is not None
    assert torch.equal(p.fwd, rnn_native._pack_b(RW[:, :4 * H].t(), dtype))
    assert torch.equal(p.bwd, rnn_native._pack_b(RW[:, :4 * H], dtype))
    assert torch.equal(p.peep, RW[:, 4 * H:].t().float())
