"""GPU numerics of the in-tree MFMA GEMM (csrc/gemm.hip) against a plain fp32 torch reference.

Covers the four operand layouts (K- vs M/N-contiguous A and B, i.e. every transpose combination), bf16 / fp16 /
fp32 inputs, fp32 / bf16 outputs, bias (per column / per row), activations, beta-accumulate, column-major
('f'-order) destinations, 3-D batches, split-K, odd shapes (generic kernel) and the bench shapes of BERT-base,
the char-LSTM and the ResNet-50 classifier. Asymmetric random operands (guide §3: A=I with asymmetric B catches a
transposed C-write).
"""
import pytest
import torch

from deeplearning4j_amd.ops import fallback, gemm

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ref(a, b, bias=None, bias_dim=1, act=None, alpha=1.0, beta=0.0, c0=None):
    r = alpha * (a.float() @ b.float())
    if bias is not None:
        r = r + (bias.float().reshape(1, -1) if bias_dim == 1 else bias.float().reshape(-1, 1))
    if beta:
        r = r + beta * c0.float()
    return gemm._torch_act(r, act)


def _tol(dt, K):
    if dt == torch.float32:
        return 1e-4 * max(1.0, K ** 0.5)
    return (2e-2 if dt == torch.bfloat16 else 4e-3) * max(1.0, (K / 64) ** 0.5)


def _mk(shape, dt, contig_last=True):
    """Operand with the requested logical shape; contig_last=False gives the transposed-view layout."""
    if contig_last:
        return torch.randn(*shape, device=DEV).to(dt)
    return torch.randn(*shape[::-1], device=DEV).to(dt).t()


def _check(out, ref, dt, K, what=""):
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= _tol(dt, K) * scale, f"{what}: max err {err} vs scale {scale}"


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("a_kc", [True, False])
@pytest.mark.parametrize("b_kc", [True, False])
def test_layouts(dt, a_kc, b_kc):
    torch.manual_seed(0)
    M, N, K = 320, 264, 200
    a = _mk((M, K), dt, contig_last=a_kc)
    b = _mk((K, N), dt, contig_last=not b_kc)
    fallback.reset()
    out = gemm.mmul(a, b, out_dtype=torch.float32)
    _check(out, _ref(a, b), dt, K, f"layout a_kc={a_kc} b_kc={b_kc}")
    assert fallback.count() == 0


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(4096, 2304, 768), (4096, 768, 768), (4096, 3072, 768), (4096, 768, 3072),
                                   (768, 2304, 4096), (3072, 768, 4096), (512, 1000, 2048), (2048, 1000, 512),
                                   (4096, 1024, 256), (1024, 256, 4096), (8, 16, 64), (1, 8, 8)])
def test_bench_shapes(dt, shape):
    torch.manual_seed(1)
    M, N, K = shape
    a = torch.randn(M, K, device=DEV).to(dt)
    b = torch.randn(K, N, device=DEV).to(dt)
    out = gemm.mmul(a, b)
    _check(out, _ref(a, b), dt, K, f"shape {shape}")


@pytest.mark.parametrize("act", [None, "relu", "tanh", "sigmoid", "gelu"])
def test_epilogue_bias_act_z(act):
    torch.manual_seed(2)
    M, N, K = 777, 520, 256
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16() * 0.1
    bias = torch.randn(N, device=DEV)
    z = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    out = gemm.mmul(a, b, bias=bias, act=act, z=z)
    ref_z = _ref(a, b, bias)
    _check(z, ref_z, torch.bfloat16, K, "pre-activation")
    _check(out, gemm._torch_act(ref_z, act), torch.bfloat16, K, f"act {act}")


def test_row_bias_alpha_beta_fp32_out():
    torch.manual_seed(3)
    M, N, K = 512, 384, 1024
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16().t()
    c0 = torch.randn(M, N, device=DEV)
    bias = torch.randn(M, device=DEV)
    out = c0.clone()
    gemm.mmul(a, b, out=out, bias=bias, bias_dim=0, alpha=0.5, beta=1.0)
    _check(out, _ref(a, b, bias, 0, None, 0.5, 1.0, c0), torch.bfloat16, K, "alpha/beta/row-bias")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_column_major_destination(dt):
    """dW = x^T delta written straight into an 'f'-order [nIn, nOut] view (DL4J Dense gradient layout)."""
    torch.manual_seed(4)
    mb, nIn, nOut = 384, 200, 136
    x = torch.randn(mb, nIn, device=DEV).to(dt)
    d = torch.randn(mb, nOut, device=DEV).to(dt)
    flat = torch.zeros(nIn * nOut, device=DEV)
    view = flat.view(nOut, nIn).t()                     # column-major [nIn, nOut]
    gemm.mmul(x.t(), d, out=view)
    _check(view, _ref(x.t(), d), dt, mb, "column-major dW")


def test_batched():
    torch.manual_seed(5)
    a = torch.randn(6, 128, 64, device=DEV).bfloat16()
    b = torch.randn(6, 96, 64, device=DEV).bfloat16().transpose(1, 2)
    out = gemm.mmul(a, b, out_dtype=torch.float32)
    ref = torch.bmm(a.float(), b.float())
    _check(out, ref, torch.bfloat16, 64, "batched")


def test_split_k_deterministic():
    torch.manual_seed(6)
    a = torch.randn(256, 8192, device=DEV).bfloat16()
    b = torch.randn(8192, 256, device=DEV).bfloat16()
    o1 = gemm.mmul(a, b, out_dtype=torch.float32)
    o2 = gemm.mmul(a, b, out_dtype=torch.float32)
    assert torch.equal(o1, o2)
    _check(o1, _ref(a, b), torch.bfloat16, 8192, "split-K")


@pytest.mark.parametrize("case", ["fp32_dw", "bf16_bias_gelu", "ragged_beta", "dgelu"])
def test_split_k_in_kernel_fixup_matches_reduce(case, monkeypatch):
    """Split-K on the gemm_glds tiles: the tile's last-arriving block sums the slabs in split order inside the kernel
    (dl4j_gemm_set_splitk_fixup(1), opt-in) — bitwise equal to the separate reduce launch, and to the reference."""
    import ctypes
    from deeplearning4j_amd.ops import native
    lib = native.load()
    lib.dl4j_gemm_set_splitk_fixup.argtypes = [ctypes.c_int]
    torch.manual_seed(11)
    kw, z = {}, None
    if case == "fp32_dw":
        M, N, K, dt, cfg = 768, 3072, 4096, torch.float32, (3, 3)
    elif case == "bf16_bias_gelu":
        M, N, K, dt, cfg = 1000, 768, 3072, torch.bfloat16, (2, 4)
        kw = dict(bias=torch.randn(N, device=DEV), act="gelu")
    elif case == "ragged_beta":
        M, N, K, dt, cfg = 333, 250, 2048, torch.float32, (5, 3)
        kw = dict(beta=1.0)
    else:
        M, N, K, dt, cfg = 512, 1024, 1536, torch.bfloat16, (7, 2)
        z = torch.randn(M, N, device=DEV).bfloat16()
        kw = dict(act="dgelu", z=z)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(K, N, device=DEV).bfloat16() * 0.05
    c0 = torch.randn(M, N, device=DEV).to(dt)
    monkeypatch.setattr(gemm, "_FORCE_CFG", cfg)
    outs = []
    old = lib.dl4j_gemm_set_splitk_fixup(1)
    try:
        for mode in (1, 0):
            lib.dl4j_gemm_set_splitk_fixup(mode)
            out = c0.clone()
            gemm.mmul(a, b, out=out, **kw)
            outs.append(out)
        torch.cuda.synchronize()
    finally:
        lib.dl4j_gemm_set_splitk_fixup(old)
    assert torch.equal(outs[0], outs[1]), f"{case}: in-kernel fixup differs from the reduce kernel"
    r = a.float() @ b.float()
    if "bias" in kw:
        r = r + kw["bias"].reshape(1, -1)
    if kw.get("beta"):
        r = r + c0.float()
    if kw.get("act") == "gelu":
        r = torch.nn.functional.gelu(r)
    elif kw.get("act") == "dgelu":
        zf = z.float()
        r = r * (0.5 * (1 + torch.erf(zf / 2 ** 0.5)) + zf * torch.exp(-0.5 * zf * zf) / (2 * 3.141592653589793) ** 0.5)
    _check(outs[0], r, torch.bfloat16, K, case)


def test_identity_asymmetric():
    """A = I, asymmetric B: a transposed C-write would show."""
    n = 256
    eye = torch.eye(n, device=DEV).bfloat16()
    b = (torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) % 97).bfloat16()
    out = gemm.mmul(eye, b, out_dtype=torch.float32)
    assert torch.equal(out, b.float())


def test_odd_shapes_generic_kernel():
    torch.manual_seed(7)
    for (M, N, K) in [(3, 5, 7), (33, 17, 9), (130, 1, 70)]:
        a = torch.randn(M, K, device=DEV).bfloat16()
        b = torch.randn(K, N, device=DEV).bfloat16()
        _check(gemm.mmul(a, b, out_dtype=torch.float32), _ref(a, b), torch.bfloat16, K, f"odd {M},{N},{K}")


def test_graph_capture():
    torch.manual_seed(8)
    a = torch.randn(1024, 2048, device=DEV).bfloat16()
    b = torch.randn(2048, 512, device=DEV).bfloat16()
    out = torch.empty(1024, 512, device=DEV, dtype=torch.float32)
    gemm.mmul(a, b, out=out)                       # warm (allocates split-K workspace outside capture)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gemm.mmul(a, b, out=out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    _check(out, _ref(a, b), torch.bfloat16, 2048, "graph replay")


@pytest.mark.parametrize("cfg", [(0, 1), (1, 1), (2, 1), (3, 1), (4, 1), (4, 3), (2, 2), (5, 1), (8, 1), (9, 1),
                                 (3, 3), (7, 2)])
@pytest.mark.parametrize("a_kc", [True, False])
@pytest.mark.parametrize("b_kc", [True, False])
def test_every_tile_config(cfg, a_kc, b_kc, monkeypatch):
    """Each kernel configuration (incl. the 8-phase 256x256 one and split-K) on every layout, with M/N tails."""
    torch.manual_seed(9)
    M, N, K = 552, 328, 384
    a = _mk((M, K), torch.bfloat16, contig_last=a_kc)
    b = _mk((K, N), torch.bfloat16, contig_last=not b_kc)
    monkeypatch.setattr(gemm, "_FORCE_CFG", cfg)
    out = gemm.mmul(a, b, out_dtype=torch.float32)
    _check(out, _ref(a, b), torch.bfloat16, K, f"cfg {cfg} a_kc={a_kc} b_kc={b_kc}")


@pytest.mark.parametrize("cfg", [None, (0, 1), (1, 1), (2, 1), (3, 1), (4, 1), (5, 1), (8, 1), (9, 1)])
def test_bn_stats_epilogue(cfg, monkeypatch):
    """Per-64-row BatchNorm partial statistics from the GEMM epilogue (conv -> BN fusion) match the stored output."""
    torch.manual_seed(10)
    M, N, K = 1000, 192, 128
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16().t()
    bias = torch.randn(N, device=DEV)
    P = 2 * ((M + 127) // 128)
    ts = torch.full((3, P, N), float("nan"), device=DEV)
    monkeypatch.setattr(gemm, "_FORCE_CFG", cfg)
    out = gemm.mmul(a, b, bias=bias, stats=ts)
    y = out.float()
    for p in range(P):
        r0, r1 = p * 64, min(M, p * 64 + 64)
        if r1 <= r0:
            continue
        blk = y[r0:r1]
        sh = blk[0]
        assert torch.allclose(ts[2, p], sh, atol=0, rtol=0)
        assert torch.allclose(ts[0, p], (blk - sh).sum(0), atol=1e-2, rtol=1e-4)
        assert torch.allclose(ts[1, p], ((blk - sh) ** 2).sum(0), atol=1e-1, rtol=1e-4)


@pytest.mark.parametrize("shape", [(4096, 3072, 768), (300, 520, 256), (96, 64, 4096)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_dgelu_epilogue(shape, dt):
    """act="dgelu": out = (a @ b) * gelu'(z) with the pre-activation z READ in the epilogue (transformer FFN
    backward); z is left untouched. (96, 64, 4096) takes the split-K reduce epilogue."""
    torch.manual_seed(5)
    M, N, K = shape
    a = torch.randn(M, K, device=DEV).to(dt) * 0.1
    b = torch.randn(K, N, device=DEV).to(dt) * 0.1
    z = (torch.randn(M, N, device=DEV) * 2).to(dt)
    z0 = z.clone()
    out = gemm.mmul(a, b, act="dgelu", z=z)
    ref = (a.float() @ b.float()) * gemm._dgelu_ref(z.float())
    assert torch.equal(z, z0)
    _check(out, ref, dt, K, f"dgelu {shape}")


@pytest.mark.parametrize("K", [77, 13])
def test_zero_padded_k_operand(K):
    """kz_view operands: a K-contiguous operand whose columns K..K8-1 are zeros is read in place (no padded copy)
    with a row-major partner, and the result matches the reference."""
    torch.manual_seed(6)
    M, N = 1600, 1024
    K8 = (K + 7) // 8 * 8
    buf = torch.zeros(M, K8, device=DEV, dtype=torch.bfloat16)
    buf[:, :K] = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    a = gemm.kz_view(buf, K)
    b = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    calls = []
    orig = gemm._pad_kc
    gemm._pad_kc = lambda *args: calls.append(1) or orig(*args)
    try:
        out = gemm.mmul(a, b, out_dtype=torch.float32)
    finally:
        gemm._pad_kc = orig
    assert not calls, "the zero-padded operand was copied"
    _check(out, _ref(a, b), torch.bfloat16, K, f"kz K={K}")
    # and transposed (M-contiguous) use of the same buffer as the A of a weight gradient
    g = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    out2 = gemm.mmul(a.t(), g, out_dtype=torch.float32)
    _check(out2, _ref(a.t(), g), torch.bfloat16, M, f"kz^T K={K}")


@pytest.mark.parametrize("case", ["plain", "bias_shadow", "beta", "colmajor", "batched", "fp32_out", "gelu_z",
                                  "relu_colmajor", "dgelu"])
def test_library_candidate(case, monkeypatch):
    """The hipBLASLt candidate of the autotuner (forced here) computes the same product for every form it accepts:
    bias through the 16-bit shadow attached to an fp32 master, beta-accumulate, column-major destinations (operands
    swapped), 3-D batches, fp32 weight-gradient output, and activation epilogues run as an in-tree elementwise kernel
    after the library product (GELU with the pre-activation kept, ReLU, the GELU-backward product)."""
    torch.manual_seed(4)
    M, N, K = 384, 320, 256
    monkeypatch.setattr(gemm, "_LIB", True)                  # opt-in (DL4J_AMD_GEMM_LIB=1)
    monkeypatch.setattr(gemm, "_FORCE_CFG", gemm.LIB_CFG)
    from deeplearning4j_amd.ops import fallback
    n0 = fallback.count("gemm")
    a = _mk((M, K), torch.bfloat16)
    b = _mk((K, N), torch.bfloat16, contig_last=False)
    if case == "plain":
        _check(gemm.mmul(a, b), _ref(a, b), torch.bfloat16, K, case)
    elif case == "fp32_out":                       # weight-gradient form: 16-bit operands, fp32 column-major result
        out = torch.empty(N, M, device=DEV).t()
        _check(gemm.mmul(a, b, out=out), _ref(a, b), torch.float32, K, case)
    elif case == "bias_shadow":
        master = torch.randn(N, device=DEV)
        master._dl4j_shadow = master.to(torch.bfloat16)
        _check(gemm.mmul(a, b, bias=master), _ref(a, b, bias=master._dl4j_shadow), torch.bfloat16, K, case)
    elif case == "beta":
        c0 = torch.randn(M, N, device=DEV).to(torch.bfloat16)
        out = c0.clone()
        _check(gemm.mmul(a, b, out=out, beta=1.0), _ref(a, b, beta=1.0, c0=c0), torch.bfloat16, K, case)
    elif case == "colmajor":
        out = torch.empty(N, M, device=DEV, dtype=torch.bfloat16).t()
        _check(gemm.mmul(a, b, out=out), _ref(a, b), torch.bfloat16, K, case)
    elif case == "gelu_z":
        master = torch.randn(N, device=DEV)
        master._dl4j_shadow = master.to(torch.bfloat16)
        z = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        out = gemm.mmul(a, b, bias=master, act="gelu", z=z)
        _check(z, _ref(a, b, bias=master._dl4j_shadow), torch.bfloat16, K, "gelu pre-activation")
        _check(out, gemm._torch_act(z.float(), "gelu"), torch.bfloat16, 8, case)
    elif case == "relu_colmajor":
        out = torch.empty(N, M, device=DEV, dtype=torch.bfloat16).t()
        _check(gemm.mmul(a, b, out=out, act="relu"), _ref(a, b, act="relu"), torch.bfloat16, K, case)
    elif case == "dgelu":
        z = torch.randn(M, N, device=DEV).to(torch.bfloat16)
        out = gemm.mmul(a, b, act="dgelu", z=z)
        _check(out, _ref(a, b) * gemm._dgelu_ref(z.float()), torch.bfloat16, K, case)
    else:
        a3 = torch.randn(3, M, K, device=DEV).to(torch.bfloat16)
        b3 = torch.randn(3, K, N, device=DEV).to(torch.bfloat16)
        out = gemm.mmul(a3, b3)
        ref = torch.stack([a3[i].float() @ b3[i].float() for i in range(3)])
        assert (out.float() - ref).abs().max() <= _tol(torch.bfloat16, K) * ref.abs().max()
    assert fallback.count("gemm") > n0, "a library pick must be counted as a helper fallback"
    c16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    assert gemm._lib_gemm(a, b, c16, False, False, None, 1, "gelu", 1.0, 1.0, None, torch.bfloat16) is None
    assert gemm._lib_gemm(a, b, c16, False, False, torch.zeros(M, device=DEV, dtype=torch.bfloat16), 0, None, 1.0,
                          0.0, None, torch.bfloat16) is None      # row bias stays in-tree
    assert gemm._lib_gemm(a, b, c16, False, False, None, 1, "dgelu", 1.0, 0.0, None, torch.bfloat16) is None
    assert gemm._lib_gemm(a, b, torch.empty(M, N, device=DEV), False, False, None, 1, None, 1.0, 1.0, None,
                          torch.float32) is None          # fp32 output with beta-accumulate stays in-tree


@pytest.mark.parametrize("case", ["long_k", "bias_relu", "colmajor", "beta", "batched"])
@pytest.mark.parametrize("force", [True, False])
def test_fp32_library_candidate(case, force, monkeypatch):
    """fp32 operands: the exact-fp32 MFMA kernel and the fp32 library GEMM (the second candidate, timed per shape)
    compute the same product to fp32 accuracy for every form; the long-K weight-gradient shape of LeNet conv1
    (K = 36864 onto a 20 x 25 output, one 64x64 tile) is dispatched to the library by the measurement."""
    torch.manual_seed(9)
    monkeypatch.setattr(gemm, "_LIB", True)                  # opt-in (DL4J_AMD_GEMM_LIB=1)
    monkeypatch.setattr(gemm, "_F32_FORCE", force)
    M, N, K = (20, 25, 36864) if case == "long_k" else (300, 200, 160)
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV)
    ref = a.double() @ b.double()
    tol = 1e-4 * ref.abs().max().item() + 1e-5 * K ** 0.5
    if case in ("long_k", "colmajor"):
        out = torch.empty(M, N, device=DEV) if case == "long_k" else torch.empty(N, M, device=DEV).t()
        gemm.mmul(a, b, out=out)
    elif case == "bias_relu":
        bias = torch.randn(N, device=DEV)
        out = gemm.mmul(a, b, bias=bias, act="relu")
        ref = torch.relu(ref + bias.double())
    elif case == "beta":
        c0 = torch.randn(M, N, device=DEV)
        out = c0.clone()
        gemm.mmul(a, b, out=out, beta=1.0)
        ref = ref + c0.double()
    else:
        a3, b3 = torch.randn(3, M, K, device=DEV), torch.randn(3, K, N, device=DEV)
        out = gemm.mmul(a3, b3)
        ref = a3.double() @ b3.double()
    assert (out.double() - ref).abs().max().item() <= tol, case


@pytest.mark.parametrize("shape", [(20, 25, 36864), (300, 200, 160), (512, 1000, 2048), (2048, 1000, 512),
                                   (64, 64, 16), (1, 7, 3)])
def test_fp32_tiled_split_k_kernel(shape):
    """The in-tree exact-fp32 path (gemm_f32t: 64/128 tiles, split-K slabs + fixed-order reduce) against fp64 on the
    shapes that used to need the library: LeNet conv1's weight gradient (K = 36864 onto 20 x 25), the ResNet FC
    products, and tiny / ragged edges; the library candidate is off (default), so no fallback is counted."""
    from deeplearning4j_amd.ops import fallback
    torch.manual_seed(2)
    M, N, K = shape
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV)
    n0 = fallback.count()
    out = gemm.mmul(a, b)
    ref = a.double() @ b.double()
    tol = 1e-4 * ref.abs().max().item() + 1e-5 * K ** 0.5
    assert (out.double() - ref).abs().max().item() <= tol
    bias = torch.randn(N, device=DEV)
    out2 = gemm.mmul(a.t().contiguous().t(), b, bias=bias, act="relu")
    assert (out2.double() - torch.relu(ref + bias.double())).abs().max().item() <= tol
    assert fallback.count() == n0
