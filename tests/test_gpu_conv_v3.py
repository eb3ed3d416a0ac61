"""Round-3 implicit-GEMM conv tile engine (csrc/conv_gemm.hip): every tile variant, forward and stride-1
backward-data, against a plain fp32 torch reference; BatchNorm tile statistics from its epilogue against a separate
pass; per-shape variant choice actually used by the conv layer path (run on MI355X)."""
import pytest
import torch
import torch.nn.functional as F

from deeplearning4j_amd.ops import conv_native, native

pytestmark = pytest.mark.gpu

CASES = [
    # N, C, H, W, K, R, S, stride, pad4 (t, b, l, r), dilation
    (2, 64, 9, 9, 64, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),
    (3, 128, 7, 7, 136, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),
    (2, 64, 11, 13, 256, 1, 1, (1, 1), (0, 0, 0, 0), (1, 1)),
    (2, 192, 10, 10, 72, 3, 3, (2, 2), (1, 1, 1, 1), (1, 1)),
    (1, 64, 12, 12, 64, 3, 3, (1, 1), (2, 2, 2, 2), (2, 2)),
    (2, 64, 8, 8, 512, 5, 5, (1, 1), (2, 2, 2, 2), (1, 1)),
    (5, 128, 6, 5, 128, 3, 3, (1, 1), (0, 1, 0, 1), (1, 1)),
]


def _nv():
    return native.load().dl4j_conv_v3_num_variants()


def _data(case, seed=3):
    N, C, H, W, K, R, S, stride, pad4, dil = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, S, generator=g) * 0.1).cuda().bfloat16()
    b = torch.randn(K, generator=g).cuda()
    return x, w, b


def _ref(x, w, b, stride, pad4, dil):
    return F.conv2d(F.pad(x.float(), (pad4[2], pad4[3], pad4[0], pad4[1])), w.float(), b, stride, dilation=dil)


def _close(a, b, tol):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item() + 1e-6
    assert err <= tol * scale, f"max abs err {err} vs scale {scale}"


@pytest.mark.parametrize("case", CASES)
def test_v3_forward_every_variant(cuda, case):
    N, C, H, W, K, R, S, stride, pad4, dil = case
    x, w, b = _data(case)
    yr = _ref(x, w, b, stride, pad4, dil)
    OH, OW = yr.shape[2], yr.shape[3]
    conv_native.bump_version()
    krsc, _ = conv_native._relayout(w, True, False)
    geom = (N, H, W, C, K, R, S, stride[0], stride[1], pad4[0], pad4[2], dil[0], dil[1], OH, OW)
    for v in range(_nv()):
        y = torch.full((N, K, OH, OW), float("nan"), device=cuda).bfloat16().contiguous(
            memory_format=torch.channels_last)
        ts = conv_native._stats_buf(v, N * OH * OW, K, x.device)
        rc = conv_native._fwd_launch(v, x, krsc, b, y, geom, 0.0, ts)
        assert rc == 1, (v, rc)
        torch.cuda.synchronize()
        _close(y, yr, 2e-2)
        # the epilogue statistics reduce to the batch mean / biased variance of the stored bf16 outputs
        P = ts.shape[1]
        rows = y.permute(0, 2, 3, 1).reshape(-1, K).float()
        M = rows.shape[0]
        cnt = torch.tensor([min(64, M - 64 * p) for p in range(P)], device=cuda, dtype=torch.float32)[:, None]
        s1, s2, sh = ts[0], ts[1], ts[2]
        mean = (s1 + cnt * sh).sum(0) / M
        ex2 = (s2 + 2 * sh * s1 + cnt * sh * sh).sum(0) / M
        _close(mean, rows.mean(0), 1e-3)
        _close(ex2 - mean * mean, rows.var(0, unbiased=False), 1e-2)


@pytest.mark.parametrize("case", [c for c in CASES if c[7] == (1, 1) and c[9] == (1, 1)])
@pytest.mark.parametrize("accum", [False, True])
def test_v3_backward_data_every_variant(cuda, case, accum):
    N, C, H, W, K, R, S, stride, pad4, dil = case
    if K % 64:
        pytest.skip("transposed conv needs K % 64 == 0 on the v3 engine")
    x, w, b = _data(case)
    xr = x.float().requires_grad_(True)
    yr = _ref(xr, w, None, stride, pad4, dil)
    g = torch.Generator().manual_seed(5)
    dy = torch.randn(yr.shape, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    OH, OW = dy.shape[2], dy.shape[3]
    conv_native.bump_version()
    _, flip = conv_native._relayout(w, False, True)
    gb = (N, OH, OW, K, C, R, S, 1, 1, R - 1 - pad4[0], S - 1 - pad4[2], 1, 1, H, W)
    base = torch.randn(N, C, H, W, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    for v in range(_nv()):
        dx = base.clone() if accum else torch.empty_like(base)
        rc = conv_native._fwd_launch(v, dy, flip, None, dx, gb, 1.0 if accum else 0.0, None)
        assert rc == 0, (v, rc)
        torch.cuda.synchronize()
        want = xr.grad + (base.float() if accum else 0)
        _close(dx, want, 2e-2)


def test_layer_path_picks_a_variant_and_matches(cuda):
    case = (4, 64, 14, 14, 64, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1))
    N, C, H, W, K, R, S, stride, pad4, dil = case
    x, w, b = _data(case)
    conv_native._V3_CHOICE.clear()
    conv_native.bump_version()
    y = conv_native.conv2d_fwd(x, w, b, stride, pad4, dil, want_stats=True)
    assert any(k[0] == "fwd" for k in conv_native._V3_CHOICE), "the v3 chooser never ran"
    _close(y, _ref(x, w, b, stride, pad4, dil), 2e-2)
    assert hasattr(y, "_bn_tile_stats")


WRW_CASES = [
    (2, 64, 9, 9, 64, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),
    (3, 128, 7, 7, 136, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),
    (2, 64, 11, 13, 256, 1, 1, (1, 1), (0, 0, 0, 0), (1, 1)),
    (2, 192, 10, 10, 72, 3, 3, (2, 2), (1, 1, 1, 1), (1, 1)),
    (1, 64, 12, 12, 64, 3, 3, (1, 1), (2, 2, 2, 2), (2, 2)),
    (4, 256, 8, 8, 64, 1, 1, (2, 2), (0, 0, 0, 0), (1, 1)),
    (2, 8, 23, 23, 64, 7, 7, (2, 2), (3, 3, 3, 3), (1, 1)),
]


@pytest.mark.parametrize("case", WRW_CASES)
def test_v3_weight_gradient_every_variant(cuda, case):
    N, C, H, W, K, R, S, stride, pad4, dil = case
    x, w, _ = _data(case)
    wr = w.float().requires_grad_(True)
    yr = _ref(x, wr, None, stride, pad4, dil)
    g = torch.Generator().manual_seed(8)
    dy = torch.randn(yr.shape, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    OH, OW = dy.shape[2], dy.shape[3]
    geom = (N, H, W, C, K, R, S, stride[0], stride[1], pad4[0], pad4[2], dil[0], dil[1], OH, OW)
    nv = native.load().dl4j_conv_wrw_v3_num_variants()
    outs = []
    db_ref = dy.float().sum(dim=(0, 2, 3))
    for v in range(nv):
        dW = torch.full((K, C, R, S), 3.0, device=cuda)            # written, not accumulated
        db = torch.full((K,), 3.0, device=cuda)
        assert conv_native._wrw_v3_launch(v, x, dy, dW, geom, db if v % 2 else None) == 0
        torch.cuda.synchronize()
        _close(dW, wr.grad, 1e-2)
        if v % 2:
            _close(db, db_ref, 1e-3)
        outs.append(dW)
    again = torch.empty_like(outs[0])
    conv_native._wrw_v3_launch(0, x, dy, again, geom)
    torch.cuda.synchronize()
    assert torch.equal(again, outs[0])                               # slab reduce: bitwise reproducible


HALO_CASES = [
    # the zoo ResNet-50 weight-gradient geometries at a small batch (3x3 halo chunks of 4 / 7 rows, 2 / 4 images)
    (2, 64, 28, 28, 64, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),
    (2, 128, 14, 14, 128, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),
    (4, 256, 7, 7, 256, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),
    (8, 512, 4, 4, 512, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),
    (2, 64, 56, 56, 64, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),            # canonical stage-1 (TH = 1 chunks)
    (3, 72, 10, 10, 136, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),           # partial k / c tiles, odd N
    (2, 64, 28, 28, 256, 1, 1, (1, 1), (0, 0, 0, 0), (1, 1)),
    (2, 256, 28, 28, 64, 1, 1, (1, 1), (0, 0, 0, 0), (1, 1)),
    (2, 256, 14, 14, 512, 1, 1, (1, 1), (0, 0, 0, 0), (1, 1)),
    (2, 256, 15, 15, 128, 1, 1, (2, 2), (0, 0, 0, 0), (1, 1)),          # strided 1x1 gather, partial last chunk
    (3, 40, 9, 7, 24, 1, 1, (1, 1), (0, 0, 0, 0), (1, 1)),
]


@pytest.mark.parametrize("case", HALO_CASES)
def test_halo_weight_gradient(cuda, case):
    """csrc/conv_wrw.hip: every applicable variant and split count (auto, /2, x2) against the fp32 torch weight
    gradient; conv-bias partials against sum(dY); bitwise reproducible."""
    N, C, H, W, K, R, S, stride, pad4, dil = case
    x, w, _ = _data(case)
    wr = w.float().requires_grad_(True)
    yr = _ref(x, wr, None, stride, pad4, dil)
    g = torch.Generator().manual_seed(8)
    dy = torch.randn(yr.shape, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    OH, OW = dy.shape[2], dy.shape[3]
    geom = (N, H, W, C, K, R, S, stride[0], stride[1], pad4[0], pad4[2], dil[0], dil[1], OH, OW)
    cands = conv_native._halo_candidates(geom)
    assert cands, "no halo variant accepted the shape"
    db_ref = dy.float().sum(dim=(0, 2, 3))
    for i, c in enumerate(cands):
        dW = torch.full((K, C, R, S), 3.0, device=cuda)
        db = torch.full((K,), 3.0, device=cuda)
        assert conv_native._wrw_launch(c, x, dy, dW, geom, db if i % 2 == 0 else None) == 0, c
        torch.cuda.synchronize()
        _close(dW, wr.grad, 1e-2)
        if i % 2 == 0:
            _close(db, db_ref, 1e-3)
        again = torch.empty_like(dW)
        conv_native._wrw_launch(c, x, dy, again, geom)
        torch.cuda.synchronize()
        assert torch.equal(again, dW), c


@pytest.mark.parametrize("case,splits", [(HALO_CASES[0], 1), (HALO_CASES[0], 9), (HALO_CASES[0], 64),
                                         (HALO_CASES[5], 7), (HALO_CASES[6], 100), (HALO_CASES[9], 13)])
def test_halo_in_kernel_tree_reduce(cuda, case, splits):
    """csrc/conv_wrw.hip tree_reduce: the split slabs summed inside wrw_halo by the last-arriving block of each tree
    node (fan-in 8 default, 2 = deepest tree, 64 = one level) against the separate wrw_halo_reduce launch (fan 0) and
    the fp32 torch weight gradient; weight and bias gradients bitwise reproducible for every fan-in, including single
    split, partial last groups and partial k / c tiles."""
    import ctypes
    lib = native.load()
    lib.dl4j_conv_wrw_set_tree.argtypes = [ctypes.c_int]
    N, C, H, W, K, R, S, stride, pad4, dil = case
    x, w, _ = _data(case)
    wr = w.float().requires_grad_(True)
    yr = _ref(x, wr, None, stride, pad4, dil)
    g = torch.Generator().manual_seed(9)
    dy = torch.randn(yr.shape, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    geom = (N, H, W, C, K, R, S, stride[0], stride[1], pad4[0], pad4[2], dil[0], dil[1], dy.shape[2], dy.shape[3])
    var = conv_native._halo_candidates(geom)[0][1]
    db_ref = dy.float().sum(dim=(0, 2, 3))
    old = lib.dl4j_conv_wrw_set_tree(8)
    res = {}
    try:
        for fan in (0, 8, 2, 64):
            lib.dl4j_conv_wrw_set_tree(fan)
            outs = []
            for _ in range(2):
                dW = torch.full((K, C, R, S), 3.0, device=cuda)
                db = torch.full((K,), 3.0, device=cuda)
                assert conv_native._wrw_launch(("halo", var, splits), x, dy, dW, geom, db) == 0
                torch.cuda.synchronize()
                outs.append((dW, db))
            assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), fan
            _close(outs[0][0], wr.grad, 1e-2)
            _close(outs[0][1], db_ref, 1e-3)
            res[fan] = outs[0]
    finally:
        lib.dl4j_conv_wrw_set_tree(old)
    for fan in (8, 2, 64):
        torch.testing.assert_close(res[fan][0], res[0][0], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(res[fan][1], res[0][1], rtol=1e-5, atol=1e-4)


def test_halo_rejects_unsupported_shapes():
    lib = native.load()
    import ctypes
    sp = ctypes.c_int(0)
    # 3x3 stride 2 and 5x5 are not halo shapes: the chooser must see 0 and fall back
    assert lib.dl4j_conv_wrw_halo_ws_floats(2, 9, 9, 64, 64, 3, 3, 2, 2, 1, 1, 1, 1, 5, 5, 0, 0, ctypes.byref(sp)) == 0
    assert lib.dl4j_conv_wrw_halo_ws_floats(2, 9, 9, 64, 64, 5, 5, 1, 1, 2, 2, 1, 1, 9, 9, 0, 0, ctypes.byref(sp)) == 0


@pytest.mark.parametrize("N,H", [(2, 20), (16, 50), (8, 256), (9, 256)])
def test_conv_tile_statistics_feed_batchnorm(cuda, N, H):
    """Conv epilogue tile statistics -> BN forward at partial counts that take each fold path: one block (P <= 32),
    128-row fold blocks (P = 625), the single-launch limit (P = 8192) and the two-stage reduce above it (P = 9216).
    Running mean / var and the normalised output against fp32 torch (reference NN:nn/layers/normalization/
    BatchNormalization.java:250-370)."""
    from deeplearning4j_amd import ops
    C = K = 64
    g = torch.Generator().manual_seed(4)
    x = (torch.randn(N, C, H, H, generator=g) + 0.2).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 3, 3, generator=g) * 0.05).cuda().bfloat16()
    y = conv_native.conv2d_fwd(x, w, None, (1, 1), (1, 1, 1, 1), (1, 1), want_stats=True)
    assert hasattr(y, "_bn_tile_stats")
    gamma = (torch.rand(K, generator=g) + 0.5).cuda()
    beta = torch.randn(K, generator=g).cuda()
    rm, rv = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
    out, ctx = ops.bn_forward(y, gamma, beta, rm, rv, True, 0.9, 1e-5, True)
    yf = y.float()
    mean = yf.mean(dim=(0, 2, 3))
    var = yf.var(dim=(0, 2, 3), unbiased=False)
    _close(rm, 0.1 * mean, 1e-4)
    _close(rv, 0.9 + 0.1 * (var + 1e-5), 1e-4)
    ref = torch.relu((yf - mean.view(1, -1, 1, 1)) * torch.rsqrt(var + 1e-5).view(1, -1, 1, 1) * gamma.view(1, -1, 1, 1)
                     + beta.view(1, -1, 1, 1))
    _close(out, ref, 3e-2)
