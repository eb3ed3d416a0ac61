"""Convolution through the hand-written MFMA implicit-GEMM kernels (``csrc/conv_igemm.hip``).

Coverage (everything else returns ``None`` and ``ops.conv`` uses the library path):
  * forward:        bf16 NHWC, C_in % 8 == 0, C_out % 4 == 0, any kernel/stride/padding/dilation
  * backward-data:  stride 1 (any kernel, padding) via the flipped-weight transposed conv;
                    1x1 kernels with any stride and no padding via a strided-scatter GEMM
  * backward-weight: C_in % 8 == 0, C_out % 8 == 0, any geometry; fp32 result accumulated straight into the
                    network's flat gradient view (DL4J [K][C][R][S] order), conv-bias gradient fused.
Weights are re-laid-out once per parameter version (KRSC for forward, flipped CRSK for backward-data).
"""
import ctypes
import weakref
import contextlib
import os

import numpy as np

import torch

from ..memory import arena

from . import native, nd4j_kernels, side_stream, tunedb
from .native import _ptr, _stream, c_int, c_ll, c_void_p

native.register_sig("dl4j_conv_w_relayout", [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p])
native.register_sig("dl4j_conv_w_relayout_batched", [c_void_p, c_int, c_ll, c_void_p])
native.register_sig("dl4j_conv_relayout_job_bytes", [])
native.register_sig("dl4j_conv_relayout_per_block", [])
native.register_sig("dl4j_conv_w_relayout_tiled", [c_void_p, c_int, c_ll, c_void_p])
native.register_sig("dl4j_conv_relayout_tile_job_bytes", [])
native.register_sig("dl4j_conv_relayout_tile_max_rs", [])
native.register_sig("dl4j_conv_fwd", [c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 15 + [c_void_p, c_void_p])
native.register_sig("dl4j_conv_bwd_data_s1", [c_void_p, c_void_p, c_void_p] + [c_int] * 12 + [c_void_p])
native.register_sig("dl4j_conv_bwd_data_1x1", [c_void_p, c_void_p, c_void_p] + [c_int] * 9 + [c_void_p])
native.register_sig("dl4j_conv_wrw", [c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 16 + [c_void_p])
native.register_sig("dl4j_conv_set_variant", [c_int])
native.register_sig("dl4j_conv_set_wrw_variant", [c_int])
native.register_sig("dl4j_conv_set_wrw_remap", [c_int])
native.register_sig("dl4j_conv_wrw_permute", [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p])
native.register_sig("dl4j_conv_wrw_det", [c_void_p] * 5 + [c_int] * 17 + [c_void_p])
native.register_sig("dl4j_conv_wrw_det_floats", [c_int] * 8, restype=c_ll)
native.register_sig("dl4j_conv_fwd_v3", [c_int, c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 15 +
                    [ctypes.c_float, c_void_p, c_int, c_void_p])
native.register_sig("dl4j_conv_v3_num_variants", [])
native.register_sig("dl4j_conv_v3_default_variant", [c_ll, c_int])
native.register_sig("dl4j_conv_wrw_v3_num_variants", [])
native.register_sig("dl4j_conv_wrw_v3_ws_floats", [c_int] * 9 + [ctypes.POINTER(c_int)], restype=c_ll)
native.register_sig("dl4j_conv_wrw_v3", [c_int] + [c_void_p] * 5 + [c_int] * 17 + [c_void_p])
native.register_sig("dl4j_conv_wrw_halo_ws_floats", [c_int] * 17 + [ctypes.POINTER(c_int)], restype=c_ll)
native.register_sig("dl4j_conv_wrw_halo", [c_int] + [c_void_p] * 5 + [c_int] * 17 + [c_void_p])

# Optional per-shape override of the weight-gradient split count (tuning): {(N,H,W,C,K,R,S,stride): splits}
WRW_SPLITS = {}

# Bumped by every parameter update (BaseNetwork._apply_update / setParams): invalidates relayout caches.
WEIGHT_VERSION = [0]
_cache = {}
_wrw_ws = {}   # (K, R, S, C, device) -> fp32 KRSC accumulation workspace, kept zero by the permute kernel


def deterministic():
    """DL4J_AMD_DETERMINISTIC=1: conv weight gradients without float atomics (per-split slabs + fixed-order reduce),
    so a training step is bitwise reproducible (the data-parallel equivalence tests rely on it)."""
    return os.environ.get("DL4J_AMD_DETERMINISTIC", "0") == "1"


_det_ws = {}


def _det_scratch(nfloats, device):
    # one growing slab per (device, stream): the side-stream weight gradients never share it with the main stream
    key = (str(device), torch.cuda.current_stream(device).stream_id if device.type == "cuda" else 0)
    t = _det_ws.get(key)
    if t is None or t.numel() < nfloats:
        t = _det_ws[key] = torch.empty(int(nfloats), dtype=torch.float32, device=device)
    return t


def _zeroed_wrw_ws(K, R, S, C, device):
    # keyed by stream too: weight gradients on the overlap stream (ops/side_stream.py) and on the main stream must
    # never share an accumulator
    key = (K, R, S, C, str(device), torch.cuda.current_stream(device).stream_id if device.type == "cuda" else 0)
    ws = _wrw_ws.get(key)
    if ws is None:
        ws = torch.zeros((K, R, S, C), dtype=torch.float32, device=device)
        _wrw_ws[key] = ws
    return ws


def set_kernel_variant(v):
    """1 = LDS-DMA pipelined forward/backward-data kernel (default), 0 = register-staged kernel (A/B testing)."""
    native.load().dl4j_conv_set_variant(int(v))


def set_wrw_variant(v):
    """0 = register-staged weight-gradient kernel (default), 1 = LDS-DMA pipelined variant."""
    native.load().dl4j_conv_set_wrw_variant(int(v))


def set_wrw_remap(v):
    """1 = XCD-aware weight-gradient block order (default), 0 = plain launch order (A/B only)."""
    native.load().dl4j_conv_set_wrw_remap(int(v))


def bump_version():
    WEIGHT_VERSION[0] += 1


# Parameter buffers whose every modification bumps WEIGHT_VERSION (a network's flat params / compute shadow).
# Weights anywhere else (SameDiff variables, ad-hoc op calls, temporaries) are relaid out on every call: their
# address may be reused by a different tensor and nothing reports their updates.
_MANAGED = {}


def register_managed(buf):
    _MANAGED[buf.data_ptr()] = (buf.data_ptr() + buf.numel() * buf.element_size(), weakref.ref(buf))


def is_managed(ptr):
    for s, (e, r) in list(_MANAGED.items()):
        if r() is None:
            del _MANAGED[s]
        elif s <= ptr < e:
            return True
    return False


class _WEnt:
    """Kernel-layout copies of one conv weight: persistent buffers (stable addresses for HIP graphs, no allocator
    churn) plus the weight version each copy was last written for."""
    __slots__ = ("krsc", "flip", "vk", "vf")

    def __init__(self):
        self.krsc = self.flip = None
        self.vk = self.vf = -1


def _ent(w):
    key = (w.data_ptr(), tuple(w.shape))
    e = _cache.get(key)
    if e is None:
        e = _cache[key] = _WEnt()
    return e


def _relayout(w, want_krsc, want_flip):
    e = _ent(w)
    v = WEIGHT_VERSION[0]
    K, C, R, S = w.shape
    if R * S == 1 and w.is_contiguous():
        e.krsc = w.view(K, 1, 1, C)                    # [K][C][1][1] is already [K][R][S][C]
        want_krsc = False
    fresh = not is_managed(w.data_ptr())
    need_k = want_krsc and (fresh or e.vk != v)
    need_f = want_flip and (fresh or e.vf != v)
    if need_k or need_f:
        if need_k and e.krsc is None:
            e.krsc = torch.empty((K, R, S, C), dtype=w.dtype, device=w.device)
        if need_f and e.flip is None:
            e.flip = torch.empty((C, R, S, K), dtype=w.dtype, device=w.device)
        wc = w.contiguous()
        rc = native.load().dl4j_conv_w_relayout(_ptr(wc), _ptr(e.krsc if need_k else None),
                                                _ptr(e.flip if need_f else None), K, C, R, S, _stream())
        native._check(rc, "conv_w_relayout")
        if need_k:
            e.vk = v
        if need_f:
            e.vf = v
    return e.krsc, e.flip


_plans = {}


def relayout_all(weights, want_flip=True):
    """Refresh the kernel-layout copies of every eligible conv weight in ONE launch ahead of the forward pass; the
    per-conv lazy path then finds fresh copies. Returns the number of weights.

    The LDS-tiled kernel (dl4j_conv_w_relayout_tiled) serves every weight with at most 16 taps; a 1x1 weight's KRSC
    layout is the weight itself (a view, never copied), only its transposed copy is refreshed."""
    ws = [w for w in weights if w.dtype in _KDT and w.is_cuda and w.dim() == 4 and w.is_contiguous()
          and w.shape[1] % 8 == 0 and w.shape[0] % 4 == 0]
    if not ws:
        return 0
    lib = native.load()
    if _TILED_RELAYOUT and all(w.shape[2] * w.shape[3] <= lib.dl4j_conv_relayout_tile_max_rs() and
                               w.data_ptr() % 16 == 0 for w in ws):   # 16-byte tile loads
        return _relayout_all_tiled(ws, want_flip, lib)
    key = (tuple((w.data_ptr(), tuple(w.shape)) for w in ws), bool(want_flip))
    plan = _plans.get(key)
    if plan is None:
        per_block = lib.dl4j_conv_relayout_per_block()
        assert lib.dl4j_conv_relayout_job_bytes() == 56
        jt = np.dtype([("W", "<u8"), ("out", "<u8"), ("K", "<i4"), ("C", "<i4"), ("R", "<i4"), ("S", "<i4"),
                       ("kind", "<i4"), ("pad", "<i4"), ("first", "<i8"), ("n", "<i8")])
        rows, ents, nblk = [], [], 0
        for w in ws:
            K, C, R, S = w.shape
            e = _ent(w)
            if e.krsc is None:
                e.krsc = torch.empty((K, R, S, C), dtype=w.dtype, device=w.device)
            flip_ok = want_flip and K % 8 == 0
            if flip_ok and e.flip is None:
                e.flip = torch.empty((C, R, S, K), dtype=w.dtype, device=w.device)
            n = K * C * R * S
            outs = [(0, e.krsc)] + ([(1, e.flip)] if flip_ok else [])
            for kind, buf in outs:
                rows.append((w.data_ptr(), buf.data_ptr(), K, C, R, S, kind, 0, nblk, n))
                nblk += (n + per_block - 1) // per_block
            ents.append((e, flip_ok))
        arr = np.array(rows, dtype=jt)
        dev_jobs = torch.from_numpy(arr.view(np.uint8).copy()).to(ws[0].device)
        plan = [dev_jobs, len(rows), nblk, ents, -1]
        _plans[key] = plan
    dev_jobs, njobs, nblk, ents, done_v = plan
    if done_v == WEIGHT_VERSION[0]:
        return len(ws)                      # already fresh (e.g. several forward passes between updates)
    rc = lib.dl4j_conv_w_relayout_batched(_ptr(dev_jobs), njobs, nblk, _stream())
    native._check(rc, "conv_w_relayout_batched")
    v = WEIGHT_VERSION[0]
    plan[4] = v
    for e, flip_ok in ents:
        e.vk = v
        if flip_ok:
            e.vf = v
    return len(ws)


_TILED_RELAYOUT = os.environ.get("DL4J_AMD_RELAYOUT_TILED", "1") == "1"
_RLT_K, _RLT_C = 64, 32


def _relayout_all_tiled(ws, want_flip, lib):
    key = ("tiled", tuple((w.data_ptr(), tuple(w.shape)) for w in ws), bool(want_flip))
    plan = _plans.get(key)
    if plan is None:
        assert lib.dl4j_conv_relayout_tile_job_bytes() == 48
        jt = np.dtype([("W", "<u8"), ("krsc", "<u8"), ("flip", "<u8"), ("K", "<i4"), ("C", "<i4"), ("RS", "<i4"),
                       ("tiles_c", "<i4"), ("first", "<i8")])
        rows, ents, nblk = [], [], 0
        for w in ws:
            K, C, R, S = w.shape
            e = _ent(w)
            if R * S == 1:
                e.krsc = w.view(K, 1, 1, C)             # already the kernel layout
            elif e.krsc is None:
                e.krsc = torch.empty((K, R, S, C), dtype=w.dtype, device=w.device)
            flip_ok = want_flip and K % 8 == 0
            if flip_ok and e.flip is None:
                e.flip = torch.empty((C, R, S, K), dtype=w.dtype, device=w.device)
            tk, tc = (K + _RLT_K - 1) // _RLT_K, (C + _RLT_C - 1) // _RLT_C
            rows.append((w.data_ptr(), 0 if R * S == 1 else e.krsc.data_ptr(), e.flip.data_ptr() if flip_ok else 0,
                         K, C, R * S, tc, nblk))
            nblk += tk * tc
            ents.append((e, flip_ok))
        arr = np.array(rows, dtype=jt)
        dev_jobs = torch.from_numpy(arr.view(np.uint8).copy()).to(ws[0].device)
        plan = [dev_jobs, len(rows), nblk, ents, -1]
        _plans[key] = plan
    dev_jobs, njobs, nblk, ents, done_v = plan
    if done_v == WEIGHT_VERSION[0]:
        return len(ws)
    native._check(lib.dl4j_conv_w_relayout_tiled(_ptr(dev_jobs), njobs, nblk, _stream()), "conv_w_relayout_tiled")
    v = WEIGHT_VERSION[0]
    plan[4] = v
    for e, flip_ok in ents:
        e.vk = v
        if flip_ok:
            e.vf = v
    return len(ws)


_KDT = (torch.bfloat16, torch.float16)


def _ok_act(t):
    return t.dtype in _KDT and t.dim() == 4 and t.is_cuda


def _dtc(t):
    """Kernel dtype code: 1 bf16, 2 fp16."""
    return 2 if t.dtype == torch.float16 else 1


def _q(t):
    """Channel granularity the kernels need: bf16 runs every shape (round-2 kernels as the fallback tile), fp16 only
    the round-3 engines, whose reduction tiles are 64 channels deep."""
    return 64 if t.dtype == torch.float16 else 8


def _cl(t):
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


def _out_hw(H, W, R, S, stride, pad4, dilation):
    pt, pb, pl, pr = pad4
    OH = (H + pt + pb - ((R - 1) * dilation[0] + 1)) // stride[0] + 1
    OW = (W + pl + pr - ((S - 1) * dilation[1] + 1)) // stride[1] + 1
    return OH, OW


def _conv2d_fwd(x, w, b, stride, pad4, dilation, want_stats=False, use_gemm=True):
    """want_stats: also emit per-tile BatchNorm statistics of the output from the kernel epilogue; they are attached
    to the result as ``y._bn_tile_stats = (planes [3, P, K] fp32, P)`` for a consuming training-mode BN layer."""
    if not (_ok_act(x) and w.dtype == x.dtype):
        return None
    N, C, H, W = x.shape
    K, Cw, R, S = w.shape
    fp16 = x.dtype == torch.float16
    if C == 3 and not fp16 and os.environ.get("DL4J_AMD_KERNEL_STEM", "1") == "1":
        from . import conv_stem
        if conv_stem.supported(_cl(x), w, b, stride, pad4, dilation):
            y = conv_stem.forward(_cl(x), w, want_stats)
            if y is not None:
                return y
    if C != Cw or C % 8 != 0 or K % 4 != 0:
        return None
    OH, OW = _out_hw(H, W, R, S, stride, pad4, dilation)
    if OH <= 0 or OW <= 0:
        return None
    if _is_pointwise(R, S, stride, pad4, dilation) and use_gemm:
        # 1x1 stride-1 conv in NHWC is a plain GEMM: Y[M, K] = X[M, C] . W[K, C]^T on the 8-phase MFMA kernel, bias
        # and the BatchNorm tile statistics in its epilogue; no weight relayout ([K][C][1][1] is already K-major)
        from .gemm import mmul
        x = _cl(x)
        M = N * H * W
        y = arena.empty((N, K, H, W), x.dtype, x.device, channels_last=True)
        ts = None
        if want_stats and C % 64 == 0 and K % 8 == 0:
            P = 2 * ((M + 127) // 128)
            ts = torch.empty((3, P, K), dtype=torch.float32, device=x.device)
        mmul(x.permute(0, 2, 3, 1).reshape(M, C), w.reshape(K, C).t(),
             out=y.permute(0, 2, 3, 1).reshape(M, K), bias=b.float() if b is not None else None, stats=ts)
        if ts is not None:
            y._bn_tile_stats = (ts, ts.shape[1])
        return y
    if fp16 and not _v3_ok(C, K, R, S):
        return None                                    # fp16 runs on the round-3 engine only
    krsc, _ = _relayout(w, True, False)
    x = _cl(x)
    y = arena.empty((N, K, OH, OW), x.dtype, x.device, channels_last=True)
    bias = b.float().contiguous() if b is not None else None
    stats = want_stats and C % 32 == 0 and R * S <= 64 and K % 8 == 0
    geom = (N, H, W, C, K, R, S, stride[0], stride[1], pad4[0], pad4[2], dilation[0], dilation[1], OH, OW)
    v = -1
    if _v3_ok(C, K, R, S):
        key = ("fwd", geom, bias is not None, stats, x.dtype)
        v = _v3_pick(key, lambda var, out, t: _fwd_launch(var, x, krsc, bias, out, geom, 0.0, t),
                     y, lambda var: _stats_buf(var, N * OH * OW, K, x.device, geom) if stats else None)
    ts = _stats_buf(v, N * OH * OW, K, x.device, geom) if stats else None
    rc = _fwd_launch(v, x, krsc, bias, y, geom, 0.0, ts)
    if rc == 1:
        _attach_tile_stats(y, ts, v, geom)
        rc = 0
    native._check(rc, "conv_fwd")
    return y


# ------------------------------------------------------------------ round-3 tile engine (csrc/conv_gemm.hip)
V3 = os.environ.get("DL4J_AMD_CONV_V3", "1") == "1"
_V3_CHOICE = {}     # (direction, geometry, ...) -> variant id (-1 = round-2 kernel in csrc/conv_igemm.hip)


def _v3_ok(C, K, R, S):
    return V3 and C % 64 == 0 and K % 8 == 0 and R * S <= 64


def _stats_buf(variant, M, K, device, geom=None):
    # BatchNorm tile partials, 64-row partials: the round-2 kernel pads to whole 128-row tiles; the halo kernel writes
    # one partial per pixel chunk
    if variant == HALO_VAR:
        P, _ = _halo_plan(geom)
        if not P:
            return None
    else:
        P = (M + 63) // 64 if variant >= 0 else 2 * ((M + 127) // 128)
    return torch.empty((3, P, K), dtype=torch.float32, device=device)


STREAM_VAR = 100     # persistent loader/consumer conv kernel (csrc/gemm_stream.hip conv_stream), a tuner candidate
HALO_VAR = 101       # halo-staged 3x3 / 64-channel kernel (csrc/conv_halo.hip), a tuner candidate
native.register_sig("dl4j_conv_halo_plan", [c_int] * 15 + [ctypes.POINTER(c_int)], restype=c_ll)
native.register_sig("dl4j_conv_halo", [c_int, c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 15 +
                    [ctypes.c_float, c_void_p, c_void_p])
_HALO_PLANS = {}


def _halo_plan(geom):
    """(chunks, pixels per chunk) of dl4j_conv_halo for a geometry, (0, 0) when it is not that kernel's."""
    r = _HALO_PLANS.get(geom)
    if r is None:
        pc = ctypes.c_int(0)
        n = native.load().dl4j_conv_halo_plan(*geom, ctypes.byref(pc))
        r = _HALO_PLANS[geom] = (int(n), int(pc.value)) if n > 0 else (0, 0)
    return r


def _attach_tile_stats(y, ts, variant, geom):
    """The producer's BN tile statistics for a consuming training BN layer (ops/native.py _tile_rpp)."""
    if variant == HALO_VAR:
        y._bn_tile_stats = (ts, ts.shape[1], _halo_plan(geom)[1])
    else:
        y._bn_tile_stats = (ts, ts.shape[1])


def _fwd_launch(variant, x, wk, bias, y, geom, beta, ts):
    """One conv launch on the chosen kernel. Returns 1 when BN tile statistics were written to ts, 0 when not, a
    negative code / HIP error otherwise."""
    lib = native.load()
    if variant == HALO_VAR:
        if ts is not None and ts.shape[1] != _halo_plan(geom)[0]:
            return -1
        rc = lib.dl4j_conv_halo(_dtc(x), _ptr(x), _ptr(wk), _ptr(bias), _ptr(y), *geom, float(beta), _ptr(ts),
                                _stream())
        return 1 if (rc == 0 and ts is not None) else rc
    if variant == STREAM_VAR:
        native.register_sig("dl4j_conv_stream", [c_int, c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 15 +
                            [ctypes.c_float, c_void_p, c_void_p])
        rc = lib.dl4j_conv_stream(_dtc(x), _ptr(x), _ptr(wk), _ptr(bias), _ptr(y), *geom, float(beta), _ptr(ts),
                                  _stream())
        return 1 if (rc == 0 and ts is not None) else rc
    if variant >= 0:
        rc = lib.dl4j_conv_fwd_v3(_dtc(x), _ptr(x), _ptr(wk), _ptr(bias), _ptr(y), *geom, float(beta), _ptr(ts),
                                  variant, _stream())
        return 1 if (rc == 0 and ts is not None) else rc
    N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW = geom
    if beta != 0.0 or x.dtype != torch.bfloat16:
        return -1
    return lib.dl4j_conv_fwd(_ptr(x), _ptr(wk), _ptr(bias), _ptr(y), N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH,
                             OW, _ptr(ts), _stream())


def _v3_pick(key, launch, out, make_ts, allow_r2=True):
    """Per-shape kernel choice: the first eager call times every tile variant of the round-3 engine and the round-2
    kernel on scratch outputs (inline on this stream) and keeps the fastest; calls under HIP-graph capture, or with
    DL4J_AMD_CONV_TUNE=0, use the remembered choice or the engine's default tile."""
    v = _V3_CHOICE.get(key)
    if v is not None:
        return v
    v = tunedb.lookup("conv_v3", key)
    if v is not None:
        _V3_CHOICE[key] = v
        return v
    lib = native.load()
    geom = key[1]
    M, K = geom[0] * geom[13] * geom[14], geom[4]
    if torch.cuda.is_current_stream_capturing() or os.environ.get("DL4J_AMD_CONV_TUNE", "1") != "1":
        return lib.dl4j_conv_v3_default_variant(M, K)
    # allow_r2=False: the round-2 kernel lacks an epilogue the caller needs (BN-backward sums), so its lower kernel
    # time would not be the lower step time
    cands = list(range(lib.dl4j_conv_v3_num_variants())) + [STREAM_VAR, HALO_VAR] + \
        ([-1] if out.dtype == torch.bfloat16 and allow_r2 else [])
    scratch = torch.empty_like(out)
    if key[0] == "bwd_acc":
        scratch.copy_(out)
    best, bt = None, None
    with side_stream.suspended():
        for var in cands:
            ts = make_ts(var)
            if launch(var, scratch, ts) not in (0, 1):
                continue
            t = _timed(lambda: launch(var, scratch, ts), reps=tunedb.reps(3))
            if bt is None or t < bt:
                best, bt = var, t
    v = _V3_CHOICE[key] = best if best is not None else -1
    tunedb.record("conv_v3", key, v)
    return v


def _conv2d_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db, gW=None, gb=None, grads_zeroed=False,
                dx_accum=None, gemm_dx=True, gemm_dw=True):
    """grads_zeroed: the caller guarantees gW/gb (flat-gradient views) are already zero (the network clears the
    whole flat gradient with one fill per step), so no per-layer memset is launched.
    dx_accum: an existing channels-last bf16 gradient of x (another consumer's contribution); when the bwd-data
    kernel can take it, the result is accumulated into it in the kernel epilogue and it is returned as dx."""
    if not (_ok_act(x) and _ok_act(dy) and w.dtype == x.dtype and dy.dtype == x.dtype):
        return None
    N, C, H, W = x.shape
    K, Cw, R, S = w.shape
    fp16 = x.dtype == torch.float16
    if C == 3 and not fp16 and not need_dx and need_dw and os.environ.get("DL4J_AMD_KERNEL_STEM", "1") == "1":
        from . import conv_stem
        if conv_stem.supported(_cl(x), w, None, stride, pad4, dilation) and _cl(dy).shape[1] == 64:
            r = conv_stem.backward_weight(_cl(x), _cl(dy), gW, gb, need_db)
            if r != "unsupported":
                return None, r[0], r[1]
    if C != Cw or C % 8 != 0 or K % 8 != 0:
        return None
    OH, OW = dy.shape[2], dy.shape[3]
    bnb = getattr(x, "_bn_bwd_req", None) if need_dx else None   # x is a training BN layer's output (ops/native.py)
    x = _cl(x)
    dy = _cl(dy)
    adt = x.dtype
    lib = native.load()
    dx = None
    pw = _is_pointwise(R, S, stride, pad4, dilation)
    if dx_accum is not None and hasattr(dx_accum, "_bn_bwd_stats"):
        del dx_accum._bn_bwd_stats                     # about to be summed into: its BN-backward sums go stale
    if bnb is not None and (adt not in (torch.bfloat16, torch.float16) or tuple(bnb[0].shape) != (N * H * W, C) or
                            bnb[0].dtype != adt or (dx_accum is not None and native.BNB_MODE < 2)):
        bnb = None
    if need_dx and pw and gemm_dx:
        from .gemm import mmul
        M = N * H * W
        acc = dx_accum is not None and dx_accum.dtype == adt and tuple(dx_accum.shape) == (N, C, H, W) \
            and dx_accum.is_contiguous(memory_format=torch.channels_last)
        dx = dx_accum if acc else arena.empty((N, C, H, W), adt, x.device, channels_last=True)
        # dX[M, C] = dY[M, K] . W[K, C]  (+= the other consumer's gradient through beta)
        if bnb is not None and (acc or dx_accum is None):
            # ... with the consuming BN layer's backward partial sums (of the stored sum) from the epilogue
            planes = torch.empty((2, (M + 63) // 64, C), dtype=torch.float32, device=x.device)
            with native.bnb_armed(bnb):
                mmul(dy.permute(0, 2, 3, 1).reshape(M, K), w.reshape(K, C), out=dx.permute(0, 2, 3, 1).reshape(M, C),
                     beta=1.0 if acc else 0.0, stats=planes, stats_tag="bnb_acc" if acc else "bnb")
            native.bnb_tag(dx, planes, bnb)
        else:
            mmul(dy.permute(0, 2, 3, 1).reshape(M, K), w.reshape(K, C), out=dx.permute(0, 2, 3, 1).reshape(M, C),
                 beta=1.0 if acc else 0.0)
    elif need_dx:
        s1 = tuple(stride) == (1, 1) and tuple(dilation) == (1, 1)
        pure_1x1 = R == 1 and S == 1 and not any(pad4) and tuple(dilation) == (1, 1)
        acc = dx_accum is not None and dx_accum.dtype == adt and tuple(dx_accum.shape) == (N, C, H, W) \
            and dx_accum.is_contiguous(memory_format=torch.channels_last)
        if s1 and (H, W) == _out_hw_inv(OH, OW, R, S, pad4, H, W) and (not fp16 or _v3_ok(K, C, R, S)):
            _, flip = _relayout(w, False, True)
            dx = dx_accum if acc else arena.empty((N, C, H, W), adt, x.device, channels_last=True)
            # transposed conv: "input" dY (OH x OW x K), flipped CRSK weights, pad' = R-1-pad, output H x W x C
            geo_b = (N, OH, OW, K, C, R, S, 1, 1, R - 1 - pad4[0], S - 1 - pad4[2], 1, 1, H, W)

            def bwd_launch(var, out, ts):
                if var >= 0:
                    return _fwd_launch(var, dy, flip, None, out, geo_b, 1.0 if acc else 0.0, ts)
                return lib.dl4j_conv_bwd_data_s1(_ptr(dy), _ptr(flip), _ptr(out), N, H, W, C, K, R, S, pad4[0],
                                                 pad4[2], OH, OW, int(acc), _stream())
            v = -1
            P = (N * H * W + 63) // 64
            mk = (lambda var: torch.empty((2, P, C), dtype=torch.float32, device=x.device) if var >= 0 else None) \
                if bnb is not None else (lambda var: None)
            with (native.bnb_armed(bnb) if bnb is not None else contextlib.nullcontext()):
                if _v3_ok(K, C, R, S):
                    v = _v3_pick(("bwd_acc" if acc else "bwd", geo_b, adt, bnb is not None), bwd_launch, dx, mk,
                                 allow_r2=bnb is None)
                planes = mk(v)
                rc = bwd_launch(v, dx, planes)
            if rc == 1:
                native.bnb_tag(dx, planes, bnb)
                rc = 0
            native._check(rc, "conv_bwd_data_s1")
        elif pure_1x1 and stride[0] == stride[1] and not fp16:
            _, flip = _relayout(w, False, True)
            if acc:
                dx = dx_accum                                # only the strided rows are touched (+=)
            else:
                dx = nd4j_kernels.zero_(torch.empty((N, C, H, W), dtype=torch.bfloat16, device=x.device,
                                                    memory_format=torch.channels_last))
            rc = lib.dl4j_conv_bwd_data_1x1(_ptr(dy), _ptr(flip), _ptr(dx), N, H, W, C, K, stride[0], OH, OW,
                                            int(acc), _stream())
            native._check(rc, "conv_bwd_data_1x1")
        elif max(stride) > 1 and (ph := _phase_plan(H, W, OH, OW, R, S, stride, pad4, dilation)) is not None and \
                all(_v3_ok(K, C, p[2], p[3]) or not fp16 for p in ph):
            dx = _bwd_data_phases(dy, w, ph, N, H, W, C, K, OH, OW, stride, dx_accum if acc else None, adt)
        elif tuple(dilation) == (1, 1) and max(stride) > 1 and pad4[0] <= R - 1 and pad4[1] <= R - 1 and \
                pad4[2] <= S - 1 and pad4[3] <= S - 1 and \
                H >= (OH - 1) * stride[0] + R - pad4[0] - pad4[1] and W >= (OW - 1) * stride[1] + S - pad4[2] - pad4[3]:
            # strided bwd-data = stride-1 transposed conv of the zero-interleaved dY (extended by the rows / cols
            # no window reached) on the MFMA kernel: s^2 more MACs than a phase-split kernel, but never the library
            sh, sw = stride
            eh = H - ((OH - 1) * sh + R - pad4[0] - pad4[1])
            ew = W - ((OW - 1) * sw + S - pad4[2] - pad4[3])
            dyz = nd4j_kernels.zero_(torch.empty((N, K, (OH - 1) * sh + 1 + eh, (OW - 1) * sw + 1 + ew), dtype=adt,
                                                 device=x.device, memory_format=torch.channels_last))
            dyz[:, :, :(OH - 1) * sh + 1:sh, :(OW - 1) * sw + 1:sw] = dy
            dx = _conv2d_bwd(x, w, dyz, (1, 1), pad4, dilation, True, False, False, dx_accum=dx_accum)[0]
        else:
            from .conv import _sym
            from .fallback import record
            import torch.nn.functional as F
            record("conv", f"bwd-data stride {tuple(stride)} kernel {R}x{S}: library path")
            sym = _sym(pad4)
            xin = x if sym else F.pad(x, (pad4[2], pad4[3], pad4[0], pad4[1]))
            padding = [pad4[0], pad4[2]] if sym else [0, 0]
            dx, _, _ = torch.ops.aten.convolution_backward(dy, xin, w, None, list(stride), padding, list(dilation),
                                                           False, [0, 0], 1, [True, False, False])
            if not sym:
                dx = dx[:, :, pad4[0]:pad4[0] + H, pad4[2]:pad4[2] + W]
    if not need_dw:
        return dx, None, None
    directw = gW is not None and gW.dtype == torch.float32 and gW.is_contiguous()
    directb = gb is not None and gb.dtype == torch.float32 and gb.is_contiguous()
    if directw and (directb or not need_db) and side_stream.active():
        # dW only writes the persistent fp32 gradient views: run it on the overlap stream next to dX
        side_stream.run(lambda: _conv2d_wrw(x, dy, N, H, W, C, K, R, S, OH, OW, stride, pad4, dilation, need_db, gW,
                                            gb, grads_zeroed, pw and gemm_dw), x, dy)
        return dx, None, None
    dW_out, db_out = _conv2d_wrw(x, dy, N, H, W, C, K, R, S, OH, OW, stride, pad4, dilation, need_db, gW, gb,
                                 grads_zeroed, pw and gemm_dw)
    return dx, dW_out, db_out


_PHASE = os.environ.get("DL4J_AMD_CONV_PHASE", "1") == "1"


def _phase_1d(n_in, n_out, R, s, p):
    """Phases of a stride-s bwd-data along one dimension. Input index i has phase f = (i + p) mod s and receives only
    the taps r = f + s*t (t < R_f = ceil((R - f) / s)) from dY rows base_f + j - t, i = i0 + s*j. Each phase is
    therefore a stride-1 transposed conv of dY with the sub-kernel w[f::s] and top pad ``base_f``. Returns
    [(i0, n_f, R_f, u0, base_f)] (u0: first tap of the sub-kernel in the flipped full kernel), or None when a phase
    needs a negative pad."""
    out = []
    for f in range(s):
        i0 = (f - p) % s
        n_f = (n_in - i0 + s - 1) // s if i0 < n_in else 0
        R_f = (R - f + s - 1) // s if f < R else 0
        base = (i0 + p - f) // s
        if n_f and R_f and R_f - 1 - base < 0:
            return None
        out.append((i0, n_f, R_f, R - 1 - f - s * (R_f - 1) if R_f else 0, base))
    return out


def _phase_plan(H, W, OH, OW, R, S, stride, pad4, dilation):
    """Phase-split plan of a strided bwd-data (s^2 stride-1 sub-problems, s^2 fewer MACs than zero-interleaving dY);
    None when it does not apply. Entries: (i0h, i0w, Rf, Sf, Hf, Wf, u0h, u0w, pad_h, pad_w) per non-empty phase."""
    if not _PHASE or tuple(dilation) != (1, 1):
        return None
    ph = _phase_1d(H, OH, R, stride[0], pad4[0])
    pw = _phase_1d(W, OW, S, stride[1], pad4[2])
    if ph is None or pw is None:
        return None
    plan = []
    for (i0h, nh, Rf, u0h, bh) in ph:
        for (i0w, nw, Sf, u0w, bw) in pw:
            if nh and nw:
                plan.append((i0h, i0w, Rf, Sf, nh, nw, u0h, u0w, Rf - 1 - bh, Sf - 1 - bw))
    return plan


def _bwd_data_phases(dy, w, plan, N, H, W, C, K, OH, OW, stride, dx_accum, adt):
    """Strided bwd-data as one stride-1 transposed conv per phase (sub-kernels sliced out of the flipped [C,R,S,K]
    weight), each written to a dense phase buffer and scattered into the strided positions of dX."""
    lib = native.load()
    sh, sw = stride
    _, flip = _relayout(w, False, True)
    zero_taps = any(p[2] == 0 or p[3] == 0 for p in plan)
    if dx_accum is not None:
        dx = dx_accum
    else:
        dx = arena.empty((N, C, H, W), adt, dy.device, channels_last=True)
        if zero_taps or len(plan) < sh * sw:
            from .nd4j_kernels import zero_
            zero_(dx)
    for (i0h, i0w, Rf, Sf, Hf, Wf, u0h, u0w, pth, ptw) in plan:
        if Rf == 0 or Sf == 0:
            continue
        sub = flip[:, u0h::sh, u0w::sw, :][:, :Rf, :Sf, :].contiguous()
        buf = torch.empty((N, C, Hf, Wf), dtype=adt, device=dy.device, memory_format=torch.channels_last)
        geo = (N, OH, OW, K, C, Rf, Sf, 1, 1, pth, ptw, 1, 1, Hf, Wf)

        def launch(var, out, _ts, sub=sub, geo=geo, Rf=Rf, Sf=Sf, pth=pth, ptw=ptw, Hf=Hf, Wf=Wf):
            if var >= 0:
                return _fwd_launch(var, dy, sub, None, out, geo, 0.0, None)
            return lib.dl4j_conv_bwd_data_s1(_ptr(dy), _ptr(sub), _ptr(out), N, Hf, Wf, C, K, Rf, Sf, Rf - 1 - pth,
                                             Sf - 1 - ptw, OH, OW, 0, _stream())
        v = -1
        if _v3_ok(K, C, Rf, Sf):
            v = _v3_pick(("bwd_phase", geo, adt), launch, buf, lambda var: None)
        native._check(launch(v, buf, None), "conv_bwd_data_phase")
        view = dx[:, :, i0h::sh, i0w::sw]
        if dx_accum is not None:
            view.add_(buf)
        else:
            view.copy_(buf)
    return dx


def _conv2d_wrw(x, dy, N, H, W, C, K, R, S, OH, OW, stride, pad4, dilation, need_db, gW, gb, grads_zeroed, use_gemm):
    """Weight (and bias) gradient of a channels-last bf16 conv; returns (dW, db), each None when it was written
    straight into the given fp32 view."""
    lib = native.load()
    dW_out = db_out = None
    if use_gemm:
        # dW[K, C] = dY^T[K, M] . X[M, C], fp32 straight into the flat-gradient view; bias = column sums of dY
        from .gemm import mmul
        M = N * H * W
        direct = gW is not None and gW.dtype == torch.float32 and gW.is_contiguous()
        dWt = gW if direct else torch.empty((K, C, R, S), dtype=torch.float32, device=x.device)
        dy_rows = dy.permute(0, 2, 3, 1).reshape(M, K)
        mmul(dy_rows.t(), x.permute(0, 2, 3, 1).reshape(M, C), out=dWt.reshape(K, C))
        dW_out = None if direct else dWt
        if need_db:
            directb = gb is not None and gb.dtype == torch.float32 and gb.is_contiguous()
            dbt = gb.reshape(-1) if directb else torch.empty(K, dtype=torch.float32, device=x.device)
            native.channel_sum(dy_rows, out=dbt)
            db_out = None if directb else dbt
        return dW_out, db_out
    direct = gW is not None and gW.dtype == torch.float32 and gW.is_contiguous()
    dWt = gW if direct else torch.empty((K, C, R, S), dtype=torch.float32, device=x.device)
    geom = (N, H, W, C, K, R, S, stride[0], stride[1], pad4[0], pad4[2], dilation[0], dilation[1], OH, OW)
    v = _wrw_pick(geom, x, dy, dWt, need_db, grads_zeroed) if V3 else ("r2",)
    if v[0] != "r2":
        # round-3 engines (tile-engine v3 / halo): per-split fp32 slabs + fixed-order reduce into the DL4J layout
        db_out = dbt = None
        if need_db:
            directb = gb is not None and gb.dtype == torch.float32 and gb.is_contiguous()
            dbt = gb.reshape(-1) if directb else torch.empty(K, dtype=torch.float32, device=x.device)
            db_out = None if directb else dbt
        native._check(_wrw_launch(v, x, dy, dWt, geom, dbt), "conv_wrw_" + v[0])
        return (None if direct else dWt), db_out
    return _conv2d_wrw_r2(x, dy, N, H, W, C, K, R, S, OH, OW, stride, pad4, dilation, need_db, gW, gb,
                          grads_zeroed, dWt, direct)


_WRW_CHOICE = {}
HALO = os.environ.get("DL4J_AMD_WRW_HALO", "1") == "1"


def _wrw_launch(choice, x, dy, dWt, geom, db=None):
    """choice: ("v3", variant) tile engine (csrc/conv_gemm.hip) or ("halo", variant, splits) halo-staged engine
    (csrc/conv_wrw.hip); returns the kernel status (-1: shape not supported)."""
    lib = native.load()
    N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW = geom
    sp = ctypes.c_int(0)
    if choice[0] == "halo":
        var, splits = choice[1], choice[2]
        nf = lib.dl4j_conv_wrw_halo_ws_floats(N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW, var, splits,
                                              ctypes.byref(sp))
        if nf <= 0:
            return -1
        ws = _det_scratch(nf, x.device)
        return lib.dl4j_conv_wrw_halo(_dtc(x), _ptr(x), _ptr(dy), _ptr(dWt), _ptr(db), _ptr(ws), *geom, var, splits,
                                      _stream())
    var = choice[1]
    nf = lib.dl4j_conv_wrw_v3_ws_floats(N, C, K, R, S, OH, OW, var, 0, ctypes.byref(sp))
    ws = _det_scratch(nf, x.device)
    return lib.dl4j_conv_wrw_v3(_dtc(x), _ptr(x), _ptr(dy), _ptr(dWt), _ptr(db), _ptr(ws), *geom, var, 0, _stream())


def _wrw_v3_launch(var, x, dy, dWt, geom, db=None):
    return _wrw_launch(("v3", var), x, dy, dWt, geom, db)


def _halo_candidates(geom):
    """Applicable halo-engine variants with their default split count and half / double of it."""
    if not HALO:
        return []
    lib = native.load()
    N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW = geom
    out = []
    for var in (1, 2, 3, 4):
        sp = ctypes.c_int(0)
        if lib.dl4j_conv_wrw_halo_ws_floats(N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW, var, 0,
                                            ctypes.byref(sp)) <= 0:
            continue
        for s in sorted({sp.value, max(1, sp.value // 2), 2 * sp.value}):
            out.append(("halo", var, s))
    return out


def _wrw_pick(geom, x, dy, dWt, need_db, grads_zeroed):
    """Per-shape weight-gradient kernel: the first eager call times the halo engine (variants x split counts), the
    round-3 tile variants and the round-2 atomic kernel (on scratch outputs, inline on this stream) and keeps the
    fastest. Deterministic mode excludes the round-2 atomic kernel. Under HIP-graph capture: the remembered choice,
    else the first halo candidate, else tile variant 0."""
    det = deterministic()
    key = (geom, det, x.dtype)
    v = _WRW_CHOICE.get(key)
    if v is not None:
        return v
    v = tunedb.lookup("conv_wrw", key)
    if v is not None:
        _WRW_CHOICE[key] = v
        return v
    lib = native.load()
    halo = _halo_candidates(geom)
    if torch.cuda.is_current_stream_capturing() or os.environ.get("DL4J_AMD_CONV_TUNE", "1") != "1":
        return halo[0] if halo else ("v3", 0)
    N, H, W, C, K, R, S, sh, sw, ph, pw, dh, dw, OH, OW = geom
    scratch = torch.empty_like(dWt)
    sdb = torch.empty(K, dtype=torch.float32, device=dWt.device) if need_db else None
    r2 = [] if det or x.dtype != torch.bfloat16 else [("r2",)]
    cands = halo + [("v3", i) for i in range(lib.dl4j_conv_wrw_v3_num_variants())] + r2
    best, bt = None, None
    with side_stream.suspended():
        for c in cands:
            if c[0] != "r2":
                def run(c=c):
                    return _wrw_launch(c, x, dy, scratch, geom, sdb)
            else:
                def run():
                    return _conv2d_wrw_r2(x, dy, N, H, W, C, K, R, S, OH, OW, (sh, sw), (ph, 0, pw, 0), (dh, dw),
                                          need_db, scratch, sdb, False, scratch, True) and 0
            if (run() or 0) != 0:
                continue
            t = _timed(run, reps=tunedb.reps(3))
            if bt is None or t < bt:
                best, bt = c, t
    v = _WRW_CHOICE[key] = best if best is not None else (("r2",) if x.dtype == torch.bfloat16 else ("v3", 0))
    tunedb.record("conv_wrw", key, v)
    return v


def _conv2d_wrw_r2(x, dy, N, H, W, C, K, R, S, OH, OW, stride, pad4, dilation, need_db, gW, gb, grads_zeroed, dWt,
                   direct):
    """Round-2 weight-gradient kernel (csrc/conv_igemm.hip): fp32 atomics into a KRSC workspace + permute, or the
    deterministic per-split slab variant."""
    lib = native.load()
    db_out = None
    if deterministic():
        # per-split fp32 slabs + fixed-order reduce straight into the DL4J layout: bitwise reproducible
        dbt = None
        if need_db:
            directb = gb is not None and gb.dtype == torch.float32 and gb.is_contiguous()
            dbt = gb.reshape(-1) if directb else torch.empty(K, dtype=torch.float32, device=x.device)
        splits = WRW_SPLITS.get((N, H, W, C, K, R, S, tuple(stride)), 0)
        nf = lib.dl4j_conv_wrw_det_floats(N, C, K, R, S, OH, OW, splits)
        part = _det_scratch(nf, x.device)
        rc = lib.dl4j_conv_wrw_det(_ptr(x), _ptr(dy), _ptr(dWt), _ptr(dbt), _ptr(part), N, H, W, C, K, R, S,
                                   stride[0], stride[1], pad4[0], pad4[2], dilation[0], dilation[1], OH, OW, splits,
                                   _stream())
        native._check(rc, "conv_wrw_det")
        db_out = None
        if need_db:
            db_out = None if (gb is not None and gb.dtype == torch.float32 and gb.is_contiguous()) else dbt
        return (None if direct else dWt), db_out
    # the kernel accumulates in [K][R][S][C]; identical to DL4J's [K][C][R][S] when R == S == 1
    if R == 1 and S == 1:
        ws = dWt
        if not (direct and grads_zeroed):
            nd4j_kernels.zero_(ws)
    else:
        ws = _zeroed_wrw_ws(K, R, S, C, x.device)
    dbt = None
    if need_db:
        directb = gb is not None and gb.dtype == torch.float32 and gb.is_contiguous()
        dbt = gb.reshape(-1) if directb else torch.empty(K, dtype=torch.float32, device=x.device)
        if not (directb and grads_zeroed):
            nd4j_kernels.zero_(dbt)
    splits = _wrw_splits(lib, x, dy, ws, dbt, N, H, W, C, K, R, S, stride, pad4, dilation, OH, OW)
    rc = lib.dl4j_conv_wrw(_ptr(x), _ptr(dy), _ptr(ws), _ptr(dbt), N, H, W, C, K, R, S, stride[0], stride[1],
                           pad4[0], pad4[2], dilation[0], dilation[1], OH, OW, splits, _stream())
    native._check(rc, "conv_wrw")
    if ws is not dWt:
        rc = lib.dl4j_conv_wrw_permute(_ptr(ws), _ptr(dWt), K, C, R, S, 1, _stream())
        native._check(rc, "conv_wrw_permute")
    dW_out = None if direct else dWt
    if need_db:
        db_out = None if (gb is not None and gb.dtype == torch.float32 and gb.is_contiguous()) else dbt
    return dW_out, db_out


def _wrw_default_splits(M, K, RSC):
    """Mirror of dl4j_conv_wrw's split heuristic (~1.5 workgroups per CU, >= 8 k-steps per split)."""
    tiles = ((K + 127) // 128) * ((RSC + 127) // 128)
    maxs = max(1, (M + 8 * 32 - 1) // (8 * 32))
    return max(1, min((384 + tiles - 1) // tiles, maxs)), maxs


def _wrw_splits(lib, x, dy, ws, dbt, N, H, W, C, K, R, S, stride, pad4, dilation, OH, OW):
    """Per-shape pixel-split count of the weight-gradient kernel. The first eager call of a shape times the heuristic
    count and its neighbours (x0.5, x2, x4: fill vs fp32-atomic epilogue traffic trade differently per shape) on a
    scratch accumulator and keeps the fastest; graph-captured calls use the remembered value (heuristic if none)."""
    key = (N, H, W, C, K, R, S, tuple(stride))
    sp = WRW_SPLITS.get(key)
    if sp is not None:
        return sp
    if torch.cuda.is_current_stream_capturing() or os.environ.get("DL4J_AMD_CONV_TUNE", "1") != "1":
        return 0
    s0, maxs = _wrw_default_splits(N * OH * OW, K, R * S * C)
    cands = sorted({c for c in (s0 // 2, s0, 2 * s0, 4 * s0) if 1 <= c <= maxs})
    scratch = torch.zeros_like(ws)
    sdb = torch.zeros_like(dbt) if dbt is not None else None

    def run(c):
        return lambda: native._check(
            lib.dl4j_conv_wrw(_ptr(x), _ptr(dy), _ptr(scratch), _ptr(sdb), N, H, W, C, K, R, S, stride[0], stride[1],
                              pad4[0], pad4[2], dilation[0], dilation[1], OH, OW, c, _stream()), "conv_wrw")
    best = min(cands, key=lambda c: _timed(run(c), reps=3))
    WRW_SPLITS[key] = best
    return best


GEMM_1X1 = os.environ.get("DL4J_AMD_CONV1X1_GEMM", "1") == "1"


def _is_pointwise(R, S, stride, pad4, dilation):
    return R == 1 and S == 1 and tuple(stride) == (1, 1) and not any(pad4) and tuple(dilation) == (1, 1)


# ------------------------------------------------------------------ per-shape choice: GEMM vs implicit-GEMM kernel
# A 1x1 stride-1 conv runs either as a plain GEMM (ops/gemm.py) or on the implicit-GEMM conv kernels; which one is
# faster depends on the shape (small K/N layers are streaming-bound and favour different tiles). The first eager
# call of each (direction, shape) times both on scratch outputs and remembers the winner; calls made while a HIP
# graph is being captured use the remembered choice (GEMM when none).
_CHOICE = {}


def _timed(fn, reps=2):
    """GPU milliseconds per call with the host enqueue hidden (ops/timing.py)."""
    from .timing import gpu_time
    return gpu_time(fn, reps=reps)


def _choose(key, run_gemm, run_old):
    c = _CHOICE.get(key)
    if c is None:
        if not GEMM_1X1:
            return False
        c = tunedb.lookup("conv_1x1", key)
        if c is not None:
            _CHOICE[key] = c
            return c
        if torch.cuda.is_current_stream_capturing() or os.environ.get("DL4J_AMD_CONV_TUNE", "1") != "1":
            return True
        # candidates run inline on this stream: on the overlap stream they would still be writing their scratch
        # outputs after those are freed, and the main-stream timing events would not cover them
        with side_stream.suspended():
            tg, to = _timed(run_gemm, reps=tunedb.reps(2)), _timed(run_old, reps=tunedb.reps(2))
        c = _CHOICE[key] = tg <= to
        tunedb.record("conv_1x1", key, c)
    return c


def _pad_ch(t, n, dim=1, cl=False):
    """Zero-pad dim ``dim`` (channels of a 4-D activation with ``cl``=channels-last, or a weight's K / C dim)
    up to ``n``."""
    if t.shape[dim] == n:
        return t
    if cl and dim == 1 and t.dim() == 4 and t.is_cuda:
        y = nd4j_kernels.channels_last_copy(t, n)                   # pad + layout in one in-tree launch
        if y is not None:
            return y
    shp = list(t.shape)
    shp[dim] = n
    out = nd4j_kernels.zero_(torch.empty(shp, dtype=t.dtype, device=t.device,
                                         memory_format=torch.channels_last if cl else torch.contiguous_format))
    out.narrow(dim, 0, t.shape[dim]).copy_(t)
    return out


def _r8(n):
    return (n + 7) // 8 * 8


def _rq(n, q):
    return (n + q - 1) // q * q


def _stem_case(x, w, b, stride, pad4, dilation):
    if x.shape[1] != 3 or os.environ.get("DL4J_AMD_KERNEL_STEM", "1") != "1":
        return False
    from . import conv_stem
    return conv_stem.supported(_cl(x), w, b, stride, pad4, dilation)


def conv2d_fwd(x, w, b, stride, pad4, dilation, want_stats=False):
    """want_stats: also emit per-tile BatchNorm statistics of the output from the kernel epilogue; they are attached
    to the result as ``y._bn_tile_stats = (planes [3, P, K] fp32, P)`` for a consuming training-mode BN layer.
    Input channel counts that are not a multiple of 8 (RGB / small first layers: AlexNet, LeNet, GoogLeNet stems)
    are zero-padded to the next multiple of 8 so they still run on the MFMA kernels (exact: zero channels add 0)."""
    if _ok_act(x) and x.dim() == 4 and w.dim() == 4 and w.dtype == x.dtype and x.shape[1] == w.shape[1] \
            and x.shape[1] % _q(x) and not (x.dtype == torch.bfloat16 and _stem_case(x, w, b, stride, pad4, dilation)):
        C8 = _rq(x.shape[1], _q(x))
        return conv2d_fwd(_pad_ch(_cl(x), C8, cl=True), _pad_ch(w, C8), b, stride, pad4, dilation, want_stats)
    if _ok_act(x) and x.dim() == 4 and w.dim() == 4 and w.dtype == x.dtype and w.shape[0] % (4 if x.dtype ==
                                                                                               torch.bfloat16 else 8):
        K = w.shape[0]
        K8 = _r8(K)
        bp = _pad_ch(b.reshape(-1), K8, 0) if b is not None else None
        y = conv2d_fwd(x, _pad_ch(w, K8, 0), bp, stride, pad4, dilation, want_stats)
        if y is None:
            return None
        out = y[:, :K].contiguous(memory_format=torch.channels_last)
        if hasattr(y, "_bn_tile_stats"):
            ts, P = y._bn_tile_stats
            out._bn_tile_stats = (ts[:, :, :K].contiguous(), P)
        return out
    use = True
    if _ok_act(x) and x.dim() == 4 and w.dim() == 4 and w.shape[2] == 1 and w.shape[3] == 1 and \
            _is_pointwise(1, 1, stride, pad4, dilation):
        key = ("fwd", tuple(x.shape), tuple(w.shape), b is not None, bool(want_stats), x.dtype)
        use = _choose(key, lambda: _conv2d_fwd(x, w, b, stride, pad4, dilation, want_stats, True),
                      lambda: _conv2d_fwd(x, w, b, stride, pad4, dilation, want_stats, False))
    return _conv2d_fwd(x, w, b, stride, pad4, dilation, want_stats, use)


def conv2d_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db, gW=None, gb=None, grads_zeroed=False,
               dx_accum=None):
    """grads_zeroed: the caller guarantees gW/gb (flat-gradient views) are already zero (the network clears the
    whole flat gradient with one fill per step), so no per-layer memset is launched.
    dx_accum: an existing channels-last bf16 gradient of x (another consumer's contribution); when the bwd-data
    kernel can take it, the result is accumulated into it in the kernel epilogue and it is returned as dx.
    Channel counts (C or K) that are not a multiple of 8 are zero-padded (see ``conv2d_fwd``); the padded weight
    gradient is cropped into ``gW``."""
    if _ok_act(x) and _ok_act(dy) and x.dim() == 4 and w.dim() == 4 and w.dtype == x.dtype and \
            x.shape[1] == w.shape[1] and (x.shape[1] % _q(x) or w.shape[0] % _q(x)) and \
            not (x.dtype == torch.bfloat16 and x.shape[1] == 3 and not need_dx and
                 _stem_case(x, w, None, stride, pad4, dilation)):
        return _conv2d_bwd_padded(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db, gW, gb, dx_accum)
    gdx = gdw = True
    if _ok_act(x) and _ok_act(dy) and w.dim() == 4 and w.shape[2] == 1 and w.shape[3] == 1 and \
            _is_pointwise(1, 1, stride, pad4, dilation):
        shp = (tuple(x.shape), tuple(w.shape), x.dtype)
        # scratch copies / buffers are made inside the candidates, i.e. only on the one timed call per shape
        # (an unconditional clone of dx_accum here was a full-activation copy per conv per step)
        def _acc_copy():
            return dx_accum.clone() if dx_accum is not None else None
        if need_dx:
            gdx = _choose(("dx", shp, dx_accum is not None),
                          lambda: _conv2d_bwd(x, w, dy, stride, pad4, dilation, True, False, False,
                                              dx_accum=_acc_copy(), gemm_dx=True),
                          lambda: _conv2d_bwd(x, w, dy, stride, pad4, dilation, True, False, False,
                                              dx_accum=_acc_copy(), gemm_dx=False))
        if need_dw:
            K, C = w.shape[0], w.shape[1]

            def _sw():
                return torch.zeros((K, C, 1, 1), dtype=torch.float32, device=x.device)

            def _sb():
                return torch.zeros((K,), dtype=torch.float32, device=x.device) if need_db else None
            gdw = _choose(("dw", shp, need_db),
                          lambda: _conv2d_bwd(x, w, dy, stride, pad4, dilation, False, True, need_db, _sw(), _sb(),
                                              True, gemm_dw=True),
                          lambda: _conv2d_bwd(x, w, dy, stride, pad4, dilation, False, True, need_db, _sw(), _sb(),
                                              True, gemm_dw=False))
    return _conv2d_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db, gW, gb, grads_zeroed, dx_accum,
                       gdx, gdw)


def _conv2d_bwd_padded(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db, gW, gb, dx_accum):
    K, C = w.shape[0], w.shape[1]
    C8, K8 = _rq(C, _q(x)), _rq(K, _q(x))
    xp = _pad_ch(_cl(x), C8, cl=True)
    wp = _pad_ch(_pad_ch(w, C8, 1), K8, 0)
    dyp = _pad_ch(_cl(dy), K8, cl=True)
    r = conv2d_bwd(xp, wp, dyp, stride, pad4, dilation, need_dx, need_dw, need_db)
    if r is None:
        return None
    dx, dW, db = r
    if dx is not None:
        dx = dx[:, :C].contiguous(memory_format=torch.channels_last)
        if dx_accum is not None:
            dx = dx_accum.add_(dx)
    if dW is not None:
        dW = dW[:K, :C]
        if gW is not None:
            gW.copy_(dW.reshape(gW.shape))
            dW = None
    if db is not None:
        db = db[:K]
        if gb is not None:
            gb.copy_(db.reshape(gb.shape))
            db = None
    return dx, dW, db


def _out_hw_inv(OH, OW, R, S, pad4, H, W):
    """For stride 1: the input size that the transposed conv reproduces (must equal H, W)."""
    pt, pb, pl, pr = pad4
    return OH - 1 + R - pt - pb, OW - 1 + S - pl - pr


_ = ctypes
