"""ctypes bindings of ``libdl4j_amd_kernels.so`` (gfx950 HIP kernels, C ABI) + torch-facing wrappers.

Every wrapper launches on torch's current HIP stream (so HIP-graph capture and stream ordering work),
allocates outputs/workspaces through torch's caching allocator, and returns ``None`` when a shape is
outside what the kernel supports (the caller then uses the torch/library path).
"""
import ctypes
import os

import threading

import numpy as np
import torch

from .build import KERNEL_LIB

_lib = None
c_void_p, c_int, c_ll, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(KERNEL_LIB):
        if os.environ.get("DL4J_AMD_AUTOBUILD", "1") == "1":
            from .build import build_kernels
            build_kernels(verbose=False)
        else:
            raise FileNotFoundError(KERNEL_LIB)
    lib = ctypes.CDLL(KERNEL_LIB)
    sigs = {
        "dl4j_fused_update": [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float,
                              c_int, c_void_p, c_void_p, c_void_p],
        "dl4j_update_chunk": [],
        "dl4j_segdesc_size": [],
        "dl4j_bn_workspace_floats": [c_ll, c_int],
        "dl4j_bn_fwd": [c_int, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p, c_void_p, c_float, c_float,
                        c_void_p, c_void_p, c_float, c_float, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
        "dl4j_bn_bwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p, c_void_p,
                        c_void_p, c_int, c_void_p, c_void_p, c_void_p],
        "dl4j_softmax_xent": [c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_float,
                              c_void_p],
        "dl4j_pool_fwd": [c_int, c_int, c_void_p, c_void_p, c_void_p] + [c_int] * 12 + [c_void_p],
        "dl4j_pool_bwd": [c_int, c_int, c_void_p, c_void_p, c_void_p] + [c_int] * 12 + [c_void_p],
    }
    for name, args in sigs.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = c_int
    for name, (args, restype) in _EXTRA_SIGS.items():
        if hasattr(lib, name):
            f = getattr(lib, name)
            f.argtypes = args
            f.restype = restype
    _lib = lib
    return lib


_EXTRA_SIGS = {}


def register_sig(name, args, restype=c_int):
    _EXTRA_SIGS[name] = (args, restype)
    if _lib is not None and hasattr(_lib, name):
        f = getattr(_lib, name)
        f.argtypes = args
        f.restype = restype


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_dev = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """Handle of the current HIP stream (the one torch.cuda.current_stream() names, incl. stream contexts and graph
    capture): two C calls instead of the Python stream object — kernel launches pay this on every call."""
    if _raw_stream is not None and _cur_dev is not None:
        return _raw_stream(_cur_dev())
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_CAPTURE_DEBUG = os.environ.get("DL4J_AMD_CAPTURE_DEBUG", "0") == "1"
_hip = None


def capture_status():
    """hipStreamIsCapturing of torch's current stream: 0 none, 1 active, 2 invalidated."""
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipStreamIsCapturing.argtypes = [c_void_p, ctypes.POINTER(c_int)]
    st = c_int(0)
    _hip.hipStreamIsCapturing(c_void_p(_stream()), ctypes.byref(st))
    return st.value


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"HIP kernel {what} failed with code {rc}")
    if _CAPTURE_DEBUG and capture_status() == 2:
        raise RuntimeError(f"stream capture invalidated at/after native call {what}")


def _dt(t):
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    return None


def _as_rows_nhwc(x):
    """View a 4-D channels-last (or 2-D row-major) tensor as [M, C] rows without copying; None if impossible."""
    if x.dim() == 2:
        return x if x.is_contiguous() else None
    if x.dim() == 4:
        if x.is_contiguous(memory_format=torch.channels_last):
            return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1])
        return None
    return None


def _ae(shape, dtype, device, channels_last=False):
    """Per-iteration buffer from the open training workspace (memory/arena.py; the LOOP_FF_BP arena, or a captured
    HIP graph's own arena), else from the caching allocator."""
    from ..memory import arena
    return arena.empty(tuple(shape), dtype, device, channels_last=channels_last)


def _like_rows(x):
    return _ae(x.shape, x.dtype, x.device, channels_last=x.dim() == 4)


# ------------------------------------------------------------------------------------ fused updater
class _SegTableCache:
    """Device copy of the updater's per-segment table. Eager: refreshed (pinned host -> device, async) only when
    the hyperparameters change (schedules, Adam bias correction). Under HIP-graph capture each graph gets its own
    pinned/device slot; the captured graph contains the copy from that slot's pinned buffer, so updating the
    pinned bytes before a replay feeds the new iteration's hyperparameters into the graph."""

    def __init__(self):
        self.slots = {}
        self.btab = None
        self.nblocks = 0


class _Slot:
    def __init__(self, nbytes, device):
        self.pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.bytes = None
        self.event = None     # completes when the last copy out of ``pinned`` has finished


_SEG_DTYPE = np.dtype([("p_off", "<i8"), ("n", "<i8"), ("st_off", "<i8"), ("in_block", "<i8"), ("block_n", "<i8"),
                       ("op", "<i4"), ("pad", "<i4"), ("h", "<f4", 4), ("l1", "<f4"), ("l2", "<f4"),
                       ("gn_mode", "<i4"), ("gn_b0", "<i4"), ("gn_b1", "<i4"), ("gn_thr", "<f4")])


def _gn_block_ranges(plan, chunk):
    """Per segment: the [first, last) update-block range (btab rows) of its gradient-normalization group."""
    cached = plan.__dict__.get("_gn_ranges")
    if cached is not None and cached[0] == chunk:
        return cached[1]
    first, b = [], 0
    for sg in plan.segments:
        first.append(b)
        b += (sg.n + chunk - 1) // chunk
    first.append(b)
    span = {}
    for i, sg in enumerate(plan.segments):
        key = sg.gn_group if sg.gn_group is not None else ("seg", i)
        lo, hi = span.get(key, (first[i], first[i + 1]))
        span[key] = (min(lo, first[i]), max(hi, first[i + 1]))
    ranges = [span[sg.gn_group if sg.gn_group is not None else ("seg", i)] for i, sg in enumerate(plan.segments)]
    plan._gn_ranges = (chunk, ranges)
    return ranges

class _ThreadSlot(threading.local):
    """``GRAPH_SLOT[0]``: the graph slot THIS host thread is capturing (None = eager). Thread-local, so the
    in-process ParallelWrapper's workers (one thread per GPU) can capture their replicas' steps concurrently
    without seeing each other's slot."""

    def __init__(self):
        self.v = None

    def __getitem__(self, i):
        if i != 0:
            raise IndexError(i)
        return self.v

    def __setitem__(self, i, val):
        if i != 0:
            raise IndexError(i)
        self.v = val


# graph slot currently being captured / replayed by this thread (None = eager)
GRAPH_SLOT = _ThreadSlot()


def seg_table_bytes(plan, iteration, epoch):
    from ..nn.conf.updaters import kernel_params
    segs = plan.segments
    arr = np.zeros(len(segs), dtype=_SEG_DTYPE)
    ranges = _gn_block_ranges(plan, load().dl4j_update_chunk())
    for i, s in enumerate(segs):
        op, h0, h1, h2, h3 = kernel_params(s.updater, iteration, epoch)
        arr[i] = (s.p_off, s.n, s.st_off, s.in_block, s.block_n, op, 0, (h0, h1, h2, h3), s.l1, s.l2,
                  getattr(s, "gn_mode", 0), ranges[i][0], ranges[i][1], getattr(s, "gn_thr", 1.0))
    return arr.tobytes()


def _slot(cache, key, nbytes, device):
    st = cache.slots.get(key)
    if st is None or st.dev.numel() != nbytes or st.dev.device != device:
        st = _Slot(nbytes, device)
        cache.slots[key] = st
    return st


def _write_pinned(st, b):
    if st.event is not None:
        st.event.synchronize()          # the previous async copy out of this pinned buffer has finished
    st.pinned.numpy()[:] = np.frombuffer(b, dtype=np.uint8)
    st.bytes = b


def prepare_graph_slots(plan, device, iteration, epoch, nslots=2):
    """Allocate the pinned/device table slots BEFORE capture (pinned host allocation is not capturable)."""
    cache = plan.__dict__.setdefault("_native_cache", _SegTableCache())
    b = seg_table_bytes(plan, iteration, epoch)
    for k in range(nslots):
        st = _slot(cache, ("graph", k), len(b), device)
        _write_pinned(st, b)


def refresh_graph_table(plan, slot, iteration, epoch):
    """Before replaying graph ``slot``: put this iteration's hyperparameters into its pinned buffer."""
    cache = plan.__dict__.get("_native_cache")
    st = cache.slots[("graph", slot)]
    b = seg_table_bytes(plan, iteration, epoch)
    if b != st.bytes:
        _write_pinned(st, b)


def mark_graph_replayed(plan, slot):
    cache = plan.__dict__.get("_native_cache")
    st = cache.slots[("graph", slot)]
    if st.event is None:
        st.event = torch.cuda.Event()
    st.event.record()


def fused_update(plan, params, grad, state, iteration, epoch, div, shadow, write_update, reg_out=None):
    lib = load()
    if lib.dl4j_segdesc_size() != _SEG_DTYPE.itemsize:
        raise RuntimeError("SegDesc layout mismatch between python and HIP")
    segs = plan.segments
    b = seg_table_bytes(plan, iteration, epoch)
    cache = plan.__dict__.setdefault("_native_cache", _SegTableCache())
    gslot = GRAPH_SLOT[0]
    if gslot is None:
        st = _slot(cache, "eager", len(b), params.device)
        if st.bytes != b:
            _write_pinned(st, b)
            st.dev.copy_(st.pinned, non_blocking=True)
            if st.event is None:
                st.event = torch.cuda.Event()
            st.event.record()
    else:                                  # capturing: the copy from this slot's pinned buffer is a graph node
        st = cache.slots.get(("graph", gslot))
        if st is None or st.dev.numel() != len(b):
            raise RuntimeError("graph table slot not prepared before capture (prepare_graph_slots)")
        if st.bytes != b:
            st.pinned.numpy()[:] = np.frombuffer(b, dtype=np.uint8)
            st.bytes = b
        st.dev.copy_(st.pinned, non_blocking=True)
    if cache.btab is None or cache.btab.device != params.device:
        chunk = lib.dl4j_update_chunk()
        rows = [(si, ci) for si, s in enumerate(segs) for ci in range((s.n + chunk - 1) // chunk)]
        cache.btab = torch.tensor(rows if rows else [(0, 0)], dtype=torch.int32).to(params.device)
        cache.nblocks = len(rows)
    sk = 0
    if shadow is not None:
        sk = {torch.bfloat16: 1, torch.float16: 2}.get(shadow.dtype)
        if sk is None:
            return False
    gn_part = None
    if any(getattr(sg, "gn_mode", 0) in (1, 2, 4, 5) for sg in segs):
        gn_part = getattr(cache, "gn_partial", None)
        if gn_part is None or gn_part.numel() < cache.nblocks or gn_part.device != params.device:
            gn_part = cache.gn_partial = torch.empty(max(cache.nblocks, 1), dtype=torch.float32,
                                                     device=params.device)
    reg_part = None
    if reg_out is not None:
        # per-block regularisation partials, summed in a fixed order below: a reproducible score (no float atomics)
        reg_part = getattr(cache, "reg_partial", None)
        if reg_part is None or reg_part.numel() < cache.nblocks or reg_part.device != params.device:
            reg_part = cache.reg_partial = torch.empty(max(cache.nblocks, 1), dtype=torch.float32,
                                                       device=params.device)
        register_sig("dl4j_fused_update_regpart", [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                                   c_int, c_float, c_int, c_void_p, c_void_p, c_void_p])
        rc = lib.dl4j_fused_update_regpart(_ptr(st.dev), _ptr(cache.btab), cache.nblocks, _ptr(params), _ptr(grad),
                                           _ptr(state), _ptr(shadow), sk, 1.0 / div, 1 if write_update else 0,
                                           _ptr(reg_part), _ptr(gn_part), _stream())
        _check(rc, "fused_update")
        score_reduce(reg_part[:cache.nblocks], 0.0, 1.0, out=reg_out.reshape(-1)[:1])
    else:
        rc = lib.dl4j_fused_update(_ptr(st.dev), _ptr(cache.btab), cache.nblocks, _ptr(params), _ptr(grad),
                                   _ptr(state), _ptr(shadow), sk, 1.0 / div, 1 if write_update else 0, None,
                                   _ptr(gn_part), _stream())
        _check(rc, "fused_update")
    from . import rnn_native
    rnn_native.check_step_guard(params.device)     # a timed-out cooperative LSTM launch skips the update: report it
    return True


def score_reduce(s, add, scale, reg=None, reg_scale=0.0, out=None):
    """out[0] = (sum(s) + add) * scale + reg[0] * reg_scale on one HIP block (fixed order; csrc/softmax_xent.hip).
    s: contiguous fp32 CUDA tensor; returns ``out`` (a fresh 0-d tensor when not given)."""
    lib = load()
    register_sig("dl4j_score_reduce", [c_void_p, c_ll, c_float, c_float, c_void_p, c_float, c_void_p, c_void_p])
    if out is None:
        out = torch.empty((), dtype=torch.float32, device=s.device)
    rc = lib.dl4j_score_reduce(_ptr(s), s.numel(), float(add), float(scale), _ptr(reg), float(reg_scale), _ptr(out),
                               _stream())
    _check(rc, "score_reduce")
    return out


def score_reduce_ok(*ts):
    return all(t is None or (torch.is_tensor(t) and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous())
               for t in ts) and load() is not None


# ------------------------------------------------------------------------------------------ batch norm
def _rows_like(t, ref):
    """``t`` as [M, C] rows in the same memory layout as ``ref`` (converting if needed)."""
    if t.dim() == 4 and not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    elif t.dim() == 2 and not t.is_contiguous():
        t = t.contiguous()
    return t.to(ref.dtype)


def bn_fwd(x, gamma, beta, run_mean, run_var, training, decay, eps, relu, residual=None, rctx=None,
           stats_only=False):
    """``stats_only``: training statistics + running-stat update + context, no output (a shortcut BN whose apply
    the residual consumer does: returns (x, ctx)). ``rctx``: that shortcut BN's context — ``residual`` is then its
    raw input and the apply computes relu(bn(x) + bn_r(residual))."""
    dt = _dt16(x)
    xr = _as_rows_nhwc(x) if dt is not None else None
    if xr is None:
        return None
    M, C = xr.shape
    if C % 8 != 0 or C // 8 > 256 or run_mean.dtype != torch.float32:
        return None
    if (stats_only or rctx is not None) and not (training and dt in (1, 2)):
        return None
    lib = load()
    if rctx is not None:
        return _bn_fwd_rbn(lib, x, xr, dt, M, C, gamma, beta, run_mean, run_var, decay, eps, residual, rctx)
    y = None if stats_only else _like_rows(x)
    ws = _ae((lib.dl4j_bn_workspace_floats(M, C),), torch.float32, x.device)
    ctx = _ae((4 * C,), torch.float32, x.device)
    g = gamma if torch.is_tensor(gamma) else None
    b = beta if torch.is_tensor(beta) else None
    res = _rows_like(residual, x) if residual is not None else None
    # training with a fused residual: bn_apply writes the ReLU bitmask (1 bit per element) so the backward pass
    # never re-reads the residual
    mask = _ae((M * C // 8,), torch.uint8, x.device) if res is not None and training else None
    ts = getattr(x, "_bn_tile_stats", None)
    rpp = _tile_rpp(ts, M, C) if training and dt in (1, 2) else None
    if rpp is not None:
        # statistics already reduced per tile by the producing conv kernel's epilogue
        register_sig("dl4j_bn_fwd_tiles", [c_int, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p, c_ll, c_int,
                                           c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p, c_float, c_float,
                                           c_int, c_void_p, c_void_p, c_void_p, c_void_p])
        register_sig("dl4j_bn_tiles_workspace_floats", [c_ll, c_int])
        lib.dl4j_bn_tiles_workspace_floats.restype = c_ll
        wst = _ae((lib.dl4j_bn_tiles_workspace_floats(ts[1], C),), torch.float32, x.device)
        rc = lib.dl4j_bn_fwd_tiles(dt, _ptr(xr), _ptr(res), _ptr(y), M, C, _ptr(ts[0]), ts[1], rpp, _ptr(g), _ptr(b),
                                   float(gamma) if g is None else 1.0, float(beta) if b is None else 0.0,
                                   _ptr(run_mean), _ptr(run_var), float(decay), float(eps), 1 if relu else 0,
                                   _ptr(wst), _ptr(ctx), _ptr(mask), _stream())
        _check(rc, "bn_fwd_tiles")
        if stats_only:
            return x, ("NATIVE_STATS", x, ctx, False, M, C, None, None)
        _bnb_request(y, xr, ctx, relu, res, mask, training, dt)
        return y, ("NATIVE", x, ctx, relu, M, C, res, mask)
    rc = lib.dl4j_bn_fwd(dt, _ptr(xr), _ptr(res), _ptr(y), M, C, _ptr(g), _ptr(b),
                         float(gamma) if g is None else 1.0, float(beta) if b is None else 0.0, _ptr(run_mean),
                         _ptr(run_var), float(decay), float(eps), 1 if training else 0, 1 if relu else 0, _ptr(ws),
                         _ptr(ctx), _ptr(mask), _stream())
    _check(rc, "bn_fwd")
    if stats_only:
        return x, ("NATIVE_STATS", x, ctx, False, M, C, None, None)
    _bnb_request(y, xr, ctx, relu, res, mask, training, dt)
    return y, ("NATIVE", x, ctx, relu, M, C, res, mask)


def _tile_rpp(ts, M, C):
    """Rows per partial of a producer's BN tile statistics ``(planes [3, P, C], P[, rpp])`` that cover the M rows of
    this BN input, else None: 64-row partials (the implicit-GEMM / GEMM epilogues, P = 2 * ceil(M / 128)) or one
    partial per chunk of rpp rows (dl4j_conv_halo, P = ceil(M / rpp))."""
    if ts is None or ts[0].shape[2] != C:
        return None
    rpp = ts[2] if len(ts) > 2 else 64
    if rpp == 64:
        return 64 if ts[1] == 2 * ((M + 127) // 128) else None
    return rpp if ts[1] == (M + rpp - 1) // rpp else None


def _bn_fwd_rbn(lib, x, xr, dt, M, C, gamma, beta, run_mean, run_var, decay, eps, residual, rctx):
    """Residual BN apply with the shortcut BN folded in (csrc/batchnorm.hip dl4j_bn_fwd_rbn)."""
    y = _like_rows(x)
    ctx = _ae((4 * C,), torch.float32, x.device)
    g = gamma if torch.is_tensor(gamma) else None
    b = beta if torch.is_tensor(beta) else None
    res = _rows_like(residual, x)
    mask = _ae((M * C // 8,), torch.uint8, x.device)
    ts = getattr(x, "_bn_tile_stats", None)
    rpp = _tile_rpp(ts, M, C)
    tiles = rpp is not None
    register_sig("dl4j_bn_fwd_rbn", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p, c_void_p,
                                     c_float, c_float, c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_ll, c_int, c_void_p])
    if tiles:
        register_sig("dl4j_bn_tiles_workspace_floats", [c_ll, c_int])
        lib.dl4j_bn_tiles_workspace_floats.restype = c_ll
        ws = _ae((lib.dl4j_bn_tiles_workspace_floats(ts[1], C),), torch.float32, x.device)
    else:
        ws = _ae((lib.dl4j_bn_workspace_floats(M, C),), torch.float32, x.device)
    rc = lib.dl4j_bn_fwd_rbn(dt, _ptr(xr), _ptr(res), _ptr(rctx), _ptr(y), M, C, _ptr(g), _ptr(b),
                             float(gamma) if g is None else 1.0, float(beta) if b is None else 0.0, _ptr(run_mean),
                             _ptr(run_var), float(decay), float(eps), _ptr(ws), _ptr(ctx), _ptr(mask),
                             _ptr(ts[0]) if tiles else None, ts[1] if tiles else 0, rpp if tiles else 0, _stream())
    _check(rc, "bn_fwd_rbn")
    return y, ("NATIVE", x, ctx, True, M, C, res, mask, rctx)


# ------------------------------------------------------------------ BN backward sums from the producer's epilogue
# A training BN layer tags its output with ``_bn_bwd_req = (x rows, ctx, relu, mask)`` (mask: the forward's ReLU
# bitmask of a layer with a fused residual). The conv / GEMM that consumes that output computes, in the epilogue of its
# backward-data launch, the BN backward partial sums of the dX it stores (csrc/mfma_tile.h epi_bnbwd_wave; when it sums
# into another consumer's gradient, of the stored sum) and tags dX with ``_bn_bwd_stats``; bn_bwd then folds those
# planes (dl4j_bn_bwd_planes) instead of re-reading dy and x in bn_bwd_partial. A later contribution to that gradient
# (a kernel summing into it drops the tag; a torch sum makes a new, untagged tensor), an in-place edit (version
# counter), or a layout the kernels do not take leaves no valid tag, and the full backward runs.
# DL4J_AMD_BN_BWD_EPILOGUE: 0 off (default), 1 plain BN layers only (no fused residual, no fan-out sum), 2 also residual
# layers and summed gradients (their epilogue reads the old sum and the mask besides x: no less traffic than
# bn_bwd_partial). Off by default: on the ResNet-50 bench (bf16, batch 512) mode 0 / 1 / 2 measured 31.1k / 30.5k /
# 29.1k images/s (profiles/r3_bench_bnbmode*.log) — bn_bwd_partial already streams at ~5 TB/s, and the epilogue's
# exposed load latency costs more than the dy re-read it saves.
BNB_MODE = int(os.environ.get("DL4J_AMD_BN_BWD_EPILOGUE", "0") or 0)
BNB = BNB_MODE > 0


def _bnb_request(y, xr, ctx, relu, res, mask, training, dt):
    if BNB and training and (res is None or (mask is not None and BNB_MODE >= 2)) and dt in (1, 2) and \
            xr.dim() == 2:
        y._bn_bwd_req = (xr, ctx, bool(relu), mask)


class bnb_armed:
    """Context manager: arms the BN-backward epilogue (dl4j_bnb_arm) for the GEMM / conv launches in its body that
    pass a statistics buffer; always disarmed on exit."""

    def __init__(self, req):
        self.req = req

    def __enter__(self):
        register_sig("dl4j_bnb_arm", [c_void_p, c_void_p, c_void_p, c_int])
        xr, ctx, relu, mask = self.req
        load().dl4j_bnb_arm(_ptr(xr), _ptr(ctx), _ptr(mask), 3 if mask is not None else (2 if relu else 1))
        return self

    def __exit__(self, *exc):
        load().dl4j_bnb_arm(None, None, None, 0)
        return False


def bnb_tag(dx, planes, req):
    """Marks dx as carrying BN-backward planes for the BN layer whose forward context is req[1]."""
    dx._bn_bwd_stats = (planes, req[1], planes.shape[1], dx._version)


def _bnb_planes(dy, c, res, M, C, mask=None):
    st = getattr(dy, "_bn_bwd_stats", None)
    if st is None or (res is not None and mask is None):
        return None
    planes, ctx_t, P, ver = st
    if ctx_t is not c or ver != dy._version or P != (M + 63) // 64 or tuple(planes.shape) != (2, P, C):
        return None
    return planes


def bn_bwd(dy, ctx, dgamma_out=None, dbeta_out=None, rgrads=None):
    """``rgrads``: (dgamma, dbeta) outputs of the folded-in shortcut BN (ctx from _bn_fwd_rbn); dres is then the
    gradient w.r.t. that BN's input. Returns (dx, dgamma, dbeta, dres) and, with rgrads, fills them."""
    _, x, c, relu, M, C, res, mask = ctx[:8]
    rctx = ctx[8] if len(ctx) > 8 else None
    planes = _bnb_planes(dy, c, res, M, C, mask) if rctx is None else None
    dy = _rows_like(dy, x)
    lib = load()
    dx = _like_rows(x)
    dres = _like_rows(x) if res is not None else None
    ok = lambda t: t is not None and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == C  # noqa
    dgamma = dgamma_out if ok(dgamma_out) else _ae((C,), torch.float32, x.device)
    dbeta = dbeta_out if ok(dbeta_out) else _ae((C,), torch.float32, x.device)
    if rctx is not None:
        rg = rgrads if rgrads is not None else (None, None)
        dg2 = rg[0] if ok(rg[0]) else _ae((C,), torch.float32, x.device)
        db2 = rg[1] if ok(rg[1]) else _ae((C,), torch.float32, x.device)
        register_sig("dl4j_bn_bwd_rbn_workspace_floats", [c_ll, c_int])
        lib.dl4j_bn_bwd_rbn_workspace_floats.restype = c_ll
        register_sig("dl4j_bn_bwd_rbn", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p])
        ws = _ae((lib.dl4j_bn_bwd_rbn_workspace_floats(M, C),), torch.float32, x.device)
        rc = lib.dl4j_bn_bwd_rbn(_dt16(x), _ptr(x), _ptr(res), _ptr(dy), _ptr(dx), _ptr(dres), M, C, _ptr(c),
                                 _ptr(dgamma), _ptr(dbeta), _ptr(rctx), _ptr(dg2), _ptr(db2), _ptr(ws), _ptr(mask),
                                 _stream())
        _check(rc, "bn_bwd_rbn")
        if rgrads is not None:
            for dst, src in zip(rgrads, (dg2, db2)):
                if dst is not None and dst is not src:
                    dst.copy_(src.reshape(dst.shape))
        return dx, dgamma, dbeta, dres
    if planes is not None:
        register_sig("dl4j_bn_bwd_planes_workspace_floats", [c_ll, c_int])
        lib.dl4j_bn_bwd_planes_workspace_floats.restype = c_ll
        register_sig("dl4j_bn_bwd_planes", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int,
                                            c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_ll, c_void_p, c_void_p])
        P = planes.shape[1]
        ws = _ae((lib.dl4j_bn_bwd_planes_workspace_floats(P, C),), torch.float32, x.device)
        rc = lib.dl4j_bn_bwd_planes(_dt16(x), _ptr(x), _ptr(dy), _ptr(dx), _ptr(dres), _ptr(mask if dres is not None
                                                                                               else None), M, C,
                                    _ptr(c), _ptr(dgamma), _ptr(dbeta), 1 if relu else 0, _ptr(planes), P, _ptr(ws),
                                    _stream())
        _check(rc, "bn_bwd_planes")
        return dx, dgamma, dbeta, dres
    ws = _ae((lib.dl4j_bn_workspace_floats(M, C),), torch.float32, x.device)
    rc = lib.dl4j_bn_bwd(_dt16(x), _ptr(x), _ptr(res), _ptr(dy), _ptr(dx), _ptr(dres), M, C, _ptr(c), _ptr(dgamma),
                         _ptr(dbeta), 1 if relu else 0, _ptr(ws), _ptr(mask), _stream())
    _check(rc, "bn_bwd")
    return dx, dgamma, dbeta, dres


def bn_pool_fwd(x, gamma, beta, run_mean, run_var, training, decay, eps, kernel, stride, pad4):
    """Fused BN -> ReLU -> max pool (csrc/batchnorm.hip bnpool_*). x: NHWC conv output. Returns (y_pooled, ctx)."""
    dt = _dt16(x)
    if dt is None or x.dim() != 4 or not torch.is_tensor(gamma) or run_mean.dtype != torch.float32:
        return None
    if not x.is_contiguous(memory_format=torch.channels_last):
        return None
    N, C, H, W = x.shape
    if C % 8 != 0 or C // 8 > 256:
        return None
    kh, kw = kernel
    sh, sw = stride
    pt, pb, pl, pr = pad4
    OH = (H + pt + pb - kh) // sh + 1
    OW = (W + pl + pr - kw) // sw + 1
    if OH < 1 or OW < 1 or kh * kw > 127:
        return None
    lib = load()
    register_sig("dl4j_bn_pool_fwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 12 +
                 [c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p, c_float, c_float, c_int, c_void_p, c_ll,
                  c_int, c_void_p, c_void_p, c_void_p])
    y = _ae((N, C, OH, OW), x.dtype, x.device, channels_last=True)
    am = _ae((N * OH * OW * C,), torch.uint8, x.device) if training else None
    xh = _ae((N, C, OH, OW), x.dtype, x.device, channels_last=True) if training else None
    ts = getattr(x, "_bn_tile_stats", None)
    M = N * H * W
    rpp = ts[2] if ts is not None and len(ts) > 2 else 64
    if not (training and ts is not None and dt in (1, 2) and ts[0].shape[2] == C and
            (ts[1] * rpp == M if rpp != 64 else ts[1] == 2 * ((M + 127) // 128))):
        ts = None
    nws = lib.dl4j_bn_workspace_floats(M, C)
    if ts is not None:
        register_sig("dl4j_bn_tiles_workspace_floats", [c_ll, c_int])
        lib.dl4j_bn_tiles_workspace_floats.restype = c_ll
        nws = max(nws, lib.dl4j_bn_tiles_workspace_floats(ts[1], C))
    ws = _ae((nws,), torch.float32, x.device)
    ctx = _ae((4 * C,), torch.float32, x.device)
    b = beta if torch.is_tensor(beta) else None
    rc = lib.dl4j_bn_pool_fwd(dt, _ptr(x), _ptr(y), _ptr(am), _ptr(xh), N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl,
                              _ptr(gamma), _ptr(b), 1.0, float(beta) if b is None else 0.0, _ptr(run_mean),
                              _ptr(run_var), float(decay), float(eps), 1 if training else 0,
                              _ptr(ts[0] if ts is not None else None), int(ts[1]) if ts is not None else 0, int(rpp),
                              _ptr(ws), _ptr(ctx), _stream())
    if rc == -1:
        return None
    _check(rc, "bn_pool_fwd")
    return y, ("NATIVE_POOL", x, ctx, am, xh, (kh, kw, sh, sw, pt, pl), (OH, OW))


def bn_pool_bwd(dy, ctx, dgamma_out=None, dbeta_out=None):
    _, x, c, am, xh, (kh, kw, sh, sw, pt, pl), (OH, OW) = ctx
    N, C, H, W = x.shape
    dy = _rows_like(dy, xh)
    lib = load()
    register_sig("dl4j_bn_pool_bwd", [c_int] + [c_void_p] * 5 + [c_int] * 12 + [c_void_p] * 4 + [c_void_p])
    dx = _ae(x.shape, x.dtype, x.device, channels_last=True)
    ok = lambda t: t is not None and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == C  # noqa
    dgamma = dgamma_out if ok(dgamma_out) else _ae((C,), torch.float32, x.device)
    dbeta = dbeta_out if ok(dbeta_out) else _ae((C,), torch.float32, x.device)
    ws = _ae((lib.dl4j_bn_workspace_floats(N * OH * OW, C),), torch.float32, x.device)
    rc = lib.dl4j_bn_pool_bwd(_dt16(x), _ptr(x), _ptr(dy), _ptr(am), _ptr(xh), _ptr(dx), N, H, W, C, OH, OW, kh, kw,
                              sh, sw, pt, pl, _ptr(c), _ptr(dgamma), _ptr(dbeta), _ptr(ws), _stream())
    _check(rc, "bn_pool_bwd")
    return dx, dgamma, dbeta


# ------------------------------------------------------------------------------------------ softmax-xent
def _dt16(t):
    """Element-type code for the kernels that also take fp16 (LayerNorm, GELU, attention, softmax-xent,
    channel sums, updater shadow): 0 fp32, 1 bf16, 2 fp16."""
    return {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}.get(t.dtype)


def softmax_xent(logits, labels, clip_eps, row_mask=None):
    """row_mask: optional fp32 per-row mask ([B] or [B, 1]) applied to each row's score and gradient."""
    dt = _dt16(logits)
    if dt is None or not logits.is_contiguous():
        return None
    B, V = logits.shape
    lab = labels.contiguous().float()
    grad = _ae(logits.shape, logits.dtype, logits.device)
    score = _ae((B,), torch.float32, logits.device)
    if row_mask is not None:
        m = row_mask.reshape(-1).to(torch.float32).contiguous()
        if m.numel() != B:
            return None
        register_sig("dl4j_softmax_xent_masked", [c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                                  c_void_p, c_float, c_void_p])
        rc = load().dl4j_softmax_xent_masked(dt, _ptr(logits), _ptr(lab), B, V, _ptr(grad), _ptr(score), _ptr(m),
                                             float(clip_eps or 0.0), _stream())
        _check(rc, "softmax_xent_masked")
        return score, grad, None
    rc = load().dl4j_softmax_xent(dt, _ptr(logits), _ptr(lab), B, V, _ptr(grad), _ptr(score), None,
                                  float(clip_eps or 0.0), _stream())
    _check(rc, "softmax_xent")
    return score, grad, None


def softmax_xent_strided(logits, y, mb, ys, clip_eps):
    """Fused softmax + MCXENT over the rows of ``logits`` [B, V] (unit column stride) with labels read in place from
    fp32 ``y`` at strides ys = (per-example, per-time-step, per-class) for row r = t*mb + b. Returns (score [B] fp32,
    gradient [B, V]); when V % 8 != 0 the gradient is a zero-padded ``kz_view`` GEMM operand (ops/gemm.py)."""
    dt = _dt16(logits)
    if dt is None or logits.dim() != 2 or logits.stride(1) != 1 or y.dtype != torch.float32 or not y.is_cuda:
        return None
    B, V = logits.shape
    register_sig("dl4j_softmax_xent_strided", [c_int, c_void_p, c_int, c_void_p, c_ll, c_ll, c_ll, c_int, c_int, c_int,
                                               c_void_p, c_int, c_void_p, c_float, c_void_p])
    from ..memory import arena
    from .gemm import kz_view
    V8 = (V + 7) // 8 * 8
    buf = arena.empty((B, V8), logits.dtype, logits.device)
    score = arena.empty((B,), torch.float32, logits.device)
    rc = load().dl4j_softmax_xent_strided(dt, _ptr(logits), logits.stride(0) if B > 1 else V, _ptr(y), int(ys[0]),
                                          int(ys[1]), int(ys[2]), int(mb), B, V, _ptr(buf), V8, _ptr(score),
                                          float(clip_eps or 0.0), _stream())
    _check(rc, "softmax_xent_strided")
    return score, (kz_view(buf, V) if V8 != V else buf)


# ------------------------------------------------------------------------------------------ pooling
def pool2d_fwd(x, ptype, kernel, stride, pad4):
    dt = _dt16(x)
    if dt is None or x.dim() != 4 or x.shape[1] % 8 != 0:
        return None
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    N, C, H, W = x.shape
    pt, pb, pl, pr = pad4
    kh, kw = kernel
    sh, sw = stride
    OH = (H + pt + pb - kh) // sh + 1
    OW = (W + pl + pr - kw) // sw + 1
    y = _ae((N, C, OH, OW), x.dtype, x.device, channels_last=True)
    mode = 0 if ptype == "MAX" else 1
    am = _ae((N * OH * OW * C if mode == 0 else 8,), torch.uint8, x.device)
    rc = load().dl4j_pool_fwd(dt, mode, _ptr(x), _ptr(y), _ptr(am), N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl,
                              _stream())
    _check(rc, "pool_fwd")
    return y, ("NATIVE", mode, am, x.shape, x.dtype, (kh, kw, sh, sw, pt, pl), (OH, OW))


def pool2d_bwd(dy, ctx):
    _, mode, am, xshape, xdt, (kh, kw, sh, sw, pt, pl), (OH, OW) = ctx
    N, C, H, W = xshape
    dy = dy.to(xdt).contiguous(memory_format=torch.channels_last)
    dx = _ae(xshape, xdt, dy.device, channels_last=True)
    rc = load().dl4j_pool_bwd({torch.bfloat16: 1, torch.float16: 2}.get(xdt, 0), mode, _ptr(dy), _ptr(am), _ptr(dx), N, H, W, C, OH,
                              OW, kh, kw, sh, sw, pt, pl, _stream())
    _check(rc, "pool_bwd")
    return dx


# ------------------------------------------------------------------------------------------ conv (MFMA)
def conv2d_fwd(x, w, b, stride, pad4, dilation, want_stats=False):
    from . import conv_native
    return conv_native.conv2d_fwd(x, w, b, stride, pad4, dilation, want_stats)


def conv2d_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db, gW=None, gb=None, grads_zeroed=False,
               dx_accum=None):
    from . import conv_native
    return conv_native.conv2d_bwd(x, w, dy, stride, pad4, dilation, need_dx, need_dw, need_db, gW, gb,
                                  grads_zeroed, dx_accum)


def segment_stats(flat, offsets, bins=0):
    """Per-segment {mean, std, meanAbs, min, max} (+ optional ``bins``-bin histograms over [min, max]) of a flat
    fp32/bf16 CUDA tensor, one fused HIP launch for all segments (csrc/stats.hip). ``offsets``: list of nseg+1
    element offsets. Returns (stats [nseg, 5] float32, hist [nseg, bins] int64 or None) on the device."""
    lib = load()
    register_sig("dl4j_segment_stats", [c_int, c_void_p, c_void_p, c_int, c_ll, c_void_p, c_void_p, c_int,
                                        c_void_p, c_void_p])
    dt = _dt(flat)
    if dt is None or not flat.is_contiguous():
        raise ValueError("segment_stats needs a contiguous fp32/bf16 tensor")
    nseg = len(offsets) - 1
    if offsets[0] < 0 or offsets[-1] > flat.numel() or any(b < a for a, b in zip(offsets[:-1], offsets[1:])):
        raise IndexError("segment offsets outside the flat array")
    dev = flat.device
    off = torch.tensor(offsets, dtype=torch.int64, device=dev)
    ws = torch.empty(5 * nseg, dtype=torch.float32, device=dev)
    out = torch.empty(nseg, 5, dtype=torch.float32, device=dev)
    hist = torch.empty(nseg, bins, dtype=torch.int32, device=dev) if bins > 0 else None
    maxlen = max(b - a for a, b in zip(offsets[:-1], offsets[1:])) if nseg else 0
    rc = lib.dl4j_segment_stats(dt, _ptr(flat), _ptr(off), nseg, maxlen, _ptr(ws), _ptr(out), bins, _ptr(hist),
                                c_void_p(_stream()))
    _check(rc, "segment_stats")
    return out, (hist.to(torch.int64) if hist is not None else None)


def channel_sum(rows, out=None):
    """fp32 column sums of a contiguous [M, C] fp32/bf16 CUDA matrix (dl4j_channel_sum); None if unsupported.
    ``out``: optional contiguous fp32 [C] destination (e.g. a flat-gradient view)."""
    dt = _dt16(rows)
    if dt is None or rows.dim() != 2 or not rows.is_contiguous() or rows.shape[1] == 0:
        return None
    lib = load()
    register_sig("dl4j_channel_sum", [c_int, c_void_p, c_ll, c_int, c_void_p, c_void_p, c_void_p])
    register_sig("dl4j_channel_sum_ws_floats", [c_ll, c_int], restype=c_ll)
    if out is None or not (out.is_contiguous() and out.dtype == torch.float32 and out.numel() == rows.shape[1]):
        out = torch.empty(rows.shape[1], dtype=torch.float32, device=rows.device)
    ws = _scratch(lib.dl4j_channel_sum_ws_floats(rows.shape[0], rows.shape[1]), rows.device)
    _check(lib.dl4j_channel_sum(dt, _ptr(rows), rows.shape[0], rows.shape[1], _ptr(out), _ptr(ws),
                                c_void_p(_stream())), "channel_sum")
    return out


_scratch_bufs = {}


def _scratch(nfloats, device):
    """Growing fp32 scratch per (device, stream) for kernels that reduce through partial rows. A stream's work is
    ordered, so consecutive launches may reuse it; the overlap stream gets its own."""
    key = (str(device), torch.cuda.current_stream(device).stream_id if device.type == "cuda" else 0)
    t = _scratch_bufs.get(key)
    if t is None or t.numel() < nfloats:
        t = _scratch_bufs[key] = torch.empty(max(int(nfloats), 1 << 16), dtype=torch.float32, device=device)
    return t
