"""Whole-sequence fused LSTM / GravesLSTM kernels (csrc/lstm.hip): the MI355X counterpart of the reference's cuDNN
``LSTMHelper`` (deeplearning4j-cuda/.../recurrent/CudnnLSTMHelper.java; SPI at nn/layers/recurrent/LSTM.java:66).

``lstm_seq_fwd`` runs the recurrence of all T steps in one launch (one workgroup per 16 minibatch rows, MFMA
h·RW, fused gates + peepholes + mask, cell state in registers). ``lstm_seq_bwd`` runs the backward time loop
(gate deltas + dh = dz·RWᵀ per step) and returns the fp32 gate deltas for the weight GEMMs. Both return
``None`` when the shape/dtype is outside the kernels (the caller then runs the per-step path).
"""
import ctypes
import threading

import torch

from . import native, nd4j_kernels
from ..memory import arena
from .native import _check, _ptr, _stream, c_int, c_void_p

_SIG_FWD = [c_int] + [c_void_p] * 12 + [c_int, c_int, c_int, c_void_p]
_SIG_BWD = [c_int, c_void_p, c_int] + [c_void_p] * 11 + [c_int, c_int, c_int, c_int, c_void_p]
_SIG_PACK = [c_int, c_void_p, ctypes.c_longlong, ctypes.c_longlong, c_int, c_void_p, c_void_p, c_void_p, c_void_p]


_DTC = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def supported(H, dtype):
    if dtype in (torch.bfloat16, torch.float16):
        ok_k = H % 32 == 0
    elif dtype == torch.float32:
        ok_k = H % 16 == 0
    else:
        return False
    if not ok_k:
        return False
    return H // 16 <= 16 or (H % 32 == 0 and H // 32 <= 16) or (H % 64 == 0 and H // 64 <= 16)


def _pack_b(m, dt):
    """[N, K] matrix (B[k][n] = m[n][k]) -> the kernels' fragment-packed layout [N/16][K/KC][64 lanes][FE]: lane
    l of k-step s holds m[16*tile + (l & 15)][KC*s + FE*(l >> 4) + j], j < FE, so each wave load is contiguous."""
    fe = 8 if dt in (torch.bfloat16, torch.float16) else 4
    N, K = m.shape
    return (m.to(dt).reshape(N // 16, 16, K // (4 * fe), 4, fe).permute(0, 2, 3, 1, 4).contiguous())


def _f32c(t):
    return None if t is None else t.detach().to(torch.float32).contiguous()


def _eps_arg(t):
    """(tensor, dtype code) for the backward kernels' eps operand: fp32 / bf16 / fp16 are read as they are."""
    t = t.detach()
    if t.dtype not in _DTC:
        t = t.to(torch.float32)
    return t.contiguous(), _DTC[t.dtype]


class RWPacks:
    """The sequence kernels' packed recurrent weights for one layer and one weight version (one TBPTT window):
    forward B = RWᵀ, backward B = RW, fp32 peepholes [3, H] — built by ONE launch (csrc/lstm_glue.hip
    lstm_pack_rw_kernel) in the forward pass and reused by the backward pass."""
    __slots__ = ("fwd", "bwd", "peep", "H", "dtype")

    def __init__(self, fwd, bwd, peep, H, dtype):
        self.fwd, self.bwd, self.peep, self.H, self.dtype = fwd, bwd, peep, H, dtype


def pack_rw(RW, H, peephole, need_bwd=True):
    """RWPacks for the [H, 4H(+3)] weight view, or None when the kernels do not take this dtype/H."""
    dt = RW.dtype
    if not RW.is_cuda or not supported(H, dt) or RW.dim() != 2 or RW.shape[0] != H:
        return None
    lib = native.load()
    native.register_sig("dl4j_lstm_pack_rw", _SIG_PACK)
    fe = 8 if dt in (torch.bfloat16, torch.float16) else 4
    shape = lambda n, k: (n // 16, k // (4 * fe), 4, 16, fe)  # noqa: E731
    fwd = arena.empty(shape(4 * H, H), dt, RW.device)
    bwd = arena.empty(shape(H, 4 * H), dt, RW.device) if need_bwd else None
    peep = arena.empty((3, H), torch.float32, RW.device) if peephole else None
    rc = lib.dl4j_lstm_pack_rw(_DTC[dt], _ptr(RW), RW.stride(0), RW.stride(1), H, _ptr(fwd), _ptr(bwd), _ptr(peep),
                               _stream())
    if rc == -1:
        return None
    _check(rc, "lstm_pack_rw")
    return RWPacks(fwd, bwd, peep, H, dt)


_SIG_COOP = [c_void_p] * 14 + [c_int, c_int, c_int, ctypes.c_uint, c_int, c_void_p]


_DEV_TAG = 0xFFFFFFFF          # csrc/lstm_coop.hip kDevTag: granule tags tracked on the device (no per-launch memset)


class _CoopBuf:
    """Persistent exchange buffer + control words of the cooperative kernels: err[0] sticky hand-off timeout flag,
    err[1] device-side tag base, err[2] finished-workgroup counter. ``next_tag`` is None while the contents are
    undefined (the next launch zeroes them). A pinned host copy of the error word is refreshed asynchronously after
    every eager launch and checked before the next one, so a hand-off timeout surfaces as an exception instead of
    silently wrong results."""

    def __init__(self, nbytes, device):
        self.exch = torch.empty(nbytes // 8, dtype=torch.int64, device=device)
        self.err = torch.empty(4, dtype=torch.int32, device=device)
        # pinned host copy, created by the first EAGER launch (pinned allocation is illegal while a stream captures:
        # the capture stream gets a buffer of its own)
        self.err_host = None
        self.err_ev = None
        self.next_tag = None                               # None: contents undefined -> the next launch zeroes them


class CoopTimeoutError(RuntimeError):
    pass


_coop_bufs = {}
# Buffers are never freed once handed to a launch: a captured HIP graph embeds their addresses (exchange memset +
# kernel arguments), so a buffer outgrown by a later, bigger launch is retired here instead of going back to the
# caching allocator (replaying a graph must never write into memory another tensor owns).
_RETIRED = []
_lock = threading.Lock()


def _coop_buf(kind, nbytes, device, steps):
    """(buffer, tag argument, reset) for one launch. Buffers are per (kind, device, stream) so concurrent
    ParallelInference workers on one device never share granules. Tags live on the device (_DEV_TAG), so only a
    buffer's first launch zeroes it. A HIP-graph capture reuses an already-initialised buffer of the device's default
    stream (the stream its replays run on) when one is big enough, so the captured graph holds no memset node."""
    capturing = torch.cuda.is_current_stream_capturing()
    key = (kind, str(device), torch.cuda.current_stream(device).cuda_stream)
    with _lock:
        if capturing and key not in _coop_bufs:
            dkey = (kind, str(device), torch.cuda.default_stream(device).cuda_stream)
            d = _coop_bufs.get(dkey)
            if d is not None and d.exch.numel() * 8 >= nbytes and d.next_tag is not None:
                _coop_bufs[key] = d
        b = _coop_bufs.get(key)
        if b is None or b.exch.numel() * 8 < nbytes:
            if b is not None:
                _RETIRED.append(b)
            b = _coop_bufs[key] = _CoopBuf(nbytes, device)
        if not capturing and b.err_ev is not None and b.err_ev.query() and int(b.err_host[0]) != 0:
            b.err_ev = None
            b.next_tag = None
            raise CoopTimeoutError(f"cooperative LSTM {kind} kernel: a cross-workgroup hand-off timed out (the "
                                   "workgroups were not co-resident); results of that launch are invalid")
        if b.next_tag is None:                             # contents undefined: this launch zeroes them
            b.next_tag = 0
            return b, _DEV_TAG, 1
        return b, _DEV_TAG, 0


def _post_launch(b):
    """Eager launches: queue an async copy of the error word into pinned memory (checked at the next launch)."""
    if torch.cuda.is_current_stream_capturing():
        return
    if b.err_host is None:
        b.err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    b.err_host.copy_(b.err[:1], non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    b.err_ev = ev


def check_coop_errors():
    """Synchronously raise if any cooperative LSTM launch so far hit a hand-off timeout."""
    for b in list(_coop_bufs.values()):
        if b.err_ev is not None and b.err_host is not None:
            b.err_ev.synchronize()
            if int(b.err_host[0]) != 0:
                raise CoopTimeoutError("cooperative LSTM kernel: a cross-workgroup hand-off timed out")


# ---- launch mode and step guard (csrc/lstm_coop.hip)
# counts components that run kernels on OTHER streams during training (data-parallel comm streams, in-process
# multi-worker trainers); while any is live, and while the conv weight-gradient overlap stream is active, the
# cooperative kernels use the cooperative launch so that every workgroup is co-resident.
CONCURRENT_STREAMS = [0]
_guard = {}          # device index -> deque of (pinned int32 snapshot, event), oldest first
_GUARD_DEPTH = 8     # snapshots allowed in flight before the host blocks on the oldest one
USED_COOP = [False]


def _concurrent_streams():
    from . import side_stream
    if CONCURRENT_STREAMS[0] > 0 or side_stream.active():
        return True
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _launch_mode(lib):
    native.register_sig("dl4j_lstm_coop_launch_mode", [c_int])
    lib.dl4j_lstm_coop_launch_mode(1 if _concurrent_streams() else -1)
    USED_COOP[0] = True


def check_step_guard(device):
    """Called once per training step after the fused update has been queued. Every step queues a snapshot of the
    device-wide step guard (set by a timed-out cooperative LSTM launch; the fused updater then skips updates) into a
    FIFO; every snapshot whose event has completed is checked, oldest first, and once ``_GUARD_DEPTH`` snapshots are
    pending the host blocks on the oldest. So a timeout is reported at most ``_GUARD_DEPTH`` steps late even when the
    host runs far ahead of the GPU (HIP-graph replay, no listener syncing): the guard is cleared and CoopTimeoutError
    raised."""
    if not USED_COOP[0] or device is None or device.type != "cuda" or torch.cuda.is_current_stream_capturing():
        return
    import collections
    lib = native.load()
    native.register_sig("dl4j_lstm_step_guard", [])
    native.register_sig("dl4j_lstm_step_guard_reset", [c_void_p])
    lib.dl4j_lstm_step_guard.restype = c_void_p
    q = _guard.get(device.index)
    if q is None:
        q = _guard[device.index] = collections.deque()
    tripped = False
    while q and (len(q) >= _GUARD_DEPTH or q[0][1].query()):
        snap, ev = q.popleft()
        ev.synchronize()
        if int(snap[0]) != 0:
            tripped = True
    if tripped:
        lib.dl4j_lstm_step_guard_reset(c_void_p(_stream()))
        q.clear()                      # younger snapshots may hold the same (now cleared) trip
        raise CoopTimeoutError("cooperative LSTM kernel: a cross-workgroup hand-off timed out; the fused updater "
                               "skipped the update of every step since (parameters unchanged)")
    ptr = lib.dl4j_lstm_step_guard()
    if not ptr:
        return
    import ctypes as _ct
    snap = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    hip = _hip()
    hip.hipMemcpyAsync(_ct.c_void_p(snap.data_ptr()), _ct.c_void_p(ptr), _ct.c_size_t(4), 2, _ct.c_void_p(_stream()))
    ev = torch.cuda.Event()
    ev.record()
    q.append((snap, ev))


_hiplib = []


def _hip():
    if not _hiplib:
        import ctypes as _ct
        lib = _ct.CDLL("libamdhip64.so")
        lib.hipMemcpyAsync.argtypes = [_ct.c_void_p, _ct.c_void_p, _ct.c_size_t, _ct.c_int, _ct.c_void_p]
        lib.hipMemcpyAsync.restype = _ct.c_int
        _hiplib.append(lib)
    return _hiplib[0]


def _coop_enabled():
    import os
    return os.environ.get("DL4J_AMD_LSTM_COOP", "1") == "1"


def _fwd_coop(lib, zx, rwt, peep, h0c, c0c, m, out, out16, gates, call, hT, cT, T, mb, H):
    """Cooperative multi-workgroup kernel (csrc/lstm_coop.hip, RW resident in LDS); False if it does not apply."""
    native.register_sig("dl4j_lstm_fwd_coop", _SIG_COOP)
    native.register_sig("dl4j_lstm_coop_exch_bytes", [c_int, c_int])
    lib.dl4j_lstm_coop_exch_bytes.restype = ctypes.c_longlong
    nbytes = lib.dl4j_lstm_coop_exch_bytes(mb, H)
    b, base, reset = _coop_buf("fwd", nbytes, zx.device, T)
    _launch_mode(lib)
    rc = lib.dl4j_lstm_fwd_coop(_ptr(zx), _ptr(rwt), _ptr(peep), _ptr(h0c), _ptr(c0c), _ptr(m), _ptr(out),
                                _ptr(out16), _ptr(gates), _ptr(call), _ptr(hT), _ptr(cT), _ptr(b.exch), _ptr(b.err), T, mb, H, base, reset,
                                c_void_p(_stream()))
    if rc != 0:
        b.next_tag = None
        return False
    _post_launch(b)
    global last_coop_err
    last_coop_err = b.err[:1]                            # device word: 1 = a hand-off wait timed out (sticky)
    return True


last_coop_err = None

_SIG_BWD_COOP = [c_void_p, c_int] + [c_void_p] * 13 + [c_int, c_int, c_int, c_int, ctypes.c_uint, c_int, c_void_p]


def _bwd_coop(lib, e, edt, gates, call, c0c, rw, peep, m, dhl, dcl, dz, dh0, dc0, T, mb, H, t_end):
    """Cooperative backward (csrc/lstm_coop.hip: K-split partial dh exchange, RW slice resident in LDS)."""
    native.register_sig("dl4j_lstm_bwd_coop", _SIG_BWD_COOP)
    native.register_sig("dl4j_lstm_coop_bwd_exch_bytes", [c_int, c_int])
    lib.dl4j_lstm_coop_bwd_exch_bytes.restype = ctypes.c_longlong
    nbytes = lib.dl4j_lstm_coop_bwd_exch_bytes(mb, H)
    b, base, reset = _coop_buf("bwd", nbytes, e.device, T)
    _launch_mode(lib)
    rc = lib.dl4j_lstm_bwd_coop(_ptr(e), edt, _ptr(gates), _ptr(call), _ptr(c0c), _ptr(rw), _ptr(peep), _ptr(m), _ptr(dhl),
                                _ptr(dcl), _ptr(dz), _ptr(dh0), _ptr(dc0), _ptr(b.exch), _ptr(b.err), T, mb, H,
                                int(t_end), base, reset, c_void_p(_stream()))
    if rc != 0:
        b.next_tag = None
        return False
    _post_launch(b)
    global last_coop_bwd_err
    last_coop_bwd_err = b.err[:1]
    return True


last_coop_bwd_err = None


def lstm_seq_fwd(zx, RW, H, peephole, h0=None, c0=None, mask=None, need_cache=True, packs=None, out16=False):
    """zx: [T, mb, 4H] (compute dtype, = x·W + b); RW: [H, 4H(+3)] view; packs: RWPacks of RW (else packed here).
    Returns (out [T, mb, H] fp32, hT, cT, gates [T,mb,4H] fp32 | None, call [T,mb,H] fp32 | None, out16) or None;
    out16 (with ``out16=True``) is h in the compute dtype, written by the same kernel (the next layer's input)."""
    T, mb, H4 = zx.shape
    dt = zx.dtype
    if H4 != 4 * H or not supported(H, dt) or T < 1 or mb < 1:
        return None
    lib = native.load()
    native.register_sig("dl4j_lstm_fwd", _SIG_FWD)
    dev = zx.device
    zx = zx.contiguous()
    if packs is not None and packs.dtype == dt and packs.H == H:
        rwt, peep = packs.fwd, packs.peep
    else:
        rwt = _pack_b(RW[:, :4 * H].t(), dt)                         # B[k][n] = RW[k][n], n over 4H
        peep = RW[:, 4 * H:4 * H + 3].t().to(torch.float32).contiguous() if peephole else None
    h0c, c0c = _f32c(h0), _f32c(c0)
    m = _f32c(mask.reshape(mb, -1)) if mask is not None else None
    if m is not None and m.shape[1] != T:
        return None
    # per-call working memory (outputs, gate / cell caches for backward) from the open training / TBPTT arena
    # (memory/arena.py: the reference's LOOP_LSTM working memory); the carried state hT / cT is not carved
    out = arena.empty((T, mb, H), torch.float32, dev)
    o16 = arena.empty((T, mb, H), dt, dev) if out16 and dt != torch.float32 else None
    hT = torch.empty(mb, H, device=dev, dtype=torch.float32)
    cT = torch.empty(mb, H, device=dev, dtype=torch.float32)
    gates = arena.empty((T, mb, 4 * H), torch.float32, dev) if need_cache else None
    call = arena.empty((T, mb, H), torch.float32, dev) if need_cache else None
    if dt == torch.bfloat16 and H in (256, 512) and _coop_enabled() and \
            _fwd_coop(lib, zx, rwt, peep, h0c, c0c, m, out, o16, gates, call, hT, cT, T, mb, H):
        return out, hT, cT, gates, call, o16
    rc = lib.dl4j_lstm_fwd(_DTC.get(dt, 0), _ptr(zx), _ptr(rwt), _ptr(peep), _ptr(h0c), _ptr(c0c),
                           _ptr(m), _ptr(out), _ptr(o16), _ptr(gates), _ptr(call), _ptr(hT), _ptr(cT), T, mb, H,
                           c_void_p(_stream()))
    if rc == -1:
        return None
    _check(rc, "lstm_fwd")
    return out, hT, cT, gates, call, o16


def lstm_seq_bwd(eps_tmh, gates, call, c0, RW, H, peephole, mask=None, dh_last=None, dc_last=None, t_end=0,
                 packs=None):
    """eps_tmh: [T, mb, H] (any float dtype). Returns (dz [T, mb, 4H] fp32, dh0, dc0) or None."""
    T, mb, _ = eps_tmh.shape
    dt = RW.dtype
    if not supported(H, dt) or t_end >= T:
        return None
    lib = native.load()
    native.register_sig("dl4j_lstm_bwd", _SIG_BWD)
    dev = eps_tmh.device
    e, edt = _eps_arg(eps_tmh)
    if packs is not None and packs.bwd is not None and packs.dtype == dt and packs.H == H:
        rw, peep = packs.bwd, packs.peep
    else:
        rw = _pack_b(RW[:, :4 * H], dt)                               # dh = dz·RWᵀ: B[k][n] = RW[n][k], k over 4H
        peep = RW[:, 4 * H:4 * H + 3].t().to(torch.float32).contiguous() if peephole else None
    m = _f32c(mask.reshape(mb, -1)) if mask is not None else None
    dz = arena.empty((T, mb, 4 * H), torch.float32, dev)
    if t_end > 0:
        dz.zero_()
    dh0 = torch.empty(mb, H, device=dev, dtype=torch.float32)
    dc0 = torch.empty(mb, H, device=dev, dtype=torch.float32)
    if dt == torch.bfloat16 and H in (256, 512) and _coop_enabled() and \
            _bwd_coop(lib, e, edt, gates, call, _f32c(c0), rw, peep, m, _f32c(dh_last), _f32c(dc_last), dz, dh0, dc0, T, mb,
                      H, t_end):
        return dz, dh0, dc0
    rc = lib.dl4j_lstm_bwd(_DTC.get(dt, 0), _ptr(e), edt, _ptr(gates), _ptr(call), _ptr(_f32c(c0)),
                           _ptr(rw), _ptr(peep), _ptr(m), _ptr(_f32c(dh_last)), _ptr(_f32c(dc_last)), _ptr(dz),
                           _ptr(dh0), _ptr(dc0), T, mb, H, int(t_end), c_void_p(_stream()))
    if rc == -1:
        return None
    _check(rc, "lstm_bwd")
    return dz, dh0, dc0




def lstm_bwd_prep(dz, out, h0, call, c0, peephole, dtype):
    """One-launch LSTM backward glue (csrc/lstm_glue.hip): dz [T, mb, 4H] fp32, out / call [T, mb, H] fp32 (h_t,
    c_t), h0 / c0 [mb, H] or None -> (dz in ``dtype`` [T*mb, 4H], h_{t-1} in ``dtype`` [T*mb, H], db [4H] fp32,
    peephole grads [3, H] fp32). None when the dtype is not bf16/fp16."""
    dt = {torch.bfloat16: 1, torch.float16: 2}.get(dtype)
    if dt is None or dz.dtype != torch.float32 or out.dtype != torch.float32 or call.dtype != torch.float32:
        return None
    T, mb, G = dz.shape
    H = G // 4
    R = T * mb
    lib = native.load()
    native.register_sig("dl4j_lstm_bwd_prep", [c_int] + [c_void_p] * 9 + [c_int, c_int, c_int, c_int, c_void_p])
    dzb = torch.empty(R, G, dtype=dtype, device=dz.device)
    hpb = torch.empty(R, H, dtype=dtype, device=dz.device)
    acc = nd4j_kernels.zero_(torch.empty(G + 3 * H, dtype=torch.float32, device=dz.device))   # both accumulators
    db, dpeep = acc[:G], acc[G:].view(3, H)
    dzc, oc, cc = dz.contiguous(), out.contiguous(), call.contiguous()
    h0f, c0f = _f32c(h0), _f32c(c0)
    rc = lib.dl4j_lstm_bwd_prep(dt, _ptr(dzc), _ptr(oc), _ptr(h0f), _ptr(cc), _ptr(c0f), _ptr(dzb), _ptr(hpb), _ptr(db),
                                _ptr(dpeep), R, mb, H, int(bool(peephole)), _stream())
    _check(rc, "lstm_bwd_prep")
    return dzb, hpb, db, dpeep


# ---- pipelined two-layer stack (csrc/lstm_coop.hip lstm_fwd_stack2 / lstm_bwd_stack2)
_P = ctypes.c_void_p
STACK_LAUNCHES = [0, 0]        # successful stacked forward / backward launches (tests, profiling)


class _Stack2Fwd(ctypes.Structure):
    _fields_ = [(n, _P) for n in ("zx1", "rw1", "rw2", "w2", "b2", "peep1", "peep2", "h0_1", "c0_1", "h0_2", "c0_2",
                                  "mask", "out1", "o16_1", "gates1", "call1", "hT1", "cT1", "out2", "o16_2",
                                  "gates2", "call2", "hT2", "cT2", "exch", "err")] + \
        [("Tn", c_int), ("mb", c_int), ("timeout", ctypes.c_longlong), ("tag_arg", ctypes.c_uint),
         ("exch_words", ctypes.c_longlong)]


class _Stack2Bwd(ctypes.Structure):
    _fields_ = [("eps2", _P), ("eps_dt", c_int), ("pad_", c_int)] + \
        [(n, _P) for n in ("gates1", "call1", "c0_1", "gates2", "call2", "c0_2", "rw1", "rw2", "w2", "peep1",
                           "peep2", "mask", "dhl1", "dcl1", "dhl2", "dcl2", "dz1", "dz2", "dh0_1", "dc0_1",
                           "dh0_2", "dc0_2", "exch", "err")] + \
        [("Tn", c_int), ("mb", c_int), ("t_end", c_int), ("timeout", ctypes.c_longlong), ("tag_arg", ctypes.c_uint),
         ("exch_words", ctypes.c_longlong)]


def _stack_enabled():
    import os
    return os.environ.get("DL4J_AMD_LSTM_STACK", "1") == "1" and _coop_enabled()


def stack2_supported(H, dtype, T):
    if not _stack_enabled() or dtype != torch.bfloat16 or H != 256:
        return False
    lib = native.load()
    native.register_sig("dl4j_lstm_stack2_max_t", [])
    return 1 <= T <= lib.dl4j_lstm_stack2_max_t()


def _p(t):
    return None if t is None else c_void_p(t.data_ptr())


def lstm2_seq_fwd(zx1, packs1, packs2, w2pack, b2, H, h0s, c0s, mask, need_cache=True):
    """Both layers of a two-layer LSTM stack in ONE pipelined launch. zx1: [T, mb, 4H] bf16 (= x·W1 + b1); packs1 /
    packs2: RWPacks of RW1 / RW2; w2pack: RWPacks-style packing of W2 ([H, 4H]); b2: [4H] fp32. Returns
    ([out, hT, cT, gates, call, out16] for layer 1, [...] for layer 2) or None when the stack kernel does not apply."""
    T, mb, H4 = zx1.shape
    if not stack2_supported(H, zx1.dtype, T) or H4 != 4 * H:
        return None
    lib = native.load()
    native.register_sig("dl4j_lstm_fwd_stack2", [c_void_p, c_int, c_int, c_void_p])
    native.register_sig("dl4j_lstm_stack2_exch_bytes", [c_int, c_int, c_int, c_int])
    native.register_sig("dl4j_lstm_stack2_struct_bytes", [c_int])
    lib.dl4j_lstm_stack2_exch_bytes.restype = ctypes.c_longlong
    assert lib.dl4j_lstm_stack2_struct_bytes(0) == ctypes.sizeof(_Stack2Fwd)
    dev = zx1.device
    m = _f32c(mask.reshape(mb, -1)) if mask is not None else None
    if m is not None and m.shape[1] != T:
        return None
    outs = []
    for _ in range(2):
        outs.append([arena.empty((T, mb, H), torch.float32, dev), torch.empty(mb, H, device=dev, dtype=torch.float32),
                     torch.empty(mb, H, device=dev, dtype=torch.float32),
                     arena.empty((T, mb, 4 * H), torch.float32, dev) if need_cache else None,
                     arena.empty((T, mb, H), torch.float32, dev) if need_cache else None,
                     arena.empty((T, mb, H), zx1.dtype, dev)])
    nbytes = lib.dl4j_lstm_stack2_exch_bytes(mb, H, T, 0)
    b, base, reset = _coop_buf("stack_fwd", nbytes, dev, T)
    _launch_mode(lib)
    h = [_f32c(x) for x in h0s]
    c = [_f32c(x) for x in c0s]
    b2c = b2.detach().to(torch.float32).contiguous()
    zx1 = zx1.contiguous()
    a = _Stack2Fwd(zx1=_p(zx1), rw1=_p(packs1.fwd), rw2=_p(packs2.fwd), w2=_p(w2pack.fwd), b2=_p(b2c),
                   peep1=_p(packs1.peep), peep2=_p(packs2.peep), h0_1=_p(h[0]), c0_1=_p(c[0]), h0_2=_p(h[1]),
                   c0_2=_p(c[1]), mask=_p(m), out1=_p(outs[0][0]), o16_1=_p(outs[0][5]), gates1=_p(outs[0][3]),
                   call1=_p(outs[0][4]), hT1=_p(outs[0][1]), cT1=_p(outs[0][2]), out2=_p(outs[1][0]),
                   o16_2=_p(outs[1][5]), gates2=_p(outs[1][3]), call2=_p(outs[1][4]), hT2=_p(outs[1][1]),
                   cT2=_p(outs[1][2]), exch=_p(b.exch), err=_p(b.err), Tn=T, mb=mb, timeout=0, tag_arg=base,
                   exch_words=0)
    rc = lib.dl4j_lstm_fwd_stack2(ctypes.byref(a), H, reset, c_void_p(_stream()))
    if rc != 0:
        b.next_tag = None
        return None
    _post_launch(b)
    STACK_LAUNCHES[0] += 1
    return outs[0], outs[1]


def lstm2_seq_bwd(eps2_tmh, cache1, cache2, packs1, packs2, w2pack, H, mask=None, t_end=0, dh_last=(None, None),
                  dc_last=(None, None)):
    """Backward of a two-layer stack in ONE pipelined launch (layer 1's eps is formed inside from layer 2's gate
    deltas). eps2_tmh: [T, mb, H] gradient of layer 2's output. Returns (dz1, dz2 [T, mb, 4H] fp32, (dh0, dc0) of
    layer 1, (dh0, dc0) of layer 2) or None."""
    T, mb, _ = eps2_tmh.shape
    if not stack2_supported(H, packs1.dtype, T) or t_end >= T:
        return None
    lib = native.load()
    native.register_sig("dl4j_lstm_bwd_stack2", [c_void_p, c_int, c_int, c_void_p])
    native.register_sig("dl4j_lstm_stack2_exch_bytes", [c_int, c_int, c_int, c_int])
    native.register_sig("dl4j_lstm_stack2_struct_bytes", [c_int])
    lib.dl4j_lstm_stack2_exch_bytes.restype = ctypes.c_longlong
    assert lib.dl4j_lstm_stack2_struct_bytes(1) == ctypes.sizeof(_Stack2Bwd)
    dev = eps2_tmh.device
    e, edt = _eps_arg(eps2_tmh)
    m = _f32c(mask.reshape(mb, -1)) if mask is not None else None
    dz = [arena.empty((T, mb, 4 * H), torch.float32, dev) for _ in range(2)]
    if t_end > 0:
        for d in dz:
            d.zero_()
    st = [(torch.empty(mb, H, device=dev, dtype=torch.float32), torch.empty(mb, H, device=dev, dtype=torch.float32))
          for _ in range(2)]
    nbytes = lib.dl4j_lstm_stack2_exch_bytes(mb, H, T, 1)
    b, base, reset = _coop_buf("stack_bwd", nbytes, dev, T)
    _launch_mode(lib)
    c01, c02 = _f32c(cache1["c0"]), _f32c(cache2["c0"])
    dl = [_f32c(x) for x in dh_last]
    cl = [_f32c(x) for x in dc_last]
    a = _Stack2Bwd(eps2=_p(e), eps_dt=edt, pad_=0, gates1=_p(cache1["gates"]), call1=_p(cache1["call"]), c0_1=_p(c01),
                   gates2=_p(cache2["gates"]), call2=_p(cache2["call"]), c0_2=_p(c02), rw1=_p(packs1.bwd),
                   rw2=_p(packs2.bwd), w2=_p(w2pack.bwd), peep1=_p(packs1.peep), peep2=_p(packs2.peep), mask=_p(m),
                   dhl1=_p(dl[0]), dcl1=_p(cl[0]), dhl2=_p(dl[1]), dcl2=_p(cl[1]), dz1=_p(dz[0]), dz2=_p(dz[1]),
                   dh0_1=_p(st[0][0]), dc0_1=_p(st[0][1]), dh0_2=_p(st[1][0]), dc0_2=_p(st[1][1]), exch=_p(b.exch),
                   err=_p(b.err), Tn=T, mb=mb, t_end=int(t_end), timeout=0, tag_arg=base, exch_words=0)
    rc = lib.dl4j_lstm_bwd_stack2(ctypes.byref(a), H, reset, c_void_p(_stream()))
    if rc != 0:
        b.next_tag = None
        return None
    _post_launch(b)
    STACK_LAUNCHES[1] += 1
    return dz[0], dz[1], st[0], st[1]
