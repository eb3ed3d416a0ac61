"""Threshold / bitmap compression of update vectors (the reference's encoded gradient sharing:
NN:optimize/solvers/accumulation/EncodingHandler.java:114-191, libnd4j thresholdEncode/Decode, bitmapEncode/Decode).

Message = int32 tensor: [count, n, threshold-bits, type(0 sparse / 1 bitmap), payload...]; see csrc/threshold.hip.
GPU tensors use the HIP kernels (deterministic in-order stream compaction); CPU tensors use the C++ runtime
(csrc/runtime/threshold.cpp). Encoding subtracts what it emits from the residual in place.
"""
import torch

from . import native, runtime
from .dispatch import use_native
from .native import _ptr, _stream, c_float, c_int, c_ll, c_void_p

HEADER = 4
SPARSE, BITMAP = 0, 1

native.register_sig("dl4j_threshold_encode", [c_void_p, c_ll, c_float, c_void_p, c_int, c_void_p, c_void_p])
native.register_sig("dl4j_threshold_count", [c_void_p, c_ll, c_float, c_void_p, c_void_p, c_void_p])
native.register_sig("dl4j_threshold_decode", [c_void_p, c_void_p, c_int, c_float, c_void_p])
native.register_sig("dl4j_bitmap_encode", [c_void_p, c_ll, c_float, c_void_p, c_void_p, c_void_p])
native.register_sig("dl4j_bitmap_decode", [c_void_p, c_ll, c_void_p, c_float, c_void_p])
native.register_sig("dl4j_decode_any", [c_void_p, c_ll, c_int, c_void_p, c_float, c_void_p])


def _ws_ints(n):
    return (n + 2047) // 2048 + 1


def bitmap_capacity(n):
    return HEADER + (n + 15) // 16


def _check_flat(r):
    if r.dtype != torch.float32 or not r.is_contiguous():
        raise ValueError("compression works on contiguous fp32 vectors")


def threshold_count(residual, threshold):
    """Number of entries with |r| >= threshold (one small D2H copy on GPU)."""
    _check_flat(residual)
    n = residual.numel()
    if use_native(residual, "compression"):
        lib = native.load()
        ws = torch.empty(_ws_ints(n), dtype=torch.int32, device=residual.device)
        hdr = torch.empty(HEADER, dtype=torch.int32, device=residual.device)
        native._check(lib.dl4j_threshold_count(_ptr(residual), n, float(threshold), _ptr(ws), _ptr(hdr), _stream()),
                      "threshold_count")
        return int(hdr[0].item())
    rt = runtime.load()
    if rt is not None:
        return int(rt.rt_threshold_count(runtime.ptr(residual), n, float(threshold)))
    return int((residual.abs() >= threshold).sum())


def threshold_encode(residual, threshold, capacity=None):
    """Sparse threshold encoding (at most ``capacity`` entries, default n/16)."""
    _check_flat(residual)
    n = residual.numel()
    cap = int(capacity if capacity is not None else max(1, n // 16))
    out = torch.zeros(HEADER + cap, dtype=torch.int32, device=residual.device)
    if use_native(residual, "compression"):
        lib = native.load()
        ws = torch.empty(_ws_ints(n), dtype=torch.int32, device=residual.device)
        native._check(lib.dl4j_threshold_encode(_ptr(residual), n, float(threshold), _ptr(out), cap, _ptr(ws),
                                                _stream()), "threshold_encode")
        return out
    rt = runtime.load()
    if rt is not None:
        rt.rt_threshold_encode(runtime.ptr(residual), n, float(threshold), runtime.ptr(out), cap)
        return out
    idx = ((residual >= threshold) | (residual <= -threshold)).nonzero().reshape(-1)[:cap]
    sgn = torch.sign(residual[idx])
    out[HEADER:HEADER + idx.numel()] = ((idx + 1) * sgn).to(torch.int32)
    residual[idx] -= sgn * threshold
    out[0], out[1], out[2], out[3] = idx.numel(), n, _fbits(threshold), SPARSE
    return out


def bitmap_encode(residual, threshold):
    _check_flat(residual)
    n = residual.numel()
    out = torch.zeros(bitmap_capacity(n), dtype=torch.int32, device=residual.device)
    if use_native(residual, "compression"):
        lib = native.load()
        cnt = torch.zeros(1, dtype=torch.int32, device=residual.device)
        native._check(lib.dl4j_bitmap_encode(_ptr(residual), n, float(threshold), _ptr(out), _ptr(cnt), _stream()),
                      "bitmap_encode")
        return out
    rt = runtime.load()
    if rt is None:
        raise RuntimeError("bitmap encoding on CPU needs the C++ runtime library")
    rt.rt_bitmap_encode(runtime.ptr(residual), n, float(threshold), runtime.ptr(out))
    return out


def decode(message, target, scale=1.0):
    """target += decoded(message) * scale (either encoding)."""
    _check_flat(target)
    if use_native(target, "compression"):
        lib = native.load()
        msg = message.to(target.device).contiguous()
        native._check(lib.dl4j_decode_any(_ptr(msg), target.numel(), msg.numel() - HEADER, _ptr(target), float(scale),
                                          _stream()), "decode")
        return target
    rt = runtime.load()
    msg = message.cpu().contiguous()
    if rt is not None:
        if int(msg[3]) == BITMAP:
            rt.rt_bitmap_decode(runtime.ptr(msg), runtime.ptr(target), float(scale))
        else:
            rt.rt_threshold_decode(runtime.ptr(msg), runtime.ptr(target), float(scale))
        return target
    cnt = int(msg[0])
    thr = _bitsf(int(msg[2])) * scale
    e = msg[HEADER:HEADER + cnt].long()
    target.index_add_(0, e.abs() - 1, torch.sign(e).to(target.dtype) * thr)
    return target


def _fbits(f):
    import struct
    return struct.unpack("<i", struct.pack("<f", float(f)))[0]


def _bitsf(i):
    import struct
    return struct.unpack("<f", struct.pack("<i", int(i)))[0]
