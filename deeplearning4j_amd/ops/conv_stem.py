"""ResNet stem convolution (7x7 / stride 2 / pad 3, 3 -> 64 channels, NHWC bf16) on the dedicated MFMA kernel in
csrc/conv_stem.hip (the generic implicit-GEMM kernels need C % 8 == 0). Weight layout for the kernel: B[k][n] with
k = r*24 + s*3 + c (K padded to 192), fragment-packed as [4 n-tiles][6 k-steps][64 lanes][8]."""
import ctypes

import torch

from . import native
from .native import _ptr, _stream, c_int, c_void_p

_packed = {}


def supported(x, w, b, stride, pad4, dilation):
    if not (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    N, C, H, W = x.shape
    if tuple(w.shape) != (64, 3, 7, 7) or C != 3 or b is not None:
        return False
    if tuple(stride) != (2, 2) or tuple(pad4) != (3, 3, 3, 3) or tuple(dilation) != (1, 1):
        return False
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    return OH % 4 == 0 and (4 * OW) % 64 == 0 and x.is_contiguous(memory_format=torch.channels_last)


def pack_weights(w):
    """[64, 3, 7, 7] -> fragment-packed bf16 [4, 6, 64, 8] (cached per weight buffer and weight version)."""
    from .conv_native import WEIGHT_VERSION, is_managed
    key = (w.data_ptr(), str(w.device))
    ent = _packed.get(key)
    if ent is None:
        ent = _packed[key] = {"pk": torch.empty(4, 6, 64, 8, dtype=torch.bfloat16, device=w.device), "v": -1}
    if ent["v"] != WEIGHT_VERSION[0] or not is_managed(w.data_ptr()):
        lib = native.load()
        native.register_sig("dl4j_stem_pack_weights", [c_void_p, c_void_p] + [ctypes.c_longlong] * 4 + [c_void_p])
        rc = lib.dl4j_stem_pack_weights(_ptr(w), _ptr(ent["pk"]), *[int(t) for t in w.stride()], c_void_p(_stream()))
        native._check(rc, "stem_pack_weights")
        ent["v"] = WEIGHT_VERSION[0]
    return ent["pk"]


def pack_weights_reference(w):
    """The packing as torch ops (tests compare the kernel against it)."""
    k = torch.arange(147, device=w.device)
    r, rem = k // 21, k % 21
    full = torch.zeros(192, 64, dtype=w.dtype, device=w.device)
    full.index_copy_(0, r * 24 + rem, w.permute(2, 3, 1, 0).reshape(147, 64))
    return full.view(6, 4, 8, 4, 16).permute(3, 0, 1, 4, 2).reshape(4, 6, 64, 8).contiguous()


def forward(x, w, want_stats=False):
    N, _, H, W = x.shape
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    lib = native.load()
    native.register_sig("dl4j_stem_conv_fwd", [c_void_p] * 4 + [c_int] * 5 + [c_void_p])
    y = torch.empty((N, 64, OH, OW), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    ts = torch.empty((3, N * OH, 64), dtype=torch.float32, device=x.device) if want_stats else None
    rc = lib.dl4j_stem_conv_fwd(_ptr(x), _ptr(pack_weights(w)), _ptr(y), _ptr(ts), N, H, W, OH, OW,
                                c_void_p(_stream()))
    if rc == -1:
        return None
    native._check(rc, "stem_conv_fwd")
    if ts is not None:
        y._bn_tile_stats = (ts, ts.shape[1], OW)                # one partial per output row
    return y


_ws = {}


def backward_weight(x, dy, gW=None, gb=None, need_db=False):
    """dW (and db) of the stem conv. Writes into the fp32 gradient views gW / gb when given (overwrite); returns
    (dW_or_None, db_or_None) like conv_native.conv2d_bwd (None = written in place)."""
    N, _, H, W = x.shape
    OH, OW = dy.shape[2], dy.shape[3]
    lib = native.load()
    native.register_sig("dl4j_stem_conv_wrw", [c_void_p] * 5 + [c_int] * 5 + [c_void_p])
    native.register_sig("dl4j_stem_wrw_workspace_floats", [c_int, c_int])
    lib.dl4j_stem_wrw_workspace_floats.restype = ctypes.c_longlong
    key = str(x.device)
    nws = lib.dl4j_stem_wrw_workspace_floats(N, OH)
    ws = _ws.get(key)
    if ws is None or ws.numel() < nws:
        ws = _ws[key] = torch.empty(nws, dtype=torch.float32, device=x.device)
    direct = gW is not None and gW.dtype == torch.float32 and gW.is_contiguous() and gW.numel() == 64 * 147
    dW = gW if direct else torch.empty((64, 3, 7, 7), dtype=torch.float32, device=x.device)
    db = None
    if need_db:
        directb = gb is not None and gb.dtype == torch.float32 and gb.is_contiguous() and gb.numel() == 64
        db = gb.reshape(-1) if directb else torch.empty(64, dtype=torch.float32, device=x.device)
    rc = lib.dl4j_stem_conv_wrw(_ptr(x), _ptr(dy), _ptr(dW), _ptr(db), _ptr(ws), N, H, W, OH, OW,
                                c_void_p(_stream()))
    if rc == -1:
        return "unsupported"
    native._check(rc, "stem_conv_wrw")
    db_out = None
    if need_db:
        db_out = None if (gb is not None and db.data_ptr() == gb.data_ptr()) else db
    return (None if direct else dW), db_out
