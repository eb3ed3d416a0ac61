"""ctypes binding of ``libdl4j_amd_runtime.so`` — host (CPU) C++ runtime pieces (csrc/runtime/*.cpp):
threshold/bitmap codec for CPU tensors, tree/t-SNE helpers, data-loader helpers."""
import ctypes
import os

from .build import RUNTIME_LIB

_rt = None
c_void_p, c_int, c_ll, c_float, c_double = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, \
    ctypes.c_double

_SIGS = {
    "rt_threshold_count": ([c_void_p, c_ll, c_float], c_ll),
    "rt_threshold_encode": ([c_void_p, c_ll, c_float, c_void_p, c_int], c_int),
    "rt_threshold_decode": ([c_void_p, c_void_p, c_float], None),
    "rt_bitmap_encode": ([c_void_p, c_ll, c_float, c_void_p], c_int),
    "rt_bitmap_decode": ([c_void_p, c_void_p, c_float], None),
    "rt_ws_create": ([c_ll, c_ll, c_ll, c_double, c_int, c_int, c_int], c_ll),
    "rt_ws_destroy": ([c_ll], None),
    "rt_ws_alloc": ([c_ll, c_ll, ctypes.POINTER(c_ll), ctypes.POINTER(c_ll)], c_int),
    "rt_ws_cycle_end": ([c_ll], c_ll),
    "rt_ws_set_capacity": ([c_ll, c_ll], c_int),
    "rt_ws_generation": ([c_ll], c_ll),
    "rt_ws_stats": ([c_ll, ctypes.POINTER(c_ll)], c_int),
}


def register(name, args, res):
    _SIGS[name] = (args, res)
    if _rt is not None and hasattr(_rt, name):
        f = getattr(_rt, name)
        f.argtypes, f.restype = args, res


def load():
    """Load (building on first use if needed) the host runtime library; None if no C++ toolchain."""
    global _rt
    if _rt is not None:
        return _rt
    if not os.path.exists(RUNTIME_LIB):
        try:
            from .build import build_runtime
            build_runtime(verbose=False)
        except Exception:
            return None
    lib = ctypes.CDLL(RUNTIME_LIB)
    for name, (args, res) in _SIGS.items():
        if hasattr(lib, name):
            f = getattr(lib, name)
            f.argtypes, f.restype = args, res
    _rt = lib
    return lib


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())
