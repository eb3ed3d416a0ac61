"""N1 native engine bindings (csrc/engine.hip): devices, streams, events, HIP graphs, the stream-ordered caching
device allocator and the op registry of the kernel library.

The reference gets this layer from libnd4j's CUDA backend (nd4j-cuda AffinityManager / CudaContext streams, the
AtomicAllocator memory handler and the NativeOps op table). Here it is C++ over the HIP runtime
with a ctypes C ABI; framework tensors can live in its memory through DLPack (``Allocator.empty``), which is how the
workspace arenas (memory/workspace.py) get their device buffers.
"""
import ctypes
import threading

import torch

from ..ops import native as _native

c_int, c_ll, c_void_p, c_float = ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_float


class DeviceProps(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 128), ("arch", ctypes.c_char * 64), ("cus", c_int), ("xcds", c_int),
                ("warp", c_int), ("max_threads", c_int), ("lds_per_block", c_int), ("clock_khz", c_int),
                ("mem_clock_khz", c_int), ("bus_width", c_int), ("pci_bus", c_int), ("total_mem", c_ll),
                ("l2_bytes", c_ll), ("lds_per_cu", c_ll)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["name"] = d["name"].decode(errors="replace")
        d["arch"] = d["arch"].decode(errors="replace")
        return d


_SIGS = {
    "dl4j_rt_device_count": ([], c_int),
    "dl4j_rt_device_props": ([c_int, ctypes.POINTER(DeviceProps)], c_int),
    "dl4j_rt_set_device": ([c_int], c_int),
    "dl4j_rt_get_device": ([], c_int),
    "dl4j_rt_device_sync": ([c_int], c_int),
    "dl4j_rt_mem_info": ([c_int, ctypes.POINTER(c_ll), ctypes.POINTER(c_ll)], c_int),
    "dl4j_rt_stream_create": ([c_int, c_int, ctypes.POINTER(c_void_p)], c_int),
    "dl4j_rt_stream_destroy": ([c_void_p], c_int),
    "dl4j_rt_stream_sync": ([c_void_p], c_int),
    "dl4j_rt_stream_query": ([c_void_p], c_int),
    "dl4j_rt_stream_wait_event": ([c_void_p, c_void_p], c_int),
    "dl4j_rt_event_create": ([c_int, ctypes.POINTER(c_void_p)], c_int),
    "dl4j_rt_event_destroy": ([c_void_p], c_int),
    "dl4j_rt_event_record": ([c_void_p, c_void_p], c_int),
    "dl4j_rt_event_sync": ([c_void_p], c_int),
    "dl4j_rt_event_query": ([c_void_p], c_int),
    "dl4j_rt_event_elapsed": ([c_void_p, c_void_p, ctypes.POINTER(c_float)], c_int),
    "dl4j_rt_capture_begin": ([c_void_p, c_int, c_int], c_int),
    "dl4j_rt_capture_end": ([c_void_p, c_int, ctypes.POINTER(c_void_p)], c_int),
    "dl4j_rt_graph_launch": ([c_void_p, c_void_p], c_int),
    "dl4j_rt_graph_node_count": ([c_void_p], c_ll),
    "dl4j_rt_graph_destroy": ([c_void_p], c_int),
    "dl4j_rt_malloc": ([c_int, c_ll, c_void_p, ctypes.POINTER(c_void_p)], c_int),
    "dl4j_rt_free": ([c_int, c_void_p], c_int),
    "dl4j_rt_record_stream": ([c_int, c_void_p, c_void_p], c_int),
    "dl4j_rt_free_pool": ([c_int, c_int], c_int),
    "dl4j_rt_empty_cache": ([c_int], c_ll),
    "dl4j_rt_alloc_stats": ([c_int, ctypes.POINTER(c_ll)], c_int),
    "dl4j_rt_reset_peak": ([c_int], c_int),
    "dl4j_rt_dlpack_empty": ([c_int, c_int, ctypes.POINTER(c_ll), c_int, c_int, c_void_p, ctypes.POINTER(c_int)],
                             c_void_p),
    "dl4j_rt_op_count": ([], c_int),
    "dl4j_rt_op_info": ([c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                         ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_void_p)], c_int),
}
_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                L = _native.load()
                for name, (args, res) in _SIGS.items():
                    f = getattr(L, name)
                    f.argtypes = args
                    f.restype = res
                _lib = L
    return _lib


class EngineError(RuntimeError):
    pass


def _ok(rc, what):
    if rc != 0:
        raise EngineError(f"{what} failed with code {rc}")


# ---------------------------------------------------------------------------------------------------------- devices
def device_count():
    n = lib().dl4j_rt_device_count()
    return max(n, 0)


def device_props(dev=0):
    p = DeviceProps()
    _ok(lib().dl4j_rt_device_props(dev, ctypes.byref(p)), "device_props")
    return p.as_dict()


def mem_info(dev=0):
    f, t = c_ll(), c_ll()
    _ok(lib().dl4j_rt_mem_info(dev, ctypes.byref(f), ctypes.byref(t)), "mem_info")
    return f.value, t.value


def synchronize(dev=0):
    _ok(lib().dl4j_rt_device_sync(dev), "device_sync")


# --------------------------------------------------------------------------------------------------- streams/events
class Stream:
    """A native HIP stream (non-blocking; ``high_priority`` for latency-critical work such as gradient
    communication). ``torch_stream()`` wraps it for torch so framework kernels can be enqueued on it."""

    def __init__(self, device=0, high_priority=False, handle=None, cus=0):
        """``cus`` > 0: restrict the stream's kernels to that many CUs (hardware queue CU mask, spread evenly)."""
        self.device = device
        self._own = handle is None
        if handle is None:
            h = c_void_p()
            if cus > 0:
                _ok(lib().dl4j_rt_stream_create_cumask(device, int(cus), ctypes.byref(h)), "stream_create_cumask")
            else:
                _ok(lib().dl4j_rt_stream_create(device, 1 if high_priority else 0, ctypes.byref(h)), "stream_create")
            handle = h.value
        self.handle = handle

    def cu_count(self):
        r = lib().dl4j_rt_stream_cu_count(self.ptr)
        if r < 0:
            raise EngineError(f"stream_cu_count {r}")
        return r

    @property
    def ptr(self):
        return c_void_p(self.handle)

    def synchronize(self):
        _ok(lib().dl4j_rt_stream_sync(self.ptr), "stream_sync")

    def query(self):
        r = lib().dl4j_rt_stream_query(self.ptr)
        if r < 0:
            raise EngineError(f"stream_query {r}")
        return bool(r)

    def wait_event(self, ev):
        _ok(lib().dl4j_rt_stream_wait_event(self.ptr, ev.ptr), "stream_wait_event")

    def torch_stream(self):
        return torch.cuda.ExternalStream(self.handle, device=torch.device("cuda", self.device))

    def close(self):
        if self._own and self.handle:
            lib().dl4j_rt_stream_destroy(self.ptr)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Event:
    def __init__(self, timing=True):
        h = c_void_p()
        _ok(lib().dl4j_rt_event_create(1 if timing else 0, ctypes.byref(h)), "event_create")
        self.handle = h.value

    @property
    def ptr(self):
        return c_void_p(self.handle)

    def record(self, stream):
        _ok(lib().dl4j_rt_event_record(self.ptr, stream.ptr), "event_record")

    def synchronize(self):
        _ok(lib().dl4j_rt_event_sync(self.ptr), "event_sync")

    def query(self):
        return lib().dl4j_rt_event_query(self.ptr) == 1

    def elapsed_ms(self, end):
        ms = c_float()
        _ok(lib().dl4j_rt_event_elapsed(self.ptr, end.ptr, ctypes.byref(ms)), "event_elapsed")
        return ms.value

    def __del__(self):
        try:
            if self.handle:
                lib().dl4j_rt_event_destroy(self.ptr)
        except Exception:
            pass


# ------------------------------------------------------------------------------------------------------------ graphs
class Graph:
    """Capture everything enqueued on ``stream`` between ``capture_begin`` / ``capture_end`` into a HIP graph;
    allocations made through the engine allocator on that stream during the capture come from a private pool that
    stays reserved until the graph is destroyed."""

    CAPTURE_GLOBAL, CAPTURE_THREAD_LOCAL, CAPTURE_RELAXED = 0, 1, 2

    def __init__(self, stream):
        self.stream = stream
        self.handle = None

    def capture_begin(self, mode=CAPTURE_THREAD_LOCAL):
        _ok(lib().dl4j_rt_capture_begin(self.stream.ptr, self.stream.device, mode), "capture_begin")

    def capture_end(self):
        h = c_void_p()
        _ok(lib().dl4j_rt_capture_end(self.stream.ptr, self.stream.device, ctypes.byref(h)), "capture_end")
        self.handle = h.value

    def replay(self, stream=None):
        _ok(lib().dl4j_rt_graph_launch(c_void_p(self.handle), (stream or self.stream).ptr), "graph_launch")

    def num_nodes(self):
        return lib().dl4j_rt_graph_node_count(c_void_p(self.handle))

    def destroy(self):
        if self.handle:
            lib().dl4j_rt_graph_destroy(c_void_p(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# --------------------------------------------------------------------------------------------------------- allocator
_DL_CODES = {torch.float32: (2, 32), torch.float16: (2, 16), torch.bfloat16: (4, 16), torch.float64: (2, 64),
             torch.int32: (0, 32), torch.int64: (0, 64), torch.int8: (0, 8), torch.uint8: (1, 8),
             torch.int16: (0, 16)}

_PyCapsule_New = ctypes.pythonapi.PyCapsule_New
_PyCapsule_New.restype = ctypes.py_object
_PyCapsule_New.argtypes = [c_void_p, ctypes.c_char_p, c_void_p]


class Allocator:
    """Per-device stream-ordered caching allocator (csrc/engine.hip). ``empty`` returns a torch tensor whose memory is
    an engine block (DLPack, freed back to the engine when the tensor dies)."""

    def __init__(self, device=0):
        self.device = device

    def malloc(self, nbytes, stream=None):
        p = c_void_p()
        r = lib().dl4j_rt_malloc(self.device, int(nbytes), stream.ptr if stream is not None else None,
                                 ctypes.byref(p))
        if r == -2:
            raise EngineError("allocation inside a capture that its pool cannot serve (warm the stream up first)")
        _ok(r, "malloc")
        return p.value

    def free(self, ptr):
        _ok(lib().dl4j_rt_free(self.device, c_void_p(ptr)), "free")

    def record_stream(self, ptr, stream):
        _ok(lib().dl4j_rt_record_stream(self.device, c_void_p(ptr), stream.ptr), "record_stream")

    def empty(self, shape, dtype=torch.uint8, stream=None):
        """Contiguous torch tensor over an engine block; ``stream`` (engine Stream, default: the null stream) is the
        stream the block is ordered on."""
        shape = tuple(int(s) for s in shape)
        code, bits = _DL_CODES[dtype]
        arr = (c_ll * max(1, len(shape)))(*shape)
        err = c_int()
        h = lib().dl4j_rt_dlpack_empty(self.device, len(shape), arr, code, bits,
                                       stream.ptr if stream is not None else None, ctypes.byref(err))
        if not h:
            raise EngineError(f"dlpack_empty failed with code {err.value}")
        cap = _PyCapsule_New(h, b"dltensor", None)
        return torch.utils.dlpack.from_dlpack(cap)

    def stats(self):
        v = (c_ll * 7)()
        _ok(lib().dl4j_rt_alloc_stats(self.device, v), "alloc_stats")
        keys = ("allocated", "reserved", "peak", "segments", "allocs", "cache_hits", "frees")
        return dict(zip(keys, list(v)))

    def reset_peak(self):
        lib().dl4j_rt_reset_peak(self.device)

    def empty_cache(self):
        return lib().dl4j_rt_empty_cache(self.device)


_allocators = {}


def allocator(device=0):
    a = _allocators.get(device)
    if a is None:
        a = _allocators[device] = Allocator(device)
    return a


def device_buffer(nbytes, device):
    """uint8 device buffer of ``nbytes`` from the engine allocator (None when the engine cannot serve it, e.g. no
    GPU, or inside a torch graph capture; the caller then allocates through torch)."""
    dev = torch.device(device)
    if dev.type != "cuda" or torch.cuda.is_current_stream_capturing():
        return None
    try:
        return allocator(dev.index or 0).empty((max(int(nbytes), 1),), torch.uint8)[:int(nbytes)]
    except Exception:
        return None


# ------------------------------------------------------------------------------------------------------- op registry
def ops():
    """[(name, signature, description, has_entry_point)] of the kernel library's op table."""
    L = lib()
    out = []
    for i in range(L.dl4j_rt_op_count()):
        n, s, w, f = ctypes.c_char_p(), ctypes.c_char_p(), ctypes.c_char_p(), c_void_p()
        if L.dl4j_rt_op_info(i, ctypes.byref(n), ctypes.byref(s), ctypes.byref(w), ctypes.byref(f)) == 0:
            out.append((n.value.decode(), s.value.decode(), w.value.decode(), bool(f.value)))
    return out
