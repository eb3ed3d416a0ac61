"""Direct RCCL communicators (``ncclCommInitAll`` over the xGMI mesh of one node) and an in-process
host loopback with the same interface (multi-worker logic testable with fewer GPUs).

The reference averages replicas with ``Nd4j.averageAndPropagate`` inside one JVM (PW:ParallelWrapper.java:316-376)
and shares encoded updates through in-memory queues (EncodedGradientsAccumulator.java:485-521). Here:

* :class:`RcclComm` binds RCCL's C API with ctypes — the copy of ``librccl.so`` that torch itself links, so the
  process holds ONE RCCL instance. Two ways to build communicators:
    - :meth:`RcclComm.init_all` (``ncclCommInitAll``): one process, one communicator per GPU, each driven by its own
      host thread — the reference's thread-per-device ParallelWrapper (parallel/inprocess.py);
    - :meth:`RcclComm.from_process_group` (``ncclGetUniqueId`` on rank 0, the 128-byte id exchanged through the
      torch.distributed store, ``ncclCommInitRank`` everywhere) — one process per GPU, bypassing ProcessGroupNCCL.
  Every collective is enqueued on the caller's current HIP stream (torch's), so it orders with the surrounding
  kernels without host waits and can be captured into a HIP graph.
* :class:`LoopbackComm` implements the same calls for N threads of one process on host (or one-device) tensors:
  deposit, barrier, sum in fixed rank order. Deterministic; used by the CPU tests of the in-process wrapper.
"""
import ctypes
import os
import threading

import torch

_NCCL_DT = {torch.float32: 7, torch.float16: 6, torch.bfloat16: 9, torch.float64: 8, torch.int32: 2,
            torch.int64: 4, torch.uint8: 1, torch.int8: 0}
_NCCL_OP = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


class NcclUniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


class RcclError(RuntimeError):
    pass


_lib = None


def library_path():
    """torch's bundled librccl (already mapped into the process), else the ROCm install's."""
    cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"), "/opt/rocm/lib/librccl.so"]
    for c in cands:
        if os.path.exists(c):
            return c
    return None


def available():
    return library_path() is not None and torch.cuda.is_available()


def _load():
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if path is None:
        raise RcclError("librccl.so not found")
    lib = ctypes.CDLL(path)
    vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(NcclUniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), ci, NcclUniqueId, ci]
    lib.ncclCommInitAll.argtypes = [ctypes.POINTER(vp), ci, ctypes.POINTER(ci)]
    lib.ncclAllReduce.argtypes = [vp, vp, sz, ci, ci, vp, vp]
    lib.ncclBroadcast.argtypes = [vp, vp, sz, ci, ci, vp, vp]
    lib.ncclAllGather.argtypes = [vp, vp, sz, ci, vp, vp]
    lib.ncclReduceScatter.argtypes = [vp, vp, sz, ci, ci, vp, vp]
    lib.ncclCommDestroy.argtypes = [vp]
    lib.ncclCommAbort.argtypes = [vp]
    lib.ncclCommGetAsyncError.argtypes = [vp, ctypes.POINTER(ci)]
    lib.ncclGetErrorString.argtypes = [ci]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    lib.ncclGroupStart.argtypes = []
    lib.ncclGroupEnd.argtypes = []
    for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommInitAll", "ncclAllReduce", "ncclBroadcast",
              "ncclAllGather", "ncclReduceScatter", "ncclCommDestroy", "ncclCommAbort", "ncclCommGetAsyncError",
              "ncclGroupStart", "ncclGroupEnd"):
        getattr(lib, f).restype = ci
    _lib = lib
    return lib


def _check(rc, what):
    if rc != 0:
        msg = _load().ncclGetErrorString(rc)
        raise RcclError(f"{what} failed: {msg.decode() if msg else rc}")


def unique_id():
    uid = NcclUniqueId()
    _check(_load().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    # raw 128 bytes: reading the c_char array field would stop at the first NUL byte
    return ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid))


class RcclComm:
    """One rank of an RCCL communicator. Collectives run on ``stream`` (default: torch's current stream of the
    communicator's device) and are asynchronous with respect to the host."""

    def __init__(self, handle, rank, nranks, device):
        self._h = ctypes.c_void_p(handle)
        self.rank, self.nranks, self.device = rank, nranks, torch.device(device)
        self._aborted = False

    # --------------------------------------------------------------------------------------------- creation
    @staticmethod
    def init_all(device_indices):
        """``ncclCommInitAll``: one communicator per listed GPU, all owned by this process."""
        lib = _load()
        n = len(device_indices)
        comms = (ctypes.c_void_p * n)()
        devs = (ctypes.c_int * n)(*device_indices)
        _check(lib.ncclCommInitAll(comms, n, devs), "ncclCommInitAll")
        return [RcclComm(comms[i], i, n, torch.device("cuda", d)) for i, d in enumerate(device_indices)]

    @staticmethod
    def init_rank(nranks, rank, uid, device):
        """``ncclCommInitRank`` with an id from :func:`unique_id` (the same bytes on every rank)."""
        lib = _load()
        u = NcclUniqueId()
        if len(uid) != ctypes.sizeof(u):
            raise RcclError(f"unique id must be {ctypes.sizeof(u)} bytes, got {len(uid)}")
        ctypes.memmove(ctypes.addressof(u), uid, len(uid))
        h = ctypes.c_void_p()
        dev = torch.device(device)
        with torch.cuda.device(dev):
            _check(lib.ncclCommInitRank(ctypes.byref(h), nranks, u, rank), "ncclCommInitRank")
        return RcclComm(h.value, rank, nranks, dev)

    @staticmethod
    def from_process_group(device=None, key="dl4j_amd/rccl_uid"):
        """A communicator over the ranks of the initialised torch.distributed default group: rank 0 draws the
        unique id and publishes it in the group's store, every rank joins with ncclCommInitRank."""
        import torch.distributed as dist
        from torch.distributed import distributed_c10d as c10d
        store = c10d._get_default_store()
        r, w = dist.get_rank(), dist.get_world_size()
        if r == 0:
            store.set(key, unique_id())
        uid = store.get(key)
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        return RcclComm.init_rank(w, r, uid, dev)

    # --------------------------------------------------------------------------------------------- collectives
    def _stream(self, stream):
        if stream is not None:
            return ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _dt(self, t):
        dt = _NCCL_DT.get(t.dtype)
        if dt is None:
            raise RcclError(f"unsupported dtype {t.dtype}")
        if not t.is_contiguous() or t.device != self.device:
            raise RcclError("tensor must be contiguous and on the communicator's device")
        return dt

    def all_reduce(self, t, op="sum", out=None, stream=None):
        """In place (or into ``out``): elementwise reduction over all ranks."""
        out = t if out is None else out
        _check(_load().ncclAllReduce(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()), t.numel(),
                                     self._dt(t), _NCCL_OP[op], self._h, self._stream(stream)), "ncclAllReduce")
        return out

    def broadcast(self, t, root=0, stream=None):
        _check(_load().ncclBroadcast(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()), t.numel(),
                                     self._dt(t), root, self._h, self._stream(stream)), "ncclBroadcast")
        return t

    def all_gather(self, send, recv, stream=None):
        """recv (nranks x send.numel() elements) <- every rank's send, in rank order."""
        assert recv.numel() == send.numel() * self.nranks
        _check(_load().ncclAllGather(ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(recv.data_ptr()),
                                     send.numel(), self._dt(send), self._h, self._stream(stream)), "ncclAllGather")
        return recv

    def reduce_scatter(self, send, recv, op="sum", stream=None):
        assert send.numel() == recv.numel() * self.nranks
        _check(_load().ncclReduceScatter(ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(recv.data_ptr()),
                                         recv.numel(), self._dt(send), _NCCL_OP[op], self._h,
                                         self._stream(stream)), "ncclReduceScatter")
        return recv

    # --------------------------------------------------------------------------------------------- health
    def async_error(self):
        """RCCL's asynchronous error code (0 = ncclSuccess); the watchdog polls it."""
        e = ctypes.c_int(0)
        _check(_load().ncclCommGetAsyncError(self._h, ctypes.byref(e)), "ncclCommGetAsyncError")
        return e.value

    def abort(self):
        if not self._aborted and self._h:
            _load().ncclCommAbort(self._h)
            self._aborted = True

    def destroy(self):
        if not self._aborted and self._h:
            _load().ncclCommDestroy(self._h)
            self._aborted = True

    @staticmethod
    def group(fn):
        """Run ``fn`` (issuing several collectives) between ncclGroupStart / ncclGroupEnd."""
        lib = _load()
        _check(lib.ncclGroupStart(), "ncclGroupStart")
        try:
            return fn()
        finally:
            _check(lib.ncclGroupEnd(), "ncclGroupEnd")


class _LoopbackState:
    def __init__(self, n):
        self.n = n
        self.slots = [None] * n
        self.barrier = threading.Barrier(n)


class LoopbackComm:
    """The RcclComm interface for N threads of one process, over host memory: each collective deposits the
    rank's tensor, waits at a barrier, combines the slots in rank order (identical bits on every rank) and waits
    again before anyone may overwrite its slot. ``abort`` breaks the barrier so every waiting rank raises."""

    def __init__(self, state, rank):
        self._s, self.rank, self.nranks = state, rank, state.n
        self.device = torch.device("cpu")

    @staticmethod
    def create(n):
        st = _LoopbackState(n)
        return [LoopbackComm(st, r) for r in range(n)]

    def _sync(self):
        try:
            self._s.barrier.wait()
        except threading.BrokenBarrierError as e:
            raise RcclError("loopback communicator aborted") from e

    def all_reduce(self, t, op="sum", out=None, stream=None):
        out = t if out is None else out
        self._s.slots[self.rank] = t
        self._sync()
        acc = self._s.slots[0].clone()
        for r in range(1, self.nranks):
            x = self._s.slots[r].to(acc.device)
            if op in ("sum", "avg"):
                acc += x
            elif op == "max":
                torch.maximum(acc, x, out=acc)
            elif op == "min":
                torch.minimum(acc, x, out=acc)
            elif op == "prod":
                acc *= x
        if op == "avg":
            acc /= self.nranks
        self._sync()
        out.copy_(acc)
        return out

    def broadcast(self, t, root=0, stream=None):
        self._s.slots[self.rank] = t
        self._sync()
        src = self._s.slots[root].clone()
        self._sync()
        t.copy_(src)
        return t

    def all_gather(self, send, recv, stream=None):
        self._s.slots[self.rank] = send
        self._sync()
        parts = [self._s.slots[r].reshape(-1).clone() for r in range(self.nranks)]
        self._sync()
        recv.reshape(-1).copy_(torch.cat(parts))
        return recv

    def reduce_scatter(self, send, recv, op="sum", stream=None):
        full = send.clone()
        self.all_reduce(full, op)
        n = recv.numel()
        recv.reshape(-1).copy_(full.reshape(-1)[self.rank * n:(self.rank + 1) * n])
        return recv

    def async_error(self):
        return 1 if self._s.barrier.broken else 0

    def abort(self):
        self._s.barrier.abort()

    def destroy(self):
        pass

    @staticmethod
    def group(fn):
        return fn()
