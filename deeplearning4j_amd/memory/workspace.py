"""MemoryWorkspace: named, cycle-scoped arenas in device memory (ND4J workspaces as DL4J uses them,
SURVEY §2.2 "Workspaces contract": NN:nn/graph/ComputationGraph.java:107-136, NN:nn/multilayer/MultiLayerNetwork.java:
126-144; SCOPE_PANIC tests CORET:nn/misc/WorkspaceTests.java:36-41).

Design (MI355X-first): one device buffer per (thread, workspace id), carved by the native bump allocator
(csrc/runtime/workspace.cpp) — aligned sub-allocations, cycle reset, FIRST_LOOP / OVER_TIME learning with
overallocation, spill accounting and a generation counter per cycle. Arrays handed out are plain torch views
of the buffer, so kernels and HIP-graph capture see ordinary device pointers. The default size limit is derived
from the device's free HBM (288 GB on an MI355X) instead of the reference's small host-tuned defaults.

SCOPE_PANIC: every array carved from a workspace remembers (workspace, generation). Using it after its cycle
ended (workspace closed and re-opened, or reset) raises :class:`ND4JWorkspaceException`, the reference's
"Op [...] X argument uses leaked workspace pointer" check.
"""
import contextlib
import ctypes
import enum
import threading
import weakref

import torch

from ..ops import runtime as _rt



def _device_buffer(nbytes, device):
    """The workspace's device memory: a block of the native engine's caching allocator (csrc/engine.hip, the N1
    layer) on the GPU, a torch tensor elsewhere (or when the engine cannot serve the request)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda":
        try:
            from ..runtime import device_buffer
            t = device_buffer(nbytes, dev)
            if t is not None:
                return t
        except Exception:
            pass
    return torch.empty(nbytes, dtype=torch.uint8, device=dev)

class AllocationPolicy(enum.Enum):
    STRICT = 0
    OVERALLOCATE = 1


class LearningPolicy(enum.Enum):
    NONE = 0
    FIRST_LOOP = 1
    OVER_TIME = 2


class ResetPolicy(enum.Enum):
    BLOCK_LEFT = 0
    ENDOFBUFFER_REACHED = 1


class SpillPolicy(enum.Enum):
    EXTERNAL = 0
    REALLOCATE = 1
    FAIL = 2


class MirroringPolicy(enum.Enum):
    FULL = 0
    HOST_ONLY = 1


class LocationPolicy(enum.Enum):
    RAM = 0
    MMAP = 1


class ND4JWorkspaceException(RuntimeError):
    pass


class WorkspaceConfiguration:
    """Builder-configured workspace policy (ND4J WorkspaceConfiguration)."""

    def __init__(self, initialSize=0, maxSize=0, overallocationLimit=0.0, policyAllocation=AllocationPolicy.OVERALLOCATE,
                 policyLearning=LearningPolicy.FIRST_LOOP, policyReset=ResetPolicy.BLOCK_LEFT,
                 policySpill=SpillPolicy.EXTERNAL, policyMirroring=MirroringPolicy.FULL,
                 policyLocation=LocationPolicy.RAM, cyclesBeforeInitialization=0, alignment=256):
        self.initialSize = int(initialSize)
        self.maxSize = int(maxSize)
        self.overallocationLimit = float(overallocationLimit)
        self.policyAllocation = policyAllocation
        self.policyLearning = policyLearning
        self.policyReset = policyReset
        self.policySpill = policySpill
        self.policyMirroring = policyMirroring
        self.policyLocation = policyLocation
        self.cyclesBeforeInitialization = int(cyclesBeforeInitialization)
        self.alignment = int(alignment)

    class Builder:
        def __init__(self):
            self._kw = {}

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)

            def setter(v):
                self._kw[name] = v
                return self
            return setter

        def build(self):
            return WorkspaceConfiguration(**self._kw)

    @staticmethod
    def builder():
        return WorkspaceConfiguration.Builder()


def default_max_bytes(device=None, fraction=0.5):
    """Size cap for one workspace: a fraction of the free device memory (≈288 GB HBM3E on an MI355X)."""
    if device is not None and torch.device(device).type == "cuda" and torch.cuda.is_available():
        free, _total = torch.cuda.mem_get_info(torch.device(device))
        return int(free * fraction)
    return 0


_registry = {}   # id(tensor) -> (weakref(tensor), workspace, generation); entries drop with their tensor


def _register(t, ws, gen):
    key = id(t)
    _registry[key] = (weakref.ref(t, lambda _r, k=key: _registry.pop(k, None)), ws, gen)


def _lookup(t):
    rec = _registry.get(id(t))
    if rec is None or rec[0]() is not t:
        return None
    return rec[1], rec[2]


class MemoryWorkspace:
    """One named arena. Use as a context manager (``notifyScopeEntered`` / ``notifyScopeLeft``) or via
    :meth:`WorkspaceManager.getAndActivateWorkspace`."""

    def __init__(self, conf, ws_id, device=None, manager=None):
        self.conf = conf
        self.id = ws_id
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.manager = manager
        lib = _rt.load()
        if lib is None:
            raise RuntimeError("native runtime library unavailable (workspace arena)")
        self._lib = lib
        maxb = conf.maxSize or default_max_bytes(self.device)
        overalloc = conf.overallocationLimit if conf.policyAllocation == AllocationPolicy.OVERALLOCATE else 0.0
        self._h = lib.rt_ws_create(conf.initialSize, maxb, conf.alignment, overalloc, conf.policyLearning.value,
                                   conf.policyReset.value, conf.cyclesBeforeInitialization)
        self._buf = _device_buffer(max(conf.initialSize, 0), self.device) if conf.initialSize > 0 else None
        self.active = False
        self.parent = None
        self.external_bytes = 0
        # frozen: the buffer never moves (a captured HIP graph holds its addresses): no growth at cycle end, and an
        # allocation beyond it spills to the caching allocator (captured into the graph's own pool)
        self.frozen = False

    # ------------------------------------------------------------------ scope
    def notifyScopeEntered(self):
        if self.manager is not None:
            self.parent = self.manager._current
            self.manager._current = self
        self.active = True
        return self

    def notifyScopeLeft(self):
        self.active = False
        if self.manager is not None and self.manager._current is self:
            self.manager._current = self.parent
        want = self._lib.rt_ws_cycle_end(self._h)
        cap = self._buf.numel() if self._buf is not None else 0
        if want > cap and not self.frozen:
            self._buf = None                                  # the old block returns to the engine first
            if self.device.type == "cuda":
                # ... and the engine hands it back to the driver (hipFree, which also waits for every stream that
                # may still read it, the weight-gradient overlap stream included), so the caching allocator of torch
                # can reuse the memory instead of failing while the engine sits on a free segment
                try:
                    from ..runtime import allocator
                    allocator(self.device.index or 0).empty_cache()
                except Exception:
                    pass
            self._buf = _device_buffer(want, self.device)
            self._lib.rt_ws_set_capacity(self._h, want)
        self.external_bytes = 0

    close = notifyScopeLeft

    def __enter__(self):
        return self.notifyScopeEntered()

    def __exit__(self, *a):
        self.notifyScopeLeft()
        return False

    def isScopeActive(self):
        return self.active

    def getId(self):
        return self.id

    # ------------------------------------------------------------------ allocation
    def create(self, shape, dtype=torch.float32, zero=False):
        """A [shape] array carved from this workspace (or spilled per policySpill)."""
        if not self.active:
            raise ND4JWorkspaceException(f"workspace {self.id} is not open")
        shape = tuple(int(s) for s in (shape if isinstance(shape, (list, tuple)) else (shape,)))
        n = 1
        for s in shape:
            n *= s
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        off = _rt.c_ll(0)
        gen = _rt.c_ll(0)
        rc = self._lib.rt_ws_alloc(self._h, nbytes, ctypes.byref(off), ctypes.byref(gen))
        if rc == 0 and self._buf is not None and off.value + nbytes <= self._buf.numel():
            t = self._buf[off.value:off.value + nbytes].view(dtype).view(shape)
        else:
            if self.conf.policySpill == SpillPolicy.FAIL and not self.frozen:
                raise ND4JWorkspaceException(f"workspace {self.id}: allocation of {nbytes} bytes exceeds the arena "
                                             f"and policySpill=FAIL")
            t = torch.empty(shape, dtype=dtype, device=self.device)   # EXTERNAL / REALLOCATE: grown at cycle end
            self.external_bytes += nbytes
        if zero:
            t.zero_()
        _register(t, self, gen.value)
        return t

    def getGeneration(self):
        return self._lib.rt_ws_generation(self._h)

    def stats(self):
        out = (ctypes.c_longlong * 10)()
        self._lib.rt_ws_stats(self._h, out)
        keys = ["capacity", "offset", "cyclePeak", "maxPeak", "spilled", "spilledTotal", "allocations", "cycles",
                "generation", "learned"]
        return dict(zip(keys, list(out)))

    def getCurrentSize(self):
        return self.stats()["capacity"]

    def getPrimaryOffset(self):
        return self.stats()["offset"]

    def destroyWorkspace(self):
        self._buf = None
        if self._h:
            self._lib.rt_ws_destroy(self._h)
            self._h = 0

    def __del__(self):
        try:
            self.destroyWorkspace()
        except Exception:
            pass


def owner_of(t):
    return _lookup(t)


def check_scope(t, where="array"):
    """SCOPE_PANIC: raise if ``t`` was carved from a workspace cycle that has since ended."""
    rec = _lookup(t)
    if rec is None:
        return
    ws, gen = rec
    if not ws.active or ws.getGeneration() != gen:
        raise ND4JWorkspaceException(f"Op [{where}] uses leaked workspace pointer from workspace [{ws.id}] "
                                     f"(generation {gen}, current {ws.getGeneration()}, open={ws.active})")


def leverageTo(t, ws_id, manager=None):
    """Copy ``t`` into the (open) workspace ``ws_id`` of this thread; detached copy if it is not open."""
    manager = manager or getWorkspaceManager()
    ws = manager._ws.get(ws_id)
    if ws is None or not ws.active:
        return detach(t)
    out = ws.create(t.shape, t.dtype)
    out.copy_(t)
    return out


def detach(t):
    """A copy of ``t`` that belongs to no workspace."""
    return t.clone()


class WorkspaceManager:
    """Per-thread workspace registry (Nd4j.getWorkspaceManager())."""

    def __init__(self):
        self._ws = {}
        self._current = None

    def getWorkspaceForCurrentThread(self, conf=None, ws_id="DEFAULT", device=None):
        ws = self._ws.get(ws_id)
        if ws is None:
            ws = MemoryWorkspace(conf or WorkspaceConfiguration(), ws_id, device, self)
            self._ws[ws_id] = ws
        return ws

    def getAndActivateWorkspace(self, conf=None, ws_id="DEFAULT", device=None):
        return self.getWorkspaceForCurrentThread(conf, ws_id, device).notifyScopeEntered()

    def checkIfWorkspaceExists(self, ws_id):
        return ws_id in self._ws

    def checkIfWorkspaceExistsAndActive(self, ws_id):
        ws = self._ws.get(ws_id)
        return ws is not None and ws.active

    def getCurrentWorkspace(self):
        return self._current

    @contextlib.contextmanager
    def scopeOutOfWorkspaces(self):
        prev = self._current
        self._current = None
        try:
            yield
        finally:
            self._current = prev

    def destroyAllWorkspacesForCurrentThread(self):
        for ws in self._ws.values():
            ws.destroyWorkspace()
        self._ws = {}
        self._current = None

    def printAllocationStatisticsForCurrentThread(self):
        lines = [f"{k}: {v.stats()}" for k, v in self._ws.items()]
        s = "\n".join(lines)
        print(s)
        return s


_tls = threading.local()


def getWorkspaceManager():
    m = getattr(_tls, "mgr", None)
    if m is None:
        m = _tls.mgr = WorkspaceManager()
    return m


# Workspace ids the reference's networks use (ComputationGraph.java:107-136 / MultiLayerNetwork.java:126-144)
WS_LAYER_WORKING_MEM = "WS_LAYER_WORKING_MEM"
WS_ALL_LAYERS_ACT = "WS_ALL_LAYERS_ACT"
WS_RNN_LOOP_WORKING_MEM = "WS_RNN_LOOP_WORKING_MEM"
WS_OUTPUT_MEM = "WS_OUTPUT_MEM"
LOOP_EXTERNAL = "LOOP_EXTERNAL"
LOOP_FF = "LOOP_FF"
LOOP_BP = "LOOP_BP"
LOOP_TBPTT = "LOOP_TBPTT"
LOOP_CACHE = "LOOP_CACHE"
LOOP_LSTM = "LOOP_LSTM"
