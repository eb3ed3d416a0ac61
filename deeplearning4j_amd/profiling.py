"""Tracing / profiling / numerical panics.

Reference behaviour being replaced:
* ND4J ``OpExecutioner.ProfilingMode`` — DISABLED / NAN_PANIC / INF_PANIC / ANY_PANIC / SCOPE_PANIC /
  OPERATIONS / ALL, set with ``Nd4j.getExecutioner().setProfilingMode`` (on in every core test,
  CORET:BaseDL4JTest.java:11-16); ``commit()`` as the device sync point (PW:trainer/DefaultTrainer.java:141).
* ``PerformanceListener`` / ``SleepyTrainingListener`` phase tracing (NN:optimize/listeners/*), the Spark
  ``EventStats`` HTML timeline (SPK:stats/StatsUtils.java:72-105).

MI355X-native equivalents:
* **roctx ranges** (``libroctx64``) around every layer forward/backward, the updater and collectives, so a
  ``rocprofv3 --marker-trace`` run attributes kernels to layers.
* **Panic checks**: after each layer forward/backward, one ``dl4j_nonfinite_count`` launch (csrc/checks.hip)
  counts NaN/Inf over the layer output and its gradient views; a hit raises :class:`ND4JOpProfilerException`
  naming the layer and phase. SCOPE_PANIC checks workspace-scoped arrays against their arena generation
  (``deeplearning4j_amd.memory``).
* **Per-layer HIP-event timing + Chrome trace export** (``chrome://tracing`` / Perfetto JSON) replacing the Spark
  HTML timeline; :class:`LayerTimingListener` aggregates per-layer milliseconds.

Everything is off by default: the hooks are two attribute checks per layer call, and captured HIP-graph steps
run no Python at all.
"""
import ctypes
import enum
import json
import os
import threading
import time

import torch


class ProfilingMode(enum.Enum):
    DISABLED = 0
    NAN_PANIC = 1
    INF_PANIC = 2
    ANY_PANIC = 3
    SCOPE_PANIC = 4
    OPERATIONS = 5
    METHODS = 6
    ALL = 7

    @staticmethod
    def of(v):
        if isinstance(v, ProfilingMode):
            return v
        return ProfilingMode[str(v).upper()]


class ND4JOpProfilerException(RuntimeError):
    """Raised by the NaN/Inf panic checks (reference: ND4JOpProfilerException / ND4JIllegalStateException)."""


# ------------------------------------------------------------------------------------------------ roctx
class _Roctx:
    def __init__(self):
        self.lib = None
        self.tried = False

    def load(self):
        if not self.tried:
            self.tried = True
            for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    self.lib = lib
                    break
                except OSError:
                    continue
        return self.lib

    def push(self, msg):
        lib = self.load()
        if lib is not None:
            lib.roctxRangePushA(msg.encode())

    def pop(self):
        if self.lib is not None:
            self.lib.roctxRangePop()

    def mark(self, msg):
        lib = self.load()
        if lib is not None:
            lib.roctxMarkA(msg.encode())


roctx = _Roctx()


# ------------------------------------------------------------------------------------------------ checks
class _CheckSeg(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("n", ctypes.c_longlong), ("dtype", ctypes.c_int), ("pad", ctypes.c_int)]


def nonfinite_counts(tensors):
    """[(nan_count, inf_count)] per tensor. GPU fp32/bf16 tensors go through one native launch; the rest use torch."""
    out = [None] * len(tensors)
    gpu = []
    for i, t in enumerate(tensors):
        if t is None or not torch.is_tensor(t) or not t.is_floating_point() or t.numel() == 0:
            out[i] = (0, 0)
        elif t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous():
            gpu.append(i)
        else:
            tf = t.detach()
            out[i] = (int(torch.isnan(tf).sum()), int(torch.isinf(tf).sum()))
    if gpu:
        from .ops import native
        lib = native.load()
        native.register_sig("dl4j_nonfinite_count", [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_longlong, ctypes.c_void_p])
        arr = (_CheckSeg * len(gpu))()
        maxn = 0
        for j, i in enumerate(gpu):
            t = tensors[i]
            arr[j].ptr, arr[j].n, arr[j].dtype = t.data_ptr(), t.numel(), 1 if t.dtype == torch.bfloat16 else 0
            maxn = max(maxn, t.numel())
        dev = tensors[gpu[0]].device
        seg_dev = torch.empty(ctypes.sizeof(arr), dtype=torch.uint8, device=dev)
        counts = torch.empty(2 * len(gpu), dtype=torch.int64, device=dev)
        rc = lib.dl4j_nonfinite_count(ctypes.cast(arr, ctypes.c_void_p), len(gpu), ctypes.c_void_p(seg_dev.data_ptr()),
                                      ctypes.c_void_p(counts.data_ptr()), maxn,
                                      ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        if rc != 0:
            raise RuntimeError(f"dl4j_nonfinite_count failed ({rc})")
        c = counts.cpu().tolist()                                    # synchronises: panic mode only
        for j, i in enumerate(gpu):
            out[i] = (c[2 * j], c[2 * j + 1])
    return out


# ------------------------------------------------------------------------------------------------ executioner
class _Event:
    __slots__ = ("name", "cat", "t0", "t1", "e0", "e1", "tid")


class OpExecutioner:
    """The ``Nd4j.getExecutioner()`` surface DL4J code and tests use: profiling mode, commit(), trace capture."""

    def __init__(self):
        self.mode = ProfilingMode.DISABLED
        self.roctx_enabled = os.environ.get("DL4J_AMD_ROCTX", "0") == "1"
        self.tracing = False
        self._events = []
        self._lock = threading.Lock()
        self._base = None
        self._stack = threading.local()

    # ------------------------------------------------------------------ configuration
    def setProfilingMode(self, mode):
        self.mode = ProfilingMode.of(mode)
        _refresh_active()

    def getProfilingMode(self):
        return self.mode

    def enableRoctx(self, on=True):
        self.roctx_enabled = bool(on)
        _refresh_active()

    def commit(self):
        """Device sync point (reference GridExecutioner.commit before device hand-offs)."""
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def panics(self):
        return self.mode in (ProfilingMode.NAN_PANIC, ProfilingMode.INF_PANIC, ProfilingMode.ANY_PANIC,
                             ProfilingMode.ALL)

    # ------------------------------------------------------------------ tracing
    def startTrace(self):
        with self._lock:
            self._events = []
            self._base = None
        self.tracing = True
        _refresh_active()

    def stopTrace(self):
        self.tracing = False
        _refresh_active()
        return self.resolve()

    def _now_event(self, device):
        if device is not None and device.type == "cuda":
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return None

    def begin(self, name, cat, device=None):
        tok = None
        if self.roctx_enabled:
            roctx.push(f"{cat}:{name}")
        if self.tracing:
            ev = _Event()
            ev.name, ev.cat, ev.tid = name, cat, threading.get_ident() & 0xFFFF
            ev.t0 = time.perf_counter()
            ev.e0 = self._now_event(device)
            if self._base is None:
                self._base = (ev.t0, ev.e0)
            tok = ev
        return tok

    def end(self, tok, device=None):
        if self.roctx_enabled:
            roctx.pop()
        if tok is not None:
            tok.e1 = self._now_event(device)
            tok.t1 = time.perf_counter()
            with self._lock:
                self._events.append(tok)

    def resolve(self):
        """Chrome-trace events [{name, cat, ph: X, ts, dur, pid, tid}] with device time from HIP events."""
        self.commit()
        out = []
        with self._lock:
            evs, base = list(self._events), self._base
        if base is None:
            return out
        t_base, e_base = base
        for ev in evs:
            if ev.e0 is not None and ev.e1 is not None and e_base is not None:
                ts = e_base.elapsed_time(ev.e0) * 1000.0
                dur = ev.e0.elapsed_time(ev.e1) * 1000.0
            else:
                ts = (ev.t0 - t_base) * 1e6
                dur = (ev.t1 - ev.t0) * 1e6
            out.append({"name": ev.name, "cat": ev.cat, "ph": "X", "ts": round(ts, 3), "dur": round(max(dur, 0.0), 3),
                        "pid": os.getpid(), "tid": ev.tid})
        return out

    def exportChromeTrace(self, path, events=None):
        events = self.resolve() if events is None else events
        with open(path, "w") as fh:
            json.dump({"traceEvents": events, "displayTimeUnit": "ms"}, fh)
        return path

    # ------------------------------------------------------------------ panic checks
    def check(self, where, tensors):
        if not self.panics():
            return
        counts = nonfinite_counts(tensors)
        nan = sum(c[0] for c in counts)
        inf = sum(c[1] for c in counts)
        m = self.mode
        if nan and m in (ProfilingMode.NAN_PANIC, ProfilingMode.ANY_PANIC, ProfilingMode.ALL):
            raise ND4JOpProfilerException(f"P.A.N.I.C.! Op.Z() contains {nan} NaN value(s): {where}")
        if inf and m in (ProfilingMode.INF_PANIC, ProfilingMode.ANY_PANIC, ProfilingMode.ALL):
            raise ND4JOpProfilerException(f"P.A.N.I.C.! Op.Z() contains {inf} Inf value(s): {where}")


_executioner = OpExecutioner()
ACTIVE = False          # hot-path switch read by the network loops


def _refresh_active():
    global ACTIVE
    e = _executioner
    ACTIVE = bool(e.roctx_enabled or e.tracing or e.mode != ProfilingMode.DISABLED)


_refresh_active()


def getExecutioner():
    return _executioner


def _flat(x):
    if x is None:
        return []
    if torch.is_tensor(x):
        return [x.contiguous() if not x.is_contiguous() else x]
    if isinstance(x, dict):
        return [t for v in x.values() for t in _flat(v)]
    if isinstance(x, (list, tuple)):
        return [t for v in x for t in _flat(v)]
    return []


def layer_begin(kind, name, layer):
    """Hook before a layer forward ('fwd') / backward ('bwd'). Returns a token for layer_end."""
    dev = getattr(getattr(layer, "net", None), "device", None)
    return _executioner.begin(f"{name}:{type(layer).__name__}", kind, dev), dev


def layer_end(tok, kind, name, layer, out):
    t, dev = tok
    _executioner.end(t, dev)
    if _executioner.panics():
        ts = _flat(out)
        if kind == "bwd":
            ts += _flat(getattr(layer, "grads", None))
        _executioner.check(f"layer {name} ({type(layer).__name__}) {'forward' if kind == 'fwd' else 'backward'}", ts)
    if _executioner.mode == ProfilingMode.SCOPE_PANIC:
        from .memory import workspace
        for t_ in _flat(out):
            workspace.check_scope(t_, f"layer {name} output")


class range_:
    """``with profiling.range_("updater"):`` — a roctx range + trace event around any region."""

    def __init__(self, name, cat="region", device=None):
        self.name, self.cat, self.device = name, cat, device

    def __enter__(self):
        self.tok = _executioner.begin(self.name, self.cat, self.device) if ACTIVE else None
        self.on = ACTIVE
        return self

    def __exit__(self, *a):
        if self.on:
            _executioner.end(self.tok, self.device)
        return False


# ------------------------------------------------------------------------------------------------ listener
class LayerTimingListener:
    """Per-layer forward/backward device time (HIP events), aggregated every ``frequency`` iterations.
    ``exportChromeTrace(path)`` writes the collected timeline (replacement for the Spark HTML timeline)."""

    def __init__(self, frequency=1):
        self.frequency = max(1, int(frequency))
        self.totals = {}
        self.counts = {}
        self.iterations = 0
        self.events = []
        _executioner.startTrace()

    def iterationDone(self, model, iteration, epoch):
        if iteration % self.frequency:
            return
        evs = _executioner.resolve()
        self.events.extend(evs)
        with _executioner._lock:
            _executioner._events = []
            _executioner._base = None
        for e in evs:
            k = (e["cat"], e["name"])
            self.totals[k] = self.totals.get(k, 0.0) + e["dur"] / 1000.0
            self.counts[k] = self.counts.get(k, 0) + 1
        self.iterations += self.frequency

    def stats(self):
        """{(phase, layer): mean ms per call}."""
        return {k: self.totals[k] / self.counts[k] for k in self.totals}

    def summary(self, top=20):
        rows = sorted(self.stats().items(), key=lambda kv: -kv[1])[:top]
        return "\n".join(f"{c:>4} {n:<48} {ms:9.3f} ms" for (c, n), ms in rows)

    def exportChromeTrace(self, path):
        return _executioner.exportChromeTrace(path, self.events)

    def close(self):
        _executioner.stopTrace()
