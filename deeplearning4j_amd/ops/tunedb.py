"""Persistent kernel-choice database (the framework's perf-db, in the role of MIOpen's find-db / hipBLASLt's tuning
files): the autotuners' per-shape decisions — GEMM tile configuration x split-K (ops/gemm.py), convolution tile
variant, weight-gradient engine, 1x1-conv GEMM-vs-implicit-GEMM (ops/conv_native.py) — keyed by (table, problem
key) for one GPU architecture.

* Lookup: ``deeplearning4j_amd/ops/tunedb/<arch>.json`` (or ``DL4J_AMD_TUNE_DB``) is read once; a shape found there
  is not re-timed, so a fresh process takes the recorded choice at its first call (no tuning pass in the first
  step, and the same kernels run from one process to the next instead of whatever won a 3-repetition timing on that
  run). ``DL4J_AMD_TUNE_DB=off`` disables the database,
  ``DL4J_AMD_TUNE_DB_SKIP=gemm`` only the named tables.
* Record: with ``DL4J_AMD_TUNE_RECORD=<file>`` every decision the autotuners make is added to that file at exit
  (merged with what it already holds); ``DL4J_AMD_TUNE_REPS`` raises the timing repetitions for such a run.
* Entries carry the schema version below; a file with another version is ignored (tile configuration ids changed).
* The file also records the compute-unit count of the device it was timed on; on a device of the same architecture
  with another CU count (a partitioned or binned part) the decisions are ignored and the autotuners re-time.
* A recorded choice a kernel refuses at launch (non-zero return code) is dropped with ``forget`` and the caller
  falls back to its planner / autotuner instead of failing.
"""
import atexit
import json
import os
import threading

import torch

VERSION = 2                 # bump when kernel-configuration ids or key layouts change
_lock = threading.Lock()
_db = None                  # {table: {repr(key): value}}
_recorded = {}
_path_used = None


def _arch():
    try:
        if not torch.cuda.is_available():
            return None
        return torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName.split(":")[0]
    except Exception:       # noqa: BLE001 — no device / no properties: no database
        return None


def _cus():
    try:
        if not torch.cuda.is_available():
            return None
        return int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
    except Exception:       # noqa: BLE001
        return None


def default_path(arch=None):
    arch = arch or _arch()
    return None if arch is None else os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunedb",
                                                  f"{arch}.json")


def _load():
    global _db, _path_used
    if _db is not None:
        return _db
    with _lock:
        if _db is not None:
            return _db
        env = os.environ.get("DL4J_AMD_TUNE_DB")
        db = {}
        if env != "off":
            p = env or default_path()
            if p and os.path.exists(p):
                try:
                    with open(p) as fh:
                        data = json.load(fh)
                    cus, want = data.get("cus"), _cus()
                    if data.get("version") == VERSION and (cus is None or want is None or cus == want):
                        db = data.get("tables", {})
                        _path_used = p
                except (OSError, ValueError):
                    db = {}
        _db = db
        return _db


def _jsonable(v):
    return list(_jsonable(x) for x in v) if isinstance(v, tuple) else v


def _native(v):
    return tuple(_native(x) for x in v) if isinstance(v, list) else v


def _skipped():
    return {t for t in os.environ.get("DL4J_AMD_TUNE_DB_SKIP", "").split(",") if t}


def lookup(table, key):
    """The recorded choice for ``key`` (tuples come back as tuples), or None. Tables named in
    ``DL4J_AMD_TUNE_DB_SKIP`` (comma-separated) are re-timed instead (re-recording one table after a kernel change)."""
    if table in _skipped():
        return None
    v = _load().get(table, {}).get(repr(key))
    return None if v is None else _native(v)


def forget(table, key):
    """Drop a loaded decision (a kernel refused it at launch), so the next call re-plans or re-times."""
    with _lock:
        _load().get(table, {}).pop(repr(key), None)
        _recorded.get(table, {}).pop(repr(key), None)


def record(table, key, value):
    """Remember an autotuner decision (kept in memory; written at exit when DL4J_AMD_TUNE_RECORD is set)."""
    with _lock:
        _recorded.setdefault(table, {})[repr(key)] = _jsonable(value)


def reps(default):
    try:
        return max(default, int(os.environ.get("DL4J_AMD_TUNE_REPS", default)))
    except ValueError:
        return default


def save(path, arch=None):
    """Merge the decisions of this process into ``path`` (same-version entries already there are kept)."""
    data = {"version": VERSION, "arch": arch or _arch(), "cus": _cus(), "tables": {}}
    if os.path.exists(path):
        try:
            with open(path) as fh:
                old = json.load(fh)
            if old.get("version") == VERSION:
                data["tables"] = old.get("tables", {})
        except (OSError, ValueError):
            pass
    with _lock:
        for t, kv in _recorded.items():
            data["tables"].setdefault(t, {}).update(kv)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        json.dump(data, fh, indent=0, sort_keys=True)
    os.replace(tmp, path)
    return sum(len(v) for v in data["tables"].values())


def loaded_from():
    _load()
    return _path_used


def _at_exit():
    p = os.environ.get("DL4J_AMD_TUNE_RECORD")
    if p and _recorded:
        try:
            save(p)
        except OSError:
            pass


atexit.register(_at_exit)
