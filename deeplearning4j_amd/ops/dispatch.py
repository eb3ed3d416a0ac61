"""Kernel dispatch policy.

On an MI355X the hot ops run hand-written HIP kernels from ``libdl4j_amd_kernels.so`` (built from
``csrc/*.hip`` for gfx950, loaded with ctypes; see ``deeplearning4j_amd.ops.native``). On CPU the
same ops run the plain-torch reference implementations in this package (the numerics oracle).

Policy knobs (environment, ``DL4J_AMD_*`` namespace — the survey's ``mi355.*`` flag namespace):
  DL4J_AMD_NATIVE=0          force the torch reference path even on GPU (A/B testing)
  DL4J_AMD_ALLOW_FALLBACK=1  allow silent fallback when the native library is missing on a GPU box
                             (default: raise — a missing extension must fail loudly)
  DL4J_AMD_KERNEL_<OP>=0     disable one native op (e.g. DL4J_AMD_KERNEL_CONV=0)
"""
import os

import torch

_state = {"checked": False, "lib": None, "error": None}


def native_lib():
    if not _state["checked"]:
        _state["checked"] = True
        try:
            from . import native
            _state["lib"] = native.load()
        except Exception as e:  # pragma: no cover - depends on build
            _state["error"] = e
    return _state["lib"]


def native_enabled(op=None):
    if os.environ.get("DL4J_AMD_NATIVE", "1") == "0":
        return False
    if op is not None and os.environ.get(f"DL4J_AMD_KERNEL_{op.upper()}", "1") == "0":
        return False
    return True


def use_native(t, op=None):
    """True if tensor ``t`` should go through the HIP kernel for ``op``."""
    if not (torch.is_tensor(t) and t.is_cuda):
        return False
    if not native_enabled(op):
        return False
    lib = native_lib()
    if lib is None:
        if os.environ.get("DL4J_AMD_ALLOW_FALLBACK", "0") == "1":
            return False
        raise RuntimeError(
            "deeplearning4j_amd: HIP kernel library not loaded on a GPU run "
            f"({_state['error']!r}). Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or set DL4J_AMD_ALLOW_FALLBACK=1 to run the torch reference path.")
    return True


def stream_ptr():
    from .native import _stream
    return _stream()
