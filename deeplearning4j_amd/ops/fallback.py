"""Helper-fallback accounting (reference ConvolutionLayer.java:58,173-200 ``helperCountFail`` /
``cudnnAllowFallback``): every time a GPU op cannot run on its in-tree HIP kernel and takes a library / torch path
instead, the event is counted here per (op, reason). Networks expose the total as ``helperCountFail()``; GPU tests
assert it stays 0 on the flagship configurations.

``DL4J_AMD_STRICT_KERNELS=1`` turns a fallback into an error (useful when adding a new layer shape).
"""
import collections
import os

_COUNTS = collections.Counter()


class KernelFallbackError(RuntimeError):
    pass


def record(op, reason):
    _COUNTS[(op, reason)] += 1
    if os.environ.get("DL4J_AMD_STRICT_KERNELS", "0") == "1":
        raise KernelFallbackError(f"{op}: no in-tree HIP kernel for this call ({reason})")


def note(t, op, reason):
    """Record a fallback when ``t`` lives on the GPU (CPU tensors always take the torch reference path)."""
    import torch
    if torch.is_tensor(t) and t.is_cuda:
        record(op, reason)


def count(op=None):
    if op is None:
        return sum(_COUNTS.values())
    return sum(v for (o, _), v in _COUNTS.items() if o == op)


def summary():
    return dict(_COUNTS)


def reset():
    _COUNTS.clear()
