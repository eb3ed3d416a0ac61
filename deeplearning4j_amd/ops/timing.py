"""GPU-side timing of short kernel sequences for the per-shape kernel choosers.

Event pairs around a few eager launches measure the HOST enqueue rate when the kernels are shorter than the Python +
ctypes launch path (~30-100 us per call here), which made the choosers pick by launch overhead rather than kernel
time. ``gpu_time`` first parks the stream on a spin kernel (``torch.cuda._sleep``) long enough to cover the host-side
enqueue of all repetitions, so the bracketing events see the kernels back to back, as they run inside the HIP graph
of a training step."""
import time

import torch

_CYCLES_PER_MS = None


def _cycles_per_ms():
    global _CYCLES_PER_MS
    if _CYCLES_PER_MS is None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1000)
        e0.record()
        torch.cuda._sleep(2_000_000)
        e1.record()
        e1.synchronize()
        _CYCLES_PER_MS = 2_000_000 / max(e0.elapsed_time(e1), 1e-3)
    return _CYCLES_PER_MS


def gpu_time(fn, reps=3, warmup=1):
    """Mean GPU milliseconds of ``fn()`` (which enqueues work on the current stream)."""
    for _ in range(warmup):
        fn()
    t0 = time.perf_counter()
    fn()
    host_ms = (time.perf_counter() - t0) * 1e3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(_cycles_per_ms() * (host_ms * reps * 1.5 + 0.2)))
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps
