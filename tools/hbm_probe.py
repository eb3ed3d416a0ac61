"""HBM bandwidth probe with torch's elementwise kernels: write-only (fill), read-only (sum), read+write (copy) over
a buffer of the given size. Used to bound the write-heavy 1x1-convolution GEMMs (tools/gemm_conv1x1_bench.py).
Usage: python tools/hbm_probe.py [--mb 411]"""
import argparse

import torch


def t_of(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=411.0)
    a = ap.parse_args()
    n = int(a.mb * 1e6) // 2
    x = torch.empty(n, dtype=torch.bfloat16, device="cuda").uniform_()
    y = torch.empty_like(x)
    b = n * 2
    for name, fn, nb in (("fill (write)", lambda: y.fill_(1.0), b), ("sum (read)", lambda: x.sum(), b),
                         ("copy (read+write)", lambda: y.copy_(x), 2 * b), ("add x+x->y", lambda: torch.add(x, x, out=y), 2 * b)):
        t = t_of(fn)
        print(f"{name:20s} {b / 1e6:8.0f} MB  {t * 1e6:8.1f} us  {nb / t / 1e12:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
