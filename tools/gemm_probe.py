"""GEMM kernel probe: per-config time vs K at a fixed M x N (separates per-block fixed cost from per-K-tile cost).

python tools/gemm_probe.py [--M 4096 --N 3072] [--cfgs 4,0,2] [--ks 64,256,768,3072]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeplearning4j_amd.ops import gemm  # noqa: E402


def timeit(fn, reps=20):
    """GPU time per call: ``reps`` calls captured in one HIP graph (no host launch cost in the number)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * (1000.0 if "probe" in __file__ else 1.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--cfgs", default="4,0,1,2")
    ap.add_argument("--ks", default="64,256,768,3072")
    ap.add_argument("--outs", default="bf16,fp32")
    args = ap.parse_args()
    M, N = args.M, args.N
    for K in [int(k) for k in args.ks.split(",")]:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16().t()
        for od in args.outs.split(","):
            dt = torch.bfloat16 if od == "bf16" else torch.float32
            out = torch.empty(M, N, device="cuda", dtype=dt)
            row = [f"M={M} N={N} K={K:5d} out={od:4s}"]
            for c in [int(c) for c in args.cfgs.split(",")]:
                gemm._FORCE_CFG = (c, 1)
                us = timeit(lambda: gemm.mmul(a, b, out=out))
                row.append(f"cfg{c} {us:8.1f}us {2.0 * M * N * K / us / 1e6:7.1f}TF")
            gemm._FORCE_CFG = None
            us = timeit(lambda: out.copy_(torch.matmul(a, b)) if out.dtype != a.dtype else torch.matmul(a, b, out=out))
            row.append(f"torch {us:8.1f}us {2.0 * M * N * K / us / 1e6:7.1f}TF")
            print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
