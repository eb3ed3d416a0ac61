#!/usr/bin/env python3
"""Run one halo weight-gradient candidate on one shape a few times (for rocprofv3 --pmc passes).
Usage: python tools/wrw_halo_probe.py --shape 512,64,28,28,64,3 --variant 1 --splits 512 --reps 5"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="512,64,28,28,64,3", help="N,C,H,W,K,R (stride 1, same padding)")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from deeplearning4j_amd.ops import conv_native
    from deeplearning4j_amd.ops.timing import gpu_time
    N, C, H, W, K, R = (int(v) for v in a.shape.split(","))
    p = R // 2
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, K, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dW = torch.empty(K, C, R, R, device="cuda")
    db = torch.empty(K, device="cuda")
    geom = (N, H, W, C, K, R, R, 1, 1, p, p, 1, 1, H, W)
    c = ("halo", a.variant, a.splits)
    assert conv_native._wrw_launch(c, x, dy, dW, geom, db) == 0
    t = gpu_time(lambda: conv_native._wrw_launch(c, x, dy, dW, geom, db), reps=a.reps)
    fl = 2.0 * N * H * W * K * C * R * R
    print(f"{a.shape} variant {a.variant} splits {a.splits}: {t * 1e3:.1f} us incl. reduce, {fl / t / 1e9:.1f} TF/s",
          flush=True)


if __name__ == "__main__":
    main()
