#!/usr/bin/env python3
"""Per-shape BatchNorm kernel timing on the ResNet-50 (DL4J zoo, batch 512) BN shapes: forward (tile-stats path
skipped: stats pass + apply) and backward (partial + fold + apply), GPU-side time (ops/timing.gpu_time), effective
HBM GB/s of the bytes each pass must move.
Usage: python tools/bn_bench.py [--batch 512]"""
import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from deeplearning4j_amd.ops import native  # noqa: E402
from deeplearning4j_amd.ops.timing import gpu_time  # noqa: E402

SHAPES = [(64, 28, "nonres"), (256, 28, "res"), (128, 14, "nonres"), (512, 14, "res"), (256, 7, "nonres"),
          (1024, 7, "res"), (512, 4, "nonres"), (2048, 4, "res")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    dev = torch.device("cuda")
    print(f"{'C':>5} {'HW':>3} {'kind':>6} | {'fwd us':>7} {'GB/s':>6} | {'bwd us':>7} {'GB/s':>6} | {'partial':>7} {'apply':>7}")
    for C, hw, kind in SHAPES:
        x = torch.randn(a.batch, C, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x) if kind == "res" else None
        dy = torch.randn_like(x)
        g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y, ctx = native.bn_fwd(x, g, b, rm, rv, True, 0.9, 1e-5, True, residual=r)
        tf = gpu_time(lambda: native.bn_fwd(x, g, b, rm, rv, True, 0.9, 1e-5, True, residual=r), reps=5) * 1e3
        tb = gpu_time(lambda: native.bn_bwd(dy, ctx), reps=5) * 1e3
        n = x.numel()
        fb = n * 2 * (3 if r is None else 4) + (n // 8 if r is not None else 0)    # stats read x, apply x(+r) -> y
        bb = n * 2 * (5 if r is None else 6)                                          # partial x,dy; apply x,dy -> dx(+dres)
        print(f"{C:5d} {hw:3d} {kind:>6} | {tf:7.1f} {fb / tf / 1e3:6.0f} | {tb:7.1f} {bb / tb / 1e3:6.0f} |")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
