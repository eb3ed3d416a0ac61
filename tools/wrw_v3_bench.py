#!/usr/bin/env python3
"""Per-shape weight-gradient timing on the zoo ResNet-50 conv shapes: round-2 atomic kernel (bias fused) vs every
round-3 tile variant (slab reduce, bias fused; channel_sum alone for reference). Usage: python tools/wrw_v3_bench.py --batch 512"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.conv_bench import capture_shapes, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from deeplearning4j_amd.ops import conv_native, native
    lib = native.load()
    seen = {}
    for s in capture_shapes("dl4j"):
        seen[s] = seen.get(s, 0) + 1
    nv = lib.dl4j_conv_wrw_v3_num_variants()
    print(f"{'C,H,W':>14} {'K,R,S st':>12} cnt | {'r2+b':>7} | " + " ".join(f"{'v' + str(v):>7}" for v in range(nv)) +
          f" | {'csum':>6}  (ms)")
    tot_r2, tot_best = 0.0, 0.0
    for (xs, ws, st, pad, dil), cnt in seen.items():
        C, H, W = xs
        K, _, R, S = ws
        if C % 8 or K % 8:
            continue
        N = a.batch
        x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        OH = (H + pad[0] + pad[1] - R) // st[0] + 1
        OW = (W + pad[2] + pad[3] - S) // st[1] + 1
        dy = torch.randn(N, K, OH, OW, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        gW = torch.zeros(K, C, R, S, device="cuda")
        gb = torch.zeros(K, device="cuda")
        geom = (N, H, W, C, K, R, S, st[0], st[1], pad[0], pad[2], dil[0], dil[1], OH, OW)
        t2 = timeit(lambda: conv_native._conv2d_wrw_r2(x, dy, N, H, W, C, K, R, S, OH, OW, st, pad, dil, True, gW, gb,
                                                       False, gW, True), a.reps)
        tv = [timeit(lambda v=v: conv_native._wrw_v3_launch(v, x, dy, gW, geom, gb), a.reps) for v in range(nv)]
        tc = timeit(lambda: native.channel_sum(dy.permute(0, 2, 3, 1).reshape(-1, K), out=gb), a.reps)
        tot_r2 += cnt * t2
        tot_best += cnt * min(t2, min(tv))
        print(f"{C:4d},{H:4d},{W:4d} {K:5d},{R},{S} {st[0]} {cnt:3d} | {t2:7.3f} | " +
              " ".join(f"{t:7.3f}" for t in tv) + f" | {tc:6.3f}")
    print(f"count-weighted: r2 {tot_r2:.3f} ms, best-of {tot_best:.3f} ms")


if __name__ == "__main__":
    main()
