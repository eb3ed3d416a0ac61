#!/usr/bin/env python3
"""Per-shape weight-gradient timing on the zoo ResNet-50 conv shapes (bias gradient included everywhere):
round-2 atomic kernel, best round-3 tile variant, plain GEMM (1x1 stride 1 only) and every halo-engine candidate
(csrc/conv_wrw.hip, variant x split count). Prints TFLOP/s of the best halo candidate and count-weighted totals.
Usage: python tools/wrw_halo_bench.py --batch 512"""
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
    ap.add_argument("--variant", default="dl4j")
    a = ap.parse_args()
    from deeplearning4j_amd.ops import conv_native, native
    from deeplearning4j_amd.ops.gemm import mmul
    lib = native.load()
    seen = {}
    for s in capture_shapes(a.variant):
        seen[s] = seen.get(s, 0) + 1
    nv = lib.dl4j_conv_wrw_v3_num_variants()
    print(f"{'C,H,W':>14} {'K,R,S st':>12} cnt | {'r2':>7} {'v3best':>7} {'gemm':>7} | {'halo':>7} {'cand':>14} "
          f"{'TF/s':>6} | x", flush=True)
    tot_old, tot_new = 0.0, 0.0
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
        tv = min(timeit(lambda v=v: conv_native._wrw_v3_launch(v, x, dy, gW, geom, gb), a.reps) for v in range(nv))
        tg = float("inf")
        if R == 1 and S == 1 and st == (1, 1) and not any(pad):
            M = N * H * W
            dyr = dy.permute(0, 2, 3, 1).reshape(M, K)
            xr = x.permute(0, 2, 3, 1).reshape(M, C)

            def gemm():
                mmul(dyr.t(), xr, out=gW.reshape(K, C))
                native.channel_sum(dyr, out=gb)
            tg = timeit(gemm, a.reps)
        best_h, best_c = float("inf"), None
        for c in conv_native._halo_candidates(geom):
            if conv_native._wrw_launch(c, x, dy, gW, geom, gb) != 0:
                continue
            t = timeit(lambda c=c: conv_native._wrw_launch(c, x, dy, gW, geom, gb), a.reps)
            if t < best_h:
                best_h, best_c = t, c
        old = min(t2, tv, tg)
        tot_old += cnt * old
        tot_new += cnt * min(old, best_h)
        flops = 2.0 * N * OH * OW * K * C * R * S
        tf = flops / (best_h * 1e-3) / 1e12 if best_c else 0.0
        cs = f"{best_c[1]}/{best_c[2]}" if best_c else "-"
        print(f"{C:4d},{H:4d},{W:4d} {K:5d},{R},{S} {st[0]} {cnt:3d} | {t2:7.3f} {tv:7.3f} {tg:7.3f} | {best_h:7.3f} "
              f"{cs:>14} {tf:6.1f} | {old / best_h if best_c else 0:4.2f}", flush=True)
    print(f"count-weighted: previous best {tot_old:.3f} ms, with halo {tot_new:.3f} ms")


if __name__ == "__main__":
    main()
