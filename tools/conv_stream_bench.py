#!/usr/bin/env python3
"""Forward implicit-GEMM conv kernels per ResNet-50 shape (zoo graph, NHWC bf16, with the BN tile-statistics epilogue
the training step uses): the round-3 tile variants 0-4 of conv_glds against the persistent conv_stream kernel
(variant 100) and the halo-staged 3x3 kernel (variant 101, 64 -> 64 channels). Prints us per call for each and the best. Usage: python tools/conv_stream_bench.py [--batch 1024]"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--variant", default="dl4j")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from tools.conv_bench import capture_shapes
    from deeplearning4j_amd.ops import conv_native as CN
    from deeplearning4j_amd.ops.timing import gpu_time
    shapes = collections.Counter(capture_shapes(a.variant))
    variants = [0, 1, 2, 3, 4, CN.STREAM_VAR, CN.HALO_VAR]
    print(f"{'shape (C,H,W) -> (K,R,S) stride':40s} {'n':>2s} " + " ".join(f"{v:>7d}" for v in variants) + "  best")
    tot = collections.Counter()
    for (xs, ws, st, pad4, dil), cnt in shapes.items():
        C, H, W = xs
        K, _, R, S = ws
        if C % 64 or C == 3:
            continue
        N = a.batch
        OH = (H + pad4[0] + pad4[1] - R) // st[0] + 1
        OW = (W + pad4[2] + pad4[3] - S) // st[1] + 1
        M = N * OH * OW
        x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wk = (torch.randn(K, R, S, C, device="cuda") * 0.05).to(torch.bfloat16)
        b = torch.zeros(K, device="cuda")
        y = torch.empty(N, K, OH, OW, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ts = torch.empty(3, (M + 63) // 64, K, device="cuda")
        geom = (N, H, W, C, K, R, S, st[0], st[1], pad4[0], pad4[2], dil[0], dil[1], OH, OW)
        row = []
        for v in variants:
            tv = CN._stats_buf(v, M, K, x.device, geom)
            if tv is None or CN._fwd_launch(v, x, wk, b, y, geom, 0.0, tv) not in (0, 1):
                row.append(None)
                continue
            row.append(gpu_time(lambda: CN._fwd_launch(v, x, wk, b, y, geom, 0.0, tv), reps=a.reps, warmup=2) * 1e6)
        ok = [(t, v) for t, v in zip(row, variants) if t is not None]
        best = min(ok)[1] if ok else None
        for t, v in zip(row, variants):
            if t is not None:
                tot[v] += t * cnt
        tot["best_old"] += min(t for t, v in ok if v not in (CN.STREAM_VAR, CN.HALO_VAR)) * cnt if ok else 0
        tot["best_all"] += min(t for t, v in ok) * cnt if ok else 0
        name = f"({C},{H},{W})->({K},{R},{S}) s{st[0]}"
        print(f"{name:40s} {cnt:2d} " + " ".join(f"{t:7.1f}" if t is not None else f"{'-':>7s}" for t in row) +
              f"  {best}", flush=True)
        del x, y, ts
        torch.cuda.empty_cache()
    print("count-weighted ns: best of round-3 variants %.1f, best incl. conv_stream / conv_halo %.1f" %
          (tot["best_old"], tot["best_all"]))


if __name__ == "__main__":
    main()
