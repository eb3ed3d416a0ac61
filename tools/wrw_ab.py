#!/usr/bin/env python3
"""A/B of weight-gradient kernel block order (XCD-aware remap on/off) and kernel variant on the ResNet-50 conv
shapes. Usage on a GPU box: python tools/wrw_ab.py --batch 512"""
import argparse
import collections
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
    from deeplearning4j_amd.ops import conv_native as CN
    dev = torch.device("cuda")
    count = collections.Counter(capture_shapes("dl4j"))
    cfgs = [(0, 0), (0, 1), (1, 0), (1, 1)]   # (variant, remap)
    tot = collections.defaultdict(float)
    print(f"{'C,H,W':>14} {'K,R,S':>10} st cnt | " + " ".join(f"v{v}r{r}(us)" for v, r in cfgs))
    for (xs, ws, st, pad, dil), n in sorted(count.items(), key=lambda kv: -kv[1]):
        C, H, W = xs
        K, _, R, S = ws
        if C % 8 != 0:
            continue
        x = torch.randn(a.batch, C, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, S, device=dev) * 0.05).to(torch.bfloat16)
        y = CN.conv2d_fwd(x, w, None, st, pad, dil)
        dy = torch.randn_like(y)
        gW = torch.zeros(K, C, R, S, device=dev)
        res = []
        for v, r in cfgs:
            CN.set_wrw_variant(v)
            CN.set_wrw_remap(r)
            t = timeit(lambda: CN.conv2d_bwd(x, w, dy, st, pad, dil, False, True, False, gW), a.reps)
            res.append(t)
            tot[(v, r)] += n * t
        print(f"{C:>4},{H:>4},{W:>4} {K:>4},{R},{S} {st[0]} {n:>3} | " + " ".join(f"{t*1e3:10.0f}" for t in res),
              flush=True)
        del x, w, y, dy, gW
    CN.set_wrw_variant(0)
    CN.set_wrw_remap(1)
    print("totals ms (count-weighted):", {f"v{v}r{r}": round(t, 3) for (v, r), t in tot.items()})


if __name__ == "__main__":
    main()
