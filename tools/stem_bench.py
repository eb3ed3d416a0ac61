#!/usr/bin/env python3
"""GPU time of the ResNet-50 stem kernels at the bench shape (batch 512, 224x224x3 -> 112x112x64 -> BN+ReLU+max pool
3x3/2 -> 55x55x64): stem conv forward, stem weight gradient (+ its fixed-order reduce), fused BN+ReLU+pool forward
and backward. Median of --reps timed calls (HIP events). Usage on a GPU box: python tools/stem_bench.py [--batch 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from deeplearning4j_amd.ops import conv_stem, native
    dev = torch.device("cuda", 0)
    N = args.batch
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, 3, 224, 224, device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    y = conv_stem.forward(x, w, want_stats=True)
    dy = torch.randn(y.shape, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gW = torch.zeros(64, 3, 7, 7, device=dev)
    gb = torch.zeros(64, device=dev)
    res = {
        "stem_fwd": timed(lambda: conv_stem.forward(x, w, want_stats=True), args.reps),
        "stem_wrw": timed(lambda: conv_stem.backward_weight(x, dy, gW, gb, True), args.reps),
    }
    gamma, beta = torch.ones(64, device=dev), torch.zeros(64, device=dev)
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    r = native.bn_pool_fwd(y, gamma, beta, rm, rv, True, 0.9, 1e-5, (3, 3), (2, 2), (0, 0, 0, 0))
    if r is not None:
        p, ctx = r
        dp = torch.randn(p.shape, device=dev, generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        res["bnpool_fwd"] = timed(lambda: native.bn_pool_fwd(y, gamma, beta, rm, rv, True, 0.9, 1e-5, (3, 3), (2, 2),
                                                              (0, 0, 0, 0)), args.reps)
        dg, db = torch.empty(64, device=dev), torch.empty(64, device=dev)
        res["bnpool_bwd"] = timed(lambda: native.bn_pool_bwd(dp, ctx, dg, db), args.reps)
    for k, v in res.items():
        print(f"{k:12s} {v * 1000:8.1f} us")


if __name__ == "__main__":
    main()
