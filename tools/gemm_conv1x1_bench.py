"""1x1-convolution GEMMs of ResNet-50 (NHWC rows x channels) with the fused BatchNorm tile statistics, per tile
configuration: time (HIP-graph replay of 10 calls), achieved HBM bytes/s (A read + C write + statistics planes) and
MFMA TF/s. Shows which configuration the output-heavy (expanding, K = 64..256) products want.
Usage: python tools/gemm_conv1x1_bench.py [--cfgs 2,3,5,8,9] [--only M,N,K]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeplearning4j_amd.ops import gemm  # noqa: E402

# (name, M rows, N out channels, K in channels): zoo ResNet-50 at batch 1024 (stage 2 at 28x28) + canonical bs512
SHAPES = [
    ("zoo s2 expand 64->256", 802816, 256, 64),
    ("zoo s2 reduce 256->64", 802816, 64, 256),
    ("zoo s3 expand 128->512", 200704, 512, 128),
    ("zoo s3 reduce 512->128", 200704, 128, 512),
    ("zoo s4 expand 256->1024", 50176, 1024, 256),
    ("zoo s4 reduce 1024->256", 50176, 256, 1024),
    ("canon s2 expand 64->256", 1605632, 256, 64),
]


def timeit(fn, reps=10):
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
    return s.elapsed_time(e) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="2,3,5,6,8,9")
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    cfgs = [int(c) for c in args.cfgs.split(",")]
    dt = torch.bfloat16
    print(f"{'shape':26s} {'M':>8s} {'N':>5s} {'K':>5s}  " + "  ".join(f"cfg{c:<2d} us  TB/s" for c in cfgs))
    for name, M, N, K in SHAPES:
        if args.only and args.only != f"{M},{N},{K}":
            continue
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(dt)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(dt)     # [out, in] weights: B = w.t() is K-contiguous
        out = torch.empty(M, N, device="cuda", dtype=dt)
        P = (M + 63) // 64
        st = torch.empty(3, P, N, device="cuda", dtype=torch.float32)
        nbytes = (M * K + M * N) * 2 + 3 * P * N * 4
        row = []
        for c in cfgs:
            gemm._FORCE_CFG = (c, 1)
            try:
                t = timeit(lambda: gemm.mmul(a, w.t(), out=out, stats=st))
                row.append(f"{t * 1e6:8.1f} {nbytes / t / 1e12:5.2f}")
            except Exception as ex:   # noqa: BLE001 — an unsupported configuration for this layout
                row.append(f"{'n/a':>8s} {'':5s}")
                print(f"  cfg {c}: {type(ex).__name__}: {ex}", file=sys.stderr)
            finally:
                gemm._FORCE_CFG = None
        print(f"{name:26s} {M:8d} {N:5d} {K:5d}  " + "  ".join(row), flush=True)
        del a, w, out, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
