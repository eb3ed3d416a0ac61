#!/usr/bin/env python3
"""Skinny 1x1-conv GEMMs of the zoo ResNet-50 (M = N*H*W rows, small K or N): time every in-tree tile config (with
and without the BN-statistics epilogue) next to torch.matmul, and report GB/s of the compulsory traffic.
Usage: python tools/skinny_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeplearning4j_amd.ops import gemm as G  # noqa: E402
from deeplearning4j_amd.ops.timing import gpu_time  # noqa: E402
from deeplearning4j_amd.ops.native import _stream  # noqa: E402

SHAPES = [(401408, 64, 256), (401408, 256, 64), (401408, 64, 64), (100352, 128, 512), (100352, 512, 128),
          (25088, 256, 1024), (25088, 1024, 256), (6272, 512, 2048), (6272, 2048, 512)]


def main():
    dev = torch.device("cuda")
    lib = G._lib()
    for M, N, K in SHAPES:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()      # [N, K] k-contiguous = W of a 1x1 conv
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        P = (M + 63) // 64
        ts = torch.empty(3, P, N, device=dev)
        byt = (M * K + M * N + N * K) * 2
        t_ref = gpu_time(lambda: torch.matmul(a, b.t(), out=c), reps=10, warmup=3)
        line = [f"M={M:7d} N={N:5d} K={K:5d}  torch {t_ref*1e3:7.1f}us {byt/t_ref/1e6:6.0f}GB/s"]
        for cfg in range(6):
            for st in (False, True):
                def run(cfg=cfg, st=st):
                    return lib.dl4j_gemm(1, 1, M, N, K, 1, G._p(a), K, 1, 0, G._p(b), K, 1, 0, G._p(c), N, 0, 1.0,
                                         0.0, None, 0, 0, None, cfg, 1, None, G._p(ts) if st else None,
                                         P if st else 0, _stream())
                if run() != 0:
                    continue
                torch.cuda.synchronize()
                ref = a.float() @ b.float().t()
                err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
                if err > 2e-2:
                    line.append(f"c{cfg} BAD err={err:.3g}")
                    continue
                t = gpu_time(run, reps=10, warmup=3)
                line.append(f"c{cfg}{'s' if st else ' '} {t*1e3:6.1f}us {byt/t/1e6:5.0f}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
