#!/usr/bin/env python3
"""Probe what bounds a small conv: scaling with batch, vs hipBLASLt GEMM of the same size, vs a copy."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.conv_bench import timeit  # noqa: E402


def main():
    from deeplearning4j_amd.ops import conv_native as CN
    dev = torch.device("cuda")
    reps = int(os.environ.get("REPS", 200))
    for (C, H, K) in [(256, 7, 1024), (64, 28, 256), (128, 14, 128)]:
        for N in (256, 1024):
            R = 3 if (C, H, K) == (128, 14, 128) else 1
            pad = (1, 1, 1, 1) if R == 3 else (0, 0, 0, 0)
            x = torch.randn(N, C, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
            w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(torch.bfloat16)
            fl = 2.0 * N * H * H * K * C * R * R
            for v in (0, 1):
                CN.set_kernel_variant(v)
                CN.bump_version()
                ms = timeit(lambda: CN.conv2d_fwd(x, w, None, (1, 1), pad, (1, 1)), reps)
                print(f"conv C={C} H={H} K={K} R={R} N={N} v{v}: {ms*1e3:8.1f} us  {fl/ms/1e9:6.0f} TF/s")
            a = torch.randn(N * H * H, C * R * R, device=dev, dtype=torch.bfloat16)
            b = torch.randn(C * R * R, K, device=dev, dtype=torch.bfloat16)
            ms = timeit(lambda: a @ b, reps)
            print(f"  hipBLASLt GEMM {N*H*H}x{C*R*R}x{K}: {ms*1e3:8.1f} us  {fl/ms/1e9:6.0f} TF/s")
            y = torch.empty(N * H * H * K, device=dev, dtype=torch.bfloat16)
            ms = timeit(lambda: y.fill_(1.0), reps)
            print(f"  fill of output ({y.numel()*2/1e6:.1f} MB): {ms*1e3:8.1f} us  {y.numel()*2/ms/1e6:6.0f} GB/s")
    e = torch.empty(1, device=dev)
    ms = timeit(lambda: e.add_(1), reps)
    print(f"empty-ish kernel back-to-back: {ms*1e3:.1f} us")


if __name__ == "__main__":
    main()
