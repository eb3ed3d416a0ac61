#!/usr/bin/env python3
"""Timing probe of the halo-staged 3x3 conv (csrc/conv_halo.hip) at one shape: the full kernel and, through
DL4J_AMD_HALO_DBG, with the MFMA loop (1) and / or the read-out (2) skipped — where a chunk's time goes.
Usage: DL4J_AMD_HALO_DBG=n python tools/halo_probe.py [--batch 1024] [--hw 28]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--hw", type=int, default=28)
    a = ap.parse_args()
    from deeplearning4j_amd.ops import conv_native as CN
    from deeplearning4j_amd.ops.timing import gpu_time
    N, H = a.batch, a.hw
    x = torch.randn(N, 64, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wk = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).to(torch.bfloat16)
    y = torch.empty_like(x)
    geom = (N, H, H, 64, 64, 3, 3, 1, 1, 1, 1, 1, 1, H, H)
    ts = CN._stats_buf(CN.HALO_VAR, N * H * H, 64, x.device, geom)
    t = gpu_time(lambda: CN._fwd_launch(CN.HALO_VAR, x, wk, None, y, geom, 0.0, ts), reps=20, warmup=3) * 1e6
    print(f"dbg={os.environ.get('DL4J_AMD_HALO_DBG', '0')} N={N} HW={H}: {t / 1000:.1f} us")


if __name__ == "__main__":
    main()
