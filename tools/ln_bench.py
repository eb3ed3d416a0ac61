#!/usr/bin/env python3
"""LayerNorm backward timing (BERT-base shape M=4096, N=768, residual, dx column sums) over block caps and the two
partial-reduction kernels (fold vs reduce), GPU-side time.  Usage: python tools/ln_bench.py"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from deeplearning4j_amd.ops import transformer_native as TN  # noqa: E402
from deeplearning4j_amd.ops import native  # noqa: E402
from deeplearning4j_amd.ops.timing import gpu_time  # noqa: E402


def main():
    M, N = 4096, 768
    dev = "cuda"
    x = torch.randn(M, N, device=dev).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    g, b = torch.rand(N, device=dev) + 0.5, torch.randn(N, device=dev)
    y, mean, rstd = TN.ln_fwd(x, g, b, 1e-12, r)
    ds = torch.empty(N, device=dev)
    L = native.load()
    L.dl4j_ln_set_config.argtypes = [native.c_int, native.c_int]
    ref = None
    for cap in (512, 256, 128, 64):
        for fold in (1, 0):
            L.dl4j_ln_set_config(cap, fold)
            dx, dg, db = TN.ln_bwd(dy, x, g, mean, rstd, r, None, None, ds)
            if ref is None:
                ref = (dg.clone(), ds.clone())
            err = max((dg - ref[0]).abs().max().item(), (ds - ref[1]).abs().max().item())
            t = gpu_time(lambda: TN.ln_bwd(dy, x, g, mean, rstd, r, None, None, ds), reps=20) * 1e3
            print(f"cap {cap:4d} fold {fold}: {t:7.1f} us  (max diff vs first {err:.2e})")
    L.dl4j_ln_set_config(128, 0)


if __name__ == "__main__":
    main()
