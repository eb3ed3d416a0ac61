"""Throughput of the in-tree MFMA GEMM (ops.gemm.mmul) vs torch.matmul (hipBLASLt) on the framework's shapes.

Random uniform [-1, 1) operands (zero-filled data reads high, guide §5.4 rule 25), interleaved rounds in one
process (rule 24), median of the rounds. Prints one line per shape: TF/s of the in-tree kernels, of torch, their
ratio, and of ``mmul``'s dispatch (the autotuner's pick between the in-tree configurations and the library GEMM,
ops/gemm.py _lib_gemm) with its choice.
A second table times the BERT layer's epilogue call sites (bias from a 16-bit shadow, bias + GELU with the
pre-activation kept, the GELU-backward product, beta-accumulate) through ``mmul``: in-tree fused epilogue vs
dispatch (which may pick the library product + one in-tree elementwise kernel).
Usage: python tools/gemm_bench.py [--dtype bf16|fp16] [--rounds R] [--only NAME] [--epilogues-only]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeplearning4j_amd.ops import gemm  # noqa: E402

SHAPES = [
    # (name, M, N, K, a_layout, b_layout)  layout 'k' = reduction dim contiguous, 'm'/'n' = the other
    ("bert qkv fwd", 4096, 2304, 768, "k", "n"),
    ("bert ffn1 fwd", 4096, 3072, 768, "k", "n"),
    ("bert ffn2 fwd", 4096, 768, 3072, "k", "n"),
    ("bert o fwd", 4096, 768, 768, "k", "n"),
    ("bert ffn2 dX", 4096, 3072, 768, "k", "k"),
    ("bert ffn1 dW", 768, 3072, 4096, "m", "n"),
    ("bert qkv dW", 768, 2304, 4096, "m", "n"),
    ("bert 16k tok qkv", 16384, 2304, 768, "k", "n"),
    ("bert 16k tok ffn2", 16384, 768, 3072, "k", "n"),
    ("lstm in-proj", 8192, 1024, 256, "k", "n"),
    ("lstm dW", 256, 1024, 8192, "m", "n"),
    ("resnet fc fwd", 512, 1000, 2048, "k", "k"),
    ("resnet fc dW", 2048, 1000, 512, "m", "n"),
    ("square 4096", 4096, 4096, 4096, "k", "k"),
    ("square 8192", 8192, 8192, 8192, "k", "k"),
]


def operand(R, C, contig_last, dt):
    t = torch.rand(R, C, device="cuda") * 2 - 1 if contig_last else (torch.rand(C, R, device="cuda") * 2 - 1).t()
    return t.to(dt)


def timeit(fn, reps=20):
    """GPU time per call: ``reps`` calls captured in one HIP graph (no host launch cost in the number)."""
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
    return s.elapsed_time(e) / reps * (1000.0 if "probe" in __file__ else 1.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--epilogues-only", action="store_true")
    args = ap.parse_args()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    if not args.epilogues_only:
        plain_table(args, dt)
    epilogue_table(args, dt)


EPILOGUES = [
    # (name, M, N, K, kind)
    ("qkv fwd +bias", 4096, 2304, 768, "bias"),
    ("o fwd +bias", 4096, 768, 768, "bias"),
    ("ffn1 fwd +bias+gelu(z)", 4096, 3072, 768, "gelu"),
    ("ffn2 fwd +bias", 4096, 768, 3072, "bias"),
    ("ffn2 dX *gelu'(z)", 4096, 3072, 768, "dgelu"),
    ("ffn1 dX +=", 4096, 768, 3072, "beta"),
]


def epilogue_table(args, dt):
    print(f"{'BERT epilogue site':26s} {'M':>6s} {'N':>6s} {'K':>6s}   fused TF/s  dispatch TF/s  speedup  pick")
    for name, M, N, K, kind in EPILOGUES:
        if args.only and args.only not in name:
            continue
        a = operand(M, K, True, dt)
        b = operand(K, N, kind not in ("dgelu", "beta"), dt)       # backward: W^T views (K contiguous)
        out = torch.empty(M, N, device="cuda", dtype=dt)
        z = torch.empty(M, N, device="cuda", dtype=dt) if kind in ("gelu", "dgelu") else None
        if z is not None:
            z.copy_(torch.randn(M, N, device="cuda"))
        bias = None
        if kind in ("bias", "gelu"):
            bias = torch.randn(N, device="cuda")
            bias._dl4j_shadow = bias.to(dt)
        kw = dict(out=out, bias=bias, z=z, act={"gelu": "gelu", "dgelu": "dgelu"}.get(kind),
                  beta=1.0 if kind == "beta" else 0.0)
        flop = 2.0 * M * N * K
        reps = max(3, min(50, int(2e12 / flop)))

        def fused():
            gemm._LIB = False
            try:
                gemm.mmul(a, b, **kw)
            finally:
                gemm._LIB = True
        tf, td = [], []
        for _ in range(args.rounds):
            tf.append(timeit(fused, reps))
            td.append(timeit(lambda: gemm.mmul(a, b, **kw), reps))
        t1, t2 = sorted(tf)[len(tf) // 2], sorted(td)[len(td) // 2]
        picks = [v for k, v in gemm._TUNED.items() if k[:3] == (M, N, K) and "lib" in k]
        pick = "lib" if picks and picks[-1] == gemm.LIB_CFG else (f"cfg{picks[-1][0]}x{picks[-1][1]}" if picks else "-")
        print(f"{name:26s} {M:6d} {N:6d} {K:6d}   {flop / t1 / 1e9:10.1f}  {flop / t2 / 1e9:13.1f}  {t1 / t2:7.2f}"
              f"  {pick}", flush=True)


def plain_table(args, dt):
    print(f"{'shape':22s} {'M':>6s} {'N':>6s} {'K':>6s}   ours TF/s  torch TF/s  ratio  dispatch TF/s  pick")
    for name, M, N, K, la, lb in SHAPES:
        if args.only and args.only not in name:
            continue
        a = operand(M, K, la == "k", dt)
        b = operand(K, N, lb == "n", dt)
        out = torch.empty(M, N, device="cuda", dtype=dt)
        flop = 2.0 * M * N * K
        reps = max(3, min(50, int(2e12 / flop)))
        ours, ref, disp = [], [], []

        def intree():
            gemm._LIB = False
            try:
                gemm.mmul(a, b, out=out)
            finally:
                gemm._LIB = True
        for _ in range(args.rounds):
            ours.append(timeit(intree, reps))
            ref.append(timeit(lambda: torch.matmul(a, b, out=out), reps))
            disp.append(timeit(lambda: gemm.mmul(a, b, out=out), reps))
        to = sorted(ours)[len(ours) // 2]
        tr = sorted(ref)[len(ref) // 2]
        td = sorted(disp)[len(disp) // 2]
        picks = [v for k, v in gemm._TUNED.items() if k[:3] == (M, N, K) and "lib" in k]
        pick = "lib" if picks and picks[-1] == gemm.LIB_CFG else (f"cfg{picks[-1][0]}x{picks[-1][1]}" if picks else "-")
        print(f"{name:22s} {M:6d} {N:6d} {K:6d}   {flop / to / 1e9:9.1f}  {flop / tr / 1e9:10.1f}  {tr / to:5.2f}"
              f"  {flop / td / 1e9:13.1f}  {pick}", flush=True)


if __name__ == "__main__":
    main()
