"""Weight-gradient GEMM layouts: dW = X^T dY with X [T, in], dY [T, out] (both operands reduction-major, i.e. M- and
N-contiguous) on the in-tree kernels, against the same product with K-contiguous copies of the operands (the copy
time reported separately). Tells whether a transpose-then-GEMM candidate can pay for its copies.
Usage: python tools/gemm_layout_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeplearning4j_amd.ops import gemm  # noqa: E402

SHAPES = [("ffn1 dW", 4096, 768, 3072), ("ffn2 dW", 4096, 3072, 768), ("qkv dW", 4096, 768, 2304),
          ("o dW", 4096, 768, 768)]


def t_of(fn, reps=20):
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
    return s.elapsed_time(e) / reps * 1e3


def main():
    print(f"{'site':10s} {'T':>5s} {'in':>5s} {'out':>5s}  {'MN-major us':>11s}  {'K-major us':>10s}  {'copies us':>9s}")
    for name, T, nin, nout in SHAPES:
        x = torch.randn(T, nin, device="cuda").bfloat16()
        dy = torch.randn(T, nout, device="cuda").bfloat16()
        out = torch.empty(nin, nout, device="cuda")
        xt = x.t().contiguous()          # [in, T]: A K-contiguous
        dyt = dy.t().contiguous()        # [out, T]: B K-contiguous
        gemm.mmul(x.t(), dy, out=out)
        gemm.mmul(xt, dyt.t(), out=out)
        a = t_of(lambda: gemm.mmul(x.t(), dy, out=out))
        b = t_of(lambda: gemm.mmul(xt, dyt.t(), out=out))
        xt2, dyt2 = torch.empty_like(xt), torch.empty_like(dyt)
        c = t_of(lambda: (xt2.copy_(x.t()), dyt2.copy_(dy.t())))
        print(f"{name:10s} {T:5d} {nin:5d} {nout:5d}  {a:11.1f}  {b:10.1f}  {c:9.1f}", flush=True)


if __name__ == "__main__":
    main()
