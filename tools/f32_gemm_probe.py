"""Exact-fp32 GEMM (csrc/gemm.hip gemm_f32t) on the LeNet training shapes: time per (tile, splits) choice and the
planner's pick, against torch.matmul (the fp32 library GEMM) on the same operands. Diagnostic for the fp32 path.
Usage: python tools/f32_gemm_probe.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deeplearning4j_amd.ops import gemm as G            # noqa: E402  (registers the signatures)
from deeplearning4j_amd.ops import native                # noqa: E402
from deeplearning4j_amd.ops.timing import gpu_time      # noqa: E402

# (name, M, N, K, A layout, B layout): "r" row-major (k contiguous for A / n contiguous for B), "t" transposed view
SHAPES = [("conv1 fwd", 50176, 20, 25, "r", "t"), ("conv2 fwd", 12544, 50, 500, "r", "t"),
          ("conv2 dgrad", 12544, 500, 50, "r", "r"), ("conv2 wgrad", 50, 500, 12544, "t", "r"),
          ("conv1 wgrad", 20, 25, 50176, "t", "r"), ("dense fwd", 64, 500, 2450, "r", "r"),
          ("dense dgrad", 64, 2450, 500, "r", "t"), ("dense wgrad", 2450, 500, 64, "t", "r")]


def operand(rows, cols, layout):
    if layout == "r":
        return torch.randn(rows, cols, device="cuda")
    return torch.randn(cols, rows, device="cuda").t()


def main():
    lib = G._lib()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, M, N, K, la, lb in SHAPES:
        A, B = operand(M, K, la), operand(K, N, lb)
        C = torch.empty(M, N, device="cuda")
        tile, nsp = ctypes.c_int(0), ctypes.c_int(1)
        lib.dl4j_gemm_f32_plan(M, N, K, 1, ctypes.byref(tile), ctypes.byref(nsp))
        ref = A @ B
        res = []
        for t in (64, 128):
            for sp in (1, 2, 4, 8, 16, 32, 64, 128, 256):
                if sp > 1 and K // sp < 16:
                    continue
                ws = torch.empty(sp * M * N, device="cuda")

                def run():
                    return lib.dl4j_gemm_f32(0, 0, M, N, K, 1, ctypes.c_void_p(A.data_ptr()), A.stride(0),
                                             A.stride(1), 0, ctypes.c_void_p(B.data_ptr()), B.stride(0), B.stride(1),
                                             0, ctypes.c_void_p(C.data_ptr()), N, 0, 1.0, 0.0, None, 0, 0, None, t, sp,
                                             ctypes.c_void_p(ws.data_ptr()), s)
                if run() != 0:
                    continue
                torch.cuda.synchronize()
                err = (C - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
                res.append((gpu_time(run, reps=10, warmup=2) * 1e3, t, sp, err))   # ms -> us
        lt = gpu_time(lambda: torch.matmul(A, B, out=C), reps=10, warmup=2) * 1e3
        res.sort()
        best = res[0]
        plan = [r for r in res if r[1] == tile.value and r[2] == nsp.value]
        print(f"{name:12s} M={M:6d} N={N:5d} K={K:6d}  lib {lt:7.1f} us | best {best[0]:7.1f} us (tile {best[1]}, "
              f"splits {best[2]}, rel err {best[3]:.1e}) | planned tile {tile.value} splits {nsp.value}: "
              f"{plan[0][0] if plan else float('nan'):7.1f} us", flush=True)
        print("     " + " ".join(f"{t}/{sp}:{us:.0f}" for us, t, sp, _ in sorted(res, key=lambda r: (r[1], r[2]))),
              flush=True)


if __name__ == "__main__":
    main()
