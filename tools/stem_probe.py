#!/usr/bin/env python3
"""Time the ResNet-50 stem convolution (3->64, 7x7, stride 2, pad 3, batch 256, bf16 NHWC) three ways:
MIOpen via torch, and the native MFMA implicit-GEMM kernels on the input zero-padded to 8 channels (the padding
copy included). Forward and weight-gradient only (the stem's input needs no gradient)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    from deeplearning4j_amd.ops import conv_native as cn
    dev = torch.device("cuda")
    N = int(os.environ.get("N", 256))
    x = torch.randn(N, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16)
    y = F.conv2d(x, w, None, 2, 3)
    dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
    flops = 2 * N * 112 * 112 * 64 * 3 * 49
    ms = t(lambda: F.conv2d(x, w, None, 2, 3))
    print(f"miopen fwd  {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s")
    ms = t(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (2, 2), (3, 3), (1, 1), False, (0, 0), 1,
                                                       (False, True, False)))
    print(f"miopen wrw  {ms:.3f} ms")

    def pad8():
        return F.pad(x, (0, 0, 0, 0, 0, 5)).contiguous(memory_format=torch.channels_last)
    print(f"pad to C=8  {t(pad8):.3f} ms")
    x8 = pad8()
    w8 = F.pad(w, (0, 0, 0, 0, 0, 5)).contiguous()
    cn.bump_version()
    out = cn.conv2d_fwd(x8, w8, None, (2, 2), (3, 3, 3, 3), (1, 1))
    err = (out.float() - y.float()).abs().max().item()
    print(f"native fwd max err vs miopen {err:.4f}")
    ms = t(lambda: cn.conv2d_fwd(x8, w8, None, (2, 2), (3, 3, 3, 3), (1, 1)))
    print(f"native fwd  {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s")
    gW = torch.zeros(64, 8, 7, 7, device=dev)

    def wrw():
        gW.zero_()
        cn.conv2d_bwd(x8, w8, dy, (2, 2), (3, 3, 3, 3), (1, 1), False, True, False, gW, None, True)
    ms = t(wrw)
    print(f"native wrw  {ms:.3f} ms")
    ref = torch.ops.aten.convolution_backward(dy, x, w, None, (2, 2), (3, 3), (1, 1), False, (0, 0), 1,
                                              (False, True, False))[1]
    wrw()
    print(f"native wrw max rel err {((gW[:, :3] - ref.float()).abs().max() / ref.float().abs().max()).item():.4f}")


if __name__ == "__main__":
    main()
