#!/usr/bin/env python3
"""ResNet-50 stem (3->64, 7x7, stride 2, pad 3, NHWC bf16) as a space-to-depth 4x4 stride-1 convolution on the MFMA
implicit-GEMM kernels vs MIOpen (torch). Checks numerics of the transformed conv and times fwd + weight gradient.

Transform: input [N,3,224,224] -> pixel-unshuffle(2) [N,12,112,112] zero-padded to Cp channels; the 7x7 kernel is
embedded at offset 1 in an 8x8 kernel and folded to 4x4 taps over (dr, dc, c) channels; padding (2,1,2,1)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, reps=10):
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


def s2d_input(x, Cp):
    """[N,3,H,W] -> [N,Cp,H/2,W/2] channels-last, channel index = (dr*2 + dc)*3 + c."""
    N, C, H, W = x.shape
    y = x.reshape(N, C, H // 2, 2, W // 2, 2).permute(0, 3, 5, 1, 2, 4).reshape(N, 4 * C, H // 2, W // 2)
    if Cp > 4 * C:
        y = F.pad(y, (0, 0, 0, 0, 0, Cp - 4 * C))
    return y.contiguous(memory_format=torch.channels_last)


def s2d_weight(w, Cp):
    """[K,3,7,7] -> [K,Cp,4,4]."""
    K, C, R, S = w.shape
    w8 = F.pad(w, (1, 0, 1, 0))                                      # tap i -> i+1 in an 8x8 kernel
    w4 = w8.reshape(K, C, 4, 2, 4, 2).permute(0, 3, 5, 1, 2, 4).reshape(K, 4 * C, 4, 4)
    if Cp > 4 * C:
        w4 = F.pad(w4, (0, 0, 0, 0, 0, Cp - 4 * C))
    return w4


def main():
    from deeplearning4j_amd.ops import conv_native as cn
    dev = torch.device("cuda")
    N = int(os.environ.get("N", 512))
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, 3, 224, 224, generator=g).to(dev).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(dev).bfloat16()
    ref = F.conv2d(x, w, None, 2, 3)
    dy = torch.randn(ref.shape, generator=g).to(dev).bfloat16().contiguous(memory_format=torch.channels_last)
    flops = 2 * ref.numel() * 147
    print(f"MIOpen fwd {t(lambda: F.conv2d(x, w, None, 2, 3)):.3f} ms")
    wr = w.clone().requires_grad_(True)

    def mi_wrw():
        torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                            [False, True, False])
    print(f"MIOpen wrw {t(mi_wrw):.3f} ms")
    _ = wr
    for Cp in (16, 32):
        xs = s2d_input(x, Cp)
        ws = s2d_weight(w, Cp)
        cn.bump_version()
        y = cn.conv2d_fwd(xs, ws, None, (1, 1), (2, 1, 2, 1), (1, 1))
        err = (y.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
        tf = t(lambda: cn.conv2d_fwd(xs, ws, None, (1, 1), (2, 1, 2, 1), (1, 1)))
        tx = t(lambda: s2d_input(x, Cp))
        gW = torch.zeros(64, Cp, 4, 4, device=dev)
        tw = t(lambda: cn.conv2d_bwd(xs, ws, dy, (1, 1), (2, 1, 2, 1), (1, 1), False, True, False, gW, None))
        # weight-gradient numerics: fold back to 7x7 and compare with MIOpen's
        gW.zero_()
        cn.conv2d_bwd(xs, ws, dy, (1, 1), (2, 1, 2, 1), (1, 1), False, True, False, gW, None)
        g4 = gW[:, :12].reshape(64, 2, 2, 3, 4, 4).permute(0, 3, 4, 1, 5, 2).reshape(64, 3, 8, 8)[:, :, 1:, 1:]
        _, gref, _ = torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                         [False, True, False])
        werr = (g4 - gref.float()).abs().max().item() / gref.float().abs().max().item()
        print(f"s2d Cp={Cp}: fwd {tf:.3f} ms ({flops / tf / 1e9:.0f} TF eff) + s2d {tx:.3f} ms, wrw {tw:.3f} ms, "
              f"fwd rel err {err:.2e}, wrw rel err {werr:.2e}")


if __name__ == "__main__":
    main()
