#!/usr/bin/env python3
"""Per-shape timing of the MFMA implicit-GEMM conv kernels on the ResNet-50 conv shapes, vs MIOpen (torch).

Shapes are captured from the zoo ResNet50 graph (batch scaled to --batch). For every unique shape the native
forward, backward-data (when the network needs it) and weight-gradient kernels are timed with HIP events and
reported as ms and TFLOP/s, next to torch's (MIOpen) time for the same op. Usage on a GPU box:
    python tools/conv_bench.py --batch 256 [--variant dl4j] [--reps 20]
"""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def capture_shapes(variant):
    from deeplearning4j_amd import ops
    from deeplearning4j_amd.models import ResNet50
    shapes = []
    orig = ops.conv.conv2d_forward

    def hook(x, w, b, stride, pad4, dilation=(1, 1), groups=1, **kw):
        shapes.append((tuple(x.shape[1:]), tuple(w.shape), tuple(stride), tuple(pad4), tuple(dilation)))
        return orig(x, w, b, stride, pad4, dilation, groups, **kw)
    import deeplearning4j_amd.nn.layers.convolution as lc
    lc.ops.conv2d_forward = hook
    try:
        net = ResNet50(numLabels=1000, variant=variant).init(device=torch.device("cpu"))
        with torch.no_grad():
            net.output(torch.rand(1, 3, 224, 224))
    finally:
        lc.ops.conv2d_forward = orig
    return shapes


def timeit(fn, reps):
    """GPU ms per call, host enqueue hidden behind a spin kernel (deeplearning4j_amd/ops/timing.py)."""
    from deeplearning4j_amd.ops.timing import gpu_time
    return gpu_time(fn, reps=reps, warmup=3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--variant", default="dl4j")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--kernel-variant", type=int, default=1)
    ap.add_argument("--sweep-wrw", action="store_true", help="time the weight-gradient kernel for several splits")
    a = ap.parse_args()
    from deeplearning4j_amd.ops import conv_native as CN
    dev = torch.device("cuda")
    CN.set_kernel_variant(a.kernel_variant)
    shapes = capture_shapes(a.variant)
    count = collections.Counter(shapes)
    rows = []
    tot = collections.defaultdict(float)
    print(f"{'C,H,W':>14} {'K,R,S':>10} st  cnt | {'fwd ms':>7} {'TF':>5} {'miop':>6} | {'bwdD ms':>7} {'TF':>5} "
          f"{'miop':>6} | {'wrw ms':>7} {'TF':>5} {'miop':>6}")
    for (xs, ws, st, pad, dil), n in sorted(count.items(), key=lambda kv: -kv[1]):
        C, H, W = xs
        K, _, R, S = ws
        if C % 8 != 0:
            continue
        N = a.batch
        x = torch.randn(N, C, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, S, device=dev) * 0.05).to(torch.bfloat16)
        y = CN.conv2d_fwd(x, w, None, st, pad, dil)
        OH, OW = y.shape[2], y.shape[3]
        flops = 2.0 * N * OH * OW * K * C * R * S
        dy = torch.randn_like(y)
        gW = torch.zeros(K, C, R, S, device=dev)
        f_ms = timeit(lambda: CN.conv2d_fwd(x, w, None, st, pad, dil), a.reps)
        d_ms = timeit(lambda: CN.conv2d_bwd(x, w, dy, st, pad, dil, True, False, False), a.reps)
        w_ms = timeit(lambda: CN.conv2d_bwd(x, w, dy, st, pad, dil, False, True, False, gW), a.reps)
        if a.sweep_wrw:
            key = (N, H, W, C, K, R, S, tuple(st))
            res = []
            for sp in (1, 2, 4, 8, 16, 32, 64, 128):
                CN.WRW_SPLITS[key] = sp
                res.append((timeit(lambda: CN.conv2d_bwd(x, w, dy, st, pad, dil, False, True, False, gW), a.reps), sp))
            CN.WRW_SPLITS.pop(key)
            M = N * OH * OW
            tiles = ((K + 127) // 128) * ((R * S * C + 127) // 128)
            print(f"   wrw sweep M={M} tiles={tiles}: " + " ".join(f"{sp}:{t*1e3:.0f}us" for t, sp in res))
        sym = pad[0] == pad[1] and pad[2] == pad[3]
        if sym:
            xm = x
            mf = timeit(lambda: torch.nn.functional.conv2d(xm, w, None, st, (pad[0], pad[2]), dil), a.reps)
            md = timeit(lambda: torch.ops.aten.convolution_backward(dy, xm, w, None, list(st), [pad[0], pad[2]],
                                                                    list(dil), False, [0, 0], 1,
                                                                    [True, False, False]), a.reps)
            mw = timeit(lambda: torch.ops.aten.convolution_backward(dy, xm, w, None, list(st), [pad[0], pad[2]],
                                                                    list(dil), False, [0, 0], 1,
                                                                    [False, True, False]), a.reps)
        else:
            mf = md = mw = float("nan")
        tf = lambda ms: flops / ms / 1e9  # noqa: E731
        print(f"{C:>4},{H:>4},{W:>4} {K:>4},{R},{S} {st[0]}  {n:>3} | {f_ms:7.3f} {tf(f_ms):5.0f} {mf:6.3f} | "
              f"{d_ms:7.3f} {tf(d_ms):5.0f} {md:6.3f} | {w_ms:7.3f} {tf(w_ms):5.0f} {mw:6.3f}")
        rows.append(dict(C=C, H=H, W=W, K=K, R=R, S=S, stride=st, count=n, fwd=f_ms, bwd_data=d_ms, wrw=w_ms,
                         miopen_fwd=mf, miopen_bwd_data=md, miopen_wrw=mw, gflop=flops / 1e9))
        tot["fwd"] += n * f_ms
        tot["bwd_data"] += n * d_ms
        tot["wrw"] += n * w_ms
        tot["miopen_fwd"] += n * mf
        tot["miopen_bwd_data"] += n * md
        tot["miopen_wrw"] += n * mw
        del x, w, y, dy, gW
    print("totals (ms, weighted by count):", {k: round(v, 3) for k, v in tot.items()})
    for k, v in CN._V3_CHOICE.items():
        g = k[1]
        print(f"choice {k[0]:8s} N{g[0]} {g[3]}x{g[1]}x{g[2]} -> K{g[4]} {g[5]}x{g[6]}/{g[7]}: "
              f"{'igemm(r2)' if v < 0 else f'v3 variant {v}'}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": rows, "totals": tot}, f, indent=1)


if __name__ == "__main__":
    main()
