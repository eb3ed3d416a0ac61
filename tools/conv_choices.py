#!/usr/bin/env python3
"""Which kernel the per-shape autotuners picked for every ResNet-50 conv (after a warm-up step of the bench model):
forward / backward-data tile choice (round-3 engine variant id or -1 = round-2 implicit-GEMM kernel), 1x1 GEMM-vs-igemm
choice, and weight-gradient engine. Usage on a GPU box: python tools/conv_choices.py [--batch 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

V3_TILES = {0: "v3 256x128", 1: "v3 128x128", 2: "v3 256x64", 3: "v3 128x64", 4: "v3 128x256", -1: "r2 igemm 128x128"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.ops import conv_native as cn
    dev = torch.device("cuda", 0)
    net = ResNet50(numLabels=1000, dataType=DataType.BFLOAT16).init(device=dev)
    x = torch.rand(args.batch, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
    x = x.to(net.compute_dtype)
    y = torch.zeros(args.batch, 1000, device=dev)
    y[torch.arange(args.batch), torch.randint(0, 1000, (args.batch,))] = 1
    for _ in range(args.steps):
        net.fit(x, y)
    torch.cuda.synchronize()
    print("fwd / bwd-data tile choices (geometry N,H,W,C,K,R,S,sh,sw,ph,pw,dh,dw,OH,OW):")
    for key, v in sorted(cn._V3_CHOICE.items(), key=lambda kv: str(kv[0])):
        g = key[1]
        M = g[0] * g[13] * g[14]
        flop = 2.0 * M * g[4] * g[3] * g[5] * g[6]
        print(f"  {key[0]:10s} C={g[3]:4d} K={g[4]:4d} {g[5]}x{g[6]} s{g[7]} {g[1]}x{g[2]}->{g[13]}x{g[14]} "
              f"M={M:8d} GF={flop / 1e9:7.1f} -> {V3_TILES.get(v, v)}")
    print("1x1 GEMM-vs-igemm choices (True = GEMM):")
    for key, v in sorted(cn._CHOICE.items(), key=lambda kv: str(kv[0])):
        print(f"  {key} -> {v}")
    print("weight-gradient choices:")
    for key, v in sorted(cn._WRW_CHOICE.items(), key=lambda kv: str(kv[0])):
        print(f"  {key} -> {v}")


if __name__ == "__main__":
    main()
