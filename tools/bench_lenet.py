#!/usr/bin/env python3
"""BASELINE.json config "LeNet-MNIST MultiLayerNetwork on the CPU backend (plumbing, no GPU)": the zoo LeNet
(ZOO:model/LeNet.java: conv 5x5/20 -> maxpool -> conv 5x5/50 -> maxpool -> dense 500 -> softmax 10, AdaDelta)
trained on MNIST-shaped synthetic data (flat 784-pixel rows in [0, 1], one-hot labels; no dataset download), fp32,
on the CPU by default (``--device cuda`` runs the same network on the GPU kernels). Prints one JSON line:
images/sec over the timed steps.
Usage: python tools/bench_lenet.py [--steps K --warmup W --batch B --device cpu|cuda --graph 0|1]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--device", default="cpu", choices=["cpu", "cuda"])
    ap.add_argument("--graph", type=int, default=1, help="cuda: replay the training step as a HIP graph (the step is "
                    "launch-bound: profiles/r4_lenet_gpu.txt, 36.3k eager vs 89.9k img/s, identical final score)")
    args = ap.parse_args()
    from deeplearning4j_amd.models import LeNet
    dev = torch.device("cuda", 0) if args.device == "cuda" else torch.device("cpu")
    net = LeNet(numLabels=10).init(device=dev)
    if args.graph and dev.type == "cuda":
        net.enableHipGraphs(True, warmup=1)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(args.batch, 784, generator=g).to(dev)
    y = torch.nn.functional.one_hot(torch.randint(0, 10, (args.batch,), generator=g), 10).float().to(dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    for _ in range(args.warmup):
        net.fit(x, y)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        net.fit(x, y)
    sync()
    el = time.perf_counter() - t0
    print(json.dumps({"metric": f"images/sec LeNet-MNIST MultiLayerNetwork training on {dev.type}",
                      "value": round(args.batch * args.steps / el, 1), "unit": "images/sec", "steps": args.steps,
                      "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1000, 3), "dtype": "fp32",
                      "data": "synthetic MNIST-shaped (784 pixels, 10 classes); random-init weights",
                      "config": {"model": "LeNet (DL4J zoo)", "batch": args.batch,
                                 "hip_graph": getattr(net, "_hipgraph", None) is not None}, "final_score": net.score()}),
          flush=True)


if __name__ == "__main__":
    main()
