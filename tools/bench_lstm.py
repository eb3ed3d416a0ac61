#!/usr/bin/env python3
"""Secondary benchmark (BASELINE.json config "LSTM char-LM ... on one MI355X"): TextGenerationLSTM training
throughput in characters/sec.

Model: the reference's zoo TextGenerationLSTM (ZOO:model/TextGenerationLSTM.java:76-89): 2x GravesLSTM(256, tanh,
peepholes) -> RnnOutputLayer(MCXENT, softmax), RmsProp(0.01), l2 1e-3, truncated BPTT 50/50; the reference's
char-modelling example shape (77 characters, minibatch 32, 1000-character sequences). Synthetic one-hot data,
random-init weights. Every timed step is one fit() over a [32, 77, 1000] minibatch = 20 TBPTT segments, each a
full forward + backward + RmsProp update.

Usage: python tools/bench_lstm.py [--steps K --warmup W --batch B --length L --dtype bf16|fp32]
       DL4J_AMD_KERNEL_LSTM=0 runs the per-step (library GEMM + elementwise) path for comparison.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--length", type=int, default=1000)
    ap.add_argument("--chars", type=int, default=77)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--graph", type=int, default=1, help="replay TBPTT windows as HIP graphs (nn/hipgraph.py)")
    args = ap.parse_args()

    from deeplearning4j_amd.models import TextGenerationLSTM
    from deeplearning4j_amd.nn.conf import DataType
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    dt = DataType.BFLOAT16 if args.dtype == "bf16" else DataType.FLOAT
    net = TextGenerationLSTM(numLabels=args.chars, inputShape=[1, args.chars], hidden=args.hidden,
                             dataType=dt).init(device=dev)
    if args.graph and dev.type == "cuda":
        net.enableHipGraphs(True, warmup=1)
    g = torch.Generator().manual_seed(7)
    idx = torch.randint(0, args.chars, (args.batch, args.length + 1), generator=g)
    x = torch.nn.functional.one_hot(idx[:, :-1], args.chars).permute(0, 2, 1).float().to(dev)
    y = torch.nn.functional.one_hot(idx[:, 1:], args.chars).permute(0, 2, 1).float().to(dev)

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
    cps = args.batch * args.length * args.steps / el
    print(json.dumps({
        "metric": "characters/sec TextGenerationLSTM training (TBPTT 50) on one MI355X", "value": round(cps, 1),
        "unit": "chars/sec", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1000, 2), "higher_is_better": True, "dtype": args.dtype,
        "data": "synthetic one-hot characters; random-init weights",
        "lstm_kernel": "sequence-HIP" if os.environ.get("DL4J_AMD_KERNEL_LSTM", "1") != "0" else "per-step",
        "hip_graph": bool(args.graph and dev.type == "cuda"),
        "config": {"model": "TextGenerationLSTM (2x GravesLSTM 256)", "batch": args.batch, "seq_len": args.length,
                   "chars": args.chars, "tbptt": 50}, "final_score": net.score()}), flush=True)


if __name__ == "__main__":
    main()
