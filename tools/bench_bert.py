#!/usr/bin/env python3
"""BERT-base training throughput (BASELINE.json config "BERT-base ... (attention matmul + LayerNorm MFMA)"):
sequences/sec and tokens/sec of a full fine-tuning step (forward, backward, Adam update of all 110M params) on one
MI355X, bf16 compute / fp32 master weights, synthetic token ids, random-init weights.

  --impl dl4j   this framework: BertBase ComputationGraph (flash-attention + LayerNorm HIP kernels, fused QKV,
                in-tree MFMA GEMMs, fused HIP Adam updater)
  --impl torch  like-for-like PyTorch-ROCm comparator: transformers.BertForSequenceClassification in bf16 with
                torch.optim.AdamW(fused=True) and SDPA attention

Usage: python tools/bench_bert.py [--impl dl4j|torch] [--batch 32] [--seq 128] [--steps 10] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def run_dl4j(args, dev):
    from deeplearning4j_amd.models import BertBase
    from deeplearning4j_amd.nn.conf import DataType
    net = BertBase(numLabels=2, inputShape=[args.seq], layers=args.layers,
                   dataType={"bf16": DataType.BFLOAT16, "fp16": DataType.HALF}.get(args.dtype, DataType.FLOAT)
                   ).init(device=dev)
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 30522, (args.batch, args.seq), generator=g).to(dev)
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (args.batch,), generator=g), 2).float().to(dev)

    if args.graph:
        net.enableHipGraphs(True, warmup=2)

    def step():
        net.fit([x], [y])
    return step, net.numParams(), lambda: net.score()


def run_torch(args, dev):
    import transformers
    cfg = transformers.BertConfig(num_hidden_layers=args.layers, num_labels=2, attn_implementation="sdpa")
    model = transformers.BertForSequenceClassification(cfg).to(dev)
    if args.dtype in ("bf16", "fp16"):
        model = model.to(torch.bfloat16 if args.dtype == "bf16" else torch.float16)
    model.train()
    opt = torch.optim.AdamW(model.parameters(), lr=2e-5, fused=dev.type == "cuda")
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 30522, (args.batch, args.seq), generator=g).to(dev)
    y = torch.randint(0, 2, (args.batch,), generator=g).to(dev)
    last = {}

    def step():
        out = model(input_ids=x, labels=y)
        out.loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        last["loss"] = out.loss.detach()
    return step, sum(p.numel() for p in model.parameters()), lambda: float(last["loss"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", default="dl4j", choices=["dl4j", "torch"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--graph", type=int, default=1, help="capture the dl4j training step in HIP graphs")
    args = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    step, nparams, score = (run_dl4j if args.impl == "dl4j" else run_torch)(args, dev)
    for _ in range(args.warmup):
        step()
    _sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    _sync()
    el = time.perf_counter() - t0
    sps = args.batch * args.steps / el
    print(json.dumps({
        "metric": "BERT-base fine-tuning throughput on one MI355X", "value": round(sps * args.seq, 1),
        "unit": "tokens/sec", "sequences_per_sec": round(sps, 2), "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1000, 2), "higher_is_better": True,
        "dtype": args.dtype, "impl": args.impl, "hip_graph": bool(args.graph and args.impl == "dl4j"), "data": "synthetic token ids; random-init weights",
        "config": {"model": f"BERT-base ({args.layers} layers, 768 hidden, 12 heads) + classifier",
                   "batch": args.batch, "seq_len": args.seq, "params": nparams}, "final_score": score()}),
          flush=True)


if __name__ == "__main__":
    main()
