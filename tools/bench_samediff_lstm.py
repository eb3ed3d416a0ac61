#!/usr/bin/env python3
"""LSTM char-LM defined and trained through SameDiff (BASELINE.json config "LSTM char-LM via SameDiff on one
MI355X"): placeholders for one-hot characters, two whole-sequence LSTM layers (GravesLSTM-style peepholes, 256 units,
csrc/lstm*.hip kernels), a projection to 77 characters and sd.loss().softmaxCrossEntropy. Trained with
TrainingConfig(Adam) + sd.fit in bf16 (fp32 master weights, fused HIP updater). Each iteration is one 50-character
window of a 32-sequence batch (the SameDiff graph carries no state across windows: no TBPTT in SameDiff); a timed
step is one sd.fit call over the 20 windows of a 1000-character sequence, as the MultiLayerNetwork bench's TBPTT step
(tools/bench_lstm.py), with the iteration captured in HIP graphs (--graph 0: eager). Prints one JSON line with
characters/s. Synthetic data, random-init weights."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(dev, mb, T, V, H, seed=0):
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.samediff import SameDiff, TrainingConfig
    g = torch.Generator().manual_seed(seed)
    bf = torch.bfloat16

    def p(*shape, scale):
        return (torch.randn(*shape, generator=g) * scale).to(bf).to(dev)

    sd = SameDiff.create()
    x = sd.placeHolder("x", torch.zeros(mb, V, T, dtype=bf, device=dev))
    y = sd.placeHolder("y", torch.zeros(mb, T, V, dtype=bf, device=dev))
    h = x
    nin = V
    for i in range(2):
        W = sd.var(f"W{i}", p(nin, 4 * H, scale=nin ** -0.5))
        RW = sd.var(f"RW{i}", p(H, 4 * H + 3, scale=H ** -0.5))
        b = sd.var(f"b{i}", torch.zeros(4 * H, dtype=bf, device=dev))
        h = sd.rnn().lstmLayer(f"lstm{i}", h, W, RW, b, peephole=True)
        nin = H
    Wo = sd.var("Wo", p(H, V, scale=H ** -0.5))
    bo = sd.var("bo", torch.zeros(V, dtype=bf, device=dev))
    logits = sd.nn().linear("logits", h.permute(0, 2, 1), Wo, bo)
    sd.loss().softmaxCrossEntropy("loss", y, logits)
    sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(2e-3)).dataSetFeatureMapping("x")
                         .dataSetLabelMapping("y").build())
    return sd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--window", type=int, default=50)
    ap.add_argument("--windows", type=int, default=20, help="windows per sd.fit call (one timed step)")
    ap.add_argument("--graph", type=int, default=1)
    args = ap.parse_args()
    from deeplearning4j_amd import DataSet
    dev = torch.device("cuda", 0)
    V, H, mb, T = 77, 256, args.batch, args.window
    sd = build(dev, mb, T, V, H)
    if args.graph:
        sd.enableHipGraphs(True, warmup=2)
    g = torch.Generator().manual_seed(1)
    idx = torch.randint(0, V, (mb, T + 1), generator=g)
    X = torch.nn.functional.one_hot(idx[:, :-1], V).permute(0, 2, 1).to(torch.bfloat16).to(dev)
    Y = torch.nn.functional.one_hot(idx[:, 1:], V).to(torch.bfloat16).to(dev)
    seq = [DataSet(X, Y)] * args.windows
    for _ in range(args.warmup):
        sd.fit(seq)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = sd.fit(seq)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "characters/sec LSTM char-LM trained through SameDiff on one MI355X",
                      "value": round(mb * T * args.windows * args.steps / dt, 1), "unit": "chars/sec", "n_gpus": 1,
                      "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
                      "higher_is_better": True, "dtype": "bf16",
                      "data": "synthetic one-hot characters; random-init weights",
                      "hip_graph": bool(sd._graph is not None and sd._graph["ok"]),
                      "config": {"model": "SameDiff 2x LSTM-256 (peephole) + softmax 77", "batch": mb,
                                 "window": T, "windows_per_step": args.windows}, "loss": loss}))


if __name__ == "__main__":
    main()
