#!/usr/bin/env python3
"""BERT-base fine-tuning step through the SameDiff import (BASELINE.json "BERT-base SameDiff import"): a random-init
HuggingFace BertForSequenceClassification (12L / 768 / 12 heads, no download) is imported with importBertSameDiff in
bf16 (fp32 master weights in the fused updater), then trained with TrainingConfig(Adam) + sd.fit on synthetic token
ids. Prints one JSON line with tokens/s. The ComputationGraph path (hand-written backward) is tools/bench_bert.py."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=128)
    args = ap.parse_args()
    import transformers
    from deeplearning4j_amd import Adam, MultiDataSet
    from deeplearning4j_amd.modelimport.bert import importBertSameDiff
    from deeplearning4j_amd.samediff import TrainingConfig
    dev = torch.device("cuda", 0)
    cfg = transformers.BertConfig(num_labels=2)
    torch.manual_seed(0)
    hf = transformers.BertForSequenceClassification(cfg)
    B, T = args.batch, args.seq
    sd = importBertSameDiff(hf.state_dict(), cfg.to_dict(), seqLen=T, device=dev, dtype=torch.bfloat16, batch=B)
    del hf
    sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(2e-5)).dataSetFeatureMapping("input_ids",
                                                                                            "attention_mask")
                         .dataSetLabelMapping("labels").build())
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (B, T), generator=g).to(dev)
    am = torch.ones(B, T, device=dev)
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (B,), generator=g), 2).to(torch.bfloat16).to(dev)
    mds = MultiDataSet([ids, am], [y])
    for _ in range(args.warmup):
        sd.fit(mds)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = sd.fit(mds)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "tokens/sec BERT-base fine-tuning through the SameDiff import on one MI355X",
                      "value": round(B * T * args.steps / dt, 1), "unit": "tokens/sec", "n_gpus": 1,
                      "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
                      "higher_is_better": True, "dtype": "bf16", "data": "synthetic token ids; random-init weights",
                      "config": {"model": "BERT-base (12L/768/12H) SameDiff import", "batch": B, "seq_len": T},
                      "loss": loss}))


if __name__ == "__main__":
    main()
