#!/usr/bin/env python3
"""BERT-base fine-tuning step through the SameDiff import (BASELINE.json "BERT-base SameDiff import"): a random-init
HuggingFace BertForSequenceClassification (12L / 768 / 12 heads, no download) is imported with importBertSameDiff in
bf16 or fp16 (``--dtype``; fp32 master weights in the fused updater), then trained with TrainingConfig(Adam) + sd.fit
on synthetic token ids. Under ``torch.distributed.run --nproc-per-node N`` every rank trains its own batch and the
flat gradient is averaged over RCCL before the update (weak scaling; BASELINE config #5 is the 8-GPU fp16 run).
Prints one JSON line (rank 0) with the whole-job tokens/s. The ComputationGraph path is tools/bench_bert.py."""
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
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--graph", type=int, default=1, help="capture the training step into HIP graphs")
    args = ap.parse_args()
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    import transformers
    from deeplearning4j_amd import Adam, MultiDataSet
    from deeplearning4j_amd.modelimport.bert import importBertSameDiff
    from deeplearning4j_amd.samediff import TrainingConfig
    dev = torch.device("cuda", local)
    cfg = transformers.BertConfig(num_labels=2)
    torch.manual_seed(0)
    hf = transformers.BertForSequenceClassification(cfg)
    B, T = args.batch, args.seq
    sd = importBertSameDiff(hf.state_dict(), cfg.to_dict(), seqLen=T, device=dev, dtype=dt, batch=B)
    del hf
    sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(2e-5)).dataSetFeatureMapping("input_ids",
                                                                                            "attention_mask")
                         .dataSetLabelMapping("labels").build())
    g = torch.Generator().manual_seed(1 + rank)
    ids = torch.randint(0, cfg.vocab_size, (B, T), generator=g).to(dev)
    am = torch.ones(B, T, device=dev)
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (B,), generator=g), 2).to(dt).to(dev)
    mds = MultiDataSet([ids, am], [y])
    if args.graph:
        sd.enableHipGraphs(True, warmup=2)
    for _ in range(args.warmup):
        sd.fit(mds)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = sd.fit(mds)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    if rank == 0:
        print(json.dumps({"metric": "tokens/sec BERT-base fine-tuning through the SameDiff import (whole job)",
                          "value": round(world * B * T * args.steps / el, 1), "unit": "tokens/sec", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
                          "higher_is_better": True, "scaling": "weak", "dtype": args.dtype,
                          "data": "synthetic token ids; random-init weights",
                          "config": {"model": "BERT-base (12L/768/12H) SameDiff import", "per_gpu_batch": B,
                                     "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}"},
                          "hip_graph": bool(sd._graph is not None and sd._graph["ok"]), "loss": loss}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
