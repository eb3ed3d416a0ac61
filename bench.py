#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 ComputationGraph training throughput (images/sec, whole job).

Metric/config from BASELINE.json: "images/sec (whole node) ResNet-50 training at 1/2/4/8 MI355X",
config "ResNet-50 ComputationGraph bf16 on one MI355X (conv2d im2col+MFMA path)" and
"ResNet-50 ParallelWrapper DP=8 with RCCL gradient all-reduce over xGMI".

Model: the reference's zoo ResNet50 graph (ZOO:model/ResNet50.java: stride-2 stage 2, MAX-3x3 head,
RmsProp(0.1,0.96,1e-3), l1 1e-7, l2 5e-5) with random-init weights; synthetic 224x224x3 images and
one-hot labels (BenchmarkDataSetIterator semantics: one fixed random batch, re-fed every step).
``--variant canonical`` runs standard ResNet-50 instead. Every timed step is a full training
iteration: forward, backward, (DP) gradient all-reduce, fused RmsProp update of all 25.6M params.

Usage: python bench.py [--gpus N --steps K --warmup W --batch B]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N  (one rank per GPU, RCCL), or
plain ``python bench.py --gpus N`` for the in-process ParallelWrapper (one host thread per GPU, ncclCommInitAll).
"""
import argparse
import json
import os
import sys
import time

import torch


def _kernel_db():
    """Which kernel-choice database the autotuners consulted (ops/tunedb.py), for the JSON provenance."""
    from deeplearning4j_amd.ops import tunedb
    p = tunedb.loaded_from()
    return os.path.relpath(p, os.path.dirname(os.path.abspath(__file__))) if p else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # per-GPU batch, sized for 288 GB of HBM: the late 7x7 / 14x14 stages need a large batch to fill 256 CUs and
    # the per-step serial tail (stem, BN folds, the fused update) amortizes over more images. Measured on one MI355X
    # (profiles/r4_batch_sweep.txt): 512 -> 34.4k, 768 -> 36.5k, 1024 -> 38.2k img/s at 20.3 GiB peak,
    # 2048 -> 40.6k at 39.9 GiB. 1024 is the default; weak scaling keeps it per GPU
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BENCH_BATCH", 1024)), help="per-GPU batch")
    ap.add_argument("--variant", default=os.environ.get("BENCH_VARIANT", "dl4j"), choices=["dl4j", "canonical"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--graph", type=int, default=int(os.environ.get("BENCH_GRAPH", "0")),
                    help="capture the training step in HIP graphs (1 on, 0 off (default), -1 auto = on unless the "
                         "collectives are not capturable, i.e. gloo). Off by default for ResNet-50: the "
                         "step is not launch-bound (~520 kernels in 15 ms at batch 512) and eager launches keep the conv "
                         "weight-gradient stream concurrent with the data-gradient chain, which a replayed graph "
                         "does not (profiles/r4_eager_vs_graph.txt: 32.8-32.9k eager vs 31.3k graph img/s)")
    ap.add_argument("--comm-dtype", default=os.environ.get("BENCH_COMM_DTYPE", "fp32"), choices=["fp32", "bf16"],
                    help="gradient all-reduce dtype for N > 1")
    ap.add_argument("--comm", default=os.environ.get("BENCH_COMM", "torch"), choices=["torch", "rccl"],
                    help="N > 1 transport: torch.distributed's RCCL process group, or the framework's own RCCL "
                         "communicator (parallel/rccl.py, ncclCommInitRank with the id exchanged through the store)")
    ap.add_argument("--inprocess", type=int, default=-1,
                    help="one process, one host thread per GPU (ParallelWrapper.inProcess: replicas on GPUs 0..N-1, "
                         "RCCL communicators from ncclCommInitAll, graph-captured steps per worker). Default (-1): on "
                         "whenever --gpus N > 1 is run WITHOUT torchrun (the reference's ParallelWrapper design); "
                         "1 forces it (also at N = 1), 0 disables it. Ignored under torchrun (WORLD_SIZE set), which "
                         "runs one process per GPU over torch.distributed's RCCL group")
    args = ap.parse_args()
    under_torchrun = "WORLD_SIZE" in os.environ
    if not under_torchrun and (args.inprocess == 1 or (args.inprocess < 0 and args.gpus > 1)):
        return main_inprocess(args)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.parallel.accumulation import AllReduceGradientsAccumulator
    from deeplearning4j_amd.parallel.distributed import all_reduce_max, barrier, init_distributed

    world, rank, local, device = init_distributed()
    if world != args.gpus and rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.manual_seed(1234 + rank)

    dt = DataType.BFLOAT16 if args.dtype == "bf16" else DataType.FLOAT
    net = ResNet50(numLabels=1000, variant=args.variant, dataType=dt).init(device=device)
    acc = None
    if world > 1:
        # bucketed RCCL all-reduce overlapped with backward; captured into the step's HIP graph (nccl backend)
        comm = None
        if args.comm == "rccl" and device.type == "cuda":
            from deeplearning4j_amd.parallel.rccl import RcclComm
            comm = RcclComm.from_process_group(device)
        acc = AllReduceGradientsAccumulator(dtype=args.comm_dtype, comm=comm)
        acc.broadcast_params(net)
        net.setGradientsAccumulator(acc)

    use_graph = args.graph if args.graph >= 0 else int(device.type == "cuda" and (acc is None or acc.capturable()))
    if use_graph:
        net.enableHipGraphs(True, warmup=1)

    B = args.batch
    g = torch.Generator(device="cpu").manual_seed(42 + rank)
    x = torch.rand(B, 3, 224, 224, generator=g).to(device)
    if device.type == "cuda":
        x = x.contiguous(memory_format=torch.channels_last)
    x = x.to(net.compute_dtype)
    y = torch.zeros(B, 1000, device=device)
    y[torch.arange(B), torch.randint(0, 1000, (B,), generator=g).to(device)] = 1.0

    # experiment switch: run the training step on a high-priority stream (the weight-gradient side stream keeps
    # the default priority, so the main chain's kernels are dispatched first when both are queued)
    prio_stream = None
    if os.environ.get("DL4J_AMD_MAIN_PRIO", "0") == "1" and device.type == "cuda":
        prio_stream = torch.cuda.Stream(device, priority=-1)
        prio_stream.wait_stream(torch.cuda.current_stream(device))

    def step():
        if prio_stream is not None:
            with torch.cuda.stream(prio_stream):
                net.fit([x], [y])
        else:
            net.fit([x], [y])

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    t_w = time.perf_counter()
    for i in range(args.warmup):
        step()
        if rank == 0 and (i == 0 or time.perf_counter() - t_w > 60):
            sync()
            print(f"[bench] warmup step {i} done, score={net.score():.4f}, {time.perf_counter() - t_w:.1f}s",
                  file=sys.stderr, flush=True)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    elapsed = all_reduce_max(elapsed)
    ms = elapsed / args.steps * 1000.0
    ips = B * world * args.steps / elapsed
    final_score = net.score()
    if rank == 0:
        model_name = "ResNet-50 (DL4J zoo ResNet50 graph)" if args.variant == "dl4j" else "ResNet-50 (canonical)"
        print(json.dumps({
            "metric": "images/sec (whole node) ResNet-50 training at 1/2/4/8 MI355X",
            "value": round(ips, 2), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (random 224x224x3 images, one-hot labels; random-init weights)",
            "config": {"model": model_name, "variant": args.variant, "global_batch": B * world, "per_gpu_batch": B,
                       "seq_len": None, "image_size": 224, "parallelism": f"dp{world}", "comm": args.comm,
                       "updater": "RmsProp(0.1,0.96,1e-3) + l1 1e-7 + l2 5e-5 (fused HIP updater)",
                       "hip_graph": bool(use_graph and getattr(net, "_hipgraph", None) is not None),
                       "kernel_db": _kernel_db(),
                       "final_score": final_score, **memory_report(device)},
        }), flush=True)
    from deeplearning4j_amd.parallel.distributed import destroy
    destroy()


def memory_report(device):
    """Peak device memory of the run, counting every allocator: torch's caching allocator (parameters, gradients,
    updater state, torch-allocated activations) PLUS the engine's own allocator (csrc/engine.hip: the LOOP_FF_BP
    activation arena and other workspace blocks, which torch does not see), and the device-wide HBM in use at the
    end (hipMemGetInfo: total - free, i.e. every reservation of this process incl. RCCL / runtime buffers)."""
    if device.type != "cuda":
        return {}
    torch_peak = torch.cuda.max_memory_allocated(device)
    eng_peak = eng_reserved = 0
    try:
        from deeplearning4j_amd.runtime import allocator
        st = allocator(device.index).stats()
        eng_peak, eng_reserved = int(st["peak"]), int(st["reserved"])
    except Exception:
        pass
    free, total = torch.cuda.mem_get_info(device)
    g = 2.0 ** 30
    return {"peak_mem_gib": round((torch_peak + eng_peak) / g, 2),
            "peak_mem_torch_gib": round(torch_peak / g, 2), "peak_mem_engine_gib": round(eng_peak / g, 2),
            "engine_reserved_gib": round(eng_reserved / g, 2), "device_used_gib": round((total - free) / g, 2),
            "device_total_gib": round(total / g, 1)}


def main_inprocess(args):
    """``--inprocess``: the reference's ParallelWrapper design on one node — N worker threads in this process, each
    training a replica on its own GPU (parallel/inprocess.py), gradients all-reduced in buckets over RCCL
    (ncclCommInitAll) on a per-device comm stream overlapping backward. Same model, batch per GPU and timing rule as
    the torchrun path: W untimed warmup rounds, then K timed rounds between device synchronisations."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from deeplearning4j_amd.datasets.dataset import DataSet
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.parallel import ParallelWrapper, TrainingMode
    N = args.gpus
    torch.manual_seed(1234)
    dt = DataType.BFLOAT16 if args.dtype == "bf16" else DataType.FLOAT
    dev0 = torch.device("cuda", 0)
    net = ResNet50(numLabels=1000, variant=args.variant, dataType=dt).init(device=dev0)
    # N worker threads issuing eager launches would contend for the GIL: graphs on unless --graph 0 is explicit
    use_graph = args.graph != 0 or "--graph" not in " ".join(sys.argv)
    if use_graph:
        net.enableHipGraphs(True, warmup=1)
    B = args.batch
    g = torch.Generator(device="cpu").manual_seed(42)
    per_dev = []
    for i in range(N):            # one fixed batch per worker, already on its GPU (BenchmarkDataSetIterator)
        d = torch.device("cuda", i)
        x = torch.rand(B, 3, 224, 224, generator=g).to(d).contiguous(memory_format=torch.channels_last)
        y = torch.zeros(B, 1000, device=d)
        y[torch.arange(B), torch.randint(0, 1000, (B,), generator=g).to(d)] = 1.0
        per_dev.append(DataSet(x.to(net.compute_dtype), y))
    pw = (ParallelWrapper.Builder(net).workers(N).inProcess(True).prefetchBuffer(2 * N)
          .trainingMode(TrainingMode.SHARED_GRADIENTS).build())

    def sync():
        for i in range(N):
            torch.cuda.synchronize(i)
    t_w = time.perf_counter()
    pw.fit([per_dev[i % N] for i in range(N * max(1, args.warmup))], 1)
    sync()
    print(f"[bench] in-process warmup done, {time.perf_counter() - t_w:.1f}s", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    pw.fit([per_dev[i % N] for i in range(N * args.steps)], 1)
    sync()
    elapsed = time.perf_counter() - t0
    ms = elapsed / args.steps * 1000.0
    ips = B * N * args.steps / elapsed
    model_name = "ResNet-50 (DL4J zoo ResNet50 graph)" if args.variant == "dl4j" else "ResNet-50 (canonical)"
    print(json.dumps({
        "metric": "images/sec (whole node) ResNet-50 training at 1/2/4/8 MI355X",
        "value": round(ips, 2), "unit": "images/sec", "n_gpus": N, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (random 224x224x3 images, one-hot labels; random-init weights)",
        "config": {"model": model_name, "variant": args.variant, "global_batch": B * N, "per_gpu_batch": B,
                   "seq_len": None, "image_size": 224, "parallelism": f"dp{N} (in-process threads)",
                   "comm": "rccl (ncclCommInitAll)",
                   "updater": "RmsProp(0.1,0.96,1e-3) + l1 1e-7 + l2 5e-5 (fused HIP updater)",
                   "hip_graph": bool(use_graph and getattr(net, "_hipgraph", None) is not None),
                   "kernel_db": _kernel_db(),
                   "final_score": net.score(), **memory_report(dev0)},
    }), flush=True)


if __name__ == "__main__":
    main()
