"""Process-group plumbing: one process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm,
carried over xGMI between the 8 MI355X of a node); gloo for CPU tests.

Replaces the reference's in-JVM multi-thread averaging (Nd4j.averageAndPropagate,
PW:ParallelWrapper.java:316-376) and its Spark/Aeron transports.
"""
import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(backend=None, timeout_s=600):
    """Initialise the default process group from torchrun env vars. Returns (world, rank, local_rank, device)."""
    world, rank, local = env_world()
    if torch.cuda.is_available():
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a failed/hung RCCL collective aborts the communicator and raises instead of hanging
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if backend is None:
            # DL4J_AMD_DIST_BACKEND=gloo rehearses multi-rank runs on one GPU (RCCL needs one GPU per rank)
            backend = os.environ.get("DL4J_AMD_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return world, rank, local, device


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def world_size():
    return dist.get_world_size() if is_dist() else 1


def rank():
    return dist.get_rank() if is_dist() else 0


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x):
    if not is_dist():
        return x
    t = torch.tensor([float(x)], dtype=torch.float64,
                     device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
