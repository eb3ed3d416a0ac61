"""RCCL (torch.distributed nccl backend) on the one GPU available: the data-parallel gradient path initialised for
real, with the bucketed all-reduce accumulator forced on (world_size 1 all-reduces are identities, so the result
must equal a plain single-GPU run) and the whole training step — collectives included — captured in HIP graphs.
Multi-rank behaviour of the same code is covered by the gloo tests in test_parallel.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

import _dist_workers as W

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(net, batches, acc=None):
    if acc is not None:
        net.setGradientsAccumulator(acc)
    net.enableHipGraphs(True, warmup=1)
    for ds in batches:
        net.fit([ds.features.cuda()], [ds.labels.cuda()])
    torch.cuda.synchronize()
    return net


@pytest.mark.parametrize("comm,bf16net", [(None, False), (torch.bfloat16, False), (None, True)])
def test_nccl_world1_allreduce_in_hip_graph(comm, bf16net, monkeypatch):
    """bf16net: the conv weight gradients run on the overlap stream (ops/side_stream.py) inside the captured graph,
    joined before each RCCL bucket. DL4J_AMD_DETERMINISTIC=1 takes the conv weight gradient off float atomics, so
    the world-1 all-reduce run must reproduce the single-GPU run to fp32 rounding, not merely to an lr-sized bound."""
    monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
    from deeplearning4j_amd.parallel.accumulation import AllReduceGradientsAccumulator
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        batches = W.make_image_batches(5, 8)
        from deeplearning4j_amd.nn.conf import DataType
        dt = DataType.BFLOAT16 if bf16net else None
        ref = _train(W.make_cg(device=torch.device("cuda", 0), dtype=dt), batches)
        net = W.make_cg(device=torch.device("cuda", 0), dtype=dt)
        acc = AllReduceGradientsAccumulator(bucket_mb=0.0005, dtype=comm, force=True)
        assert acc.active and acc.capturable()
        from deeplearning4j_amd.ops import side_stream
        n0 = side_stream.LAUNCHES[0]
        net = _train(net, batches, acc)
        if bf16net:
            assert side_stream.LAUNCHES[0] > n0, "conv weight gradient never ran on the overlap stream"
        assert net._hipgraph is not None and net._hipgraph.ok, "DP step was not captured into a HIP graph"
        assert len(acc._buckets) > 2
        if bf16net:
            assert torch.allclose(net.params(), ref.params(), atol=1e-5, rtol=0)
        elif comm is None:
            assert torch.allclose(net.params(), ref.params(), atol=1e-6)
        else:
            assert torch.allclose(net.params(), ref.params(), atol=5e-3)
            assert not torch.equal(net.params(), ref.params())     # the bf16 wire format is really used
    finally:
        dist.destroy_process_group()
