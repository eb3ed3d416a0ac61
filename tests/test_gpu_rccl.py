"""Direct RCCL communicators (parallel/rccl.py) on the one GPU of the test box: ncclCommInitAll / ncclCommInitRank
world-1 cliques, every collective against its definition, a collective captured into a HIP graph, and the
bucketed gradient accumulator + in-process trainer running on an RcclComm (forced on at world 1, where the
all-reduce is an identity, so training must equal plain single-GPU training bit for bit in deterministic mode)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

import _dist_workers as W

pytestmark = pytest.mark.gpu


def _comm():
    from deeplearning4j_amd.parallel.rccl import RcclComm
    return RcclComm.init_all([0])[0]


def test_rccl_library_is_torchs_copy():
    from deeplearning4j_amd.parallel import rccl
    assert rccl.available()
    assert os.path.dirname(torch.__file__) in rccl.library_path()


def test_init_all_world1_collectives():
    c = _comm()
    try:
        assert c.nranks == 1 and c.rank == 0
        x = torch.randn(1000, device="cuda")
        y = x.clone()
        c.all_reduce(y, "sum")
        c.all_reduce(y, "avg")
        c.broadcast(y, 0)
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        for dt in (torch.bfloat16, torch.float16, torch.float64, torch.int32):
            t = (torch.arange(64, device="cuda") % 7).to(dt)
            out = torch.empty_like(t)
            c.all_reduce(t, "max", out=out)
            torch.cuda.synchronize()
            assert torch.equal(out, t)
        g = torch.empty(1000, device="cuda")
        c.all_gather(x, g)
        rs = torch.empty(1000, device="cuda")
        c.reduce_scatter(x, rs)
        torch.cuda.synchronize()
        assert torch.equal(g, x) and torch.equal(rs, x)
        assert c.async_error() == 0
    finally:
        c.destroy()


def test_rccl_allreduce_captured_in_hip_graph():
    c = _comm()
    try:
        x = torch.zeros(4096, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            x.add_(1.0)
            c.all_reduce(x)                     # warm up outside the capture
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            x.mul_(2.0)
            c.all_reduce(x, "sum")
            x.add_(1.0)
        x.fill_(1.0)
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        assert torch.allclose(x, torch.full_like(x, 7.0))   # (1*2+1)*2+1
    finally:
        c.destroy()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_from_process_group_world1():
    from deeplearning4j_amd.parallel.rccl import RcclComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        c = RcclComm.from_process_group()
        x = torch.randn(333, device="cuda", dtype=torch.bfloat16)
        y = x.clone()
        c.all_reduce(y)
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        c.destroy()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("comm_dtype", [None, torch.bfloat16])
def test_accumulator_on_rccl_comm_in_hip_graph(comm_dtype, monkeypatch):
    """Graph-captured bf16 CG training with every gradient bucket all-reduced through an RcclComm on the step's
    stream; deterministic conv weight gradients, so the result equals plain training (fp32 wire) or stays within
    the bf16 wire rounding."""
    monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.parallel.accumulation import AllReduceGradientsAccumulator
    batches = W.make_image_batches(5, 8)

    def train(acc):
        net = W.make_cg(device=torch.device("cuda", 0), dtype=DataType.BFLOAT16)
        if acc is not None:
            net.setGradientsAccumulator(acc)
        net.enableHipGraphs(True, warmup=1)
        for ds in batches:
            net.fit([ds.features.cuda()], [ds.labels.cuda()])
        torch.cuda.synchronize()
        return net
    ref = train(None)
    c = _comm()
    try:
        acc = AllReduceGradientsAccumulator(bucket_mb=0.0005, dtype=comm_dtype, force=True, comm=c)
        assert acc.active and acc.capturable() and acc.world_size == 1
        net = train(acc)
        assert net._hipgraph is not None and net._hipgraph.ok
        assert len(acc._buckets) > 2
        if comm_dtype is None:
            assert torch.allclose(net.params(), ref.params(), atol=1e-6, rtol=0)
        else:
            assert torch.allclose(net.params(), ref.params(), atol=5e-3)
            assert acc._staging is not None and len(acc._staging) == len(acc._buckets)
    finally:
        c.destroy()


def test_inprocess_trainer_on_gpu_with_rccl(monkeypatch):
    """The thread-per-device trainer with its ncclCommInitAll communicator (one worker on this box)."""
    monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.parallel import ParallelWrapper
    from deeplearning4j_amd.parallel.accumulation import AllReduceGradientsAccumulator
    from deeplearning4j_amd.parallel.inprocess import InProcessTrainer
    from deeplearning4j_amd.parallel.rccl import RcclComm
    batches = W.make_batches(6, 8)
    import copy
    proto = W.make_net(Adam(0.01))
    ref = type(proto)(copy.deepcopy(proto.conf))     # separate confs: the conf carries the iteration count
    ref.init(device=torch.device("cuda", 0))
    net = type(proto)(copy.deepcopy(proto.conf))
    net.init(ref.params().clone(), device=torch.device("cuda", 0))
    for ds in batches:
        ref.fit(ds)
    pw = ParallelWrapper.Builder(net).workers(1).build()
    comms = RcclComm.init_all([0])
    tr = InProcessTrainer(pw, devices=[torch.device("cuda", 0)], comms=comms)
    for m in tr.models:
        m.gradientsAccumulator = AllReduceGradientsAccumulator(comm=comms[0], force=True)
    tr.fit(batches, 1)
    torch.cuda.synchronize()
    assert torch.allclose(net.params(), ref.params(), atol=1e-6), (net.params() - ref.params()).abs().max()
    comms[0].destroy()
