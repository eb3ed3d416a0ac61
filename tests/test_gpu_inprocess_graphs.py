"""Concurrent HIP-graph capture by several host threads (the in-process ParallelWrapper's thread-per-GPU design,
parallel/inprocess.py): each thread captures and replays its own network's training step, with thread-local
capture mode, per-thread capture streams and graph slots (nn/hipgraph.py, ops/native.py GRAPH_SLOT). On this
one-GPU box both threads share cuda:0, so the captures and replays really run at the same time on one device; the
result must be bitwise the sequential one (deterministic conv weight gradients)."""
import threading

import pytest
import torch

import _dist_workers as W

pytestmark = pytest.mark.gpu


def _train(seed, batches, start=None, out=None, idx=None, errs=None):
    try:
        from deeplearning4j_amd.nn.conf import DataType
        torch.cuda.set_device(0)
        # each worker issues on a stream of its own, as the in-process wrapper's workers do on their own devices
        # (per-stream scratch buffers, ops/native.py _scratch)
        with torch.cuda.stream(torch.cuda.Stream(0)):
            net = W.make_cg(seed=seed, device=torch.device("cuda", 0), dtype=DataType.BFLOAT16)
            net.enableHipGraphs(True, warmup=1)
            if start is not None:
                start.wait()
            for ds in batches:
                net.fit([ds.features.cuda()], [ds.labels.cuda()])
            torch.cuda.current_stream().synchronize()
        assert net._hipgraph is not None and net._hipgraph.ok, "step was not captured"
        if out is not None:
            out[idx] = net.params().detach().clone()
        return net.params().detach().clone()
    except BaseException as e:   # noqa: BLE001
        if errs is not None:
            errs.append(e)
        raise


def test_two_threads_capture_and_replay_concurrently(monkeypatch):
    monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
    batches = W.make_image_batches(6, 8)
    ref = [_train(3, batches), _train(5, batches)]
    out = [None, None]
    errs = []
    start = threading.Barrier(2)
    ts = [threading.Thread(target=_train, args=(s, batches, start, out, i, errs)) for i, s in enumerate((3, 5))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    for i in range(2):
        assert out[i] is not None
        assert torch.equal(out[i], ref[i]), (out[i] - ref[i]).abs().max()


def test_rccl_buckets_run_on_the_comm_stream(monkeypatch):
    """The direct-RCCL accumulator forks each bucket onto its own high-priority stream and joins it before the
    update (parallel/accumulation.py); world 1, so the result equals plain training."""
    monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.parallel.accumulation import AllReduceGradientsAccumulator
    from deeplearning4j_amd.parallel.rccl import RcclComm
    batches = W.make_image_batches(5, 8)
    ref = _train(3, batches)
    c = RcclComm.init_all([0])[0]
    try:
        net = W.make_cg(seed=3, device=torch.device("cuda", 0), dtype=DataType.BFLOAT16)
        acc = AllReduceGradientsAccumulator(bucket_mb=0.0005, force=True, comm=c)
        net.setGradientsAccumulator(acc)
        net.enableHipGraphs(True, warmup=1)
        for ds in batches:
            net.fit([ds.features.cuda()], [ds.labels.cuda()])
        torch.cuda.synchronize()
        assert net._hipgraph is not None and net._hipgraph.ok
        assert 0 in acc._comm_streams and acc._comm_streams[0] != torch.cuda.current_stream(0)
        assert torch.allclose(net.params(), ref, atol=1e-6, rtol=0), (net.params() - ref).abs().max()
    finally:
        c.destroy()


def test_inprocess_replicas_inherit_graph_mode():
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.parallel.inprocess import _replica
    net = W.make_net(Adam(0.01))
    net2 = type(net)(net.conf)
    net2.init(net.params().clone(), device=torch.device("cuda", 0))
    net2.enableHipGraphs(True, warmup=3)
    r = _replica(net2, torch.device("cuda", 0))
    assert getattr(r, "_hipgraph_enabled", False) and r._hipgraph_warmup == 3
