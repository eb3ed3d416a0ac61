"""Data-parallel training and parallel inference (reference PW tests: ParallelWrapperTest.java,
ParallelInferenceTest.java; NN: EncodedGradientsAccumulatorTest.java, threshold codec tests).
Multi-process paths run with gloo, world_size 2, on CPU (the RCCL path is the same code with backend nccl)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from deeplearning4j_amd.ops import compression as C

import _dist_workers as W


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(mode, tmp_path):
    path = str(tmp_path / f"{mode}.pt")
    mp.spawn(W.run_mode, args=(2, _port(), mode, path), nprocs=2, join=True)
    return torch.load(path, weights_only=True)


def test_threshold_codec_cpu():
    g = torch.Generator().manual_seed(0)
    r = torch.randn(10000, generator=g) * 1e-3
    r0 = r.clone()
    thr = 1.5e-3
    n_expected = int((r.abs() >= thr).sum())
    assert C.threshold_count(r, thr) == n_expected
    msg = C.threshold_encode(r, thr, capacity=r.numel())
    assert int(msg[0]) == n_expected and int(msg[3]) == C.SPARSE
    idx = msg[4:4 + n_expected].long()
    assert torch.equal(idx.abs() - 1, (r0.abs() >= thr).nonzero().reshape(-1))     # in-order
    dec = C.decode(msg, torch.zeros_like(r))
    assert torch.allclose(dec + r, r0, atol=1e-7)          # decoded + residual == original
    # bitmap
    r2 = r0.clone()
    bm = C.bitmap_encode(r2, thr)
    assert bm.numel() == C.bitmap_capacity(r0.numel()) and int(bm[0]) == n_expected
    dec2 = C.decode(bm, torch.zeros_like(r0))
    assert torch.allclose(dec2, dec) and torch.allclose(r2, r)
    # capacity limit: only the first entries are emitted, the rest stay in the residual
    r3 = r0.clone()
    m3 = C.threshold_encode(r3, thr, capacity=5)
    assert int(m3[0]) == 5
    assert torch.allclose(C.decode(m3, torch.zeros_like(r0)) + r3, r0, atol=1e-7)


def test_encoding_handler_switches_modes():
    from deeplearning4j_amd.parallel import EncodingHandler
    h = EncodingHandler(threshold=1e-2)
    sparse = torch.zeros(3200)
    sparse[::100] = 0.05
    m = h.encodeUpdates(sparse.clone())
    assert int(m[3]) == C.BITMAP          # starts in bitmap mode
    assert not h.bitmapMode               # ...and switches to sparse because few values were encoded
    m = h.encodeUpdates(sparse.clone())
    assert int(m[3]) == C.SPARSE
    dense = torch.full((3200,), 0.05)
    m = h.encodeUpdates(dense)
    assert int(m[3]) == C.BITMAP and h.bitmapMode


def test_parallel_wrapper_shared_gradients_equals_large_batch(tmp_path):
    res = _run("shared", tmp_path)
    p0, p1 = res["params"]
    assert torch.equal(p0, p1)                  # replicas identical
    # single process, global batch = concat of the two ranks' batches, same number of steps
    from deeplearning4j_amd import Adam, DataSet
    net = W.make_net(Adam(0.01))
    batches = W.make_batches(8, 8)
    for _ in range(2):
        for i in range(0, 8, 2):
            a, b = batches[i], batches[i + 1]
            net.fit(DataSet(torch.cat([a.features, b.features]), torch.cat([a.labels, b.labels])))
    assert torch.allclose(net.params(), p0, atol=1e-5), (net.params() - p0).abs().max()
    assert res["iters"] == 8


def test_parallel_wrapper_averaging(tmp_path):
    res = _run("averaging", tmp_path)
    p0, p1 = res["params"]
    assert torch.allclose(p0, p1, atol=1e-6)
    init = W.make_net(__import__("deeplearning4j_amd").Adam(0.01)).params()
    assert not torch.allclose(p0, init)


def test_parallel_wrapper_encoded_updates(tmp_path):
    res = _run("encoded", tmp_path)
    p0, p1 = res["params"]
    assert torch.equal(p0, p1)                  # every rank applies the same decoded sum
    init = W.make_net(__import__("deeplearning4j_amd").Adam(0.5)).params()
    assert not torch.allclose(p0, init)


def test_parallel_inference_batched_and_sequential():
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.parallel import InferenceMode, ParallelInference
    net = W.make_net(Adam(0.01))
    xs = [torch.randn(3, 5) for _ in range(12)]
    ref = [net.output(x) for x in xs]
    for mode in (InferenceMode.BATCHED, InferenceMode.SEQUENTIAL):
        pi = ParallelInference.Builder(net).inferenceMode(mode).batchLimit(8).devices(
            [torch.device("cpu"), torch.device("cpu")]).build()
        futs = [pi.submit(x) for x in xs]
        outs = [f.result(timeout=60) for f in futs]
        pi.shutdown()
        for o, r in zip(outs, ref):
            assert torch.allclose(o, r, atol=1e-6)


@pytest.mark.skipif(os.environ.get("DL4J_AMD_SKIP_SLOW") == "1", reason="slow")
def test_wrapper_single_process_trains():
    from deeplearning4j_amd import Adam, ListDataSetIterator
    from deeplearning4j_amd.parallel import ParallelWrapper
    net = W.make_net(Adam(0.05))
    it = ListDataSetIterator(W.make_batches(4, 16), 16)
    s0 = net.score(W.make_batches(1, 64, seed=9)[0])
    ParallelWrapper.Builder(net).build().fit(it, 5)
    assert net.score(W.make_batches(1, 64, seed=9)[0]) < s0 + 0.5


@pytest.mark.parametrize("master", ["paramavg", "shared"])
def test_cluster_training_masters(tmp_path, master):
    """ParameterAveraging / Shared training masters across 2 gloo ranks: replicas end identical (rank 1 started
    from different weights), evaluation merges both shards (all 64 examples counted once)."""
    path = str(tmp_path / f"{master}.pt")
    mp.spawn(W.run_cluster, args=(2, _port(), master, path), nprocs=2, join=True)
    r = torch.load(path, weights_only=True)
    assert torch.allclose(r["params"][0], r["params"][1], atol=1e-6)
    assert r["n_eval"] == 64
    assert r["score"] == r["score"] and 0.0 <= r["acc"] <= 1.0
    if master == "paramavg":
        html = open(path + ".html").read()
        assert "fit" in html and "average" in html


def test_parallel_wrapper_main_cli(tmp_path):
    """ParallelWrapperMain: restore a model zip, train from an iterator factory, write the result."""
    import sys
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.parallel.main import main
    from deeplearning4j_amd.utils.model_serializer import ModelSerializer
    (tmp_path / "pwm_data.py").write_text(
        "import torch\nfrom deeplearning4j_amd import DataSet, ListDataSetIterator\n"
        "def make():\n    g = torch.Generator().manual_seed(0)\n    out = []\n"
        "    for _ in range(4):\n        x = torch.randn(8, 5, generator=g)\n        y = torch.zeros(8, 3)\n"
        "        y[:, 0] = 1\n        out.append(DataSet(x, y))\n    return ListDataSetIterator(out)\n")
    sys.path.insert(0, str(tmp_path))
    try:
        net = W.make_net(Adam(0.01))
        ModelSerializer.writeModel(net, str(tmp_path / "in.zip"), True)
        out = main(["--modelPath", str(tmp_path / "in.zip"), "--dataSetIteratorFactoryClazz", "pwm_data:make",
                    "--modelOutputPath", str(tmp_path / "out.zip"), "--epochs", "2"])
        assert out.getIterationCount() == 8
        re = ModelSerializer.restoreModel(str(tmp_path / "out.zip"))
        assert torch.allclose(re.params(), out.params())
    finally:
        sys.path.remove(str(tmp_path))


@pytest.mark.skipif(os.environ.get("DL4J_AMD_SKIP_SLOW") == "1", reason="slow")
@pytest.mark.parametrize("in_process", [True, False])
def test_parallel_wrapper_in_process_workers_spawn(in_process):
    """ParallelWrapper.Builder(net).workers(2).build().fit(data) from ONE plain process — worker threads (host
    loopback here, RCCL communicators on GPUs) or two child processes fed over sockets (gloo here, RCCL on GPUs) —
    train synchronously and the caller's model ends up equal to single-process training on the concatenated
    batches (the reference's in-JVM ParallelWrapper contract, PW:ParallelWrapper.java:467-565)."""
    from deeplearning4j_amd import Adam, DataSet
    from deeplearning4j_amd.parallel import ParallelWrapper
    batches = W.make_batches(8, 8)
    net = W.make_net(Adam(0.01))
    ParallelWrapper.Builder(net).workers(2).inProcess(in_process).build().fit(batches, 2)   # a plain list source
    ref = W.make_net(Adam(0.01))
    for _ in range(2):
        for i in range(0, 8, 2):
            a, b = batches[i], batches[i + 1]
            ref.fit(DataSet(torch.cat([a.features, b.features]), torch.cat([a.labels, b.labels])))
    assert torch.allclose(net.params(), ref.params(), atol=1e-5), (net.params() - ref.params()).abs().max()
    assert net.getIterationCount() == 8
    assert net.score() == net.score() and net.score() > 0      # the trained replica's score, not a stale one


def test_spawned_worker_failure_is_reported():
    """A child that dies (bad batch) makes fit raise promptly instead of blocking on the other rank's collective."""
    from deeplearning4j_amd import Adam, DataSet
    from deeplearning4j_amd.parallel import ParallelWrapper
    batches = W.make_batches(4, 8)
    batches[3] = DataSet(torch.randn(8, 7), batches[3].labels)
    net = W.make_net(Adam(0.01))
    with pytest.raises(RuntimeError, match="worker"):
        ParallelWrapper.Builder(net).workers(2).inProcess(False).build().fit(batches, 1)


def test_cg_shared_gradients_bucketed_equals_large_batch(tmp_path):
    """ComputationGraph DP-2 with several gradient buckets issued during backward == one process at 2x batch."""
    from deeplearning4j_amd import DataSet
    path = str(tmp_path / "cg.pt")
    mp.spawn(W.run_cg_shared, args=(2, _port(), path), nprocs=2, join=True)
    res = torch.load(path, weights_only=True)
    p0, p1 = res["params"]
    assert torch.equal(p0, p1)
    assert res["nbuckets"] > 2
    net = W.make_cg()
    b = W.make_image_batches(6, 4)
    for i in range(0, 6, 2):
        net.fit(DataSet(torch.cat([b[i].features, b[i + 1].features]), torch.cat([b[i].labels, b[i + 1].labels])))
    assert torch.allclose(net.params(), p0, atol=1e-5), (net.params() - p0).abs().max()


@pytest.mark.parametrize("bucket_mb", ["32", "0.00002"])
def test_samediff_data_parallel_equals_large_batch(tmp_path, monkeypatch, bucket_mb):
    """SameDiff DP-2 (gloo): each rank fits half of every batch, gradients averaged across ranks before the fused
    update == one process fitting the whole batch. With tiny buckets every variable is its own bucket, issued from
    the reverse pass the moment its gradient is final (samediff _SDGradBuckets)."""
    monkeypatch.setenv("DL4J_AMD_BUCKET_MB", bucket_mb)
    path = str(tmp_path / "sd.pt")
    mp.spawn(W.run_samediff_dp, args=(2, _port(), path), nprocs=2, join=True)
    res = torch.load(path, weights_only=True)
    p0, p1 = res["params"]
    if bucket_mb != "32":
        assert res["nbuckets"] > 2
    assert torch.equal(p0, p1)
    sd = W.make_samediff()
    for ds in W.samediff_batches():
        sd.fit(ds)
    ref = torch.cat([v.value.reshape(-1) for v in sd.trainableVariables()])
    assert torch.allclose(ref, p0, atol=1e-5), (ref - p0).abs().max()
