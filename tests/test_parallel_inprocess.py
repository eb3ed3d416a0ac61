"""In-process ParallelWrapper (parallel/inprocess.py: one host thread per device, streaming round-robin feed) over
the host loopback communicator, and world-4 gloo runs of the process-per-device path. The reference semantics are
computed in one process (reference: PW:ParallelWrapper.java:316-376, :467-565; DefaultTrainer.java:254-311)."""
import socket

import pytest
import torch
import torch.multiprocessing as mp

import _dist_workers as W


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pw(net, workers, **kw):
    from deeplearning4j_amd.parallel import ParallelWrapper, TrainingMode
    b = ParallelWrapper.Builder(net).workers(workers).inProcess(True)
    if kw.get("averaging"):
        b.trainingMode(TrainingMode.AVERAGING).averagingFrequency(kw["averaging"]).averageUpdaters(True)
    if "prefetch" in kw:
        b.prefetchBuffer(kw["prefetch"])
    return b.build()


def test_inprocess_shared_gradients_equals_large_batch():
    from deeplearning4j_amd import Adam, DataSet
    net = W.make_net(Adam(0.01))
    batches = W.make_batches(12, 8)
    _pw(net, 4).fit(batches, 2)
    ref = W.make_net(Adam(0.01))
    for _ in range(2):
        for i in range(0, 12, 4):
            grp = batches[i:i + 4]
            ref.fit(DataSet(torch.cat([b.features for b in grp]), torch.cat([b.labels for b in grp])))
    assert torch.allclose(net.params(), ref.params(), atol=1e-5), (net.params() - ref.params()).abs().max()
    assert net.getIterationCount() == 6


def test_inprocess_averaging_every_three_rounds_matches_reference():
    from deeplearning4j_amd import Adam
    net = W.make_net(Adam(0.01))
    batches = W.make_batches(12, 8)
    _pw(net, 4, averaging=3).fit(batches, 2)
    want = W.simulate_averaging(lambda: W.make_net(Adam(0.01)), batches, 4, 3, 2)
    assert torch.allclose(net.params(), want, atol=1e-6), (net.params() - want).abs().max()


def test_inprocess_streams_a_long_iterator_with_bounded_memory():
    """4k batches through a generator-backed iterator: the wrapper never holds more than prefetchBuffer + 2 x workers
    batches (queued + in training + the round being handed out; the round-1/2 launcher materialised the whole
    iterator first)."""
    from deeplearning4j_amd import Sgd
    from deeplearning4j_amd.datasets.dataset import DataSet

    class Gen:
        def __init__(self, n):
            self.n, self.i, self.made = n, 0, 0

        def reset(self):
            self.i = 0

        def hasNext(self):
            return self.i < self.n

        def next(self):
            self.i += 1
            self.made += 1
            x = torch.randn(2, 5)
            y = torch.zeros(2, 3)
            y[:, 0] = 1
            return DataSet(x, y)
    net = W.make_net(Sgd(0.01))
    it = Gen(4000)
    pw = _pw(net, 4, prefetch=8)
    pw.fit(it, 1)
    assert it.made == 4000
    assert pw._inproc.max_live <= 8 + 2 * 4, pw._inproc.max_live
    assert net.getIterationCount() == 1000


def test_inprocess_worker_failure_propagates_without_hanging():
    from deeplearning4j_amd import Adam, DataSet
    net = W.make_net(Adam(0.01))
    batches = W.make_batches(8, 8)
    batches[6] = DataSet(torch.randn(8, 7), batches[6].labels)        # wrong feature width -> worker 2 fails
    with pytest.raises(RuntimeError, match="worker 2"):
        _pw(net, 4).fit(batches, 1)


def test_inprocess_listeners_fire_on_the_callers_model():
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.optimize.listeners import CollectScoresIterationListener
    net = W.make_net(Adam(0.01))
    lst = CollectScoresIterationListener(1)
    net.setListeners(lst)
    _pw(net, 2).fit(W.make_batches(8, 8), 1)
    assert len(lst.getScoreVsIter()) == 4


def _run4(mode, tmp_path):
    path = str(tmp_path / f"{mode}.pt")
    mp.spawn(W.run_mode4, args=(4, _port(), mode, path), nprocs=4, join=True)
    return torch.load(path, weights_only=True)


def test_gloo_world4_averaging_every_three_rounds(tmp_path):
    from deeplearning4j_amd import Adam
    res = _run4("averaging3", tmp_path)
    ps = res["params"]
    for p in ps[1:]:
        assert torch.allclose(p, ps[0], atol=1e-6)
    want = W.simulate_averaging(lambda: W.make_net(Adam(0.01)), W.make_batches(12, 8), 4, 3, 2)
    assert torch.allclose(ps[0], want, atol=1e-5), (ps[0] - want).abs().max()


def test_gloo_world4_encoded_updates(tmp_path):
    from deeplearning4j_amd import Adam
    res = _run4("encoded", tmp_path)
    ps = res["params"]
    for p in ps[1:]:
        assert torch.equal(p, ps[0])                 # every rank applies the same decoded sum of 4 messages
    assert not torch.allclose(ps[0], W.make_net(Adam(0.5)).params())


def test_inprocess_partial_round_trains_on_first_workers():
    """10 batches over 4 workers: 2 full rounds + a trailing round of 2. The reference (PW:ParallelWrapper.java:
    514-578) trains the trailing batches on the first ``locker`` workers; here the idle replicas contribute zero
    gradients to the round's all-reduce and the update divides by the 2 trained batches, i.e. the trailing round is
    the large-batch step over those 2 batches, and every replica ends identical."""
    from deeplearning4j_amd import Adam, DataSet
    net = W.make_net(Adam(0.01))
    batches = W.make_batches(10, 8)
    pw = _pw(net, 4)
    pw.fit(batches, 1)
    ref = W.make_net(Adam(0.01))
    for grp in (batches[0:4], batches[4:8], batches[8:10]):
        ref.fit(DataSet(torch.cat([b.features for b in grp]), torch.cat([b.labels for b in grp])))
    assert torch.allclose(net.params(), ref.params(), atol=1e-5), (net.params() - ref.params()).abs().max()
    assert net.getIterationCount() == 3


def test_inprocess_fewer_batches_than_workers():
    """An epoch with fewer batches than workers still trains (the round-3 wrapper dropped the whole round)."""
    from deeplearning4j_amd import Sgd
    net = W.make_net(Sgd(0.1))
    before = net.params().clone()
    _pw(net, 4, averaging=1).fit(W.make_batches(3, 8), 1)
    assert not torch.allclose(net.params(), before)


def test_devices_for_refuses_mixed_gpu_cpu_replicas(monkeypatch):
    """A model on a GPU with fewer visible GPUs than workers is an error, not N-1 CPU replicas."""
    from deeplearning4j_amd.parallel import inprocess

    class M:
        device = torch.device("cuda", 0)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    with pytest.raises(RuntimeError, match="visible GPUs"):
        inprocess.devices_for(4, M())

    class C:
        device = torch.device("cpu")
    assert inprocess.devices_for(4, C()) == [torch.device("cpu")] * 4


def test_inprocess_short_trailing_batch_keeps_replicas_identical():
    """a short last batch (3 examples instead of 8) in a partial round. Every replica — trained or idle —
    divides the summed gradient by the round's total example count (8 + 3), so all replicas apply the same update
    and equal the large-batch step over the round's 11 examples."""
    from deeplearning4j_amd import Adam, DataSet
    net = W.make_net(Adam(0.01))
    batches = W.make_batches(10, 8)
    last = batches[9]
    batches[9] = DataSet(last.features[:3].clone(), last.labels[:3].clone())
    pw = _pw(net, 4)
    pw.fit(batches, 1)
    models = pw._inproc.models
    for m in models[1:]:
        assert torch.equal(m.params(), models[0].params())
    ref = W.make_net(Adam(0.01))
    for grp in (batches[0:4], batches[4:8], batches[8:10]):
        ref.fit(DataSet(torch.cat([b.features for b in grp]), torch.cat([b.labels for b in grp])))
    assert torch.allclose(net.params(), ref.params(), atol=1e-5), (net.params() - ref.params()).abs().max()


def test_inprocess_unequal_batches_in_full_round():
    """A full round whose batches differ in size: the divisor is the round's example total on every replica."""
    from deeplearning4j_amd import Sgd, DataSet
    net = W.make_net(Sgd(0.1))
    b = W.make_batches(2, 8)
    b[1] = DataSet(b[1].features[:5].clone(), b[1].labels[:5].clone())
    pw = _pw(net, 2)
    pw.fit(b, 1)
    ms = pw._inproc.models
    assert torch.equal(ms[0].params(), ms[1].params())
    ref = W.make_net(Sgd(0.1))
    ref.fit(DataSet(torch.cat([x.features for x in b]), torch.cat([x.labels for x in b])))
    assert torch.allclose(net.params(), ref.params(), atol=1e-6), (net.params() - ref.params()).abs().max()


def test_inprocess_eight_workers_bucketed_equals_large_batch():
    """8 worker threads (the 8-GPU node's thread-per-device layout) through the real in-process code path: round-robin
    feed, per-worker replicas, the bucketed all-reduce accumulator with a small bucket size (several buckets issued
    during backward) over the host loopback communicator. Every round equals one large-batch step over the round's 8
    batches, and all 8 replicas end bit-identical."""
    from deeplearning4j_amd import Adam, DataSet
    from deeplearning4j_amd.parallel import ParallelWrapper
    net = W.make_net(Adam(0.01))
    batches = W.make_batches(16, 4)
    pw = ParallelWrapper.Builder(net).workers(8).inProcess(True).bucketSizeMB(1e-4).build()
    pw.fit(batches, 1)
    ms = pw._inproc.models
    assert len(ms) == 8
    for m in ms[1:]:
        assert torch.equal(m.params(), ms[0].params())
    acc = ms[0].gradientsAccumulator
    assert acc._buckets is not None and len(acc._buckets) > 1, "expected several gradient buckets"
    ref = W.make_net(Adam(0.01))
    for i in range(0, 16, 8):
        grp = batches[i:i + 8]
        ref.fit(DataSet(torch.cat([b.features for b in grp]), torch.cat([b.labels for b in grp])))
    assert torch.allclose(net.params(), ref.params(), atol=1e-5), (net.params() - ref.params()).abs().max()
