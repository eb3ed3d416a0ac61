"""BasicGradientsAccumulator, FancyBlockingQueue and the encoded accumulator's buffer / fan-out contract.

Ports of the reference's own tests:
  * deeplearning4j-core/src/test/java/org/deeplearning4j/parallelism/FancyBlockingQueueTests.java (testFancyQueue1-4);
  * deeplearning4j-nn/src/test/java/org/deeplearning4j/optimize/solvers/accumulation/EncodedGradientsAccumulatorTest
    .java (testStore1, testEncodingLimits1);
plus a ParallelWrapper CUSTOM-mode run with a BasicGradientsAccumulator shared by 4 in-process workers (CPU)."""
import random
import threading
import time

import pytest
import torch

import _dist_workers as W


def _queue_with_512(consumers):
    from deeplearning4j_amd.parallel import FancyBlockingQueue
    q = FancyBlockingQueue(512, consumers)
    f = 0
    for x in range(512):
        q.add(x)
        f += x
    assert q.size() == 512
    return q, f


def _drain(q, nthreads, sleep=False):
    total = [0]
    lock = threading.Lock()

    def run():
        while not q.isEmpty():
            i = q.poll()
            with lock:
                total[0] += i
            if sleep:
                time.sleep(random.randint(1, 4) / 1000.0)
    ts = [threading.Thread(target=run) for _ in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    return total[0]


def test_fancy_queue_four_consumers_each_see_everything():          # testFancyQueue1
    q, f = _queue_with_512(4)
    q.registerConsumers(4)
    assert _drain(q, 4) == 4 * f
    assert q.size() == 0                                            # dropped once all 4 consumers took them


def test_fancy_queue_four_consumers_with_jitter():                  # testFancyQueue2
    q, f = _queue_with_512(4)
    q.registerConsumers(4)
    assert _drain(q, 4, sleep=True) == 4 * f


def test_fancy_queue_single_consumer():                             # testFancyQueue3
    q, f = _queue_with_512(4)
    q.registerConsumers(1)
    assert _drain(q, 1) == f


def test_fancy_queue_fallback_single_consumer_mode():               # testFancyQueue4
    q, f = _queue_with_512(4)
    q.fallbackToSingleConsumerMode(True)
    assert _drain(q, 1) == f


def test_fancy_queue_order_and_late_elements():
    from deeplearning4j_amd.parallel import FancyBlockingQueue
    q = FancyBlockingQueue(consumers=2)
    q.registerConsumers(2)
    seen = {0: [], 1: []}
    start = threading.Barrier(2)

    def run(k):
        start.wait()
        while len(seen[k]) < 10:
            e = q.poll(timeout=0.5)
            if e is not None:
                seen[k].append(e)
    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for i in range(10):
        q.put(i)
    for t in ts:
        t.join(timeout=30)
    assert seen[0] == list(range(10)) and seen[1] == list(range(10))


def test_encoded_store_and_fanout():                                # testStore1
    from deeplearning4j_amd.parallel.encoded import EncodedGradientsAccumulator, EncodingHandler
    num_params = 100000
    handler = EncodingHandler(1e-3)
    for workers in (2, 4, 8):
        size = EncodedGradientsAccumulator.getOptimalBufferSize(num_params, workers, 2)
        assert size == ((num_params // 16) + 65536) * workers * 2 * 4
        acc = EncodedGradientsAccumulator(handler, parties=workers, bufferSize=size, queueSize=2)
        for e in range(10, 400, 7):
            g = torch.zeros(num_params)
            g[:e] = 2e-3
            acc.receiveUpdate(handler.encodeUpdates(g))
            assert all(m.size() == 1 for m in acc.messages)         # replicated into every party's queue
            for m in acc.messages:
                m.clear()                                           # "just purge updates, like they were consumed"


def test_encoded_message_larger_than_buffer_share_is_refused():
    from deeplearning4j_amd.parallel.encoded import EncodedGradientsAccumulator
    acc = EncodedGradientsAccumulator(1e-3, parties=2, bufferSize=1024, queueSize=4)
    with pytest.raises(MemoryError, match="Not enough memory"):
        acc.receiveUpdate(torch.zeros(1024, dtype=torch.int32))


def test_encoding_limits():                                          # testEncodingLimits1
    from deeplearning4j_amd.parallel.encoded import EncodingHandler
    num_params = 100000
    handler = EncodingHandler(1e-3)
    for e in range(10, num_params // 5, 997):
        g = torch.zeros(num_params)
        g[:e] = 2e-3
        enc = handler.encodeUpdates(g)
        assert enc.numel() < num_params // 16 + 6, (e, int(enc[3]), enc.numel())


def test_basic_accumulator_sums_parties_updates():
    """storeUpdate from 3 threads, then applyUpdate: every party's params move by the SUM of the 3 candidates, and
    ``updates`` is cleared afterwards (BasicGradientsAccumulator.java:85-157)."""
    from deeplearning4j_amd.optimize.solvers import NegativeGradientStepFunction
    from deeplearning4j_amd.parallel import BasicGradientsAccumulator
    acc = BasicGradientsAccumulator(3)
    cands = [torch.full((5,), float(i + 1)) for i in range(3)]
    params = [torch.zeros(5) for _ in range(3)]

    def run(i):
        acc.storeUpdate(cands[i])
        acc.applyUpdate(NegativeGradientStepFunction(), params[i], None)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    for p in params:
        assert torch.equal(p, torch.full((5,), -6.0))
    assert torch.equal(acc.updates, torch.zeros(5))
    assert acc.ownCounter == 1 and acc.extCounter == 1


def test_basic_accumulator_alpha_overload():
    from deeplearning4j_amd.optimize.solvers import NegativeDefaultStepFunction
    from deeplearning4j_amd.parallel import BasicGradientsAccumulator
    acc = BasicGradientsAccumulator(1)
    p = torch.zeros(4)
    acc.storeUpdate(torch.ones(4))
    acc.applyUpdate(NegativeDefaultStepFunction(), p, None, 0.5)
    assert torch.equal(p, torch.full((4,), -0.5))


def test_parallel_wrapper_custom_basic_accumulator_in_process():
    """ParallelWrapper CUSTOM mode with ONE BasicGradientsAccumulator shared by 4 in-process workers: every replica
    applies the sum of the 4 workers' post-updater updates each round, so all replicas stay identical and equal a
    single-process simulation of that rule (Sgd: sum of per-batch SGD steps)."""
    from deeplearning4j_amd import DataSet, Sgd
    from deeplearning4j_amd.parallel import BasicGradientsAccumulator, ParallelWrapper
    net = W.make_net(Sgd(0.1))
    batches = W.make_batches(8, 8)
    pw = ParallelWrapper.Builder(net).workers(4).inProcess(True) \
        .gradientsAccumulator(BasicGradientsAccumulator(4)).build()
    pw.fit(batches, 1)
    ms = pw._inproc.models
    for m in ms[1:]:
        assert torch.equal(m.params(), ms[0].params())
    # simulate: per round, p <- p - sum_i lr * g_i / mb_i  (each worker's own SGD update)
    ref = W.make_net(Sgd(0.1))
    p = ref.params().clone()
    for r in range(2):
        total = torch.zeros_like(p)
        for b in batches[4 * r:4 * r + 4]:
            probe = W.make_net(Sgd(0.1))
            probe.setParams(p.clone())
            probe.fit(DataSet(b.features, b.labels))
            total += p - probe.params()
        p = p - total
    assert torch.allclose(ms[0].params(), p, atol=1e-6), (ms[0].params() - p).abs().max()


def test_parallel_wrapper_custom_basic_partial_round():
    """6 batches over 4 workers: the trailing round's 2 idle replicas contribute zero updates; all stay identical."""
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.parallel import BasicGradientsAccumulator, ParallelWrapper
    net = W.make_net(Adam(0.01))
    pw = ParallelWrapper.Builder(net).workers(4).inProcess(True) \
        .gradientsAccumulator(BasicGradientsAccumulator(4)).build()
    pw.fit(W.make_batches(6, 8), 1)
    ms = pw._inproc.models
    for m in ms[1:]:
        assert torch.equal(m.params(), ms[0].params())


def test_parallel_wrapper_custom_basic_two_fits():
    """A second fit starts new worker threads: the shared accumulator re-learns its parties."""
    from deeplearning4j_amd import Sgd
    from deeplearning4j_amd.parallel import BasicGradientsAccumulator, ParallelWrapper
    net = W.make_net(Sgd(0.1))
    pw = ParallelWrapper.Builder(net).workers(2).inProcess(True) \
        .gradientsAccumulator(BasicGradientsAccumulator(2)).build()
    pw.fit(W.make_batches(4, 8), 1)
    pw.fit(W.make_batches(4, 8), 1)
    assert net.getIterationCount() == 4
