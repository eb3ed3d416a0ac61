"""In-process ParallelWrapper: one host thread per device, fed round-robin from a streaming iterator.

Reference: PW:ParallelWrapper.java:123-137 (worker threads pinned to devices), :467-565 (the fit loop: the master
round-robins DataSets into per-worker queues of capacity 1, waits for all workers after every ``workers`` batches,
averages every ``averagingFrequency`` rounds), PW:trainer/DefaultTrainer.java:254-311 (replica creation: worker 0
trains the root model, the others train copies), :396-416 (worker exceptions rethrown to the master).

MI355X design:
  * replicas live on GPUs 0..N-1 of this process; their communicators come from ``ncclCommInitAll`` (RcclComm,
    parallel/rccl.py) and every collective is enqueued on the worker's own HIP stream; on a host without N GPUs the
    replicas run on the CPU over the in-process LoopbackComm (same code path, used by the CPU tests);
  * SHARED_GRADIENTS: synchronous DP — each worker's bucketed gradient all-reduce runs during its backward
    (AllReduceGradientsAccumulator with the worker's communicator), then the update with the global minibatch;
  * AVERAGING: local steps, parameters (+ updater state) all-reduced and divided by N every k rounds;
  * streaming: the master pulls one round (N batches) at a time from the iterator and hands batch i of the round to
    worker i through a queue of capacity ``prefetchBuffer // N`` (>= 1); at most ``prefetchBuffer + 2N`` batches
    (queued, in training, and the round being handed out) exist at once however long the iterator is;
  * a trailing partial round of L < N batches trains on the first L workers (reference :514-578,
    ``registerConsumers(locker)``); the other workers still run the round's collectives with a zero gradient, and
    every replica's update divides the summed gradient by the round's total example count (SHARED_GRADIENTS), so
    every replica applies the same update even when the round's batches differ in size;
  * HIP graphs: replicas inherit the caller's ``enableHipGraphs`` mode and each worker thread captures its own
    replica's step (thread-local capture mode, per-thread capture streams and graph slots, nn/hipgraph.py);
  * no per-batch host sync: each worker records an event per step and waits only for the step ``max_inflight``
    rounds back, so the next batch's host work and H2D copy overlap the GPU;
  * failure: a worker exception aborts every communicator (waiting ranks raise instead of hanging), the other
    workers are drained and the master re-raises it.
Listeners fire on worker 0, i.e. on the caller's own model (the reference attaches them to the root model too).
"""
import collections
import logging
import queue
import threading

import torch

from ..datasets.dataset import DataSet, MultiDataSet
from .accumulation import AllReduceGradientsAccumulator, average_params_and_state

log = logging.getLogger("deeplearning4j_amd")

_STOP = object()


def _replica(model, device):
    """A copy of ``model`` (config, parameters, updater state) on ``device``."""
    import copy
    net = type(model)(copy.deepcopy(model.conf))
    net.init(model.params().detach().to(device).clone(), device=device)
    st = model.updater.getStateViewArray()
    if st is not None and st.numel() > 0:
        net.updater.setStateViewArray(st.detach().to(device).clone())
    net.conf.iterationCount = model.conf.iterationCount
    net.conf.epochCount = model.conf.epochCount
    if getattr(model, "_hipgraph_enabled", False):       # replicas train exactly like the caller's model
        net.enableHipGraphs(True, warmup=getattr(model, "_hipgraph_warmup", 2))
    return net


def _fit_one(m, ds):
    if isinstance(ds, MultiDataSet):
        m._fit_batch(ds.features, ds.labels, ds.featuresMasks, ds.labelsMasks)
    elif isinstance(ds, DataSet):
        if type(m).__name__ == "ComputationGraph":
            m._fit_batch([ds.features], [ds.labels], None if ds.featuresMask is None else [ds.featuresMask],
                         None if ds.labelsMask is None else [ds.labelsMask])
        else:
            m._fit_batch(ds.features, ds.labels, ds.featuresMask, ds.labelsMask)
    else:
        raise TypeError(f"unsupported batch type {type(ds)}")


def devices_for(n, model=None):
    """GPUs 0..n-1 when this process sees at least n; the CPU for every worker when the model itself lives on the
    CPU. A model on a GPU with fewer than n GPUs visible is an error (mixing one GPU worker with CPU replicas would
    be silently far slower): use fewer workers, or one process per device (torchrun / inProcess(False))."""
    if torch.cuda.is_available() and torch.cuda.device_count() >= n:
        return [torch.device("cuda", i) for i in range(n)]
    dev = getattr(model, "device", None) if model is not None else None
    if dev is not None and torch.device(dev).type == "cuda":
        raise RuntimeError(f"in-process ParallelWrapper: {n} workers need {n} visible GPUs, this process sees "
                           f"{torch.cuda.device_count()}; reduce workers() or use one process per device")
    return [torch.device("cpu")] * n


def make_comms(devs):
    if devs[0].type == "cuda":
        from .rccl import RcclComm
        return RcclComm.init_all([d.index for d in devs])
    from .rccl import LoopbackComm
    return LoopbackComm.create(len(devs))


class InProcessTrainer:
    """Owns the replicas, communicators and worker threads of one ParallelWrapper (created on first fit)."""

    def __init__(self, wrapper, devices=None, comms=None):
        self.w = wrapper
        n = int(wrapper.workers)
        self.devices = list(devices) if devices is not None else devices_for(n, wrapper.model)
        m = wrapper.model
        if not m.initCalled:
            m.init(device=self.devices[0])
        self.comms = list(comms) if comms is not None else make_comms(self.devices)
        # worker 0 trains the caller's model (DefaultTrainer.java:248-283); the rest train copies
        self.models = [m] + [_replica(m, d) for d in self.devices[1:]]
        from .wrapper import TrainingMode
        self.shared = wrapper.trainingMode in (TrainingMode.SHARED_GRADIENTS,)
        self.custom = getattr(wrapper.accumulator, "shared_in_process", False)
        if self.custom:
            # CUSTOM mode with a thread-shared accumulator (BasicGradientsAccumulator): every replica gets the SAME
            # instance, which synchronises the worker threads itself (reference PW:ParallelWrapper.java:838-843)
            if getattr(wrapper.accumulator, "parties", n) != n:
                raise ValueError(f"accumulator built for {wrapper.accumulator.parties} parties, wrapper has {n} "
                                 "workers")
            for net in self.models:
                net.setGradientsAccumulator(wrapper.accumulator)
        elif self.shared:
            for net, c in zip(self.models, self.comms):
                net.setGradientsAccumulator(AllReduceGradientsAccumulator(wrapper.bucket_mb, comm=c))
        self.queues = [queue.Queue(maxsize=max(1, int(wrapper.prefetchBuffer) // n)) for _ in range(n)]
        self.errors = []
        self.rounds_done = [0] * n
        self.cv = threading.Condition()
        self.max_live = 0           # most batches alive at once (tests check the streaming bound)
        self._live = 0
        self._threads = []
        self.max_inflight = 2       # GPU steps a worker may have queued before it waits on the oldest one

    # ------------------------------------------------------------------------------------------------ workers
    def _run(self, i):
        net, comm, q, dev = self.models[i], self.comms[i], self.queues[i], self.devices[i]
        from .wrapper import TrainingMode
        avg = self.w.trainingMode == TrainingMode.AVERAGING
        k = self.w.averagingFrequency
        inflight = collections.deque()
        try:
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            while True:
                item = q.get()
                if item is _STOP:
                    break
                ds, rnd, active, bsz, total = item
                acc = getattr(net, "gradientsAccumulator", None)
                if acc is not None and not self.custom:
                    # every replica divides the summed gradient by the SAME count, the round's total examples (a
                    # short trailing batch or a partial round would otherwise give each replica its own divisor)
                    acc.global_batch = total
                    if active < len(self.models):
                        acc.participants = active       # partial round: replicas that trained
                try:
                    if ds is not None:
                        _fit_one(net, ds)               # the network moves the batch to its device
                    elif self.custom:
                        acc.idle_step(net)              # a zero update into the shared accumulator's barriers
                    elif self.shared:
                        net._zero_contribution_step(bsz)
                finally:
                    if acc is not None and not self.custom:
                        acc.participants = None
                        acc.global_batch = None
                if ds is not None:
                    with self.cv:
                        self._live -= 1
                if avg and (rnd + 1) % k == 0:
                    average_params_and_state(net, self.w.averageUpdaters, comm=comm)
                if dev.type == "cuda":
                    ev = torch.cuda.Event()
                    ev.record()
                    inflight.append(ev)
                    while len(inflight) > self.max_inflight:
                        inflight.popleft().synchronize()
                with self.cv:
                    self.rounds_done[i] = rnd + 1
                    self.cv.notify_all()
            while inflight:
                inflight.popleft().synchronize()
        except BaseException as e:          # noqa: BLE001 — propagated to the master
            with self.cv:
                self.errors.append((i, e))
                self.cv.notify_all()
            for c in self.comms:
                c.abort()
            if self.custom and hasattr(self.w.accumulator, "abort"):
                self.w.accumulator.abort()
            while True:                     # drain so the master's puts never block forever
                try:
                    if q.get(timeout=0.05) is _STOP:
                        break
                except queue.Empty:
                    if not any(t.is_alive() for t in self._threads if t is not threading.current_thread()):
                        break

    def _start(self):
        if self._threads:
            return
        if len(self.models) > 1 and self.devices[0].type == "cuda":
            from ..ops import rnn_native
            rnn_native.CONCURRENT_STREAMS[0] += 1      # RCCL kernels on other streams: cooperative LSTM launches
            self._concurrent = True
        if self.custom and hasattr(self.w.accumulator, "resetParties"):
            self.w.accumulator.resetParties()
        for i in range(len(self.models)):
            t = threading.Thread(target=self._run, args=(i,), name=f"dl4j-pw-worker-{i}", daemon=True)
            t.start()
            self._threads.append(t)

    def _raise_if_failed(self):
        if self.errors:
            i, e = self.errors[0]
            raise RuntimeError(f"ParallelWrapper worker {i} failed: {e!r}") from e

    # ------------------------------------------------------------------------------------------------ master
    def _put(self, i, item):
        while True:
            self._raise_if_failed()
            try:
                self.queues[i].put(item, timeout=0.1)
                return
            except queue.Full:
                continue

    def fit(self, source, numEpochs=1):
        n = len(self.models)
        m = self.models[0]
        self._start()
        rnd = 0
        try:
            for _ in range(int(numEpochs)):
                for l in m.listeners:
                    if hasattr(l, "onEpochStart"):
                        l.onEpochStart(m)
                for batch_round in _rounds(source, n):
                    L = len(batch_round)
                    bsz = _batch_size(batch_round[0])
                    total = sum(_batch_size(b) for b in batch_round)
                    with self.cv:
                        self._live += L             # pulled from the iterator and not yet trained on
                        self.max_live = max(self.max_live, self._live)
                    for i in range(n):
                        self._put(i, (batch_round[i] if i < L else None, rnd, L, bsz, total))
                    rnd += 1
                self._wait_rounds(rnd)
                for net in self.models:
                    net.incrementEpochCount()
                for l in m.listeners:
                    if hasattr(l, "onEpochEnd"):
                        l.onEpochEnd(m)
            from .wrapper import TrainingMode
            if self.w.trainingMode == TrainingMode.AVERAGING and rnd % self.w.averagingFrequency != 0:
                self._collective_all(lambda net, c: average_params_and_state(net, self.w.averageUpdaters, comm=c))
        finally:
            self.shutdown()
        self._raise_if_failed()
        return m

    def _wait_rounds(self, rnd):
        with self.cv:
            while min(self.rounds_done) < rnd and not self.errors:
                self.cv.wait(timeout=0.5)
        self._raise_if_failed()

    def _collective_all(self, fn):
        """Run fn(model_i, comm_i) on every replica concurrently (collectives need all ranks in flight)."""
        errs = []

        def run(i):
            try:
                if self.devices[i].type == "cuda":
                    torch.cuda.set_device(self.devices[i])
                fn(self.models[i], self.comms[i])
                if self.devices[i].type == "cuda":
                    torch.cuda.current_stream(self.devices[i]).synchronize()
            except BaseException as e:      # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=run, args=(i,)) for i in range(len(self.models))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]

    def shutdown(self):
        for i, t in enumerate(self._threads):
            if t.is_alive():
                try:
                    self.queues[i].put(_STOP, timeout=1.0)
                except queue.Full:
                    pass
        for t in self._threads:
            t.join(timeout=30)
        self._threads = []
        if getattr(self, "_concurrent", False):
            from ..ops import rnn_native
            rnn_native.CONCURRENT_STREAMS[0] -= 1
            self._concurrent = False


def _batch_size(ds):
    if ds is None:
        return 1
    f = ds.features
    f = f[0] if isinstance(f, (list, tuple)) else f
    return int(f.shape[0])


def _rounds(source, n):
    """Stream rounds of n batches from a DataSetIterator / MultiDataSetIterator / iterable; the last round may be
    partial (fewer than n batches)."""
    if isinstance(source, (DataSet, MultiDataSet)):
        source = [source]
    if hasattr(source, "hasNext"):
        if hasattr(source, "reset"):
            source.reset()

        def gen():
            while source.hasNext():
                yield source.next()
        it = gen()
    else:
        it = iter(source)
    buf = []
    for ds in it:
        buf.append(ds)
        if len(buf) == n:
            yield buf
            buf = []
    if buf:
        log.debug("ParallelWrapper: trailing round of %d batch(es) trains on the first %d of %d workers",
                  len(buf), len(buf), n)
        yield buf
