"""ParallelWrapper: single-node data-parallel training (reference PW:ParallelWrapper.java:123-904,
PW:trainer/DefaultTrainer.java, PW:trainer/SymmetricTrainer.java).

MI355X-first design: ONE PROCESS PER GPU (``torchrun --nproc-per-node 8``), each holding a full replica in its
own HBM, talking over RCCL/xGMI. The reference's N worker threads sharing one JVM become N ranks; the
round-robin feeding of DataSets to worker queues becomes a rank-strided view of the iterator (rank r trains on
batches r, r+W, r+2W, ...), so W consecutive batches form one synchronous step exactly as the reference's
"after every `workers` batches wait for all" loop.

Training modes (ParallelWrapper.TrainingMode):
  * SHARED_GRADIENTS (default here): synchronous DP. Dense bucketed all-reduce of the summed gradient, issued
    during backward (AllReduceGradientsAccumulator), then one fused update with the GLOBAL minibatch —
    numerically the single-GPU large-batch step.
    ``gradientsAccumulator(EncodedGradientsAccumulator(...))`` selects the reference's threshold-encoded
    update sharing instead (the post-updater update is residual-encoded and exchanged).
  * AVERAGING: local SGD; every ``averagingFrequency`` iterations parameters (and updater state when
    ``averageUpdaters``) are averaged with an all-reduce (reference Nd4j.averageAndPropagate, :316-376).
  * CUSTOM: a user accumulator (any object with begin_backward/grad_ready/reduce_gradients or apply_update).
Without an initialised process group (W == 1) the wrapper simply trains the model.
"""
import enum
import logging
import os

from ..datasets.dataset import DataSet, MultiDataSet
from .accumulation import AllReduceGradientsAccumulator, average_params_and_state
from .distributed import barrier, is_dist, rank, world_size

log = logging.getLogger("deeplearning4j_amd")


class TrainingMode(enum.Enum):
    AVERAGING = "AVERAGING"
    SHARED_GRADIENTS = "SHARED_GRADIENTS"
    CUSTOM = "CUSTOM"


class _RankShard:
    """Rank-strided view of a DataSetIterator: rank r sees batches r, r+W, ... Every rank sees the same number
    of batches (a trailing partial round is dropped) so the collectives stay matched."""

    def __init__(self, it, r, w):
        self.it, self.r, self.w = it, r, w

    def __iter__(self):
        if isinstance(self.it, (list, tuple)) or not hasattr(self.it, "hasNext"):
            src = list(self.it)                  # a list (or any iterable) of DataSets: stride it directly
            for i in range(0, len(src) - len(src) % self.w, self.w):
                yield src[i + self.r]
            return
        if hasattr(self.it, "reset"):
            self.it.reset()
        buf = []
        while self.it.hasNext():
            buf.append(self.it.next())
            if len(buf) == self.w:
                yield buf[self.r]
                buf = []


class ParallelWrapper:
    TrainingMode = TrainingMode

    def __init__(self, model, workers=None, prefetchBuffer=16, averagingFrequency=1, averageUpdaters=True,
                 reportScoreAfterAveraging=False, trainingMode=TrainingMode.SHARED_GRADIENTS,
                 gradientsAccumulator=None, bucket_mb=None, trainerContext=None, inProcess=None):
        self.model = model
        self.inProcess = inProcess
        self._inproc = None
        self.trainerContext = trainerContext
        self._trainer = None
        self.workers = workers or world_size()
        if is_dist() and self.workers != world_size():
            log.warning("ParallelWrapper: workers=%d but world size is %d; one worker per rank is used",
                        self.workers, world_size())
            self.workers = world_size()
        self.prefetchBuffer = prefetchBuffer
        self.averagingFrequency = max(1, int(averagingFrequency))
        self.averageUpdaters = averageUpdaters
        self.reportScoreAfterAveraging = reportScoreAfterAveraging
        self.trainingMode = trainingMode
        self.accumulator = gradientsAccumulator
        self.bucket_mb = bucket_mb
        self._prepared = False
        self._iter = 0
        self.listeners = []

    class Builder:
        def __init__(self, model):
            self._kw = {"model": model}

        def workers(self, n):
            self._kw["workers"] = int(n)
            return self

        def prefetchBuffer(self, n):
            self._kw["prefetchBuffer"] = int(n)
            return self

        def averagingFrequency(self, n):
            self._kw["averagingFrequency"] = int(n)
            return self

        def averageUpdaters(self, b):
            self._kw["averageUpdaters"] = bool(b)
            return self

        def reportScoreAfterAveraging(self, b):
            self._kw["reportScoreAfterAveraging"] = bool(b)
            return self

        def trainingMode(self, m):
            self._kw["trainingMode"] = TrainingMode(m) if not isinstance(m, TrainingMode) else m
            return self

        def gradientsAccumulator(self, acc):
            self._kw["gradientsAccumulator"] = acc
            self._kw.setdefault("trainingMode", TrainingMode.CUSTOM)
            return self

        def inProcess(self, b=True):
            """True: one host thread per device in this process (RCCL communicators from ncclCommInitAll, or the
            host loopback on CPU); False: one child process per device (parallel/launcher.py). Default: threads."""
            self._kw["inProcess"] = bool(b)
            return self

        def bucketSizeMB(self, mb):
            self._kw["bucket_mb"] = mb
            return self

        def trainerFactory(self, ctx):
            """A parallel.factory.TrainerContext (Default / Symmetric / ParameterServer) that owns the per-step
            synchronisation instead of trainingMode."""
            self._kw["trainerContext"] = ctx
            self._kw.setdefault("trainingMode", TrainingMode.CUSTOM)
            return self

        def build(self):
            return ParallelWrapper(**self._kw)

    def setListeners(self, *ls):
        self.model.setListeners(*ls)

    def _prepare(self):
        if self._prepared:
            return
        m = self.model
        if not m.initCalled:
            m.init()
        if is_dist():
            # every replica starts from rank 0's parameters and updater state (DefaultTrainer.java:254-311)
            AllReduceGradientsAccumulator().broadcast_params(m, 0)
        if self.trainingMode == TrainingMode.SHARED_GRADIENTS and self.accumulator is None:
            self.accumulator = AllReduceGradientsAccumulator(self.bucket_mb)
        if self.trainingMode in (TrainingMode.SHARED_GRADIENTS, TrainingMode.CUSTOM) and self.accumulator is not None:
            m.setGradientsAccumulator(self.accumulator)
        if self.trainerContext is not None:
            self.trainerContext.init(m)
            self._trainer = self.trainerContext.create(None, rank(), m, rank(), False, self, self.trainingMode,
                                                       self.averagingFrequency)
        self._prepared = True

    def fit(self, source, numEpochs=1, presharded=False):
        """Train on a DataSetIterator / MultiDataSetIterator (or a list of DataSets) for ``numEpochs``.

        Called from one plain process with ``workers > 1`` (no process group), by default the wrapper trains with
        one host thread per device in this process (parallel/inprocess.py: streaming round-robin feed, RCCL
        communicators from ncclCommInitAll; listeners fire on this model). ``inProcess(False)`` (or
        DL4J_AMD_PW_SPAWN=1) launches one child process per device instead (parallel/launcher.py: batches are
        streamed to the children over sockets; listeners do not run there). Under torchrun (a process group) every
        rank runs this method on its rank-strided share of the batches."""
        shared_acc = getattr(self.accumulator, "shared_in_process", False)
        if not is_dist() and self.workers > 1 and self.trainerContext is None and \
                (self.accumulator is None or shared_acc):
            spawn = not shared_acc and (self.inProcess is False or (self.inProcess is None and
                                                                    os.environ.get("DL4J_AMD_PW_SPAWN", "0") == "1"))
            if spawn:
                from .launcher import spawn_fit
                return spawn_fit(self, source, numEpochs)
            if self.trainingMode not in (TrainingMode.SHARED_GRADIENTS, TrainingMode.AVERAGING) and not shared_acc:
                raise ValueError("in-process ParallelWrapper supports SHARED_GRADIENTS, AVERAGING and CUSTOM "
                                 "accumulators shared between threads (BasicGradientsAccumulator); other CUSTOM "
                                 "accumulators / trainer contexts need one process per device (torchrun)")
            from .inprocess import InProcessTrainer
            if self._inproc is None:
                self._inproc = InProcessTrainer(self)
            try:
                return self._inproc.fit(source, numEpochs)
            except BaseException:
                self._inproc = None         # aborted communicators are not reusable: rebuild on the next fit
                raise
        self._prepare()
        m = self.model
        W, r = world_size(), rank()
        for _ in range(int(numEpochs)):
            for l in m.listeners:
                if hasattr(l, "onEpochStart"):
                    l.onEpochStart(m)
            if presharded:                 # a launcher child: the parent already sent only this rank's batches
                items = source
            else:
                items = _RankShard(source, r, W) if W > 1 else (source if not hasattr(source, "reset") else
                                                                _RankShard(source, 0, 1))
            for ds in items:
                self._step(ds)
            for l in m.listeners:
                if hasattr(l, "onEpochEnd"):
                    l.onEpochEnd(m)
            m.incrementEpochCount()
        if self._trainer is not None:
            self.trainerContext.finalizeTraining(m)
        elif self.trainingMode == TrainingMode.AVERAGING and self._iter % self.averagingFrequency != 0:
            average_params_and_state(m, self.averageUpdaters)       # final sync so all replicas agree
        barrier()
        return m

    def _step(self, ds):
        m = self.model
        if self._trainer is not None:
            self._trainer.feedDataSet(ds)
            self._iter += 1
            if self._iter % self.averagingFrequency == 0:
                self.trainerContext.finalizeRound(m)
            return
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
        self._iter += 1
        if self.trainingMode == TrainingMode.AVERAGING and self._iter % self.averagingFrequency == 0:
            average_params_and_state(m, self.averageUpdaters)
            if self.reportScoreAfterAveraging:
                log.info("Averaged score: %s", m.score())

    def shutdown(self):
        pass

    close = shutdown
