"""Cluster (multi-node) training masters — the MI355X replacement for dl4j-spark.

Reference: SPK:impl/multilayer/SparkDl4jMultiLayer.java (fit(RDD<DataSet>) :214, evaluate, calculateScore),
SPK:impl/graph/SparkComputationGraph.java, SPK:api/TrainingMaster.java (SPI), SPK:impl/paramavg/
ParameterAveragingTrainingMaster.java (split the data into chunks of workers*batchSizePerWorker*averagingFrequency,
workers fit ``averagingFrequency`` minibatches, parameters (+ updater state) averaged, broadcast, repeat),
SPS:training/SharedTrainingMaster.java (threshold-encoded gradient sharing between workers every iteration),
SPK:api/stats/SparkTrainingStats.java + StatsUtils.exportStatsAsHtml.

Design: Spark executors + the driver become ranks of one torch.distributed job spanning nodes (torchrun
--nnodes N --nproc-per-node 8; RCCL over xGMI inside a node and the NIC fabric across nodes). An "RDD" is any
sequence / DataSetIterator visible to every rank; each rank takes its strided shard (rank r: items r, r+W, ...),
exactly like Spark's partition-per-executor. The averaging round of ParameterAveragingTrainingMaster is an
all-reduce of the flat parameter (and updater-state) vector — one collective instead of the reference's
driver-side aggregation tree — and SharedTrainingMaster reuses the encoded/dense gradient-sharing accumulators of
ParallelWrapper. Evaluation is computed on each shard and merged with an all-gather of the evaluation state.
"""
import json
import time

import torch

from ..datasets.dataset import DataSet, DataSetIterator, ListDataSetIterator
from .accumulation import AllReduceGradientsAccumulator, average_params_and_state
from .distributed import barrier, is_dist, rank, world_size


class TrainingStats:
    """Per-phase wall-clock timings of a distributed fit (SparkTrainingStats): phase -> list of (rank, start_ms,
    duration_ms)."""

    def __init__(self):
        self.events = {}

    def add(self, phase, start, dur):
        self.events.setdefault(phase, []).append((rank(), int(start * 1000), int(dur * 1000)))

    def getKeySet(self):
        return set(self.events)

    def getValue(self, key):
        return list(self.events.get(key, []))

    def summary(self):
        out = {}
        for k, v in self.events.items():
            d = [e[2] for e in v]
            out[k] = {"count": len(d), "totalMs": sum(d), "meanMs": sum(d) / max(1, len(d))}
        return out

    def statsAsString(self):
        return json.dumps(self.summary(), indent=1, sort_keys=True)


class StatsUtils:
    @staticmethod
    def exportStatsAsHtml(stats, path):
        """Timeline + per-phase duration table (StatsUtils.exportStatsAsHtml) via the static UI components."""
        from ..ui.components import ChartTimeline, ComponentTable, StaticPageUtil
        tl = ChartTimeline("Training phases by worker")
        lanes = {}
        for phase, evs in stats.events.items():
            for r, st, d in evs:
                lanes.setdefault(f"rank {r}", []).append((st, st + max(d, 1), phase))
        for lane in sorted(lanes):
            tl.addLaneData(lane, lanes[lane])
        rows = [[k, v["count"], v["totalMs"], f"{v['meanMs']:.2f}"] for k, v in sorted(stats.summary().items())]
        table = ComponentTable(["phase", "count", "total ms", "mean ms"], rows, title="Phase durations")
        StaticPageUtil.saveHTMLFile(path, table, tl)


class TrainingMaster:
    """SPI: how a cluster of replicas trains one model."""

    def executeTraining(self, net, data):
        raise NotImplementedError

    def setCollectTrainingStats(self, b):
        self.collectTrainingStats = bool(b)

    def getTrainingStats(self):
        return self.stats


def _batches(data, batch):
    """Normalise "RDD" inputs: DataSetIterator, list of DataSets, or one big DataSet (split into ``batch``)."""
    if isinstance(data, DataSet):
        return data.batchBy(batch)
    if isinstance(data, DataSetIterator):
        data.reset()
        return [d for d in data]
    out = []
    for d in data:
        out.extend(d.batchBy(batch) if batch and d.numExamples() > batch else [d])
    return out


def _fit_one(net, ds):
    if type(net).__name__ == "ComputationGraph":
        net._fit_batch([ds.features], [ds.labels], None if ds.featuresMask is None else [ds.featuresMask],
                       None if ds.labelsMask is None else [ds.labelsMask])
    else:
        net._fit_batch(ds.features, ds.labels, ds.featuresMask, ds.labelsMask)


class ParameterAveragingTrainingMaster(TrainingMaster):
    class Builder:
        def __init__(self, rddDataSetNumExamples=1):
            self.kw = {"rddDataSetNumExamples": rddDataSetNumExamples}

        def batchSizePerWorker(self, n): self.kw["batchSizePerWorker"] = int(n); return self  # noqa: E704
        def averagingFrequency(self, n): self.kw["averagingFrequency"] = int(n); return self  # noqa: E704
        def aggregationDepth(self, n): self.kw["aggregationDepth"] = int(n); return self  # noqa: E704
        def workerPrefetchNumBatches(self, n): self.kw["workerPrefetchNumBatches"] = int(n); return self  # noqa
        def saveUpdater(self, b): self.kw["saveUpdater"] = bool(b); return self  # noqa: E704
        def collectTrainingStats(self, b): self.kw["collectTrainingStats"] = bool(b); return self  # noqa: E704
        def repartionData(self, r): return self  # noqa: E704
        def repartitionStrategy(self, r): return self  # noqa: E704
        def rddTrainingApproach(self, a): return self  # noqa: E704
        def exportDirectory(self, d): return self  # noqa: E704
        def storageLevel(self, s): return self  # noqa: E704

        def build(self):
            return ParameterAveragingTrainingMaster(**self.kw)

    def __init__(self, rddDataSetNumExamples=1, batchSizePerWorker=16, averagingFrequency=5, aggregationDepth=2,
                 workerPrefetchNumBatches=0, saveUpdater=True, collectTrainingStats=False):
        self.rddDataSetNumExamples = rddDataSetNumExamples
        self.batchSizePerWorker = batchSizePerWorker
        self.averagingFrequency = max(1, averagingFrequency)
        self.aggregationDepth = aggregationDepth
        self.saveUpdater = saveUpdater
        self.collectTrainingStats = collectTrainingStats
        self.stats = TrainingStats()

    def executeTraining(self, net, data):
        W, r = world_size(), rank()
        if is_dist():
            AllReduceGradientsAccumulator().broadcast_params(net, 0)          # broadcast initial parameters
        batches = _batches(data, self.batchSizePerWorker)
        n_rounds = len(batches) // W                                         # equal work per rank
        mine = [batches[i * W + r] for i in range(n_rounds)]
        since = 0
        for ds in mine:
            t0 = time.time()
            _fit_one(net, ds)
            if self.collectTrainingStats:
                self.stats.add("fit", t0, time.time() - t0)
            since += 1
            if since == self.averagingFrequency:
                t1 = time.time()
                average_params_and_state(net, self.saveUpdater)
                if self.collectTrainingStats:
                    self.stats.add("average", t1, time.time() - t1)
                since = 0
        if since:
            average_params_and_state(net, self.saveUpdater)
        barrier()
        return net


class SharedTrainingMaster(TrainingMaster):
    """Synchronous gradient sharing every iteration: threshold-encoded updates (EncodedGradientsAccumulator,
    the reference's Strom-style sharing) or, with ``threshold=None``, a dense bucketed all-reduce."""

    class Builder:
        def __init__(self, threshold=1e-3, rddDataSetNumExamples=1):
            self.kw = {"threshold": threshold}

        def batchSizePerWorker(self, n): self.kw["batchSizePerWorker"] = int(n); return self  # noqa: E704
        def updatesThreshold(self, t): self.kw["threshold"] = t; return self  # noqa: E704
        def thresholdAlgorithm(self, a): self.kw["threshold"] = getattr(a, "threshold", a); return self  # noqa
        def workersPerNode(self, n): return self  # noqa: E704
        def collectTrainingStats(self, b): self.kw["collectTrainingStats"] = bool(b); return self  # noqa: E704

        def build(self):
            return SharedTrainingMaster(**self.kw)

    def __init__(self, threshold=1e-3, batchSizePerWorker=16, collectTrainingStats=False):
        self.threshold = threshold
        self.batchSizePerWorker = batchSizePerWorker
        self.collectTrainingStats = collectTrainingStats
        self.stats = TrainingStats()

    def executeTraining(self, net, data):
        from .wrapper import ParallelWrapper, TrainingMode
        b = ParallelWrapper.Builder(net)
        if self.threshold is not None:
            from .encoded import EncodedGradientsAccumulator
            b = b.gradientsAccumulator(EncodedGradientsAccumulator(threshold=self.threshold))
        else:
            b = b.trainingMode(TrainingMode.SHARED_GRADIENTS)
        pw = b.build()
        t0 = time.time()
        pw.fit(ListDataSetIterator(_batches(data, self.batchSizePerWorker)))
        if self.collectTrainingStats:
            self.stats.add("fit", t0, time.time() - t0)
        return net


class SparkDl4jMultiLayer:
    """Distributed front end for a MultiLayerNetwork (same API shape as the reference's Spark wrapper; the
    ``sc`` argument is accepted for source compatibility and ignored — the cluster is the process group)."""

    def __init__(self, sc, netOrConf, trainingMaster):
        from ..nn.multilayer import MultiLayerNetwork
        if not hasattr(netOrConf, "fit"):
            netOrConf = MultiLayerNetwork(netOrConf)
            netOrConf.init()
        self.net = netOrConf
        self.tm = trainingMaster

    def getNetwork(self):
        return self.net

    def getTrainingMaster(self):
        return self.tm

    def fit(self, data, numEpochs=1):
        for _ in range(int(numEpochs)):
            self.tm.executeTraining(self.net, data)
            self.net.incrementEpochCount()
        return self.net

    fitMultiDataSet = fit

    def _local_eval(self, data, ev, batch):
        bs = _batches(data, batch)
        W, r = world_size(), rank()
        for ds in bs[r::W]:
            out = self.net.output(ds.features)
            out = out[0] if isinstance(out, list) else out
            ev.eval(ds.labels, out, ds.labelsMask) if ds.labelsMask is not None else ev.eval(ds.labels, out)
        return ev

    def _merge(self, ev):
        if not is_dist():
            return ev
        import torch.distributed as dist
        objs = [None] * world_size()
        dist.all_gather_object(objs, ev.toJson())
        merged = type(ev).fromJson(objs[0])
        for j in objs[1:]:
            merged.merge(type(ev).fromJson(j))
        return merged

    def evaluate(self, data, evaluation=None, batch=64):
        from ..eval.evaluation import Evaluation
        return self._merge(self._local_eval(data, evaluation or Evaluation(), batch))

    def doEvaluation(self, data, evaluation, batch=64):
        return self.evaluate(data, evaluation, batch)

    def evaluateRegression(self, data, batch=64):
        from ..eval.regression import RegressionEvaluation
        return self.evaluate(data, RegressionEvaluation(), batch)

    def evaluateROC(self, data, thresholdSteps=0, batch=64):
        from ..eval.roc import ROC
        return self.evaluate(data, ROC(thresholdSteps), batch)

    def calculateScore(self, data, average=True, batch=64):
        bs = _batches(data, batch)
        W, r = world_size(), rank()
        tot, n = 0.0, 0
        for ds in bs[r::W]:
            s = self.net.score(ds) if hasattr(self.net, "score") else 0.0
            tot += s * ds.numExamples()
            n += ds.numExamples()
        t = torch.tensor([tot, float(n)], dtype=torch.float64)
        if is_dist():
            import torch.distributed as dist
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else t.device
            t = t.to(dev)
            dist.all_reduce(t)
            t = t.cpu()
        return float(t[0] / t[1]) if average else float(t[0])

    def getScore(self):
        return self.net.score()


class SparkComputationGraph(SparkDl4jMultiLayer):
    def __init__(self, sc, netOrConf, trainingMaster):
        from ..nn.graph import ComputationGraph
        if not hasattr(netOrConf, "fit"):
            netOrConf = ComputationGraph(netOrConf)
            netOrConf.init()
        self.net = netOrConf
        self.tm = trainingMaster


DistributedMultiLayer = SparkDl4jMultiLayer
DistributedComputationGraph = SparkComputationGraph
