"""Early stopping: configuration, termination conditions, score calculators, model savers, trainers
(reference deeplearning4j-nn/.../earlystopping/**; trainer loop BaseEarlyStoppingTrainer.java:77-300).

Semantics kept: the score calculator runs every ``evaluateEveryNEpochs`` epochs, a lower score is better
unless the calculator says otherwise, the best model is saved through the model saver, iteration termination
conditions see each minibatch score, epoch conditions see (epoch, score), and the result records the
termination reason/details, the score per epoch, the best epoch/score and the total epoch count.
On the GPU the per-minibatch score is only read (a device sync) when iteration conditions exist.
"""
import enum
import logging
import math
import os
import time

from .datasets import DataSet, MultiDataSet

log = logging.getLogger("deeplearning4j_amd")


# ----------------------------------------------------------------------------------------- termination
class EpochTerminationCondition:
    def initialize(self):
        pass

    def terminate(self, epochNum, score, minimize=True):
        raise NotImplementedError


class IterationTerminationCondition:
    def initialize(self):
        pass

    def terminate(self, lastMiniBatchScore):
        raise NotImplementedError


class MaxEpochsTerminationCondition(EpochTerminationCondition):
    def __init__(self, maxEpochs):
        if maxEpochs <= 0:
            raise ValueError("Max number of epochs must be >= 1")
        self.maxEpochs = int(maxEpochs)

    def terminate(self, epochNum, score, minimize=True):
        return epochNum + 1 >= self.maxEpochs

    def __repr__(self):
        return f"MaxEpochsTerminationCondition({self.maxEpochs})"


class ScoreImprovementEpochTerminationCondition(EpochTerminationCondition):
    def __init__(self, maxEpochsWithNoImprovement, minImprovement=0.0):
        self.maxEpochsWithNoImprovement, self.minImprovement = int(maxEpochsWithNoImprovement), minImprovement
        self.initialize()

    def initialize(self):
        self.bestEpoch, self.bestScore = -1, float("nan")

    def terminate(self, epochNum, score, minimize=True):
        if self.bestEpoch == -1:
            self.bestEpoch, self.bestScore = epochNum, score
            return False
        improvement = (self.bestScore - score) if minimize else (score - self.bestScore)
        if improvement > self.minImprovement:
            self.bestEpoch, self.bestScore = epochNum, score
            return False
        return epochNum >= self.bestEpoch + self.maxEpochsWithNoImprovement

    def __repr__(self):
        return (f"ScoreImprovementEpochTerminationCondition(maxEpochsWithNoImprovement="
                f"{self.maxEpochsWithNoImprovement}, minImprovement={self.minImprovement})")


class BestScoreEpochTerminationCondition(EpochTerminationCondition):
    def __init__(self, bestExpectedScore, lesserBetter=True):
        self.bestExpectedScore, self.lesserBetter = bestExpectedScore, lesserBetter

    def terminate(self, epochNum, score, minimize=True):
        return score < self.bestExpectedScore if self.lesserBetter else self.bestExpectedScore < score

    def __repr__(self):
        return f"BestScoreEpochTerminationCondition({self.bestExpectedScore})"


class MaxTimeIterationTerminationCondition(IterationTerminationCondition):
    def __init__(self, maxTime, unit_seconds=1.0):
        self.maxTimeSec = float(maxTime) * unit_seconds
        self.initialize()

    def initialize(self):
        self.start = time.time()

    def terminate(self, lastMiniBatchScore):
        return time.time() - self.start >= self.maxTimeSec

    def __repr__(self):
        return f"MaxTimeIterationTerminationCondition({self.maxTimeSec}s)"


class MaxScoreIterationTerminationCondition(IterationTerminationCondition):
    def __init__(self, maxScore):
        self.maxScore = maxScore

    def terminate(self, s):
        return s > self.maxScore or math.isnan(s)

    def __repr__(self):
        return f"MaxScoreIterationTerminationCondition({self.maxScore})"


class InvalidScoreIterationTerminationCondition(IterationTerminationCondition):
    def terminate(self, s):
        return math.isnan(s) or math.isinf(s)

    def __repr__(self):
        return "InvalidScoreIterationTerminationCondition()"


# ----------------------------------------------------------------------------------------- score calculators
def _as_list(it):
    if isinstance(it, (DataSet, MultiDataSet)):
        return [it]
    it.reset()
    return it


class ScoreCalculator:
    def calculateScore(self, model):
        raise NotImplementedError

    def minimizeScore(self):
        return True


class DataSetLossCalculator(ScoreCalculator):
    """Average (or summed) loss over a held-out iterator (scorecalc/DataSetLossCalculator.java)."""

    def __init__(self, data, average=True):
        self.data, self.average = data, average

    def calculateScore(self, model):
        total, n = 0.0, 0
        for ds in _as_list(self.data):
            m = ds.numExamples() if isinstance(ds, DataSet) else ds.features[0].shape[0]
            total += model.score(ds) * m
            n += m
        return total / n if self.average and n else total


DataSetLossCalculatorCG = DataSetLossCalculator


class _EvalCalculator(ScoreCalculator):
    def __init__(self, data):
        self.data = data

    def _new(self):
        raise NotImplementedError

    def _metric(self, e):
        raise NotImplementedError

    def calculateScore(self, model):
        e = self._new()
        model.doEvaluation(self.data, e)
        return float(self._metric(e))


class ClassificationScoreCalculator(_EvalCalculator):
    """Evaluation metric on held-out data (ClassificationScoreCalculator.java); maximised except for none."""

    def __init__(self, metric, data):
        super().__init__(data)
        self.metric = metric if isinstance(metric, str) else metric.name

    def _new(self):
        from .eval import Evaluation
        return Evaluation()

    def _metric(self, e):
        return e.scoreForMetric(self.metric)

    def minimizeScore(self):
        return False


class RegressionScoreCalculator(_EvalCalculator):
    def __init__(self, metric, data):
        super().__init__(data)
        self.metric = metric if isinstance(metric, str) else metric.name

    def _new(self):
        from .eval import RegressionEvaluation
        return RegressionEvaluation()

    def _metric(self, e):
        return e.scoreForMetric(self.metric)

    def minimizeScore(self):
        return self.metric not in ("PC", "R2")


class ROCScoreCalculator(_EvalCalculator):
    class ROCType(enum.Enum):
        ROC = "ROC"
        BINARY = "BINARY"
        MULTICLASS = "MULTICLASS"

    class Metric(enum.Enum):
        AUC = "AUC"
        AUPRC = "AUPRC"

    def __init__(self, rocType, data, metric=None):
        super().__init__(data)
        self.rocType = rocType
        self.metricName = (metric or ROCScoreCalculator.Metric.AUC)

    def _new(self):
        from .eval import ROC, ROCBinary, ROCMultiClass
        return {ROCScoreCalculator.ROCType.ROC: ROC, ROCScoreCalculator.ROCType.BINARY: ROCBinary,
                ROCScoreCalculator.ROCType.MULTICLASS: ROCMultiClass}[self.rocType]()

    def _metric(self, e):
        auc = self.metricName == ROCScoreCalculator.Metric.AUC
        if self.rocType == ROCScoreCalculator.ROCType.ROC:
            return e.calculateAUC() if auc else e.calculateAUCPR()
        if self.rocType == ROCScoreCalculator.ROCType.BINARY:
            return e.calculateAverageAuc() if auc else e.calculateAverageAUCPR()
        return e.calculateAverageAUC() if auc else e.calculateAverageAUCPR()

    def minimizeScore(self):
        return False


class AutoencoderScoreCalculator(ScoreCalculator):
    """Reconstruction error of an AutoEncoder layer (or the network) on held-out data, as a regression metric."""

    def __init__(self, metric, data):
        self.metric = metric if isinstance(metric, str) else metric.name
        self.data = data

    def calculateScore(self, model):
        from .eval import RegressionEvaluation
        e = RegressionEvaluation()
        for ds in _as_list(self.data):
            x = ds.features
            out = model.output(x)
            e.eval(x.reshape(out.shape).to(out.device), out)
        return e.scoreForMetric(self.metric)


class VAEReconErrorScoreCalculator(AutoencoderScoreCalculator):
    pass


class VAEReconProbScoreCalculator(ScoreCalculator):
    """Negative mean reconstruction log-probability from a VAE layer (VAEReconProbScoreCalculator.java)."""

    def __init__(self, data, reconstructionProbNumSamples=1, logProb=True):
        self.data, self.numSamples, self.logProb = data, reconstructionProbNumSamples, logProb

    def calculateScore(self, model):
        vae = model.getLayer(0)
        total, n = 0.0, 0
        for ds in _as_list(self.data):
            lp = vae.reconstructionLogProbability(ds.features, self.numSamples)
            total += float(lp.sum())
            n += lp.numel()
        return -total / max(n, 1)


# ----------------------------------------------------------------------------------------- savers
class EarlyStoppingModelSaver:
    def saveBestModel(self, net, score):
        raise NotImplementedError

    def saveLatestModel(self, net, score):
        raise NotImplementedError

    def getBestModel(self):
        raise NotImplementedError

    def getLatestModel(self):
        raise NotImplementedError


class InMemoryModelSaver(EarlyStoppingModelSaver):
    def __init__(self):
        self.bestModel = self.latestModel = None

    def saveBestModel(self, net, score):
        self.bestModel = net.clone()

    def saveLatestModel(self, net, score):
        self.latestModel = net.clone()

    def getBestModel(self):
        return self.bestModel

    def getLatestModel(self):
        return self.latestModel


class LocalFileModelSaver(EarlyStoppingModelSaver):
    """bestModel.bin / latestModel.bin in a directory (LocalFileModelSaver.java), ModelSerializer zip format."""
    BEST, LATEST = "bestModel.bin", "latestModel.bin"

    def __init__(self, directory, saveUpdater=True):
        self.directory, self.saveUpdater = str(directory), saveUpdater
        os.makedirs(self.directory, exist_ok=True)

    def _save(self, net, name):
        from .utils.model_serializer import ModelSerializer
        p = os.path.join(self.directory, name)
        ModelSerializer.writeModel(net, p + ".tmp", self.saveUpdater)
        os.replace(p + ".tmp", p)

    def saveBestModel(self, net, score):
        self._save(net, self.BEST)

    def saveLatestModel(self, net, score):
        self._save(net, self.LATEST)

    def _load(self, name):
        from .utils.model_serializer import ModelSerializer
        p = os.path.join(self.directory, name)
        if not os.path.exists(p):
            raise FileNotFoundError(p)
        return ModelSerializer.restoreModel(p)

    def getBestModel(self):
        return self._load(self.BEST)

    def getLatestModel(self):
        return self._load(self.LATEST)


LocalFileGraphSaver = LocalFileModelSaver


# ----------------------------------------------------------------------------------------- config / result
class EarlyStoppingConfiguration:
    def __init__(self, epochTerminationConditions=None, iterationTerminationConditions=None,
                 scoreCalculator=None, modelSaver=None, evaluateEveryNEpochs=1, saveLastModel=False):
        self.epochTerminationConditions = list(epochTerminationConditions or [])
        self.iterationTerminationConditions = list(iterationTerminationConditions or [])
        self.scoreCalculator = scoreCalculator
        self.modelSaver = modelSaver or InMemoryModelSaver()
        self.evaluateEveryNEpochs = int(evaluateEveryNEpochs)
        self.saveLastModel = saveLastModel

    def validate(self):
        if not self.epochTerminationConditions and not self.iterationTerminationConditions:
            raise ValueError("Cannot conduct early stopping without a termination condition (both Iteration "
                             "and Epoch termination conditions are null/empty)")

    class Builder:
        def __init__(self):
            self._kw = {}

        def epochTerminationConditions(self, *c):
            self._kw["epochTerminationConditions"] = [x for a in c for x in (a if isinstance(a, list) else [a])]
            return self

        def iterationTerminationConditions(self, *c):
            self._kw["iterationTerminationConditions"] = [x for a in c for x in (a if isinstance(a, list) else [a])]
            return self

        def scoreCalculator(self, s):
            self._kw["scoreCalculator"] = s
            return self

        def modelSaver(self, s):
            self._kw["modelSaver"] = s
            return self

        def evaluateEveryNEpochs(self, n):
            self._kw["evaluateEveryNEpochs"] = n
            return self

        def saveLastModel(self, b):
            self._kw["saveLastModel"] = b
            return self

        def build(self):
            return EarlyStoppingConfiguration(**self._kw)


class TerminationReason(enum.Enum):
    Error = "Error"
    IterationTerminationCondition = "IterationTerminationCondition"
    EpochTerminationCondition = "EpochTerminationCondition"


class EarlyStoppingResult:
    TerminationReason = TerminationReason

    def __init__(self, terminationReason, terminationDetails, scoreVsEpoch, bestModelEpoch, bestModelScore,
                 totalEpochs, bestModel):
        self.terminationReason, self.terminationDetails = terminationReason, terminationDetails
        self.scoreVsEpoch, self.bestModelEpoch, self.bestModelScore = scoreVsEpoch, bestModelEpoch, bestModelScore
        self.totalEpochs, self.bestModel = totalEpochs, bestModel

    def getTerminationReason(self):
        return self.terminationReason

    def getTerminationDetails(self):
        return self.terminationDetails

    def getScoreVsEpoch(self):
        return self.scoreVsEpoch

    def getBestModelEpoch(self):
        return self.bestModelEpoch

    def getBestModelScore(self):
        return self.bestModelScore

    def getTotalEpochs(self):
        return self.totalEpochs

    def getBestModel(self):
        return self.bestModel

    def __repr__(self):
        return (f"EarlyStoppingResult(terminationReason={self.terminationReason.value},details="
                f"{self.terminationDetails},bestModelEpoch={self.bestModelEpoch},bestModelScore="
                f"{self.bestModelScore},totalEpochs={self.totalEpochs})")


class EarlyStoppingListener:
    def onStart(self, esConfig, net):
        pass

    def onEpoch(self, epochNum, score, esConfig, net):
        pass

    def onCompletion(self, result):
        pass


# ----------------------------------------------------------------------------------------- trainer
class EarlyStoppingTrainer:
    """Works for MultiLayerNetwork and ComputationGraph (EarlyStoppingTrainer / EarlyStoppingGraphTrainer)."""

    def __init__(self, esConfig, net, train, listener=None):
        self.esConfig, self.model, self.iterator, self.listener = esConfig, net, train, listener

    def setListener(self, l):
        self.listener = l

    def _epoch_listeners(self, start, epoch):
        self.model.setEpochCount(epoch)
        for l in self.model.getListeners():
            f = getattr(l, "onEpochStart" if start else "onEpochEnd", None)
            if f is not None:
                f(self.model)

    def fit(self):
        c = self.esConfig
        c.validate()
        sc = c.scoreCalculator
        minimize = sc.minimizeScore() if sc is not None else True
        for cond in c.iterationTerminationConditions + c.epochTerminationConditions:
            cond.initialize()
        if self.listener is not None:
            self.listener.onStart(c, self.model)
        scoreVsEpoch = {}
        bestEpoch, bestScore = -1, (float("inf") if minimize else -float("inf"))
        epoch = 0
        while True:
            self.iterator.reset()
            self._epoch_listeners(True, epoch)
            term, reason, it_count = False, None, 0
            while self.iterator.hasNext():
                ds = self.iterator.next()
                try:
                    if not self._fit_one(ds, it_count):
                        it_count += 1
                        continue
                except Exception as e:   # reference: return an Error result with the best model so far
                    log.warning("Early stopping training terminated due to exception at epoch %d, iteration %d: %s",
                                epoch, it_count, e)
                    return EarlyStoppingResult(TerminationReason.Error, repr(e), scoreVsEpoch, bestEpoch, bestScore,
                                               epoch, self._best())
                if c.iterationTerminationConditions:
                    s = self.model.score()
                    for cond in c.iterationTerminationConditions:
                        if cond.terminate(s):
                            term, reason = True, cond
                            break
                    term = self._agree(term)
                if term:
                    break
                it_count += 1
            if not self.iterator.hasNext():
                self._epoch_listeners(False, epoch)
            if term:
                log.info("Hit per iteration termination condition at epoch %d, iteration %d. Reason: %s", epoch,
                         it_count, reason)
                if c.saveLastModel:
                    c.modelSaver.saveLatestModel(self.model, 0.0)
                res = EarlyStoppingResult(TerminationReason.IterationTerminationCondition, repr(reason),
                                          scoreVsEpoch, bestEpoch, bestScore, epoch, self._best())
                if self.listener is not None:
                    self.listener.onCompletion(res)
                return res
            if (epoch == 0 and c.evaluateEveryNEpochs == 1) or epoch % c.evaluateEveryNEpochs == 0:
                score = sc.calculateScore(self.model) if sc is not None else 0.0
                scoreVsEpoch[epoch] = score
                invalid = math.isnan(score) or math.isinf(score)
                better = score < bestScore if minimize else score > bestScore
                if (sc is not None and better) or (bestEpoch == -1 and invalid):
                    bestScore, bestEpoch = score, epoch
                    c.modelSaver.saveBestModel(self.model, score)
                if c.saveLastModel:
                    c.modelSaver.saveLatestModel(self.model, score)
                if self.listener is not None:
                    self.listener.onEpoch(epoch, score, c, self.model)
                for cond in c.epochTerminationConditions:
                    if cond.terminate(epoch, score, minimize):
                        log.info("Hit epoch termination condition at epoch %d. Details: %s", epoch, cond)
                        best = self._best()
                        if best is None and c.saveLastModel:
                            best = self.model
                        res = EarlyStoppingResult(TerminationReason.EpochTerminationCondition, repr(cond),
                                                  scoreVsEpoch, bestEpoch, bestScore, epoch + 1, best)
                        if self.listener is not None:
                            self.listener.onCompletion(res)
                        return res
            epoch += 1

    def _fit_one(self, ds, it_count):
        """Fit one minibatch; returns False when this process skipped it (data-parallel sharding)."""
        self.model.fit(ds)
        return True

    def _agree(self, flag):
        return flag

    def _best(self):
        try:
            return self.esConfig.modelSaver.getBestModel()
        except FileNotFoundError:
            return None


EarlyStoppingGraphTrainer = EarlyStoppingTrainer


class EarlyStoppingParallelTrainer(EarlyStoppingTrainer):
    """Early stopping over a data-parallel ParallelWrapper (reference: deeplearning4j-scaleout-parallelwrapper
    ``EarlyStoppingParallelTrainer.java:51-120``, which wraps a ParallelWrapper with ``workers`` /
    ``averagingFrequency`` and checks termination conditions from an averaging listener).

    Here the "workers" are the ``torch.distributed`` ranks (one process per GPU, RCCL all-reduce of the flat
    gradient, or parameter averaging every ``averagingFrequency`` steps). Minibatch i of an epoch is fitted by
    rank ``i % world_size``; with shared gradients the replicas hold identical parameters, so every rank computes
    the same validation score and takes the same termination decision without extra communication. On one
    process this is exactly EarlyStoppingTrainer."""

    def __init__(self, esConfig, net, train, trainMulti=None, listener=None, workers=None, prefetchBuffer=16,
                 averagingFrequency=1, reportScoreAfterAveraging=True, useLegacyAveraging=True, trainingMode=None):
        if isinstance(listener, int) and not isinstance(listener, bool):
            # the reference's positional order (esConf, model, train, trainMulti, workers, prefetchBuffer,
            # averagingFrequency[, reportScoreAfterAveraging, useLegacyAveraging])
            listener, workers, prefetchBuffer, averagingFrequency = None, listener, \
                (workers if workers is not None else prefetchBuffer), \
                (prefetchBuffer if workers is not None else averagingFrequency)
        from .parallel.wrapper import ParallelWrapper, TrainingMode
        super().__init__(esConfig, net, train if train is not None else trainMulti, listener)
        mode = trainingMode if trainingMode is not None else TrainingMode.SHARED_GRADIENTS
        self.wrapper = ParallelWrapper(net, workers=workers, prefetchBuffer=prefetchBuffer,
                                       averagingFrequency=averagingFrequency,
                                       reportScoreAfterAveraging=reportScoreAfterAveraging, trainingMode=mode)

    def _fit_one(self, ds, it_count):
        # rank r fits batch r of every group of W consecutive batches; a trailing partial group is dropped so every
        # rank takes the same number of (collective) steps
        from .parallel.distributed import rank, world_size
        W = world_size()
        self.wrapper._prepare()
        if W == 1:
            self.wrapper._step(ds)
            return True
        if it_count == 0:
            self._group = []
        self._group.append(ds)
        if len(self._group) < W:
            return False
        mine, self._group = self._group[rank()], []
        self.wrapper._step(mine)
        return True

    def _agree(self, flag):
        # iteration scores differ per rank (different minibatches): terminate when any rank's condition fires
        from .parallel.distributed import all_reduce_max, world_size
        if world_size() == 1:
            return flag
        return bool(all_reduce_max(1.0 if flag else 0.0) > 0)

    def fit(self):
        res = super().fit()
        from .parallel.distributed import barrier
        barrier()
        if res.bestModel is None and res.terminationReason == TerminationReason.IterationTerminationCondition:
            # stopped inside the first epoch, before any score was saved: the current model is the result
            # (EarlyStoppingParallelTrainer.java:186-196)
            res.bestModel = self.model
        return res
