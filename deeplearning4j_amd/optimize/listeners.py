"""Training listeners (reference deeplearning4j-nn/.../optimize/listeners/* and optimize/api/TrainingListener.java).

Hook contract (TrainingListener.java:20-71), called by MultiLayerNetwork / ComputationGraph:
  iterationDone(model, iteration, epoch), onEpochStart(model), onEpochEnd(model),
  onForwardPass(model, activations), onGradientCalculation(model), onBackwardPass(model).
MI355X note: ``model.score()`` synchronises the device (the score lives on the GPU until read), so
listeners that read it every iteration serialize the host with the GPU; the defaults read it every
``frequency`` iterations only.
"""
import enum
import logging
import os
import time

log = logging.getLogger("deeplearning4j_amd")


class InvocationType(enum.Enum):
    """When an EvaluativeListener fires (optimize/api/InvocationType.java)."""
    EPOCH_START = "EPOCH_START"
    EPOCH_END = "EPOCH_END"
    ITERATION_END = "ITERATION_END"


class TrainingListener:
    """Base with no-op hooks (BaseTrainingListener.java)."""

    def iterationDone(self, model, iteration, epoch):
        pass

    def onEpochStart(self, model):
        pass

    def onEpochEnd(self, model):
        pass

    def onForwardPass(self, model, activations):
        pass

    def onGradientCalculation(self, model):
        pass

    def onBackwardPass(self, model):
        pass


BaseTrainingListener = TrainingListener
IterationListener = TrainingListener


class ScoreIterationListener(TrainingListener):
    """Logs the score every ``printIterations`` iterations (ScoreIterationListener.java)."""

    def __init__(self, printIterations=10):
        self.printIterations = max(1, int(printIterations))
        self.history = []

    def iterationDone(self, model, iteration, epoch):
        if iteration % self.printIterations == 0:
            s = model.score()
            self.history.append((iteration, s))
            log.info("Score at iteration %d is %s", iteration, s)


class CollectScoresIterationListener(TrainingListener):
    """Collects (iteration, score) pairs every ``frequency`` iterations (CollectScoresIterationListener.java)."""

    def __init__(self, frequency=1):
        self.frequency = max(1, int(frequency))
        self.scoreVsIter = []

    def iterationDone(self, model, iteration, epoch):
        if iteration % self.frequency == 0:
            self.scoreVsIter.append((iteration, model.score()))

    def getScoreVsIter(self):
        return list(self.scoreVsIter)

    def exportScores(self, path_or_file, delimiter=","):
        lines = ["Iteration" + delimiter + "Score"] + [f"{i}{delimiter}{s}" for i, s in self.scoreVsIter]
        text = "\n".join(lines) + "\n"
        if hasattr(path_or_file, "write"):
            path_or_file.write(text)
        else:
            with open(path_or_file, "w") as f:
                f.write(text)


class PerformanceListener(TrainingListener):
    """Samples/sec, batches/sec, iteration time, ETL time (PerformanceListener.java:60-122). Times are wall-clock
    between consecutive iterationDone calls; with ``synchronize`` the device is synchronised first so the time is
    the true step time rather than the host enqueue time."""

    def __init__(self, frequency=1, reportScore=False, reportSample=True, reportBatch=True, reportIteration=True,
                 reportTime=True, reportEtl=True, synchronize=True):
        self.frequency = max(1, int(frequency))
        self.reportScore, self.reportSample, self.reportBatch = reportScore, reportSample, reportBatch
        self.reportIteration, self.reportTime, self.reportEtl = reportIteration, reportTime, reportEtl
        self.synchronize = synchronize
        self.lastTime = None
        self.samplesPerSec = 0.0
        self.batchesPerSec = 0.0
        self.records = []

    class Builder:
        def __init__(self):
            self._kw = {}

        def setFrequency(self, f):
            self._kw["frequency"] = f
            return self

        def reportScore(self, b):
            self._kw["reportScore"] = b
            return self

        def reportSample(self, b):
            self._kw["reportSample"] = b
            return self

        def reportBatch(self, b):
            self._kw["reportBatch"] = b
            return self

        def reportIteration(self, b):
            self._kw["reportIteration"] = b
            return self

        def reportTime(self, b):
            self._kw["reportTime"] = b
            return self

        def reportETL(self, b):
            self._kw["reportEtl"] = b
            return self

        def build(self):
            return PerformanceListener(**self._kw)

    def _now(self, model):
        if self.synchronize:
            dev = getattr(model, "device", None)
            if dev is not None and getattr(dev, "type", "cpu") == "cuda":
                import torch
                torch.cuda.synchronize(dev)
        return time.perf_counter()

    def iterationDone(self, model, iteration, epoch):
        now = self._now(model)
        if self.lastTime is None:
            self.lastTime = now
            return
        if iteration % self.frequency == 0:
            dt = max(now - self.lastTime, 1e-9)
            n = getattr(model, "_mb", None) or 0
            self.samplesPerSec = n / dt
            self.batchesPerSec = 1.0 / dt
            parts = []
            if self.reportEtl:
                parts.append(f"ETL: {getattr(model, 'lastEtlTime', 0):.0f} ms")
            if self.reportIteration:
                parts.append(f"iteration {iteration}")
            if self.reportTime:
                parts.append(f"iteration time: {dt * 1000:.1f} ms")
            if self.reportSample:
                parts.append(f"samples/sec: {self.samplesPerSec:.3f}")
            if self.reportBatch:
                parts.append(f"batches/sec: {self.batchesPerSec:.3f}")
            rec = {"iteration": iteration, "time_ms": dt * 1000, "samples_per_sec": self.samplesPerSec,
                   "batches_per_sec": self.batchesPerSec}
            if self.reportScore:
                rec["score"] = model.score()
                parts.append(f"score: {rec['score']}")
            self.records.append(rec)
            log.info("; ".join(parts) + ";")
        self.lastTime = now


class TimeIterationListener(TrainingListener):
    """Logs remaining-time estimates given the total iteration count (TimeIterationListener.java)."""

    def __init__(self, iterationCount):
        self.iterationCount = int(iterationCount)
        self.start = time.time()
        self.iterationCounter = 0
        self.lastEstimate = None

    def iterationDone(self, model, iteration, epoch):
        self.iterationCounter += 1
        elapsed = time.time() - self.start
        remaining = (self.iterationCount - self.iterationCounter) * elapsed / self.iterationCounter
        self.lastEstimate = remaining
        log.info("Remaining time : %d mn - End expected at : %s", int(remaining / 60),
                 time.ctime(time.time() + remaining))


class ParamAndGradientIterationListener(TrainingListener):
    """Per-parameter mean / min / max / mean-abs of params and gradients (and the update direction, i.e. the
    gradient view after the updater) every ``iterations`` iterations; optional tab-delimited file output
    (ParamAndGradientIterationListener.java). Statistics are reduced on the device in one pass per tensor."""

    def __init__(self, iterations=1, printHeader=True, printMean=True, printMinMax=True, printMeanAbsValue=True,
                 outputToConsole=True, outputToFile=False, outputToLogger=True, file=None, delimiter="\t"):
        self.iterations = max(1, int(iterations))
        self.printHeader, self.printMean, self.printMinMax = printHeader, printMean, printMinMax
        self.printMeanAbsValue, self.outputToConsole, self.outputToFile = printMeanAbsValue, outputToConsole, \
            outputToFile
        self.outputToLogger, self.file, self.delimiter = outputToLogger, file, delimiter
        self.rows = []
        self._wrote_header = False

    class _Builder:
        def __init__(self):
            self._kw = {}

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)

            def setter(v=True):
                self._kw[name] = v
                return self
            return setter

        def build(self):
            return ParamAndGradientIterationListener(**self._kw)

    @classmethod
    def builder(cls):
        """Fluent builder with the reference's property names (ParamAndGradientIterationListener.builder())."""
        return cls._Builder()

    def _stat_names(self):
        names = []
        if self.printMean:
            names.append("mean")
        if self.printMinMax:
            names += ["min", "max"]
        if self.printMeanAbsValue:
            names.append("meanAbsValue")
        return names

    def _stats(self, t):
        import torch
        t = t.detach().float().reshape(-1)
        if t.numel() == 0:
            return []
        vals = []
        if self.printMean:
            vals.append(t.mean())
        if self.printMinMax:
            vals += [t.min(), t.max()]
        if self.printMeanAbsValue:
            vals.append(t.abs().mean())
        return torch.stack(vals).cpu().tolist()

    def iterationDone(self, model, iteration, epoch):
        if iteration % self.iterations != 0:
            return
        params = model.paramTable()
        grads = model.gradient().gradientForVariable() if hasattr(model, "gradient") else {}
        row = [iteration, model.score()]
        header = ["n", "score"]
        stat_names = self._stat_names()
        for k, p in params.items():
            if p.numel() == 0:
                continue
            header += [f"param_{k}_{n}" for n in stat_names]
            row += self._stats(p)
            g = grads.get(k)
            if g is not None and g.numel() > 0:
                header += [f"grad_{k}_{n}" for n in stat_names]
                row += self._stats(g)
        self.rows.append(row)
        line = self.delimiter.join(str(x) for x in row)
        if self.outputToFile and self.file:
            with open(self.file, "a") as f:
                if self.printHeader and not self._wrote_header:
                    f.write(self.delimiter.join(header) + "\n")
                    self._wrote_header = True
                f.write(line + "\n")
        if self.outputToConsole:
            print(line)
        if self.outputToLogger:
            log.info(line)


class ComposableIterationListener(TrainingListener):
    """Fans every hook out to a list of listeners (ComposableIterationListener.java)."""

    def __init__(self, *listeners):
        self.listeners = [x for l in listeners for x in (l if isinstance(l, (list, tuple)) else [l])]

    def iterationDone(self, model, iteration, epoch):
        for l in self.listeners:
            l.iterationDone(model, iteration, epoch)

    def onEpochStart(self, model):
        for l in self.listeners:
            getattr(l, "onEpochStart", lambda m: None)(model)

    def onEpochEnd(self, model):
        for l in self.listeners:
            getattr(l, "onEpochEnd", lambda m: None)(model)

    def onForwardPass(self, model, activations):
        for l in self.listeners:
            getattr(l, "onForwardPass", lambda m, a: None)(model, activations)

    def onGradientCalculation(self, model):
        for l in self.listeners:
            getattr(l, "onGradientCalculation", lambda m: None)(model)

    def onBackwardPass(self, model):
        for l in self.listeners:
            getattr(l, "onBackwardPass", lambda m: None)(model)


class EvaluativeListener(TrainingListener):
    """Runs evaluations on held-out data every ``frequency`` invocations of ``invocationType``
    (EvaluativeListener.java). ``callback(listener, model, invocationCount, evaluations)`` is optional."""

    def __init__(self, data, frequency=1, invocationType=InvocationType.ITERATION_END, *evaluations, callback=None):
        from ..eval import Evaluation
        self.data = data
        self.frequency = max(1, int(frequency))
        self.invocationType = invocationType
        self.evaluations = list(evaluations) or [Evaluation()]
        self.callback = callback
        self.invocationCount = 0
        self.lastEvaluations = None

    def _invoke(self, model):
        self.invocationCount += 1
        if self.invocationCount % self.frequency != 0:
            return
        for e in self.evaluations:
            e.reset()
        if hasattr(model, "doEvaluation"):
            model.doEvaluation(self.data, *self.evaluations)
        self.lastEvaluations = list(self.evaluations)
        for e in self.evaluations:
            log.info("Evaluation at invocation %d:\n%s", self.invocationCount, e.stats())
        if self.callback is not None:
            self.callback(self, model, self.invocationCount, self.evaluations)

    def iterationDone(self, model, iteration, epoch):
        if self.invocationType == InvocationType.ITERATION_END:
            self._invoke(model)

    def onEpochStart(self, model):
        if self.invocationType == InvocationType.EPOCH_START:
            self._invoke(model)

    def onEpochEnd(self, model):
        if self.invocationType == InvocationType.EPOCH_END:
            self._invoke(model)


class SleepyTrainingListener(TrainingListener):
    """Latency injection per training phase (SleepyTrainingListener.java): sleeps ``timer*`` ms in each hook.
    TimeMode.SIMPLE always sleeps the full amount; ADDITIVE sleeps only the remainder so the phase takes at
    least that long (fault/latency injection for data-parallel straggler tests)."""

    class TimeMode(enum.Enum):
        SIMPLE = "SIMPLE"
        ADDITIVE = "ADDITIVE"

    def __init__(self, timerIteration=0, timerEpochStart=0, timerEpochEnd=0, timerFF=0, timerBP=0,
                 timerGradient=0, timeMode=None):
        self.timerIteration, self.timerES, self.timerEE = timerIteration, timerEpochStart, timerEpochEnd
        self.timerFF, self.timerBP, self.timerGradient = timerFF, timerBP, timerGradient
        self.timeMode = timeMode or SleepyTrainingListener.TimeMode.SIMPLE
        self._last = {}

    def _sleep(self, key, ms):
        if ms <= 0:
            return
        now = time.time() * 1000
        if self.timeMode == SleepyTrainingListener.TimeMode.ADDITIVE and key in self._last:
            ms = ms - (now - self._last[key])
        if ms > 0:
            time.sleep(ms / 1000.0)
        self._last[key] = time.time() * 1000

    def iterationDone(self, model, iteration, epoch):
        self._sleep("it", self.timerIteration)

    def onEpochStart(self, model):
        self._sleep("es", self.timerES)

    def onEpochEnd(self, model):
        self._sleep("ee", self.timerEE)

    def onForwardPass(self, model, activations):
        self._sleep("ff", self.timerFF)

    def onBackwardPass(self, model):
        self._sleep("bp", self.timerBP)

    def onGradientCalculation(self, model):
        self._sleep("gc", self.timerGradient)


# ----------------------------------------------------------------------------------------------- checkpoints
class Checkpoint:
    """One row of checkpointInfo.txt (listeners/checkpoint/Checkpoint.java)."""
    HEADER = "checkpointNum,timestamp,iteration,epoch,modelType,filename"

    def __init__(self, checkpointNum, timestamp, iteration, epoch, modelType, filename=None):
        self.checkpointNum, self.timestamp, self.iteration = int(checkpointNum), int(timestamp), int(iteration)
        self.epoch, self.modelType, self.filename = int(epoch), modelType, filename

    def toFileString(self):
        return f"{self.checkpointNum},{self.timestamp},{self.iteration},{self.epoch},{self.modelType},{self.filename}"

    @staticmethod
    def fromFileString(s):
        a = s.strip().split(",")
        return Checkpoint(int(a[0]), int(a[1]), int(a[2]), int(a[3]), a[4], a[5])

    def getCheckpointNum(self):
        return self.checkpointNum

    def getIteration(self):
        return self.iteration

    def getEpoch(self):
        return self.epoch

    def getFilename(self):
        return self.filename

    def __repr__(self):
        return f"Checkpoint({self.toFileString()})"


class CheckpointListener(TrainingListener):
    """Periodic model checkpoints: every N epochs / N iterations / wall-clock interval, with keepAll, keepLast(n)
    or keepLastAndEvery(n, m) retention; files ``checkpoint_<n>_<ModelType>.zip`` + ``checkpointInfo.txt``
    (listeners/checkpoint/CheckpointListener.java:79-344). With data parallelism only rank 0 writes."""
    MODEL_TYPES = ("MultiLayerNetwork", "ComputationGraph", "Model")

    def __init__(self, rootDir, keepMode="ALL", keepLast=0, keepEvery=0, logSaving=True, saveEveryNEpochs=None,
                 saveEveryNIterations=None, saveEveryNIterSinceLast=False, saveEveryMs=None,
                 saveEverySinceLast=False, saveUpdater=True):
        self.rootDir = str(rootDir)
        os.makedirs(self.rootDir, exist_ok=True)
        self.keepMode, self.keepLast, self.keepEvery = keepMode, keepLast, keepEvery
        self.logSaving = logSaving
        self.saveEveryNEpochs, self.saveEveryNIterations = saveEveryNEpochs, saveEveryNIterations
        self.saveEveryNIterSinceLast = saveEveryNIterSinceLast
        self.saveEveryMs, self.saveEverySinceLast = saveEveryMs, saveEverySinceLast
        self.saveUpdater = saveUpdater
        self.recordFile = os.path.join(self.rootDir, "checkpointInfo.txt")
        self.lastCheckpointNum = -1
        for c in self.availableCheckpoints():     # resume numbering after a restart
            self.lastCheckpointNum = max(self.lastCheckpointNum, c.checkpointNum)
        self._last = None
        self.startTime = None
        self.startIter = None
        self._lastTimedSave = None

    class Builder:
        def __init__(self, rootDir):
            self._kw = {"rootDir": rootDir}

        def keepAll(self):
            self._kw["keepMode"] = "ALL"
            return self

        def keepLast(self, n):
            self._kw.update(keepMode="LAST", keepLast=int(n))
            return self

        def keepLastAndEvery(self, nLast, everyN):
            self._kw.update(keepMode="LAST_AND_EVERY", keepLast=int(nLast), keepEvery=int(everyN))
            return self

        def logSaving(self, b):
            self._kw["logSaving"] = b
            return self

        def saveEveryEpoch(self):
            return self.saveEveryNEpochs(1)

        def saveEveryNEpochs(self, n):
            self._kw["saveEveryNEpochs"] = int(n)
            return self

        def saveEveryNIterations(self, n, sinceLast=False):
            self._kw.update(saveEveryNIterations=int(n), saveEveryNIterSinceLast=sinceLast)
            return self

        def saveEvery(self, amount, unit_seconds=1.0, sinceLast=False):
            self._kw.update(saveEveryMs=float(amount) * unit_seconds * 1000.0, saveEverySinceLast=sinceLast)
            return self

        def build(self):
            return CheckpointListener(**self._kw)

    @staticmethod
    def _rank0():
        try:
            import torch.distributed as dist
            return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
        except Exception:
            return True

    @staticmethod
    def _model_type(model):
        n = type(model).__name__
        return n if n in ("MultiLayerNetwork", "ComputationGraph") else "Model"

    def onEpochEnd(self, model):
        done = model.getEpochCount() + 1
        if self.saveEveryNEpochs and done > 0 and done % self.saveEveryNEpochs == 0:
            self._save(model)

    def iterationDone(self, model, iteration, epoch):
        if self.startTime is None:
            self.startTime, self.startIter = time.time() * 1000, iteration
            return
        if self.saveEveryNIterations:
            if self.saveEveryNIterSinceLast:
                last = self._last.iteration if self._last else self.startIter
                if iteration - last >= self.saveEveryNIterations:
                    self._save(model)
                    return
            elif iteration > 0 and iteration % self.saveEveryNIterations == 0:
                self._save(model)
                return
        if self.saveEveryMs:
            now = time.time() * 1000
            if self.saveEverySinceLast:
                last = self._last.timestamp if self._last else self.startTime
                if now - last >= self.saveEveryMs:
                    self._save(model)
            else:
                last = self._lastTimedSave if self._lastTimedSave is not None else self.startTime
                if now - last > self.saveEveryMs:
                    self._save(model)
                    self._lastTimedSave = now

    def _save(self, model):
        if not self._rank0():
            return
        from ..utils.model_serializer import ModelSerializer
        if not os.path.exists(self.recordFile):
            with open(self.recordFile, "w") as f:
                f.write(Checkpoint.HEADER + "\n")
        self.lastCheckpointNum += 1
        c = Checkpoint(self.lastCheckpointNum, int(time.time() * 1000), model.getIterationCount(),
                       model.getEpochCount(), self._model_type(model))
        c.filename = f"checkpoint_{c.checkpointNum}_{c.modelType}.zip"
        path = os.path.join(self.rootDir, c.filename)
        tmp = path + ".tmp"
        ModelSerializer.writeModel(model, tmp, self.saveUpdater)
        os.replace(tmp, path)                  # atomic: a crash never leaves a torn checkpoint
        with open(self.recordFile, "a") as f:
            f.write(c.toFileString() + "\n")
        if self.logSaving:
            log.info("Model checkpoint saved: epoch %d, iteration %d, path: %s", c.epoch, c.iteration, path)
        self._last = c
        if self.keepMode == "LAST":
            cps = self.availableCheckpoints()
            while len(cps) > self.keepLast:
                os.remove(self.getFileForCheckpoint(cps.pop(0)))
        elif self.keepMode == "LAST_AND_EVERY":
            for cp in self.availableCheckpoints():
                if cp.checkpointNum > 0 and (cp.checkpointNum + 1) % self.keepEvery == 0:
                    continue
                if cp.checkpointNum > self.lastCheckpointNum - self.keepLast:
                    continue
                os.remove(self.getFileForCheckpoint(cp))

    def availableCheckpoints(self):
        if not os.path.exists(self.recordFile):
            return []
        with open(self.recordFile) as f:
            lines = f.read().splitlines()[1:]
        out = []
        for ln in lines:
            if ln.strip():
                c = Checkpoint.fromFileString(ln)
                if os.path.exists(os.path.join(self.rootDir, c.filename)):
                    out.append(c)
        return out

    def lastCheckpoint(self):
        a = self.availableCheckpoints()
        return a[-1] if a else None

    def getFileForCheckpoint(self, c):
        num = c.checkpointNum if isinstance(c, Checkpoint) else int(c)
        if num < 0:
            raise ValueError(f"Invalid checkpoint number: {num}")
        for t in self.MODEL_TYPES:
            p = os.path.join(self.rootDir, f"checkpoint_{num}_{t}.zip")
            if os.path.exists(p):
                return p
        raise FileNotFoundError(f"Model file for checkpoint {num} does not exist")

    def loadCheckpoint(self, c, loadUpdater=True, device=None):
        from ..utils.model_serializer import ModelSerializer
        return ModelSerializer.restoreModel(self.getFileForCheckpoint(c), loadUpdater, device)

    @staticmethod
    def loadCheckpointMLN(rootDir, num):
        return CheckpointListener(rootDir).loadCheckpoint(num)

    loadCheckpointCG = loadCheckpointMLN

    @staticmethod
    def loadLastCheckpointMLN(rootDir):
        cl = CheckpointListener(rootDir)
        last = cl.lastCheckpoint()
        return None if last is None else cl.loadCheckpoint(last)

    loadLastCheckpointCG = loadLastCheckpointMLN
