"""StatsListener: training statistics for the UI / storage.

Reference: UIM:stats/BaseStatsListener.java (init report: software / hardware / model info; per-report: score,
learning rates, memory, performance, GC, and for parameters / gradients / updates / activations: histograms,
mean, stdev and mean magnitude per (layer, param)), stats/api/{StatsUpdateConfiguration, StatsInitializationConfiguration,
StatsType, SummaryType, Histogram}.java.

MI355X mapping: every summary over the flat parameter / gradient / update arrays is ONE fused HIP launch covering all
(layer, param) segments (dl4j_segment_stats in csrc/stats.hip: mean, stdev, mean |x|, min, max + histograms), and
one device->host copy per report — no per-parameter reductions or syncs. Gradients are summarised in
onGradientCalculation (before the updater), updates in iterationDone (the fused updater leaves the applied update in
the gradient buffer, as the reference does).
"""
import gc
import os
import platform
import socket
import time
import uuid

import torch

from ..optimize.listeners import TrainingListener
from .storage import Persistable, StorageMetaData

TYPE_ID = "StatsListener"


class StatsType:
    Parameters, Gradients, Updates, Activations = "Parameters", "Gradients", "Updates", "Activations"


class SummaryType:
    Mean, Stdev, MeanMagnitudes = "Mean", "Stdev", "MeanMagnitudes"


class StatsUpdateConfiguration:
    def __init__(self, reportingFrequency=1, collectPerformanceStats=True, collectMemoryStats=True,
                 collectGarbageCollectionStats=True, collectLearningRates=True, collectHistograms=None,
                 collectMean=None, collectStdev=None, collectMeanMagnitudes=None, numHistogramBins=20):
        self.reportingFrequency = max(1, int(reportingFrequency))
        self.collectPerformanceStats = collectPerformanceStats
        self.collectMemoryStats = collectMemoryStats
        self.collectGarbageCollectionStats = collectGarbageCollectionStats
        self.collectLearningRates = collectLearningRates
        allt = {StatsType.Parameters, StatsType.Gradients, StatsType.Updates, StatsType.Activations}
        self.collectHistograms = set(allt if collectHistograms is None else collectHistograms)
        self.collectMean = set(allt if collectMean is None else collectMean)
        self.collectStdev = set(allt if collectStdev is None else collectStdev)
        self.collectMeanMagnitudes = set(allt if collectMeanMagnitudes is None else collectMeanMagnitudes)
        self.numHistogramBins = int(numHistogramBins)

    def wants(self, st):
        return st in self.collectHistograms or st in self.collectMean or st in self.collectStdev or \
            st in self.collectMeanMagnitudes

    class Builder:
        def __init__(self):
            self.kw = {}

        def reportingFrequency(self, n): self.kw["reportingFrequency"] = n; return self  # noqa: E704
        def collectPerformanceStats(self, b): self.kw["collectPerformanceStats"] = b; return self  # noqa: E704
        def collectMemoryStats(self, b): self.kw["collectMemoryStats"] = b; return self  # noqa: E704
        def collectGarbageCollectionStats(self, b): self.kw["collectGarbageCollectionStats"] = b; return self  # noqa
        def collectLearningRates(self, b): self.kw["collectLearningRates"] = b; return self  # noqa: E704
        def numHistogramBins(self, n): self.kw["numHistogramBins"] = n; return self  # noqa: E704

        def collectHistograms(self, *types):
            self.kw["collectHistograms"] = set(types)
            return self

        def collectMean(self, *types):
            self.kw["collectMean"] = set(types)
            return self

        def collectStdev(self, *types):
            self.kw["collectStdev"] = set(types)
            return self

        def collectMeanMagnitudes(self, *types):
            self.kw["collectMeanMagnitudes"] = set(types)
            return self

        def build(self):
            return StatsUpdateConfiguration(**self.kw)


DefaultStatsUpdateConfiguration = StatsUpdateConfiguration


class StatsInitializationConfiguration:
    def __init__(self, collectSoftwareInfo=True, collectHardwareInfo=True, collectModelInfo=True):
        self.collectSoftwareInfo = collectSoftwareInfo
        self.collectHardwareInfo = collectHardwareInfo
        self.collectModelInfo = collectModelInfo


DefaultStatsInitializationConfiguration = StatsInitializationConfiguration


def _segments(net):
    """(names, element offsets) of every parameter view inside the flat parameter array, in flat order."""
    flat = net.flattenedParams
    base = flat.data_ptr()
    es = flat.element_size()
    segs = []
    for k, v in net.paramTable().items():
        if v.numel() == 0:
            continue
        segs.append(((v.data_ptr() - base) // es, k, v.numel()))
    segs.sort()
    names = [k for _, k, _ in segs]
    offs = [o for o, _, _ in segs] + [segs[-1][0] + segs[-1][2]] if segs else [0]
    return names, offs


def summarize(flat, names, offs, bins):
    """{name: {mean, stdev, meanMagnitude, min, max, histogram?}} for segments of a flat array (one fused HIP
    launch on GPU; torch reductions on CPU)."""
    if flat.is_cuda:
        from ..ops import native
        stats, hist = native.segment_stats(flat.contiguous(), offs, bins)
        stats = stats.cpu().tolist()
        hist = hist.cpu().tolist() if hist is not None else None
    else:
        stats, hist = [], [] if bins else None
        f = flat.detach().float().reshape(-1)
        for a, b in zip(offs[:-1], offs[1:]):
            x = f[a:b]
            mn, mx = float(x.min()), float(x.max())
            stats.append([float(x.mean()), float(x.std(unbiased=False)), float(x.abs().mean()), mn, mx])
            if bins:
                h = torch.histc(x, bins, mn, mx) if mx > mn else torch.zeros(bins).index_fill_(0, torch.tensor([0]),
                                                                                                 float(x.numel()))
                hist.append([int(v) for v in h.tolist()])
    out = {}
    for i, n in enumerate(names):
        m, s, mm, lo, hi = stats[i]
        d = {"mean": m, "stdev": s, "meanMagnitude": mm, "min": lo, "max": hi}
        if hist is not None:
            d["histogram"] = {"min": lo, "max": hi, "bins": bins, "counts": hist[i]}
        out[n] = d
    return out


def _select(summary, st, cfg):
    out = {}
    for k, d in summary.items():
        e = {}
        if st in cfg.collectMean:
            e["mean"] = d["mean"]
        if st in cfg.collectStdev:
            e["stdev"] = d["stdev"]
        if st in cfg.collectMeanMagnitudes:
            e["meanMagnitude"] = d["meanMagnitude"]
        if st in cfg.collectHistograms and "histogram" in d:
            e["histogram"] = d["histogram"]
        out[k] = e
    return out


class StatsListener(TrainingListener):
    def __init__(self, router, listenerFrequency=None, updateConfig=None, initConfig=None, sessionID=None,
                 workerID=None):
        self.router = router
        self.updateConfig = updateConfig or StatsUpdateConfiguration(
            reportingFrequency=listenerFrequency if listenerFrequency else 1)
        if listenerFrequency:
            self.updateConfig.reportingFrequency = int(listenerFrequency)
        self.initConfig = initConfig or StatsInitializationConfiguration()
        self.sessionID = sessionID or str(uuid.uuid4())
        self.workerID = workerID or f"{socket.gethostname()}_{os.getpid()}_{os.environ.get('RANK', '0')}"
        self._init_done = False
        self._t0 = None
        self._last_t = None
        self._last_iter = 0
        self._examples = 0
        self._minibatches = 0
        self._grad_summary = None
        self._act_summary = None
        self._gc_prev = None

    # ------------------------------------------------------------------ helpers
    def _will_report(self, model):
        return (model.conf.iterationCount + 1) % self.updateConfig.reportingFrequency == 0

    def _init_report(self, model):
        ic = self.initConfig
        d = {}
        if ic.collectSoftwareInfo:
            d["software"] = {"python": platform.python_version(), "torch": torch.__version__,
                             "hip": getattr(torch.version, "hip", None), "os": platform.platform(),
                             "backend": "rocm" if torch.cuda.is_available() else "cpu"}
        if ic.collectHardwareInfo:
            hw = {"cpus": os.cpu_count(), "hostname": socket.gethostname(), "devices": []}
            if torch.cuda.is_available():
                for i in range(torch.cuda.device_count()):
                    p = torch.cuda.get_device_properties(i)
                    hw["devices"].append({"name": p.name, "totalMemory": p.total_memory,
                                          "multiProcessorCount": p.multi_processor_count})
            d["hardware"] = hw
        if ic.collectModelInfo:
            names, offs = _segments(model)
            d["model"] = {"className": type(model).__name__, "numParams": int(model.numParams()),
                          "numLayers": len(model._layer_offsets), "paramNames": names,
                          "layerNames": [str(n) for _, n, _, _ in model._layer_offsets],
                          "layerTypes": [type(i.conf).__name__ for _, _, i, _ in model._layer_offsets],
                          "configJson": model.conf.toJson() if hasattr(model.conf, "toJson") else None}
        self.router.putStorageMetaData(StorageMetaData(self.sessionID, TYPE_ID, self.workerID,
                                                       "StatsInitializationReport", "StatsReport"))
        self.router.putStaticInfo(Persistable(self.sessionID, TYPE_ID, self.workerID, data=d, kind="static"))
        self._init_done = True

    # ------------------------------------------------------------------ hooks
    def onForwardPass(self, model, activations):
        if StatsType.Activations not in (self.updateConfig.collectHistograms | self.updateConfig.collectMean |
                                         self.updateConfig.collectStdev | self.updateConfig.collectMeanMagnitudes):
            return
        if not self._will_report(model):
            return
        acts = activations if isinstance(activations, dict) else {str(i): a for i, a in enumerate(activations)}
        out = {}
        bins = self.updateConfig.numHistogramBins if StatsType.Activations in self.updateConfig.collectHistograms \
            else 0
        for k, a in acts.items():
            if not torch.is_tensor(a) or a.numel() == 0 or not a.is_floating_point():
                continue
            flat = a.detach().reshape(-1)
            if flat.dtype not in (torch.float32, torch.bfloat16):
                flat = flat.float()
            out.update(summarize(flat.contiguous(), [str(k)], [0, flat.numel()], bins))
        self._act_summary = out

    def onGradientCalculation(self, model):
        if not self.updateConfig.wants(StatsType.Gradients) or not self._will_report(model):
            return
        names, offs = _segments(model)
        bins = self.updateConfig.numHistogramBins if StatsType.Gradients in self.updateConfig.collectHistograms else 0
        self._grad_summary = summarize(model.flattenedGradients.reshape(-1), names, offs, bins)

    def iterationDone(self, model, iteration, epoch):
        now = time.time()
        if self._t0 is None:
            self._t0 = self._last_t = now
        mb = getattr(model, "_mb", None) or 0
        self._examples += int(mb)
        self._minibatches += 1
        if not self._init_done:
            self._init_report(model)
        if iteration % self.updateConfig.reportingFrequency != 0:
            return
        t_start = time.time()
        cfg = self.updateConfig
        d = {"iterationCount": int(iteration), "epochCount": int(epoch), "score": float(model.score())}
        if cfg.collectPerformanceStats:
            dt = max(now - self._last_t, 1e-9)
            iters = max(iteration - self._last_iter, 1)
            d["performance"] = {"totalRuntimeMs": int((now - self._t0) * 1000), "totalExamples": self._examples,
                                "totalMinibatches": self._minibatches,
                                "examplesPerSecond": iters * mb / dt if mb else 0.0,
                                "minibatchesPerSecond": iters / dt}
        if cfg.collectMemoryStats:
            mem = {}
            try:
                import psutil
                p = psutil.Process()
                mem["hostCurrentBytes"] = p.memory_info().rss
                mem["hostMaxBytes"] = psutil.virtual_memory().total
            except ImportError:
                pass
            if torch.cuda.is_available():
                dev = torch.cuda.current_device()
                free, total = torch.cuda.mem_get_info(dev)
                mem["deviceCurrentBytes"] = [int(torch.cuda.memory_allocated(dev))]
                mem["deviceReservedBytes"] = [int(torch.cuda.memory_reserved(dev))]
                mem["deviceMaxBytes"] = [int(total)]
            d["memory"] = mem
        if cfg.collectGarbageCollectionStats:
            st = gc.get_stats()
            cur = [(s["collections"], s["collected"]) for s in st]
            prev = self._gc_prev or [(0, 0)] * len(cur)
            d["gc"] = [{"generation": i, "deltaCount": c - pc, "deltaCollected": k - pk}
                       for i, ((c, k), (pc, pk)) in enumerate(zip(cur, prev))]
            self._gc_prev = cur
        names, offs = _segments(model)
        if cfg.collectLearningRates:
            by_off = dict(zip(offs[:-1], names))
            lrs = {}
            for sg in model.updater.plan.segments:
                n = by_off.get(sg.p_off)
                lr = sg.updater.getLearningRate(iteration, epoch) if n is not None and \
                    getattr(sg.updater, "HAS_LR", False) else None
                if lr is not None:
                    lrs[n] = float(lr)
            d["learningRates"] = lrs
        if cfg.wants(StatsType.Parameters):
            bins = cfg.numHistogramBins if StatsType.Parameters in cfg.collectHistograms else 0
            d[StatsType.Parameters] = _select(summarize(model.flattenedParams.reshape(-1), names, offs, bins),
                                              StatsType.Parameters, cfg)
        if cfg.wants(StatsType.Updates) and model.flattenedGradients is not None:
            bins = cfg.numHistogramBins if StatsType.Updates in cfg.collectHistograms else 0
            d[StatsType.Updates] = _select(summarize(model.flattenedGradients.reshape(-1), names, offs, bins),
                                           StatsType.Updates, cfg)
        if self._grad_summary is not None:
            d[StatsType.Gradients] = _select(self._grad_summary, StatsType.Gradients, cfg)
            self._grad_summary = None
        if self._act_summary is not None:
            d[StatsType.Activations] = _select(self._act_summary, StatsType.Activations, cfg)
            self._act_summary = None
        d["statsCollectionDurationMs"] = int((time.time() - t_start) * 1000)
        self.router.putUpdate(Persistable(self.sessionID, TYPE_ID, self.workerID, data=d, kind="update"))
        self._last_t, self._last_iter = now, iteration


J7StatsListener = StatsListener
