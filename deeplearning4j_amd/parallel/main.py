"""ParallelWrapperMain: command-line data-parallel training of a saved model.

Reference: PW:main/ParallelWrapperMain.java (flags --modelPath, --workers, --prefetchSize, --averagingFrequency,
--reportScore, --averageUpdaters, --dataSetIteratorFactoryClazz, --multiDataSetIteratorFactoryClazz,
--modelOutputPath, --uiUrl). Run one process per GPU:

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m deeplearning4j_amd.parallel.main \\
        --modelPath model.zip --dataSetIteratorFactoryClazz mypkg.data:make_iterator --modelOutputPath out.zip

The iterator factory is ``module:callable`` returning a DataSetIterator (the Java factory-class contract).
"""
import argparse
import importlib
import logging

log = logging.getLogger("deeplearning4j_amd")


def _factory(spec):
    """``module:callable`` returning an iterator, or ``module:Class`` of a provider factory whose create() returns
    one (the reference's DataSetIteratorProviderFactory / MultiDataSetProviderFactory classes)."""
    mod, _, fn = spec.partition(":")
    obj = getattr(importlib.import_module(mod), fn or "create")
    obj = obj() if callable(obj) else obj
    if hasattr(obj, "create") and not hasattr(obj, "__iter__") and not hasattr(obj, "next"):
        obj = obj.create()
    return obj


def main(argv=None):
    ap = argparse.ArgumentParser("ParallelWrapperMain")
    ap.add_argument("--modelPath", required=True)
    ap.add_argument("--workers", type=int, default=None)
    ap.add_argument("--prefetchSize", type=int, default=16)
    ap.add_argument("--averagingFrequency", type=int, default=1)
    ap.add_argument("--reportScore", type=lambda s: s.lower() == "true", default=False)
    ap.add_argument("--averageUpdaters", type=lambda s: s.lower() != "false", default=True)
    ap.add_argument("--legacyAveraging", type=lambda s: s.lower() == "true", default=False)
    ap.add_argument("--trainingMode", default="SHARED_GRADIENTS", choices=["SHARED_GRADIENTS", "AVERAGING"])
    ap.add_argument("--dataSetIteratorFactoryClazz", default=None)
    ap.add_argument("--multiDataSetIteratorFactoryClazz", default=None)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--modelOutputPath", default=None)
    ap.add_argument("--uiUrl", default=None)
    a = ap.parse_args(argv)
    if not (a.dataSetIteratorFactoryClazz or a.multiDataSetIteratorFactoryClazz):
        ap.error("one of --dataSetIteratorFactoryClazz / --multiDataSetIteratorFactoryClazz is required")
    from ..utils.model_serializer import ModelSerializer
    from .distributed import init_distributed, rank
    from .wrapper import ParallelWrapper, TrainingMode
    world, r, _, device = init_distributed()
    net = ModelSerializer.restoreModel(a.modelPath, device=device)
    if a.uiUrl:
        from ..ui import RemoteUIStatsStorageRouter, StatsListener
        url = a.uiUrl if a.uiUrl.startswith("http") else "http://" + a.uiUrl
        net.addListeners(StatsListener(RemoteUIStatsStorageRouter(url)))
    it = _factory(a.dataSetIteratorFactoryClazz or a.multiDataSetIteratorFactoryClazz)
    pw = (ParallelWrapper.Builder(net).workers(a.workers or world).prefetchBuffer(a.prefetchSize)
          .averagingFrequency(a.averagingFrequency).reportScoreAfterAveraging(a.reportScore)
          .averageUpdaters(a.averageUpdaters).trainingMode(TrainingMode(a.trainingMode)).build())
    pw.fit(it, a.epochs)
    if a.modelOutputPath and rank() == 0:
        ModelSerializer.writeModel(net, a.modelOutputPath, True)
        log.info("model written to %s", a.modelOutputPath)
    return net


if __name__ == "__main__":
    main()
