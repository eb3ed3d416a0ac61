"""In-process entry to node-level data parallelism (reference PW:ParallelWrapper.java:123-137 — N workers pinned to
N devices inside one JVM — and :467-565, the fit loop).

MI355X design: one process per GPU over RCCL. When ``ParallelWrapper.Builder(net).workers(N).build().fit(data)``
is called from a single ordinary Python process (no process group, N > 1), the wrapper launches N FRESH child
interpreters (``python -m deeplearning4j_amd.parallel.launcher <dir>``; nothing is forked from a process that may
already hold GPU state, nothing re-execs the parent), each pinned to one GPU, and hands them:

  * the model as a ModelSerializer ZIP (configuration + parameters + updater state),
  * the training data as CPU tensors (``torch.save`` of plain tensor lists, loaded back with weights_only=True),
  * the wrapper settings as JSON.

The children run the same ParallelWrapper.fit under torch.distributed (rank-strided data, bucketed all-reduce or
parameter averaging), rank 0 writes the trained model back, and the parent copies parameters and updater state
into the caller's network — from the caller's point of view ``fit`` trained its model on N GPUs. Backend: nccl
(RCCL over xGMI) with one GPU per worker, gloo on CPU (tests / rehearsal).
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import torch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(source):
    from ..datasets.dataset import DataSet, MultiDataSet
    if isinstance(source, (DataSet, MultiDataSet)):
        items = [source]
    elif isinstance(source, (list, tuple)):
        items = list(source)
    else:
        if hasattr(source, "reset"):
            source.reset()
        items = []
        while source.hasNext():
            items.append(source.next())
    out = []
    for ds in items:
        if isinstance(ds, MultiDataSet):
            out.append({"multi": True, "f": [t.cpu() for t in ds.features], "l": [t.cpu() for t in ds.labels],
                        "fm": [None if t is None else t.cpu() for t in (ds.featuresMasks or [])],
                        "lm": [None if t is None else t.cpu() for t in (ds.labelsMasks or [])]})
        else:
            out.append({"multi": False, "f": [ds.features.cpu()], "l": [ds.labels.cpu()],
                        "fm": [None if ds.featuresMask is None else ds.featuresMask.cpu()],
                        "lm": [None if ds.labelsMask is None else ds.labelsMask.cpu()]})
    return out


def _to_datasets(raw):
    from ..datasets.dataset import DataSet, MultiDataSet
    res = []
    for r in raw:
        if r["multi"]:
            res.append(MultiDataSet(r["f"], r["l"], r["fm"] or None, r["lm"] or None))
        else:
            res.append(DataSet(r["f"][0], r["l"][0], r["fm"][0], r["lm"][0]))
    return res


def spawn_fit(wrapper, source, numEpochs=1, timeout_s=None):
    """Train ``wrapper.model`` with ``wrapper.workers`` child processes; returns the (updated) model."""
    from ..utils.model_serializer import ModelSerializer
    W = int(wrapper.workers)
    m = wrapper.model
    if not m.initCalled:
        m.init()
    ngpu = torch.cuda.device_count() if torch.cuda.is_available() else 0
    backend = os.environ.get("DL4J_AMD_DIST_BACKEND") or ("nccl" if ngpu >= W else "gloo")
    work = tempfile.mkdtemp(prefix="dl4j_pw_")
    ModelSerializer.writeModel(m, os.path.join(work, "model.zip"), True)
    torch.save(_batches(source), os.path.join(work, "data.pt"))
    cfg = {"workers": W, "trainingMode": wrapper.trainingMode.value, "averagingFrequency": wrapper.averagingFrequency,
           "averageUpdaters": wrapper.averageUpdaters, "bucket_mb": wrapper.bucket_mb, "numEpochs": int(numEpochs),
           "backend": backend, "kind": type(m).__name__}
    with open(os.path.join(work, "config.json"), "w") as f:
        json.dump(cfg, f)
    port = _free_port()
    procs = []
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for r in range(W):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(W), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DL4J_AMD_DIST_BACKEND=backend,
                   PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
        if backend == "gloo":
            env.setdefault("OMP_NUM_THREADS", "1")
        procs.append(subprocess.Popen([sys.executable, "-m", "deeplearning4j_amd.parallel.launcher", work], env=env))
    failed = None
    try:
        for r, p in enumerate(procs):
            rc = p.wait(timeout=timeout_s)
            if rc != 0 and failed is None:
                failed = (r, rc)
                for q in procs:
                    if q.poll() is None:
                        q.kill()
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    if failed is not None:
        raise RuntimeError(f"ParallelWrapper worker {failed[0]} exited with code {failed[1]} (work dir {work})")
    trained = ModelSerializer.restoreModel(os.path.join(work, "out.zip"), True, device=m.device)
    with torch.no_grad():
        m.flattenedParams.copy_(trained.flattenedParams.to(m.flattenedParams.device))
        us, ts = getattr(m.updater, "state", None), getattr(trained.updater, "state", None)
        if us is not None and ts is not None and us.numel() == ts.numel():
            us.copy_(ts.to(us.device))
        m.sync_shadow()
    m.conf.iterationCount = trained.conf.iterationCount
    m.conf.epochCount = trained.conf.epochCount
    if hasattr(m, "_bump_weight_version"):
        m._bump_weight_version()
    return m


def _worker(work):
    from ..utils.model_serializer import ModelSerializer
    from .distributed import destroy, init_distributed, rank
    from .wrapper import ParallelWrapper, TrainingMode
    with open(os.path.join(work, "config.json")) as f:
        cfg = json.load(f)
    if cfg["backend"] == "gloo":
        torch.set_num_threads(1)
    world, r, local, device = init_distributed(backend=cfg["backend"])
    if cfg["backend"] == "gloo":
        device = torch.device("cpu")
    net = ModelSerializer.restoreModel(os.path.join(work, "model.zip"), True, device=device)
    data = _to_datasets(torch.load(os.path.join(work, "data.pt"), weights_only=True))
    pw = ParallelWrapper(net, workers=cfg["workers"], trainingMode=TrainingMode(cfg["trainingMode"]),
                         averagingFrequency=cfg["averagingFrequency"], averageUpdaters=cfg["averageUpdaters"],
                         bucket_mb=cfg["bucket_mb"])
    pw.fit(data, cfg["numEpochs"])
    if rank() == 0:
        ModelSerializer.writeModel(net, os.path.join(work, "out.zip"), True)
    destroy()


if __name__ == "__main__":
    _worker(sys.argv[1])
