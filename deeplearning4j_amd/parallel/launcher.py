"""Process-per-device entry to node-level data parallelism (opt-in: ``ParallelWrapper.Builder.inProcess(False)`` or
DL4J_AMD_PW_SPAWN=1; the default is the in-process thread-per-device trainer, parallel/inprocess.py).

Reference: PW:ParallelWrapper.java:123-137 (N workers pinned to N devices) and :467-565 (the fit loop: the master
hands DataSets round-robin to the workers). Here the workers are N FRESH child interpreters
(``python -m deeplearning4j_amd.parallel.launcher <dir>``; nothing is forked from a process that may hold GPU state,
nothing re-execs the parent), one per GPU, in one torch.distributed group (nccl = RCCL over xGMI, gloo on CPU).

  * the model goes to the children once, as a ModelSerializer ZIP (configuration + parameters + updater state);
  * the data is STREAMED: the parent pulls complete rounds of N batches from the caller's iterator and sends batch i
    of each round to child i over a local socket (length-prefixed ``torch.save`` frames, loaded back with
    weights_only=True). A child's socket buffer is the only backlog, so the parent never holds more than one round
    however long the iterator is;
  * the parent polls EVERY child while streaming and while waiting: the first non-zero exit kills the others and
    raises (a crashed rank can no longer leave the parent blocked on another rank's collective);
  * rank 0 writes the trained model back; the parent copies parameters, updater state, iteration / epoch counts and
    the last score into the caller's network and removes the work directory.
Listeners attached to the caller's model do not run in the children (a warning says so); use the in-process mode
for listener-driven training.
"""
import io
import json
import logging
import os
import shutil
import socket
import struct
import subprocess
import sys
import tempfile
import time

import torch

log = logging.getLogger("deeplearning4j_amd")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ---------------------------------------------------------------------------------------------- wire format
def _pack(ds):
    from ..datasets.dataset import MultiDataSet
    if isinstance(ds, MultiDataSet):
        d = {"multi": True, "f": [t.cpu() for t in ds.features], "l": [t.cpu() for t in ds.labels],
             "fm": [None if t is None else t.cpu() for t in (ds.featuresMasks or [])],
             "lm": [None if t is None else t.cpu() for t in (ds.labelsMasks or [])]}
    else:
        d = {"multi": False, "f": [ds.features.cpu()], "l": [ds.labels.cpu()],
             "fm": [None if ds.featuresMask is None else ds.featuresMask.cpu()],
             "lm": [None if ds.labelsMask is None else ds.labelsMask.cpu()]}
    buf = io.BytesIO()
    torch.save(d, buf)
    return buf.getvalue()


def _unpack(b):
    from ..datasets.dataset import DataSet, MultiDataSet
    r = torch.load(io.BytesIO(b), weights_only=True)
    if r["multi"]:
        return MultiDataSet(r["f"], r["l"], r["fm"] or None, r["lm"] or None)
    return DataSet(r["f"][0], r["l"][0], r["fm"][0], r["lm"][0])


def _send(sock, kind, payload=b""):
    sock.sendall(kind + struct.pack("<Q", len(payload)) + payload)


def _recv_exact(sock, n):
    out = bytearray()
    while len(out) < n:
        chunk = sock.recv(min(1 << 20, n - len(out)))
        if not chunk:
            raise ConnectionError("ParallelWrapper feed closed")
        out += chunk
    return bytes(out)


def _recv(sock):
    hdr = _recv_exact(sock, 9)
    kind, n = hdr[:1], struct.unpack("<Q", hdr[1:])[0]
    return kind, (_recv_exact(sock, n) if n else b"")


class SocketFeed:
    """A child's view of the stream: iterating yields this rank's batches of one epoch (until the epoch marker)."""

    def __init__(self, sock):
        self.sock = sock
        self.done = False

    def __iter__(self):
        while True:
            kind, payload = _recv(self.sock)
            if kind == b"B":
                yield _unpack(payload)
            elif kind == b"E":
                return
            else:                                   # b"Q": no more epochs
                self.done = True
                return


# ---------------------------------------------------------------------------------------------- parent
def spawn_fit(wrapper, source, numEpochs=1, timeout_s=None):
    """Train ``wrapper.model`` with ``wrapper.workers`` child processes; returns the (updated) model."""
    from ..utils.model_serializer import ModelSerializer
    from .inprocess import _rounds
    W = int(wrapper.workers)
    m = wrapper.model
    if not m.initCalled:
        m.init()
    if m.listeners:
        log.warning("ParallelWrapper (process per device): listeners of the caller's model do not run in the worker "
                    "processes; use inProcess(True) for listener-driven training")
    ngpu = torch.cuda.device_count() if torch.cuda.is_available() else 0
    backend = os.environ.get("DL4J_AMD_DIST_BACKEND") or ("nccl" if ngpu >= W else "gloo")
    work = tempfile.mkdtemp(prefix="dl4j_pw_")
    procs, conns = [], []
    srv = socket.socket()
    try:
        ModelSerializer.writeModel(m, os.path.join(work, "model.zip"), True)
        srv.bind(("127.0.0.1", 0))
        srv.listen(W)
        srv.settimeout(1.0)
        feed_port = srv.getsockname()[1]
        cfg = {"workers": W, "trainingMode": wrapper.trainingMode.value,
               "averagingFrequency": wrapper.averagingFrequency, "averageUpdaters": wrapper.averageUpdaters,
               "bucket_mb": wrapper.bucket_mb, "numEpochs": int(numEpochs), "backend": backend,
               "kind": type(m).__name__, "feed_port": feed_port}
        with open(os.path.join(work, "config.json"), "w") as f:
            json.dump(cfg, f)
        port = _free_port()
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        for r in range(W):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(W), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port), DL4J_AMD_DIST_BACKEND=backend,
                       PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
            if backend == "gloo":
                env.setdefault("OMP_NUM_THREADS", "1")
            procs.append(subprocess.Popen([sys.executable, "-m", "deeplearning4j_amd.parallel.launcher", work],
                                          env=env))
        conns = [None] * W
        t0 = time.time()
        while any(c is None for c in conns):
            _check_children(procs)
            if timeout_s is not None and time.time() - t0 > timeout_s:
                raise TimeoutError("ParallelWrapper workers did not connect")
            try:
                c, _ = srv.accept()
            except socket.timeout:
                continue
            c.settimeout(None)
            r = struct.unpack("<I", _recv_exact(c, 4))[0]
            conns[r] = c
        for _ in range(int(numEpochs)):
            for rnd in _rounds(source, W):
                _check_children(procs)
                for i, ds in enumerate(rnd):
                    _send(conns[i], b"B", _pack(ds))
            for c in conns:
                _send(c, b"E")
        for c in conns:
            _send(c, b"Q")
        while any(p.poll() is None for p in procs):
            _check_children(procs)
            time.sleep(0.05)
        _check_children(procs)
        trained = ModelSerializer.restoreModel(os.path.join(work, "out.zip"), True, device=m.device)
        with torch.no_grad():
            m.flattenedParams.copy_(trained.flattenedParams.to(m.flattenedParams.device))
            us, ts = getattr(m.updater, "state", None), getattr(trained.updater, "state", None)
            if us is not None and ts is not None and us.numel() == ts.numel():
                us.copy_(ts.to(us.device))
            m.sync_shadow()
        m.conf.iterationCount = trained.conf.iterationCount
        m.conf.epochCount = trained.conf.epochCount
        score_path = os.path.join(work, "score.json")
        if os.path.exists(score_path):
            with open(score_path) as f:
                m.setScore(json.load(f)["score"])
        if hasattr(m, "_bump_weight_version"):
            m._bump_weight_version()
        return m
    finally:
        for c in conns:
            if c is not None:
                c.close()
        srv.close()
        for q in procs:
            if q.poll() is None:
                q.kill()
                q.wait()
        shutil.rmtree(work, ignore_errors=True)


def _check_children(procs):
    for r, p in enumerate(procs):
        rc = p.poll()
        if rc is not None and rc != 0:
            for q in procs:
                if q.poll() is None:
                    q.kill()
            raise RuntimeError(f"ParallelWrapper worker {r} exited with code {rc}")


# ---------------------------------------------------------------------------------------------- child
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
    sock = socket.create_connection(("127.0.0.1", cfg["feed_port"]))
    sock.sendall(struct.pack("<I", r))
    net = ModelSerializer.restoreModel(os.path.join(work, "model.zip"), True, device=device)
    pw = ParallelWrapper(net, workers=cfg["workers"], trainingMode=TrainingMode(cfg["trainingMode"]),
                         averagingFrequency=cfg["averagingFrequency"], averageUpdaters=cfg["averageUpdaters"],
                         bucket_mb=cfg["bucket_mb"])
    feed = SocketFeed(sock)
    pw.fit(feed, cfg["numEpochs"], presharded=True)
    if not feed.done:
        _recv(sock)                                 # the final quit frame
    if rank() == 0:
        ModelSerializer.writeModel(net, os.path.join(work, "out.zip"), True)
        with open(os.path.join(work, "score.json"), "w") as f:
            json.dump({"score": float(net.score())}, f)
    sock.close()
    destroy()


if __name__ == "__main__":
    _worker(sys.argv[1])
