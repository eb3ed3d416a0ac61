"""ParallelInference: serving with one model replica per GPU and a dynamic batcher
(reference PW:ParallelInference.java:65-440, observers/BatchedInferenceObservable).

Modes:
  * SEQUENTIAL: requests are dealt round-robin to the replicas; each runs them one by one.
  * BATCHED (default): a collector thread coalesces concurrently submitted requests (up to ``batchLimit``
    examples, waiting at most ``maxLatencyMs`` for more) into ONE forward pass, then splits the output back.
Replicas live on cuda:0..N-1 (or the CPU); each worker thread owns one replica and a dedicated HIP stream,
so the GPUs run concurrently while the Python threads only enqueue work. Inputs are staged through
pinned host memory and copied with non_blocking=True. ``output(x)`` blocks and returns the result;
``submit(x)`` returns a Future.
"""
import enum
import queue
import threading
from concurrent.futures import Future

import torch


class InferenceMode(enum.Enum):
    SEQUENTIAL = "SEQUENTIAL"
    BATCHED = "BATCHED"


class _Request:
    __slots__ = ("x", "future", "n")

    def __init__(self, x, fut):
        self.x, self.future, self.n = x, fut, x.shape[0]


class Pair(tuple):
    """(first, second) with the reference's getters (org.nd4j.linalg.primitives.Pair)."""

    def __new__(cls, first, second):
        return super().__new__(cls, (first, second))

    def getFirst(self):
        return self[0]

    def getSecond(self):
        return self[1]


def _rows(a):
    a = torch.as_tensor(a)
    return a.reshape(1, -1) if a.dim() <= 1 else a


class BatchedInferenceObservable:
    """Request batcher of the BATCHED mode as a standalone object (reference PW:inference/observers/
    BatchedInferenceObservable.java): ``addInput(arrays, masks)`` queues one request (rank-1 arrays are single rows);
    ``getInputBatches()`` stacks consecutive requests along dimension 0 into as few batches as possible — a new batch
    starts when an array's trailing shape, the mask layout or the example limit changes — and remembers each batch's
    request range; after the forward passes, ``setOutputBatches([...])`` + ``getOutputs()`` split every batched
    output back into one array list per request, in request order."""

    def __init__(self, batchLimit=None):
        self.batchLimit = batchLimit
        self.inputs = []                      # per request: (list of arrays, list of masks or None)
        self.outputBatchInputArrays = []      # per batch: [first request, last request]
        self.outputBatches = None
        self.counter = 0

    def addInput(self, inputs, masks=None):
        self.inputs.append(([_rows(a) for a in inputs], None if masks is None else [
            None if m is None else _rows(m) for m in masks]))
        self.counter += 1

    def getCounter(self):
        return self.counter

    def setCounter(self, n):
        self.counter = int(n)

    @staticmethod
    def _key(req):
        arrays, masks = req
        return (tuple(tuple(a.shape[1:]) for a in arrays),
                None if masks is None else tuple(None if m is None else tuple(m.shape[1:]) for m in masks))

    def getInputBatches(self):
        out, self.outputBatchInputArrays = [], []
        start = 0
        while start < len(self.inputs):
            key, n, end = self._key(self.inputs[start]), self.inputs[start][0][0].shape[0], start + 1
            while end < len(self.inputs) and self._key(self.inputs[end]) == key:
                m = self.inputs[end][0][0].shape[0]
                if self.batchLimit is not None and n + m > self.batchLimit:
                    break
                n += m
                end += 1
            reqs = self.inputs[start:end]
            feats = [torch.cat([r[0][j] for r in reqs], 0) for j in range(len(reqs[0][0]))]
            masks = None
            if reqs[0][1] is not None:
                masks = [None if reqs[0][1][j] is None else torch.cat([r[1][j] for r in reqs], 0)
                         for j in range(len(reqs[0][1]))]
            out.append(Pair(feats, masks))
            self.outputBatchInputArrays.append([start, end - 1])
            start = end
        return out

    def setOutputBatches(self, batches):
        self.outputBatches = [list(b) for b in batches]

    def getOutputs(self):
        if self.outputBatches is None or len(self.outputBatches) != len(self.outputBatchInputArrays):
            raise RuntimeError("output batches do not match the input batches")
        res = []
        for outs, (a, b) in zip(self.outputBatches, self.outputBatchInputArrays):
            off = 0
            for r in range(a, b + 1):
                n = self.inputs[r][0][0].shape[0]
                res.append([o[off:off + n] for o in outs])
                off += n
        return res[:self.counter] if self.counter else res


class ParallelInference:
    InferenceMode = InferenceMode

    def __init__(self, model, workers=None, inferenceMode=InferenceMode.BATCHED, batchLimit=32, queueLimit=64,
                 maxLatencyMs=2.0, devices=None):
        self.model = model
        if devices is None:
            n = torch.cuda.device_count() if torch.cuda.is_available() else 0
            devices = [torch.device("cuda", i) for i in range(n)] or [torch.device("cpu")]
            if workers:
                devices = [devices[i % len(devices)] for i in range(int(workers))]
        self.devices = devices
        self.mode = inferenceMode
        self.batchLimit, self.maxLatency = int(batchLimit), float(maxLatencyMs) / 1000.0
        self._q = queue.Queue(maxsize=int(queueLimit))
        self._replicas = [self._replica(d) for d in devices]
        self._stop = False
        self._rr = 0
        self._worker_qs = [queue.Queue(maxsize=4) for _ in devices]
        self._threads = [threading.Thread(target=self._worker, args=(i,), daemon=True) for i in range(len(devices))]
        for t in self._threads:
            t.start()
        self._collector = threading.Thread(target=self._collect, daemon=True)
        self._collector.start()

    class Builder:
        def __init__(self, model):
            self._kw = {"model": model}

        def workers(self, n):
            self._kw["workers"] = int(n)
            return self

        def inferenceMode(self, m):
            self._kw["inferenceMode"] = InferenceMode(m) if not isinstance(m, InferenceMode) else m
            return self

        def batchLimit(self, n):
            self._kw["batchLimit"] = int(n)
            return self

        def queueLimit(self, n):
            self._kw["queueLimit"] = int(n)
            return self

        def maxLatencyMs(self, ms):
            self._kw["maxLatencyMs"] = float(ms)
            return self

        def devices(self, d):
            self._kw["devices"] = list(d)
            return self

        def build(self):
            return ParallelInference(**self._kw)

    def _replica(self, device):
        m = self.model
        if getattr(m, "device", None) == device:
            return m
        from ..utils.model_serializer import ModelSerializer
        import io
        buf = io.BytesIO()
        ModelSerializer.writeModel(m, buf, False)
        buf.seek(0)
        return ModelSerializer.restoreModel(buf, False, device=device)

    # ------------------------------------------------------------------ client API
    def submit(self, x):
        fut = Future()
        x = torch.as_tensor(x)
        self._q.put(_Request(x, fut))
        return fut

    def output(self, x):
        return self.submit(x).result()

    def updateModel(self, model):
        """Swap in new weights on every replica (reference ParallelInference.updateModel)."""
        self.model = model
        self._replicas = [self._replica(d) for d in self.devices]

    def shutdown(self):
        self._stop = True
        self._q.put(None)
        for q in self._worker_qs:
            q.put(None)

    # ------------------------------------------------------------------ internals
    def _collect(self):
        import time
        while not self._stop:
            first = self._q.get()
            if first is None:
                break
            batch = [first]
            n = first.n
            if self.mode == InferenceMode.BATCHED:
                deadline = time.perf_counter() + self.maxLatency
                while n < self.batchLimit:
                    rem = deadline - time.perf_counter()
                    if rem <= 0:
                        break
                    try:
                        r = self._q.get(timeout=rem)
                    except queue.Empty:
                        break
                    if r is None:
                        self._stop = True
                        break
                    if n + r.n > self.batchLimit and n > 0:
                        self._dispatch(batch)
                        batch, n = [r], r.n
                        continue
                    batch.append(r)
                    n += r.n
            self._dispatch(batch)

    def _dispatch(self, batch):
        i = self._rr % len(self._worker_qs)
        self._rr += 1
        self._worker_qs[i].put(batch)

    def _worker(self, i):
        dev = self.devices[i]
        stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        while True:
            batch = self._worker_qs[i].get()
            if batch is None:
                break
            try:
                # requests of differing feature shapes go through separate forward passes
                ob = BatchedInferenceObservable()
                for r in batch:
                    ob.addInput([r.x])
                outs = []
                for b in ob.getInputBatches():
                    x = b.getFirst()[0]
                    if dev.type == "cuda":
                        with torch.cuda.device(dev), torch.cuda.stream(stream):
                            xd = x.pin_memory().to(dev, non_blocking=True) if not x.is_cuda else x.to(dev)
                            out = self._replicas[i].output(xd)
                            out = out.to("cpu", non_blocking=False)
                    else:
                        out = self._replicas[i].output(x)
                    outs.append([out])
                ob.setOutputBatches(outs)
                for r, o in zip(batch, ob.getOutputs()):
                    r.future.set_result(o[0])
            except Exception as e:      # deliver the failure to every waiting caller
                for r in batch:
                    if not r.future.done():
                        r.future.set_exception(e)
