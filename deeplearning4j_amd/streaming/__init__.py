"""Streaming / serving (replacement for dl4j-streaming): NDArray pub/sub routes, record converters and
the model-serving route, plus an HTTP model server.

Reference: ``NDArrayPubSubRoute`` / ``NDArrayPublisher`` / ``NDArrayConsumer`` move base64-encoded ``Nd4j.write``
arrays over Kafka topics through Camel (STRM:kafka/*); ``DL4jServeRouteBuilder`` consumes arrays from a topic,
restores a ModelSerializer zip, runs ``output`` and publishes the result (STRM:routes/DL4jServeRouteBuilder.java:
48-92); ``CSVRecordToINDArray`` / ``CSVRecordToDataSet`` convert DataVec records (STRM:conversion/*).

Topics are served either by an in-process :class:`Broker` (thread-safe, many producers / consumers per topic) or by
a Kafka cluster through :class:`~deeplearning4j_amd.streaming.kafka.KafkaBroker`, which speaks the Kafka wire
protocol itself (no client library in the image; ``streaming/kafka.py``). Either way the message format is the
reference's: base64 of the ND4J binary array codec, so payloads interoperate. :class:`ModelServer` exposes the same serve route over HTTP
(FastAPI) with dynamic batching through :class:`~deeplearning4j_amd.parallel.ParallelInference` on the GPU.
"""
import base64
import queue
import threading

import numpy as np
import torch

from ..utils import nd4j_io


# ------------------------------------------------------------------------------------------------ serde
class NDArrayType:
    """Base64 <-> array (the Kafka message body of the reference's NDArrayType)."""

    @staticmethod
    def toBase64(arr):
        t = torch.as_tensor(arr).detach().cpu()
        return base64.b64encode(nd4j_io.to_bytes(t)).decode("ascii")

    @staticmethod
    def fromBase64(s):
        return nd4j_io.from_bytes(base64.b64decode(s))


# ------------------------------------------------------------------------------------------------ broker
class Broker:
    """In-process topic broker: every subscriber of a topic gets every message published after it subscribed."""

    def __init__(self):
        self._subs = {}
        self._lock = threading.Lock()

    def subscribe(self, topic, maxsize=0):
        q = queue.Queue(maxsize)
        with self._lock:
            self._subs.setdefault(topic, []).append(q)
        return q

    def unsubscribe(self, topic, q):
        with self._lock:
            if q in self._subs.get(topic, []):
                self._subs[topic].remove(q)

    def publish(self, topic, message):
        with self._lock:
            subs = list(self._subs.get(topic, []))
        for q in subs:
            q.put(message)
        return len(subs)


_default_broker = Broker()


def KafkaBroker(bootstrap, **kw):
    """A Broker over a Kafka cluster (``"host:port[,host:port]"``); see ``streaming/kafka.py``."""
    from .kafka import KafkaBroker as _K
    return _K(bootstrap, **kw)


def default_broker():
    return _default_broker


class NDArrayPublisher:
    def __init__(self, topic, broker=None):
        self.topic = topic
        self.broker = broker or _default_broker

    def publish(self, arr):
        arrs = arr if isinstance(arr, (list, tuple)) else [arr]
        for a in arrs:
            self.broker.publish(self.topic, NDArrayType.toBase64(a))


class NDArrayConsumer:
    def __init__(self, topic, broker=None):
        self.topic = topic
        self.broker = broker or _default_broker
        self._q = self.broker.subscribe(topic)

    def getArrays(self, n=1, timeout=10.0):
        return [NDArrayType.fromBase64(self._q.get(timeout=timeout)) for _ in range(n)]

    def getINDArray(self, timeout=10.0):
        return self.getArrays(1, timeout)[0]

    def close(self):
        self.broker.unsubscribe(self.topic, self._q)


class _Route:
    """A consumer thread: take a message from ``src``, apply ``process``, publish to ``dst``."""

    def __init__(self, broker, src, dst, process):
        self.broker, self.src, self.dst, self.process = broker, src, dst, process
        self._q = broker.subscribe(src)
        self._stop = threading.Event()
        self._t = None
        self.processed = 0
        self.errors = []

    def start(self):
        self._t = threading.Thread(target=self._run, daemon=True, name=f"route-{self.src}")
        self._t.start()
        return self

    def _run(self):
        while not self._stop.is_set():
            try:
                msg = self._q.get(timeout=0.05)
            except queue.Empty:
                continue
            try:
                out = self.process(msg)
                if out is not None and self.dst is not None:
                    self.broker.publish(self.dst, out)
                self.processed += 1
            except Exception as e:  # noqa: BLE001 - a bad message must not kill the route
                self.errors.append(e)

    def stop(self):
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2.0)
        self.broker.unsubscribe(self.src, self._q)


class NDArrayPubSubRoute:
    """Route arrays from ``publishTopic`` to ``subscribeTopic``, optionally transforming each array."""

    def __init__(self, publishTopic, subscribeTopic, transform=None, broker=None):
        self.broker = broker or _default_broker
        fn = transform or (lambda a: a)
        self.route = _Route(self.broker, publishTopic, subscribeTopic,
                            lambda m: NDArrayType.toBase64(fn(NDArrayType.fromBase64(m))))

    def start(self):
        self.route.start()
        return self

    def stop(self):
        self.route.stop()


# ------------------------------------------------------------------------------------------------ converters
class RecordToNDArray:
    def convert(self, records):
        raise NotImplementedError


class CSVRecordToINDArray(RecordToNDArray):
    """List of CSV records (lists of numbers or strings) -> [n, cols] float array."""

    def convert(self, records):
        rows = [[float(v) for v in (r.split(",") if isinstance(r, str) else r)] for r in records]
        return torch.tensor(rows, dtype=torch.float32)


class NDArrayRecordToNDArray(RecordToNDArray):
    def convert(self, records):
        return torch.cat([torch.as_tensor(r).reshape(1, -1).float() for r in records], dim=0)


class RecordToDataSet:
    def convert(self, records, numLabels):
        raise NotImplementedError


class CSVRecordToDataSet(RecordToDataSet):
    """CSV records whose LAST column is the class index -> DataSet(features, one-hot labels)."""

    def convert(self, records, numLabels):
        from ..datasets import DataSet
        m = CSVRecordToINDArray().convert(records)
        x, cls = m[:, :-1], m[:, -1].long()
        y = torch.zeros(m.shape[0], numLabels)
        y[torch.arange(m.shape[0]), cls] = 1.0
        return DataSet(x, y)


# ------------------------------------------------------------------------------------------------ serve route
def _load_model(modelUri, device=None):
    from ..utils.model_serializer import ModelSerializer
    return ModelSerializer.restoreModel(modelUri, False, device)


def _model_output(model, x):
    from ..nn.graph import ComputationGraph
    with torch.no_grad():
        out = model.output(x)
    if isinstance(model, ComputationGraph) or isinstance(out, (list, tuple)):
        out = out[0]
    return out.float().cpu()


class DL4jServeRouteBuilder:
    """Builder for the serving route: consume base64 arrays from ``consumingTopic``, run the restored model, publish
    base64 outputs to ``outputTopic`` (STRM:routes/DL4jServeRouteBuilder.java:48-92). Fluent setters:
    ``modelUri``, ``model``, ``consumingTopic``, ``outputTopic``, ``beforeProcessor``, ``finalProcessor``,
    ``broker``, ``device``."""

    _KEYS = ("modelUri", "model", "consumingTopic", "outputTopic", "beforeProcessor", "finalProcessor", "broker",
             "device")

    def __init__(self):
        self._cfg = {"consumingTopic": "input", "outputTopic": "output"}

    def __getattr__(self, name):
        if name not in DL4jServeRouteBuilder._KEYS:
            raise AttributeError(name)

        def setter(v):
            self._cfg[name] = v
            return self
        return setter

    def build(self):
        c = self._cfg
        model = c.get("model") or _load_model(c["modelUri"], c.get("device"))
        before, final = c.get("beforeProcessor"), c.get("finalProcessor")

        def process(msg):
            x = NDArrayType.fromBase64(msg)
            if before is not None:
                x = before(x)
            out = _model_output(model, x)
            if final is not None:
                out = final(out)
            return NDArrayType.toBase64(out)
        return _Route(c.get("broker") or _default_broker, c["consumingTopic"], c["outputTopic"], process)


# ------------------------------------------------------------------------------------------------ HTTP server
class ModelServer:
    """HTTP serving of a model: ``POST /predict`` with ``{"ndarray": <base64 Nd4j>}`` or ``{"array": [[...]]}``;
    responses carry both encodings. Requests are batched dynamically by ParallelInference (BATCHED mode)."""

    def __init__(self, model, batchLimit=64, workers=1, maxLatencyMs=2):
        from ..parallel import InferenceMode, ParallelInference
        self.model = model
        self.pi = ParallelInference.Builder(model).inferenceMode(InferenceMode.BATCHED).batchLimit(batchLimit) \
            .workers(workers).maxLatencyMs(maxLatencyMs).build()
        self.app = self._make_app()

    def _make_app(self):
        from fastapi import FastAPI, HTTPException
        app = FastAPI(title="deeplearning4j_amd model server")
        pi = self.pi

        @app.get("/health")
        def health():
            return {"status": "ok"}

        @app.post("/predict")
        def predict(body: dict):
            if "ndarray" in body:
                x = NDArrayType.fromBase64(body["ndarray"])
            elif "array" in body:
                x = torch.as_tensor(np.asarray(body["array"], dtype=np.float32))
            else:
                raise HTTPException(status_code=400, detail="expected 'ndarray' (base64) or 'array'")
            out = pi.output(x)
            if isinstance(out, (list, tuple)):
                out = out[0]
            out = torch.as_tensor(out).float().cpu()
            return {"array": out.tolist(), "ndarray": NDArrayType.toBase64(out)}
        return app

    def serve(self, host="127.0.0.1", port=9008):
        import uvicorn
        uvicorn.run(self.app, host=host, port=port, log_level="warning")

    def shutdown(self):
        self.pi.shutdown()

