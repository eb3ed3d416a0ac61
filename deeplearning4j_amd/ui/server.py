"""Training UI server.

Reference: PLAY:play/PlayUIServer.java:53-278 (UIServer.getInstance(), attach/detach StatsStorage,
enableRemoteListener, port flag / org.deeplearning4j.ui.port, the module list and its routes). The server is a stdlib
threaded HTTP server assembled from UI modules (ui/modules.py): train (overview / model / system / help pages, their
JSON data, session + worker selection, language switch), convolutional activations, t-SNE, remote receiver and the
default redirect; plus the flat JSON API (/api/sessions, /api/overview, /api/model, /api/system, /api/tsne).
Attached storages forward their events to the modules that registered for the event's type ID.
"""
import json
import math
import os
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .modules import (ConvolutionalListenerModule, DefaultModule, RemoteReceiverModule, Request, Response,
                      TrainModule, TsneModule)
from .storage import InMemoryStatsStorage, StatsStorageEvent
from .stats import TYPE_ID


def _sessions(storages):
    out = []
    for st in storages:
        for s in st.listSessionIDs():
            out.append((s, st))
    return out


def overview(storage, sid):
    score, perf, ratios, mem = [], [], {}, []
    for w in storage.listWorkerIDsForSessionAndType(sid, TYPE_ID):
        for t in storage.getAllUpdateTimes(sid, TYPE_ID, w):
            r = storage.getUpdate(sid, TYPE_ID, w, t)
            it = r.get("iterationCount")
            score.append([it, r.get("score")])
            p = r.get("performance")
            if p:
                perf.append([it, p.get("examplesPerSecond"), p.get("minibatchesPerSecond")])
            P, U = r.get("Parameters") or {}, r.get("Updates") or {}
            for k in P:
                pm = P[k].get("meanMagnitude")
                um = (U.get(k) or {}).get("meanMagnitude")
                if pm and um is not None and pm > 0 and um > 0:
                    ratios.setdefault(k, []).append([it, math.log10(um / pm)])
            m = r.get("memory")
            if m:
                mem.append([it, m.get("hostCurrentBytes"), (m.get("deviceCurrentBytes") or [None])[0]])
    return {"score": score, "performance": perf, "updateRatios": ratios, "memory": mem}


def model_view(storage, sid, param=None):
    latest = None
    for w in storage.listWorkerIDsForSessionAndType(sid, TYPE_ID):
        r = storage.getLatestUpdate(sid, TYPE_ID, w)
        if r is not None and (latest is None or r.timeStamp > latest.timeStamp):
            latest = r
    static = None
    infos = storage.getAllStaticInfos(sid, TYPE_ID)
    if infos:
        static = infos[0].data.get("model")
    out = {"model": static, "latest": None}
    if latest is not None:
        d = latest.data
        sel = {}
        for st in ("Parameters", "Gradients", "Updates", "Activations"):
            block = d.get(st) or {}
            sel[st] = {k: v for k, v in block.items() if param is None or k == param}
        out["latest"] = {"iteration": d.get("iterationCount"), "stats": sel, "learningRates": d.get("learningRates")}
    return out


def system_view(storage, sid):
    infos = storage.getAllStaticInfos(sid, TYPE_ID)
    return {"workers": [{"worker": i.workerID, "hardware": i.data.get("hardware"),
                         "software": i.data.get("software")} for i in infos],
            "memory": overview(storage, sid)["memory"]}


class UIServer:
    _instance = None
    _lock = threading.Lock()

    def __init__(self, port=None):
        self.port = int(port if port is not None else os.environ.get("ORG_DEEPLEARNING4J_UI_PORT", 9000))
        self.storages = []
        self.remote_storage = None
        self.tsne = {}
        self.httpd = None
        self.modules = [DefaultModule(), TrainModule(self), ConvolutionalListenerModule(self), TsneModule(self),
                        RemoteReceiverModule(self)]
        self._routes = [r for m in self.modules for r in m.getRoutes()]
        self._listeners = {}

    @staticmethod
    def getInstance(port=None):
        with UIServer._lock:
            if UIServer._instance is None:
                UIServer._instance = UIServer(port).start()
            return UIServer._instance

    def attach(self, storage):
        if storage not in self.storages:
            self.storages.append(storage)
            for m in self.modules:
                m.onAttach(storage)
            if hasattr(storage, "registerStatsStorageListener"):
                lst = _ModuleEventRouter(self.modules)
                self._listeners[id(storage)] = lst
                storage.registerStatsStorageListener(lst)

    def detach(self, storage):
        self.storages = [s for s in self.storages if s is not storage]
        lst = self._listeners.pop(id(storage), None)
        if lst is not None and hasattr(storage, "deregisterStatsStorageListener"):
            storage.deregisterStatsStorageListener(lst)
        for m in self.modules:
            m.onDetach(storage)

    def getModules(self):
        return list(self.modules)

    def dispatch(self, method, raw_path, body=b""):
        """Route one request through the modules (then the flat /api endpoints); returns a Response."""
        u = urllib.parse.urlparse(raw_path)
        q = dict(urllib.parse.parse_qsl(u.query))
        path = u.path.rstrip("/") or "/"
        req = Request(method, path, q, body)
        for r in self._routes:
            params = r.match(method, path)
            if params is not None:
                return r.fn(req, params)
        if method == "GET":
            if path == "/api/sessions":
                return Response.ok([s for s, _ in _sessions(self.storages)])
            if path == "/api/tsne":
                return Response.ok(self.tsne)
            if path in ("/api/overview", "/api/model", "/api/system"):
                st = self._find(q.get("sid", ""))
                if st is None:
                    return Response.not_found("unknown session")
                if path == "/api/overview":
                    return Response.ok(overview(st, q["sid"]))
                if path == "/api/model":
                    return Response.ok(model_view(st, q["sid"], q.get("param")))
                return Response.ok(system_view(st, q["sid"]))
        return Response.not_found()

    def isAttached(self, storage):
        return storage in self.storages

    def getStatsStorageInstances(self):
        return list(self.storages)

    def enableRemoteListener(self, storage=None, multiSession=True):
        self.remote_storage = storage or InMemoryStatsStorage()
        self.attach(self.remote_storage)

    def disableRemoteListener(self):
        if self.remote_storage is not None:
            self.detach(self.remote_storage)
        self.remote_storage = None

    def isRemoteListenerEnabled(self):
        return self.remote_storage is not None

    def getAddress(self):
        return f"http://127.0.0.1:{self.port}"

    def getPort(self):
        return self.port

    def _find(self, sid):
        for s, st in _sessions(self.storages):
            if s == sid:
                return st
        return None

    def _handler(self):
        ui = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _serve(self, method):
                n = int(self.headers.get("Content-Length", 0) or 0)
                body = self.rfile.read(n) if n else b""
                r = ui.dispatch(method, self.path, body)
                self.send_response(r.code)
                self.send_header("Content-Type", r.ctype)
                for k, v in r.headers.items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(r.body)))
                self.end_headers()
                self.wfile.write(r.body)

            def do_GET(self):
                self._serve("GET")

            def do_POST(self):
                self._serve("POST")
        return H

    def start(self):
        self.httpd = ThreadingHTTPServer(("127.0.0.1", self.port), self._handler())
        self.port = self.httpd.server_address[1]
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self

    def stop(self):
        if self.httpd is not None:
            self.httpd.shutdown()
            self.httpd.server_close()
            self.httpd = None
        with UIServer._lock:
            if UIServer._instance is self:
                UIServer._instance = None


class _ModuleEventRouter:
    """StatsStorage listener forwarding each event to the modules registered for its type ID."""

    def __init__(self, modules):
        self.modules = modules

    def notify(self, event):
        for m in self.modules:
            if getattr(event, "typeID", None) in m.getCallbackTypeIDs():
                m.reportStorageEvents([event])


_ = StatsStorageEvent
