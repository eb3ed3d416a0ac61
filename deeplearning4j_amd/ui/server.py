"""Training UI server.

Reference: PLAY:play/PlayUIServer.java (UIServer.getInstance(), attach/detach StatsStorage, enableRemoteListener,
port flag / org.deeplearning4j.ui.port), modules train (overview: score vs iteration, update:parameter ratios,
examples/sec; model: per-layer parameter/update stats and histograms; system: memory and hardware/software info),
tsne (upload and view coordinates) and remote receiver (RemoteReceiverModule: POST records from
RemoteUIStatsStorageRouter). Stdlib threaded HTTP server serving JSON APIs plus one self-contained HTML page
(inline SVG charts; no external assets, the box has no network).
"""
import json
import math
import os
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .storage import InMemoryStatsStorage, Persistable, StatsStorageEvent
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


_PAGE = """<!doctype html><html><head><meta charset="utf-8"><title>DL4J-AMD Training UI</title>
<style>body{font-family:sans-serif;margin:16px;background:#fafafa}h2{margin:8px 0}.c{background:#fff;border:1px solid
#ddd;padding:8px;margin:8px 0}svg{background:#fff}table{border-collapse:collapse}td,th{border:1px solid #ddd;
padding:2px 6px;font-size:12px}</style></head><body>
<h2>Training overview</h2><div>Session: <select id="sid"></select></div>
<div class="c"><b>Score vs iteration</b><div id="score"></div></div>
<div class="c"><b>log10(update : parameter) mean magnitude ratio</b><div id="ratio"></div></div>
<div class="c"><b>Examples / second</b><div id="perf"></div></div>
<div class="c"><b>Model (latest report)</b><div id="model"></div></div>
<div class="c"><b>System</b><pre id="sys"></pre></div>
<script>
function line(el, series, w, h){var xs=[],ys=[];series.forEach(function(s){s.pts.forEach(function(p){if(p[1]!=null){
xs.push(p[0]);ys.push(p[1]);}})});if(!xs.length){el.innerHTML='(no data)';return;}var x0=Math.min.apply(null,xs),
x1=Math.max.apply(null,xs),y0=Math.min.apply(null,ys),y1=Math.max.apply(null,ys);if(x1==x0)x1=x0+1;if(y1==y0)y1=y0+1;
var svg='<svg width="'+w+'" height="'+h+'">';var cols=['#1f77b4','#ff7f0e','#2ca02c','#d62728','#9467bd','#8c564b'];
series.forEach(function(s,i){var d=s.pts.filter(function(p){return p[1]!=null}).map(function(p){return ((p[0]-x0)/(x1-x0)
*(w-50)+40).toFixed(1)+','+(h-20-(p[1]-y0)/(y1-y0)*(h-30)).toFixed(1)}).join(' ');svg+='<polyline fill="none" stroke="'+
cols[i%cols.length]+'" points="'+d+'"/>';});svg+='<text x="2" y="12" font-size="10">'+y1.toPrecision(4)+'</text><text x="2"'
+' y="'+(h-22)+'" font-size="10">'+y0.toPrecision(4)+'</text></svg>';el.innerHTML=svg;}
function load(){var sid=document.getElementById('sid').value;fetch('api/overview?sid='+sid).then(function(r){return r.json()})
.then(function(d){line(document.getElementById('score'),[{pts:d.score}],700,220);var rs=[];for(var k in d.updateRatios)
rs.push({pts:d.updateRatios[k]});line(document.getElementById('ratio'),rs,700,220);line(document.getElementById('perf'),
[{pts:d.performance}],700,160);});fetch('api/model?sid='+sid).then(function(r){return r.json()}).then(function(d){
if(!d.latest){return;}var t='<table><tr><th>param</th><th>mean</th><th>stdev</th><th>mean |x|</th><th>update mean |x|</th>'
+'</tr>';var P=d.latest.stats.Parameters,U=d.latest.stats.Updates||{};for(var k in P){t+='<tr><td>'+k+'</td><td>'+
(P[k].mean||0).toExponential(3)+'</td><td>'+(P[k].stdev||0).toExponential(3)+'</td><td>'+(P[k].meanMagnitude||0)
.toExponential(3)+'</td><td>'+((U[k]||{}).meanMagnitude||0).toExponential(3)+'</td></tr>';}document.getElementById('model')
.innerHTML='iteration '+d.latest.iteration+t+'</table>';});fetch('api/system?sid='+sid).then(function(r){return r.json()})
.then(function(d){document.getElementById('sys').textContent=JSON.stringify(d.workers,null,1);});}
fetch('api/sessions').then(function(r){return r.json()}).then(function(s){var e=document.getElementById('sid');
s.forEach(function(x){var o=document.createElement('option');o.value=x;o.text=x;e.appendChild(o);});e.onchange=load;
load();setInterval(load,5000);});
</script></body></html>"""


class UIServer:
    _instance = None
    _lock = threading.Lock()

    def __init__(self, port=None):
        self.port = int(port if port is not None else os.environ.get("ORG_DEEPLEARNING4J_UI_PORT", 9000))
        self.storages = []
        self.remote_storage = None
        self.tsne = {}
        self.httpd = None

    @staticmethod
    def getInstance(port=None):
        with UIServer._lock:
            if UIServer._instance is None:
                UIServer._instance = UIServer(port).start()
            return UIServer._instance

    def attach(self, storage):
        if storage not in self.storages:
            self.storages.append(storage)

    def detach(self, storage):
        self.storages = [s for s in self.storages if s is not storage]

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

            def _send(self, code, body, ctype="application/json"):
                b = body if isinstance(body, bytes) else (body.encode() if isinstance(body, str) else
                                                          json.dumps(body).encode())
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def do_GET(self):
                u = urllib.parse.urlparse(self.path)
                q = dict(urllib.parse.parse_qsl(u.query))
                path = u.path.rstrip("/") or "/"
                if path in ("/", "/train", "/train/overview"):
                    return self._send(200, _PAGE, "text/html; charset=utf-8")
                if path == "/api/sessions":
                    return self._send(200, [s for s, _ in _sessions(ui.storages)])
                if path == "/api/tsne":
                    return self._send(200, ui.tsne)
                st = ui._find(q.get("sid", ""))
                if st is None:
                    return self._send(404, {"error": "unknown session"})
                if path == "/api/overview":
                    return self._send(200, overview(st, q["sid"]))
                if path == "/api/model":
                    return self._send(200, model_view(st, q["sid"], q.get("param")))
                if path == "/api/system":
                    return self._send(200, system_view(st, q["sid"]))
                return self._send(404, {"error": "not found"})

            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0))
                raw = self.rfile.read(n)
                if self.path == "/remoteReceive":
                    if ui.remote_storage is None:
                        return self._send(403, {"error": "remote listener not enabled"})
                    try:
                        msg = json.loads(raw)
                        r = Persistable.decode(json.dumps(msg["record"]))
                        {"meta": ui.remote_storage.putStorageMetaData, "static": ui.remote_storage.putStaticInfo,
                         "update": ui.remote_storage.putUpdate}[msg["type"]](r)
                        return self._send(200, {"status": "ok"})
                    except (KeyError, ValueError) as e:
                        return self._send(400, {"error": str(e)})
                if self.path.startswith("/tsne/upload"):
                    name = dict(urllib.parse.parse_qsl(urllib.parse.urlparse(self.path).query)).get("name", "upload")
                    rows = []
                    for line in raw.decode("utf-8").splitlines():
                        p = line.strip().split(",")
                        if len(p) >= 3:
                            rows.append([float(p[0]), float(p[1]), ",".join(p[2:]).strip()])
                    ui.tsne[name] = rows
                    return self._send(200, {"status": "ok", "points": len(rows)})
                return self._send(404, {"error": "not found"})
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


_ = StatsStorageEvent
