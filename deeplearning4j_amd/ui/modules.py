"""UI modules: the route sets the training UI server is assembled from (reference PLAY:api/UIModule.java, Route.java;
PLAY:module/train/TrainModule.java:94-117, module/convolutional/ConvolutionalListenerModule.java:48-50,
module/tsne/TsneModule.java:45-50, module/remote/RemoteReceiverModule.java:58, module/defaultModule/DefaultModule.java:30).

A module lists ``Route(method, pattern, fn)`` entries; ``:name`` path segments are captured into ``params``. Handlers
get a ``Request`` and return a ``Response``. The pages are self-contained HTML (inline SVG charts drawn by a few lines
of script; no external assets, the box has no network) that poll the module's JSON endpoints, labelled through the
i18n provider.
"""
import json
import math
import os
import time
import urllib.parse

from .i18n import DefaultI18N
from .stats import TYPE_ID
from .storage import Persistable


class Request:
    def __init__(self, method, path, query=None, body=b""):
        self.method, self.path, self.query, self.body = method, path, dict(query or {}), body


class Response:
    def __init__(self, code=200, body=b"", ctype="application/json", headers=None):
        self.code, self.ctype, self.headers = code, ctype, dict(headers or {})
        if isinstance(body, bytes):
            self.body = body
        elif isinstance(body, str):
            self.body = body.encode("utf-8")
        else:
            self.body = json.dumps(body).encode("utf-8")

    @staticmethod
    def ok(body, ctype="application/json"):
        """JSON (any value, strings included) unless another content type is given."""
        if ctype == "application/json" and not isinstance(body, bytes):
            body = json.dumps(body)
        return Response(200, body, ctype)

    @staticmethod
    def html(text):
        return Response(200, text, "text/html; charset=utf-8")

    @staticmethod
    def redirect(to):
        return Response(302, b"", "text/plain", {"Location": to})

    @staticmethod
    def not_found(msg="not found"):
        return Response(404, {"error": msg})


class Route:
    def __init__(self, method, pattern, fn):
        self.method, self.pattern, self.fn = method, pattern, fn
        self.parts = [p for p in pattern.split("/") if p]

    def match(self, method, path):
        if method != self.method:
            return None
        segs = [p for p in path.split("/") if p]
        if len(segs) != len(self.parts):
            return None
        params = {}
        for want, got in zip(self.parts, segs):
            if want.startswith(":"):
                params[want[1:]] = urllib.parse.unquote(got)
            elif want != got:
                return None
        return params


class UIModule:
    """A set of routes plus the StatsStorage type IDs whose events the module wants."""

    def getRoutes(self):
        return []

    def getCallbackTypeIDs(self):
        return []

    def reportStorageEvents(self, events):
        pass

    def onAttach(self, storage):
        pass

    def onDetach(self, storage):
        pass


# ------------------------------------------------------------------------------------------------------ shared HTML
_CSS = ("body{font-family:sans-serif;margin:0;background:#fafafa}nav{background:#24323e;padding:6px 12px}"
        "nav a{color:#fff;margin-right:14px;text-decoration:none}nav select{margin-left:8px}main{padding:12px}"
        ".c{background:#fff;border:1px solid #ddd;padding:8px;margin:8px 0}svg{background:#fff}"
        "table{border-collapse:collapse}td,th{border:1px solid #ddd;padding:2px 6px;font-size:12px}"
        ".l{cursor:pointer;color:#1f5fa8}")

_JS_LINE = """function E(s){return String(s).replace(/[&<>"']/g,function(c){return '&#'+c.charCodeAt(0)+';'});}
function line(el,series,w,h){var xs=[],ys=[];series.forEach(function(s){s.pts.forEach(function(p){
if(p[1]!=null&&isFinite(p[1])){xs.push(p[0]);ys.push(p[1]);}})});if(!xs.length){el.innerHTML='(no data)';return;}
var x0=Math.min.apply(null,xs),x1=Math.max.apply(null,xs),y0=Math.min.apply(null,ys),y1=Math.max.apply(null,ys);
if(x1==x0)x1=x0+1;if(y1==y0)y1=y0+1;var svg='<svg width="'+w+'" height="'+h+'">';
var cols=['#1f77b4','#ff7f0e','#2ca02c','#d62728','#9467bd','#8c564b'];series.forEach(function(s,i){
var d=s.pts.filter(function(p){return p[1]!=null&&isFinite(p[1])}).map(function(p){return((p[0]-x0)/(x1-x0)*(w-50)+40)
.toFixed(1)+','+(h-20-(p[1]-y0)/(y1-y0)*(h-30)).toFixed(1)}).join(' ');svg+='<polyline fill="none" stroke="'+
cols[i%cols.length]+'" points="'+d+'"/>';if(s.name)svg+='<text x="'+(w-140)+'" y="'+(14+12*i)+'" font-size="10" fill="'+
cols[i%cols.length]+'">'+s.name+'</text>';});svg+='<text x="2" y="12" font-size="10">'+y1.toPrecision(4)+
'</text><text x="2" y="'+(h-22)+'" font-size="10">'+y0.toPrecision(4)+'</text></svg>';el.innerHTML=svg;}
function bars(el,h,w,hh){if(!h||!h.counts){el.innerHTML='(no histogram)';return;}var m=Math.max.apply(null,h.counts)||1,
n=h.counts.length,bw=(w-40)/n,svg='<svg width="'+w+'" height="'+hh+'">';h.counts.forEach(function(c,i){var y=c/m*(hh-20);
svg+='<rect x="'+(30+i*bw).toFixed(1)+'" y="'+(hh-15-y).toFixed(1)+'" width="'+Math.max(1,bw-1).toFixed(1)+
'" height="'+y.toFixed(1)+'" fill="#1f77b4"/>';});svg+='<text x="2" y="'+(hh-2)+'" font-size="10">'+h.min.toPrecision(3)+
'</text><text x="'+(w-60)+'" y="'+(hh-2)+'" font-size="10">'+h.max.toPrecision(3)+'</text></svg>';el.innerHTML=svg;}
function J(u){return fetch(u).then(function(r){return r.json()})}"""


def _page(title_key, body, script, i18n):
    t = i18n.messages()
    langs = "".join(f'<option value="{c}"{" selected" if c == i18n.getDefaultLanguage() else ""}>{c}</option>'
                    for c in i18n.languages())
    nav = (f'<nav><a href="/train/overview">{t["train.nav.overview"]}</a><a href="/train/model">'
           f'{t["train.nav.model"]}</a><a href="/train/system">{t["train.nav.system"]}</a><a href="/train/help">'
           f'{t["train.nav.help"]}</a><a href="/activations">{t["activations.title"]}</a><a href="/tsne">'
           f'{t["tsne.title"]}</a><span style="color:#fff">{t["train.nav.session"]}:</span><select id="sess">'
           f'</select><span style="color:#fff;margin-left:12px">{t["train.nav.language"]}:</span>'
           f'<select id="lang" onchange="fetch(\'/setlang/\'+this.value).then(function(){{location.reload()}})">'
           f'{langs}</select></nav>')
    sess = ("J('/train/sessions/all').then(function(s){var e=document.getElementById('sess');J('/train/sessions/current')"
            ".then(function(c){s.forEach(function(x){var o=document.createElement('option');o.value=x;o.text=x;"
            "if(x==c.sessionId)o.selected=true;e.appendChild(o);});e.onchange=function(){fetch('/train/sessions/set/'+"
            "encodeURIComponent(e.value)).then(function(){load()})};load();setInterval(load,5000);});});")
    return (f'<!doctype html><html><head><meta charset="utf-8"><title>{t["train.pagetitle"]} - {t[title_key]}'
            f'</title><style>{_CSS}</style></head><body>{nav}<main><h2>{t[title_key]}</h2>{body}</main>'
            f'<script>{_JS_LINE}\n{script}\n{sess}</script></body></html>')


# ------------------------------------------------------------------------------------------------------ train module
class TrainModule(UIModule):
    """Overview / model / system / help pages and their JSON data, session and worker selection
    (reference TrainModule.java:94-117)."""

    def __init__(self, server):
        self.server = server
        self.current_session = None
        self.current_worker = 0
        self.i18n = DefaultI18N.getInstance()

    def getCallbackTypeIDs(self):
        return [TYPE_ID]

    def getRoutes(self):
        return [Route("GET", "/train", lambda r, p: Response.redirect("/train/overview")),
                Route("GET", "/train/overview", lambda r, p: Response.html(self.overview_page())),
                Route("GET", "/train/overview/data", lambda r, p: self._data(self.overview_data)),
                Route("GET", "/train/model", lambda r, p: Response.html(self.model_page())),
                Route("GET", "/train/model/graph", lambda r, p: self._data(self.model_graph)),
                Route("GET", "/train/model/data/:layerId", lambda r, p: self._data(self.model_data, p["layerId"])),
                Route("GET", "/train/system", lambda r, p: Response.html(self.system_page())),
                Route("GET", "/train/system/data", lambda r, p: self._data(self.system_data)),
                Route("GET", "/train/help", lambda r, p: Response.html(self.help_page())),
                Route("GET", "/train/sessions/current", lambda r, p: Response.ok({"sessionId": self.session()})),
                Route("GET", "/train/sessions/all", lambda r, p: Response.ok(self.sessions())),
                Route("GET", "/train/sessions/info", lambda r, p: Response.ok(self.sessions_info())),
                Route("GET", "/train/sessions/set/:to", lambda r, p: self.set_session(p["to"])),
                Route("GET", "/train/sessions/lastUpdate/:sessionId",
                      lambda r, p: Response.ok(self.last_update(p["sessionId"]))),
                Route("GET", "/train/workers/currentByIdx", lambda r, p: Response.ok(self.current_worker)),
                Route("GET", "/train/workers/setByIdx/:to", lambda r, p: self.set_worker(p["to"])),
                Route("GET", "/setlang/:to", lambda r, p: self.set_lang(p["to"])),
                Route("GET", "/lang/getCurrent", lambda r, p: Response.ok(self.i18n.getDefaultLanguage()))]

    # -- sessions
    def sessions(self):
        out = []
        for st in self.server.storages:
            for s in st.listSessionIDs():
                if s not in out and st.listTypeIDsForSession(s).__contains__(TYPE_ID):
                    out.append(s)
        return out

    def _storage(self, sid):
        for st in self.server.storages:
            if sid in st.listSessionIDs():
                return st
        return None

    def session(self):
        all_ = self.sessions()
        if self.current_session not in all_:
            # default: the session with the most recent update
            best, bt = None, -1
            for s in all_:
                t = self.last_update(s)
                if t > bt:
                    best, bt = s, t
            self.current_session = best
        return self.current_session

    def set_session(self, sid):
        if sid not in self.sessions():
            return Response.not_found(f"unknown session {sid}")
        self.current_session = sid
        self.current_worker = 0
        return Response.ok({"sessionId": sid})

    def set_worker(self, to):
        try:
            self.current_worker = int(to)
        except ValueError:
            return Response(400, {"error": f"bad worker index {to!r}"})
        return Response.ok(self.current_worker)

    def set_lang(self, lang):
        try:
            self.i18n.setDefaultLanguage(lang)
        except ValueError as e:
            return Response(400, {"error": str(e)})
        return Response.ok({"language": lang})

    def workers(self, sid):
        st = self._storage(sid)
        return [] if st is None else sorted(st.listWorkerIDsForSessionAndType(sid, TYPE_ID))

    def last_update(self, sid):
        st = self._storage(sid)
        if st is None:
            return -1
        ts = [r.timeStamp for w in st.listWorkerIDsForSessionAndType(sid, TYPE_ID)
              for r in [st.getLatestUpdate(sid, TYPE_ID, w)] if r is not None]
        return max(ts) if ts else -1

    def sessions_info(self):
        out = {}
        for s in self.sessions():
            st = self._storage(s)
            ws = self.workers(s)
            out[s] = {"numWorkers": len(ws), "workers": ws, "lastUpdate": self.last_update(s),
                      "numUpdates": st.getNumUpdateRecordsFor(s)}
        return out

    def _worker(self, sid):
        ws = self.workers(sid)
        return ws[min(self.current_worker, len(ws) - 1)] if ws else None

    def _updates(self, sid):
        st, w = self._storage(sid), self._worker(sid)
        if st is None or w is None:
            return []
        return [st.getUpdate(sid, TYPE_ID, w, t) for t in st.getAllUpdateTimes(sid, TYPE_ID, w)]

    def _static(self, sid):
        st = self._storage(sid)
        infos = st.getAllStaticInfos(sid, TYPE_ID) if st is not None else []
        w = self._worker(sid)
        for i in infos:
            if i.workerID == w:
                return i.data
        return infos[0].data if infos else {}

    def _data(self, fn, *args):
        sid = self.session()
        if sid is None:
            return Response.ok({"sessionId": None})
        return Response.ok(fn(sid, *args))

    # -- overview
    def overview_data(self, sid):
        ups = self._updates(sid)
        score, perf, ratios, stdev_act = [], [], {}, {}
        for r in ups:
            d = r.data
            it = d.get("iterationCount")
            score.append([it, d.get("score")])
            p = d.get("performance") or {}
            if p:
                perf.append([it, p.get("examplesPerSecond"), p.get("minibatchesPerSecond")])
            P, U = d.get("Parameters") or {}, d.get("Updates") or {}
            for k in P:
                pm, um = P[k].get("meanMagnitude"), (U.get(k) or {}).get("meanMagnitude")
                if pm and um and pm > 0 and um > 0:
                    ratios.setdefault(k, []).append([it, math.log10(um / pm)])
            for k, a in (d.get("Activations") or {}).items():
                if a.get("stdev") is not None:
                    stdev_act.setdefault(k, []).append([it, a["stdev"]])
        model = self._static(sid).get("model") or {}
        last = ups[-1].data if ups else {}
        lp = last.get("performance") or {}
        first_t = ups[0].timeStamp if ups else None
        return {"sessionId": sid, "score": score, "performance": perf, "updateRatios": ratios,
                "stdevActivations": stdev_act,
                "perfTable": {"startTime": first_t, "totalRuntimeMs": lp.get("totalRuntimeMs"),
                              "lastUpdate": ups[-1].timeStamp if ups else None,
                              "totalParamUpdates": last.get("iterationCount"),
                              "updatesPerSec": lp.get("minibatchesPerSecond"),
                              "examplesPerSec": lp.get("examplesPerSecond")},
                "modelTable": {"modelType": model.get("className"), "nLayers": model.get("numLayers"),
                               "nParams": model.get("numParams")}}

    def overview_page(self):
        t = self.i18n.messages()
        body = (f'<div class="c"><b>{t["train.overview.chart.scoreTitle"]}</b><div id="score"></div></div>'
                f'<div class="c"><b>{t["train.overview.chart.updateRatioTitle"]}</b><div id="ratio"></div></div>'
                f'<div class="c"><b>{t["train.overview.chart.perfTitle"]}</b><div id="perf"></div></div>'
                '<div class="c"><table id="tabs"></table></div>')
        rows = [("train.overview.modeltable.modeltype", "modelTable", "modelType"),
                ("train.overview.modeltable.nLayers", "modelTable", "nLayers"),
                ("train.overview.modeltable.nParams", "modelTable", "nParams"),
                ("train.overview.perftable.totalParamUpdates", "perfTable", "totalParamUpdates"),
                ("train.overview.perftable.totalRuntime", "perfTable", "totalRuntimeMs"),
                ("train.overview.perftable.examplesPerSec", "perfTable", "examplesPerSec")]
        spec = json.dumps([[t[k], a, b] for k, a, b in rows])
        script = ("function load(){J('/train/overview/data').then(function(d){if(!d.score)return;"
                  "line(document.getElementById('score'),[{pts:d.score}],720,220);var rs=[];for(var k in d.updateRatios)"
                  "rs.push({name:k,pts:d.updateRatios[k]});line(document.getElementById('ratio'),rs,720,220);"
                  "line(document.getElementById('perf'),[{pts:d.performance}],720,160);var h='';"
                  f"{spec}.forEach(function(r){{h+='<tr><th>'+E(r[0])+'</th><td>'+E(d[r[1]][r[2]])+'</td></tr>';}});"
                  "document.getElementById('tabs').innerHTML=h;});}")
        return _page("train.overview.title", body, script, self.i18n)

    # -- model
    def model_graph(self, sid):
        """{vertexNames, vertexTypes, vertexInputs (indices), layerIds}: the MultiLayerNetwork chain or the
        ComputationGraph vertex DAG from the stored configuration."""
        model = self._static(sid).get("model") or {}
        names = list(model.get("layerNames") or [])
        types = list(model.get("layerTypes") or [])
        conf = model.get("configJson")
        inputs = [[i - 1] if i > 0 else [] for i in range(len(names))]
        if conf and model.get("className") == "ComputationGraph":
            try:
                c = json.loads(conf)
                vin = c.get("vertexInputs") or {}
                nets = list(c.get("networkInputs") or [])
                order = nets + [n for n in vin if n not in nets]
                vtypes = {n: (v.get("@class") or type(v).__name__) if isinstance(v, dict) else str(v)
                          for n, v in (c.get("vertices") or {}).items()}
                idx = {n: i for i, n in enumerate(order)}
                names = order
                types = ["Input" if n in nets else vtypes.get(n, "Vertex") for n in order]
                inputs = [[idx[i] for i in vin.get(n, []) if i in idx] for n in order]
            except (ValueError, AttributeError):
                pass
        return {"vertexNames": names, "vertexTypes": types, "vertexInputs": inputs,
                "layerIds": list(model.get("layerNames") or [])}

    def model_data(self, sid, layer_id):
        """Per-parameter mean-magnitude series of this layer (parameters and updates), its learning rates and the
        latest histograms."""
        model = self._static(sid).get("model") or {}
        names = list(model.get("layerNames") or [])
        # statistics are keyed "<layer index or name>_<param>" (ui/stats.py _segments)
        prefs = [f"{layer_id}_"] + ([f"{names.index(layer_id)}_"] if layer_id in names else [])
        ups = self._updates(sid)

        def strip(k):
            for pf in prefs:
                if k.startswith(pf):
                    return k[len(pf):]
            return None
        mm = {}
        lr = []
        for r in ups:
            d = r.data
            it = d.get("iterationCount")
            for st in ("Parameters", "Updates", "Gradients"):
                for k, v in (d.get(st) or {}).items():
                    pk = strip(k)
                    if pk is not None and v.get("meanMagnitude") is not None:
                        mm.setdefault(f"{st}:{pk}", []).append([it, v["meanMagnitude"]])
            lrs = d.get("learningRates") or {}
            vals = [v for k, v in lrs.items() if strip(k) is not None or k == layer_id]
            if vals:
                lr.append([it, vals[0]])
        hist = {}
        if ups:
            d = ups[-1].data
            for st in ("Parameters", "Updates", "Gradients", "Activations"):
                for k, v in (d.get(st) or {}).items():
                    pk = strip(k)
                    if (pk is not None or k == layer_id) and "histogram" in v:
                        hist[f"{st}:{pk if pk is not None else k}"] = v["histogram"]
        info = {"layerName": layer_id, "layerType": (model.get("layerTypes") or [None] * len(names))[
            names.index(layer_id)] if layer_id in names else None,
            "params": sorted({k.split(":", 1)[1] for k in mm})}
        return {"layerInfo": info, "meanMagnitudes": mm, "learningRates": lr, "histograms": hist}

    def model_page(self):
        t = self.i18n.messages()
        body = ('<div class="c" style="float:left;width:220px"><b>Layers</b><div id="layers"></div></div>'
                '<div style="margin-left:240px"><div class="c"><b>' + t["train.model.layerInfoTable.title"] +
                '</b><pre id="info"></pre></div><div class="c"><b>' + t["train.model.meanmag.title"] +
                '</b><div id="mm"></div></div><div class="c"><b>' + t["train.model.lrChart.title"] +
                '</b><div id="lr"></div></div><div class="c"><b>' + t["train.model.paramHistChart.title"] +
                '</b><div id="hist"></div></div></div>')
        script = ("var cur=null;function show(id){cur=id;J('/train/model/data/'+encodeURIComponent(id)).then(function(d){"
                  "if(!d.layerInfo)return;document.getElementById('info').textContent=JSON.stringify(d.layerInfo,null,1);"
                  "var s=[];for(var k in d.meanMagnitudes)s.push({name:k,pts:d.meanMagnitudes[k]});"
                  "line(document.getElementById('mm'),s,640,220);line(document.getElementById('lr'),[{pts:d.learningRates}],"
                  "640,140);var h=document.getElementById('hist');h.innerHTML='';for(var k in d.histograms){"
                  "var e=document.createElement('div');h.appendChild(document.createTextNode(k));h.appendChild(e);"
                  "bars(e,d.histograms[k],640,120);}});}"
                  "function load(){J('/train/model/graph').then(function(g){if(!g.vertexNames)return;var h='';"
                  "window._vn=g.vertexNames;g.vertexNames.forEach(function(n,i){h+='<div class=\"l\" onclick=\"show(_vn['+i+'])\">'+"
                  "E(n)+' <small>'+E(g.vertexTypes[i])+'</small></div>';});document.getElementById('layers').innerHTML=h;"
                  "if(cur==null&&g.layerIds.length)cur=g.layerIds[0];if(cur!=null)show(cur);});}")
        return _page("train.model.title", body, script, self.i18n)

    # -- system
    def system_data(self, sid):
        st = self._storage(sid)
        infos = st.getAllStaticInfos(sid, TYPE_ID) if st is not None else []
        mem = []
        for r in self._updates(sid):
            m = r.data.get("memory")
            if m:
                mem.append([r.data.get("iterationCount"), m.get("hostCurrentBytes"),
                            (m.get("deviceCurrentBytes") or [None])[0]])
        return {"workers": [{"worker": i.workerID, "hardware": i.data.get("hardware"),
                             "software": i.data.get("software")} for i in infos], "memory": mem}

    def system_page(self):
        t = self.i18n.messages()
        body = (f'<div class="c"><b>{t["train.system.chart.memory"]}</b><div id="mem"></div></div>'
                f'<div class="c"><b>{t["train.system.hwTable.title"]}</b><pre id="hw"></pre></div>'
                f'<div class="c"><b>{t["train.system.swTable.title"]}</b><pre id="sw"></pre></div>')
        script = ("function load(){J('/train/system/data').then(function(d){if(!d.workers)return;"
                  "line(document.getElementById('mem'),[{name:'host',pts:d.memory.map(function(m){return[m[0],m[1]]})},"
                  "{name:'device',pts:d.memory.map(function(m){return[m[0],m[2]]})}],720,200);"
                  "document.getElementById('hw').textContent=JSON.stringify(d.workers.map(function(w){return w.hardware}),"
                  "null,1);document.getElementById('sw').textContent=JSON.stringify(d.workers.map(function(w){"
                  "return w.software}),null,1);});}")
        return _page("train.system.title", body, script, self.i18n)

    def help_page(self):
        t = self.i18n.messages()
        return _page("train.help.title", f'<div class="c">{t["train.help.text"]}</div>', "function load(){}",
                     self.i18n)


# ------------------------------------------------------------------------------------------------------ other modules
class DefaultModule(UIModule):
    def getRoutes(self):
        return [Route("GET", "/", lambda r, p: Response.redirect("/train/overview"))]


CONV_TYPE_ID = "ConvolutionalListener"


class ConvolutionalListenerModule(UIModule):
    """Latest activation grids published by ConvolutionalIterationListener (ui/convolutional.py) through a stats
    router: ``/activations`` page, ``/activations/data`` (iteration + per-layer image URLs) and the PNG bytes."""

    def __init__(self, server):
        self.server = server
        self.i18n = DefaultI18N.getInstance()

    def getCallbackTypeIDs(self):
        return [CONV_TYPE_ID]

    def latest(self):
        best = None
        for st in self.server.storages:
            for s in st.listSessionIDs():
                for w in st.listWorkerIDsForSessionAndType(s, CONV_TYPE_ID):
                    r = st.getLatestUpdate(s, CONV_TYPE_ID, w)
                    if r is not None and (best is None or r.timeStamp > best.timeStamp):
                        best = r
        return best

    def getRoutes(self):
        return [Route("GET", "/activations", lambda r, p: Response.html(self.page())),
                Route("GET", "/activations/data", lambda r, p: Response.ok(self.data())),
                Route("GET", "/activations/image/:layer", lambda r, p: self.image(p["layer"]))]

    def data(self):
        r = self.latest()
        if r is None:
            return {"iteration": None, "images": {}}
        imgs = r.data.get("images") or {}
        return {"iteration": r.data.get("iteration"),
                "images": {k: "/activations/image/" + urllib.parse.quote(str(k)) for k in imgs}}

    def image(self, layer):
        r = self.latest()
        path = (r.data.get("images") or {}).get(layer) if r is not None else None
        if not path or not os.path.isfile(path):
            return Response.not_found(f"no activation image for layer {layer}")
        with open(path, "rb") as fh:
            return Response(200, fh.read(), "image/png")

    def page(self):
        script = ("function load(){J('/activations/data').then(function(d){var h='iteration '+d.iteration;"
                  "for(var k in d.images)h+='<div class=\"c\"><b>'+E(k)+'</b><br><img style=\"image-rendering:pixelated;"
                  "width:512px\" src=\"'+E(d.images[k])+'?t='+Date.now()+'\"></div>';document.getElementById('acts')"
                  ".innerHTML=h;});}")
        return _page("activations.title", '<div id="acts"></div>', script, self.i18n)


class TsneModule(UIModule):
    """Uploaded 2-D embeddings (``x,y,label`` per line) per session (reference TsneModule.java:45-50)."""

    def __init__(self, server):
        self.server = server
        self.i18n = DefaultI18N.getInstance()

    @staticmethod
    def parse(text):
        rows = []
        for line in text.splitlines():
            p = line.strip().split(",")
            if len(p) >= 3:
                rows.append([float(p[0]), float(p[1]), ",".join(p[2:]).strip()])
            elif len(p) == 2 and p[0]:
                rows.append([float(p[0]), float(p[1]), ""])
        return rows

    def getRoutes(self):
        return [Route("GET", "/tsne", lambda r, p: Response.html(self.page())),
                Route("GET", "/tsne/sessions", lambda r, p: Response.ok(sorted(self.server.tsne))),
                Route("GET", "/tsne/coords/:sid", lambda r, p: self.coords(p["sid"])),
                Route("POST", "/tsne/upload", lambda r, p: self.post(r.query.get("name", "upload"), r.body)),
                Route("POST", "/tsne/post/:sid", lambda r, p: self.post(p["sid"], r.body))]

    def coords(self, sid):
        if sid not in self.server.tsne:
            return Response.not_found(f"unknown t-SNE session {sid}")
        return Response.ok(self.server.tsne[sid])

    def post(self, sid, body):
        try:
            rows = self.parse(body.decode("utf-8"))
        except (UnicodeDecodeError, ValueError) as e:
            return Response(400, {"error": str(e)})
        self.server.tsne[sid] = rows
        return Response.ok({"status": "ok", "points": len(rows)})

    def page(self):
        t = self.i18n.messages()
        body = (f'<div class="c">{t["tsne.upload"]}<br><textarea id="csv" rows="4" cols="60"></textarea>'
                '<button onclick="fetch(\'/tsne/post/\'+encodeURIComponent(document.getElementById(\'nm\').value),'
                '{method:\'POST\',body:document.getElementById(\'csv\').value}).then(function(){load()})">Upload</button>'
                ' name <input id="nm" value="upload"></div><div class="c"><select id="ts"></select><div id="plot"></div>'
                '</div>')
        script = ("function draw(sid){J('/tsne/coords/'+encodeURIComponent(sid)).then(function(rows){var xs=rows.map("
                  "function(r){return r[0]}),ys=rows.map(function(r){return r[1]});var x0=Math.min.apply(null,xs),"
                  "x1=Math.max.apply(null,xs),y0=Math.min.apply(null,ys),y1=Math.max.apply(null,ys);if(x1==x0)x1++;"
                  "if(y1==y0)y1++;var s='<svg width=\"720\" height=\"480\">';rows.forEach(function(r){var x=20+(r[0]-x0)/"
                  "(x1-x0)*680,y=460-(r[1]-y0)/(y1-y0)*440;s+='<circle cx=\"'+x.toFixed(1)+'\" cy=\"'+y.toFixed(1)+"
                  "'\" r=\"2\" fill=\"#1f77b4\"/><text x=\"'+(x+3).toFixed(1)+'\" y=\"'+y.toFixed(1)+'\" font-size=\"9\">'"
                  "+E(r[2])+'</text>';});document.getElementById('plot').innerHTML=s+'</svg>';});}"
                  "function load(){J('/tsne/sessions').then(function(ss){var e=document.getElementById('ts');"
                  "e.innerHTML='';ss.forEach(function(x){var o=document.createElement('option');o.value=x;o.text=x;"
                  "e.appendChild(o);});e.onchange=function(){draw(e.value)};if(ss.length)draw(ss[0]);});}")
        return _page("tsne.title", body, script, self.i18n)


class RemoteReceiverModule(UIModule):
    """``POST /remoteReceive``: records posted by RemoteUIStatsStorageRouter go into the server's remote storage
    (reference RemoteReceiverModule.java:58-120)."""

    def __init__(self, server):
        self.server = server

    def getRoutes(self):
        return [Route("POST", "/remoteReceive", lambda r, p: self.receive(r.body))]

    def receive(self, raw):
        st = self.server.remote_storage
        if st is None:
            return Response(403, {"error": "remote listener not enabled"})
        try:
            msg = json.loads(raw)
            rec = Persistable.decode(json.dumps(msg["record"]))
            {"meta": st.putStorageMetaData, "static": st.putStaticInfo, "update": st.putUpdate}[msg["type"]](rec)
        except (KeyError, ValueError, TypeError) as e:
            return Response(400, {"error": str(e)})
        return Response.ok({"status": "ok", "received": time.time()})
