"""Nearest-neighbours REST server and client.

Reference: deeplearning4j-nearestneighbor-server NearestNeighborsServer.java (flags --ndarrayPath (comma-separated
2-D chunks), --labelsPath, --nearestNeighborsPort, --similarityFunction, --invert; POST /knn {k, inputIndex};
POST /knnnew {ndarray: base64 ND4J binary, k, forceFillK}; responses {"results": [{index, distance, label?}]}) and
deeplearning4j-nearestneighbors-client NearestNeighborsClient.java.
Stdlib threading HTTP server; the index is a native VP-tree (or GPU brute force with ``--gpu``).
"""
import argparse
import base64
import json
import threading
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np
import torch

from ..utils import nd4j_io
from .distances import knn_bruteforce
from .vptree import VPTree


def to_base64(arr):
    return base64.b64encode(nd4j_io.to_bytes(torch.as_tensor(arr))).decode("ascii")


def from_base64(s):
    return nd4j_io.from_bytes(base64.b64decode(s))


class NearestNeighborsServer:
    def __init__(self, points, labels=None, similarityFunction="euclidean", invert=False, port=9000, gpu=False):
        self.points = torch.as_tensor(points, dtype=torch.float32)
        if self.points.dim() != 2:
            raise ValueError("NearestNeighborsServer assumes 2D points")
        self.labels = list(labels or [])
        if self.labels and len(self.labels) != self.points.shape[0]:
            raise ValueError(f"Number of labels must match number of rows in points matrix "
                             f"(expected {self.points.shape[0]}, found {len(self.labels)})")
        self.fn, self.invert, self.port = similarityFunction, invert, port
        self.gpu = gpu and torch.cuda.is_available()
        if self.gpu:
            self.dev_points = self.points.cuda()
        else:
            self.tree = VPTree(self.points, similarityFunction, invert)
        self.httpd = None

    def search(self, query, k):
        q = torch.as_tensor(query, dtype=torch.float32).reshape(1, -1)
        if self.gpu:
            i, d = knn_bruteforce(self.dev_points, q.cuda(), k, self.fn, self.invert)
            idx, dist = i[0].cpu().tolist(), d[0].cpu().tolist()
        else:
            res, dist = self.tree.search(q, k)
            idx = [r.getIndex() for r in res]
        out = []
        for i, d in zip(idx, dist):
            r = {"index": int(i), "distance": float(d)}
            if self.labels:
                r["label"] = self.labels[i]
            out.append(r)
        return out

    def _handler(self):
        srv = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _reply(self, code, obj):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_POST(self):
                try:
                    n = int(self.headers.get("Content-Length", 0))
                    req = json.loads(self.rfile.read(n) or b"null")
                    if req is None:
                        return self._reply(400, {"status": "invalid json passed."})
                    if self.path == "/knn":
                        q = srv.points[int(req["inputIndex"])]
                        return self._reply(200, {"results": srv.search(q, int(req["k"]))})
                    if self.path == "/knnnew":
                        q = from_base64(req["ndarray"])
                        return self._reply(200, {"results": srv.search(q, int(req["k"]))})
                    return self._reply(404, {"status": "unknown route"})
                except Exception as e:  # noqa: BLE001 - report to the client like the reference (500)
                    return self._reply(500, {"status": str(e)})
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

    @staticmethod
    def main(argv=None):
        ap = argparse.ArgumentParser("NearestNeighborsServer")
        ap.add_argument("--ndarrayPath", required=True, help="comma-separated .npy / ND4J binary 2-D chunks")
        ap.add_argument("--labelsPath", default=None)
        ap.add_argument("--nearestNeighborsPort", type=int, default=9000)
        ap.add_argument("--similarityFunction", default="euclidean")
        ap.add_argument("--invert", action="store_true")
        ap.add_argument("--gpu", action="store_true")
        a = ap.parse_args(argv)
        chunks = []
        for p in a.ndarrayPath.split(","):
            if p.endswith(".npy"):
                chunks.append(torch.from_numpy(np.load(p, allow_pickle=False)))
            else:
                with open(p, "rb") as fh:
                    chunks.append(nd4j_io.read(fh))
        labels = None
        if a.labelsPath:
            labels = []
            for p in a.labelsPath.split(","):
                with open(p, encoding="utf-8") as fh:
                    labels.extend(l.rstrip("\n") for l in fh)
        srv = NearestNeighborsServer(torch.cat(chunks), labels, a.similarityFunction, a.invert,
                                     a.nearestNeighborsPort, a.gpu).start()
        print(f"NearestNeighborsServer listening on 127.0.0.1:{srv.port}")
        try:
            threading.Event().wait()
        except KeyboardInterrupt:
            srv.stop()


class NearestNeighborsClient:
    def __init__(self, url):
        self.url = url.rstrip("/")

    def _post(self, route, obj):
        req = urllib.request.Request(self.url + route, json.dumps(obj).encode(),
                                     {"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=30) as r:
            return json.loads(r.read())

    def knn(self, index, k):
        return self._post("/knn", {"inputIndex": int(index), "k": int(k)})["results"]

    def knnNew(self, k, arr, forceFillK=False):
        return self._post("/knnnew", {"ndarray": to_base64(arr), "k": int(k), "forceFillK": bool(forceFillK)})[
            "results"]


if __name__ == "__main__":
    NearestNeighborsServer.main()
