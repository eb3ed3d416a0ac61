"""Vantage-point tree (native C++ build + tau-pruned k-NN search, multi-threaded over queries).

Reference: nearestneighbor-core clustering/vptree/VPTree.java (constructors (items, similarityFunction, invert,
workers), search(target, k, results, distances)), VPTreeFillSearch.java (always returns exactly k results),
sptree/DataPoint.java. Results here are ordered nearest-first.
"""
import ctypes
import os

import numpy as np
import torch

from ..ops import runtime as RT
from .distances import DISTANCES

c_void_p, c_int, c_ull, c_double = ctypes.c_void_p, ctypes.c_int, ctypes.c_ulonglong, ctypes.c_double
RT.register("rt_vptree_build", [c_void_p, c_int, c_int, c_int, c_int, c_ull], c_void_p)
RT.register("rt_vptree_free", [c_void_p], None)
RT.register("rt_vptree_knn", [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int], None)


class DataPoint:
    def __init__(self, index, point, invert=False):
        self.index = int(index)
        self.point = point
        self.invert = invert

    def getIndex(self):
        return self.index

    def getPoint(self):
        return self.point

    def __eq__(self, o):
        return isinstance(o, DataPoint) and o.index == self.index

    def __hash__(self):
        return hash(self.index)

    def __repr__(self):
        return f"DataPoint({self.index})"


def _as_np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().float().numpy()
    return np.asarray(x, dtype=np.float32)


class VPTree:
    EUCLIDEAN = "euclidean"

    def __init__(self, items, similarityFunction="euclidean", invert=False, workers=None, seed=12345):
        if isinstance(similarityFunction, bool):          # VPTree(points, invert)
            similarityFunction, invert = "euclidean", similarityFunction
        if isinstance(items, (list, tuple)) and items and isinstance(items[0], DataPoint):
            items = np.stack([_as_np(p.point).reshape(-1) for p in items])
        self.items = np.ascontiguousarray(_as_np(items), dtype=np.float32)
        if self.items.ndim != 2:
            raise ValueError("VPTree items must be a 2-D [n, d] array")
        self.similarityFunction = similarityFunction
        self.invert = bool(invert)
        self.workers = workers or min(8, os.cpu_count() or 1)
        self._rt = RT.load()
        self._h = None
        n, d = self.items.shape
        # Cosine is not a metric, so tau-pruning on it can miss neighbours. On unit vectors
        # |a-b|^2 = 2 (1 - cos), a monotone map: build the tree on normalised rows with the euclidean metric
        # and convert the distances back — exact. "dot" has no such map: it is answered by brute force.
        self._cos = similarityFunction in ("cosinedistance", "cosinesimilarity")
        self._brute = similarityFunction == "dot"
        if self._brute:
            return
        data = self.items
        if self._cos:
            data = np.ascontiguousarray(data / np.maximum(np.linalg.norm(data, axis=1, keepdims=True), 1e-30))
        self._tree_data = data
        self._h = self._rt.rt_vptree_build(ctypes.c_void_p(data.ctypes.data), n, d,
                                           0 if self._cos else DISTANCES.get(similarityFunction, 0),
                                           0 if self._cos else int(self.invert), seed)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._rt.rt_vptree_free(h)
            self._h = None

    def getItems(self):
        return torch.from_numpy(self.items)

    def knn(self, queries, k):
        """Batched search: (indices [nq,k] int32, distances [nq,k]) nearest-first (-1 / inf padding)."""
        q = np.ascontiguousarray(_as_np(queries).reshape(-1, self.items.shape[1]), dtype=np.float32)
        k = min(int(k), self.items.shape[0])
        if self._brute:
            from .distances import knn_bruteforce
            i, d = knn_bruteforce(torch.from_numpy(self.items), torch.from_numpy(q), k, "dot", self.invert)
            return i.numpy().astype(np.int32), d.numpy()
        if self._cos:
            q = np.ascontiguousarray(q / np.maximum(np.linalg.norm(q, axis=1, keepdims=True), 1e-30))
        idx = np.empty((q.shape[0], k), np.int32)
        dist = np.empty((q.shape[0], k), np.float32)
        self._rt.rt_vptree_knn(self._h, ctypes.c_void_p(q.ctypes.data), q.shape[0], k,
                               ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(dist.ctypes.data), self.workers)
        if self._cos:
            cd = 0.5 * dist * dist
            dist = np.where(idx >= 0, cd if self.similarityFunction == "cosinedistance" else 1.0 - cd, dist)
            if self.similarityFunction == "cosinesimilarity" and self.invert:
                dist = -dist
        return idx, dist

    def search(self, target, k, results=None, distances=None):
        t = _as_np(target)
        if t.ndim > 2 or (t.ndim == 2 and t.shape[0] != 1) or t.reshape(-1).shape[0] != self.items.shape[1]:
            raise ValueError(f"Target for search should have shape [1, {self.items.shape[1]}] but got {t.shape}")
        idx, dist = self.knn(t, k)
        res = [DataPoint(i, torch.from_numpy(self.items[i])) for i in idx[0] if i >= 0]
        ds = [float(d) for i, d in zip(idx[0], dist[0]) if i >= 0]
        if results is not None:
            results.clear()
            results.extend(res)
        if distances is not None:
            distances.clear()
            distances.extend(ds)
        return res, ds

    def distance(self, a, b):
        from .distances import pairwise
        d = float(pairwise(torch.as_tensor(_as_np(a)).reshape(1, -1), torch.as_tensor(_as_np(b)).reshape(1, -1),
                           self.similarityFunction)[0, 0])
        return -d if self.invert else d


class VPTreeFillSearch:
    """k-NN that always returns k results (VPTreeFillSearch.java)."""

    def __init__(self, vpTree, k, target):
        self.tree, self.k, self.target = vpTree, k, target
        self.results, self.distances = [], []

    def search(self):
        self.tree.search(self.target, self.k, self.results, self.distances)
        return self.results

    def getResults(self):
        return self.results

    def getDistances(self):
        return self.distances
