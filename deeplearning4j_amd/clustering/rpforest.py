"""Random-projection trees / forest for approximate nearest neighbours (RPForest.java, RPTree.java, RPUtils.java).

Each tree splits a node's points at the median of their projection on a random Gaussian direction until a leaf holds
at most ``maxSize`` points. A query descends every tree to a leaf; the union of leaves is re-ranked exactly with the
requested distance (one small GEMM on the data's device).
"""
import numpy as np
import torch

from .distances import SIMILARITIES, pairwise


class RPUtils:
    @staticmethod
    def computeDistance(function, x, y, result=None):
        """One distance (RPUtils.computeDistance): euclidean / manhattan / cosinedistance / cosinesimilarity / dot /
        jaccard / hamming between two vectors."""
        xv = torch.as_tensor(getattr(x, "tensor", x), dtype=torch.float64).reshape(1, -1)
        yv = torch.as_tensor(getattr(y, "tensor", y), dtype=torch.float64).reshape(1, -1)
        return float(pairwise(xv, yv, function)[0, 0])

    @staticmethod
    def computeDistanceMulti(function, x, y, result=None):
        """Distances from vector x to every row of y (RPUtils.computeDistanceMulti); written into ``result`` when
        given, and returned."""
        xv = torch.as_tensor(getattr(x, "tensor", x), dtype=torch.float64).reshape(1, -1)
        ym = torch.as_tensor(getattr(y, "tensor", y), dtype=torch.float64).reshape(-1, xv.shape[1])
        d = pairwise(xv, ym, function)[0]
        if result is not None:
            r = getattr(result, "tensor", result)
            r.reshape(-1).copy_(d.to(r.dtype))
            return result
        return d

    @staticmethod
    def getAllCandidates(x, trees):
        cand = set()
        for t in trees:
            cand.update(t.getCandidates(x))
        return sorted(cand)

    @staticmethod
    def queryAllWithDistances(toQuery, X, trees, n, similarityFunction):
        cand = RPUtils.getAllCandidates(toQuery, trees)
        if not cand:
            return []
        q = torch.as_tensor(toQuery, dtype=torch.float32, device=X.device).reshape(1, -1)
        d = pairwise(q, X[torch.as_tensor(cand, device=X.device)], similarityFunction)[0]
        if similarityFunction in SIMILARITIES:
            d = -d
        order = torch.argsort(d)[:n].cpu().tolist()
        dl = d.cpu().tolist()
        return [(dl[i], cand[i]) for i in order]


class RPTree:
    def __init__(self, dim, maxSize, similarityFunction="euclidean", seed=12345):
        self.dim, self.maxSize, self.sim = dim, maxSize, similarityFunction
        self.rng = np.random.RandomState(seed)
        self.nodes = []          # (direction, threshold, left, right, indices|None)

    def buildTree(self, x):
        X = x.detach().cpu().double().numpy() if isinstance(x, torch.Tensor) else np.asarray(x, np.float64)
        self.X = X
        self.nodes = []
        self.root = self._build(np.arange(X.shape[0]))
        return self

    def _build(self, idx):
        nid = len(self.nodes)
        self.nodes.append(None)
        if len(idx) <= self.maxSize:
            self.nodes[nid] = (None, 0.0, -1, -1, idx)
            return nid
        w = self.rng.randn(self.dim)
        proj = self.X[idx] @ w
        thr = float(np.median(proj))
        left, right = idx[proj <= thr], idx[proj > thr]
        if len(left) == 0 or len(right) == 0:          # degenerate split (duplicates): make a leaf
            self.nodes[nid] = (None, 0.0, -1, -1, idx)
            return nid
        l = self._build(left)
        r = self._build(right)
        self.nodes[nid] = (w, thr, l, r, None)
        return nid

    def getCandidates(self, target):
        t = target.detach().cpu().double().numpy() if isinstance(target, torch.Tensor) else np.asarray(target)
        t = t.reshape(-1)
        n = self.root
        while True:
            w, thr, l, r, idx = self.nodes[n]
            if idx is not None:
                return idx.tolist()
            n = l if float(t @ w) <= thr else r

    def getLeaves(self):
        return [nd[4] for nd in self.nodes if nd[4] is not None]


class RPForest:
    def __init__(self, numTrees, maxSize, similarityFunction="euclidean", seed=12345):
        self.numTrees, self.maxSize, self.sim, self.seed = numTrees, maxSize, similarityFunction, seed
        self.trees = []
        self.data = None

    def fit(self, x):
        self.data = torch.as_tensor(x, dtype=torch.float32)
        self.trees = [RPTree(self.data.shape[1], self.maxSize, self.sim, self.seed + i).buildTree(self.data)
                      for i in range(self.numTrees)]
        return self

    def getAllCandidates(self, input):
        return RPUtils.getAllCandidates(input, self.trees)

    def queryWithDistances(self, query, numResults):
        return RPUtils.queryAllWithDistances(query, self.data, self.trees, numResults, self.sim)

    def queryAll(self, toQuery, n):
        return [i for _, i in self.queryWithDistances(toQuery, n)]
