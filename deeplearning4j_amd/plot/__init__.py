"""t-SNE: exact (dense, GPU) and Barnes-Hut (sparse P from a native VP-tree k-NN, native SP-tree gradient).

Reference: deeplearning4j-manifold/deeplearning4j-tsne plot/Tsne.java and plot/BarnesHutTsne.java (defaults: maxIter
1000, perplexity 30, theta 0.5, momentum 0.5 -> 0.8 at switchMomentumIteration 100, early exaggeration x12 until
stopLyingIteration 250, gains +0.2 / x0.8 with minGain 0.01, learning rate 500, optional AdaGrad, normalize;
symmetrized P = (P + P^T) / sum; saveAsFile writes "y1,y2,...,label" lines).

MI355X mapping: exact t-SNE is O(N^2) dense algebra — the affinity matrix, Student-t kernel and gradient are GEMMs
and elementwise passes on the GPU. Barnes-Hut keeps the tree work on the host in C++ (csrc/runtime/trees.cpp).
"""
import math

import numpy as np
import scipy.sparse as sp
import torch

from ..clustering.sptree import bh_gradient
from ..clustering.vptree import VPTree
from ..ops import runtime as RT
import ctypes

RT.register("rt_tsne_row_probs", [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_void_p, ctypes.c_int], None)


def _prep(x, normalize, usePca, pcaDims=50):
    X = torch.as_tensor(x).double()
    if normalize:
        X = (X - X.min()) / (X.max() - X.min()).clamp_min(1e-12)
        X = X - X.mean(0, keepdim=True)
    if usePca and X.shape[1] > pcaDims:
        U, S, V = torch.pca_lowrank(X, q=pcaDims, center=True)
        X = X @ V[:, :pcaDims]
    return X


def _dense_affinities(X, perplexity, tol=1e-5, iters=60):
    """Row-wise Gaussian conditionals with per-row precision found by vectorised bisection (all rows at once)."""
    N = X.shape[0]
    D = torch.cdist(X, X) ** 2
    D.fill_diagonal_(0)
    target = math.log(perplexity)
    beta = torch.ones(N, 1, dtype=X.dtype, device=X.device)
    lo = torch.full_like(beta, -float("inf"))
    hi = torch.full_like(beta, float("inf"))
    eye = torch.eye(N, dtype=torch.bool, device=X.device)
    for _ in range(iters):
        P = torch.exp(-D * beta).masked_fill(eye, 0)
        s = P.sum(1, keepdim=True).clamp_min(1e-300)
        H = torch.log(s) + beta * (D * P).sum(1, keepdim=True) / s
        diff = H - target
        if float(diff.abs().max()) < tol:
            break
        up = diff > 0
        lo = torch.where(up, beta, lo)
        hi = torch.where(up, hi, beta)
        beta = torch.where(up, torch.where(torch.isinf(hi), beta * 2, (beta + hi) / 2),
                           torch.where(torch.isinf(lo), beta / 2, (beta + lo) / 2))
    P = P / s
    return P


class _TsneBase:
    def __init__(self, **kw):
        self.maxIter = 1000
        self.realMin = 1e-12
        self.initialMomentum = 0.5
        self.finalMomentum = 0.8
        self.momentum = 0.5             # current momentum (the schedule moves it initial -> final at the switch)
        self.minGain = 1e-2
        self.switchMomentumIteration = 100
        self.normalize = True
        self.usePca = False
        self.stopLyingIteration = 250
        self.tolerance = 1e-5
        self.learningRate = 500.0
        self.useAdaGrad = False
        self.perplexity = 30.0
        self.theta = 0.5
        self.numDimensions = 2
        self.similarityFunction = "euclidean"
        self.invert = False
        self.seed = 12345
        self.device = None
        self.Y = None
        self.listeners = []
        self.scores = []
        for k, v in kw.items():
            setattr(self, k, v)

    class Builder:
        TARGET = None

        def __init__(self):
            self.kw = {}

        def _s(self, k, v):
            self.kw[k] = v
            return self

        def setMaxIter(self, v): return self._s("maxIter", int(v))  # noqa: E704
        def setRealMin(self, v): return self._s("realMin", float(v))  # noqa: E704
        def setInitialMomentum(self, v): return self._s("initialMomentum", float(v))  # noqa: E704
        def setFinalMomentum(self, v): return self._s("finalMomentum", float(v))  # noqa: E704
        def setMomentum(self, v): return self._s("momentum", float(v))  # noqa: E704
        def setSwitchMomentumIteration(self, v): return self._s("switchMomentumIteration", int(v))  # noqa: E704
        def normalize(self, v): return self._s("normalize", bool(v))  # noqa: E704
        def usePca(self, v): return self._s("usePca", bool(v))  # noqa: E704
        def stopLyingIteration(self, v): return self._s("stopLyingIteration", int(v))  # noqa: E704
        def tolerance(self, v): return self._s("tolerance", float(v))  # noqa: E704
        def learningRate(self, v): return self._s("learningRate", float(v))  # noqa: E704
        def useAdaGrad(self, v): return self._s("useAdaGrad", bool(v))  # noqa: E704
        def perplexity(self, v): return self._s("perplexity", float(v))  # noqa: E704
        def minGain(self, v): return self._s("minGain", float(v))  # noqa: E704
        def theta(self, v): return self._s("theta", float(v))  # noqa: E704
        def numDimension(self, v): return self._s("numDimensions", int(v))  # noqa: E704
        def similarityFunction(self, v): return self._s("similarityFunction", str(v))  # noqa: E704
        def invertDistanceMetric(self, v): return self._s("invert", bool(v))  # noqa: E704
        def seed(self, v): return self._s("seed", int(v))  # noqa: E704
        def device(self, d): return self._s("device", d)  # noqa: E704
        def workspaceMode(self, m): return self  # noqa: E704
        def vpTreeWorkers(self, n): return self  # noqa: E704

        def build(self):
            return self.TARGET(**self.kw)

    def getTheta(self):
        return self.theta

    def isInvert(self):
        return self.invert

    def getSimiarlityFunction(self):        # the reference's spelling
        return self.similarityFunction

    getSimilarityFunction = getSimiarlityFunction

    def getPerplexity(self):
        return self.perplexity

    def setListeners(self, *ls):
        self.listeners = list(ls[0] if len(ls) == 1 and isinstance(ls[0], (list, tuple)) else ls)

    def _dev(self):
        if self.device is not None:
            return torch.device(self.device)
        return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")

    def _update(self, Y, grad, inc, gains, hist, momentum):
        same = torch.sign(grad) == torch.sign(inc)
        gains.copy_(torch.where(same, gains * 0.8, gains + 0.2).clamp_min(self.minGain))
        step = gains * grad
        if self.useAdaGrad:
            hist += step * step
            step = self.learningRate * step / (hist.sqrt() + 1e-6)
        else:
            step = step * self.learningRate
        inc.mul_(momentum).sub_(step)
        Y += inc

    def getData(self):
        return self.Y

    getY = getData

    def saveAsFile(self, labels, path):
        Y = self.Y.detach().cpu().numpy()
        with open(path, "w", encoding="utf-8") as fh:
            for i in range(min(len(labels), Y.shape[0])):
                if labels[i] is None:
                    continue
                fh.write(",".join(repr(float(v)) for v in Y[i]) + "," + str(labels[i]) + " \n")

    def plot(self, matrix, nDims, labels, path):
        self.fit(matrix, nDims)
        self.saveAsFile(labels, path)

    def score(self):
        return self.scores[-1] if self.scores else float("nan")


class Tsne(_TsneBase):
    """Exact t-SNE on the GPU (dense P and Q)."""

    def calculate(self, X, nDims=None, perplexity=None):
        if nDims is not None:
            self.numDimensions = nDims
        if perplexity is not None:
            self.perplexity = perplexity
        dev = self._dev()
        Xp = _prep(X, self.normalize, self.usePca).to(dev)
        N = Xp.shape[0]
        P = _dense_affinities(Xp, self.perplexity, self.tolerance)
        P = (P + P.t())
        P = (P / P.sum()).clamp_min(self.realMin)
        P = P * 4.0                                          # early exaggeration (Tsne.java)
        g = torch.Generator().manual_seed(self.seed)
        Y = (torch.randn(N, self.numDimensions, generator=g, dtype=torch.float64) * 1e-4).to(dev)
        inc = torch.zeros_like(Y)
        gains = torch.ones_like(Y)
        hist = torch.zeros_like(Y)
        momentum = self.initialMomentum
        eye = torch.eye(N, dtype=torch.bool, device=dev)
        for it in range(self.maxIter):
            num = 1.0 / (1.0 + torch.cdist(Y, Y) ** 2)
            num = num.masked_fill(eye, 0)
            Q = (num / num.sum()).clamp_min(self.realMin)
            W = (P - Q) * num
            grad = 4.0 * (W.sum(1, keepdim=True) * Y - W @ Y)
            if it == self.switchMomentumIteration:
                momentum = self.finalMomentum
            if it == self.stopLyingIteration:
                P = P / 4.0
            self._update(Y, grad, inc, gains, hist, momentum)
            Y -= Y.mean(0, keepdim=True)
            if it % 50 == 0 or it == self.maxIter - 1:
                self.scores.append(float((P * torch.log(P / Q)).sum()))
            for l in self.listeners:
                l.iterationDone(self, it, 0)
        self.Y = Y
        return Y

    def fit(self, X, nDims=None):
        self.calculate(X, nDims)
        return self


class BarnesHutTsne(_TsneBase):
    """O(N log N) t-SNE: k-NN (3*perplexity) affinities from the native VP-tree, Barnes-Hut forces from the native
    SP-tree; theta == 0 falls back to the exact solver (as the reference does)."""

    def computeGaussianPerplexity(self, X, perplexity):
        N = X.shape[0]
        K = min(N - 1, int(3 * perplexity))
        Xn = X.detach().cpu().float().numpy()
        tree = VPTree(Xn, "euclidean")
        idx, dist = tree.knn(Xn, K + 1)
        idx, dist = idx[:, 1:], np.ascontiguousarray(dist[:, 1:])       # drop self
        probs = np.empty_like(dist)
        RT.load().rt_tsne_row_probs(ctypes.c_void_p(dist.ctypes.data), N, K, float(perplexity), float(self.tolerance),
                                    ctypes.c_void_p(probs.ctypes.data), 8)
        rows = np.repeat(np.arange(N), K)
        P = sp.csr_matrix((probs.reshape(-1).astype(np.float64), (rows, idx.reshape(-1))), shape=(N, N))
        self.rows, self.cols, self.vals = P.indptr, P.indices, P.data
        return P

    def symmetrized(self, P):
        S = (P + P.T).tocsr()
        S.sum_duplicates()
        return S

    def fit(self, X, nDims=None):
        if nDims is not None:
            self.numDimensions = nDims
        if self.theta == 0.0:
            t = Tsne(**{k: getattr(self, k) for k in ("maxIter", "realMin", "initialMomentum", "finalMomentum",
                                                      "minGain", "switchMomentumIteration", "normalize", "usePca",
                                                      "stopLyingIteration", "tolerance", "learningRate",
                                                      "useAdaGrad", "perplexity", "numDimensions", "seed",
                                                      "device")})
            self.Y = t.calculate(X)
            self.scores = t.scores
            return self
        Xp = _prep(X, self.normalize, self.usePca)
        N = Xp.shape[0]
        P = self.symmetrized(self.computeGaussianPerplexity(Xp, self.perplexity))
        P = P / P.sum()
        rowP = P.indptr.astype(np.int64)
        colP = P.indices.astype(np.int32)
        valP = P.data.astype(np.float64) * 12.0
        self.rows, self.cols, self.vals = rowP, colP, valP
        rng = np.random.RandomState(self.seed)
        Y = rng.randn(N, self.numDimensions) * 1e-3 if self.Y is None else \
            np.asarray(self.Y.detach().cpu() if isinstance(self.Y, torch.Tensor) else self.Y, np.float64)
        Yt = torch.from_numpy(Y)
        inc = torch.zeros_like(Yt)
        gains = torch.ones_like(Yt)
        hist = torch.zeros_like(Yt)
        momentum = self.initialMomentum
        for it in range(self.maxIter):
            dY, sumQ = bh_gradient(Yt.numpy(), rowP, colP, valP, self.theta)
            if it == self.switchMomentumIteration:
                momentum = self.finalMomentum
            if it == self.stopLyingIteration:
                valP = valP / 12.0
            self._update(Yt, torch.from_numpy(dY), inc, gains, hist, momentum)
            Yt -= Yt.mean(0, keepdim=True)
            if it % 50 == 0 or it == self.maxIter - 1:
                self.scores.append(self._kl(Yt.numpy(), rowP, colP, valP, sumQ))
            for l in self.listeners:
                l.iterationDone(self, it, 0)
        self.vals = valP
        self.Y = Yt
        return self

    @staticmethod
    def _kl(Y, rowP, colP, valP, sumQ):
        rows = np.repeat(np.arange(len(rowP) - 1), np.diff(rowP))
        d = ((Y[rows] - Y[colP]) ** 2).sum(1)
        q = (1.0 / (1.0 + d)) / sumQ
        return float((valP * np.log((valP + 1e-12) / (q + 1e-12))).sum())


Tsne.Builder = type("Builder", (_TsneBase.Builder,), {"TARGET": Tsne})
BarnesHutTsne.Builder = type("Builder", (_TsneBase.Builder,), {"TARGET": BarnesHutTsne})
