"""Space-partitioning tree (Barnes-Hut) and its 2-D quad-tree specialisation — native C++ (trees.cpp).

Reference: clustering/sptree/SpTree.java (computeNonEdgeForces(pointIndex, theta, negativeForce, sumQ),
computeEdgeForces(rowP, colP, valP, N, posF), getDepth, centre of mass), clustering/quadtree/QuadTree.java.
"""
import ctypes

import numpy as np
import torch

from ..ops import runtime as RT

c_void_p, c_int, c_double, c_ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_longlong
RT.register("rt_sptree_build", [c_void_p, c_int, c_int], c_void_p)
RT.register("rt_sptree_free", [c_void_p], None)
RT.register("rt_sptree_depth", [c_void_p], c_int)
RT.register("rt_sptree_cum", [c_void_p], c_int)
RT.register("rt_sptree_com", [c_void_p, c_void_p], None)
RT.register("rt_sptree_nonedge", [c_void_p, c_int, c_double, c_void_p], c_double)
RT.register("rt_bhtsne_gradient", [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_double, c_void_p, c_int],
            c_double)


class SpTree:
    def __init__(self, data):
        Y = data.detach().cpu().double().numpy() if isinstance(data, torch.Tensor) else np.asarray(data, np.float64)
        self.Y = np.ascontiguousarray(Y)
        self.N, self.D = self.Y.shape
        if not 1 <= self.D <= 3:
            raise ValueError("SpTree supports 1-3 dimensions")
        self._rt = RT.load()
        self._h = self._rt.rt_sptree_build(ctypes.c_void_p(self.Y.ctypes.data), self.N, self.D)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._rt.rt_sptree_free(h)
            self._h = None

    def getDepth(self):
        return self._rt.rt_sptree_depth(self._h)

    def getCumSize(self):
        return self._rt.rt_sptree_cum(self._h)

    def getCenterOfMass(self):
        out = np.zeros(self.D)
        self._rt.rt_sptree_com(self._h, ctypes.c_void_p(out.ctypes.data))
        return out

    def computeNonEdgeForces(self, pointIndex, theta, negativeForce=None):
        """Adds the Barnes-Hut repulsive force on one point into ``negativeForce`` (len D); returns its sum-Q part."""
        f = np.zeros(self.D) if negativeForce is None else negativeForce
        buf = np.ascontiguousarray(f, dtype=np.float64)
        s = self._rt.rt_sptree_nonedge(self._h, int(pointIndex), float(theta), ctypes.c_void_p(buf.ctypes.data))
        if negativeForce is not None:
            negativeForce[...] = buf
        return s, buf

    @staticmethod
    def computeEdgeForces(Y, rowP, colP, valP):
        """Attractive forces sum_j p_ij q_ij (y_i - y_j) for a CSR P (numpy, vectorised)."""
        Y = np.asarray(Y, np.float64)
        rows = np.repeat(np.arange(len(rowP) - 1), np.diff(rowP))
        diff = Y[rows] - Y[colP]
        q = 1.0 / (1.0 + (diff * diff).sum(1))
        posF = np.zeros_like(Y)
        np.add.at(posF, rows, (valP * q)[:, None] * diff)
        return posF

    def isCorrect(self):
        return self.getCumSize() == self.N


class QuadTree(SpTree):
    def __init__(self, data):
        super().__init__(data)
        if self.D != 2:
            raise ValueError("QuadTree is 2-D")


def bh_gradient(Y, rowP, colP, valP, theta, nthreads=8):
    """Full Barnes-Hut t-SNE gradient (native): returns (dY [N, D] float64, sumQ)."""
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    rowP = np.ascontiguousarray(rowP, dtype=np.int64)
    colP = np.ascontiguousarray(colP, dtype=np.int32)
    valP = np.ascontiguousarray(valP, dtype=np.float64)
    dY = np.empty_like(Y)
    rt = RT.load()
    s = rt.rt_bhtsne_gradient(ctypes.c_void_p(Y.ctypes.data), Y.shape[0], Y.shape[1], ctypes.c_void_p(rowP.ctypes.data),
                              ctypes.c_void_p(colP.ctypes.data), ctypes.c_void_p(valP.ctypes.data), float(theta),
                              ctypes.c_void_p(dY.ctypes.data), nthreads)
    return dY, s
