"""KD-tree with incremental insert/delete, nearest and radius search (KDTree.java, HyperRect.java).

Pointer-based dynamic tree for low-dimensional points (the reference's use); bulk k-NN over large point sets should
use the VP-tree (native) or knn_bruteforce (GPU) instead.
"""
import numpy as np


class HyperRect:
    def __init__(self, lo, hi):
        self.lo = np.array(lo, dtype=np.float64)
        self.hi = np.array(hi, dtype=np.float64)

    @staticmethod
    def point(p):
        return HyperRect(p, p)

    def enlargeTo(self, p):
        self.lo = np.minimum(self.lo, p)
        self.hi = np.maximum(self.hi, p)

    def minDistance(self, p):
        d = np.maximum(self.lo - p, 0) + np.maximum(p - self.hi, 0)
        return float(np.sqrt((d * d).sum()))

    def contains(self, p):
        return bool(np.all(self.lo <= p) and np.all(p <= self.hi))


class KDTree:
    GREATER = 1
    LESS = 0

    class KDNode:
        def __init__(self, point):
            self.point = point
            self.left = self.right = self.parent = None

        def getPoint(self):
            return self.point

        def getLeft(self):
            return self.left

        def getRight(self):
            return self.right

        def getParent(self):
            return self.parent

    def __init__(self, dims):
        self.dims = dims
        self.root = None
        self.rect = None
        self._size = 0

    @staticmethod
    def _vec(p):
        import torch
        if isinstance(p, torch.Tensor):
            p = p.detach().cpu().double().numpy()
        return np.asarray(p, dtype=np.float64).reshape(-1)

    def insert(self, point):
        p = self._vec(point)
        if p.shape[0] != self.dims:
            raise ValueError(f"point must have {self.dims} dimensions")
        node = KDTree.KDNode(p)
        self._size += 1
        if self.rect is None:
            self.rect = HyperRect.point(p)
        else:
            self.rect.enlargeTo(p)
        if self.root is None:
            self.root = node
            return
        cur, depth = self.root, 0
        while True:
            ax = depth % self.dims
            if p[ax] <= cur.point[ax]:
                if cur.left is None:
                    cur.left, node.parent = node, cur
                    return
                cur = cur.left
            else:
                if cur.right is None:
                    cur.right, node.parent = node, cur
                    return
                cur = cur.right
            depth += 1

    def size(self):
        return self._size

    def _all(self, node, out):
        if node is None:
            return
        out.append(node.point)
        self._all(node.left, out)
        self._all(node.right, out)

    def delete(self, point):
        """Remove one occurrence of ``point`` (rebuilds the affected subtree); returns the removed node or None."""
        p = self._vec(point)
        pts = []
        self._all(self.root, pts)
        for i, q in enumerate(pts):
            if np.array_equal(q, p):
                del pts[i]
                self.root, self.rect, self._size = None, None, 0
                for r in pts:
                    self.insert(r)
                return KDTree.KDNode(p)
        return None

    def nn(self, point):
        """(distance, point) of the nearest stored point."""
        q = self._vec(point)
        best = [np.inf, None]

        def rec(node, depth):
            if node is None:
                return
            d = float(np.sqrt(((node.point - q) ** 2).sum()))
            if d < best[0]:
                best[0], best[1] = d, node.point
            ax = depth % self.dims
            diff = q[ax] - node.point[ax]
            near, far = (node.left, node.right) if diff <= 0 else (node.right, node.left)
            rec(near, depth + 1)
            if abs(diff) < best[0]:
                rec(far, depth + 1)
        rec(self.root, 0)
        return best[0], best[1]

    def knn(self, point, distance):
        """All stored points within ``distance`` of ``point`` as (distance, point), nearest first."""
        q = self._vec(point)
        out = []

        def rec(node, depth):
            if node is None:
                return
            d = float(np.sqrt(((node.point - q) ** 2).sum()))
            if d <= distance:
                out.append((d, node.point))
            ax = depth % self.dims
            diff = q[ax] - node.point[ax]
            if diff <= distance:
                rec(node.left, depth + 1)
            if -diff <= distance:
                rec(node.right, depth + 1)
        rec(self.root, 0)
        out.sort(key=lambda t: t[0])
        return out
