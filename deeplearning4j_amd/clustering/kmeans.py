"""k-means and the cluster model (Point / Cluster / ClusterSet / strategies / termination conditions).

Reference: clustering/kmeans/KMeansClustering.java (setup(clusterCount, maxIterations | minVariationRate,
distanceFunction, inverse)), algorithm/BaseClusteringAlgorithm.java (k-means++-style seeding: first centre random,
next centres drawn with probability ~ squared distance to the nearest centre; classify / refresh centres / remove
empty clusters and split the most spread-out clusters), cluster/*.java, strategy/*.java, condition/*.java,
info/ClusterSetInfo.java.

MI355X mapping: all points live in one [N, d] tensor on the device; each iteration is one distance GEMM
([N, k]), an argmin, and a scatter-add (index_add_) for the new centres — no per-point host work.
"""
import math

import numpy as np
import torch

from .distances import SIMILARITIES, pairwise


class Point:
    def __init__(self, id=None, label=None, array=None):
        if array is None and isinstance(id, (torch.Tensor, np.ndarray, list)):
            id, array = None, id
        self.id = id
        self.label = label
        self.array = torch.as_tensor(np.asarray(array, dtype=np.float32) if not isinstance(array, torch.Tensor)
                                     else array).reshape(-1).float()

    def getArray(self):
        return self.array

    def getId(self):
        return self.id

    def getLabel(self):
        return self.label

    @staticmethod
    def toPoints(matrix):
        m = torch.as_tensor(matrix)
        return [Point(str(i), None, m[i]) for i in range(m.shape[0])]


class PointClassification:
    def __init__(self, cluster, distanceFromCenter, newLocation):
        self.cluster, self.distanceFromCenter, self.newLocation = cluster, distanceFromCenter, newLocation

    def getCluster(self):
        return self.cluster

    def getDistanceFromCenter(self):
        return self.distanceFromCenter

    def isNewLocation(self):
        return self.newLocation


class Cluster:
    def __init__(self, center=None, distanceFunction="euclidean", inverse=False, id=None):
        self.center = center
        self.points = []
        self.distanceFunction = distanceFunction
        self.inverse = inverse
        self.id = id
        self.label = None

    def getCenter(self):
        return self.center

    def setCenter(self, c):
        self.center = c

    def getPoints(self):
        return list(self.points)

    def addPoint(self, p, moveCenter=False):
        self.points.append(p)
        if moveCenter:
            n = len(self.points)
            self.center = Point(self.center.id, None, self.center.array * ((n - 1) / n) + p.array / n)

    def removePoints(self):
        self.points = []

    def isEmpty(self):
        return not self.points

    def getId(self):
        return self.id

    def getDistanceToCenter(self, p):
        d = float(pairwise(p.array.reshape(1, -1), self.center.array.reshape(1, -1), self.distanceFunction)[0, 0])
        return -d if self.inverse else d


class ClusterSet:
    def __init__(self, distanceFunction="euclidean", inverse=False):
        self.distanceFunction = distanceFunction
        self.inverse = inverse
        self.clusters = []
        self.pointDistribution = {}

    def getClusters(self):
        return list(self.clusters)

    def getClusterCount(self):
        return len(self.clusters)

    def addNewClusterWithCenter(self, center):
        c = Cluster(center, self.distanceFunction, self.inverse, id=len(self.clusters))
        self.clusters.append(c)
        return c

    def getCenters(self):
        return torch.stack([c.center.array for c in self.clusters])

    def _sign(self):
        return -1.0 if (self.inverse or self.distanceFunction in SIMILARITIES) else 1.0

    def nearestCluster(self, point):
        d = pairwise(point.array.reshape(1, -1), self.getCenters().to(point.array.device), self.distanceFunction)[0]
        i = int(torch.argmin(d * self._sign()))
        return self.clusters[i], float(d[i])

    def classifyPoint(self, point, moveClusterCenter=False):
        c, d = self.nearestCluster(point)
        prev = self.pointDistribution.get(point.id)
        new = prev != c.id
        self.pointDistribution[point.id] = c.id
        c.addPoint(point, moveClusterCenter)
        return PointClassification(c, d, new)

    def classifyPoints(self, points, moveClusterCenter=False):
        for p in points:
            self.classifyPoint(p, moveClusterCenter)

    def getMostPopulatedClusters(self, count):
        return sorted(self.clusters, key=lambda c: -len(c.points))[:count]

    def removePoints(self):
        for c in self.clusters:
            c.removePoints()

    def getClusterForPoint(self, point):
        cid = self.pointDistribution.get(point.id)
        return None if cid is None else self.clusters[cid]


# ------------------------------------------------------------------------------------- conditions / strategies
class FixedIterationCountCondition:
    def __init__(self, n):
        self.n = n

    @staticmethod
    def iterationCountGreaterThan(n):
        return FixedIterationCountCondition(n)

    def isSatisfied(self, history):
        return history.iteration >= self.n


class VarianceVariationCondition:
    """Stops when the relative change of the mean point-to-centre variance is below ``rate`` for ``period``
    consecutive iterations."""

    def __init__(self, rate, period=1):
        self.rate, self.period = rate, period

    @staticmethod
    def varianceVariationLessThan(rate, period=1):
        return VarianceVariationCondition(rate, period)

    def isSatisfied(self, history):
        v = history.variances
        if len(v) <= self.period:
            return False
        for j in range(1, self.period + 1):
            a, b = v[-j - 1], v[-j]
            if a == 0 or abs(b - a) / abs(a) >= self.rate:
                return False
        return True


class ConvergenceCondition:
    """Stops when the fraction of points that changed cluster is below ``rate``."""

    def __init__(self, rate):
        self.rate = rate

    @staticmethod
    def distributionVariationRateLessThan(rate):
        return ConvergenceCondition(rate)

    def isSatisfied(self, history):
        return history.iteration > 1 and history.moved_fraction < self.rate


class _History:
    def __init__(self):
        self.iteration = 0
        self.variances = []
        self.moved_fraction = 1.0


class FixedClusterCountStrategy:
    def __init__(self, clusterCount, distanceFunction="euclidean", inverse=False):
        self.initialClusterCount = clusterCount
        self.distanceFunction = distanceFunction
        self.inverse = inverse
        self.allowEmptyClusters = False
        self.terminationCondition = None

    @staticmethod
    def setup(clusterCount, distanceFunction="euclidean", inverse=False):
        return FixedClusterCountStrategy(clusterCount, distanceFunction, inverse)

    def endWhenIterationCountEquals(self, n):
        self.terminationCondition = FixedIterationCountCondition(n)
        return self

    def endWhenDistributionVariationRateLessThan(self, rate):
        self.terminationCondition = ConvergenceCondition(rate)
        return self

    def endWhenVarianceVariationRateLessThan(self, rate, period=1):
        self.terminationCondition = VarianceVariationCondition(rate, period)
        return self

    def getInitialClusterCount(self):
        return self.initialClusterCount

    def getDistanceFunction(self):
        return self.distanceFunction

    def inverseDistanceCalculation(self):
        return self.inverse


class OptimisationStrategy(FixedClusterCountStrategy):
    """Fixed count + optimisation target (e.g. keep the mean point-to-centre distance under a value by splitting
    the most spread-out clusters)."""

    def __init__(self, clusterCount, distanceFunction="euclidean", inverse=False):
        super().__init__(clusterCount, distanceFunction, inverse)
        self.maxAverageDistance = None

    def optimize(self, kind, value):
        if kind in ("MINIMIZE_AVERAGE_POINT_TO_CENTER_DISTANCE", "MINIMIZE_MAXIMUM_POINT_TO_CENTER_DISTANCE"):
            self.maxAverageDistance = float(value)
        return self


class ClusterUtils:
    @staticmethod
    def assign(X, centers, fn, inverse):
        d = pairwise(X, centers, fn)
        sign = -1.0 if (inverse or fn in SIMILARITIES) else 1.0
        idx = torch.argmin(d * sign, dim=1)
        return idx, d.gather(1, idx[:, None])[:, 0]

    @staticmethod
    def refreshCenters(X, idx, k, old):
        sums = torch.zeros(k, X.shape[1], device=X.device, dtype=X.dtype).index_add_(0, idx, X)
        cnt = torch.bincount(idx, minlength=k).to(X.dtype)
        new = torch.where(cnt[:, None] > 0, sums / cnt.clamp_min(1)[:, None], old)
        return new, cnt


class KMeansClustering:
    def __init__(self, strategy, seed=None):
        self.strategy = strategy
        self.seed = seed
        self.history = _History()
        self.clusterSet = None

    @staticmethod
    def setup(clusterCount, maxIterOrRate, distanceFunction="euclidean", inverse=False, allowEmptyClusters=False,
              seed=None):
        s = FixedClusterCountStrategy.setup(clusterCount, distanceFunction, inverse)
        if isinstance(maxIterOrRate, int):
            s.endWhenIterationCountEquals(maxIterOrRate)
        else:
            s.endWhenDistributionVariationRateLessThan(float(maxIterOrRate))
        s.allowEmptyClusters = allowEmptyClusters
        return KMeansClustering(s, seed)

    def _seed_centers(self, X, k, gen):
        """k-means++ seeding (first centre uniform, then ~ squared distance to the nearest centre), greedy variant:
        2 + log(k) candidates per step, keeping the one that lowers the potential most."""
        n = X.shape[0]
        fn, inv = self.strategy.distanceFunction, self.strategy.inverse
        sign = -1.0 if (inv or fn in SIMILARITIES) else 1.0

        def sqd(c):
            d = pairwise(X, c.reshape(1, -1), fn)[:, 0] * sign
            return d * d
        first = int(torch.randint(n, (1,), generator=gen))
        centers = [X[first]]
        dx = sqd(X[first])
        trials = 2 + int(math.log(max(k, 2)))
        while len(centers) < min(k, n):
            w = dx.clamp_min(0).double().cpu()
            if float(w.sum()) <= 0:
                break
            cand = torch.multinomial(w / w.sum(), trials, replacement=True, generator=gen).tolist()
            best = None
            for i in cand:
                nd = torch.minimum(dx, sqd(X[i]))
                pot = float(nd.sum())
                if best is None or pot < best[0]:
                    best = (pot, i, nd)
            centers.append(X[best[1]])
            dx = best[2]
        return torch.stack(centers)

    def applyTo(self, points, device=None):
        """Cluster a list of Points (or an [N, d] tensor); returns the ClusterSet."""
        if isinstance(points, torch.Tensor):
            points = Point.toPoints(points)
        dev = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        X = torch.stack([p.array for p in points]).to(dev)
        s = self.strategy
        k = s.initialClusterCount
        gen = torch.Generator().manual_seed(self.seed if self.seed is not None else 12345)
        C = self._seed_centers(X, k, gen).to(dev)
        hist = self.history = _History()
        prev = None
        cond = s.terminationCondition or FixedIterationCountCondition(100)
        while True:
            hist.iteration += 1
            idx, dist = ClusterUtils.assign(X, C, s.distanceFunction, s.inverse)
            C, cnt = ClusterUtils.refreshCenters(X, idx, C.shape[0], C)
            if not s.allowEmptyClusters and bool((cnt == 0).any()):
                # re-seed empty clusters at the points farthest from their centre (split most spread-out)
                empty = torch.nonzero(cnt == 0)[:, 0]
                far = torch.topk(dist.abs(), len(empty)).indices
                C[empty] = X[far]
            hist.variances.append(float((dist * dist).mean()))
            hist.moved_fraction = 1.0 if prev is None else float((idx != prev).float().mean())
            prev = idx
            if cond.isSatisfied(hist) or hist.iteration >= 10000:
                break
        cs = ClusterSet(s.distanceFunction, s.inverse)
        for j in range(C.shape[0]):
            cs.addNewClusterWithCenter(Point(f"center_{j}", None, C[j].cpu()))
        idx = idx.cpu().tolist()
        for p, j in zip(points, idx):
            cs.clusters[j].points.append(p)
            cs.pointDistribution[p.id] = j
        self.clusterSet = cs
        self.centers = C
        return cs

    def getClusterSet(self):
        return self.clusterSet


_ = math
