"""Nearest neighbours and clustering.

Reference: deeplearning4j-nearestneighbors-parent/nearestneighbor-core (clustering/vptree, kdtree, lsh,
randomprojection, kmeans, cluster, strategy, condition, sptree, quadtree) and the REST server
(deeplearning4j-nearestneighbor-server NearestNeighborsServer.java: POST /knn, /knnnew).

MI355X split: tree structures (VP-tree, SP/quad-tree) are pointer-chasing host work in C++
(csrc/runtime/trees.cpp); dense work — brute-force k-NN, k-means assignment, LSH hashing — is GEMM-shaped and runs
on the GPU through torch (rocBLAS/hipBLASLt GEMM + top-k) whenever the data lives there.
"""
from .distances import DISTANCES, pairwise, knn_bruteforce  # noqa: F401
from .vptree import DataPoint, VPTree, VPTreeFillSearch  # noqa: F401
from .kdtree import HyperRect, KDTree  # noqa: F401
from .lsh import RandomProjectionLSH  # noqa: F401
from .rpforest import RPForest, RPTree, RPUtils  # noqa: F401
from .kmeans import (Cluster, ClusterSet, ClusterUtils, ConvergenceCondition, FixedClusterCountStrategy,  # noqa
                     FixedIterationCountCondition, KMeansClustering, OptimisationStrategy, Point,
                     PointClassification, VarianceVariationCondition)
from .sptree import QuadTree, SpTree  # noqa: F401
