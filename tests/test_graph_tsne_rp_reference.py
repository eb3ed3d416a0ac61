"""Small ports, after the reference's TestGraphLoadingWeighted (deeplearning4j-graph/src/test/java/org/deeplearning4j/
graph/data/TestGraphLoadingWeighted.java:20-95), RPUtilsTest (nearestneighbor-core/src/test/java/org/deeplearning4j/
clustering/randomprojection/RPUtilsTest.java:12-25) and BarnesHutTsneTest (deeplearning4j-core/src/test/java/org/
deeplearning4j/plot/BarnesHutTsneTest.java:30-100): the reference's WeightedGraph.txt loads as a directed weighted
graph with the expected out-degrees, targets and weights, and equals the graph built through an EdgeLineProcessor +
VertexFactory; batched distances equal per-row distances; Barnes-Hut t-SNE builder fields are kept and a 10-iteration
fit runs on 100 x 784 inputs (the reference reads mnist2500_X.txt, which this tree does not hold: a seeded stand-in of
that shape). CPU."""
import torch

from deeplearning4j_amd.clustering import RPUtils
from deeplearning4j_amd.graph import GraphLoader, StringVertexFactory, WeightedEdgeLineProcessor
from deeplearning4j_amd.plot import BarnesHutTsne

from _ref_fixtures import path as _ref_path

WEIGHTED = _ref_path("deeplearning4j-graph/src/test/resources/WeightedGraph.txt")


def test_weighted_directed():
    g = GraphLoader.loadWeightedEdgeListFile(WEIGHTED, 9, ",", True, ["//"])
    assert g.numVertices() == 9
    assert [g.getVertexDegree(i) for i in range(9)] == [2, 2, 1, 2, 2, 1, 1, 1, 1]
    edges = [[1, 3], [2, 4], [5], [4, 6], [5, 7], [8], [7], [8], [0]]
    weights = [[1, 3], [12, 14], [25], [34, 36], [45, 47], [58], [67], [78], [80]]
    for i in range(9):
        out = g.getEdgesOut(i)
        assert len(out) == len(edges[i])
        for e in out:
            assert e.getFrom() == i and e.getTo() in edges[i]
            assert e.getValue() == weights[i][edges[i].index(e.getTo())]


def test_weighted_directed_v2():
    g = GraphLoader.loadWeightedEdgeListFile(WEIGHTED, 9, ",", True, False, ["//"])
    assert g.numVertices() == 9
    g2 = GraphLoader.loadGraph(WEIGHTED, WeightedEdgeLineProcessor(",", True, ["//"]), StringVertexFactory(), 9, False)
    assert g == g2


def test_rp_distance_compute_batch():
    x = torch.linspace(1, 4, 4)
    y = torch.linspace(1, 16, 16).reshape(4, 4)
    result = torch.zeros(4)
    d = RPUtils.computeDistanceMulti("euclidean", x, y, result)
    for i in range(4):
        assert abs(RPUtils.computeDistance("euclidean", x, y[i]) - float(d[i])) < 1e-3
    assert torch.equal(result, d)


def test_tsne_fit_runs():
    torch.manual_seed(123)
    b = BarnesHutTsne.Builder().stopLyingIteration(10).setMaxIter(10).theta(0.5).learningRate(500) \
        .useAdaGrad(False).build()
    g = torch.Generator().manual_seed(123)
    data = (torch.rand(100, 784, generator=g) < 0.2).double()
    b.fit(data)
    y = b.getData() if hasattr(b, "getData") else b.Y
    assert tuple(y.shape) == (100, 2) and torch.isfinite(torch.as_tensor(y)).all()


def test_tsne_builder_fields():
    b = (BarnesHutTsne.Builder().theta(0).invertDistanceMetric(False).similarityFunction("euclidean").setMaxIter(1)
         .setRealMin(1.0).setInitialMomentum(2.0).setFinalMomentum(3.0).setMomentum(4.0).setSwitchMomentumIteration(1)
         .normalize(False).stopLyingIteration(100).tolerance(1e-1).learningRate(100).perplexity(1.0).minGain(1.0)
         .build())
    assert b.getTheta() == 0 and b.isInvert() is False and b.getSimiarlityFunction() == "euclidean"
    assert b.maxIter == 1 and b.realMin == 1.0 and b.initialMomentum == 2.0 and b.finalMomentum == 3.0
    assert b.momentum == 4.0 and b.switchMomentumIteration == 1 and b.normalize is False
    assert b.stopLyingIteration == 100 and b.tolerance == 1e-1 and b.learningRate == 100
    assert b.useAdaGrad is False and b.getPerplexity() == 1.0 and b.minGain == 1.0
