"""Graph vertices at the vertex level, after the reference's TestGraphNodes
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/graph/TestGraphNodes.java:134-545): SubsetVertex (2-D and
4-D), LastTimeStepVertex (with and without a per-example mask), DuplicateToTimeSeriesVertex, StackVertex and
UnstackVertex forward / backward, L2Vertex against the hand-written distance and its derivative, and the graph JSON
round trip of configurations using them. fp64, CPU."""
import pytest
import torch

import deeplearning4j_amd as D


def _rand(*shape, seed=12345):
    return torch.rand(*shape, generator=torch.Generator().manual_seed(seed), dtype=torch.float64)


@pytest.mark.parametrize("shape", [(5, 10), (5, 10, 3, 3)])
def test_subset_vertex(shape):
    v = D.SubsetVertex(4, 7)
    x = _rand(*shape)
    out, ctx = v.forward([x])
    assert torch.equal(out, x[:, 4:8])
    (back,) = v.backward(out, ctx)
    assert tuple(back.shape) == tuple(x.shape)
    assert torch.count_nonzero(back[:, :4]) == 0 and torch.count_nonzero(back[:, 8:]) == 0
    assert torch.equal(back[:, 4:8], out)


def _last_ts_conf():
    return (D.NeuralNetConfiguration.Builder().graphBuilder().addInputs("in")
            .addVertex("lastTS", D.LastTimeStepVertex("in"), "in")
            .addLayer("out", D.OutputLayer.Builder().nIn(5).nOut(1).build(), "lastTS").setOutputs("out").build())


def test_last_time_step_vertex():
    conf = _last_ts_conf()
    g = D.ComputationGraph(conf)
    g.init()
    v = g.conf.vertices["lastTS"]
    x = _rand(3, 5, 6)
    out, ctx = v.forward([x], True)
    assert torch.equal(out, x[:, :, 5])
    (eps,) = v.backward(out, ctx)
    assert tuple(eps.shape) == (3, 5, 6)
    assert torch.count_nonzero(eps[:, :, :5]) == 0 and torch.equal(eps[:, :, 5], out)
    mask = torch.tensor([[1, 1, 1, 0, 0, 0], [1, 1, 1, 1, 0, 0], [1, 1, 1, 1, 1, 0]], dtype=torch.float64)
    out, ctx = v.forward([x], True, [mask])
    assert torch.equal(out, torch.stack([x[0, :, 2], x[1, :, 3], x[2, :, 4]]))
    (eps,) = v.backward(out, ctx)
    assert torch.equal(eps[1, :, 3], out[1]) and torch.count_nonzero(eps[1, :, 4:]) == 0
    # through the network: the masked last step feeds the output layer
    g.setLayerMaskArrays([mask], None)
    assert torch.allclose(g.feedForward([x.float()], False)["lastTS"].double(), out, atol=1e-6)
    assert D.ComputationGraphConfiguration.fromJson(conf.toJson()).toJson() == conf.toJson()


def test_duplicate_to_time_series_vertex():
    conf = (D.NeuralNetConfiguration.Builder().graphBuilder().addInputs("in2d", "in3d")
            .addVertex("duplicateTS", D.DuplicateToTimeSeriesVertex("in3d"), "in2d")
            .addLayer("out", D.RnnOutputLayer.Builder().nIn(5).nOut(1).build(), "duplicateTS")
            .addLayer("out3d", D.RnnOutputLayer.Builder().nIn(2).nOut(1).build(), "in3d")
            .setOutputs("out", "out3d").build())
    g = D.ComputationGraph(conf)
    g.init()
    in2d, in3d = _rand(3, 5), _rand(3, 2, 7, seed=1)
    acts = g.feedForward([in2d.float(), in3d.float()], False)
    exp = in2d.unsqueeze(2).expand(3, 5, 7)
    assert torch.allclose(acts["duplicateTS"].double(), exp, atol=1e-6)
    v = g.conf.vertices["duplicateTS"]
    out, ctx = v.forward([in2d], T=7)
    assert torch.equal(out, exp)
    (back,) = v.backward(exp, ctx)
    assert torch.allclose(back, exp.sum(2))
    assert D.ComputationGraphConfiguration.fromJson(conf.toJson()).toJson() == conf.toJson()


def test_stack_and_unstack_vertices():
    ins = [_rand(5, 2, seed=i) for i in range(3)]
    stack = D.StackVertex()
    out, ctx = stack.forward(ins)
    for i in range(3):
        assert torch.equal(out[5 * i:5 * (i + 1)], ins[i])
    back = stack.backward(out, ctx)
    for i in range(3):
        assert torch.equal(back[i], ins[i])
    for shape in [(15, 2), (15, 10, 3, 3)]:
        x = _rand(*shape, seed=7)
        for k in range(3):
            u = D.UnstackVertex(k, 3)
            o, c = u.forward([x])
            assert torch.equal(o, x[5 * k:5 * (k + 1)])
            (b,) = u.backward(o, c)
            assert torch.equal(b[5 * k:5 * (k + 1)], o)
            assert torch.count_nonzero(b) == torch.count_nonzero(o)


def test_l2_vertex():
    a, b = _rand(5, 2, seed=1), _rand(5, 2, seed=2)
    v = D.L2Vertex()
    out, ctx = v.forward([a, b])
    exp = torch.sqrt(((a - b) ** 2).sum(1, keepdim=True))
    assert torch.allclose(out, exp, atol=1e-14)
    eps = _rand(5, 1, seed=3)                         # dL/dlambda
    da, db = v.backward(eps, ctx)
    exp_da = (a - b) * (eps / exp)                    # d||a-b||/da = (a-b)/||a-b||
    assert torch.allclose(da, exp_da, atol=1e-12)
    assert torch.allclose(db, -exp_da, atol=1e-12)
