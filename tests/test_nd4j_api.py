"""ND4J-compatible INDArray / Nd4j / Transforms surface (CPU; semantics from the reference's ND4J usage)."""
import io

import numpy as np
import pytest
import torch

from deeplearning4j_amd.nd4j import INDArray, NDArrayIndex, Nd4j, Transforms


@pytest.fixture(autouse=True)
def _cpu(monkeypatch):
    monkeypatch.setenv("DL4J_AMD_ND4J_DEVICE", "cpu")


def test_create_orders_and_vectors():
    v = Nd4j.create([1.0, 2.0, 3.0])
    assert v.shape() == [1, 3] and v.isRowVector() and v.isVector()
    c = Nd4j.create([1.0, 2, 3, 4, 5, 6], [2, 3])
    f = Nd4j.create([1.0, 2, 3, 4, 5, 6], [2, 3], "f")
    assert c.ordering() == "c" and f.ordering() == "f"
    np.testing.assert_array_equal(np.asarray(c), [[1, 2, 3], [4, 5, 6]])
    np.testing.assert_array_equal(np.asarray(f), [[1, 3, 5], [2, 4, 6]])
    assert f.stride() == [1, 2]
    assert c.dup("f").ordering() == "f" and c.dup("f").equals(c)
    z = Nd4j.zeros(2, 4, "f")
    assert z.ordering() == "f" and z.sumNumber() == 0
    assert Nd4j.ones(3, 2).sumNumber() == 6
    assert Nd4j.valueArrayOf([2, 2], 7.0).meanNumber() == 7
    assert Nd4j.scalar(3.5).getDouble(0) == 3.5
    assert Nd4j.eye(3).sumNumber() == 3
    assert Nd4j.linspace(0, 1, 5).getDouble(0, 4) == 1.0
    assert Nd4j.arange(4).shape() == [1, 4]


def test_reshape_ravel_f_order():
    a = Nd4j.create([1.0, 2, 3, 4, 5, 6], [2, 3])
    np.testing.assert_array_equal(np.asarray(a.ravel("f")), [[1, 4, 2, 5, 3, 6]])
    np.testing.assert_array_equal(np.asarray(a.reshape("f", 3, 2)), [[1, 5], [4, 3], [2, 6]])
    np.testing.assert_array_equal(np.asarray(a.reshape(3, 2)), [[1, 2], [3, 4], [5, 6]])
    assert a.transpose().shape() == [3, 2] and a.transpose().ordering() == "f"
    assert a.permute(1, 0).equals(a.transpose())


def test_views_and_in_place_ops():
    a = Nd4j.create([1.0, 2, 3, 4, 5, 6], [2, 3])
    a.getRow(1).addi(10)                                        # view: writes through
    np.testing.assert_array_equal(np.asarray(a), [[1, 2, 3], [14, 15, 16]])
    a.getColumn(0).muli(0)
    assert a.getDouble(1, 0) == 0
    sub = a.get(NDArrayIndex.all(), NDArrayIndex.interval(1, 3))
    assert sub.shape() == [2, 2]
    sub.assign(1.0)
    np.testing.assert_array_equal(np.asarray(a), [[0, 1, 1], [0, 1, 1]])
    a.putScalar(0, 0, 9.0)
    a.putScalar(5, -1.0)                                        # linear index, c order
    assert a.getDouble(0, 0) == 9 and a.getDouble(1, 2) == -1
    p = a.get(NDArrayIndex.point(1), NDArrayIndex.all())
    assert p.shape() == [1, 3]
    sel = a.get(NDArrayIndex.all(), NDArrayIndex.indices(0, 2))
    assert sel.shape() == [2, 2]
    a.putRow(0, Nd4j.create([7.0, 8.0, 9.0]))
    np.testing.assert_array_equal(np.asarray(a.getRow(0)), [[7, 8, 9]])


def test_arithmetic_and_vector_broadcasts():
    a = Nd4j.create([1.0, 2, 3, 4], [2, 2])
    b = Nd4j.create([10.0, 20, 30, 40], [2, 2])
    assert a.add(b).sumNumber() == 110 and a.sumNumber() == 10
    assert a.rsub(1).getDouble(0, 0) == 0 and a.rdiv(4).getDouble(1, 1) == 1
    r = Nd4j.create([1.0, 2.0])
    np.testing.assert_array_equal(np.asarray(a.addRowVector(r)), [[2, 4], [4, 6]])
    np.testing.assert_array_equal(np.asarray(a.addColumnVector(r.transpose())), [[2, 3], [5, 6]])
    np.testing.assert_array_equal(np.asarray(a.divRowVector(r)), [[1, 1], [3, 2]])
    c = a.dup()
    c.muliColumnVector(Nd4j.create([[2.0], [3.0]]))
    np.testing.assert_array_equal(np.asarray(c), [[2, 4], [9, 12]])
    np.testing.assert_allclose(np.asarray(a.mmul(b)), np.asarray(a) @ np.asarray(b))
    np.testing.assert_allclose(np.asarray(a @ b + 1), np.asarray(a) @ np.asarray(b) + 1)
    assert a.dot(a) == 30
    assert a.gt(2).sumNumber() == 2 and a.eq(a).sumNumber() == 4
    d = a.dup()
    d += 1
    d *= 2
    assert d.sumNumber() == 28
    out = Nd4j.zeros(2, 2)
    Nd4j.gemm(a, b, True, False, out)
    np.testing.assert_allclose(np.asarray(out), np.asarray(a).T @ np.asarray(b))


def test_reductions():
    x = np.arange(24, dtype=np.float64).reshape(2, 3, 4)
    a = Nd4j.create(x)
    np.testing.assert_allclose(np.asarray(a.sum(0)), x.sum(0))
    np.testing.assert_allclose(np.asarray(a.mean(1, 2)), x.mean((1, 2)).reshape(1, -1))
    np.testing.assert_allclose(np.asarray(a.std(2)), x.std(2, ddof=1))
    np.testing.assert_allclose(np.asarray(a.var(False, 2)), x.var(2))
    np.testing.assert_allclose(np.asarray(a.norm2(2)), np.sqrt((x ** 2).sum(2)))
    np.testing.assert_allclose(np.asarray(a.norm1(0)), np.abs(x).sum(0))
    np.testing.assert_allclose(np.asarray(a.max(2)), x.max(2))
    m = Nd4j.create([[1.0, 5.0, 2.0], [7.0, 0.0, 3.0]])
    np.testing.assert_array_equal(np.asarray(m.argMax(1)), [[1, 0]])
    assert m.maxNumber() == 7 and m.minNumber() == 0 and m.norm2Number() == pytest.approx(np.sqrt(88))
    assert m.sum().shape() == [1, 1]
    assert a.tensorsAlongDimension(1, 2) == 2
    np.testing.assert_array_equal(np.asarray(a.tensorAlongDimension(1, 1, 2)), x[1])
    np.testing.assert_array_equal(np.asarray(a.tensorAlongDimension(2, 0)), x[:, 0, 2])
    np.testing.assert_array_equal(np.asarray(m.cumsum(1)), np.cumsum(np.asarray(m), 1))


def test_transforms():
    a = Nd4j.create([[-1.0, 0.0, 2.0]])
    np.testing.assert_allclose(np.asarray(Transforms.sigmoid(a)), 1 / (1 + np.exp([[1.0, 0.0, -2.0]])), rtol=1e-6)
    np.testing.assert_allclose(np.asarray(Transforms.relu(a)), [[0, 0, 2]])
    np.testing.assert_allclose(np.asarray(Transforms.pow(a, 2)), [[1, 0, 4]])
    np.testing.assert_allclose(np.asarray(Transforms.max(a, 0.5)), [[0.5, 0.5, 2]])
    s = Transforms.softmax(Nd4j.create([[1.0, 2.0, 3.0]]))
    assert s.sumNumber() == pytest.approx(1.0)
    b = a.dup()
    Transforms.abs(b, False)                                   # in place
    assert b.minNumber() == 0 and b.sumNumber() == 3
    u, v = Nd4j.create([1.0, 0.0]), Nd4j.create([1.0, 1.0])
    assert Transforms.cosineSim(u, v) == pytest.approx(1 / np.sqrt(2))
    assert Transforms.euclideanDistance(u, v) == pytest.approx(1.0)
    assert Transforms.manhattanDistance(u, v) == pytest.approx(1.0)
    assert Transforms.unitVec(Nd4j.create([3.0, 4.0])).norm2Number() == pytest.approx(1.0)
    sims = Transforms.allCosineSimilarities(Nd4j.create([[1.0, 0.0], [0.0, 1.0]]), Nd4j.create([[1.0, 1.0]]))
    assert sims.shape() == [2, 1]


def test_stacking_flatten_average():
    a, b = Nd4j.ones(2, 2), Nd4j.zeros(2, 2)
    assert Nd4j.hstack(a, b).shape() == [2, 4] and Nd4j.vstack([a, b]).shape() == [4, 2]
    assert Nd4j.concat(0, a, b).shape() == [4, 2] and Nd4j.stack(0, a, b).shape() == [2, 2, 2]
    flat = Nd4j.toFlattened(Nd4j.create([1.0, 2, 3, 4], [2, 2]), Nd4j.create([5.0, 6.0]))
    np.testing.assert_array_equal(np.asarray(flat), [[1, 2, 3, 4, 5, 6]])
    flat_f = Nd4j.toFlattened([Nd4j.create([1.0, 2, 3, 4], [2, 2])], order="f")
    np.testing.assert_array_equal(np.asarray(flat_f), [[1, 3, 2, 4]])
    xs = [Nd4j.create([1.0, 3.0]), Nd4j.create([3.0, 5.0])]
    Nd4j.averageAndPropagate(None, xs)
    assert xs[0].equals(xs[1]) and xs[0].getDouble(0, 0) == 2
    s = Nd4j.sort(Nd4j.create([[3.0, 1.0, 2.0]]), 1, True)
    np.testing.assert_array_equal(np.asarray(s), [[1, 2, 3]])


def test_binary_codec_round_trip(tmp_path):
    a = Nd4j.create([1.0, 2, 3, 4, 5, 6], [2, 3], "f")
    buf = io.BytesIO()
    Nd4j.write(a, buf, "f")
    buf.seek(0)
    b = Nd4j.readArray(buf)
    assert isinstance(b, INDArray) and b.equals(a)
    p = str(tmp_path / "a.bin")
    Nd4j.saveBinary(a, p)
    assert Nd4j.readBinary(p).equals(a)
    t = str(tmp_path / "a.txt")
    Nd4j.writeTxt(a, t)
    assert Nd4j.readTxt(t).equals(a)


def test_indarrays_feed_networks():
    from deeplearning4j_amd import (Activation, DataSet, DenseLayer, LossFunction, MultiLayerNetwork,
                                    NeuralNetConfiguration, OutputLayer, Sgd)
    conf = (NeuralNetConfiguration.Builder().seed(1).updater(Sgd(0.1)).list()
            .layer(0, DenseLayer.Builder().nIn(4).nOut(5).activation(Activation.TANH).build())
            .layer(1, OutputLayer.Builder(LossFunction.MSE).nIn(5).nOut(2).activation(Activation.IDENTITY).build())
            .build())
    net = MultiLayerNetwork(conf)
    net.init(device=torch.device("cpu"))
    Nd4j.getRandom().setSeed(3)
    x, y = Nd4j.rand(8, 4), Nd4j.rand(8, 2)
    net.fit(DataSet(x, y))
    out = net.output(x)
    assert tuple(out.shape) == (8, 2)
    assert Nd4j.getAffinityManager().getNumberOfDevices() >= 1
