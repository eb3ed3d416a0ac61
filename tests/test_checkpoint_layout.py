"""ModelSerializer ``coefficients.bin`` byte layout, pinned per parameter initializer.

For every initializer the expected flat parameter vector is built BY HAND from the reference's layout rules (not
from this framework's ParamSpec tables), the network's parameter views are filled with distinct values, and the
checkpoint bytes must equal an independently assembled ND4J ``Nd4j.write`` stream of that vector; restoring must give
back every value. Reference layouts:
  * Dense / Output / Embedding (DefaultParamInitializer.java:114-146): W [nIn, nOut] stored 'f', then b [1, nOut]
  * Convolution (ConvolutionParamInitializer.java:118-122): b [1, nOut] FIRST, then W [nOut, nIn, kH, kW] 'c'
  * LSTM (LSTMParamInitializer.java:126-167): W [nIn, 4H] 'f', RW [H, 4H] 'f', b [1, 4H]
  * GravesLSTM (GravesLSTMParamInitializer): as LSTM with RW [H, 4H + 3] (peepholes)
  * BatchNormalization (BatchNormalizationParamInitializer.java:88-102): gamma, beta, mean, var, each [1, C]
ND4J stream (Nd4j.write, big-endian DataOutputStream): shape-info buffer UTF(alloc) | int n | UTF("INT") | n ints
[rank, shape, stride, offset, ews, order] followed by the data buffer UTF(alloc) | int n | UTF("FLOAT") | n floats.
"""
import io
import struct
import zipfile

import numpy as np
import pytest
import torch


def _utf(s):
    b = s.encode()
    return struct.pack(">H", len(b)) + b


def nd4j_row_bytes(flat):
    """Nd4j.write of a [1, P] 'c' float row vector, assembled independently of utils/nd4j_io.py."""
    P = flat.size
    info = [2, 1, P, P, 1, 0, 1, ord("c")]
    out = _utf("HEAP") + struct.pack(">i", len(info)) + _utf("INT") + struct.pack(f">{len(info)}i", *info)
    out += _utf("HEAP") + struct.pack(">i", P) + _utf("FLOAT") + np.asarray(flat, dtype=">f4").tobytes()
    return out


def _vals(shape, base):
    n = int(np.prod(shape))
    return (np.arange(n, dtype=np.float64).reshape(shape) * 0.25 + base).astype(np.float32)


def _net(layers, kind="mln", input_type=None):
    from deeplearning4j_amd import MultiLayerNetwork, NeuralNetConfiguration
    b = NeuralNetConfiguration.Builder().seed(1).list()
    for i, l in enumerate(layers):
        b = b.layer(i, l)
    if input_type is not None:
        b = b.setInputType(input_type)
    net = MultiLayerNetwork(b.build())
    net.init()
    return net


def _fill(net, values):
    """values: {param key: logical ndarray}; writes through the network's parameter views."""
    table = net.paramTable()
    with torch.no_grad():
        for k, v in values.items():
            view = table[k]
            assert tuple(view.shape) == v.shape, (k, tuple(view.shape), v.shape)
            view.copy_(torch.from_numpy(v))
    net.sync_shadow()


def _check(net, expected_flat, values, tmp_path):
    from deeplearning4j_amd.utils.model_serializer import ModelSerializer
    got = net.params().detach().reshape(-1).numpy()
    assert got.shape == expected_flat.shape
    assert np.array_equal(got, expected_flat)
    path = str(tmp_path / "m.zip")
    ModelSerializer.writeModel(net, path, False)
    with zipfile.ZipFile(path) as z:
        data = z.read("coefficients.bin")
    assert data == nd4j_row_bytes(expected_flat)
    back = ModelSerializer.restoreMultiLayerNetwork(path, False)
    table = back.paramTable()
    for k, v in values.items():
        assert np.array_equal(table[k].detach().numpy(), v), k


def f_order(a):
    return np.asarray(a).reshape(-1, order="F")


def test_dense_and_output_layout(tmp_path):
    from deeplearning4j_amd import DenseLayer, LossFunction, OutputLayer
    net = _net([DenseLayer.Builder().nIn(3).nOut(4).build(),
                OutputLayer.Builder(LossFunction.MSE).nIn(4).nOut(2).build()])
    v = {"0_W": _vals((3, 4), 1), "0_b": _vals((1, 4), 100), "1_W": _vals((4, 2), 200), "1_b": _vals((1, 2), 300)}
    _fill(net, v)
    want = np.concatenate([f_order(v["0_W"]), v["0_b"].ravel(), f_order(v["1_W"]), v["1_b"].ravel()])
    _check(net, want, v, tmp_path)


def test_convolution_layout_bias_first(tmp_path):
    from deeplearning4j_amd import LossFunction, OutputLayer
    from deeplearning4j_amd.nn.conf.inputs import InputType
    from deeplearning4j_amd.nn.conf.layers import ConvolutionLayer
    net = _net([ConvolutionLayer.Builder(2, 3).nIn(2).nOut(3).build(),
                OutputLayer.Builder(LossFunction.MSE).nOut(2).build()], input_type=InputType.convolutional(4, 5, 2))
    v = {"0_W": _vals((3, 2, 2, 3), 1), "0_b": _vals((1, 3), 500)}
    n_out_in = net.paramTable()["1_W"].shape
    v["1_W"] = _vals(tuple(n_out_in), 700)
    v["1_b"] = _vals((1, 2), 900)
    _fill(net, v)
    want = np.concatenate([v["0_b"].ravel(), v["0_W"].reshape(-1), f_order(v["1_W"]), v["1_b"].ravel()])
    _check(net, want, v, tmp_path)


@pytest.mark.parametrize("graves", [False, True])
def test_lstm_layout(tmp_path, graves):
    from deeplearning4j_amd import LossFunction
    from deeplearning4j_amd.nn.conf.layers import LSTM, GravesLSTM, RnnOutputLayer
    H, nIn = 3, 2
    L = GravesLSTM if graves else LSTM
    net = _net([L.Builder().nIn(nIn).nOut(H).build(),
                RnnOutputLayer.Builder(LossFunction.MSE).nIn(H).nOut(2).build()])
    rw_cols = 4 * H + (3 if graves else 0)
    v = {"0_W": _vals((nIn, 4 * H), 1), "0_RW": _vals((H, rw_cols), 50), "0_b": _vals((1, 4 * H), 150),
         "1_W": _vals((H, 2), 300), "1_b": _vals((1, 2), 400)}
    _fill(net, v)
    want = np.concatenate([f_order(v["0_W"]), f_order(v["0_RW"]), v["0_b"].ravel(), f_order(v["1_W"]),
                           v["1_b"].ravel()])
    _check(net, want, v, tmp_path)


def test_batchnorm_layout(tmp_path):
    from deeplearning4j_amd import DenseLayer, LossFunction, OutputLayer
    from deeplearning4j_amd.nn.conf.layers import BatchNormalization
    net = _net([DenseLayer.Builder().nIn(2).nOut(3).build(), BatchNormalization.Builder().nOut(3).build(),
                OutputLayer.Builder(LossFunction.MSE).nIn(3).nOut(2).build()])
    keys = [k for k in net.paramTable() if k.startswith("1_")]
    assert keys == ["1_gamma", "1_beta", "1_mean", "1_var"], keys
    v = {"0_W": _vals((2, 3), 1), "0_b": _vals((1, 3), 10), "1_gamma": _vals((1, 3), 20),
         "1_beta": _vals((1, 3), 30), "1_mean": _vals((1, 3), 40), "1_var": _vals((1, 3), 50),
         "2_W": _vals((3, 2), 60), "2_b": _vals((1, 2), 70)}
    _fill(net, v)
    want = np.concatenate([f_order(v["0_W"]), v["0_b"].ravel(), v["1_gamma"].ravel(), v["1_beta"].ravel(),
                           v["1_mean"].ravel(), v["1_var"].ravel(), f_order(v["2_W"]), v["2_b"].ravel()])
    _check(net, want, v, tmp_path)


def test_embedding_layout(tmp_path):
    from deeplearning4j_amd import LossFunction, OutputLayer
    from deeplearning4j_amd.nn.conf.layers import EmbeddingLayer
    net = _net([EmbeddingLayer.Builder().nIn(5).nOut(3).build(),
                OutputLayer.Builder(LossFunction.MSE).nIn(3).nOut(2).build()])
    v = {"0_W": _vals((5, 3), 1), "0_b": _vals((1, 3), 40), "1_W": _vals((3, 2), 80), "1_b": _vals((1, 2), 90)}
    _fill(net, v)
    want = np.concatenate([f_order(v["0_W"]), v["0_b"].ravel(), f_order(v["1_W"]), v["1_b"].ravel()])
    _check(net, want, v, tmp_path)


def test_codec_matches_independent_stream():
    from deeplearning4j_amd.utils import nd4j_io
    flat = _vals((1, 17), -3).ravel()
    assert nd4j_io.to_bytes(torch.from_numpy(flat).reshape(1, -1)) == nd4j_row_bytes(flat)
    back = nd4j_io.from_bytes(nd4j_row_bytes(flat))
    assert np.array_equal(back.reshape(-1).numpy(), flat)
    _ = io
