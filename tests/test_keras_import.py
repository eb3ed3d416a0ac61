"""Keras import on the reference's own HDF5 fixtures (KER test resources weights/*.h5, read with our HDF5 parser).

Shape checks mirror KerasWeightSettingTests.java (dense W [4,6], conv W [6,5,3,3], embedding+LSTM output
[42,6,10] ...). Numerics: the imported network's output is compared with an independent numpy forward written
in Keras semantics (channels-last tensors, Keras gate order, hard_sigmoid, Theano true convolution) directly
from the raw Keras weight arrays. No Keras is installed and the fixtures hold no reference outputs, so agreement
with Keras itself is "parity unpinned" beyond these semantics.
"""
import glob
import os

import numpy as np
import pytest
import torch

from deeplearning4j_amd.modelimport import hdf5
from deeplearning4j_amd.modelimport.keras import (KerasLayer, KerasModelImport, UnsupportedKerasConfigurationException,
                                                   space_to_depth_mapper)
from _ref_fixtures import path as _ref_path

R = _ref_path("deeplearning4j-modelimport/src/test/resources/weights") + "/"
pytestmark = pytest.mark.skipif(not os.path.isdir(R), reason="reference fixtures not present")
CPU = torch.device("cpu")


def _kw(path, layer):
    f = hdf5.File(path)
    root = f["model_weights"] if "model_weights" in f else f
    g = root[layer]
    out = {}
    for n in g.attrs["weight_names"]:
        k = n.split("/")[-1].split(":")[0]
        if n.count("/") >= 2:
            k = n.split("/")[-2] + "/" + k
        elif k.startswith(layer + "_"):
            k = k[len(layer) + 1:]
        out[k] = np.asarray(g[n].read(), dtype=np.float64)
    return out


def _names(path):
    f = hdf5.File(path)
    root = f["model_weights"] if "model_weights" in f else f
    return list(root.attrs["layer_names"])


def _fixtures(prefix):
    return sorted(glob.glob(R + prefix + "_t*.h5"))


def _import(p):
    return KerasModelImport.importKerasModelAndWeights(p, device=CPU)


def _out(net, x):
    return net.output(torch.as_tensor(x, dtype=torch.float32)).detach().double().numpy()


def _theano(p):
    return "theano_2" in p          # Keras 2 files record the backend; Keras 1 files are imported as TensorFlow


def _conv2d_keras(x, k, b, theano):
    """x [n,h,w,c], k [kh,kw,c,o] -> valid conv, channels-last."""
    if theano:
        k = k[::-1, ::-1]
    n, H, W, C = x.shape
    kh, kw, _, O = k.shape
    out = np.zeros((n, H - kh + 1, W - kw + 1, O))
    for i in range(H - kh + 1):
        for j in range(W - kw + 1):
            out[:, i, j] = np.einsum("nabc,abco->no", x[:, i:i + kh, j:j + kw], k)
    return out + b


def _hs(z):
    return np.clip(0.2 * z + 0.5, 0, 1)


def _split4(a, H):
    return [a[..., i * H:(i + 1) * H] for i in range(4)]


def _lstm_keras(x, kw, prefix=""):
    """x [n,T,f]; Keras gate order i,f,c,o; returns all h [n,T,H]."""
    if prefix + "kernel" in kw:
        U = kw[prefix + "recurrent_kernel"]
        H = U.shape[0]
        Wi, Wf, Wc, Wo = _split4(kw[prefix + "kernel"], H)
        Ui, Uf, Uc, Uo = _split4(U, H)
        bi, bf, bc, bo = _split4(kw[prefix + "bias"], H)
    else:
        Wi, Wf, Wc, Wo = (kw[prefix + "W_" + g] for g in "ifco")
        Ui, Uf, Uc, Uo = (kw[prefix + "U_" + g] for g in "ifco")
        bi, bf, bc, bo = (kw[prefix + "b_" + g] for g in "ifco")
        H = Ui.shape[0]
    n, T, _ = x.shape
    h = np.zeros((n, H))
    c = np.zeros((n, H))
    hs = []
    for t in range(T):
        xt = x[:, t]
        i = _hs(xt @ Wi + h @ Ui + bi)
        f = _hs(xt @ Wf + h @ Uf + bf)
        g = np.tanh(xt @ Wc + h @ Uc + bc)
        o = _hs(xt @ Wo + h @ Uo + bo)
        c = f * c + i * g
        h = o * np.tanh(c)
        hs.append(h)
    return np.stack(hs, 1)


def test_all_fixtures_import():
    KerasLayer.registerCustomLayer("Lambda", space_to_depth_mapper(2))
    try:
        n = 0
        for p in sorted(glob.glob(R + "*.h5")):
            net = _import(p)
            assert net.numParams() >= 0
            n += 1
        assert n == 35
    finally:
        KerasLayer.clearCustomLayers()


def test_lambda_requires_registration():
    with pytest.raises(UnsupportedKerasConfigurationException):
        _import(R + "space_to_depth_simple_tensorflow_2.h5")


@pytest.mark.parametrize("p", _fixtures("dense"))
def test_dense(p):
    net = _import(p)
    assert tuple(net.layers[0].params["W"].shape) == (4, 6)
    kw = _kw(p, _names(p)[0])
    x = np.random.RandomState(0).randn(3, 4)
    ref = x @ kw["kernel" if "kernel" in kw else "W"] + kw["bias" if "bias" in kw else "b"]
    np.testing.assert_allclose(_out(net, x), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("p", _fixtures("conv2d"))
def test_conv2d(p):
    net = _import(p)
    assert tuple(net.layers[0].params["W"].shape) == (6, 5, 3, 3)
    kw = _kw(p, _names(p)[0])
    k = kw.get("kernel", kw.get("W"))
    b = kw.get("bias", kw.get("b"))
    x = np.random.RandomState(1).randn(2, 5, 5, 5)             # NHWC as Keras sees it
    ref = _conv2d_keras(x, k, b, _theano(p))
    got = _out(net, x.transpose(0, 3, 1, 2)).transpose(0, 2, 3, 1)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("p", _fixtures("batch_to_conv2d"))
def test_dense_reshape_bn_conv(p):
    net = _import(p)
    names = _names(p)
    import json
    cfg = json.loads(hdf5.File(p).attrs["model_config"])
    layers = cfg["config"] if isinstance(cfg["config"], list) else cfg["config"]["layers"]
    target = layers[1]["config"]["target_shape"]
    eps = layers[2]["config"]["epsilon"]
    dense = _kw(p, names[0])
    bn = _kw(p, names[2])
    conv = _kw(p, names[3])
    x = np.random.RandomState(2).randn(3, 100)
    h = x @ dense.get("kernel", dense.get("W")) + dense.get("bias", dense.get("b"))
    h = h.reshape(3, *target)
    mean = bn.get("moving_mean", bn.get("running_mean"))
    var = bn.get("moving_variance", bn.get("running_std"))
    h = (h - mean) / np.sqrt(var + eps) * bn["gamma"] + bn["beta"]
    ref = _conv2d_keras(h, conv.get("kernel", conv.get("W")), conv.get("bias", conv.get("b")), _theano(p))
    got = _out(net, x).transpose(0, 2, 3, 1)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("p", _fixtures("lstm"))
def test_lstm_last_step(p):
    net = _import(p)
    kw = _kw(p, _names(p)[0])
    x = np.random.RandomState(3).randn(2, 4, 1)
    ref = _lstm_keras(x, kw)[:, -1]
    got = _out(net, x.transpose(0, 2, 1))
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("p", _fixtures("simple_rnn"))
def test_simple_rnn(p):
    net = _import(p)
    kw = _kw(p, _names(p)[0])
    W = kw.get("kernel", kw.get("W"))
    U = kw.get("recurrent_kernel", kw.get("U"))
    b = kw.get("bias", kw.get("b"))
    x = np.random.RandomState(4).randn(2, 4, 1)
    h = np.zeros((2, U.shape[0]))
    for t in range(4):
        h = np.tanh(x[:, t] @ W + h @ U + b)
    np.testing.assert_allclose(_out(net, x.transpose(0, 2, 1)), h, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("p", _fixtures("embedding_lstm"))
def test_embedding_lstm(p):
    net = _import(p)
    names = _names(p)
    emb = _kw(p, names[0])
    lstm = _kw(p, names[1])
    idx = np.random.RandomState(5).randint(0, emb.get("embeddings", emb.get("W")).shape[0], size=(42, 10))
    E = emb.get("embeddings", emb.get("W"))
    ref = _lstm_keras(E[idx], lstm)                          # [n, T, H]
    got = _out(net, idx.astype(np.float32))
    assert got.shape == (42, 6, 10)
    np.testing.assert_allclose(got.transpose(0, 2, 1), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("p", _fixtures("embedding_conv1d"))
def test_embedding_conv1d(p):
    net = _import(p)
    names = _names(p)
    E = _kw(p, names[0])
    E = E.get("embeddings", E.get("W"))
    conv = _kw(p, names[1])
    k = conv.get("kernel", conv.get("W"))
    if k.ndim == 4:
        k = k[:, 0]
    b = conv.get("bias", conv.get("b"))
    if _theano(p):
        k = k[::-1]
    idx = np.random.RandomState(6).randint(0, E.shape[0], size=(3, 10))
    x = E[idx]                                                   # [n, T, E]
    K = k.shape[0]
    ref = np.stack([np.einsum("nkc,kco->no", x[:, t:t + K], k) for t in range(10 - K + 1)], 1) + b
    got = _out(net, idx.astype(np.float32))                      # [n, O, T']
    np.testing.assert_allclose(got.transpose(0, 2, 1), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("p", _fixtures("bidirectional_lstm"))
def test_bidirectional_lstm(p):
    net = _import(p)
    kw = _kw(p, _names(p)[0])
    x = np.random.RandomState(7).randn(2, 4, 10)
    def sub(d):
        pre = d + "_lstm_1"
        return {k[len(pre) + 1:]: v for k, v in kw.items() if k.startswith(pre)}
    fwd = _lstm_keras(x, sub("forward"))
    bwd = _lstm_keras(x[:, ::-1], sub("backward"))[:, ::-1]
    ref = np.concatenate([fwd, bwd], -1)
    got = _out(net, x.transpose(0, 2, 1)).transpose(0, 2, 1)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


def _s2d_tf(x, b):
    n, H, W, C = x.shape
    return x.reshape(n, H // b, b, W // b, b, C).transpose(0, 1, 3, 2, 4, 5).reshape(n, H // b, W // b, b * b * C)


def test_space_to_depth_custom_lambda():
    KerasLayer.registerCustomLayer("Lambda", space_to_depth_mapper(2))
    try:
        for p in _fixtures("space_to_depth_simple"):
            net = _import(p)
            x = np.random.RandomState(8).randn(10, 6, 6, 4)
            got = _out(net, x.transpose(0, 3, 1, 2))
            assert got.shape == (10, 16, 3, 3)
            np.testing.assert_allclose(got.transpose(0, 2, 3, 1), _s2d_tf(x, 2), atol=1e-6)
        net = _import(R + "space_to_depth_graph_tensorflow_2.h5")
        x1 = np.random.RandomState(9).randn(10, 6, 6, 4)
        x2 = np.random.RandomState(10).randn(10, 3, 3, 16)
        out = net.output(torch.as_tensor(x1.transpose(0, 3, 1, 2), dtype=torch.float32),
                         torch.as_tensor(x2.transpose(0, 3, 1, 2), dtype=torch.float32))
        out = out[0] if isinstance(out, (list, tuple)) else out
        got = out.double().numpy().transpose(0, 2, 3, 1)
        assert got.shape == (10, 3, 3, 32)
        np.testing.assert_allclose(got, np.concatenate([_s2d_tf(x1, 2), x2], -1), atol=1e-6)
    finally:
        KerasLayer.clearCustomLayers()


def test_space_to_depth_gradient_roundtrip():
    from deeplearning4j_amd.nn.conf import layers as L
    from deeplearning4j_amd.nn.conf.inputs import InputType
    from deeplearning4j_amd.nn.conf.network import NeuralNetConfiguration
    from deeplearning4j_amd.nn.multilayer import MultiLayerNetwork
    conf = NeuralNetConfiguration.Builder().list().layer(0, L.SpaceToDepthLayer(blockSize=2)) \
        .setInputType(InputType.convolutional(4, 4, 3)).build()
    net = MultiLayerNetwork(conf)
    net.init(device=CPU)
    impl = net.layers[0]
    x = torch.randn(2, 3, 4, 4)
    y = impl.activate(x)
    _, back = impl.backpropGradient(y)
    assert torch.equal(back, x)


def test_training_config_adds_loss_layer():
    import json
    from deeplearning4j_amd.modelimport.keras import KerasModel
    cfg = {"class_name": "Sequential", "config": [
        {"class_name": "Dense", "config": {"name": "d1", "units": 5, "activation": "relu",
                                           "batch_input_shape": [None, 3]}},
        {"class_name": "Dense", "config": {"name": "d2", "units": 2, "activation": "softmax"}}]}
    km = KerasModel(cfg, None, json.dumps({"loss": "categorical_crossentropy"}))
    net = km.getMultiLayerNetwork(False, CPU)
    assert type(net.layers[-1].conf).__name__ == "LossLayer"
    x = torch.randn(4, 3)
    y = torch.eye(2)[torch.tensor([0, 1, 0, 1])]
    net.fit(x, y)
    assert np.isfinite(net.score())


def test_model_guesser_h5():
    from deeplearning4j_amd.utils.model_serializer import ModelGuesser, guess_model_type
    p = R + "dense_tensorflow_2.h5"
    assert guess_model_type(p) == "keras"
    net = ModelGuesser.loadModelGuess(p)
    assert net.numParams() == 30
