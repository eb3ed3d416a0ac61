"""Per-layer Keras import, after the reference's Keras layer tests
(deeplearning4j-modelimport/src/test/java/org/deeplearning4j/nn/modelimport/keras/layers/**: KerasDenseTest,
KerasConvolution1DTest / 2DTest, KerasAtrousConvolution1DTest / 2DTest, KerasDeconvolution2DTest,
KerasSeparableConvolution2DTest, KerasCropping2DTest, KerasZeroPadding1DTest / 2DTest, KerasUpsampling1DTest / 2DTest,
KerasPooling1DTest / 2DTest, KerasActivationLayer (LeakyReLU), KerasDropoutTest, KerasAlphaDropoutTest,
KerasGaussianDropoutTest, KerasGaussianNoiseTest, KerasBatchNormalizationTest, KerasEmbeddingTest, KerasLSTMTest,
KerasSimpleRnnTest, KerasBidirectionalTest): one Keras layer config map, in its Keras 1 and Keras 2 field spellings,
becomes a DL4J layer with the layer name, activation, weight init (glorot_normal -> XAVIER), L1 / L2 weight
regularisation, dropout (Keras fraction p -> retain probability 1 - p), kernel / stride / dilation / padding /
cropping / size fields, LSTM forget-gate bias, and MaskZero wrapping behind a mask_zero Embedding. CPU."""
import pytest
import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.modelimport.keras import KerasLayer
from deeplearning4j_amd.nn.conf import layers as L
from deeplearning4j_amd.nn.conf.regularization import AlphaDropout, Dropout, GaussianDropout, GaussianNoise

NAME, L1, L2, DROP, N_OUT = "test_layer", 0.01, 0.02, 0.3, 13
KERNEL, STRIDE, DILATION = [1, 2], [3, 4], [2, 2]

K1 = dict(init="init", wreg="W_regularizer", out="output_dim", filters="nb_filter", strides="subsample",
          border="border_mode", dilation="atrous_rate", dropout_w="dropout_W", inner_init="inner_init",
          inner_act="inner_activation", filter_len="filter_length", sub_len="subsample_length", pool1="pool_length",
          pool1_stride="stride", up1="length", rate="p", gauss="sigma", emb_init="init")
K2 = dict(init="kernel_initializer", wreg="kernel_regularizer", out="units", filters="filters", strides="strides",
          border="padding", dilation="dilation_rate", dropout_w="dropout", inner_init="recurrent_initializer",
          inner_act="recurrent_activation", filter_len="kernel_size", sub_len="strides", pool1="pool_size",
          pool1_stride="strides", up1="size", rate="rate", gauss="stddev", emb_init="embeddings_initializer")
VERSIONS = [(1, K1), (2, K2)]


def _init(v):
    return "glorot_normal" if v == 1 else {"class_name": "glorot_normal"}


def _layer(cls, cfg, v, prev=None):
    return KerasLayer.fromConfig({"class_name": cls, "config": dict(cfg, name=NAME), "keras_version": v},
                                 previousLayer=prev)


def _common(f, v, **extra):
    return dict({"activation": "linear", f["init"]: _init(v), f["wreg"]: {"l1": L1, "l2": L2}, "dropout": DROP},
                **extra)


def _check_common(layer):
    assert str(layer.getActivationFn()) == "identity"
    assert layer.getLayerName() == NAME
    assert layer.getWeightInit() == D.WeightInit.XAVIER
    assert layer.getL1() == L1 and layer.getL2() == L2
    assert layer.getIDropout() == Dropout(1 - DROP)


@pytest.mark.parametrize("v,f", VERSIONS)
def test_dense(v, f):
    layer = _layer("Dense", _common(f, v, **{f["out"]: N_OUT}), v)
    _check_common(layer)
    assert layer.getNOut() == N_OUT


@pytest.mark.parametrize("v,f", VERSIONS)
@pytest.mark.parametrize("dilation", [False, True])
def test_convolution_2d(v, f, dilation):
    if dilation and v == 1:
        pytest.skip("the reference tests dilation with Keras 2 fields only")
    cfg = _common(f, v, **{f["strides"]: STRIDE, f["filters"]: N_OUT, f["border"]: "valid"})
    if v == 1:
        cfg.update(nb_row=KERNEL[0], nb_col=KERNEL[1])
    else:
        cfg["kernel_size"] = KERNEL
    if dilation:
        cfg[f["dilation"]] = DILATION
    layer = _layer("Convolution2D" if v == 1 else "Conv2D", cfg, v)
    _check_common(layer)
    assert list(layer.getKernelSize()) == KERNEL and list(layer.getStride()) == STRIDE
    assert layer.getNOut() == N_OUT and layer.getConvolutionMode() == D.ConvolutionMode.Truncate
    assert list(layer.getPadding()) == [0, 0]
    if dilation:
        assert list(layer.getDilation()) == DILATION


@pytest.mark.parametrize("v,f", VERSIONS)
def test_atrous_convolution_2d(v, f):
    cfg = _common(f, v, **{f["strides"]: STRIDE, f["filters"]: N_OUT, f["border"]: "valid",
                           "atrous_rate": DILATION, "nb_row": KERNEL[0], "nb_col": KERNEL[1]})
    layer = _layer("AtrousConvolution2D", cfg, 1)
    _check_common(layer)
    assert list(layer.getDilation()) == DILATION and list(layer.getKernelSize()) == KERNEL


@pytest.mark.parametrize("v,f", VERSIONS)
@pytest.mark.parametrize("cls", ["conv", "atrous"])
def test_convolution_1d(v, f, cls):
    cfg = _common(f, v, **{f["filter_len"]: KERNEL[0] if v == 1 else [KERNEL[0]],
                           f["sub_len"]: STRIDE[0] if v == 1 else [STRIDE[0]], f["filters"]: N_OUT,
                           f["border"]: "valid"})
    if cls == "atrous":
        cfg[f["dilation"]] = DILATION[0] if v == 1 else [DILATION[0]]
    name = {"conv": ("Convolution1D", "Conv1D"), "atrous": ("AtrousConvolution1D", "Conv1D")}[cls][v - 1]
    layer = _layer(name, cfg, v)
    _check_common(layer)
    assert layer.getKernelSize()[0] == KERNEL[0] and layer.getStride()[0] == STRIDE[0]
    assert layer.getNOut() == N_OUT and layer.getConvolutionMode() == D.ConvolutionMode.Truncate
    assert layer.getPadding()[0] == 0
    if cls == "atrous":
        assert layer.getDilation()[0] == DILATION[0]


@pytest.mark.parametrize("v,f", VERSIONS)
def test_deconvolution_2d(v, f):
    cfg = _common(f, v, **{f["strides"]: STRIDE, f["filters"]: N_OUT, f["border"]: "valid", "kernel_size": KERNEL})
    layer = _layer("Deconvolution2D" if v == 1 else "Conv2DTranspose", cfg, v)
    assert isinstance(layer, L.Deconvolution2D)
    _check_common(layer)
    assert list(layer.getKernelSize()) == KERNEL and list(layer.getStride()) == STRIDE


@pytest.mark.parametrize("v,f", VERSIONS)
def test_separable_convolution_2d(v, f):
    cfg = {"activation": "linear", "depthwise_initializer": _init(v), "pointwise_initializer": _init(v),
           "depthwise_regularizer": {"l1": L1, "l2": L2}, "dropout": DROP, "depth_multiplier": 3,
           f["strides"]: STRIDE, f["filters"]: N_OUT, f["border"]: "valid", "kernel_size": KERNEL,
           f["dilation"]: DILATION}
    layer = _layer("SeparableConvolution2D" if v == 1 else "SeparableConv2D", cfg, v)
    assert isinstance(layer, L.SeparableConvolution2D)
    _check_common(layer)
    assert layer.getDepthMultiplier() == 3 and list(layer.getDilation()) == DILATION


@pytest.mark.parametrize("v", [1, 2])
def test_cropping_and_zero_padding_2d(v):
    c = _layer("Cropping2D", {"cropping": [2, 3]}, v)
    assert c.getLayerName() == NAME and list(c.getCropping()) == [2, 2, 3, 3]
    c = _layer("Cropping2D", {"cropping": 2}, v)
    assert list(c.getCropping())[:2] == [2, 2]
    z = _layer("ZeroPadding2D", {"padding": [2, 3]}, v)
    assert z.getLayerName() == NAME and list(z.getPadding()) == [2, 2, 3, 3]
    z = _layer("ZeroPadding2D", {"padding": 2}, v)
    assert list(z.getPadding())[:2] == [2, 2]


@pytest.mark.parametrize("v", [1, 2])
def test_zero_padding_1d_and_upsampling(v):
    z = _layer("ZeroPadding1D", {"padding": 2}, v)
    assert z.getLayerName() == NAME and z.getPadding()[0] == 2
    f = K1 if v == 1 else K2
    u1 = _layer("UpSampling1D", {f["up1"]: 4}, v)
    assert u1.getLayerName() == NAME and list(u1.getSize()) == [4]
    u2 = _layer("UpSampling2D", {"size": [2, 2]}, v)
    assert u2.getLayerName() == NAME and list(u2.getSize()) == [2, 2]


@pytest.mark.parametrize("v,f", VERSIONS)
def test_pooling(v, f):
    p2 = _layer("MaxPooling2D", {"pool_size": KERNEL, "strides": STRIDE, f["border"]: "valid"}, v)
    assert p2.getLayerName() == NAME and list(p2.getKernelSize()) == KERNEL and list(p2.getStride()) == STRIDE
    assert p2.getPoolingType() == D.PoolingType.MAX and p2.getConvolutionMode() == D.ConvolutionMode.Truncate
    assert list(p2.getPadding()) == [0, 0]
    p1 = _layer("MaxPooling1D", {f["pool1"]: KERNEL[0] if v == 1 else [KERNEL[0]],
                                 f["pool1_stride"]: STRIDE[0] if v == 1 else [STRIDE[0]], f["border"]: "valid"}, v)
    assert p1.getKernelSize()[0] == KERNEL[0] and p1.getStride()[0] == STRIDE[0]
    assert p1.getPoolingType() == D.PoolingType.MAX and p1.getPadding()[0] == 0


def test_leaky_relu_activation_layer():
    layer = _layer("LeakyReLU", {"alpha": 0.3}, 2)
    assert str(layer.getActivationFn()) == "leakyrelu(a=0.3)" and layer.getLayerName() == NAME


@pytest.mark.parametrize("v,f", VERSIONS)
def test_dropout_family(v, f):
    assert _layer("Dropout", {f["rate"]: DROP}, v).getIDropout() == Dropout(1 - DROP)
    assert _layer("AlphaDropout", {f["rate"]: DROP}, v).getIDropout() == AlphaDropout(1 - DROP)
    assert _layer("GaussianDropout", {f["rate"]: DROP}, v).getIDropout() == GaussianDropout(DROP)
    layer = _layer("GaussianNoise", {f["gauss"]: 0.4}, v)
    assert layer.getIDropout() == GaussianNoise(0.4) and layer.getLayerName() == NAME


@pytest.mark.parametrize("v", [1, 2])
def test_batch_normalization(v):
    layer = _layer("BatchNormalization", {"epsilon": 1e-5, "momentum": 0.99, "gamma_regularizer": None,
                                          "beta_regularizer": None, "mode": 0, "axis": 3}, v)
    assert layer.getLayerName() == NAME and layer.getEps() == 1e-5


def _lstm_cfg(f, v, rs, cls="LSTM"):
    cfg = {"activation": "linear", f["inner_act"]: "hard_sigmoid", f["inner_init"]: _init(v), f["init"]: _init(v),
           f["wreg"]: {"l1": L1, "l2": L2}, "return_sequences": rs, f["dropout_w"]: DROP,
           ("dropout_U" if v == 1 else "recurrent_dropout"): 0.0, f["out"]: N_OUT, "unroll": True}
    if cls == "LSTM":
        cfg["forget_bias_init"] = "one"
    return cfg


@pytest.mark.parametrize("v,f", VERSIONS)
@pytest.mark.parametrize("rs", [True, False])
def test_lstm(v, f, rs):
    layer = _layer("LSTM", _lstm_cfg(f, v, rs), v)
    if not rs:
        assert isinstance(layer, L.LastTimeStep)
        assert layer.getOutputType(0, D.InputType.recurrent(1337)) == D.InputType.feedForward(N_OUT)
        layer = layer.underlying
    else:
        assert layer.getOutputType(0, D.InputType.recurrent(1337)) == D.InputType.recurrent(N_OUT)
    assert isinstance(layer, L.LSTM)
    _check_common(layer)
    assert layer.getForgetGateBiasInit() == 1.0 and layer.getNOut() == N_OUT
    assert str(layer.getGateActivationFn()) == "hardsigmoid"


@pytest.mark.parametrize("v,f", VERSIONS)
@pytest.mark.parametrize("mask_zero", [False, True])
def test_lstm_behind_mask_zero_embedding(v, f, mask_zero):
    emb = {"class_name": "Embedding", "config": {"name": "emb", "input_dim": 10, "output_dim": 10,
                                                 "mask_zero": mask_zero}, "keras_version": v}
    layer = _layer("LSTM", _lstm_cfg(f, v, True), v, prev=emb)
    assert isinstance(layer, L.MaskZeroLayer) == mask_zero


@pytest.mark.parametrize("v,f", VERSIONS)
def test_simple_rnn(v, f):
    layer = _layer("SimpleRNN", _lstm_cfg(f, v, True, "SimpleRNN"), v)
    assert isinstance(layer, L.SimpleRnn)
    _check_common(layer)
    assert layer.getNOut() == N_OUT


@pytest.mark.parametrize("v,f", VERSIONS)
def test_bidirectional(v, f):
    cfg = {"merge_mode": "sum", "layer": {"class_name": "LSTM", "config": dict(_lstm_cfg(f, v, True), name=NAME)}}
    layer = _layer("Bidirectional", cfg, v)
    assert isinstance(layer, L.Bidirectional)
    assert str(layer.getMode()).upper().endswith("ADD")
    inner = layer.underlying
    _check_common(inner)
    assert inner.getForgetGateBiasInit() == 1.0


@pytest.mark.parametrize("v,f", VERSIONS)
@pytest.mark.parametrize("mask_zero", [False, True])
def test_embedding(v, f, mask_zero):
    cfg = {"input_dim": 10, "output_dim": 10, "batch_input_shape": [100, 20], f["emb_init"]: _init(v),
           "mask_zero": mask_zero}
    layer = _layer("Embedding", cfg, v)
    assert layer.getLayerName() == NAME and layer.getWeightInit() == D.WeightInit.XAVIER
    assert layer.numParams() == 10 * 10


def test_embedding_set_weights_mask_zero():
    """Importing weights through a mask_zero Embedding zeroes the padding token's row."""
    import json
    model = {"class_name": "Sequential", "config": [
        {"class_name": "Embedding", "config": {"name": "emb", "input_dim": 100, "output_dim": 20, "mask_zero": True,
                                               "batch_input_shape": [None, 5], "input_length": 5}},
        {"class_name": "LSTM", "config": {"name": "lstm", "units": 4, "return_sequences": False,
                                          "activation": "tanh", "recurrent_activation": "hard_sigmoid"}}]}
    from deeplearning4j_amd.modelimport.keras import KerasModel
    km = KerasModel(json.dumps(model), keras_version="2.1")
    conf, setters = km._sequential()
    net = D.MultiLayerNetwork(conf)
    net.init()
    assert isinstance(net.getLayer(1).conf.underlying, L.MaskZeroLayer)
    m = dict(setters)[0]
    m.setter(net.getLayer(0).params, {"embeddings": torch.ones(100, 20).numpy()})
    w = net.getLayer(0).params["W"]
    assert int((w[0] == 0).sum()) == 20 and float(w[1:].min()) == 1.0
