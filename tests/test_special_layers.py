"""Specialised layers: SameDiff-lite layers, self-attention, AutoEncoder / VAE (supervised + pretraining),
YOLOv2 output layer. Gradient checks in double precision as the reference does
(CORET: gradientcheck/{VaeGradientCheckTests,YoloGradientCheckTests}.java, nn/layers/samediff/TestSameDiffDense.java,
nn/layers/variational/TestVAE.java, nn/layers/objdetect/TestYolo2OutputLayer.java)."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.gradientcheck import checkGradients
from deeplearning4j_amd.nn.conf import SameDiffLayerConf
from deeplearning4j_amd.nn.layers.objdetect import YoloUtils

DEV = torch.device("cpu")


def _onehot(n, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    y = torch.zeros(n, k, dtype=torch.float64)
    y[torch.arange(n), torch.randint(0, k, (n,), generator=g)] = 1
    return y


def _mln(layers, updater=None, inputType=None, dtype=DataType.DOUBLE, **kw):
    b = (NeuralNetConfiguration.Builder().seed(123).dataType(dtype).updater(updater or NoOp())
         .weightInit(NormalDistribution(0, 1)).list())
    for i, l in enumerate(layers):
        b.layer(i, l)
    if inputType is not None:
        b.setInputType(inputType)
    for k, v in kw.items():
        getattr(b, k)(v)
    net = MultiLayerNetwork(b.build())
    net.init(device=DEV)
    return net


class SameDiffDense(SameDiffLayerConf):
    """The reference's test layer (CORET: nn/layers/samediff/testlayers/SameDiffDense.java), written against
    the SameDiff-lite API."""

    def defineParameters(self, params):
        params.clear()
        params.addWeightParam("W", [self.nIn, self.nOut])
        params.addBiasParam("b", [1, self.nOut])

    def defineLayer(self, sd, layerInput, paramTable):
        z = sd.mmul("mmul", layerInput, paramTable["W"]).add("z", paramTable["b"])
        return [Activation.TANH.asSameDiff("out", sd, z)]


def test_samediff_dense_gradients_and_equivalence():
    net = _mln([SameDiffDense(nIn=4, nOut=5),
                OutputLayer.Builder(LossFunction.MCXENT).nIn(5).nOut(3).activation(Activation.SOFTMAX).build()])
    x = torch.randn(6, 4, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=_onehot(6, 3), print_results=True)
    # same params as a DenseLayer network -> identical output
    ref = _mln([DenseLayer.Builder().nIn(4).nOut(5).activation(Activation.TANH).build(),
                OutputLayer.Builder(LossFunction.MCXENT).nIn(5).nOut(3).activation(Activation.SOFTMAX).build()])
    ref.layers[0].params["W"].copy_(net.layers[0].params["W"])
    ref.layers[0].params["b"].copy_(net.layers[0].params["b"])
    ref.layers[1].params["W"].copy_(net.layers[1].params["W"])
    ref.layers[1].params["b"].copy_(net.layers[1].params["b"])
    assert torch.allclose(ref.output(x), net.output(x))


def test_self_attention_gradients():
    net = _mln([SelfAttentionLayer.Builder().nIn(6).nOut(6).nHeads(2).activation(Activation.IDENTITY).build(),
                RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(6).nOut(3).activation(Activation.SOFTMAX).build()])
    x = torch.randn(2, 6, 5, dtype=torch.float64)
    y = torch.zeros(2, 3, 5, dtype=torch.float64)
    y[:, 0, :] = 1
    # the key bias has an exactly-zero gradient (softmax shift invariance): allow numerical noise there
    assert checkGradients(net, input=x, labels=y, print_results=True, minAbsoluteError=1e-7)


@pytest.mark.parametrize("causal,masked", [(True, False), (False, True), (True, True)])
def test_self_attention_gradients_causal_and_masked(causal, masked):
    """The hand-derived backward (nn/layers/attention.py, ops/transformer_native.attention_bwd_explicit) against
    fp64 numerical gradients, with a causal mask and / or padded keys (masked query rows produce zeros)."""
    net = _mln([SelfAttentionLayer.Builder().nIn(6).nOut(6).nHeads(3).causal(causal)
                .activation(Activation.TANH).build(),
                RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(6).nOut(3).activation(Activation.SOFTMAX).build()])
    x = torch.randn(3, 6, 5, dtype=torch.float64)
    y = torch.zeros(3, 3, 5, dtype=torch.float64)
    y[:, 1, :] = 1
    mask = None
    if masked:
        mask = torch.ones(3, 5, dtype=torch.float64)
        mask[1, 3:] = 0
        mask[2, 1:] = 0
    assert checkGradients(net, input=x, labels=y, inputMask=mask, labelMask=mask, print_results=True,
                          minAbsoluteError=1e-7)


def test_autoencoder_supervised_gradients_and_pretrain():
    ae = AutoEncoder.Builder().nIn(6).nOut(4).activation(Activation.SIGMOID).corruptionLevel(0.0).build()
    net = _mln([ae, OutputLayer.Builder(LossFunction.MSE).nIn(4).nOut(2).activation(Activation.IDENTITY).build()])
    x = torch.rand(5, 6, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=torch.randn(5, 2, dtype=torch.float64), print_results=True)
    # layer-wise pretraining reduces the reconstruction error and only touches layer 0
    net2 = _mln([AutoEncoder.Builder().nIn(6).nOut(4).activation(Activation.SIGMOID).corruptionLevel(0.1)
                 .weightInit(WeightInit.XAVIER).lossFunction(LossFunction.MSE).build(),
                 OutputLayer.Builder(LossFunction.MSE).nIn(4).nOut(2).activation(Activation.IDENTITY).build()],
                updater=Adam(1.0), dtype=DataType.FLOAT)     # DL4J divides the Adam update by the minibatch
    g = torch.Generator().manual_seed(1)
    data = torch.sigmoid(3 * torch.randn(64, 2, generator=g) @ torch.randn(2, 6, generator=g))   # low rank
    w_out = net2.layers[1].params["W"].clone()
    l0 = net2.layers[0]
    err0 = ((l0.reconstruct(data) - data) ** 2).mean().item()
    net2.pretrainLayer(0, DataSet(data, torch.zeros(64, 2)), numEpochs=200)
    err1 = ((l0.reconstruct(data) - data) ** 2).mean().item()
    assert err1 < err0 * 0.8, (err0, err1)
    assert torch.equal(net2.layers[1].params["W"], w_out)


def test_vae_supervised_gradients_and_pretraining():
    vae = (VariationalAutoencoder.Builder().nIn(5).nOut(3).encoderLayerSizes([4]).decoderLayerSizes([4])
           .activation(Activation.TANH).pzxActivationFn(Activation.IDENTITY)
           .outputDistribution(GaussianReconstructionDistribution(Activation.IDENTITY)).build())
    net = _mln([vae, OutputLayer.Builder(LossFunction.MSE).nIn(3).nOut(2).activation(Activation.IDENTITY).build()])
    x = torch.randn(4, 5, dtype=torch.float64)
    assert checkGradients(net, input=x, labels=torch.randn(4, 2, dtype=torch.float64), print_results=True)
    # pretraining lowers the negative ELBO; generative API works
    for dist in (BernoulliReconstructionDistribution(Activation.SIGMOID),
                 GaussianReconstructionDistribution(Activation.TANH)):
        v = (VariationalAutoencoder.Builder().nIn(8).nOut(2).encoderLayerSizes([16]).decoderLayerSizes([16])
             .activation(Activation.TANH).outputDistribution(dist).build())
        n2 = _mln([v, OutputLayer.Builder(LossFunction.MSE).nIn(2).nOut(1).activation(Activation.IDENTITY).build()],
                  updater=Adam(1.0), dtype=DataType.FLOAT)
        g = torch.Generator().manual_seed(0)
        data = (torch.rand(128, 8, generator=g) > 0.5).float()
        lp0 = n2.layers[0].reconstructionLogProbability(data, 4).mean().item()
        n2.pretrainLayer(0, DataSet(data, torch.zeros(128, 1)), numEpochs=150)
        lp1 = n2.layers[0].reconstructionLogProbability(data, 4).mean().item()
        assert lp1 > lp0, (type(dist).__name__, lp0, lp1)
        z = torch.randn(3, 2)
        assert n2.layers[0].generateAtMeanGivenZ(z).shape == (3, 8)
        assert n2.layers[0].generateRandomGivenZ(z).shape == (3, 8)


def _yolo_labels(mb, C, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    lab = torch.zeros(mb, 4 + C, H, W, dtype=torch.float64)
    for e in range(mb):
        for _ in range(2):
            cx, cy = torch.rand(2, generator=g) * torch.tensor([W - 1.0, H - 1.0]) + 0.5
            w_, h_ = torch.rand(2, generator=g) * 1.5 + 0.3
            gx, gy = int(cx), int(cy)
            lab[e, 0:4, gy, gx] = torch.tensor([cx - w_ / 2, cy - h_ / 2, cx + w_ / 2, cy + h_ / 2])
            lab[e, 4 + int(torch.randint(0, C, (1,), generator=g)), gy, gx] = 1
    return lab


def test_yolo2_gradients_and_detection():
    B, C, H, W = 2, 3, 4, 4
    priors = [[1.0, 1.5], [2.0, 1.0]]
    net = _mln([ConvolutionLayer.Builder([1, 1]).nIn(2).nOut(B * (5 + C)).activation(Activation.IDENTITY).build(),
                Yolo2OutputLayer(boundingBoxes=priors)],
               inputType=InputType.convolutional(H, W, 2))
    x = torch.randn(2, 2, H, W, dtype=torch.float64) * 0.5
    assert checkGradients(net, input=x, labels=_yolo_labels(2, C, H, W), print_results=True)
    out = net.output(x)
    assert out.shape == (2, B * (5 + C), H, W)
    objs = YoloUtils.getPredictedObjects(priors, out, 0.0, 0.5)
    assert objs and all(0 <= o.getPredictedClass() < C for o in objs)


@pytest.mark.parametrize("pt", ["AVG", "SUM"])
def test_global_pooling_channels_last_fast_path(pt):
    """The channels-last AVG/SUM fast path equals the generic strided reduction (values and gradients)."""
    from deeplearning4j_amd.nn.conf import layers as L
    from deeplearning4j_amd.nn.layers.pooling import GlobalPoolingLayerImpl
    conf = L.GlobalPoolingLayer(poolingType=pt)
    impl = GlobalPoolingLayerImpl(conf)
    x = torch.randn(3, 5, 4, 6)
    xc = x.contiguous(memory_format=torch.channels_last)
    out_fast = impl.activate(xc)
    assert impl._fast is not None
    eps = torch.randn_like(out_fast)
    _, g_fast = impl.backpropGradient(eps)
    out_ref = impl.activate(x)
    assert impl._fast is None
    _, g_ref = impl.backpropGradient(eps)
    torch.testing.assert_close(out_fast, out_ref)
    torch.testing.assert_close(g_fast, g_ref)


def test_zero_padding_folded_into_conv(monkeypatch):
    """The graph planner folds ZeroPadding -> Conv(Truncate) into the conv's padding: same outputs, same gradients
    as materialising the padded tensor (asymmetric padding included)."""
    from deeplearning4j_amd.nn.conf import (ConvolutionLayer, ConvolutionMode, InputType, NeuralNetConfiguration,
                                            OutputLayer, ZeroPaddingLayer, LossFunction, Activation, Sgd)
    from deeplearning4j_amd.nn.graph import ComputationGraph

    def build():
        g = NeuralNetConfiguration.Builder().seed(3).updater(Sgd(0.1)).convolutionMode(ConvolutionMode.Truncate) \
            .graphBuilder().addInputs("in").setInputTypes(InputType.convolutional(9, 8, 2))
        g.addLayer("zp", ZeroPaddingLayer.Builder(1, 2, 0, 3).build(), "in")
        g.addLayer("c", ConvolutionLayer.Builder([3, 3], [2, 2]).nOut(4).build(), "zp")
        g.addLayer("out", OutputLayer.Builder(LossFunction.MSE).nOut(2).activation(Activation.IDENTITY).build(), "c")
        net = ComputationGraph(g.setOutputs("out").build())
        net.init(device=torch.device("cpu"))
        return net
    x = torch.randn(3, 2, 9, 8)
    y = torch.randn(3, 2)
    monkeypatch.setenv("DL4J_AMD_FOLD_PAD", "1")
    a = build()
    assert a.layers_by_name["c"].extra_pad4 == (1, 2, 0, 3)
    monkeypatch.setenv("DL4J_AMD_FOLD_PAD", "0")
    b = build()
    assert b.layers_by_name["c"].extra_pad4 is None
    torch.testing.assert_close(a.output(x)[0] if isinstance(a.output(x), list) else a.output(x),
                               b.output(x)[0] if isinstance(b.output(x), list) else b.output(x))
    a.fit([x], [y])
    b.fit([x], [y])
    torch.testing.assert_close(a.params(), b.params())


def test_conv_bias_deferred_into_batchnorm(monkeypatch):
    """Conv(+bias) -> BN: skipping the bias add in training (BN adds (1-decay)*b to its running mean) gives the
    same training outputs, parameters, running statistics and inference outputs as the plain computation."""
    from deeplearning4j_amd.nn.conf import (BatchNormalization, ConvolutionLayer, InputType, NeuralNetConfiguration,
                                            OutputLayer, LossFunction, Activation, Sgd)
    from deeplearning4j_amd.nn.graph import ComputationGraph

    def build():
        g = NeuralNetConfiguration.Builder().seed(5).updater(Sgd(0.05)).activation(Activation.IDENTITY) \
            .graphBuilder().addInputs("in") \
            .setInputTypes(InputType.convolutional(6, 6, 3))
        g.addLayer("c", ConvolutionLayer.Builder([3, 3]).nOut(4).biasInit(0.3).build(), "in")
        g.addLayer("bn", BatchNormalization.Builder().decay(0.8).build(), "c")
        g.addLayer("out", OutputLayer.Builder(LossFunction.MSE).nOut(2).activation(Activation.IDENTITY).build(), "bn")
        net = ComputationGraph(g.setOutputs("out").build())
        net.init(device=torch.device("cpu"))
        return net
    x = torch.randn(5, 3, 6, 6)
    y = torch.randn(5, 2)
    monkeypatch.setenv("DL4J_AMD_DEFER_BIAS", "1")
    a = build()
    assert a.layers_by_name["c"].defer_bias      # nIn = 3: the library-conv case
    monkeypatch.setenv("DL4J_AMD_DEFER_BIAS", "0")
    b = build()
    assert not b.layers_by_name["c"].defer_bias
    for _ in range(3):
        a.fit([x], [y])
        b.fit([x], [y])
    torch.testing.assert_close(a.params(), b.params(), rtol=1e-5, atol=1e-6)
    oa, ob = a.output(x), b.output(x)
    oa = oa[0] if isinstance(oa, list) else oa
    ob = ob[0] if isinstance(ob, list) else ob
    torch.testing.assert_close(oa, ob, rtol=1e-5, atol=1e-6)


def test_samediff_native_ops_cpu_reference():
    """SameDiff lstmLayer / layerNorm / fusedSelfAttention (CPU reference path) agree with the layer runtimes."""
    from deeplearning4j_amd.nn.conf.activations import ActivationSigmoid, ActivationTanH
    from deeplearning4j_amd.nn.layers import recurrent as R
    from deeplearning4j_amd.samediff import SameDiff
    g = torch.Generator().manual_seed(0)
    mb, nIn, T, H = 3, 5, 7, 8
    x = torch.randn(mb, nIn, T, generator=g, dtype=torch.float64)
    W = torch.randn(nIn, 4 * H, generator=g, dtype=torch.float64) * 0.4
    RW = torch.randn(H, 4 * H + 3, generator=g, dtype=torch.float64) * 0.4
    b = torch.randn(4 * H, generator=g, dtype=torch.float64) * 0.1
    sd = SameDiff.create()
    out = sd.rnn().lstmLayer("h", sd.var("x", x), sd.var("W", W), sd.var("RW", RW), sd.var("b", b), peephole=True)
    ref, _, _ = R._lstm_fwd(x, W, RW, b, None, None, H, True, ActivationTanH(), ActivationSigmoid(), None, False)
    assert torch.allclose(out.value, ref, atol=1e-10)
    e = torch.randn(4, 6, 16, generator=g, dtype=torch.float64)
    ln = sd.nn().layerNorm("ln", sd.var("e", e), sd.var("g", torch.ones(16, dtype=torch.float64)),
                           sd.var("bb", torch.zeros(16, dtype=torch.float64)), 1e-5)
    assert torch.allclose(ln.value, torch.nn.functional.layer_norm(e, (16,), eps=1e-5))
    qkv = torch.randn(2, 5, 3 * 8, generator=g, dtype=torch.float64)
    att = sd.nn().fusedSelfAttention("att", sd.var("qkv", qkv), 2)
    assert att.value.shape == (2, 5, 8)
