"""Hand-derived backward passes of the VAE, AutoEncoder and YOLOv2 output layers, checked in fp64.

Each gradient is compared two ways: against central finite differences of the layer's own score (the reference's
gradient-check method, CORET gradientcheck/{VaeGradientCheckTests,YoloGradientCheckTests}.java), and against
torch.autograd applied to an independent copy of the forward expression kept in this file. Stochastic paths
(VAE reparameterisation noise, AutoEncoder input corruption) are made repeatable by reseeding torch's RNG before
every evaluation."""
import itertools

import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.nn.conf.losses import LossMSE
from deeplearning4j_amd.nn.conf.variational import (BernoulliReconstructionDistribution,
                                                    CompositeReconstructionDistribution,
                                                    ExponentialReconstructionDistribution,
                                                    GaussianReconstructionDistribution, LossFunctionWrapper)

D = torch.float64


def _mln(layers, inputType=None):
    b = (NeuralNetConfiguration.Builder().seed(7).dataType(DataType.DOUBLE).updater(NoOp())
         .weightInit(NormalDistribution(0, 0.5)).list())
    for i, l in enumerate(layers):
        b.layer(i, l)
    if inputType is not None:
        b.setInputType(inputType)
    net = MultiLayerNetwork(b.build())
    net.init(device=torch.device("cpu"))
    return net


def _fd_check(layer, score_fn, keys, h=1e-6, rtol=1e-5, atol=1e-8):
    """Central differences of ``score_fn`` (a scalar of the current layer params) vs layer.grads."""
    analytic = {k: layer.grads[k].clone() for k in keys}
    for k in keys:
        p = layer.params[k]                        # parameter views may be 'f'-ordered: index, don't flatten
        ga = analytic[k].reshape(p.shape)
        for idx in itertools.product(*[range(n) for n in p.shape]):
            old = p[idx].item()
            p[idx] = old + h
            sp = score_fn()
            p[idx] = old - h
            sm = score_fn()
            p[idx] = old
            num = (sp - sm) / (2 * h)
            a = ga[idx].item()
            assert abs(num - a) <= atol + rtol * max(abs(num), abs(a)), (k, idx, num, a)


# ------------------------------------------------------------------------------- reconstruction distributions
@pytest.mark.parametrize("dist,kind", [
    (GaussianReconstructionDistribution(Activation.IDENTITY), "real"),
    (GaussianReconstructionDistribution(Activation.TANH), "real"),
    (BernoulliReconstructionDistribution(Activation.SIGMOID), "binary"),
    (ExponentialReconstructionDistribution(Activation.TANH), "positive"),
    (LossFunctionWrapper(Activation.SIGMOID, LossMSE()), "binary"),
    (CompositeReconstructionDistribution.Builder()
     .addDistribution(2, GaussianReconstructionDistribution(Activation.IDENTITY))
     .addDistribution(3, BernoulliReconstructionDistribution(Activation.SIGMOID)).build(), "mixed"),
])
def test_distribution_gradient_matches_autograd(dist, kind):
    g = torch.Generator().manual_seed(3)
    n = 5
    x = {"real": torch.randn(6, n, generator=g, dtype=D),
         "binary": (torch.rand(6, n, generator=g) > 0.5).to(D),
         "positive": torch.rand(6, n, generator=g, dtype=D) * 2,
         "mixed": torch.cat([torch.randn(6, 2, generator=g, dtype=D),
                             (torch.rand(6, 3, generator=g) > 0.5).to(D)], 1)}[kind]
    pre = torch.randn(6, dist.distributionInputSize(n), generator=g, dtype=D).requires_grad_(True)
    (ref,) = torch.autograd.grad(dist.exampleNegLogProbability(x, pre).sum(), [pre])
    got = dist.gradient(x, pre.detach())
    torch.testing.assert_close(got, ref, rtol=1e-10, atol=1e-12)


# ------------------------------------------------------------------------------- VAE
def _vae_net(dist, enc=(4, 3), dec=(3,), pzx=Activation.IDENTITY, ns=1):
    vae = (VariationalAutoencoder.Builder().nIn(5).nOut(2).encoderLayerSizes(list(enc))
           .decoderLayerSizes(list(dec)).activation(Activation.TANH).pzxActivationFn(pzx)
           .outputDistribution(dist).numSamples(ns).build())
    return _mln([vae, OutputLayer.Builder(LossFunction.MSE).nIn(2).nOut(2).activation(Activation.IDENTITY).build()])


def _vae_autograd_reference(layer, x, seed):
    """Independent autograd version of the negative ELBO (the pre-round-3 implementation)."""
    c = layer.conf
    keys = list(layer.params)
    p = {k: layer.params[k].detach().clone().requires_grad_(True) for k in keys}
    act, pzx = c.activation, layer._pzx_act()
    mb = x.shape[0]
    torch.manual_seed(seed)
    with torch.enable_grad():
        h = x
        for i in range(len(c.encoderLayerSizes)):
            h = act.getActivation(h @ p[f"e{i}W"] + p[f"e{i}b"], True)
        mean = pzx.getActivation(h @ p["pZXMeanW"] + p["pZXMeanb"], True)
        logs2 = pzx.getActivation(h @ p["pZXLogStd2W"] + p["pZXLogStd2b"], True)
        loss = -0.5 / mb * (1.0 + logs2 - mean * mean - logs2.exp()).sum()
        ns = max(1, int(c.numSamples or 1))
        for _ in range(ns):
            z = mean + (0.5 * logs2).exp() * torch.randn_like(mean)
            d = z
            for i in range(len(c.decoderLayerSizes)):
                d = act.getActivation(d @ p[f"d{i}W"] + p[f"d{i}b"], True)
            loss = loss + layer._dist().negLogProbability(x, d @ p["pXZW"] + p["pXZb"], True) / ns
        grads = torch.autograd.grad(loss * mb, [p[k] for k in keys])
    return float(loss.detach()), dict(zip(keys, grads))


@pytest.mark.parametrize("case", ["gauss", "bern_2samples", "composite_tanh_pzx", "lossfn_nodecoder"])
def test_vae_pretrain_gradient(case):
    dist, kw = {
        "gauss": (GaussianReconstructionDistribution(Activation.TANH), {}),
        "bern_2samples": (BernoulliReconstructionDistribution(Activation.SIGMOID), {"ns": 2}),
        "composite_tanh_pzx": (CompositeReconstructionDistribution.Builder()
                               .addDistribution(2, GaussianReconstructionDistribution(Activation.IDENTITY))
                               .addDistribution(3, ExponentialReconstructionDistribution(Activation.TANH)).build(),
                               {"pzx": Activation.TANH, "enc": (4,)}),
        "lossfn_nodecoder": (LossFunctionWrapper(Activation.SIGMOID, LossMSE()), {"dec": ()}),
    }[case]
    net = _vae_net(dist, **kw)
    layer = net.layers[0]
    g = torch.Generator().manual_seed(11)
    x = torch.rand(4, 5, generator=g, dtype=D)
    if case == "gauss":
        x = torch.randn(4, 5, generator=g, dtype=D)
    seed = 1234
    mb = x.shape[0]

    def score():
        torch.manual_seed(seed)
        return layer.computePretrainGradientAndScore(x) * mb

    s = score()
    ref_s, ref_g = _vae_autograd_reference(layer, x, seed)
    assert abs(s / mb - ref_s) < 1e-12
    for k, v in ref_g.items():
        torch.testing.assert_close(layer.grads[k].reshape(v.shape), v, rtol=1e-9, atol=1e-12)
    score()                                         # re-establish layer.grads at the unperturbed point
    _fd_check(layer, score, list(layer.params))


def test_vae_supervised_backward_two_encoder_layers():
    net = _vae_net(GaussianReconstructionDistribution(Activation.IDENTITY), enc=(6, 4), pzx=Activation.TANH)
    x = torch.randn(5, 5, dtype=D)
    y = torch.randn(5, 2, dtype=D)
    from deeplearning4j_amd.gradientcheck import checkGradients
    assert checkGradients(net, input=x, labels=y)
    # decoder / log-variance parameters are pretrain-only: zero supervised gradient
    net.computeGradientAndScore(x, y)
    layer = net.layers[0]
    for k in layer.grads:
        if k.startswith("d") or k.startswith("pXZ") or k.startswith("pZXLogStd2"):
            assert torch.count_nonzero(layer.grads[k]) == 0, k


# ------------------------------------------------------------------------------- AutoEncoder
@pytest.mark.parametrize("act,corrupt,sparsity,loss", [
    (Activation.SIGMOID, 0.0, 0.0, LossFunction.MSE),
    (Activation.SIGMOID, 0.3, 0.1, LossFunction.XENT),
    (Activation.TANH, 0.2, 0.0, LossFunction.L2),
])
def test_autoencoder_pretrain_gradient(act, corrupt, sparsity, loss):
    ae = (AutoEncoder.Builder().nIn(6).nOut(4).activation(act).corruptionLevel(corrupt).sparsity(sparsity)
          .lossFunction(loss).build())
    net = _mln([ae, OutputLayer.Builder(LossFunction.MSE).nIn(4).nOut(2).activation(Activation.IDENTITY).build()])
    layer = net.layers[0]
    x = torch.rand(5, 6, generator=torch.Generator().manual_seed(2), dtype=D)
    mb = x.shape[0]

    def score():
        torch.manual_seed(99)
        return layer.computePretrainGradientAndScore(x) * mb

    score()
    # autograd reference of the same objective
    p = {k: layer.params[k].detach().clone().requires_grad_(True) for k in ("W", "b", "vb")}
    torch.manual_seed(99)
    xin = x * (torch.rand_like(x) >= corrupt).to(D) if corrupt > 0 else x
    a = layer.conf.activation
    with torch.enable_grad():
        yy = a.getActivation(xin @ p["W"] + p["b"], True)
        L = layer._loss().computeScore(x, yy @ p["W"].t() + p["vb"], a, None, False)
        if sparsity > 0:
            rh = yy.mean(0).clamp(1e-6, 1 - 1e-6)
            L = L + mb * (sparsity * torch.log(sparsity / rh) + (1 - sparsity) * torch.log((1 - sparsity) / (1 - rh))).sum()
        ref = torch.autograd.grad(L, [p["W"], p["b"], p["vb"]])
    for k, r in zip(("W", "b", "vb"), ref):
        torch.testing.assert_close(layer.grads[k].reshape(r.shape), r, rtol=1e-9, atol=1e-12)
    _fd_check(layer, score, ["W", "b", "vb"])


# ------------------------------------------------------------------------------- YOLOv2
def _yolo_case(seed, B=2, C=3, H=4, W=4, mb=2):
    g = torch.Generator().manual_seed(seed)
    lab = torch.zeros(mb, 4 + C, H, W, dtype=D)
    for e in range(mb):
        for _ in range(3):
            cx, cy = torch.rand(2, generator=g, dtype=D) * torch.tensor([W - 1.0, H - 1.0], dtype=D) + 0.5
            w_, h_ = torch.rand(2, generator=g, dtype=D) * 1.5 + 0.4
            gx, gy = int(cx), int(cy)
            lab[e, :, gy, gx] = 0
            lab[e, 0:4, gy, gx] = torch.stack([cx - w_ / 2, cy - h_ / 2, cx + w_ / 2, cy + h_ / 2])
            lab[e, 4 + int(torch.randint(0, C, (1,), generator=g)), gy, gx] = 1
    x = torch.randn(mb, B * (5 + C), H, W, generator=g, dtype=D) * 0.6
    return x, lab


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_yolo2_explicit_gradient_matches_autograd_and_fd(seed):
    from deeplearning4j_amd.nn.conf.layers import Yolo2OutputLayer as Conf
    from deeplearning4j_amd.nn.layers.objdetect import Yolo2OutputLayerImpl
    priors = [[1.0, 1.5], [2.0, 1.0]]
    conf = Conf(boundingBoxes=priors)
    if seed == 2:
        conf.lossPositionScale = LossMSE()
        conf.lambdaNoObj = 0.7
        conf.lambdaCoord = 3.0
    impl = Yolo2OutputLayerImpl(conf)
    x, lab = _yolo_case(seed)
    loss, gx = impl._loss(x, lab, need_grad=True)
    xr = x.clone().requires_grad_(True)
    with torch.enable_grad():
        (ref,) = torch.autograd.grad(impl._loss(xr, lab), [xr])
    torch.testing.assert_close(gx, ref, rtol=1e-9, atol=1e-12)
    # the IOU path is live (the gradient differs from one with the IOU label held constant)
    resp_cells = lab[:, 4:].sum(1) > 0
    assert resp_cells.any()
    h = 1e-6
    flat = x.view(-1)
    idx = torch.randperm(flat.numel(), generator=torch.Generator().manual_seed(seed))[:120]
    for i in idx.tolist():
        old = flat[i].item()
        flat[i] = old + h
        sp = float(impl._loss(x, lab))
        flat[i] = old - h
        sm = float(impl._loss(x, lab))
        flat[i] = old
        num = (sp - sm) / (2 * h)
        got = gx.reshape(-1)[i].item()
        assert abs(num - got) <= 1e-8 + 1e-5 * max(abs(num), abs(got)), (i, num, got)


def test_yolo2_iou_term_contributes():
    """With lambdaCoord = 0 the xy/wh gradients can only come through the IOU confidence label: they must be
    nonzero on responsible anchors (and still match finite differences, covered above)."""
    from deeplearning4j_amd.nn.conf.layers import Yolo2OutputLayer as Conf
    from deeplearning4j_amd.nn.layers.objdetect import Yolo2OutputLayerImpl
    conf = Conf(boundingBoxes=[[1.0, 1.5], [2.0, 1.0]])
    conf.lambdaCoord = 0.0
    impl = Yolo2OutputLayerImpl(conf)
    x, lab = _yolo_case(5)
    _, g = impl._loss(x, lab, need_grad=True)
    g5 = g.reshape(2, 2, 8, 4, 4)
    obj = (lab[:, 4:].sum(1) > 0)
    assert torch.count_nonzero(g5[:, :, 0:4][obj.unsqueeze(1).unsqueeze(2).expand(2, 2, 4, 4, 4)]) > 0
    assert torch.count_nonzero(g5[:, :, 0:4][~obj.unsqueeze(1).unsqueeze(2).expand(2, 2, 4, 4, 4)]) == 0
