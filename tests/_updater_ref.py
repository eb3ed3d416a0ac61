"""Expected updater outputs written out exactly as the reference's TestUpdaters computes them by hand
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/updater/TestUpdaters.java: AdaDelta :61-131, AdaGrad
:133-165, Adam :167-220, Nadam :222-292, Nesterovs :350-371, RmsProp :400-420, Sgd :460-472, NoOp :480-506), and a
driver that pushes a known gradient through a network's real update path (host reference on CPU, the fused HIP
updater kernel on GPU) for two iterations and returns the applied updates (params_before - params_after)."""
import math

import torch


def expected(kind, hp, grads):
    """Sequence of expected updates for the gradients ``grads`` (one per iteration), fp64."""
    g0 = grads[0]
    out = []
    if kind == "sgd":
        return [hp["lr"] * g for g in grads]
    if kind == "noop":
        return [g.clone() for g in grads]          # TestUpdaters.testNoOpUpdater: the gradient passes unchanged
    if kind == "adagrad":
        h = torch.zeros_like(g0)
        for g in grads:
            h = h + g * g
            out.append(hp["lr"] * g / torch.sqrt(h + hp["eps"]))
        return out
    if kind == "adadelta":
        msg, msdx = torch.zeros_like(g0), torch.zeros_like(g0)
        for g in grads:
            msg = msg * hp["rho"] + g * g * (1 - hp["rho"])
            u = torch.sqrt(msdx + hp["eps"]) / torch.sqrt(msg + hp["eps"]) * g
            msdx = msdx * hp["rho"] + u * u * (1 - hp["rho"])
            out.append(u)
        return out
    if kind == "adam":
        m, v = torch.zeros_like(g0), torch.zeros_like(g0)
        for it, g in enumerate(grads):
            b1t, b2t = hp["b1"] ** (it + 1), hp["b2"] ** (it + 1)
            alphat = hp["lr"] * math.sqrt(1 - b2t) / (1 - b1t)
            m = m * hp["b1"] + g * (1 - hp["b1"])
            v = v * hp["b2"] + g * g * (1 - hp["b2"])
            out.append(m * alphat / (torch.sqrt(v) + hp["eps"]))
        return out
    if kind == "nadam":
        m, v = torch.zeros_like(g0), torch.zeros_like(g0)
        for it, g in enumerate(grads):
            b1t = hp["b1"] ** (it + 1)
            omb1g = g * (1 - hp["b1"])
            m = m * hp["b1"] + omb1g
            v = v * hp["b2"] + g * g * (1 - hp["b2"])
            alphat = (m * hp["b1"] / (1 - b1t) + omb1g / (1 - b1t)) * hp["lr"]
            out.append(alphat / (torch.sqrt(v) + hp["eps"]))
        return out
    if kind == "nesterovs":
        v = torch.zeros_like(g0)
        for g in grads:
            vprev = v
            v = v * hp["mu"] - g * hp["lr"]
            out.append(vprev * hp["mu"] + v * (-hp["mu"] - 1))
        return out
    if kind == "rmsprop":
        c = torch.zeros_like(g0)
        for g in grads:
            c = c * hp["decay"] + g * g * (1 - hp["decay"])
            out.append(g * hp["lr"] / torch.sqrt(c + hp["eps"]))
        return out
    raise ValueError(kind)


CASES = {
    "sgd": dict(lr=0.05),
    "noop": dict(),
    "adagrad": dict(lr=1e-2, eps=1e-6),
    "adadelta": dict(rho=0.85, eps=1e-6),
    "adam": dict(lr=0.01, b1=0.8, b2=0.888, eps=1e-8),
    "nadam": dict(lr=0.01, b1=0.8, b2=0.888, eps=1e-8),
    "nesterovs": dict(lr=1e-2, mu=0.6),
    "rmsprop": dict(lr=0.01, decay=0.25, eps=1e-8),
}


def make_updater(kind, hp):
    from deeplearning4j_amd.nn.conf import updaters as U
    return {
        "sgd": lambda: U.Sgd(learningRate=hp["lr"]),
        "noop": lambda: U.NoOp(),
        "adagrad": lambda: U.AdaGrad(learningRate=hp["lr"], epsilon=hp["eps"]),
        "adadelta": lambda: U.AdaDelta(rho=hp["rho"], epsilon=hp["eps"]),
        "adam": lambda: U.Adam(learningRate=hp["lr"], beta1=hp["b1"], beta2=hp["b2"], epsilon=hp["eps"]),
        "nadam": lambda: U.Nadam(learningRate=hp["lr"], beta1=hp["b1"], beta2=hp["b2"], epsilon=hp["eps"]),
        "nesterovs": lambda: U.Nesterovs(learningRate=hp["lr"], momentum=hp["mu"]),
        "rmsprop": lambda: U.RmsProp(learningRate=hp["lr"], rmsDecay=hp["decay"], epsilon=hp["eps"]),
    }[kind]()


def run_network_updates(kind, device):
    """Two updates through net._apply_update_kernels with fixed gradients; returns (actual, expected) lists."""
    from deeplearning4j_amd import Activation, LossFunction, MultiLayerNetwork, NeuralNetConfiguration
    from deeplearning4j_amd.nn.conf.layers import DenseLayer, OutputLayer
    hp = CASES[kind]
    conf = (NeuralNetConfiguration.Builder().seed(12345).updater(make_updater(kind, hp)).list()
            .layer(0, DenseLayer.Builder().nIn(4).nOut(5).activation(Activation.TANH).build())
            .layer(1, OutputLayer.Builder(LossFunction.MSE).nIn(5).nOut(3).activation(Activation.IDENTITY).build())
            .build())
    net = MultiLayerNetwork(conf)
    net.init(device=torch.device(device))
    n = net.numParams()
    gen = torch.Generator().manual_seed(7)
    grads = [torch.randn(n, generator=gen, dtype=torch.float64) * 0.5 for _ in range(2)]
    actual = []
    for it, g in enumerate(grads):
        net.conf.iterationCount = it
        before = net.flattenedParams.detach().double().cpu().clone()
        net.flattenedGradients.copy_(g.to(net.flattenedGradients.dtype))
        net._apply_update_kernels(1)
        if device != "cpu":
            torch.cuda.synchronize()
        actual.append(before - net.flattenedParams.detach().double().cpu())
    return actual, expected(kind, hp, grads)
