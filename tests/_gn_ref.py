"""Reference semantics of DL4J gradient normalization (BaseMultiLayerUpdater.java:322-382), computed by hand on the
raw summed gradient of each layer, for the CPU and GPU tests of the fused updater."""
import torch


def make_net(gn, thr, device=None, seed=5):
    from deeplearning4j_amd import (Activation, DenseLayer, LossFunction, MultiLayerNetwork, NeuralNetConfiguration,
                                    OutputLayer, Sgd)
    conf = (NeuralNetConfiguration.Builder().seed(seed).updater(Sgd(0.5)).gradientNormalization(gn)
            .gradientNormalizationThreshold(thr).list()
            .layer(0, DenseLayer.Builder().nIn(6).nOut(9).activation(Activation.TANH).build())
            .layer(1, DenseLayer.Builder().nIn(9).nOut(7).activation(Activation.TANH).build())
            .layer(2, OutputLayer.Builder(LossFunction.MCXENT).nIn(7).nOut(3).activation(Activation.SOFTMAX).build())
            .build())
    net = MultiLayerNetwork(conf)
    net.init(device=device or torch.device("cpu"))
    return net


def data(device=None, bs=10):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(bs, 6, generator=g) * 3
    y = torch.zeros(bs, 3)
    y[torch.arange(bs), torch.randint(0, 3, (bs,), generator=g)] = 1
    return x.to(device or "cpu"), y.to(device or "cpu")


def expected_step(net, x, y, gn, thr, lr=0.5):
    """params after one SGD step with gradient normalization, from the raw gradient of computeGradientAndScore."""
    from deeplearning4j_amd.nn.conf.enums import GradientNormalization as G
    p0 = net.params().detach().clone().double().reshape(-1)
    net.computeGradientAndScore(x, y)
    g = net.getGradientsViewArray().detach().clone().double().reshape(-1)
    table = net.paramTable()
    base = net.params().data_ptr()
    layers = {}
    for key, v in table.items():
        li = key.split("_")[0]
        off = (v.data_ptr() - base) // v.element_size()
        layers.setdefault(li, []).append((off, v.numel()))
    for li, parts in layers.items():
        views = [g[o:o + n] for o, n in parts]
        if gn == G.RenormalizeL2PerLayer:
            nrm = torch.sqrt(sum((v ** 2).sum() for v in views))
            for v in views:
                v /= nrm
        elif gn == G.RenormalizeL2PerParamType:
            for v in views:
                v /= v.norm()
        elif gn == G.ClipElementWiseAbsoluteValue:
            for v in views:
                v.clamp_(-thr, thr)
        elif gn == G.ClipL2PerLayer:
            nrm = torch.sqrt(sum((v ** 2).sum() for v in views))
            if nrm > thr:
                for v in views:
                    v *= thr / nrm
        elif gn == G.ClipL2PerParamType:
            for v in views:
                n = v.norm()
                if n > thr:
                    v *= thr / n
    return p0 - lr * g / x.shape[0]
