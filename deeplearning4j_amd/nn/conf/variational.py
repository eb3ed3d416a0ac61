"""Reconstruction distributions p(x|z) for the VariationalAutoencoder layer
(reference nn/conf/layers/variational/{Gaussian,Bernoulli,Exponential,Composite}ReconstructionDistribution.java,
LossFunctionWrapper.java). Each maps the decoder's pre-output ("distribution parameters") to a negative log
likelihood (``exampleNegLogProbability``) and gives its hand-derived gradient with respect to that pre-output
(``gradient``, reference ReconstructionDistribution.gradient) for the VAE's explicit backward pass."""
import math

import torch

from .activations import ActivationIdentity, ActivationSigmoid, to_activation
from .base import Config
from .losses import to_loss

NEG_HALF_LOG_2PI = -0.5 * math.log(2 * math.pi)


class ReconstructionDistribution(Config):
    def hasLossFunction(self):
        return False

    def distributionInputSize(self, dataSize):
        raise NotImplementedError

    def exampleNegLogProbability(self, x, preOut):
        """Per-example negative log probability [mb]."""
        raise NotImplementedError

    def negLogProbability(self, x, preOut, average=True):
        s = self.exampleNegLogProbability(x, preOut).sum()
        return s / x.shape[0] if average else s

    def gradient(self, x, preOut):
        """d(sum of exampleNegLogProbability) / d preOut."""
        raise NotImplementedError

    def generateAtMean(self, preOut):
        raise NotImplementedError

    def generateRandom(self, preOut):
        raise NotImplementedError


class GaussianReconstructionDistribution(ReconstructionDistribution):
    """preOut = [mean | log(sigma^2)] after the activation (Gaussian...Distribution.java)."""
    FIELDS = {"activationFn": None}
    _CONVERTERS = {"activationFn": to_activation}

    def __init__(self, activationFn=None, **kw):
        super().__init__(activationFn=activationFn or ActivationIdentity(), **kw)

    def distributionInputSize(self, dataSize):
        return 2 * dataSize

    def _split(self, preOut):
        out = self.activationFn.getActivation(preOut, True)
        n = out.shape[1] // 2
        return out[:, :n], out[:, n:]

    def exampleNegLogProbability(self, x, preOut):
        mean, logs2 = self._split(preOut)
        n = mean.shape[1]
        return 0.5 * logs2.sum(1) - n * NEG_HALF_LOG_2PI + ((x - mean) ** 2 / logs2.exp() / 2).sum(1)

    def gradient(self, x, preOut):
        mean, logs2 = self._split(preOut)
        inv = (-logs2).exp()
        d = x - mean
        dmean = -d * inv                                  # d/dmean of (x - mean)^2 / (2 sigma^2)
        dlogs2 = 0.5 - 0.5 * d * d * inv                  # d/dlog(sigma^2) of 0.5 log(sigma^2) + (x-mean)^2 e^-ls / 2
        return self.activationFn.backprop(preOut, torch.cat([dmean, dlogs2], dim=1))

    def generateAtMean(self, preOut):
        return self._split(preOut)[0]

    def generateRandom(self, preOut):
        mean, logs2 = self._split(preOut)
        return mean + torch.randn_like(mean) * (0.5 * logs2).exp()


class BernoulliReconstructionDistribution(ReconstructionDistribution):
    FIELDS = {"activationFn": None}
    _CONVERTERS = {"activationFn": to_activation}

    def __init__(self, activationFn=None, **kw):
        super().__init__(activationFn=activationFn or ActivationSigmoid(), **kw)

    def distributionInputSize(self, dataSize):
        return dataSize

    def exampleNegLogProbability(self, x, preOut):
        p = self.activationFn.getActivation(preOut, True).clamp(1e-5, 1 - 1e-5)
        return -(x * p.log() + (1 - x) * (1 - p).log()).sum(1)

    def gradient(self, x, preOut):
        q = self.activationFn.getActivation(preOut, True)
        inside = ((q >= 1e-5) & (q <= 1 - 1e-5)).to(q.dtype)          # the clamp passes no gradient outside
        p = q.clamp(1e-5, 1 - 1e-5)
        dp = (-x / p + (1 - x) / (1 - p)) * inside
        return self.activationFn.backprop(preOut, dp)

    def generateAtMean(self, preOut):
        return self.activationFn.getActivation(preOut, False)

    def generateRandom(self, preOut):
        p = self.activationFn.getActivation(preOut, False)
        return (torch.rand_like(p) < p).to(p.dtype)


class ExponentialReconstructionDistribution(ReconstructionDistribution):
    """lambda = exp(act(preOut)); log p(x) = log(lambda) - lambda * x."""
    FIELDS = {"activationFn": None}
    _CONVERTERS = {"activationFn": to_activation}

    def __init__(self, activationFn=None, **kw):
        super().__init__(activationFn=activationFn or ActivationIdentity(), **kw)

    def distributionInputSize(self, dataSize):
        return dataSize

    def exampleNegLogProbability(self, x, preOut):
        gamma = self.activationFn.getActivation(preOut, True)
        return -(gamma - gamma.exp() * x).sum(1)

    def gradient(self, x, preOut):
        gamma = self.activationFn.getActivation(preOut, True)
        return self.activationFn.backprop(preOut, gamma.exp() * x - 1.0)

    def generateAtMean(self, preOut):
        return 1.0 / self.activationFn.getActivation(preOut, False).exp()

    def generateRandom(self, preOut):
        lam = self.activationFn.getActivation(preOut, False).exp()
        u = torch.rand_like(lam)
        return -torch.log(1 - u) / lam


class CompositeReconstructionDistribution(ReconstructionDistribution):
    """Different distributions for consecutive column ranges of the data."""
    FIELDS = {"distributionSizes": [], "reconstructionDistributions": []}

    class Builder:
        def __init__(self):
            self.sizes, self.dists = [], []

        def addDistribution(self, size, dist):
            self.sizes.append(int(size))
            self.dists.append(dist)
            return self

        def build(self):
            return CompositeReconstructionDistribution(distributionSizes=self.sizes,
                                                       reconstructionDistributions=self.dists)

    def hasLossFunction(self):
        return any(d.hasLossFunction() for d in self.reconstructionDistributions)

    def distributionInputSize(self, dataSize):
        return sum(d.distributionInputSize(s) for s, d in zip(self.distributionSizes, self.reconstructionDistributions))

    def _chunks(self, x, preOut):
        xi = pi = 0
        for s, d in zip(self.distributionSizes, self.reconstructionDistributions):
            ps = d.distributionInputSize(s)
            yield d, (x[:, xi:xi + s] if x is not None else None), preOut[:, pi:pi + ps]
            xi += s
            pi += ps

    def exampleNegLogProbability(self, x, preOut):
        return sum(d.exampleNegLogProbability(xs, ps) for d, xs, ps in self._chunks(x, preOut))

    def gradient(self, x, preOut):
        return torch.cat([d.gradient(xs, ps) for d, xs, ps in self._chunks(x, preOut)], dim=1)

    def generateAtMean(self, preOut):
        return torch.cat([d.generateAtMean(ps) for d, _, ps in self._chunks(None, preOut)], dim=1)

    def generateRandom(self, preOut):
        return torch.cat([d.generateRandom(ps) for d, _, ps in self._chunks(None, preOut)], dim=1)


class LossFunctionWrapper(ReconstructionDistribution):
    """Use an ordinary loss function as the 'reconstruction distribution' (not a true probability)."""
    FIELDS = {"activationFn": None, "lossFunction": None}
    _CONVERTERS = {"activationFn": to_activation, "lossFunction": to_loss}

    def __init__(self, activationFn=None, lossFunction=None, **kw):
        """Reference LossFunctionWrapper(IActivation activationFn, ILossFunction lossFunction)."""
        super().__init__(activationFn=activationFn or ActivationIdentity(), lossFunction=lossFunction, **kw)

    def hasLossFunction(self):
        return True

    def distributionInputSize(self, dataSize):
        return dataSize

    def exampleNegLogProbability(self, x, preOut):
        return self.lossFunction.computeScoreArray(x, preOut, self.activationFn, None)

    def gradient(self, x, preOut):
        return self.lossFunction.computeGradient(x, preOut, self.activationFn, None)

    def generateAtMean(self, preOut):
        return self.activationFn.getActivation(preOut, False)

    def generateRandom(self, preOut):
        return self.generateAtMean(preOut)
