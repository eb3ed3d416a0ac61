"""Reconstruction distributions p(x|z) for the VariationalAutoencoder layer
(reference nn/conf/layers/variational/{Gaussian,Bernoulli,Exponential,Composite}ReconstructionDistribution.java,
LossFunctionWrapper.java). Each maps the decoder's pre-output ("distribution parameters") to a negative log
likelihood; gradients come from autograd in the VAE runtime, so only the forward math lives here."""
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

    def generateAtMean(self, preOut):
        return torch.cat([d.generateAtMean(ps) for d, _, ps in self._chunks(None, preOut)], dim=1)

    def generateRandom(self, preOut):
        return torch.cat([d.generateRandom(ps) for d, _, ps in self._chunks(None, preOut)], dim=1)


class LossFunctionWrapper(ReconstructionDistribution):
    """Use an ordinary loss function as the 'reconstruction distribution' (not a true probability)."""
    FIELDS = {"activationFn": None, "lossFunction": None}
    _CONVERTERS = {"activationFn": to_activation, "lossFunction": to_loss}

    def hasLossFunction(self):
        return True

    def distributionInputSize(self, dataSize):
        return dataSize

    def exampleNegLogProbability(self, x, preOut):
        return self.lossFunction.computeScoreArray(x, preOut, self.activationFn, None)

    def generateAtMean(self, preOut):
        return self.activationFn.getActivation(preOut, False)

    def generateRandom(self, preOut):
        return self.generateAtMean(preOut)
