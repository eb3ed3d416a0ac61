"""Variational autoencoder runtime (reference nn/layers/variational/VariationalAutoencoder.java).

Supervised use (inside a network, after pretraining): output = pzxActivationFn(mean pre-output of q(z|x)),
backprop through the encoder + p(z|x)-mean parameters only; decoder / p(x|z) / log-variance parameters get a
zero gradient (they are pretrain parameters, conf isPretrainParam).
Pretraining (``computePretrainGradientAndScore``): negative ELBO with the reparameterisation trick,
score = KL(q(z|x) || N(0,I)) / mb + mean over ``numSamples`` of -log p(x|z) / mb (reference :176-240,
activation applied to both the mean and log-variance pre-outputs), gradients by autograd.
Also: reconstructionLogProbability / reconstructionProbability (importance-sampled, reference
reconstructionLogProbability), generateAtMeanGivenZ, generateRandomGivenZ, reconstructionError.
"""
import math

import torch

from .base import LayerImpl


class VariationalAutoencoderImpl(LayerImpl):
    def isPretrainLayer(self):
        return True

    def _dist(self):
        from ..conf.variational import GaussianReconstructionDistribution
        return self.conf.outputDistribution or GaussianReconstructionDistribution()

    def _pzx_act(self):
        from ..conf.activations import ActivationIdentity
        return self.conf.pzxActivationFn or ActivationIdentity()

    def _encode(self, x, p, training):
        h = x
        for i in range(len(self.conf.encoderLayerSizes)):
            h = self.conf.activation.getActivation(h @ p[f"e{i}W"] + p[f"e{i}b"], training)
        act = self._pzx_act()
        mean = act.getActivation(h @ p["pZXMeanW"] + p["pZXMeanb"], training)
        logs2 = act.getActivation(h @ p["pZXLogStd2W"] + p["pZXLogStd2b"], training)
        return mean, logs2

    def _decode_pre(self, z, p, training=False):
        h = z
        for i in range(len(self.conf.decoderLayerSizes)):
            h = self.conf.activation.getActivation(h @ p[f"d{i}W"] + p[f"d{i}b"], training)
        return h @ p["pXZW"] + p["pXZb"]

    def _p(self, dtype, keys=None, grad=False):
        out = {}
        for k, v in self.params.items():
            t = v.detach().to(dtype)
            if grad and (keys is None or k in keys):
                t = t.clone().requires_grad_(True)
            out[k] = t
        return out

    # ------------------------------------------------------------------ supervised path
    def _enc_keys(self):
        return [k for k in self.params if k.startswith("e") or k.startswith("pZXMean")]

    def activate(self, x, training=False, mask=None, **kw):
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        dt = self.params["pZXMeanW"].dtype
        with torch.no_grad():
            mean, _ = self._encode(x.to(dt), self._p(dt), training)
        return mean.to(x.dtype) if x.is_floating_point() else mean

    def backpropGradient(self, eps, **kw):
        dt = self.params["pZXMeanW"].dtype
        keys = self._enc_keys()
        p = self._p(dt, keys, True)
        x = self.input.detach().to(dt).requires_grad_(True)
        with torch.enable_grad():
            mean, _ = self._encode(x, p, True)
            grads = torch.autograd.grad(mean, [x] + [p[k] for k in keys], eps.to(dt))
        for k in self.grads:
            self.grads[k].zero_()
        for k, g in zip(keys, grads[1:]):
            self.grads[k].copy_(g.reshape(self.grads[k].shape))
        return self.make_gradient(), self.backpropDropOut(grads[0].to(self.input.dtype))

    # ------------------------------------------------------------------ pretraining
    def computePretrainGradientAndScore(self, x):
        c = self.conf
        dt = self.params["pZXMeanW"].dtype
        keys = list(self.params)
        p = self._p(dt, keys, True)
        x = x.to(dt)
        mb = x.shape[0]
        ns = max(1, int(c.numSamples or 1))
        dist = self._dist()
        with torch.enable_grad():
            mean, logs2 = self._encode(x, p, True)
            kl = -0.5 / mb * (1.0 + logs2 - mean * mean - logs2.exp()).sum()
            rec = 0.0
            sigma = (0.5 * logs2).exp()
            for _ in range(ns):
                z = mean + sigma * torch.randn_like(mean)
                rec = rec + dist.negLogProbability(x, self._decode_pre(z, p, True), True) / ns
            loss = kl + rec
            grads = torch.autograd.grad(loss * mb, [p[k] for k in keys], allow_unused=True)
        for k, g in zip(keys, grads):
            if g is None:
                self.grads[k].zero_()
            else:
                self.grads[k].copy_(g.reshape(self.grads[k].shape))
        return float(loss.detach())

    # ------------------------------------------------------------------ generative API
    def reconstructionLogProbability(self, data, numSamples=1):
        if self._dist().hasLossFunction():
            raise ValueError("Cannot calculate reconstruction log probability when using a LossFunctionWrapper "
                             "reconstruction distribution")
        dt = self.params["pZXMeanW"].dtype
        with torch.no_grad():
            x = data.to(dt)
            p = self._p(dt)
            mean, logs2 = self._encode(x, p, False)
            sigma = (0.5 * logs2).exp()
            dist = self._dist()
            lps = []
            for _ in range(int(numSamples)):
                z = mean + sigma * torch.randn_like(mean)
                lps.append(-dist.exampleNegLogProbability(x, self._decode_pre(z, p)))
            lp = torch.stack(lps, 0)
            return torch.logsumexp(lp, 0) - math.log(len(lps))

    def reconstructionProbability(self, data, numSamples=1):
        return self.reconstructionLogProbability(data, numSamples).exp()

    def generateAtMeanGivenZ(self, z):
        dt = self.params["pXZW"].dtype
        with torch.no_grad():
            return self._dist().generateAtMean(self._decode_pre(z.to(dt), self._p(dt)))

    def generateRandomGivenZ(self, z):
        dt = self.params["pXZW"].dtype
        with torch.no_grad():
            return self._dist().generateRandom(self._decode_pre(z.to(dt), self._p(dt)))

    def hasLossFunction(self):
        return self._dist().hasLossFunction()

    def reconstructionError(self, data):
        if not self.hasLossFunction():
            raise ValueError("reconstructionError requires a LossFunctionWrapper reconstruction distribution")
        dt = self.params["pZXMeanW"].dtype
        with torch.no_grad():
            x = data.to(dt)
            p = self._p(dt)
            mean, _ = self._encode(x, p, False)
            return self._dist().exampleNegLogProbability(x, self._decode_pre(mean, p))
