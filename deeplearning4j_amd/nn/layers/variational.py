"""Variational autoencoder runtime (reference nn/layers/variational/VariationalAutoencoder.java).

Supervised use (inside a network, after pretraining): output = pzxActivationFn(mean pre-output of q(z|x)),
backprop through the encoder + p(z|x)-mean parameters only; decoder / p(x|z) / log-variance parameters get a
zero gradient (they are pretrain parameters, conf isPretrainParam).
Pretraining (``computePretrainGradientAndScore``): negative ELBO with the reparameterisation trick,
score = KL(q(z|x) || N(0,I)) / mb + mean over ``numSamples`` of -log p(x|z) / mb (reference :176-240,
activation applied to both the mean and log-variance pre-outputs).
Both paths are hand-derived backward passes (reference VariationalAutoencoder.backpropGradient :807-880 and
computeGradientAndScore :176-360): dKL/dmean = mean, dKL/dlog(s^2) = (exp(log s^2) - 1) / 2, the reconstruction
distribution supplies d(-log p(x|z))/d(decoder pre-output) (conf/variational.py ``gradient``), and the
reparameterisation z = mean + exp(log s^2 / 2) * eps routes dz into dmean += dz, dlog(s^2) += dz * eps * s / 2.
tests/test_explicit_backward.py checks every parameter gradient against a finite-difference fp64 gradient check.
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

    def _encode(self, x, p, training, cache=None):
        """Encoder forward; with ``cache`` (a list) records (input, pre-activation) per dense step for backward."""
        h = x
        act = self.conf.activation
        for i in range(len(self.conf.encoderLayerSizes)):
            z = h @ p[f"e{i}W"] + p[f"e{i}b"]
            if cache is not None:
                cache.append((h, z))
            h = act.getActivation(z, training)
        pzx = self._pzx_act()
        zm = h @ p["pZXMeanW"] + p["pZXMeanb"]
        zl = h @ p["pZXLogStd2W"] + p["pZXLogStd2b"]
        if cache is not None:
            cache.append((h, zm, zl))
        return pzx.getActivation(zm, training), pzx.getActivation(zl, training)

    def _decode_pre(self, z, p, training=False, cache=None):
        h = z
        for i in range(len(self.conf.decoderLayerSizes)):
            a = h @ p[f"d{i}W"] + p[f"d{i}b"]
            if cache is not None:
                cache.append((h, a))
            h = self.conf.activation.getActivation(a, training)
        if cache is not None:
            cache.append(h)
        return h @ p["pXZW"] + p["pXZb"]

    @staticmethod
    def _acc_grad(g, k, val):
        g[k] = val if k not in g else g[k] + val

    def _dense_back(self, g, wk, bk, h_in, dz, W):
        """Dense step y = h_in @ W + b: accumulate dW/db into ``g`` and return dL/dh_in."""
        self._acc_grad(g, wk, h_in.t() @ dz)
        self._acc_grad(g, bk, dz.sum(0, keepdim=True))
        return dz @ W.t()

    def _decoder_back(self, cache, dpre, p, g):
        """Backward through the decoder stack from d/d(p(x|z) pre-output); returns dL/dz."""
        dh = self._dense_back(g, "pXZW", "pXZb", cache[-1], dpre, p["pXZW"])
        act = self.conf.activation
        for i in reversed(range(len(self.conf.decoderLayerSizes))):
            h_in, a = cache[i]
            dh = self._dense_back(g, f"d{i}W", f"d{i}b", h_in, act.backprop(a, dh), p[f"d{i}W"])
        return dh

    def _encoder_back(self, cache, dmean, dlogs2, p, g):
        """Backward from d/dmean (and d/dlog s^2 unless None) of q(z|x) to dL/dx."""
        pzx = self._pzx_act()
        h, zm, zl = cache[-1]
        dh = self._dense_back(g, "pZXMeanW", "pZXMeanb", h, pzx.backprop(zm, dmean), p["pZXMeanW"])
        if dlogs2 is not None:
            dh = dh + self._dense_back(g, "pZXLogStd2W", "pZXLogStd2b", h, pzx.backprop(zl, dlogs2),
                                       p["pZXLogStd2W"])
        act = self.conf.activation
        for i in reversed(range(len(self.conf.encoderLayerSizes))):
            h_in, z = cache[i]
            dh = self._dense_back(g, f"e{i}W", f"e{i}b", h_in, act.backprop(z, dh), p[f"e{i}W"])
        return dh

    def _store_grads(self, g):
        for k in self.grads:
            if k in g:
                self.grads[k].copy_(g[k].reshape(self.grads[k].shape))
            else:
                self.grads[k].zero_()

    def _p(self, dtype):
        return {k: v.detach().to(dtype) for k, v in self.params.items()}

    # ------------------------------------------------------------------ supervised path
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
        p = self._p(dt)
        cache = []
        with torch.no_grad():
            self._encode(self.input.to(dt), p, True, cache)
            g = {}
            dx = self._encoder_back(cache, eps.to(dt), None, p, g)
        self._store_grads(g)                              # decoder / log-variance params: zero (pretrain only)
        return self.make_gradient(), self.backpropDropOut(dx.to(self.input.dtype))

    # ------------------------------------------------------------------ pretraining
    def computePretrainGradientAndScore(self, x):
        c = self.conf
        dt = self.params["pZXMeanW"].dtype
        p = self._p(dt)
        x = x.to(dt)
        mb = x.shape[0]
        ns = max(1, int(c.numSamples or 1))
        dist = self._dist()
        g = {}
        with torch.no_grad():
            enc = []
            mean, logs2 = self._encode(x, p, True, enc)
            e_ls = logs2.exp()
            kl = -0.5 / mb * (1.0 + logs2 - mean * mean - e_ls).sum()
            dmean = mean.clone()                          # gradients of mb * (KL + reconstruction) / mb-scaled score
            dlogs2 = 0.5 * (e_ls - 1.0)
            sigma = (0.5 * logs2).exp()
            rec = 0.0
            for _ in range(ns):
                eps = torch.randn_like(mean)
                z = mean + sigma * eps
                dec = []
                pre = self._decode_pre(z, p, True, dec)
                rec = rec + dist.negLogProbability(x, pre, True) / ns
                dz = self._decoder_back(dec, dist.gradient(x, pre) / ns, p, g)
                dmean += dz
                dlogs2 += dz * eps * (0.5 * sigma)
            self._encoder_back(enc, dmean, dlogs2, p, g)
            loss = kl + rec
        self._store_grads(g)
        return float(loss)

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
