"""AutoEncoder runtime (reference nn/layers/feedforward/autoencoder/AutoEncoder.java, BasePretrainNetwork.java).

Supervised use (inside a network): behaves as a dense layer y = act(xW + b); the visible bias ``vb`` is a
pretrain-only parameter and gets a zero gradient (BasePretrainNetwork.backpropGradient).
Layer-wise pretraining (``computePretrainGradientAndScore``): input corrupted by zeroing a ``corruptionLevel``
fraction of entries, encode y = act(x~ W + b), decode z = act(y W^T + vb) with tied weights, loss =
lossFunction(x, z_pre) (+ KL sparsity penalty when ``sparsity`` > 0); gradients of all three parameters
come from autograd and land in the flat gradient views. Parity with the reference's hand-written
pretrain gradient is unpinned (its sign convention predates the current updater path); tests check that
pretraining decreases the reconstruction loss.
"""
import torch

from .feedforward import DenseLayerImpl


class AutoEncoderImpl(DenseLayerImpl):
    def backpropGradient(self, eps):
        g, e = super().backpropGradient(eps)
        self.grads["vb"].zero_()
        return g, e

    def isPretrainLayer(self):
        return True

    def _loss(self):
        from ..conf.losses import LossMSE
        return self.conf.lossFunction or LossMSE()

    def encode(self, x, training=False):
        W, b = self.params["W"], self.params["b"]
        return self.conf.activation.getActivation(x.to(W.dtype) @ W + b, training)

    def decode(self, y):
        W, vb = self.params["W"], self.params["vb"]
        return self.conf.activation.getActivation(y @ W.t() + vb, False)

    def reconstruct(self, x):
        return self.decode(self.encode(x))

    def computePretrainGradientAndScore(self, x):
        c = self.conf
        keys = ["W", "b", "vb"]
        p = {k: self.params[k].detach().clone().requires_grad_(True) for k in keys}
        x = x.to(p["W"].dtype)
        if c.corruptionLevel and c.corruptionLevel > 0:
            x_in = x * (torch.rand_like(x) >= c.corruptionLevel).to(x.dtype)
        else:
            x_in = x
        with torch.enable_grad():
            y = c.activation.getActivation(x_in @ p["W"] + p["b"], True)
            z_pre = y @ p["W"].t() + p["vb"]
            loss = self._loss().computeScore(x, z_pre, c.activation, None, False)
            if c.sparsity and c.sparsity > 0:
                rho_hat = y.mean(0).clamp(1e-6, 1 - 1e-6)
                rho = c.sparsity
                loss = loss + x.shape[0] * (rho * torch.log(rho / rho_hat) +
                                            (1 - rho) * torch.log((1 - rho) / (1 - rho_hat))).sum()
            grads = torch.autograd.grad(loss, [p[k] for k in keys])
        for k, gk in zip(keys, grads):
            self.grads[k].copy_(gk.reshape(self.grads[k].shape))
        return float(loss.detach()) / x.shape[0]
