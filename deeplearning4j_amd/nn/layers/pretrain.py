"""AutoEncoder runtime (reference nn/layers/feedforward/autoencoder/AutoEncoder.java, BasePretrainNetwork.java).

Supervised use (inside a network): behaves as a dense layer y = act(xW + b); the visible bias ``vb`` is a
pretrain-only parameter and gets a zero gradient (BasePretrainNetwork.backpropGradient).
Layer-wise pretraining (``computePretrainGradientAndScore``): input corrupted by zeroing a ``corruptionLevel``
fraction of entries, encode y = act(x~ W + b), decode z = act(y W^T + vb) with tied weights, loss =
lossFunction(x, z_pre) (+ KL sparsity penalty when ``sparsity`` > 0). The gradient is derived by hand
(reference AutoEncoder.computeGradientAndScore / BasePretrainNetwork): dz = lossFunction.computeGradient(x, z_pre),
dvb = sum(dz), dW = dz^T y (decoder use of the tied weight) + x~^T dy_pre (encoder use), dy = dz W + the
sparsity term, dy_pre = act'(dy), db = sum(dy_pre). tests/test_explicit_backward.py gradient-checks it in fp64.
The reference's own pretrain update predates its current updater sign convention, so parity there is unpinned;
tests also check that pretraining decreases the reconstruction loss.
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
        W, b, vb = (self.params[k].detach() for k in ("W", "b", "vb"))
        x = x.to(W.dtype)
        if c.corruptionLevel and c.corruptionLevel > 0:
            x_in = x * (torch.rand_like(x) >= c.corruptionLevel).to(x.dtype)
        else:
            x_in = x
        act = c.activation
        lossfn = self._loss()
        with torch.no_grad():
            a = x_in @ W + b
            y = act.getActivation(a, True)
            z_pre = y @ W.t() + vb
            loss = lossfn.computeScore(x, z_pre, act, None, False)
            dz = lossfn.computeGradient(x, z_pre, act, None).to(W.dtype)
            dW = dz.t() @ y
            dvb = dz.sum(0)
            dy = dz @ W
            if c.sparsity and c.sparsity > 0:
                m = y.mean(0)
                rho_hat = m.clamp(1e-6, 1 - 1e-6)
                rho = c.sparsity
                loss = loss + x.shape[0] * (rho * torch.log(rho / rho_hat) +
                                            (1 - rho) * torch.log((1 - rho) / (1 - rho_hat))).sum()
                inside = ((m >= 1e-6) & (m <= 1 - 1e-6)).to(y.dtype)
                dy = dy + (-rho / rho_hat + (1 - rho) / (1 - rho_hat)) * inside      # d(mb * KL)/d(mean) / mb
            da = act.backprop(a, dy)
            dW += x_in.t() @ da
            db = da.sum(0)
        for k, gk in (("W", dW), ("b", db), ("vb", dvb)):
            self.grads[k].copy_(gk.reshape(self.grads[k].shape))
        return float(loss) / x.shape[0]
