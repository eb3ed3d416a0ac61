"""Multi-head self-attention over recurrent-format activations [mb, nIn, T].

Not in the reference snapshot (no attention/LayerNorm layers exist there); added for the
transformer configs the rebuild targets. Q/K/V projections are one fused [nIn, 3d] GEMM on the
channels-last [mb*T, nIn] view; the attention core is ``scaled_dot_product_attention`` (flash / memory-
efficient attention kernels on ROCm), the output projection a second GEMM. Backward re-runs the cheap
projections under autograd from the saved input (activation recomputation instead of storing Q/K/V).
Feature masks [mb, T] mask padded keys; masked query rows are zeroed.
"""
import torch
import torch.nn.functional as F

from .base import LayerImpl


class SelfAttentionLayerImpl(LayerImpl):
    def _fwd(self, x, mask, p):
        c = self.conf
        mb, nIn, T = x.shape
        hs = c.headSize or (c.nOut // c.nHeads)
        H = c.nHeads
        xt = x.permute(0, 2, 1)                                   # [mb, T, nIn]
        w = torch.cat([p["Wq"], p["Wk"], p["Wv"]], dim=1)        # one fused projection GEMM
        b = torch.cat([p["bq"], p["bk"], p["bv"]], dim=1).reshape(-1)
        qkv = torch.addmm(b, xt.reshape(-1, nIn), w).reshape(mb, T, 3, H, hs)
        q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)           # [mb, H, T, hs]
        attn_mask = None
        if mask is not None:
            attn_mask = (mask.to(torch.bool)).reshape(mb, 1, 1, T)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask, is_causal=bool(c.causal) and mask is None)
        o = o.permute(0, 2, 1, 3).reshape(mb * T, H * hs)
        y = torch.addmm(p["bo"].reshape(-1), o, p["Wo"]).reshape(mb, T, -1)
        if mask is not None:
            y = y * mask.to(y.dtype).reshape(mb, T, 1)
        return y.permute(0, 2, 1)

    def _p(self, dtype, grad=False):
        out = {}
        for k, v in self.params.items():
            t = v.detach().to(dtype)
            out[k] = t.requires_grad_(grad)
        return out

    def activate(self, x, training=False, mask=None, **kw):
        self.input = x
        self.maskArray = mask
        with torch.no_grad():
            y = self._fwd(x, mask, self._p(x.dtype))
        return self.conf.activation.getActivation(y, training) if self.conf.activation is not None else y

    def backpropGradient(self, eps, **kw):
        x = self.input.detach().requires_grad_(True)
        p = self._p(x.dtype, True)
        with torch.enable_grad():
            y = self._fwd(x, self.maskArray, p)
            if self.conf.activation is not None:
                y = self.conf.activation.getActivation(y, True)
            keys = list(p)
            grads = torch.autograd.grad(y, [x] + [p[k] for k in keys], eps.to(y.dtype))
        for k, g in zip(keys, grads[1:]):
            self.grads[k].copy_(g.reshape(self.grads[k].shape))
        return self.make_gradient(), grads[0]
