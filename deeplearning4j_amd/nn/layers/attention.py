"""Multi-head self-attention over recurrent-format activations [mb, nIn, T].

Not in the reference snapshot (no attention/LayerNorm layers exist there); added for the
transformer configs the rebuild targets. Everything runs on the in-tree kernels with a
hand-derived backward (no torch.autograd):

  forward   X = x^T [mb*T, nIn];  QKV = X [Wq|Wk|Wv] + [bq|bk|bv]  (three GEMMs writing the column blocks of one
            [mb*T, 3d] buffer, bias in the epilogue);  O = attention(QKV)  (flash kernel csrc/attention.hip for
            bf16 / fp16 with head size 64 / 128, else the explicit reference, counted as a fallback on the GPU);
            Y = O Wo + bo;  masked query rows zeroed;  y = act(Y^T)
  backward  dY = act'(.) eps (masked rows zeroed);  dWo = O^T dY, dbo = colsum(dY);  dO = dY Wo^T;
            dQKV = attention_bwd(dO) (flash backward kernel, or P-based explicit backward);
            dW{q,k,v} = X^T dQ/dK/dV, db{q,k,v} = colsums;  dX = dQ Wq^T + dK Wk^T + dV Wv^T (beta-accumulated GEMMs)
Feature masks [mb, T] mask padded keys; masked query rows produce zeros.
"""
import torch

from .base import LayerImpl, bias_grad_, matmul, weight_grad_
from ...ops.gemm import mmul


class SelfAttentionLayerImpl(LayerImpl):
    def type(self):
        return "RECURRENT"

    def _dims(self):
        c = self.conf
        hs = c.headSize or (c.nOut // c.nHeads)
        return c.nHeads, hs, c.nHeads * hs

    def _attn_fwd(self, qkv, mb, T, H, mask):
        from ...ops import transformer_native as TN
        from ...ops import use_native
        q3 = qkv.reshape(mb, T, -1)
        if q3.is_cuda and q3.dtype in (torch.bfloat16, torch.float16) and use_native(q3, "attention") \
                and TN.attn_supported(q3, H):
            out, lse = TN.attn_fwd(q3, H, mask, bool(self.conf.causal))
            return out, ("native", out, lse)
        if q3.is_cuda:
            from ...ops import fallback
            fallback.record("attention", f"SelfAttentionLayer head size {q3.shape[-1] // (3 * H)} / {q3.dtype}")
        out, ctx = TN.attention_fwd_explicit(q3, H, mask, bool(self.conf.causal))
        return out, ("explicit", ctx)

    def _attn_bwd(self, qkv, do, mb, T, H, mask, ctx):
        from ...ops import transformer_native as TN
        if ctx[0] == "native":
            return TN.attn_bwd(qkv.reshape(mb, T, -1), ctx[1], ctx[2], do.reshape(mb, T, -1), H, mask,
                               bool(self.conf.causal))
        return TN.attention_bwd_explicit(ctx[1], do.reshape(mb, T, -1), qkv.dtype)

    def activate(self, x, training=False, mask=None, **kw):
        self.training = training
        mb, nIn, T = x.shape
        H, hs, d = self._dims()
        dt = self.W("Wq").dtype
        X = x.permute(0, 2, 1).reshape(mb * T, nIn).to(dt).contiguous()
        qkv = torch.empty(mb * T, 3 * d, dtype=dt, device=x.device)
        for i, (wk, bk) in enumerate((("Wq", "bq"), ("Wk", "bk"), ("Wv", "bv"))):
            mmul(X, self.W(wk), out=qkv[:, i * d:(i + 1) * d], bias=self.Wbias(bk).reshape(-1))
        m = mask.reshape(mb, T) if mask is not None else None
        o, actx = self._attn_fwd(qkv, mb, T, H, m)
        o2 = o.reshape(mb * T, d)
        Y = matmul(o2, self.W("Wo"), bias=self.Wbias("bo"))
        if m is not None:
            Y = Y * m.reshape(mb * T, 1).to(Y.dtype)
        z = Y.reshape(mb, T, -1).permute(0, 2, 1)
        self.input = x
        self.maskArray = mask
        if training:
            self._c = (X, qkv, actx, o2, m, mb, T)
        self._z = z
        return self.conf.activation.getActivation(z, training) if self.conf.activation is not None else z

    def backpropGradient(self, eps, **kw):
        X, qkv, actx, o2, m, mb, T = self._c
        H, hs, d = self._dims()
        dz = self.conf.activation.backprop(self._z, eps.to(self._z.dtype)) if self.conf.activation is not None \
            else eps
        dt = X.dtype
        dY = dz.permute(0, 2, 1).reshape(mb * T, -1).to(dt)
        if m is not None:
            dY = dY * m.reshape(mb * T, 1).to(dt)
        dY = dY.contiguous()
        weight_grad_(self.grads["Wo"], o2.t(), dY)
        bias_grad_(self.grads["bo"], dY)
        dO = matmul(dY, self.W("Wo").t())
        dqkv = self._attn_bwd(qkv, dO, mb, T, H, m, actx).reshape(mb * T, 3 * d)
        if not dqkv.is_contiguous():
            dqkv = dqkv.contiguous()
        Xt = X.t()
        dX = None
        for i, (wk, bk) in enumerate((("Wq", "bq"), ("Wk", "bk"), ("Wv", "bv"))):
            g = dqkv[:, i * d:(i + 1) * d]
            weight_grad_(self.grads[wk], Xt, g)
            bias_grad_(self.grads[bk], g.contiguous() if g.is_cuda else g)
            if dX is None:
                dX = mmul(g, self.W(wk).t())
            else:
                mmul(g, self.W(wk).t(), out=dX, beta=1.0)
        self._c = None
        eps_prev = dX.reshape(mb, T, -1).permute(0, 2, 1)
        return self.make_gradient(), eps_prev
