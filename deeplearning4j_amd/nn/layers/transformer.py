"""Transformer runtime layers: BERT embeddings, post-LN encoder block, [CLS] pooler.

Not in the reference snapshot (no attention or LayerNorm there); they implement the BERT-base
config of BASELINE.json on the same layer SPI (activate / backpropGradient writing into flat gradient views).

MI355X structure of one encoder block (token-major [B*T, E] activations, bf16 compute, fp32 master weights):
  qkv = x·Wqkv + b          one fused projection GEMM (in-tree MFMA GEMM, bias in the epilogue)
  ctx = attention(qkv)      flash-style HIP kernel reading Q/K/V in place (csrc/attention.hip)
  h1  = LN(ctx·Wo + bo + x) output GEMM + LayerNorm-with-residual HIP kernel (csrc/layernorm.hip)
  h2  = LN(gelu(h1·W1 + b1)·W2 + b2 + h1)
The backward is written out by hand (no autograd): GEMMs produce fp32 weight gradients straight into the flat
gradient views, attention/LN backward are the matching HIP kernels, and the residual gradients are summed in
place. Activations cross layer boundaries as [mb, E, T] *views* of token-major memory, so stacking blocks costs
no transposes. On CPU (and fp64 gradient checks) the same math runs on plain torch ops.
"""
import math

import torch
import torch.nn.functional as F

from ... import ops
from .base import LayerImpl, copy_grad_, matmul, weight_grad_
from ...ops.gemm import mmul


def _native(x, op):
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and ops.use_native(x, op)


def _wgrad(view, a, b):
    """view <- aᵀ·b on the in-tree GEMM: fp32 accumulation written straight into the fp32 gradient view."""
    weight_grad_(view, a.t(), b)


def _bsum(view, d):
    """view <- column sums of d, accumulated in the view's precision without a converted copy of d."""
    if d.is_cuda and view.is_contiguous() and view.dtype == torch.float32 and ops.use_native(d, "bias_grad"):
        from ...ops import native
        if native.channel_sum(d.contiguous(), out=view.view(-1)) is not None:
            return
    if view.is_contiguous():
        torch.sum(d, 0, dtype=view.dtype, out=view.view(-1))
    else:
        copy_grad_(view, d.sum(0, dtype=view.dtype))


def _gelu_fwd(z):
    if _native(z, "gelu"):
        from ...ops import transformer_native as TN
        r = TN.gelu(z)
        if r is not None:
            return r
    return F.gelu(z)


def _gelu_bwd(z, dy):
    if _native(z, "gelu"):
        from ...ops import transformer_native as TN
        r = TN.gelu(z, dy.to(z.dtype).contiguous())
        if r is not None:
            return r
    zf = z.float() if z.dtype != torch.float64 else z
    cdf = 0.5 * (1.0 + torch.erf(zf * (1.0 / math.sqrt(2.0))))
    pdf = torch.exp(-0.5 * zf * zf) * (1.0 / math.sqrt(2.0 * math.pi))
    return (dy.to(zf.dtype) * (cdf + zf * pdf)).to(z.dtype)


# ------------------------------------------------------------------------------------------------ LN helpers
def _ln_fwd(x, res, g, b, eps):
    if _native(x, "layernorm"):
        from ...ops import transformer_native as TN
        r = TN.ln_fwd(x, g, b, eps, res)
        if r is not None:
            y, mean, rstd = r
            return y, ("native", mean, rstd)
    s = x if res is None else x + res
    sf = s.float() if s.dtype != torch.float64 else s
    mean = sf.mean(-1, keepdim=True)
    rstd = torch.rsqrt(sf.var(-1, unbiased=False, keepdim=True) + eps)
    xhat = (sf - mean) * rstd
    y = xhat * g.reshape(-1).to(sf.dtype) + b.reshape(-1).to(sf.dtype)
    return y.to(x.dtype), ("torch", xhat, rstd)


def _ln_bwd(dy, x, res, g, ctx, gview=None, bview=None, dsum_view=None):
    """-> ds (gradient of x and of res); dgamma / dbeta land in the gradient views. ``dsum_view``: the producing dense
    layer's bias-gradient view, filled with the column sums of ds by the LayerNorm backward kernel itself when it
    can (returns with ``dsum_view`` handled), else by _bsum."""
    if ctx[0] == "native":
        from ...ops import transformer_native as TN
        dsv = dsum_view.view(-1) if dsum_view is not None and dsum_view.is_contiguous() and \
            dsum_view.dtype == torch.float32 else None
        ds, dg, db = TN.ln_bwd(dy, x, g, ctx[1], ctx[2], res, gview, bview, dsv)
        if dg.data_ptr() != gview.data_ptr():
            copy_grad_(gview, dg)
        if db.data_ptr() != bview.data_ptr():
            copy_grad_(bview, db)
        if dsum_view is not None and dsv is None:
            _bsum(dsum_view, ds)
        return ds
    _, xhat, rstd = ctx
    d = dy.to(xhat.dtype)
    dg = (d * xhat).sum(0)
    db = d.sum(0)
    dxh = d * g.reshape(-1).to(xhat.dtype)
    ds = rstd * (dxh - dxh.mean(-1, keepdim=True) - xhat * (dxh * xhat).mean(-1, keepdim=True))
    copy_grad_(gview, dg)
    copy_grad_(bview, db)
    ds = ds.to(x.dtype)
    if dsum_view is not None:
        _bsum(dsum_view, ds)
    return ds


# ------------------------------------------------------------------------------------------------ attention
def _attn_fwd(qkv, B, T, H, mask, causal):
    from ...ops import transformer_native as TN
    if _native(qkv, "attention"):
        q3 = qkv.reshape(B, T, -1)
        if TN.attn_supported(q3, H):
            out, lse = TN.attn_fwd(q3, H, mask, causal)
            return out.reshape(B * T, -1), ("native", out, lse)
    if qkv.is_cuda:
        from ...ops import fallback
        fallback.record("attention", f"head size {qkv.shape[-1] // (3 * H)} / dtype {qkv.dtype}: explicit torch path")
    o, ctx = TN.attention_fwd_explicit(qkv.reshape(B, T, -1), H, mask, causal)
    return o.reshape(B * T, -1), ("explicit", ctx)


def _attn_bwd(dctx, qkv, B, T, H, mask, causal, ctx):
    from ...ops import transformer_native as TN
    if ctx[0] == "native":
        return TN.attn_bwd(qkv.reshape(B, T, -1), ctx[1], ctx[2], dctx.reshape(B, T, -1), H, mask,
                           causal).reshape(B * T, -1)
    return TN.attention_bwd_explicit(ctx[1], dctx.reshape(B, T, -1), qkv.dtype).reshape(B * T, -1)


def _token_major(x):
    """[mb, E, T] (possibly a permuted view of token-major memory) -> contiguous [mb*T, E] (no copy when it is)."""
    mb, E, T = x.shape
    return x.permute(0, 2, 1).reshape(mb * T, E)


class TransformerEncoderLayerImpl(LayerImpl):
    def type(self):
        return "RECURRENT"

    def activate(self, x, training=False, mask=None, **kw):
        c = self.conf
        self.training = training
        B, E, T = x.shape
        H = c.nHeads
        dt = self.W("Wqkv").dtype
        xt = _token_major(x).to(dt)
        m = mask.reshape(B, T) if mask is not None else None
        qkv = matmul(xt, self.W("Wqkv"), bias=self.Wbias("bqkv"))
        ctx, actx = _attn_fwd(qkv, B, T, H, m, c.causal)
        a = matmul(ctx, self.W("Wo"), bias=self.Wbias("bo"))
        h1, ln1 = _ln_fwd(a, xt, self.params["ln1g"], self.params["ln1b"], c.layerNormEps)
        # FFN-1 with bias + exact GELU fused into the GEMM epilogue; the pre-activation z1 is kept for backward
        z1 = torch.empty(h1.shape[0], self.W("W1").shape[1], dtype=h1.dtype, device=h1.device)
        f = matmul(h1, self.W("W1"), bias=self.Wbias("b1"), act="gelu", z=z1)
        f2 = matmul(f, self.W("W2"), bias=self.Wbias("b2"))
        y, ln2 = _ln_fwd(f2, h1, self.params["ln2g"], self.params["ln2b"], c.layerNormEps)
        self.maskArray = mask
        if training:
            self._c = (xt, qkv, actx, ctx, a, ln1, h1, z1, f, f2, ln2, B, T, m)
        self.input = x
        return y.reshape(B, T, E).permute(0, 2, 1)

    def backpropGradient(self, eps, **kw):
        c = self.conf
        xt, qkv, actx, ctx, a, ln1, h1, z1, f, f2, ln2, B, T, m = self._c
        self._c = None
        g = self.grads
        dt = xt.dtype
        dy = _token_major(eps).to(dt)
        ds2 = _ln_bwd(dy, f2, h1, self.params["ln2g"], ln2, g["ln2g"], g["ln2b"], g["b2"])   # + b2 gradient
        _wgrad(g["W2"], f, ds2)
        if _native(ds2, "gemm") and z1.dtype == ds2.dtype:
            # GELU backward in the GEMM epilogue: dz1 = (ds2 · W2ᵀ) * gelu'(z1)
            dz1 = mmul(ds2, self.W("W2").t(), act="dgelu", z=z1)
        else:
            dz1 = _gelu_bwd(z1, matmul(ds2, self.W("W2").t()))
        _wgrad(g["W1"], h1, dz1)
        _bsum(g["b1"], dz1)
        dh1 = mmul(dz1, self.W("W1").t(), out=ds2, beta=1.0)          # residual gradient summed in place
        ds1 = _ln_bwd(dh1, a, xt, self.params["ln1g"], ln1, g["ln1g"], g["ln1b"], g["bo"])   # + bo gradient
        _wgrad(g["Wo"], ctx, ds1)
        dctx = matmul(ds1, self.W("Wo").t())
        dqkv = _attn_bwd(dctx, qkv, B, T, c.nHeads, m, c.causal, actx)
        _wgrad(g["Wqkv"], xt, dqkv)
        _bsum(g["bqkv"], dqkv)
        dx = mmul(dqkv, self.W("Wqkv").t(), out=ds1, beta=1.0)
        E = dx.shape[1]
        return self.make_gradient(), dx.reshape(B, T, E).permute(0, 2, 1)


class BertEmbeddingLayerImpl(LayerImpl):
    def type(self):
        return "RECURRENT"

    def activate(self, x, training=False, mask=None, **kw):
        c = self.conf
        if x.dim() == 3:
            x = x[:, 0, :]
        idx = x.long()
        B, T = idx.shape
        dt = self.W("Wword").dtype
        from ...ops import nn_misc
        e = nn_misc.bert_embed_forward(self.W("Wword"), self.W("Wpos"), self.W("Wtype"), idx) if idx.is_cuda else None
        if e is None:
            e = self.W("Wword")[idx.reshape(-1)] + self.W("Wpos")[:T].repeat(B, 1) + self.W("Wtype")[0].reshape(1, -1)
            e = e.to(dt).contiguous()
        y, ln = _ln_fwd(e, None, self.params["lng"], self.params["lnb"], c.layerNormEps)
        if training:
            self._c = (idx, e, ln, B, T)
        return y.reshape(B, T, -1).permute(0, 2, 1)

    def backpropGradient(self, eps, **kw):
        idx, e, ln, B, T = self._c
        self._c = None
        dy = _token_major(eps).to(e.dtype)
        g = self.grads
        de = _ln_bwd(dy, e, None, self.params["lng"], ln, g["lng"], g["lnb"])
        from ...ops import nd4j_kernels as NK
        from ...ops import nn_misc
        if de.is_cuda and g["Wword"].dtype == torch.float32:
            # word rows: scatter-add of the 16-bit row gradients into the fp32 view (in-tree kernel, no fp32 copy
            # of de); position / type rows: deterministic column sums written in place
            if getattr(self.net, "_grads_zeroed", False):
                nn_misc.embedding_backward_(g["Wword"], idx, de)     # flat gradient already cleared this step
            else:
                gw = NK.zero_(torch.empty_like(g["Wword"]))
                nn_misc.embedding_backward_(gw, idx, de)
                copy_grad_(g["Wword"], gw)
            if nn_misc.bert_embed_backward_pt(de.contiguous(), g["Wpos"], g["Wtype"], B, T):
                return self.make_gradient(), None
        de = de.to(g["Wword"].dtype)
        if getattr(self.net, "_grads_zeroed", False) and g["Wword"].is_contiguous():
            g["Wword"].index_add_(0, idx.reshape(-1), de)          # flat gradient already cleared this step
        else:
            gw = torch.zeros_like(g["Wword"])
            gw.index_add_(0, idx.reshape(-1), de)
            copy_grad_(g["Wword"], gw)
        copy_grad_(g["Wpos"][:T], de.reshape(B, T, -1).sum(0).to(g["Wpos"].dtype))
        if g["Wpos"].shape[0] > T:
            g["Wpos"][T:].zero_()
        gt = torch.zeros_like(g["Wtype"])
        gt[0] = de.sum(0)
        copy_grad_(g["Wtype"], gt)
        return self.make_gradient(), None

    def feedForwardMaskArray(self, mask, state, mb):
        self.maskArray = mask
        return mask, state


class BertPoolerLayerImpl(LayerImpl):
    def activate(self, x, training=False, mask=None, **kw):
        from ...ops import nd4j_kernels as NK
        self.input = x
        x0 = x[:, :, 0].to(self.W("W").dtype)
        if training and x0.is_cuda:
            # keep the pre-activation: backward is eps * tanh'(z) on the in-tree derivative kernel (the GEMM
            # epilogue stores a pre-activation for GELU only)
            z = matmul(x0, self.W("W"), bias=self.Wbias("b"))
            y = NK.transform(z, "tanh")
            if y is not None:
                self._c = (x0, z, None, x.shape)
                return y
            y = torch.tanh(z)
        else:
            y = matmul(x0, self.W("W"), bias=self.Wbias("b"), act="tanh")
        if training:
            self._c = (x0, None, y, x.shape)
        return y

    def backpropGradient(self, eps, **kw):
        from ...ops import nd4j_kernels as NK
        x0, z, y, shape = self._c
        self._c = None
        dz = NK.transform_bp(z, eps.to(z.dtype), "tanh") if z is not None else None
        if dz is None:
            y = torch.tanh(z) if y is None else y
            dz = eps.to(y.dtype) * (1 - y * y)
        _wgrad(self.grads["W"], x0, dz)
        _bsum(self.grads["b"], dz)
        B, E, T = shape
        if x0.is_cuda:
            # token-major [B, T, E] storage returned as a [B, E, T] view, so the encoder below reads it without a
            # transposing copy; only token 0 receives a gradient
            dxt = NK.zero_(torch.empty((B, T, E), dtype=x0.dtype, device=x0.device))
            mmul(dz, self.W("W").t(), out=dxt[:, 0, :])
            return self.make_gradient(), dxt.permute(0, 2, 1)
        dx = torch.zeros(shape, dtype=x0.dtype, device=x0.device)
        dx[:, :, 0] = matmul(dz, self.W("W").t())
        return self.make_gradient(), dx

    def feedForwardMaskArray(self, mask, state, mb):
        return None, state
