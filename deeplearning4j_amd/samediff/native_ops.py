"""Autograd wrappers that route SameDiff-lite ops through the framework's HIP kernels on the GPU:
the whole-sequence LSTM (csrc/lstm.hip), flash-style self attention (csrc/attention.hip) and LayerNorm
(csrc/layernorm.hip). On CPU tensors (or shapes the kernels do not cover) the same ops run as differentiable
torch reference code, so graphs are portable and the GPU path can be checked against the CPU one.
"""
import torch
import torch.nn.functional as F

from .. import ops


# ------------------------------------------------------------------------------------------------ LSTM
class _LSTMSeq(torch.autograd.Function):
    """zx [T, mb, 4H] (= x·W + b, compute dtype), RW [H, 4H(+3)] -> h for all steps [T, mb, H] fp32."""

    @staticmethod
    def forward(ctx, zx, RW, h0, c0, H, peephole):
        from ..ops import rnn_native
        r = rnn_native.lstm_seq_fwd(zx.detach(), RW.detach(), H, peephole, h0, c0, None, True)
        out, hT, cT, gates, call = r
        ctx.save_for_backward(RW, out, gates, call, h0 if h0 is not None else torch.empty(0),
                              c0 if c0 is not None else torch.empty(0))
        ctx.H, ctx.peephole, ctx.has_h0, ctx.has_c0 = H, peephole, h0 is not None, c0 is not None
        ctx.zx_dtype = zx.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..ops import rnn_native
        RW, out, gates, call, h0, c0 = ctx.saved_tensors
        H = ctx.H
        T, mb, _ = out.shape
        c0v = c0 if ctx.has_c0 else None
        dz, dh0, dc0 = rnn_native.lstm_seq_bwd(dout, gates, call, c0v, RW, H, ctx.peephole)
        h0f = h0.float().reshape(1, mb, H) if ctx.has_h0 else torch.zeros(1, mb, H, device=out.device)
        hprev = torch.cat([h0f, out[:-1]], 0).reshape(T * mb, H)
        dzf = dz.reshape(T * mb, 4 * H)
        dRW = hprev.t() @ dzf
        if ctx.peephole:
            c0f = c0.float().reshape(1, mb, H) if ctx.has_c0 else torch.zeros(1, mb, H, device=out.device)
            cprev = torch.cat([c0f, call[:-1]], 0)
            dzf_, dzo_, dzg_ = dz[:, :, H:2 * H], dz[:, :, 2 * H:3 * H], dz[:, :, 3 * H:]
            dRW = torch.cat([dRW, (dzf_ * cprev).sum((0, 1)).reshape(-1, 1), (dzo_ * call).sum((0, 1)).reshape(-1, 1),
                             (dzg_ * cprev).sum((0, 1)).reshape(-1, 1)], dim=1)
        return (dz.to(ctx.zx_dtype), dRW.to(RW.dtype), dh0 if ctx.has_h0 else None, dc0 if ctx.has_c0 else None,
                None, None)


def lstm_layer(x, W, RW, b, h0=None, c0=None, peephole=False):
    """x [mb, nIn, T] -> h [mb, H, T]. DL4J gate order [a|f|o|g], tanh cell/output activation, sigmoid gates."""
    mb, nIn, T = x.shape
    H = RW.shape[0]
    dt = W.dtype
    zx = (x.permute(2, 0, 1).reshape(T * mb, nIn).to(dt) @ W + b.reshape(1, -1).to(dt)).reshape(T, mb, 4 * H)
    from ..ops import rnn_native
    if x.is_cuda and rnn_native.supported(H, dt) and ops.use_native(x, "lstm"):
        out = _LSTMSeq.apply(zx, RW, h0, c0, H, peephole)
        return out.permute(1, 2, 0).to(x.dtype)
    # differentiable reference (CPU / unsupported shapes)
    h = torch.zeros(mb, H, dtype=zx.dtype, device=x.device) if h0 is None else h0.to(zx.dtype)
    c = torch.zeros(mb, H, dtype=zx.dtype, device=x.device) if c0 is None else c0.to(zx.dtype)
    outs = []
    for t in range(T):
        z = zx[t] + h @ RW[:, :4 * H]
        za, zf, zo, zg = z[:, :H], z[:, H:2 * H], z[:, 2 * H:3 * H], z[:, 3 * H:]
        if peephole:
            zf = zf + c * RW[:, 4 * H]
            zg = zg + c * RW[:, 4 * H + 2]
        c = torch.sigmoid(zf) * c + torch.sigmoid(zg) * torch.tanh(za)
        if peephole:
            zo = zo + c * RW[:, 4 * H + 1]
        h = torch.sigmoid(zo) * torch.tanh(c)
        outs.append(h)
    return torch.stack(outs, 2)


# ------------------------------------------------------------------------------------------------ LayerNorm
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        from ..ops import transformer_native as TN
        shp = x.shape
        x2 = x.detach().reshape(-1, shp[-1]).contiguous()
        y, mean, rstd = TN.ln_fwd(x2, gamma.detach(), beta.detach(), eps)
        ctx.save_for_backward(x2, gamma, mean, rstd)
        ctx.shp = shp
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, dy):
        from ..ops import transformer_native as TN
        x2, gamma, mean, rstd = ctx.saved_tensors
        dx, dg, db = TN.ln_bwd(dy.reshape(x2.shape).contiguous(), x2, gamma, mean, rstd)
        return dx.reshape(ctx.shp), dg.to(gamma.dtype).reshape(gamma.shape), db.to(gamma.dtype).reshape(gamma.shape), \
            None


def layer_norm(x, gamma, beta, eps=1e-5):
    from ..ops import transformer_native as TN
    N = x.shape[-1]
    if gamma is not None and beta is not None and TN.ln_supported(x.contiguous(), N) and ops.use_native(x, "layernorm"):
        return _LayerNorm.apply(x.contiguous(), gamma.reshape(-1), beta.reshape(-1), eps)
    return F.layer_norm(x, (N,), gamma.reshape(-1) if gamma is not None else None,
                        beta.reshape(-1) if beta is not None else None, eps)


# ------------------------------------------------------------------------------------------------ attention
def self_attention(qkv, nHeads, mask=None, causal=False):
    """Fused-layout self attention: qkv [B, T, 3E] -> [B, T, E]."""
    from ..ops import transformer_native as TN
    if TN.attn_supported(qkv.contiguous(), nHeads) and ops.use_native(qkv, "attention"):
        return TN.FlashAttention.apply(qkv.contiguous(), nHeads, mask, causal)
    return TN.attention_reference(qkv, nHeads, mask, causal).to(qkv.dtype)
