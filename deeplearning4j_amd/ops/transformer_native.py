"""ctypes wrappers of the transformer kernels: flash-style attention (csrc/attention.hip) and LayerNorm with fused
residual add (csrc/layernorm.hip). Each returns ``None`` when the shape/dtype is outside the kernel so callers can
use the reference path; on a GPU box with the library missing, ``ops.use_native`` raises instead."""
import torch

from . import native
from .native import _check, _ptr, _stream, c_float, c_int, c_ll, c_void_p

_SIGS = {
    "dl4j_attn_fwd_dt": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_int,
                         c_void_p],
    "dl4j_attn_bwd_dt": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                         c_int, c_int, c_float, c_int, c_void_p],
    "dl4j_ln_fwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_float,
                    c_void_p],
    "dl4j_ln_bwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                    c_void_p, c_void_p, c_ll, c_int, c_void_p],
    "dl4j_ln_partial_rows": [c_ll],
}


def _lib():
    lib = native.load()
    for k, v in _SIGS.items():
        native.register_sig(k, v)
    lib.dl4j_ln_partial_rows.restype = c_ll
    return lib


# ------------------------------------------------------------------------------------------------ attention
def attn_supported(qkv, H):
    if not (qkv.is_cuda and qkv.dtype in (torch.bfloat16, torch.float16) and qkv.dim() == 3 and qkv.is_contiguous()):
        return False
    E3 = qkv.shape[2]
    if E3 % (3 * H):
        return False
    return (E3 // (3 * H)) in (64, 128)


def attn_fwd(qkv, H, mask=None, causal=False, scale=None):
    """qkv [B, T, 3E] bf16/fp16 contiguous -> (out [B, T, E] same dtype, lse [B, H, T] fp32)."""
    B, T, E3 = qkv.shape
    D = E3 // (3 * H)
    scale = float(scale if scale is not None else D ** -0.5)
    out = torch.empty(B, T, E3 // 3, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(B, H, T, device=qkv.device, dtype=torch.float32)
    m = None if mask is None else mask.reshape(B, T).to(torch.float32).contiguous()
    rc = _lib().dl4j_attn_fwd_dt(_dt(qkv), _ptr(qkv), _ptr(m), _ptr(out), _ptr(lse), B, T, H, D, scale,
                                 int(bool(causal)), c_void_p(_stream()))
    if rc == -1:
        return None
    _check(rc, "attn_fwd")
    return out, lse


def attn_bwd(qkv, out, lse, dout, H, mask=None, causal=False, scale=None):
    """Returns dqkv [B, T, 3E] in qkv's dtype (dQ, dK, dV in the fused projection layout)."""
    B, T, E3 = qkv.shape
    D = E3 // (3 * H)
    scale = float(scale if scale is not None else D ** -0.5)
    dout = dout.to(qkv.dtype).contiguous()
    dqkv = torch.empty_like(qkv)
    ws = torch.empty(B, H, T, device=qkv.device, dtype=torch.float32)
    m = None if mask is None else mask.reshape(B, T).to(torch.float32).contiguous()
    rc = _lib().dl4j_attn_bwd_dt(_dt(qkv), _ptr(qkv), _ptr(out), _ptr(dout), _ptr(m), _ptr(lse), _ptr(ws), _ptr(dqkv),
                                 B, T, H, D, scale, int(bool(causal)), c_void_p(_stream()))
    if rc == -1:
        return None
    _check(rc, "attn_bwd")
    return dqkv


class FlashAttention(torch.autograd.Function):
    """Autograd wrapper (used when the transformer block runs under autograd, e.g. SameDiff graphs)."""

    @staticmethod
    def forward(ctx, qkv, H, mask, causal):
        out, lse = attn_fwd(qkv, H, mask, causal)
        ctx.save_for_backward(qkv, out, lse, mask if mask is not None else torch.empty(0))
        ctx.H, ctx.causal, ctx.has_mask = H, causal, mask is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, mask = ctx.saved_tensors
        dqkv = attn_bwd(qkv, out, lse, dout, ctx.H, mask if ctx.has_mask else None, ctx.causal)
        return dqkv, None, None, None


def attention_reference(qkv, H, mask=None, causal=False, scale=None):
    """Plain-torch fp32 attention on the same layout (the numerics oracle)."""
    B, T, E3 = qkv.shape
    E = E3 // 3
    D = E // H
    scale = scale if scale is not None else D ** -0.5
    cd = torch.float64 if qkv.dtype == torch.float64 else torch.float32
    q, k, v = qkv.to(cd).reshape(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
    s = (q @ k.transpose(-1, -2)) * scale
    keep = torch.ones(B, 1, T, T, dtype=torch.bool, device=qkv.device)
    if mask is not None:
        keep = keep & (mask.reshape(B, 1, 1, T) != 0)
    if causal:
        keep = keep & torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril().reshape(1, 1, T, T)
    s = s.masked_fill(~keep, float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)
    o = p @ v
    return o.permute(0, 2, 1, 3).reshape(B, T, E)


def attention_fwd_explicit(qkv, H, mask=None, causal=False, scale=None):
    """Attention core with an explicitly derived backward (no torch.autograd): the path for shapes / dtypes outside
    the flash kernel (CPU, fp32 / fp64, head sizes other than 64 / 128). qkv [B, T, 3E] in the fused projection
    layout. Returns (out [B, T, E] in qkv's dtype, ctx) for attention_bwd_explicit; ctx keeps the probabilities
    P [B, H, T, T] (fp32, or fp64 for fp64 inputs)."""
    B, T, E3 = qkv.shape
    E = E3 // 3
    D = E // H
    scale = float(scale if scale is not None else D ** -0.5)
    cd = torch.float64 if qkv.dtype == torch.float64 else torch.float32
    q, k, v = qkv.to(cd).reshape(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)      # [B, H, T, D]
    s = (q @ k.transpose(-1, -2)) * scale
    keep = None
    if mask is not None:
        keep = (mask.reshape(B, 1, 1, T) != 0)
    if causal:
        tri = torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril().reshape(1, 1, T, T)
        keep = tri if keep is None else (keep & tri)
    if keep is not None:
        s = s.masked_fill(~keep, float("-inf"))
    p = torch.softmax(s, dim=-1).nan_to_num(0.0)          # fully masked rows: zero output
    o = p @ v
    out = o.permute(0, 2, 1, 3).reshape(B, T, E).to(qkv.dtype)
    return out, (q, k, v, p, scale)


def attention_bwd_explicit(ctx, dout, qkv_dtype):
    """dqkv [B, T, 3E] for attention_fwd_explicit:  dV = P^T dO,  dP = dO V^T,  dS = P * (dP - rowsum(dP * P)),
    dQ = scale dS K,  dK = scale dS^T Q."""
    q, k, v, p, scale = ctx
    B, H, T, D = q.shape
    do = dout.to(q.dtype).reshape(B, T, H, D).permute(0, 2, 1, 3)
    dv = p.transpose(-1, -2) @ do
    dp = do @ v.transpose(-1, -2)
    ds = p * (dp - (dp * p).sum(-1, keepdim=True))
    dq = (ds @ k) * scale
    dk = (ds.transpose(-1, -2) @ q) * scale
    dqkv = torch.stack([dq, dk, dv], 0).permute(1, 3, 0, 2, 4).reshape(B, T, 3 * H * D)
    return dqkv.to(qkv_dtype)


# ------------------------------------------------------------------------------------------------ layernorm
def _dt(t):
    return {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}.get(t.dtype)


def ln_supported(x, N):
    return x.is_cuda and _dt(x) is not None and x.is_contiguous() and N % 8 == 0 and N <= 4096


def ln_fwd(x, gamma, beta, eps, residual=None):
    """x (+ residual) [M, N] -> (y [M, N] same dtype, mean [M], rstd [M])."""
    N = x.shape[-1]
    M = x.numel() // N
    y = torch.empty_like(x)
    mean = torch.empty(M, device=x.device, dtype=torch.float32)
    rstd = torch.empty(M, device=x.device, dtype=torch.float32)
    g = gamma.reshape(-1).to(torch.float32).contiguous()
    b = beta.reshape(-1).to(torch.float32).contiguous()
    r = None if residual is None else residual.to(x.dtype).contiguous()
    rc = _lib().dl4j_ln_fwd(_dt(x), _ptr(x), _ptr(r), _ptr(g), _ptr(b), _ptr(y), _ptr(mean), _ptr(rstd), M, N,
                            float(eps), c_void_p(_stream()))
    if rc == -1:
        return None
    _check(rc, "ln_fwd")
    return y, mean, rstd


def ln_bwd(dy, x, gamma, mean, rstd, residual=None, dgamma_out=None, dbeta_out=None, dsum_out=None):
    """-> (dx [M, N] (also the residual's gradient), dgamma [N] fp32, dbeta [N] fp32). ``dgamma_out`` /
    ``dbeta_out``: contiguous fp32 views (e.g. the flat gradient) the kernel writes directly. ``dsum_out``: optional
    contiguous fp32 [N] view receiving the column sums of dx (the producing dense layer's bias gradient)."""
    N = x.shape[-1]
    M = x.numel() // N
    lib = _lib()
    P = lib.dl4j_ln_partial_rows(M)
    part = torch.empty(P * 3 * N, device=x.device, dtype=torch.float32)
    dx = torch.empty_like(x)
    ok = lambda t: t is not None and t.is_contiguous() and t.dtype == torch.float32 and t.numel() == N  # noqa: E731
    dg = dgamma_out.view(-1) if ok(dgamma_out) else torch.empty(N, device=x.device, dtype=torch.float32)
    db = dbeta_out.view(-1) if ok(dbeta_out) else torch.empty(N, device=x.device, dtype=torch.float32)
    g = gamma.reshape(-1).to(torch.float32).contiguous()
    r = None if residual is None else residual.to(x.dtype).contiguous()
    rc = lib.dl4j_ln_bwd(_dt(x), _ptr(dy.to(x.dtype).contiguous()), _ptr(x), _ptr(r), _ptr(g), _ptr(mean), _ptr(rstd),
                         _ptr(dx), _ptr(part), _ptr(dg), _ptr(db), _ptr(dsum_out), M, N, c_void_p(_stream()))
    if rc == -1:
        return None
    _check(rc, "ln_bwd")
    return dx, dg, db



# ------------------------------------------------------------------------------------------------ GELU
def gelu(z, dy=None):
    """Exact GELU (dy None) or its backward dy * gelu'(z) on the fused HIP kernel; None if unsupported."""
    native.register_sig("dl4j_gelu", [c_int, c_void_p, c_void_p, c_void_p, c_ll, c_void_p])
    d = _dt(z)
    if d is None or not z.is_contiguous() or (dy is not None and (dy.dtype != z.dtype or not dy.is_contiguous())):
        return None
    out = torch.empty_like(z)
    rc = native.load().dl4j_gelu(d, _ptr(z), _ptr(dy), _ptr(out), z.numel(), c_void_p(_stream()))
    if rc == -1:
        return None
    _check(rc, "gelu")
    return out
