"""SameDiff op registry with explicit reverse-mode derivatives (the reference's DifferentialFunction.doDiff contract,
NN:nn/layers/samediff/SameDiffLayer.java:58-87,195-215 execAndEndResult / execBackwards).

Every op is a pair of plain functions on device tensors — ``forward(inputs, attrs) -> (output, ctx)`` and
``backward(ctx, grad_out, inputs, attrs) -> [grad per input or None]`` — registered under a stable name, so a graph
is data (op name + input variable names + JSON attributes): it can be re-executed for new placeholder values,
differentiated without torch.autograd, and saved / loaded. The heavy ops dispatch to the framework's kernels in both
directions: ``mmul``/``linear`` -> in-tree MFMA GEMM (ops/gemm.py), ``conv2d`` -> implicit-GEMM conv kernels
(ops/conv.py), pooling, ``layerNorm`` / ``fusedSelfAttention`` -> LayerNorm / flash-attention HIP kernels,
``lstmLayer`` -> whole-sequence LSTM HIP kernels, ``softmaxCrossEntropy`` -> fused softmax-xent kernel. On CPU
tensors (and fp64 gradient checks) the same ops run their torch reference math.
"""
import math
import threading

import torch
import torch.nn.functional as F

from .. import ops

REGISTRY = {}
_TLS = threading.local()


def set_sinks(sinks, done=None, dsum=None, nograd=None, acc=None):
    """Gradient destinations of the op whose backward runs next: {input position: contiguous fp32 tensor shaped like
    that input} (SameDiff._backward sets them for variables only this op reads). ``done``: input positions whose
    sink an earlier backward already filled; ``dsum``: an fp32 sink for the column sums of this LayerNorm's input
    gradient (the producing linear's bias gradient). ``acc``: {input position: the partial gradient other consumers
    already produced} that the backward may accumulate into in place (then it reports it with ``acc_used``)."""
    _TLS.sinks = sinks
    _TLS.done = done
    _TLS.dsum = dsum
    _TLS.dsum_written = False
    _TLS.nograd = nograd
    _TLS.acc = acc
    _TLS.acc_used = set()


def acc_target(i):
    """The partial gradient of input ``i`` this backward may add its contribution into (in place), or None."""
    a = getattr(_TLS, "acc", None)
    return None if not a else a.get(i)


def mark_acc_used(i):
    _TLS.acc_used.add(i)


def acc_used():
    return getattr(_TLS, "acc_used", set())


def need_grad(i):
    """False when the reverse pass will discard input ``i``'s gradient (a placeholder or constant nobody asked the
    gradient of): the op may return None for it instead of computing it."""
    n = getattr(_TLS, "nograd", None)
    return not n or i not in n


def sink_done(i):
    d = getattr(_TLS, "done", None)
    return bool(d) and i in d


def dsum_written():
    return getattr(_TLS, "dsum_written", False)


def grad_sink(i):
    """The destination input ``i``'s gradient should be written to, or None (write a fresh tensor). A backward that
    uses it returns that same tensor as the gradient."""
    s = getattr(_TLS, "sinks", None)
    return None if not s else s.get(i)


def master(t):
    """The fp32 master copy of a mixed-precision trainable variable (SameDiff training keeps it in the flat parameter
    buffer, the 16-bit value is its shadow), else ``t`` itself."""
    if t is None:
        return None
    m = getattr(t, "_dl4j_master", None)
    return t if m is None else m


class OpDef:
    def __init__(self, name, fwd, bwd):
        self.name, self.fwd, self.bwd = name, fwd, bwd


def register(name):
    def deco(pair):
        fwd, bwd = pair
        REGISTRY[name] = OpDef(name, fwd, bwd)
        return pair
    return deco


def _unbroadcast(g, shape):
    """Sum a broadcast gradient back to ``shape``."""
    if g is None:
        return None
    shape = tuple(shape)
    if tuple(g.shape) == shape:
        return g
    while g.dim() > len(shape):
        g = g.sum(0)
    for i, s in enumerate(shape):
        if s == 1 and g.shape[i] != 1:
            g = g.sum(i, keepdim=True)
    return g.reshape(shape)


def _shape(x):
    return tuple(x.shape) if torch.is_tensor(x) else ()


def _g(g, x):
    """Gradient for input ``x`` (None for python scalars / non-float inputs)."""
    if not torch.is_tensor(x) or not x.is_floating_point():
        return None
    return _unbroadcast(g, x.shape).to(x.dtype)


# ----------------------------------------------------------------------------------------------- elementwise
def _binary(name, f, da, db):
    def fwd(ins, at):
        a, b = ins
        return f(a, b), None

    def bwd(ctx, g, ins, at):
        a, b = ins
        return [_g(da(g, a, b), a), _g(db(g, a, b), b)]
    register(name)((fwd, bwd))


_binary("add", lambda a, b: a + b, lambda g, a, b: g, lambda g, a, b: g)
_binary("sub", lambda a, b: a - b, lambda g, a, b: g, lambda g, a, b: -g)
_binary("mul", lambda a, b: a * b, lambda g, a, b: g * b, lambda g, a, b: g * a)
_binary("div", lambda a, b: a / b, lambda g, a, b: g / b, lambda g, a, b: -g * a / (b * b))
_binary("rsub", lambda a, b: b - a, lambda g, a, b: -g, lambda g, a, b: g)
_binary("rdiv", lambda a, b: b / a, lambda g, a, b: -g * b / (a * a), lambda g, a, b: g / a)


def _unary(name, f, df_xy):
    """df_xy(g, x, y) -> dL/dx."""
    def fwd(ins, at):
        y = f(ins[0], at)
        return y, y

    def bwd(ctx, g, ins, at):
        return [df_xy(g, ins[0], ctx, at).to(ins[0].dtype)]
    register(name)((fwd, bwd))


_SQRT2 = math.sqrt(2.0)
_unary("neg", lambda x, a: -x, lambda g, x, y, a: -g)
_unary("identity", lambda x, a: x, lambda g, x, y, a: g)
_unary("exp", lambda x, a: torch.exp(x), lambda g, x, y, a: g * y)
_unary("log", lambda x, a: torch.log(x), lambda g, x, y, a: g / x)
_unary("sqrt", lambda x, a: torch.sqrt(x), lambda g, x, y, a: g / (2 * y))
_unary("square", lambda x, a: x * x, lambda g, x, y, a: 2 * g * x)
_unary("abs", lambda x, a: torch.abs(x), lambda g, x, y, a: g * torch.sign(x))
_unary("pow", lambda x, a: x ** a["p"], lambda g, x, y, a: g * a["p"] * x ** (a["p"] - 1))
_unary("relu", lambda x, a: torch.relu(x), lambda g, x, y, a: g * (x > 0).to(g.dtype))
_unary("sigmoid", lambda x, a: torch.sigmoid(x), lambda g, x, y, a: g * y * (1 - y))
_unary("tanh", lambda x, a: torch.tanh(x), lambda g, x, y, a: g * (1 - y * y))
_unary("softplus", lambda x, a: F.softplus(x), lambda g, x, y, a: g * torch.sigmoid(x))
_unary("elu", lambda x, a: F.elu(x), lambda g, x, y, a: g * torch.where(x > 0, torch.ones_like(x), y + 1))
_unary("leakyRelu", lambda x, a: F.leaky_relu(x, a.get("alpha", 0.01)),
       lambda g, x, y, a: g * torch.where(x > 0, torch.ones_like(x), torch.full_like(x, a.get("alpha", 0.01))))
def _gelu(z, dy=None):
    """Exact GELU or its backward on the fused HIP kernel (GPU bf16/fp32), torch reference otherwise."""
    if z.is_cuda and ops.use_native(z, "gelu"):
        from ..ops import transformer_native as TN
        r = TN.gelu(z.contiguous(), None if dy is None else dy.to(z.dtype).contiguous())
        if r is not None:
            return r
    if dy is None:
        return 0.5 * z * (1 + torch.erf(z / _SQRT2))
    return (dy * (0.5 * (1 + torch.erf(z / _SQRT2)) + z * torch.exp(-0.5 * z * z) / math.sqrt(2 * math.pi))).to(z.dtype)


register("gelu")((lambda ins, at: (_gelu(ins[0]), None), lambda ctx, g, ins, at: [_gelu(ins[0], g)]))
_unary("softmax", lambda x, a: torch.softmax(x, dim=-1),
       lambda g, x, y, a: y * (g - (g * y).sum(-1, keepdim=True)))


# activation by DL4J IActivation (forward getActivation, backward IActivation.backprop)
def _act_obj(at):
    from ..nn.conf.activations import to_activation
    from ..nn.conf.base import _decode
    a = at["act"]
    return to_activation(_decode(a) if isinstance(a, dict) else a)


def _act_fwd(ins, at):
    return _act_obj(at).getActivation(ins[0], True), None


def _act_bwd(ctx, g, ins, at):
    return [_act_obj(at).backprop(ins[0], g).to(ins[0].dtype)]


register("activation")((_act_fwd, _act_bwd))


# ----------------------------------------------------------------------------------------------- linear algebra
def _mm(a, b, out_dtype=None):
    from ..ops.gemm import bias_vec, mmul
    if a.dim() <= 3 and b.dim() <= 3 and a.dim() >= 2 and b.dim() >= 2:
        return mmul(a, b, out_dtype=out_dtype)
    return torch.matmul(a, b)


def _mmul_fwd(ins, at):
    a, b = ins
    return _mm(a, b), None


def _mmul_bwd(ctx, g, ins, at):
    a, b = ins
    g = g.to(a.dtype)
    da = _mm(g, b.transpose(-1, -2))
    db = _mm(a.transpose(-1, -2), g)
    return [_unbroadcast(da, a.shape), _unbroadcast(db, b.shape)]


register("mmul")((_mmul_fwd, _mmul_bwd))


def _param_acc(w):
    return torch.float64 if w.dtype == torch.float64 else torch.float32


def _colsum(g2, out=None):
    """fp32 column sums of a [M, N] gradient (channel-sum HIP kernel on the GPU); ``out``: optional fp32 sink."""
    if g2.is_cuda and g2.dtype in (torch.bfloat16, torch.float16, torch.float32) and g2.shape[1] % 8 == 0:
        from ..ops import native
        r = native.channel_sum(g2.contiguous(), out=None if out is None else out.view(-1))
        if r is not None:
            return r
    r = g2.to(_param_acc(g2)).sum(0)
    return r if out is None else out.view(-1).copy_(r)


def _linear_fwd(ins, at):
    """y = act(x . w + b); attr ``act`` ("gelu", set by SameDiff's fusion pass for linear -> gelu) runs the
    activation in the GEMM epilogue and keeps the pre-activation for the backward."""
    x, w, b = ins
    from ..ops.gemm import bias_vec, mmul
    bias = None if b is None else bias_vec(master(b))
    act = at.get("act")
    lead = x.shape[:-1]
    if x.dim() > 2 and w.dim() == 2:
        # [.., K] activations as one [rows, K] GEMM (not a batched one: a plain 2-D product can also take the library
        # candidate, and one launch covers every row)
        x = x.reshape(-1, x.shape[-1])
    if act is None:
        return mmul(x, w, bias=bias).reshape(lead + (w.shape[-1],)), None
    if x.is_cuda:
        z = torch.empty(x.shape[:-1] + (w.shape[1],), dtype=x.dtype, device=x.device)
        y = mmul(x, w, bias=bias, act=act, z=z)
        return y.reshape(lead + (w.shape[-1],)), z.reshape(lead + (w.shape[-1],))
    z = mmul(x, w, bias=bias)
    return _gelu(z).reshape(lead + (w.shape[-1],)), z.reshape(lead + (w.shape[-1],))


def _linear_bwd(ctx, g, ins, at):
    x, w, b = ins
    if at.get("act") is not None:
        g = _gelu(ctx, g.to(ctx.dtype))
    g2 = g.to(x.dtype).reshape(-1, g.shape[-1])
    x2 = x.reshape(-1, x.shape[-1])
    acc = acc_target(0)
    if acc is not None and acc.dtype == x.dtype and acc.shape == x.shape and acc.is_contiguous() and x.is_cuda:
        # the residual branch's gradient is already there: dx summed into it by the GEMM (beta = 1), no add launch
        from ..ops.gemm import mmul
        mmul(g2, w.t(), out=acc.view(-1, acc.shape[-1]), beta=1.0)
        mark_acc_used(0)
        dx = acc
    else:
        dx = _mm(g2, w.t()).reshape(x.shape)
    sw, sb = grad_sink(1), grad_sink(2)
    if sw is not None and x.is_cuda and w.dim() == 2:
        from ..ops.gemm import mmul
        dw = mmul(x2.t(), g2, out=sw)                  # straight into the flat gradient (fp32 epilogue)
    else:
        dw = _mm(x2.t(), g2, out_dtype=None if w.dtype == torch.float64 else torch.float32)
    if b is None:
        db = None
    elif sb is not None and sink_done(2):
        db = sb.reshape(b.shape)                      # written by the consuming LayerNorm's backward (dsum)
    else:
        db = _colsum(g2, sb).reshape(b.shape)
    return [dx, dw, db]


register("linear")((_linear_fwd, _linear_bwd))


# ----------------------------------------------------------------------------------------------- shape / reduce
def _dims(at, x):
    d = at.get("dims") or []
    return tuple(d) if d else tuple(range(x.dim()))


register("sum")((lambda ins, at: (ins[0].sum(dim=_dims(at, ins[0])), None),
                 lambda ctx, g, ins, at: [_expand_back(g, ins[0], _dims(at, ins[0]))]))
register("mean")((lambda ins, at: (ins[0].mean(dim=_dims(at, ins[0])), None),
                  lambda ctx, g, ins, at: [_expand_back(g, ins[0], _dims(at, ins[0])) /
                                           math.prod(ins[0].shape[d] for d in _dims(at, ins[0]))]))


def _expand_back(g, x, dims):
    shp = list(x.shape)
    for d in sorted(d % x.dim() for d in dims):
        shp[d] = 1
    return g.reshape(shp).expand(x.shape).to(x.dtype)


register("reshape")((lambda ins, at: (ins[0].reshape(*at["shape"]), None),
                     lambda ctx, g, ins, at: [g.reshape(ins[0].shape)]))
register("permute")((lambda ins, at: (ins[0].permute(*at["dims"]), None),
                     lambda ctx, g, ins, at: [g.permute(*_inv_perm(at["dims"]))]))
register("transpose")((lambda ins, at: (ins[0].transpose(-1, -2), None),
                       lambda ctx, g, ins, at: [g.transpose(-1, -2)]))


def _inv_perm(p):
    inv = [0] * len(p)
    for i, d in enumerate(p):
        inv[d] = i
    return inv


def _idx(at):
    out = []
    for e in at["idx"]:
        if isinstance(e, dict) and "slice" in e:
            out.append(slice(*e["slice"]))
        elif e is None:
            out.append(None)
        else:
            out.append(e)
    return tuple(out)


def _get_bwd(ctx, g, ins, at):
    dx = torch.zeros_like(ins[0])
    dx[_idx(at)] += g.to(dx.dtype)
    return [dx]


register("get")((lambda ins, at: (ins[0][_idx(at)], None), _get_bwd))


def _concat_fwd(ins, at):
    return torch.cat(ins, dim=at["dim"]), None


def _concat_bwd(ctx, g, ins, at):
    sizes = [t.shape[at["dim"]] for t in ins]
    return list(torch.split(g, sizes, dim=at["dim"]))


register("concat")((_concat_fwd, _concat_bwd))


def _gather_fwd(ins, at):
    p, i = ins
    if at.get("axis", 0) == 0:
        if p.dim() == 2:
            from ..ops.nn_misc import embedding_forward
            return embedding_forward(p, i), None
        return p.index_select(0, i.long().reshape(-1)).reshape(tuple(i.shape) + tuple(p.shape[1:])), None
    return torch.index_select(p, at["axis"], i.long().reshape(-1)), None


def _gather_bwd(ctx, g, ins, at):
    p, i = ins
    sp = grad_sink(0)
    dp = sp.zero_() if sp is not None else torch.zeros(p.shape, dtype=_param_acc(p), device=p.device)
    ax = at.get("axis", 0)
    if ax == 0:
        from ..ops.nn_misc import embedding_backward_
        if p.dim() == 2:
            embedding_backward_(dp, i, g)
        else:
            dp.index_add_(0, i.long().reshape(-1), g.reshape(-1, *p.shape[1:]).to(dp.dtype))
    else:
        dp.index_add_(ax, i.long().reshape(-1), g.to(dp.dtype))
    return [dp, None]


register("gather")((_gather_fwd, _gather_bwd))


# ----------------------------------------------------------------------------------------------- NN blocks
def _ln_fwd(ins, at):
    """LayerNorm over the last dim of x (+ residual: the 4th input, set by SameDiff's fusion pass for
    add -> layerNorm, summed inside the LayerNorm kernel)."""
    x, gamma, beta = ins[:3]
    gamma, beta = master(gamma), master(beta)
    res = ins[3] if len(ins) > 3 else None
    eps = at.get("eps", 1e-5)
    N = x.shape[-1]
    from ..ops import transformer_native as TN
    x2 = x.reshape(-1, N).contiguous()
    if gamma is not None and beta is not None and TN.ln_supported(x2, N) and ops.use_native(x, "layernorm") and \
            (res is None or res.dtype == x.dtype):
        r2 = None if res is None else res.reshape(-1, N).contiguous()
        y, mean, rstd = TN.ln_fwd(x2, gamma.reshape(-1), beta.reshape(-1), eps, r2)
        return y.reshape(x.shape), ("native", x2, r2, mean, rstd)
    if res is not None:
        x2 = x2 + res.reshape(-1, N)
    xf = x2.float() if x.dtype != torch.float64 else x2
    mean = xf.mean(-1, keepdim=True)
    rstd = torch.rsqrt(((xf - mean) ** 2).mean(-1, keepdim=True) + eps)
    xh = (xf - mean) * rstd
    y = xh * (gamma.reshape(-1).to(xf.dtype) if gamma is not None else 1) + \
        (beta.reshape(-1).to(xf.dtype) if beta is not None else 0)
    return y.to(x.dtype).reshape(x.shape), ("ref", xh, rstd)


def _ln_bwd(ctx, g, ins, at):
    x, gamma, beta = ins[:3]
    res = ins[3] if len(ins) > 3 else None
    N = x.shape[-1]
    g2 = g.reshape(-1, N).contiguous()
    if ctx[0] == "native":
        from ..ops import transformer_native as TN
        _, x2, r2, mean, rstd = ctx
        dsum = getattr(_TLS, "dsum", None)
        dx, dg, db = TN.ln_bwd(g2.to(x.dtype), x2, master(gamma).reshape(-1), mean, rstd, r2,
                               dgamma_out=grad_sink(1), dbeta_out=grad_sink(2), dsum_out=dsum)
        if dsum is not None:
            _TLS.dsum_written = True
        dx = dx.reshape(x.shape)
        out = [dx, dg.reshape(gamma.shape), db.reshape(beta.shape)]
        return out + ([dx.to(res.dtype)] if res is not None else [])
    _, xh, rstd = ctx
    gf = g2.to(xh.dtype)
    gam = gamma.reshape(-1).to(xh.dtype) if gamma is not None else torch.ones(N, dtype=xh.dtype, device=xh.device)
    dxh = gf * gam
    dx = rstd * (dxh - dxh.mean(-1, keepdim=True) - xh * (dxh * xh).mean(-1, keepdim=True))
    dg = None if gamma is None else (gf * xh).sum(0).reshape(gamma.shape)
    db = None if beta is None else gf.sum(0).reshape(beta.shape)
    dx = dx.to(x.dtype).reshape(x.shape)
    return [dx, dg, db] + ([dx.to(res.dtype)] if res is not None else [])


register("layerNorm")((_ln_fwd, _ln_bwd))


def _attn_fwd(ins, at):
    qkv, mask = ins
    from ..ops import transformer_native as TN
    H, causal = at["nHeads"], at.get("causal", False)
    q = qkv.contiguous()
    if TN.attn_supported(q, H) and ops.use_native(qkv, "attention"):
        out, lse = TN.attn_fwd(q, H, mask, causal)
        return out, ("native", q, out, lse)
    B, T, E3 = qkv.shape
    E = E3 // 3
    D = E // H
    cd = torch.float64 if qkv.dtype == torch.float64 else torch.float32
    qq, kk, vv = qkv.to(cd).reshape(B, T, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
    s = (qq @ kk.transpose(-1, -2)) * (D ** -0.5)
    keep = torch.ones(B, 1, T, T, dtype=torch.bool, device=qkv.device)
    if mask is not None:
        keep = keep & (mask.reshape(B, 1, 1, T) != 0)
    if causal:
        keep = keep & torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril().reshape(1, 1, T, T)
    p = torch.softmax(s.masked_fill(~keep, float("-inf")), dim=-1).nan_to_num(0.0)
    o = (p @ vv).permute(0, 2, 1, 3).reshape(B, T, E)
    return o.to(qkv.dtype), ("ref", qq, kk, vv, p)


def _attn_bwd(ctx, g, ins, at):
    qkv, mask = ins
    H, causal = at["nHeads"], at.get("causal", False)
    if ctx[0] == "native":
        from ..ops import transformer_native as TN
        _, q, out, lse = ctx
        return [TN.attn_bwd(q, out, lse, g.to(q.dtype).contiguous(), H, mask, causal), None]
    _, qq, kk, vv, p = ctx
    B, T, E3 = qkv.shape
    E = E3 // 3
    D = E // H
    go = g.to(p.dtype).reshape(B, T, H, D).permute(0, 2, 1, 3)
    dv = p.transpose(-1, -2) @ go
    dp = go @ vv.transpose(-1, -2)
    ds = p * (dp - (dp * p).sum(-1, keepdim=True)) * (D ** -0.5)
    dq = ds @ kk
    dk = ds.transpose(-1, -2) @ qq
    dqkv = torch.stack([dq, dk, dv], 0).permute(1, 3, 0, 2, 4).reshape(B, T, E3)
    return [dqkv.to(qkv.dtype), None]


register("fusedSelfAttention")((_attn_fwd, _attn_bwd))


def _conv_fwd(ins, at):
    x, w, b = ins
    from ..ops.conv import conv2d_forward
    st, pd, dl = at.get("stride", [1, 1]), at.get("padding", [0, 0]), at.get("dilation", [1, 1])
    y = conv2d_forward(x, w, b.reshape(-1) if b is not None else None, st, (pd[0], pd[0], pd[1], pd[1]), dl)
    return y, None


def _conv_bwd(ctx, g, ins, at):
    x, w, b = ins
    from ..ops.conv import conv2d_backward
    st, pd, dl = at.get("stride", [1, 1]), at.get("padding", [0, 0]), at.get("dilation", [1, 1])
    gW = torch.zeros(w.shape, dtype=torch.float32 if w.dtype != torch.float64 else w.dtype, device=w.device)
    gb = None if b is None else torch.zeros(b.numel(), dtype=gW.dtype, device=w.device)
    g = g.to(x.dtype)
    if x.is_cuda and g.dim() == 4:
        g = g.contiguous(memory_format=torch.channels_last)
    dx, dw, db = conv2d_backward(x, w, g, st, (pd[0], pd[0], pd[1], pd[1]), dl, True, True, b is not None,
                                 gW=gW, gb=gb, grads_zeroed=True)
    dw = gW if dw is None else dw
    db = gb if db is None else db
    return [dx, dw.reshape(w.shape), None if b is None else db.reshape(b.shape)]


register("conv2d")((_conv_fwd, _conv_bwd))


def _pool(kind):
    def fwd(ins, at):
        from ..ops.pool import pool2d_forward
        k, s, p = at["kernel"], at["stride"], at.get("padding", [0, 0])
        y, ctx = pool2d_forward(ins[0], kind, k, s, (p[0], p[0], p[1], p[1]))
        return y, ctx

    def bwd(ctx, g, ins, at):
        from ..ops.pool import pool2d_backward
        return [pool2d_backward(g.to(ins[0].dtype), ctx)]
    return fwd, bwd


register("maxPooling2d")(_pool("MAX"))
register("avgPooling2d")(_pool("AVG"))


def _lstm_native_grads(dz, xt, out, gates, call, h0, c0, x, W, RW, b, H, peephole, base, want_dx=None):
    """[dx, dW, dRW, db] of one lstmLayer from the sequence kernel's gate deltas dz [T, mb, 4H] fp32: one glue
    launch (bf16 dz, h_{t-1}, db, peephole sums: csrc/lstm_glue.hip) and MFMA GEMMs written straight into the
    gradient sinks (input positions base+1..base+3); dx only when the input needs a gradient. None when the glue
    does not take this dtype (the caller's generic path runs)."""
    from ..ops import rnn_native
    from ..ops.gemm import bias_vec, mmul
    prep = rnn_native.lstm_bwd_prep(dz, out, h0, call, c0, peephole, W.dtype)
    if prep is None:
        return None
    T, mb = dz.shape[0], dz.shape[1]
    dzb, hpb, db, dpeep = prep
    sw, srw, sb = grad_sink(base + 1), grad_sink(base + 2), grad_sink(base + 3)
    dW = mmul(xt.t(), dzb, out=sw) if sw is not None else mmul(xt.t(), dzb, out_dtype=torch.float32)
    gRW = srw if srw is not None else torch.empty(RW.shape, dtype=torch.float32, device=dz.device)
    mmul(hpb.t(), dzb, out=gRW[:, :4 * H])
    if peephole:
        gRW[:, 4 * H:4 * H + 3].copy_(dpeep.t())
    dbv = sb.view(-1).copy_(db) if sb is not None else db
    dx = None
    if (need_grad(base) if want_dx is None else want_dx):
        dx = mmul(dzb, W.t()).reshape(T, mb, -1).permute(1, 2, 0).to(x.dtype)
    return [dx, dW, gRW, dbv.reshape(b.shape)]


def _lstm_fwd(ins, at):
    """x [mb, nIn, T] -> h [mb, H, T]; DL4J gate order [a|f|o|g], tanh/sigmoid."""
    x, W, RW, b, h0, c0 = ins
    peephole = at.get("peephole", False)
    mb, nIn, T = x.shape
    H = RW.shape[0]
    dt = W.dtype
    from ..ops.gemm import bias_vec, mmul
    from ..ops import rnn_native
    if x.is_cuda and rnn_native.supported(H, dt) and ops.use_native(x, "lstm"):
        from ..nn.layers.recurrent import _time_major_rows
        xt = _time_major_rows(x, dt)                      # one cast/permute/pad launch, a GEMM operand in place
        zx = mmul(xt, W, bias=bias_vec(master(b))).reshape(T, mb, 4 * H)
        packs = rnn_native.pack_rw(RW, H, peephole)       # both packed images in one launch, reused by backward
        out, hT, cT, gates, call, o16 = rnn_native.lstm_seq_fwd(zx, RW, H, peephole, h0, c0, None, True, packs=packs,
                                                                out16=x.dtype == dt)
        y = o16.permute(1, 2, 0) if o16 is not None else out.permute(1, 2, 0).to(x.dtype)
        return y, ("native", xt, zx, out, gates, call, packs)
    xt = x.permute(2, 0, 1).reshape(T * mb, nIn).to(dt)
    zx = mmul(xt, W, bias=b.reshape(-1)).reshape(T, mb, 4 * H)
    cd = torch.float64 if dt == torch.float64 else torch.float32
    h = torch.zeros(mb, H, dtype=cd, device=x.device) if h0 is None else h0.to(cd)
    c = torch.zeros(mb, H, dtype=cd, device=x.device) if c0 is None else c0.to(cd)
    RWc = RW.to(cd)
    hs, cs, gs = [h], [c], []
    for t in range(T):
        z = zx[t].to(cd) + h @ RWc[:, :4 * H]
        za, zf, zo, zg = z[:, :H], z[:, H:2 * H], z[:, 2 * H:3 * H], z[:, 3 * H:]
        if peephole:
            zf = zf + c * RWc[:, 4 * H]
            zg = zg + c * RWc[:, 4 * H + 2]
        a, f, gg = torch.tanh(za), torch.sigmoid(zf), torch.sigmoid(zg)
        c = f * c + gg * a
        if peephole:
            zo = zo + c * RWc[:, 4 * H + 1]
        o = torch.sigmoid(zo)
        tc = torch.tanh(c)
        h = o * tc
        hs.append(h)
        cs.append(c)
        gs.append((a, f, o, gg, tc))
    out = torch.stack(hs[1:], 2)
    return out.to(x.dtype), ("ref", xt, hs, cs, gs)


def _lstm_bwd(ctx, g, ins, at):
    x, W, RW, b, h0, c0 = ins
    peephole = at.get("peephole", False)
    mb, nIn, T = x.shape
    H = RW.shape[0]
    from ..ops.gemm import bias_vec, mmul
    if ctx[0] == "native":
        from ..ops import rnn_native
        _, xt, zx, out, gates, call, packs = ctx
        dz, dh0, dc0 = rnn_native.lstm_seq_bwd(g.permute(2, 0, 1), gates, call, c0, RW, H, peephole, packs=packs)
        r = _lstm_native_grads(dz, xt, out, gates, call, h0, c0, x, W, RW, b, H, peephole, 0)
        if r is not None:
            return r + [None if h0 is None else dh0.to(h0.dtype), None if c0 is None else dc0.to(c0.dtype)]
        h0f = h0.float().reshape(1, mb, H) if h0 is not None else torch.zeros(1, mb, H, device=x.device)
        hprev = torch.cat([h0f, out[:-1].float()], 0).reshape(T * mb, H)
        dzf = dz.reshape(T * mb, 4 * H)
        lp = RW.dtype in (torch.bfloat16, torch.float16)
        # low-precision operands with fp32 accumulation/output keep the recurrent-weight GEMM on the MFMA kernels
        dRW = mmul(hprev.to(RW.dtype).t(), dzf.to(RW.dtype), out_dtype=torch.float32) if lp else mmul(hprev.t(), dzf)
        if peephole:
            c0f = c0.float().reshape(1, mb, H) if c0 is not None else torch.zeros(1, mb, H, device=x.device)
            cprev = torch.cat([c0f, call[:-1]], 0)
            dRW = torch.cat([dRW, (dz[:, :, H:2 * H] * cprev).sum((0, 1)).reshape(-1, 1),
                             (dz[:, :, 2 * H:3 * H] * call).sum((0, 1)).reshape(-1, 1),
                             (dz[:, :, 3 * H:] * cprev).sum((0, 1)).reshape(-1, 1)], 1)
    else:
        _, xt, hs, cs, gs = ctx
        cd = hs[0].dtype
        RWc = RW.to(cd)
        go = g.to(cd)
        dh = torch.zeros(mb, H, dtype=cd, device=x.device)
        dc = torch.zeros(mb, H, dtype=cd, device=x.device)
        dzs = [None] * T
        dpeep = [torch.zeros(H, dtype=cd, device=x.device) for _ in range(3)]
        for t in reversed(range(T)):
            a, f, o, gg, tc = gs[t]
            c_prev, c_t = cs[t], cs[t + 1]
            dh = dh + go[:, :, t]
            do = dh * tc
            dzo = do * o * (1 - o)
            dc = dc + dh * o * (1 - tc * tc)
            if peephole:
                dc = dc + dzo * RWc[:, 4 * H + 1]
                dpeep[1] += (dzo * c_t).sum(0)
            dza = dc * gg * (1 - a * a)
            dzg = dc * a * gg * (1 - gg)
            dzf = dc * c_prev * f * (1 - f)
            dz = torch.cat([dza, dzf, dzo, dzg], 1)
            dzs[t] = dz
            dc = dc * f
            if peephole:
                dc = dc + dzf * RWc[:, 4 * H] + dzg * RWc[:, 4 * H + 2]
                dpeep[0] += (dzf * c_prev).sum(0)
                dpeep[2] += (dzg * c_prev).sum(0)
            dh = dz @ RWc[:, :4 * H].t()
        dz = torch.stack(dzs, 0)
        dzf = dz.reshape(T * mb, 4 * H)
        hprev = torch.stack(hs[:-1], 0).reshape(T * mb, H)
        dRW = hprev.t() @ dzf
        if peephole:
            dRW = torch.cat([dRW] + [p.reshape(-1, 1) for p in dpeep], 1)
        dh0, dc0 = dh, dc
    dzc = dzf.to(W.dtype)
    dW = mmul(xt.t(), dzc, out_dtype=torch.float32 if W.dtype != torch.float64 else None)
    db = dzf.sum(0)
    dx = mmul(dzc, W.t()).reshape(T, mb, nIn).permute(1, 2, 0)
    return [dx.to(x.dtype), dW, dRW.reshape(RW.shape), db.reshape(b.shape),
            None if h0 is None else dh0.to(h0.dtype), None if c0 is None else dc0.to(c0.dtype)]


register("lstmLayer")((_lstm_fwd, _lstm_bwd))


# two stacked lstmLayer ops (SameDiff's fusion pass: the first one's output read only by the second): ONE pipelined
# launch per direction (csrc/lstm_coop.hip lstm_fwd_stack2 / lstm_bwd_stack2, the MultiLayerNetwork stack path)
def _lstm2_fwd(ins, at):
    x, W1, RW1, b1, W2, RW2, b2 = ins
    peephole = at.get("peephole", False)
    mb, nIn, T = x.shape
    H = RW1.shape[0]
    dt = W1.dtype
    from ..ops import rnn_native
    if x.is_cuda and x.dtype == dt and ops.use_native(x, "lstm") and rnn_native.stack2_supported(H, dt, T) and \
            RW2.shape[0] == H and tuple(W2.shape) == (H, 4 * H) and W2.dtype == dt:
        from ..nn.layers.recurrent import _time_major_rows
        from ..ops.gemm import bias_vec, mmul
        xt = _time_major_rows(x, dt)
        zx1 = mmul(xt, W1, bias=bias_vec(master(b1))).reshape(T, mb, 4 * H)
        p1, p2 = rnn_native.pack_rw(RW1, H, peephole), rnn_native.pack_rw(RW2, H, peephole)
        pw = rnn_native.pack_rw(W2, H, False)
        r = None
        if p1 is not None and p2 is not None and pw is not None:
            r = rnn_native.lstm2_seq_fwd(zx1, p1, p2, pw, master(b2).reshape(-1), H, (None, None), (None, None),
                                         None, True)
        if r is not None:
            L1, L2 = r
            return L2[5].permute(1, 2, 0), ("stack", xt, L1, L2, p1, p2, pw)
    y1, c1 = _lstm_fwd([x, W1, RW1, b1, None, None], at)
    y2, c2 = _lstm_fwd([y1, W2, RW2, b2, None, None], at)
    return y2, ("pair", y1, c1, c2)


def _lstm2_bwd(ctx, g, ins, at):
    x, W1, RW1, b1, W2, RW2, b2 = ins
    peephole = at.get("peephole", False)
    H = RW1.shape[0]
    outer = (getattr(_TLS, "sinks", None), getattr(_TLS, "nograd", None))
    sk = outer[0] or {}
    if ctx[0] == "pair":
        _, y1, c1, c2 = ctx
        try:
            _TLS.sinks, _TLS.nograd = {k - 3: v for k, v in sk.items() if k >= 4}, None
            g2 = _lstm_bwd(c2, g, [y1, W2, RW2, b2, None, None], at)
            _TLS.sinks, _TLS.nograd = {k: v for k, v in sk.items() if k <= 3}, outer[1]
            g1 = _lstm_bwd(c1, g2[0], [x, W1, RW1, b1, None, None], at)
        finally:
            _TLS.sinks, _TLS.nograd = outer
        return g1[:4] + g2[1:4]
    from ..ops import rnn_native
    _, xt, L1, L2, p1, p2, pw = ctx
    T, mb = L1[0].shape[0], L1[0].shape[1]
    r = rnn_native.lstm2_seq_bwd(g.permute(2, 0, 1), {"gates": L1[3], "call": L1[4], "c0": None},
                                 {"gates": L2[3], "call": L2[4], "c0": None}, p1, p2, pw, H)
    if r is None:
        raise RuntimeError("stacked LSTM forward ran but the stacked backward kernel rejected the shape")
    dz1, dz2, _, _ = r
    g2 = _lstm_native_grads(dz2, L1[5].reshape(T * mb, H), L2[0], L2[3], L2[4], None, None, x, W2, RW2, b2, H,
                            peephole, 3, want_dx=False)
    g1 = _lstm_native_grads(dz1, xt, L1[0], L1[3], L1[4], None, None, x, W1, RW1, b1, H, peephole, 0)
    return g1 + g2[1:]


register("lstmStack2")((_lstm2_fwd, _lstm2_bwd))


# ----------------------------------------------------------------------------------------------- losses (scalar)
def _sce_fwd(ins, at):
    y, z = ins
    ls = at.get("labelSmoothing", 0.0)
    yy = y * (1 - ls) + ls / y.shape[-1] if ls else y
    z2 = z.reshape(-1, z.shape[-1])
    from ..ops.loss import softmax_xent
    s, grad, _ = softmax_xent(z2.contiguous(), yy.reshape(-1, z.shape[-1]), None, 0.0)
    n = z2.shape[0]
    return s.sum() / n, (grad, n)


def _sce_bwd(ctx, g, ins, at):
    grad, n = ctx
    return [None, (grad.float() * (g.float() / n)).to(ins[1].dtype).reshape(ins[1].shape)]


register("softmaxCrossEntropy")((_sce_fwd, _sce_bwd))


def _mse_fwd(ins, at):
    y, z = ins
    d = z.float() - y.float() if z.dtype != torch.float64 else z - y
    return (d * d).mean(), d


def _mse_bwd(ctx, g, ins, at):
    d = ctx
    return [None, (2.0 * d * g / d.numel()).to(ins[1].dtype)]


register("meanSquaredError")((_mse_fwd, _mse_bwd))


def _log_fwd(ins, at):
    y, p = ins
    eps = at.get("epsilon", 1e-7)
    pc = p.float().clamp(eps, 1 - eps) if p.dtype != torch.float64 else p.clamp(eps, 1 - eps)
    yy = y.to(pc.dtype)
    return -(yy * torch.log(pc) + (1 - yy) * torch.log(1 - pc)).mean(), (pc, yy)


def _log_bwd(ctx, g, ins, at):
    pc, yy = ctx
    eps = at.get("epsilon", 1e-7)
    inside = ((ins[1] > eps) & (ins[1] < 1 - eps)).to(pc.dtype)
    d = (-(yy / pc) + (1 - yy) / (1 - pc)) * inside / pc.numel()
    return [None, (d * g).to(ins[1].dtype)]


register("logLoss")((_log_fwd, _log_bwd))
