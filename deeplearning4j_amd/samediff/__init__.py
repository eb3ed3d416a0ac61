"""SameDiff: a graph-building differentiable API with its own reverse-mode autodiff.

The reference's SameDiff (used through the SameDiff layer bridge, NN:nn/conf/layers/samediff/BaseSameDiffLayer.java:43,
NN:nn/layers/samediff/SameDiffLayer.java:58-87,195-215 execAndEndResult / execBackwards) records ops into a graph and
differentiates it op by op. Here every op is an entry of the registry in ``samediff/autodiff.py`` with an explicit
forward and backward (no torch.autograd); ``SameDiff`` records ``(output, op name, input variables, JSON attributes)``
and executes eagerly at definition time (so ``eval``/``getArr`` work immediately), can re-execute the recorded graph
for new placeholder values (``output``), differentiate it (``execBackwards``, ``calculateGradients``), train it
(``setTrainingConfig`` + ``fit``: reverse pass + one fused HIP updater launch over all trainable variables) and
save / load it (``save`` / ``SameDiff.load``: graph JSON + variable arrays). Heavy ops run on the framework's
kernels in both directions (GEMM, conv, pooling, LayerNorm, flash attention, LSTM, softmax-xent).
"""
import io
import json
import os
import zipfile

import torch

# reverse pass: a linear's input gradient is summed into the partial gradient other consumers already produced by the
# GEMM itself (beta = 1), instead of a separate add (DL4J_AMD_SD_ACC=0 turns it off for A/B checks)
_ACC_FUSE = os.environ.get("DL4J_AMD_SD_ACC", "1") == "1"

from .autodiff import REGISTRY


class SDVariable:
    def __init__(self, sd, name, value):
        self.sd, self.name, self.value = sd, name, value

    # ------------------------------------------------------------ arithmetic (named and anonymous forms)
    def _bin(self, name, other, op):
        if isinstance(name, (SDVariable, int, float)) or torch.is_tensor(name):
            name, other = None, name
        return self.sd._op(name, op, [self, other])

    def add(self, name, other=None):
        return self._bin(name, other, "add")

    def sub(self, name, other=None):
        return self._bin(name, other, "sub")

    def mul(self, name, other=None):
        return self._bin(name, other, "mul")

    def div(self, name, other=None):
        return self._bin(name, other, "div")

    def rsub(self, name, other=None):
        return self._bin(name, other, "rsub")

    def rdiv(self, name, other=None):
        return self._bin(name, other, "rdiv")

    def mmul(self, name, other=None):
        return self._bin(name, other, "mmul")

    def pow(self, name, p=None):
        if not isinstance(name, str) and name is not None:
            name, p = None, name
        return self.sd._op(name, "pow", [self], {"p": float(p)})

    def __add__(self, o):
        return self.add(None, o)

    def __radd__(self, o):
        return self.add(None, o)

    def __sub__(self, o):
        return self.sub(None, o)

    def __rsub__(self, o):
        return self.rsub(None, o)

    def __mul__(self, o):
        return self.mul(None, o)

    def __rmul__(self, o):
        return self.mul(None, o)

    def __truediv__(self, o):
        return self.div(None, o)

    def __matmul__(self, o):
        return self.mmul(None, o)

    def __neg__(self):
        return self.sd._op(None, "neg", [self])

    # ------------------------------------------------------------ reductions / shape
    def sum(self, *dims):
        return self.sd._op(None, "sum", [self], {"dims": list(dims)})

    def mean(self, *dims):
        return self.sd._op(None, "mean", [self], {"dims": list(dims)})

    def reshape(self, *shape):
        if len(shape) == 1 and isinstance(shape[0], (list, tuple)):
            shape = tuple(shape[0])
        return self.sd._op(None, "reshape", [self], {"shape": [int(s) for s in shape]})

    def permute(self, *dims):
        return self.sd._op(None, "permute", [self], {"dims": [int(d) for d in dims]})

    def transpose(self):
        return self.sd._op(None, "transpose", [self])

    def get(self, *idx):
        """Python-style indexing / slicing (e.g. ``h.get(slice(None), 0)`` = the first token of every row)."""
        enc = [{"slice": [i.start, i.stop, i.step]} if isinstance(i, slice) else i for i in idx]
        return self.sd._op(None, "get", [self], {"idx": enc})

    def getShape(self):
        return list(self.value.shape)

    def getArr(self):
        return self.value

    def eval(self):
        return self.value.detach()

    def gradient(self):
        """Gradient of the loss w.r.t. this variable from the last ``execBackwards`` / ``fit`` reverse pass."""
        return self.sd._last_grads.get(self.name)

    def __repr__(self):
        return f"SDVariable(name={self.name!r}, shape={list(self.value.shape)})"


class _NN:
    def __init__(self, sd):
        self.sd = sd

    def _u(self, name, x, op, attrs=None):
        if isinstance(name, SDVariable):
            name, x = None, name
        return self.sd._op(name, op, [x], attrs)

    def relu(self, name, x=None, cutoff=0.0):
        return self._u(name, x, "relu")

    def sigmoid(self, name, x=None):
        return self._u(name, x, "sigmoid")

    def tanh(self, name, x=None):
        return self._u(name, x, "tanh")

    def softmax(self, name, x=None):
        return self._u(name, x, "softmax")

    def gelu(self, name, x=None):
        return self._u(name, x, "gelu")

    def elu(self, name, x=None):
        return self._u(name, x, "elu")

    def leakyRelu(self, name, x=None, alpha=0.01):
        return self._u(name, x, "leakyRelu", {"alpha": float(alpha)})

    def softplus(self, name, x=None):
        return self._u(name, x, "softplus")

    def linear(self, name, x, w=None, b=None):
        if isinstance(name, SDVariable):
            name, x, w, b = None, name, x, w
        return self.sd._op(name, "linear", [x, w, b])

    def layerNorm(self, name, x, gain=None, bias=None, eps=1e-5):
        """LayerNorm over the last dim (LayerNorm HIP kernels on the GPU)."""
        if isinstance(name, SDVariable):
            name, x, gain, bias = None, name, x, gain
        return self.sd._op(name, "layerNorm", [x, gain, bias], {"eps": float(eps)})

    def fusedSelfAttention(self, name, qkv=None, nHeads=None, mask=None, causal=False):
        """Multi-head self attention on a fused projection qkv [B, T, 3E] -> [B, T, E] (flash-attention kernel)."""
        if isinstance(name, SDVariable):
            name, qkv, nHeads, mask = None, name, qkv, nHeads
        return self.sd._op(name, "fusedSelfAttention", [qkv, mask], {"nHeads": int(nHeads), "causal": bool(causal)})


class _RNN:
    def __init__(self, sd):
        self.sd = sd

    def lstmLayer(self, name, x, W, RW, b, h0=None, c0=None, peephole=False):
        """Whole-sequence LSTM (DL4J gate order, tanh/sigmoid): x [mb, nIn, T] -> [mb, H, T]. Runs the fused
        sequence HIP kernels on the GPU (csrc/lstm.hip); RW has 3 extra peephole columns when ``peephole``."""
        return self.sd._op(name, "lstmLayer", [x, W, RW, b, h0, c0], {"peephole": bool(peephole)})


class _CNN:
    def __init__(self, sd):
        self.sd = sd

    def conv2d(self, name, x, w, b=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1)):
        if isinstance(name, SDVariable):
            name, x, w, b = None, name, x, w
        return self.sd._op(name, "conv2d", [x, w, b], {"stride": list(stride), "padding": list(padding),
                                                          "dilation": list(dilation)})

    def maxPooling2d(self, name, x, kernel, stride, padding=(0, 0)):
        return self.sd._op(name, "maxPooling2d", [x], {"kernel": list(kernel), "stride": list(stride),
                                                        "padding": list(padding)})

    def avgPooling2d(self, name, x, kernel, stride, padding=(0, 0)):
        return self.sd._op(name, "avgPooling2d", [x], {"kernel": list(kernel), "stride": list(stride),
                                                        "padding": list(padding)})


class _Loss:
    """``sd.loss()``: reduced (mean over the minibatch) losses, registered as loss variables."""

    def __init__(self, sd):
        self.sd = sd

    def _reg(self, v):
        self.sd._loss_names.append(v.name)
        return v

    def softmaxCrossEntropy(self, name, labels, logits, weights=None, labelSmoothing=0.0):
        """Softmax over the last dimension of ``logits``; labels one-hot (or soft) of the same shape."""
        return self._reg(self.sd._op(name, "softmaxCrossEntropy", [labels, logits],
                                     {"labelSmoothing": float(labelSmoothing)}))

    def meanSquaredError(self, name, labels, predictions, weights=None):
        return self._reg(self.sd._op(name, "meanSquaredError", [labels, predictions]))

    def logLoss(self, name, labels, predictions, weights=None, epsilon=1e-7):
        return self._reg(self.sd._op(name, "logLoss", [labels, predictions], {"epsilon": float(epsilon)}))


class TrainingConfig:
    """``TrainingConfig.builder()``: updater, l2, minibatch division and the DataSet -> placeholder mappings
    (reference SameDiff TrainingConfig)."""

    def __init__(self, updater=None, l1=0.0, l2=0.0, features=(), labels=(), minimize=True):
        self.updater, self.l1, self.l2 = updater, float(l1), float(l2)
        self.dataSetFeatureMapping, self.dataSetLabelMapping = list(features), list(labels)
        self.minimize = minimize

    class Builder:
        def __init__(self):
            self._kw = {}

        def updater(self, u):
            self._kw["updater"] = u
            return self

        def l1(self, v):
            self._kw["l1"] = v
            return self

        def l2(self, v):
            self._kw["l2"] = v
            return self

        def dataSetFeatureMapping(self, *names):
            self._kw["features"] = names
            return self

        def dataSetLabelMapping(self, *names):
            self._kw["labels"] = names
            return self

        def minimize(self, b=True):
            self._kw["minimize"] = b
            return self

        def build(self):
            return TrainingConfig(**self._kw)

    @staticmethod
    def builder():
        return TrainingConfig.Builder()


class SameDiff:
    """A recorded differentiable graph (see module docstring)."""

    def __init__(self):
        self.variables = {}
        self._kind = {}                 # name -> VARIABLE | PLACEHOLDER | CONSTANT | ARRAY
        self._n = 0
        self._ops = []                  # records: (output name, op name, input refs, attrs) in definition order
        self._ctx = {}                  # output name -> saved forward context of its op
        self._placeholders = []
        self._trainable = []
        self._loss_names = []
        self._last_grads = {}
        self._plans = {}
        self._executed = None           # target set of the last planned execution (whose contexts are live)
        self.fusion = True
        self.trainingConfig = None
        self._train_state = None
        self.iterationCount = 0
        self.epochCount = 0

    @staticmethod
    def create():
        return SameDiff()

    # ------------------------------------------------------------------ definition
    def _new(self, name, value, kind):
        if name is None:
            self._n += 1
            name = f"sd_var_{self._n}"
        v = SDVariable(self, name, value)
        self.variables[name] = v
        self._kind[name] = kind
        return v

    def _ref(self, a):
        """Input reference of an op: a variable name, a python scalar, or None."""
        if a is None:
            return None
        if isinstance(a, SDVariable):
            return a.name
        if isinstance(a, (int, float, bool)):
            return {"scalar": a}
        if torch.is_tensor(a):
            return self.constant(None, a).name
        raise TypeError(f"unsupported SameDiff op input {type(a)}")

    def _val(self, r):
        if r is None:
            return None
        if isinstance(r, dict):
            return r["scalar"]
        return self.variables[r].value

    def _op(self, name, op, args, attrs=None):
        if op not in REGISTRY:
            raise KeyError(f"unknown SameDiff op {op!r}")
        refs = [self._ref(a) for a in args]
        attrs = dict(attrs or {})
        y, ctx = REGISTRY[op].fwd([self._val(r) for r in refs], attrs)
        v = self._new(name, y, "ARRAY")
        self._ctx[v.name] = ctx
        self._executed = None
        self._ops.append((v.name, op, refs, attrs))
        return v

    def var(self, name, value, *shape):
        if not torch.is_tensor(value):
            value = torch.as_tensor(value) if not shape else torch.zeros(shape)
        v = self._new(name, value, "VARIABLE")
        self._trainable.append(v.name)
        return v

    def placeHolder(self, name, value=None, *shape):
        """placeHolder(name, exampleValue) or placeHolder(name, dtype, *shape): a graph input fed by ``output`` /
        ``fit``. A shape (with -1 for the minibatch) creates a zero example value for eager definition."""
        if value is None or not torch.is_tensor(value):
            dims = [1 if d is None or d < 0 else int(d) for d in shape] if shape else [1]
            dt = value if isinstance(value, torch.dtype) else torch.float32
            value = torch.zeros(dims, dtype=dt)
        v = self._new(name, value, "PLACEHOLDER")
        self._placeholders.append(v.name)
        return v

    def constant(self, name, value):
        return self._new(name, torch.as_tensor(value).detach(), "CONSTANT")

    def loss(self):
        return _Loss(self)

    def setLossVariables(self, *names):
        self._loss_names = [n.name if isinstance(n, SDVariable) else n for n in names]

    def getLossVariables(self):
        return list(self._loss_names)

    def trainableVariables(self):
        return [self.variables[n] for n in self._trainable]

    def ops(self):
        """The recorded graph: [(output, op, inputs, attrs)]."""
        return list(self._ops)

    # ------------------------------------------------------------------ execution
    def _needed(self, targets):
        if targets is None:
            return list(self._ops)
        need = set(targets)
        keep = []
        for rec in reversed(self._ops):
            if rec[0] in need:
                keep.append(rec)
                need.update(r for r in rec[2] if isinstance(r, str))
        return keep[::-1]

    def _plan(self, targets):
        """Execution plan for ``targets``: the needed records after the fusion pass, cached per target set.

        Fusions (only where the intermediate has a single consumer and is not itself a target):
          linear -> gelu          one GEMM with the GELU in its epilogue (pre-activation kept for the backward)
          add(a, b) -> layerNorm  the residual sum done inside the LayerNorm kernel (same-shape operands)
          lstmLayer -> lstmLayer  the two recurrences pipelined in one launch per direction (lstmStack2)
        Fused-away intermediates keep their definition-time values."""
        key = (tuple(targets) if targets is not None else None, self.fusion)
        hit = self._plans.get(key)
        if hit is not None and hit[0] == len(self._ops):
            return hit[1]
        recs = self._needed(targets)
        if self.fusion:
            uses = {}
            for _, _, refs, _ in recs:
                for r in refs:
                    if isinstance(r, str):
                        uses[r] = uses.get(r, 0) + 1
            for t in targets or ():
                uses[t] = uses.get(t, 0) + 1
            prod = {r[0]: i for i, r in enumerate(recs)}
            out, drop = list(recs), set()
            for i, (o, op, refs, attrs) in enumerate(recs):
                src = refs[0] if refs and isinstance(refs[0], str) else None
                j = prod.get(src)
                if j is None or uses.get(src, 0) != 1 or j in drop:
                    continue
                po, pop, prefs, pattrs = recs[j]
                if op == "gelu" and pop == "linear" and "act" not in pattrs:
                    out[i] = (o, "linear", prefs, {**pattrs, "act": "gelu"})
                    drop.add(j)
                elif op == "lstmLayer" and pop == "lstmLayer" and refs[4:6] == [None, None] and \
                        prefs[4:6] == [None, None] and attrs.get("peephole", False) == pattrs.get("peephole", False):
                    # stacked LSTM layers: one pipelined launch per direction (autodiff lstmStack2)
                    out[i] = (o, "lstmStack2", list(prefs[:4]) + list(refs[1:4]), dict(attrs))
                    drop.add(j)
                elif op == "layerNorm" and pop == "add" and len(refs) == 3 and \
                        all(isinstance(r, str) for r in prefs):
                    a, b = (self.variables[r].value for r in prefs)
                    if a.shape == b.shape and a.dtype == b.dtype:
                        out[i] = (o, "layerNorm", [prefs[0], refs[1], refs[2], prefs[1]], dict(attrs))
                        drop.add(j)
            recs = [r for k, r in enumerate(out) if k not in drop]
        self._plans[key] = (len(self._ops), recs)
        return recs

    def _exec(self, feeds, targets=None):
        """Re-run the recorded ops (those ``targets`` depend on) with new placeholder values; saves contexts."""
        for k, v in feeds.items():
            self.variables[k].value = v
        self._executed = tuple(targets) if targets is not None else None
        for out, op, refs, attrs in self._plan(targets):
            y, ctx = REGISTRY[op].fwd([self._val(r) for r in refs], attrs)
            self.variables[out].value = y
            self._ctx[out] = ctx

    def _backward(self, seeds, wrt, targets=None, on_final=None, sinks=None):
        """Reverse pass from ``seeds`` {variable name: upstream gradient} over the recorded ops; returns
        {name: gradient} for ``wrt`` (every op's explicit backward; no torch.autograd).

        ``on_final(name, grad)``: called for each ``wrt`` variable as soon as its gradient is complete, i.e. right
        after the reverse pass has processed the EARLIEST recorded op that reads it (later ops were processed
        first). Data-parallel training uses it to start each gradient bucket's all-reduce while the rest of the
        reverse pass still runs.

        ``sinks`` {name: contiguous fp32 tensor}: destinations (views of the flat gradient buffer) for variables read
        by exactly ONE recorded op; that op's backward writes the gradient there directly (autodiff.grad_sink)
        instead of into a temporary the training step would then copy."""
        grads = dict(seeds)
        tg = targets if targets is not None else list(seeds)
        # the planned (fused) records only when their contexts come from a planned execution of these targets
        recs = self._plan(tg) if self._executed == tuple(tg) else self._needed(tg)
        if sinks:
            reads = {}
            for _, _, refs, _ in recs:
                for r in refs:
                    if isinstance(r, str) and r in sinks:
                        reads[r] = reads.get(r, 0) + 1
            sinks = {n: t for n, t in sinks.items() if reads.get(n) == 1 and n not in grads}
        from . import autodiff as _ad
        dsum_for, presunk = (self._ln_bias_fusions(recs, sinks) if sinks else {}), {}
        # inputs nobody differentiates (placeholders / constants not asked for): ops may skip their gradient
        frozen = {n for n, k in self._kind.items() if k in ("PLACEHOLDER", "CONSTANT")} - set(wrt)
        final_at = {}
        if on_final is not None:
            want = set(wrt)
            for i, (_, _, refs, _) in enumerate(recs):
                for r in refs:
                    if isinstance(r, str) and r in want and r not in final_at:
                        final_at[r] = i
            by_pos = {}
            for name, i in final_at.items():
                by_pos.setdefault(i, []).append(name)
            for name in wrt:                    # read by no op on the path to the targets: final (None) now
                if name not in final_at:
                    on_final(name, grads.get(name))
        produced_at = {rec[0]: k for k, rec in enumerate(recs)}

        def _sp(t):
            return t.untyped_storage().data_ptr() if torch.is_tensor(t) else None
        seed_ptrs = {_sp(t) for t in seeds.values()}
        for i in range(len(recs) - 1, -1, -1):
            out, op, refs, attrs = recs[i]
            g = grads.get(out)
            if g is not None:
                ins = [self._val(r) for r in refs]
                sk = {j: sinks[r] for j, r in enumerate(refs) if isinstance(r, str) and r in sinks} if sinks else None
                fz = dsum_for.get(i)
                acc = None
                if _ACC_FUSE and op == "linear" and isinstance(refs[0], str) and refs[0] not in wrt:
                    prev = grads.get(refs[0])
                    # in place only when no seed and no other pending gradient (a name whose producing op is still to
                    # come, or a returned one) shares its storage
                    if prev is not None and torch.is_tensor(prev) and _sp(prev) not in seed_ptrs and not any(
                            n != refs[0] and produced_at.get(n, -1) < i and _sp(t) == _sp(prev)
                            for n, t in grads.items()):
                        acc = {0: prev}
                _ad.set_sinks(sk, done=presunk.get(i), dsum=None if fz is None else sinks[fz[1]],
                              nograd={j for j, r in enumerate(refs) if isinstance(r, str) and r in frozen}, acc=acc)
                try:
                    gins = REGISTRY[op].bwd(self._ctx[out], g, ins, attrs)
                    if fz is not None and _ad.dsum_written():
                        presunk[fz[0]] = {2}        # the producing linear's bias gradient is already in its sink
                    used = set(_ad.acc_used())
                finally:
                    _ad.set_sinks(None)
                for j, (r, gi) in enumerate(zip(refs, gins)):
                    if gi is None or not isinstance(r, str):
                        continue
                    prev = grads.get(r)
                    if j in used:
                        grads[r] = gi                # the backward already summed into prev (gi is prev)
                    elif prev is None:
                        grads[r] = gi
                    else:
                        grads[r] = prev + gi
            if on_final is not None:
                for name in by_pos.get(i, ()):
                    on_final(name, grads.get(name))
        self._last_grads = {k: grads.get(k) for k in wrt}
        return self._last_grads

    @staticmethod
    def _ln_bias_fusions(recs, sinks):
        """{LayerNorm record index: (producing linear record index, bias variable)} for LayerNorms whose normalized
        input (x or the fused residual) is the output of a bias-carrying, activation-free linear op read by nothing
        else: LayerNorm's backward kernel emits the column sums of its input gradient, which ARE that bias gradient
        (the CG's dense -> LayerNorm fusion, csrc/layernorm.hip dsum), so the linear skips its channel-sum pass."""
        prod = {o: j for j, (o, _, _, _) in enumerate(recs)}
        reads = {}
        for _, _, refs, _ in recs:
            for r in refs:
                if isinstance(r, str):
                    reads[r] = reads.get(r, 0) + 1
        out = {}
        for j, (_, op, refs, _) in enumerate(recs):
            if op != "layerNorm":
                continue
            for pos in (0, 3):
                y = refs[pos] if pos < len(refs) else None
                pj = prod.get(y) if isinstance(y, str) else None
                if pj is None or reads.get(y) != 1:
                    continue
                _, pop, prefs, pat = recs[pj]
                if pop == "linear" and not pat.get("act") and len(prefs) > 2 and isinstance(prefs[2], str) and \
                        prefs[2] in sinks:
                    out[j] = (pj, prefs[2])
                    break
        return out

    def output(self, placeholders, *outputs):
        """Execute the recorded graph for new placeholder values; returns {name: value}."""
        names = [o.name if isinstance(o, SDVariable) else o for o in outputs]
        with torch.no_grad():
            self._exec({k: _tensor(v) for k, v in placeholders.items()}, names)
        return {n: self.variables[n].value for n in names}

    def outputSingle(self, placeholders, output):
        return next(iter(self.output(placeholders, output).values()))

    def execAndEndResult(self, out):
        return out.value.detach()

    def execBackwards(self, loss, wrt=None, placeholders=None):
        """Gradients of ``loss`` (seeded with ones) w.r.t. ``wrt`` (default: trainable variables)."""
        self._exec({k: _tensor(v) for k, v in (placeholders or {}).items()}, [loss.name])
        wrt = [w.name if isinstance(w, SDVariable) else w for w in (wrt or self.trainableVariables())]
        return self._backward({loss.name: torch.ones_like(loss.value)}, wrt, [loss.name])

    def calculateGradients(self, placeholders, *variables):
        if not self._loss_names:
            raise ValueError("no loss variables")
        self._exec({k: _tensor(v) for k, v in (placeholders or {}).items()}, self._loss_names)
        wrt = [w.name if isinstance(w, SDVariable) else w for w in variables] or list(self._trainable)
        seeds = {n: torch.ones_like(self.variables[n].value) for n in self._loss_names}
        return self._backward(seeds, wrt, list(self._loss_names))

    # ------------------------------------------------------------------ training
    def setTrainingConfig(self, cfg):
        self.trainingConfig = cfg
        self._train_state = None

    def _init_training(self):
        from ..ops.update import Segment, UpdatePlan
        cfg = self.trainingConfig
        vs = self.trainableVariables()
        dev = vs[0].value.device
        n = sum(v.value.numel() for v in vs)
        mdt = torch.float64 if all(v.value.dtype == torch.float64 for v in vs) else torch.float32
        flat = torch.empty(n, dtype=mdt, device=dev)
        # bf16 / fp16 variables train in mixed precision: fp32 master weights, the fused updater writes the 16-bit
        # copy the graph computes with (its "shadow") in the same pass
        lowp = vs[0].value.dtype
        mixed = lowp in (torch.bfloat16, torch.float16) and all(v.value.dtype == lowp for v in vs)
        shadow = torch.empty(n, dtype=lowp, device=dev) if mixed else None
        segs, off = [], 0
        for v in vs:
            k = v.value.numel()
            flat[off:off + k].copy_(v.value.detach().reshape(-1).to(mdt))
            if mixed:
                shadow[off:off + k].copy_(v.value.detach().reshape(-1))
                v.value = shadow[off:off + k].view(v.value.shape)
                # the fp32 master next to its 16-bit shadow: ops that consume parameters in fp32 (GEMM bias, LayerNorm
                # gamma / beta) read it instead of converting the shadow every step (autodiff.master)
                v.value._dl4j_master = flat[off:off + k].view(v.value.shape)
                v.value._dl4j_master._dl4j_shadow = v.value
            else:
                v.value = flat[off:off + k].view(v.value.shape)
            segs.append(Segment(off, k, 0, off, n, cfg.updater, cfg.l1, cfg.l2, 0))   # one block: state offset 0
            off += k
        state = torch.zeros(max(1, cfg.updater.stateSize(n)), dtype=mdt, device=dev)
        plan = UpdatePlan(segs, [(0, n, 0, cfg.updater)])
        self._train_state = {"flat": flat, "grad": torch.zeros_like(flat), "state": state, "plan": plan,
                             "shadow": shadow}

    def fit(self, data, numEpochs=1):
        """Train on a DataSet / MultiDataSet, an iterator of them, or a list. Returns the last loss value."""
        from ..datasets.dataset import DataSet
        from ..ops.update import fused_update
        cfg = self.trainingConfig
        if cfg is None or cfg.updater is None:
            raise ValueError("setTrainingConfig(TrainingConfig.builder().updater(...)...) first")
        if not self._loss_names:
            raise ValueError("no loss variables: use sd.loss() ops or setLossVariables")
        if self._train_state is None:
            self._init_training()
        st = self._train_state
        vs = self.trainableVariables()
        last = None
        sign = 1.0 if cfg.minimize else -1.0
        for _ in range(int(numEpochs)):
            items = [data] if isinstance(data, DataSet) or hasattr(data, "features") else data
            if hasattr(items, "reset"):
                items.reset()
            for ds in items:
                feats = ds.features if isinstance(ds.features, (list, tuple)) else [ds.features]
                labs = ds.labels if isinstance(ds.labels, (list, tuple)) else [ds.labels]
                feeds = {n: _tensor(t).to(st["flat"].device) for n, t in zip(cfg.dataSetFeatureMapping, feats)}
                feeds.update({n: _tensor(t).to(st["flat"].device) for n, t in
                              zip(cfg.dataSetLabelMapping, labs)})
                with torch.no_grad():
                    if self._graph_ready(feeds):
                        last = self._graph_replay(feeds)
                    else:
                        last = self._train_body(feeds, sign)
                        self._eager_steps += 1
                # the loss stays on the device: iterations of one fit call run back to back, without a host sync
                # between them (the A/B graph slots keep the last replay's loss valid until the call returns)
                self.iterationCount += 1
            self.epochCount += 1
        return None if last is None else float(last)

    def _train_body(self, feeds, sign):
        """One training iteration's device work: forward, reverse pass, gradient copy into the flat buffer,
        cross-rank all-reduce, fused update. Returns the summed loss as a device tensor (capturable)."""
        from ..ops.update import fused_update
        st = self._train_state
        vs = self.trainableVariables()
        self._exec(feeds, self._loss_names)
        seeds = {n: torch.full_like(self.variables[n].value, sign) for n in self._loss_names}
        if "views" not in st:
            off, st["views"] = 0, []
            for v in vs:
                st["views"].append(st["grad"][off:off + v.value.numel()].view(v.value.shape))
                off += v.value.numel()
        dp = self._dp_buckets(st)
        if dp is not None:
            # data parallel: each variable's gradient goes into the flat buffer as soon as it is final, and a bucket's
            # all-reduce starts once all of its variables are, overlapping the rest of the reverse pass
            dp.begin()
            self._backward(seeds, [v.name for v in vs], list(self._loss_names), on_final=dp.final,
                           sinks=self._grad_sinks(st, vs))
            dp.finish()
        else:
            grads = self._backward(seeds, [v.name for v in vs], list(self._loss_names),
                                   sinks=self._grad_sinks(st, vs))
            dst, src = [], []
            for v, view in zip(vs, st["views"]):
                g = grads.get(v.name)
                if g is None:
                    view.zero_()
                elif g.data_ptr() != view.data_ptr():        # gradient sinks were written in place
                    dst.append(view)
                    src.append(g.reshape(view.shape))
            if dst:
                torch._foreach_copy_(dst, src)      # one multi-tensor launch for the remaining gradients
        fused_update(st["plan"], st["flat"], st["grad"], st["state"], self.iterationCount, self.epochCount, 1,
                     mini_batch=False, shadow=st["shadow"])
        out = None
        for n in self._loss_names:
            v = self.variables[n].value.float().reshape(())
            out = v if out is None else out + v
        return out

    @staticmethod
    def _grad_sinks(st, vs):
        """{variable name: its fp32 flat-gradient view} (fp64 training keeps the copies: the GEMM writes fp32)."""
        if st["grad"].dtype != torch.float32 or os.environ.get("DL4J_AMD_SD_SINKS", "1") == "0":
            return None
        return {v.name: view for v, view in zip(vs, st["views"])}

    # ------------------------------------------------------------------ HIP graphs
    def enableHipGraphs(self, enabled=True, warmup=2):
        """Capture the training iteration into HIP graphs after ``warmup`` eager steps (fixed placeholder shapes,
        CUDA variables, no gloo all-reduce): two graphs A/B alternate so the fused updater's iteration-dependent
        table (pinned buffer + graph H2D node) is refreshed without a host sync, as nn/hipgraph.py does for
        networks. The whole step - every op's forward and explicit backward, the gradient copy, RCCL all-reduce
        and the update - replays with one launch."""
        self._graphs_on = bool(enabled)
        self._graph_warmup = int(warmup)
        self._graph = None
        return self

    _graphs_on = False
    _graph = None
    _eager_steps = 0

    def _graph_eligible(self, feeds):
        import torch.distributed as dist
        if not self._graphs_on or not all(t.is_cuda for t in feeds.values()):
            return False
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 and \
                dist.get_backend() != "nccl":
            return False
        return self._train_state["flat"].is_cuda

    def _graph_ready(self, feeds):
        if not self._graph_eligible(feeds):
            return False
        g = self._graph
        if g is not None:
            return g["ok"] and all(feeds[k].shape == g["static"][k].shape and feeds[k].dtype == g["static"][k].dtype
                                   for k in feeds)
        if self._eager_steps < self._graph_warmup:
            return False
        return self._graph_capture(feeds)

    def _graph_capture(self, feeds):
        from ..ops import native
        st = self._train_state
        sign = 1.0 if self.trainingConfig.minimize else -1.0
        static = {k: v.detach().clone() for k, v in feeds.items()}
        g = {"static": static, "graphs": [], "loss": [None, None], "k": 0, "ok": False,
             "pool": torch.cuda.graph_pool_handle()}
        native.prepare_graph_slots(st["plan"], st["flat"].device, self.iterationCount, self.epochCount)
        torch.cuda.current_stream(st["flat"].device).synchronize()
        from ..nn.hipgraph import capture, capture_gc_guard
        guard = capture_gc_guard()
        guard.__enter__()
        try:
            for slot in (0, 1):
                cg = torch.cuda.CUDAGraph()
                native.GRAPH_SLOT[0] = slot
                g["loss"][slot] = capture(cg, g["pool"], lambda: self._train_body(static, sign),
                                          st["flat"].device)
                g["graphs"].append(cg)
            g["ok"] = True
        except Exception as e:          # capture not possible for this graph: stay eager
            import logging
            logging.getLogger("deeplearning4j_amd").warning("SameDiff HIP-graph capture failed, eager steps: %s", e)
            g["ok"] = False
        finally:
            native.GRAPH_SLOT[0] = None
            guard.__exit__(None, None, None)
        self._graph = g                 # (capture only records: parameters are untouched until the first replay)
        return g["ok"]

    def _graph_replay(self, feeds):
        from ..ops import native
        g = self._graph
        st = self._train_state
        for k, v in feeds.items():
            g["static"][k].copy_(v, non_blocking=True)
        slot = g["k"] & 1
        native.refresh_graph_table(st["plan"], slot, self.iterationCount, self.epochCount)
        g["graphs"][slot].replay()
        native.mark_graph_replayed(st["plan"], slot)
        g["k"] += 1
        return g["loss"][slot]

    def _dp_buckets(self, st):
        """The data-parallel bucket plan (one process per GPU, torch.distributed over RCCL / gloo), or None when
        training on one rank. See _SDGradBuckets."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return None
        b = st.get("dp")
        if b is None:
            b = st["dp"] = _SDGradBuckets(self, st)
        return b

    # ------------------------------------------------------------------ save / load
    # ------------------------------------------------------------------ save / load
    def save(self, path, saveUpdaterState=False):
        """Graph JSON (variables with kinds / shapes / dtypes, op records, loss variables) + variable arrays
        (torch.save of a tensor dict, read back with weights_only=True)."""
        graph = {
            "format": "dl4j_amd.samediff/1",
            "variables": [{"name": n, "kind": self._kind[n], "shape": list(v.value.shape),
                           "dtype": str(v.value.dtype).replace("torch.", "")} for n, v in self.variables.items()],
            "ops": [{"output": o, "op": op, "inputs": refs, "attrs": attrs} for o, op, refs, attrs in self._ops],
            "losses": list(self._loss_names), "placeholders": list(self._placeholders),
            "trainable": list(self._trainable), "iterationCount": self.iterationCount, "epochCount": self.epochCount,
        }
        arrays = {n: v.value.detach().cpu().clone() for n, v in self.variables.items() if self._kind[n] != "ARRAY"}
        buf = io.BytesIO()
        torch.save(arrays, buf)
        with zipfile.ZipFile(path, "w") as z:
            z.writestr("graph.json", json.dumps(graph, indent=1))
            z.writestr("arrays.pt", buf.getvalue())

    @staticmethod
    def load(path, device=None):
        with zipfile.ZipFile(path) as z:
            graph = json.loads(z.read("graph.json"))
            arrays = torch.load(io.BytesIO(z.read("arrays.pt")), weights_only=True)
        sd = SameDiff()
        for vd in graph["variables"]:
            n = vd["name"]
            if vd["kind"] == "ARRAY":
                continue
            t = arrays[n].to(device) if device is not None else arrays[n]
            sd._new(n, t, vd["kind"])
        sd._placeholders = list(graph["placeholders"])
        sd._trainable = list(graph["trainable"])
        sd._loss_names = list(graph["losses"])
        sd.iterationCount, sd.epochCount = graph.get("iterationCount", 0), graph.get("epochCount", 0)
        for rec in graph["ops"]:
            y, ctx = REGISTRY[rec["op"]].fwd([sd._val(r) for r in rec["inputs"]], rec["attrs"])
            sd._new(rec["output"], y, "ARRAY")
            sd._ctx[rec["output"]] = ctx
            sd._ops.append((rec["output"], rec["op"], rec["inputs"], rec["attrs"]))
        return sd

    def getVariable(self, name):
        return self.variables[name]

    def nn(self):
        return _NN(self)

    def cnn(self):
        return _CNN(self)

    def rnn(self):
        return _RNN(self)

    # common ops in the reference's sd.xxx(name, ...) form
    def mmul(self, name, a, b=None):
        if isinstance(name, SDVariable):
            name, a, b = None, name, a
        return self._op(name, "mmul", [a, b])

    def _u(self, name, x, op, attrs=None):
        if isinstance(name, SDVariable):
            name, x = None, name
        return self._op(name, op, [x], attrs)

    def sigmoid(self, name, x=None):
        return self._u(name, x, "sigmoid")

    def tanh(self, name, x=None):
        return self._u(name, x, "tanh")

    def relu(self, name, x=None, cutoff=0.0):
        return self._u(name, x, "relu")

    def softmax(self, name, x=None):
        return self._u(name, x, "softmax")

    def exp(self, name, x=None):
        return self._u(name, x, "exp")

    def log(self, name, x=None):
        return self._u(name, x, "log")

    def sqrt(self, name, x=None):
        return self._u(name, x, "sqrt")

    def square(self, name, x=None):
        return self._u(name, x, "square")

    def abs(self, name, x=None):
        return self._u(name, x, "abs")

    def neg(self, name, x=None):
        return self._u(name, x, "neg")

    def identity(self, name, x=None):
        return self._u(name, x, "identity")

    def sum(self, name, x, *dims):
        return self._op(name, "sum", [x], {"dims": list(dims)})

    def mean(self, name, x, *dims):
        return self._op(name, "mean", [x], {"dims": list(dims)})

    def gather(self, name, params, indices, axis=0):
        """Rows of ``params`` selected by integer ``indices`` (embedding lookup when axis == 0)."""
        return self._op(name, "gather", [params, indices], {"axis": int(axis)})

    def concat(self, name, dim, *xs):
        return self._op(name, "concat", list(xs), {"dim": int(dim)})

    def activation(self, name, act, x):
        from ..nn.conf.activations import to_activation
        a = to_activation(act)
        return self._op(name, "activation", [x], {"act": a.to_dict()})


def _tensor(v):
    if hasattr(v, "toTensor"):
        return v.toTensor()
    return v if torch.is_tensor(v) else torch.as_tensor(v)


def _as_samediff(self, name, sd, x):
    """Activation.X.asSameDiff(name, sd, x) (reference Activation.asSameDiff)."""
    return sd.activation(name, self, x)


def _install():
    from ..nn.conf.activations import Activation, IActivation
    Activation.asSameDiff = _as_samediff
    IActivation.asSameDiff = _as_samediff


_install()

__all__ = ["SameDiff", "SDVariable", "TrainingConfig"]


class _SDGradBuckets:
    """Bucketed, overlapped gradient all-reduce for SameDiff data parallelism (the reference shares SameDiff
    gradients through ParallelWrapper; SURVEY §5.8: buckets overlap the reverse pass).

    The flat fp32 gradient is cut into buckets of whole variables (DL4J_AMD_BUCKET_MB, default 32 MB). The reverse
    pass reports each trainable variable the moment its gradient is final (SameDiff._backward ``on_final``); the
    gradient is copied into its flat view and, once every variable of a bucket is in, the bucket's all-reduce is
    issued asynchronously (torch.distributed: RCCL's own stream on GPUs, so it runs while the reverse pass goes on).
    ``finish`` waits for all buckets and averages by the world size. Wire dtype: DL4J_AMD_SD_COMM_DTYPE=bf16|fp16
    halves the bytes (persistent staging buffers, stable addresses for HIP-graph capture)."""

    def __init__(self, sd, st):
        import os
        self.st = st
        vs = sd.trainableVariables()
        g = st["grad"]
        per = max(1, int(float(os.environ.get("DL4J_AMD_BUCKET_MB", "32")) * (1 << 20)) // g.element_size())
        self.var_bucket = {}
        self.view = {}
        self.buckets = []            # [start, end, n_vars]
        off = 0
        cur = None
        for v, view in zip(vs, st["views"]):
            k = v.value.numel()
            if cur is None or cur[1] - cur[0] >= per:
                cur = [off, off, 0]
                self.buckets.append(cur)
            cur[1] = off + k
            cur[2] += 1
            self.var_bucket[v.name] = len(self.buckets) - 1
            self.view[v.name] = view
            off += k
        wire = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(os.environ.get("DL4J_AMD_SD_COMM_DTYPE", ""))
        self.staging = None
        if wire is not None and wire != g.dtype:
            self.staging = [torch.empty(e - s, dtype=wire, device=g.device) for s, e, _ in self.buckets]
        self.left = []
        self.pending = []

    def begin(self):
        self.left = [n for _, _, n in self.buckets]
        self.pending = []

    def final(self, name, grad):
        b = self.var_bucket.get(name)
        if b is None:
            return
        view = self.view[name]
        if grad is None:
            view.zero_()
        elif grad.data_ptr() != view.data_ptr():          # not already written in place (gradient sink)
            view.copy_(grad.reshape(view.shape))
        self.left[b] -= 1
        if self.left[b] == 0:
            self._issue(b)

    def _issue(self, b):
        import torch.distributed as dist
        s, e, _ = self.buckets[b]
        seg = self.st["grad"][s:e]
        tmp = self.staging[b] if self.staging is not None else None
        if tmp is not None:
            tmp.copy_(seg)
        work = dist.all_reduce(tmp if tmp is not None else seg, async_op=True)
        self.pending.append((work, tmp, seg))

    def finish(self):
        import torch.distributed as dist
        for b, n in enumerate(self.left):      # buckets whose variables got no report (defensive): issue now
            if n > 0:
                self.left[b] = 0
                self._issue(b)
        for work, tmp, seg in self.pending:
            work.wait()
            if tmp is not None:
                seg.copy_(tmp)
        self.pending = []
        self.st["grad"].div_(dist.get_world_size())
