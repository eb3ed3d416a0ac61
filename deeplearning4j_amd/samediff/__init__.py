"""SameDiff-lite: a define-by-run differentiable graph API for user-defined layers.

The reference's SameDiff layer bridge (nn/conf/layers/samediff/BaseSameDiffLayer.java:43,
nn/layers/samediff/SameDiffLayer.java:58-87,195-215) lets a user describe a layer's forward pass with the
``SameDiff`` op API; DL4J runs ``execAndEndResult`` forward and ``execBackwards`` for the gradients.
Here ``SameDiff`` records the same calls eagerly on PyTorch-ROCm tensors (autograd supplies the backward),
so a layer written against the reference API (``sd.mmul("mmul", x, w)``, ``z.add("z", b)``,
``Activation.TANH.asSameDiff("out", sd, z)``, ``sd.nn().relu(...)``) runs unchanged on the GPU. Only the
op surface the reference layer tests use plus the common math/NN ops is provided.
"""
import torch
import torch.nn.functional as F


class SDVariable:
    def __init__(self, sd, name, value):
        self.sd, self.name, self.value = sd, name, value

    # ------------------------------------------------------------ arithmetic (named and anonymous forms)
    def _bin(self, name, other, fn):
        if isinstance(name, (SDVariable, int, float)) or torch.is_tensor(name):
            name, other = None, name
        return self.sd._op(name, fn, self, other)

    def add(self, name, other=None):
        return self._bin(name, other, torch.add)

    def sub(self, name, other=None):
        return self._bin(name, other, torch.sub)

    def mul(self, name, other=None):
        return self._bin(name, other, torch.mul)

    def div(self, name, other=None):
        return self._bin(name, other, torch.div)

    def rsub(self, name, other=None):
        return self._bin(name, other, lambda a, b: b - a)

    def rdiv(self, name, other=None):
        return self._bin(name, other, lambda a, b: b / a)

    def mmul(self, name, other=None):
        return self._bin(name, other, torch.matmul)

    def pow(self, name, p=None):
        return self._bin(name, p, torch.pow)

    def __add__(self, o):
        return self.add(None, o)

    def __sub__(self, o):
        return self.sub(None, o)

    def __mul__(self, o):
        return self.mul(None, o)

    def __truediv__(self, o):
        return self.div(None, o)

    def __matmul__(self, o):
        return self.mmul(None, o)

    def __neg__(self):
        return self.sd._op(None, torch.neg, self)

    # ------------------------------------------------------------ reductions / shape
    def sum(self, *dims):
        return self.sd._op(None, lambda t: t.sum(dim=dims) if dims else t.sum(), self)

    def mean(self, *dims):
        return self.sd._op(None, lambda t: t.mean(dim=dims) if dims else t.mean(), self)

    def reshape(self, *shape):
        return self.sd._op(None, lambda t: t.reshape(*shape), self)

    def permute(self, *dims):
        return self.sd._op(None, lambda t: t.permute(*dims), self)

    def transpose(self):
        return self.sd._op(None, lambda t: t.transpose(-1, -2), self)

    def get(self, *idx):
        """Python-style indexing / slicing (e.g. ``h.get(slice(None), 0)`` = the first token of every row)."""
        return self.sd._op(None, lambda t: t[idx], self)

    def getShape(self):
        return list(self.value.shape)

    def getArr(self):
        return self.value

    def eval(self):
        return self.value.detach()

    def __repr__(self):
        return f"SDVariable(name={self.name!r}, shape={list(self.value.shape)})"


class _NN:
    def __init__(self, sd):
        self.sd = sd

    def _u(self, name, x, fn):
        if isinstance(name, SDVariable):
            name, x = None, name
        return self.sd._op(name, fn, x)

    def relu(self, name, x=None, cutoff=0.0):
        return self._u(name, x, lambda t: torch.relu(t - cutoff) + cutoff if cutoff else torch.relu(t))

    def sigmoid(self, name, x=None):
        return self._u(name, x, torch.sigmoid)

    def tanh(self, name, x=None):
        return self._u(name, x, torch.tanh)

    def softmax(self, name, x=None):
        return self._u(name, x, lambda t: torch.softmax(t, dim=-1))

    def gelu(self, name, x=None):
        return self._u(name, x, F.gelu)

    def elu(self, name, x=None):
        return self._u(name, x, F.elu)

    def leakyRelu(self, name, x=None, alpha=0.01):
        return self._u(name, x, lambda t: F.leaky_relu(t, alpha))

    def softplus(self, name, x=None):
        return self._u(name, x, F.softplus)

    def linear(self, name, x, w=None, b=None):
        if isinstance(name, SDVariable):
            name, x, w, b = None, name, x, w
        return self.sd._op(name, lambda a, ww, bb: a @ ww if bb is None else a @ ww + bb, x, w, b)

    def layerNorm(self, name, x, gain=None, bias=None, eps=1e-5):
        """LayerNorm over the last dim (LayerNorm HIP kernels on the GPU)."""
        if isinstance(name, SDVariable):
            name, x, gain, bias = None, name, x, gain
        from .native_ops import layer_norm
        return self.sd._op(name, lambda t, g, bb: layer_norm(t, g, bb, eps), x, gain, bias)

    def fusedSelfAttention(self, name, qkv, nHeads, mask=None, causal=False):
        """Multi-head self attention on a fused projection qkv [B, T, 3E] -> [B, T, E] (flash-attention kernel)."""
        if isinstance(name, SDVariable):
            name, qkv, nHeads = None, name, qkv
        from .native_ops import self_attention
        return self.sd._op(name, lambda q, m: self_attention(q, nHeads, m, causal), qkv, mask)


class _RNN:
    def __init__(self, sd):
        self.sd = sd

    def lstmLayer(self, name, x, W, RW, b, h0=None, c0=None, peephole=False):
        """Whole-sequence LSTM (DL4J gate order, tanh/sigmoid): x [mb, nIn, T] -> [mb, H, T]. Runs the fused
        sequence HIP kernels on the GPU (csrc/lstm.hip); RW has 3 extra peephole columns when ``peephole``."""
        from .native_ops import lstm_layer
        return self.sd._op(name, lambda x_, w_, rw_, b_, h_, c_: lstm_layer(x_, w_, rw_, b_, h_, c_, peephole),
                           x, W, RW, b, h0, c0)


class _CNN:
    def __init__(self, sd):
        self.sd = sd

    def conv2d(self, name, x, w, b=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1)):
        if isinstance(name, SDVariable):
            name, x, w, b = None, name, x, w
        return self.sd._op(name, lambda t, ww, bb: F.conv2d(t, ww, None if bb is None else bb.reshape(-1), tuple(stride),
                                                            tuple(padding), tuple(dilation)), x, w, b)

    def maxPooling2d(self, name, x, kernel, stride, padding=(0, 0)):
        return self.sd._op(name, lambda t: F.max_pool2d(t, kernel, stride, padding), x)

    def avgPooling2d(self, name, x, kernel, stride, padding=(0, 0)):
        return self.sd._op(name, lambda t: F.avg_pool2d(t, kernel, stride, padding), x)


class _Loss:
    """``sd.loss()``: reduced (mean over the minibatch) losses, registered as loss variables."""

    def __init__(self, sd):
        self.sd = sd

    def _reg(self, v):
        self.sd._loss_names.append(v.name)
        return v

    def softmaxCrossEntropy(self, name, labels, logits, weights=None, labelSmoothing=0.0):
        """Softmax over the last dimension of ``logits``; labels one-hot (or soft) of the same shape."""
        def f(y, z):
            if labelSmoothing:
                y = y * (1 - labelSmoothing) + labelSmoothing / y.shape[-1]
            lp = torch.log_softmax(z.float(), dim=-1)
            return -(y.float() * lp).sum(-1).mean()
        return self._reg(self.sd._op(name, f, labels, logits))

    def meanSquaredError(self, name, labels, predictions, weights=None):
        return self._reg(self.sd._op(name, lambda y, z: ((z.float() - y.float()) ** 2).mean(), labels, predictions))

    def logLoss(self, name, labels, predictions, weights=None, epsilon=1e-7):
        def f(y, p):
            p = p.float().clamp(epsilon, 1 - epsilon)
            return -(y * torch.log(p) + (1 - y) * torch.log(1 - p)).mean()
        return self._reg(self.sd._op(name, f, labels, predictions))


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
    """Define-by-run graph that also RECORDS every op: the values are computed eagerly on PyTorch-ROCm tensors (so
    ``execBackwards`` / ``eval`` work immediately, as in SameDiff layers), and the recorded op list can be replayed
    for new placeholder values (``output``) or trained (``setTrainingConfig`` + ``fit``; backward by autograd over the
    replayed ops, one fused HIP updater launch over all trainable variables)."""

    def __init__(self):
        self.variables = {}
        self._n = 0
        self._ops = []                  # (output name, fn, args) in definition order
        self._placeholders = []
        self._trainable = []
        self._loss_names = []
        self.trainingConfig = None
        self._train_state = None
        self.iterationCount = 0
        self.epochCount = 0

    @staticmethod
    def create():
        return SameDiff()

    def _new(self, name, value):
        if name is None:
            self._n += 1
            name = f"sd_var_{self._n}"
        v = SDVariable(self, name, value)
        self.variables[name] = v
        return v

    def _op(self, name, fn, *args):
        vals = [a.value if isinstance(a, SDVariable) else a for a in args]
        v = self._new(name, fn(*vals))
        self._ops.append((v.name, fn, args))
        return v

    def var(self, name, value):
        if not torch.is_tensor(value):
            value = torch.as_tensor(value)
        v = self._new(name, value)
        self._trainable.append(v.name)
        return v

    def placeHolder(self, name, value=None, *shape):
        """placeHolder(name, exampleValue) or placeHolder(name, dtype, *shape): a graph input fed by ``output`` /
        ``fit``. A shape (with -1 for the minibatch) creates a zero example value for eager definition."""
        if value is None or not torch.is_tensor(value):
            dims = [1 if d is None or d < 0 else int(d) for d in shape] if shape else [1]
            dt = value if isinstance(value, torch.dtype) else torch.float32
            value = torch.zeros(dims, dtype=dt)
        v = self._new(name, value)
        self._placeholders.append(v.name)
        return v

    def constant(self, name, value):
        return self._new(name, torch.as_tensor(value).detach())

    def loss(self):
        return _Loss(self)

    def setLossVariables(self, *names):
        self._loss_names = [n.name if isinstance(n, SDVariable) else n for n in names]

    def getLossVariables(self):
        return list(self._loss_names)

    def trainableVariables(self):
        return [self.variables[n] for n in self._trainable]

    # ------------------------------------------------------------------ replay
    def _replay(self, feeds, targets=None):
        """Re-run the recorded ops (only those ``targets`` depend on, when given) with new placeholder values."""
        for k, v in feeds.items():
            self.variables[k].value = v
        ops = self._ops
        if targets is not None:
            need = set(targets)
            keep = []
            for name, fn, args in reversed(self._ops):
                if name in need:
                    keep.append((name, fn, args))
                    need.update(a.name for a in args if isinstance(a, SDVariable))
            ops = keep[::-1]
        for name, fn, args in ops:
            vals = [self.variables[a.name].value if isinstance(a, SDVariable) else a for a in args]
            self.variables[name].value = fn(*vals)

    def output(self, placeholders, *outputs):
        """Replay the recorded graph for new placeholder values; returns {name: value}."""
        names = [o.name if isinstance(o, SDVariable) else o for o in outputs]
        with torch.no_grad():
            self._replay({k: _tensor(v) for k, v in placeholders.items()}, names)
        return {n: self.variables[n].value for n in names}

    def outputSingle(self, placeholders, output):
        return next(iter(self.output(placeholders, output).values()))

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
        flat = torch.empty(n, dtype=torch.float32, device=dev)
        # bf16 variables train in mixed precision: fp32 master weights, the fused updater writes the bf16 copy the
        # graph computes with (its "shadow") in the same pass
        mixed = all(v.value.dtype == torch.bfloat16 for v in vs)
        shadow = torch.empty(n, dtype=torch.bfloat16, device=dev) if mixed else None
        segs, off = [], 0
        for i, v in enumerate(vs):
            k = v.value.numel()
            flat[off:off + k].copy_(v.value.detach().reshape(-1).float())
            if mixed:
                shadow[off:off + k].copy_(v.value.detach().reshape(-1))
                v.value = shadow[off:off + k].view(v.value.shape)
            else:
                v.value = flat[off:off + k].view(v.value.shape)
            segs.append(Segment(off, k, 0, off, n, cfg.updater, cfg.l1, cfg.l2, 0))   # one block: state offset 0
            off += k
        state = torch.zeros(max(1, cfg.updater.stateSize(n)), dtype=torch.float32, device=dev)
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
                for v in vs:
                    v.value.requires_grad_(True)
                with torch.enable_grad():
                    self._replay(feeds, self._loss_names)
                    loss = sum(self.variables[n].value.float() for n in self._loss_names)
                    if not cfg.minimize:
                        loss = -loss
                    grads = torch.autograd.grad(loss, [v.value for v in vs], allow_unused=True)
                with torch.no_grad():
                    off = 0
                    for v, g in zip(vs, grads):
                        k = v.value.numel()
                        if g is None:
                            st["grad"][off:off + k].zero_()
                        else:
                            st["grad"][off:off + k].copy_(g.reshape(-1))
                        off += k
                    for v in vs:
                        v.value.requires_grad_(False)
                    fused_update(st["plan"], st["flat"], st["grad"], st["state"], self.iterationCount,
                                 self.epochCount, 1, mini_batch=False, shadow=st["shadow"])
                self.iterationCount += 1
                last = float(loss.detach())
            self.epochCount += 1
        return last

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
        return self._op(name, torch.matmul, a, b)

    def _u(self, name, x, fn):
        if isinstance(name, SDVariable):
            name, x = None, name
        return self._op(name, fn, x)

    def sigmoid(self, name, x=None):
        return self._u(name, x, torch.sigmoid)

    def tanh(self, name, x=None):
        return self._u(name, x, torch.tanh)

    def relu(self, name, x=None, cutoff=0.0):
        return self._u(name, x, torch.relu)

    def softmax(self, name, x=None):
        return self._u(name, x, lambda t: torch.softmax(t, dim=-1))

    def exp(self, name, x=None):
        return self._u(name, x, torch.exp)

    def log(self, name, x=None):
        return self._u(name, x, torch.log)

    def sqrt(self, name, x=None):
        return self._u(name, x, torch.sqrt)

    def square(self, name, x=None):
        return self._u(name, x, torch.square)

    def abs(self, name, x=None):
        return self._u(name, x, torch.abs)

    def neg(self, name, x=None):
        return self._u(name, x, torch.neg)

    def identity(self, name, x=None):
        return self._u(name, x, lambda t: t)

    def sum(self, name, x, *dims):
        return self._op(name, lambda t: t.sum(dim=dims) if dims else t.sum(), x)

    def mean(self, name, x, *dims):
        return self._op(name, lambda t: t.mean(dim=dims) if dims else t.mean(), x)

    def gather(self, name, params, indices, axis=0):
        """Rows of ``params`` selected by integer ``indices`` (embedding lookup when axis == 0)."""
        if axis == 0:
            return self._op(name, lambda p, i: torch.nn.functional.embedding(i.long(), p), params, indices)
        return self._op(name, lambda p, i: torch.index_select(p, axis, i.long().reshape(-1)), params, indices)

    def concat(self, name, dim, *xs):
        return self._op(name, lambda *ts: torch.cat(ts, dim=dim), *xs)

    def activation(self, name, act, x):
        from ..nn.conf.activations import to_activation
        a = to_activation(act)
        return self._op(name, lambda t: a.getActivation(t, True), x)

    def execAndEndResult(self, out):
        return out.value.detach()

    def execBackwards(self, loss, wrt):
        grads = torch.autograd.grad(loss.value, [w.value for w in wrt], allow_unused=True)
        return {w.name: g for w, g in zip(wrt, grads)}


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
