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
        o = other.value if isinstance(other, SDVariable) else other
        return self.sd._new(name, fn(self.value, o))

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
        return self.sd._new(None, -self.value)

    # ------------------------------------------------------------ reductions / shape
    def sum(self, *dims):
        return self.sd._new(None, self.value.sum(dim=dims) if dims else self.value.sum())

    def mean(self, *dims):
        return self.sd._new(None, self.value.mean(dim=dims) if dims else self.value.mean())

    def reshape(self, *shape):
        return self.sd._new(None, self.value.reshape(*shape))

    def permute(self, *dims):
        return self.sd._new(None, self.value.permute(*dims))

    def transpose(self):
        return self.sd._new(None, self.value.transpose(-1, -2))

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
        return self.sd._new(name, fn(x.value))

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
        out = x.value @ w.value
        if b is not None:
            out = out + b.value
        return self.sd._new(name, out)

    def layerNorm(self, name, x, gain=None, bias=None, eps=1e-5):
        """LayerNorm over the last dim (LayerNorm HIP kernels on the GPU)."""
        if isinstance(name, SDVariable):
            name, x, gain, bias = None, name, x, gain
        from .native_ops import layer_norm
        out = layer_norm(x.value, gain.value if gain is not None else None, bias.value if bias is not None else None,
                         eps)
        return self.sd._new(name, out)

    def fusedSelfAttention(self, name, qkv, nHeads, mask=None, causal=False):
        """Multi-head self attention on a fused projection qkv [B, T, 3E] -> [B, T, E] (flash-attention kernel)."""
        if isinstance(name, SDVariable):
            name, qkv, nHeads = None, name, qkv
        from .native_ops import self_attention
        m = mask.value if isinstance(mask, SDVariable) else mask
        return self.sd._new(name, self_attention(qkv.value, nHeads, m, causal))


class _RNN:
    def __init__(self, sd):
        self.sd = sd

    def lstmLayer(self, name, x, W, RW, b, h0=None, c0=None, peephole=False):
        """Whole-sequence LSTM (DL4J gate order, tanh/sigmoid): x [mb, nIn, T] -> [mb, H, T]. Runs the fused
        sequence HIP kernels on the GPU (csrc/lstm.hip); RW has 3 extra peephole columns when ``peephole``."""
        from .native_ops import lstm_layer
        v = lambda t: None if t is None else t.value  # noqa: E731
        return self.sd._new(name, lstm_layer(x.value, W.value, RW.value, b.value, v(h0), v(c0), peephole))


class _CNN:
    def __init__(self, sd):
        self.sd = sd

    def conv2d(self, name, x, w, b=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1)):
        if isinstance(name, SDVariable):
            name, x, w, b = None, name, x, w
        out = F.conv2d(x.value, w.value, None if b is None else b.value.reshape(-1), tuple(stride),
                       tuple(padding), tuple(dilation))
        return self.sd._new(name, out)

    def maxPooling2d(self, name, x, kernel, stride, padding=(0, 0)):
        return self.sd._new(name, F.max_pool2d(x.value, kernel, stride, padding))

    def avgPooling2d(self, name, x, kernel, stride, padding=(0, 0)):
        return self.sd._new(name, F.avg_pool2d(x.value, kernel, stride, padding))


class SameDiff:
    """Eager op recorder. Variables are torch tensors that carry autograd history."""

    def __init__(self):
        self.variables = {}
        self._n = 0

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

    def var(self, name, value):
        if not torch.is_tensor(value):
            value = torch.as_tensor(value)
        return self._new(name, value)

    placeHolder = var

    def constant(self, name, value):
        return self._new(name, torch.as_tensor(value).detach())

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
        return self._new(name, a.value @ b.value)

    def _u(self, name, x, fn):
        if isinstance(name, SDVariable):
            name, x = None, name
        return self._new(name, fn(x.value))

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
        return self._new(name, x.value.sum(dim=dims) if dims else x.value.sum())

    def mean(self, name, x, *dims):
        return self._new(name, x.value.mean(dim=dims) if dims else x.value.mean())

    def concat(self, name, dim, *xs):
        return self._new(name, torch.cat([x.value for x in xs], dim=dim))

    def activation(self, name, act, x):
        from ..nn.conf.activations import to_activation
        return self._new(name, to_activation(act).getActivation(x.value, True))

    def execAndEndResult(self, out):
        return out.value.detach()

    def execBackwards(self, loss, wrt):
        grads = torch.autograd.grad(loss.value, [w.value for w in wrt], allow_unused=True)
        return {w.name: g for w, g in zip(wrt, grads)}


def _as_samediff(self, name, sd, x):
    """Activation.X.asSameDiff(name, sd, x) (reference Activation.asSameDiff)."""
    return sd.activation(name, self, x)


def _install():
    from ..nn.conf.activations import Activation, IActivation
    Activation.asSameDiff = _as_samediff
    IActivation.asSameDiff = _as_samediff


_install()

__all__ = ["SameDiff", "SDVariable"]
