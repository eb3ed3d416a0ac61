"""Weight initialisation schemes and distributions.

Reference: nn/weights/WeightInit.java:68-71, nn/weights/WeightInitUtil.java:64-144 (formulas below are
the same), nn/conf/distribution/*.java.  Initialisation fills a view of the flat parameter vector
in place (no copies), as WeightInitUtil does.
"""
import math
from enum import Enum

import torch

from .base import Config, register_enum


def _jdouble(v):
    """Java's Double.toString of v (0.0, 1.0, 0.5, 1.0E-8)."""
    v = float(v)
    if v == int(v) and abs(v) < 1e7:
        return f"{v:.1f}"
    if 1e-3 <= abs(v) < 1e7:
        return repr(v)
    m, e = f"{v:.16e}".split("e")
    m = m.rstrip("0")
    m = m + "0" if m.endswith(".") else m
    return f"{m}E{int(e)}"


class Distribution(Config):
    def sample_(self, t, gen=None):
        raise NotImplementedError

    def __str__(self):
        """The reference's toString: ``NormalDistribution{mean=0.0, std=1.0}`` (nn/conf/distribution/*.java)."""
        parts = []
        for k, d in self.FIELDS.items():
            v = getattr(self, k)
            parts.append(f"{k}={_jdouble(v) if isinstance(d, float) else v}")
        return f"{type(self).__name__}{{{', '.join(parts)}}}"


class NormalDistribution(Distribution):
    FIELDS = {"mean": 0.0, "std": 1.0}

    def __init__(self, mean=0.0, std=1.0, **kw):
        super().__init__(mean=mean, std=std, **kw)

    def sample_(self, t, gen=None):
        return t.normal_(self.mean, self.std, generator=gen)


class GaussianDistribution(NormalDistribution):
    pass


class UniformDistribution(Distribution):
    FIELDS = {"lower": 0.0, "upper": 1.0}

    def __init__(self, lower=0.0, upper=1.0, **kw):
        super().__init__(lower=lower, upper=upper, **kw)

    def sample_(self, t, gen=None):
        return t.uniform_(self.lower, self.upper, generator=gen)


class ConstantDistribution(Distribution):
    FIELDS = {"value": 0.0}

    def __init__(self, value=0.0, **kw):
        super().__init__(value=value, **kw)

    def sample_(self, t, gen=None):
        return t.fill_(self.value)


class BinomialDistribution(Distribution):
    FIELDS = {"numberOfTrials": 1, "probabilityOfSuccess": 0.5}

    def __init__(self, numberOfTrials=1, probabilityOfSuccess=0.5, **kw):
        super().__init__(numberOfTrials=numberOfTrials, probabilityOfSuccess=probabilityOfSuccess, **kw)

    def sample_(self, t, gen=None):
        p = torch.full(t.shape, self.probabilityOfSuccess, dtype=torch.float64)
        s = torch.distributions.Binomial(self.numberOfTrials, p).sample()
        return t.copy_(s)


class LogNormalDistribution(Distribution):
    FIELDS = {"mean": 0.0, "std": 1.0}

    def __init__(self, mean=0.0, std=1.0, **kw):
        super().__init__(mean=mean, std=std, **kw)

    def sample_(self, t, gen=None):
        return t.log_normal_(self.mean, self.std, generator=gen)


class TruncatedNormalDistribution(Distribution):
    FIELDS = {"mean": 0.0, "std": 1.0}

    def __init__(self, mean=0.0, std=1.0, **kw):
        super().__init__(mean=mean, std=std, **kw)

    def sample_(self, t, gen=None):
        tmp = torch.empty(t.shape, dtype=torch.float32)
        torch.nn.init.trunc_normal_(tmp, self.mean, self.std, self.mean - 2 * self.std, self.mean + 2 * self.std,
                                    generator=gen)
        return t.copy_(tmp)


class OrthogonalDistribution(Distribution):
    FIELDS = {"gain": 1.0}

    def __init__(self, gain=1.0, **kw):
        super().__init__(gain=gain, **kw)

    def sample_(self, t, gen=None):
        tmp = torch.empty(t.shape if t.dim() >= 2 else (1, t.numel()), dtype=torch.float32)
        torch.nn.init.orthogonal_(tmp, self.gain, generator=gen)
        return t.copy_(tmp.reshape(t.shape))


@register_enum
class WeightInit(Enum):
    DISTRIBUTION = "DISTRIBUTION"
    ZERO = "ZERO"
    ONES = "ONES"
    SIGMOID_UNIFORM = "SIGMOID_UNIFORM"
    NORMAL = "NORMAL"
    LECUN_NORMAL = "LECUN_NORMAL"
    UNIFORM = "UNIFORM"
    XAVIER = "XAVIER"
    XAVIER_UNIFORM = "XAVIER_UNIFORM"
    XAVIER_FAN_IN = "XAVIER_FAN_IN"
    XAVIER_LEGACY = "XAVIER_LEGACY"
    RELU = "RELU"
    RELU_UNIFORM = "RELU_UNIFORM"
    IDENTITY = "IDENTITY"
    LECUN_UNIFORM = "LECUN_UNIFORM"
    VAR_SCALING_NORMAL_FAN_IN = "VAR_SCALING_NORMAL_FAN_IN"
    VAR_SCALING_NORMAL_FAN_OUT = "VAR_SCALING_NORMAL_FAN_OUT"
    VAR_SCALING_NORMAL_FAN_AVG = "VAR_SCALING_NORMAL_FAN_AVG"
    VAR_SCALING_UNIFORM_FAN_IN = "VAR_SCALING_UNIFORM_FAN_IN"
    VAR_SCALING_UNIFORM_FAN_OUT = "VAR_SCALING_UNIFORM_FAN_OUT"
    VAR_SCALING_UNIFORM_FAN_AVG = "VAR_SCALING_UNIFORM_FAN_AVG"


def init_weights_(view, fan_in, fan_out, shape, scheme, dist=None, gen=None):
    """Fill ``view`` (any shape, numel == prod(shape)) in place. Sampling happens in fp32 on the host
    generator for reproducibility across devices, then copies into the (device) view."""
    scheme = WeightInit[scheme] if isinstance(scheme, str) else scheme
    n = view.numel()
    tmp = torch.empty(n, dtype=torch.float64 if view.dtype == torch.float64 else torch.float32)

    def U(a):
        tmp.uniform_(-a, a, generator=gen)

    def N(std):
        tmp.normal_(0.0, std, generator=gen)

    W = WeightInit
    if scheme == W.DISTRIBUTION:
        if dist is None:
            raise ValueError("WeightInit.DISTRIBUTION requires a distribution (dist)")
        dist.sample_(tmp, gen)
    elif scheme == W.RELU:
        N(math.sqrt(2.0 / fan_in))
    elif scheme == W.RELU_UNIFORM:
        U(math.sqrt(6.0 / fan_in))
    elif scheme == W.SIGMOID_UNIFORM:
        U(4.0 * math.sqrt(6.0 / (fan_in + fan_out)))
    elif scheme == W.UNIFORM:
        U(1.0 / math.sqrt(fan_in))
    elif scheme == W.LECUN_UNIFORM:
        U(3.0 / math.sqrt(fan_in))
    elif scheme == W.XAVIER:
        N(math.sqrt(2.0 / (fan_in + fan_out)))
    elif scheme == W.XAVIER_UNIFORM:
        U(math.sqrt(6.0) / math.sqrt(fan_in + fan_out))
    elif scheme in (W.LECUN_NORMAL, W.NORMAL, W.XAVIER_FAN_IN, W.VAR_SCALING_NORMAL_FAN_IN):
        N(1.0 / math.sqrt(fan_in))
    elif scheme == W.XAVIER_LEGACY:
        N(1.0 / math.sqrt(shape[0] + shape[1]))
    elif scheme == W.ZERO:
        tmp.zero_()
    elif scheme == W.ONES:
        tmp.fill_(1.0)
    elif scheme == W.IDENTITY:
        if len(shape) != 2 or shape[0] != shape[1]:
            raise ValueError(f"Cannot use IDENTITY init with parameters of shape {shape}")
        tmp.copy_(torch.eye(shape[0]).reshape(-1))
    elif scheme == W.VAR_SCALING_NORMAL_FAN_OUT:
        N(1.0 / math.sqrt(fan_out))
    elif scheme == W.VAR_SCALING_NORMAL_FAN_AVG:
        N(1.0 / math.sqrt((fan_in + fan_out) / 2))
    elif scheme == W.VAR_SCALING_UNIFORM_FAN_IN:
        U(3.0 / math.sqrt(fan_in))
    elif scheme == W.VAR_SCALING_UNIFORM_FAN_OUT:
        U(3.0 / math.sqrt(fan_out))
    elif scheme == W.VAR_SCALING_UNIFORM_FAN_AVG:
        U(3.0 / math.sqrt((fan_in + fan_out) / 2))
    else:
        raise ValueError(f"Illegal weight init value: {scheme}")
    with torch.no_grad():
        view.copy_(tmp.reshape(view.shape).to(view.dtype))
    return view


def to_weight_init(w):
    if w is None or isinstance(w, WeightInit):
        return w
    return WeightInit[str(w).upper()]


class WeightInitUtil:
    """Reference nn/weights/WeightInitUtil.java: ``initWeights(fanIn, fanOut, shape, WeightInit, Distribution,
    params[, order])`` fills the given array (a view, e.g. into the flat parameter vector) in place and returns it
    reshaped to ``shape``. The random stream is the framework's generator (``Nd4j.getRandom()`` seeds it), so the same
    seed gives the same weights as an explicit sample of the scheme's distribution with that seed."""

    DEFAULT_WEIGHT_INIT_ORDER = "f"

    @staticmethod
    def initWeights(fanIn, fanOut, shape, initScheme, dist, params, order="f"):
        shape = [int(v) for v in shape]
        if params.numel() != int(math.prod(shape)):
            raise ValueError(f"params length {params.numel()} does not match shape {shape}")
        gen = _default_generator()
        flat = params.reshape(-1)
        init_weights_(flat, fanIn, fanOut, shape, initScheme, dist, gen)
        if order == "f":
            return flat.reshape(list(reversed(shape))).permute(*reversed(range(len(shape))))
        return flat.reshape(shape)


def _default_generator():
    """The ND4J facade's process-wide generator (``Nd4j.getRandom().setSeed`` seeds it)."""
    from ...nd4j.factory import _Random
    return _Random.gen()
