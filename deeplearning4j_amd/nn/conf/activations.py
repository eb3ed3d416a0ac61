"""Activation functions (ND4J IActivation equivalents) with explicit forward and backprop.

Reference usage: every layer calls ``IActivation.getActivation(z, training)`` forward and
``IActivation.backprop(z, epsilon)`` backward (reference nn/layers/BaseLayer.java:334-336,
nn/layers/BaseOutputLayer.java:173); the enum ``Activation`` maps names to instances.
Elementwise activations run as torch elementwise kernels unless fused into a producer by the
HIP path (BN+ReLU, GEMM epilogues — see ``deeplearning4j_amd.ops``).
"""
import math
from enum import Enum

import torch

from .base import Config, register_enum
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


def _kf(x, op, a0=0.0, a1=0.0):
    """GPU tensors (fp32 / bf16 / fp16, not tracked by autograd) run the ND4J transform kernel
    (csrc/nd4j_ops.hip); anything else returns None and the torch expression below is used."""
    if not (torch.is_tensor(x) and x.is_cuda):
        return None
    from deeplearning4j_amd.ops import nd4j_kernels
    return nd4j_kernels.transform(x, op, a0, a1)


def _kb(z, eps, op, a0=0.0):
    if not (torch.is_tensor(z) and z.is_cuda and torch.is_tensor(eps) and eps.dtype == z.dtype):
        return None
    from deeplearning4j_amd.ops import nd4j_kernels
    return nd4j_kernels.transform_bp(z, eps, op, a0)


class IActivation(Config):
    def getActivation(self, x, training=False):
        raise NotImplementedError

    def backprop(self, z, epsilon):
        """dL/dz given pre-activation z and dL/d(activation)."""
        raise NotImplementedError

    def __call__(self, x, training=False):
        return self.getActivation(x, training)

    def __str__(self):
        """The ND4J toString form: the lower-case activation name, with parameters when it has any
        (``sigmoid``, ``hardsigmoid``, ``leakyrelu(alpha=0.01)``)."""
        name = next((e.value.lower() for e, c in _ACT_MAP.items() if c is type(self)), type(self).__name__)
        f = self._all_fields()
        return name + ("(" + ", ".join(f"{k}={getattr(self, k)}" for k in f) + ")" if f else "")


class ActivationIdentity(IActivation):
    def getActivation(self, x, training=False):
        return x

    def backprop(self, z, epsilon):
        return epsilon


class ActivationReLU(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "relu", 0.0)
        if r is not None:
            return r
        return torch.relu(x)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "relu", 0.0)
        if r is not None:
            return r
        return torch.where(z > 0, epsilon, torch.zeros((), dtype=epsilon.dtype, device=epsilon.device))


class ActivationReLU6(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "relu6", 0.0)
        if r is not None:
            return r
        return torch.clamp(x, 0.0, 6.0)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "relu6", 0.0)
        if r is not None:
            return r
        return epsilon * ((z > 0) & (z < 6)).to(epsilon.dtype)


class ActivationLReLU(IActivation):
    FIELDS = {"alpha": 0.01}

    def __str__(self):
        return f"leakyrelu(a={self.alpha})"          # ND4J ActivationLReLU.toString

    def getActivation(self, x, training=False):
        r = _kf(x, "leakyrelu", self.alpha)
        if r is not None:
            return r
        return torch.nn.functional.leaky_relu(x, self.alpha)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "leakyrelu", self.alpha)
        if r is not None:
            return r
        return torch.where(z > 0, epsilon, epsilon * self.alpha)


class ActivationRReLU(IActivation):
    """Randomized leaky ReLU: slope ~ U(l, u) when training, (l+u)/2 at inference."""
    FIELDS = {"l": 1.0 / 8, "u": 1.0 / 3}

    def getActivation(self, x, training=False):
        if training:
            self._alpha = torch.empty_like(x).uniform_(self.l, self.u)
        else:
            self._alpha = (self.l + self.u) / 2
        return torch.where(x >= 0, x, x * self._alpha)

    def backprop(self, z, epsilon):
        a = getattr(self, "_alpha", (self.l + self.u) / 2)
        return torch.where(z >= 0, epsilon, epsilon * a)


class ActivationELU(IActivation):
    FIELDS = {"alpha": 1.0}

    def getActivation(self, x, training=False):
        r = _kf(x, "elu", self.alpha)
        if r is not None:
            return r
        return torch.nn.functional.elu(x, self.alpha)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "elu", self.alpha)
        if r is not None:
            return r
        return torch.where(z > 0, epsilon, epsilon * self.alpha * torch.exp(z))


class ActivationSELU(IActivation):
    A = 1.6732632423543772848170429916717
    S = 1.0507009873554804934193349852946

    def getActivation(self, x, training=False):
        r = _kf(x, "selu", 0.0)
        if r is not None:
            return r
        return torch.selu(x)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "selu", 0.0)
        if r is not None:
            return r
        return epsilon * torch.where(z > 0, torch.full_like(z, self.S), self.S * self.A * torch.exp(z))


class ActivationSigmoid(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "sigmoid", 0.0)
        if r is not None:
            return r
        return torch.sigmoid(x)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "sigmoid", 0.0)
        if r is not None:
            return r
        s = torch.sigmoid(z)
        return epsilon * s * (1 - s)


class ActivationHardSigmoid(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "hardsigmoid", 0.0)
        if r is not None:
            return r
        return torch.clamp(0.2 * x + 0.5, 0.0, 1.0)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "hardsigmoid", 0.0)
        if r is not None:
            return r
        return epsilon * (0.2 * ((z > -2.5) & (z < 2.5)).to(epsilon.dtype))


class ActivationTanH(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "tanh", 0.0)
        if r is not None:
            return r
        return torch.tanh(x)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "tanh", 0.0)
        if r is not None:
            return r
        t = torch.tanh(z)
        return epsilon * (1 - t * t)


class ActivationHardTanH(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "hardtanh", 0.0)
        if r is not None:
            return r
        return torch.clamp(x, -1.0, 1.0)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "hardtanh", 0.0)
        if r is not None:
            return r
        return epsilon * ((z > -1) & (z < 1)).to(epsilon.dtype)


class ActivationRationalTanh(IActivation):
    """f(x) = 1.7159 * tanh_approx(2x/3), tanh_approx(y) = sgn(y)(1 - 1/(1+|y|+y^2+1.41645 y^4))."""

    def getActivation(self, x, training=False):
        r = _kf(x, "rationaltanh", 0.0)
        if r is not None:
            return r
        y = 2.0 * x / 3.0
        a = torch.abs(y)
        return 1.7159 * torch.sign(y) * (1 - 1 / (1 + a + y * y + 1.41645 * y ** 4))

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "rationaltanh", 0.0)
        if r is not None:
            return r
        y = 2.0 * z / 3.0
        a = torch.abs(y)
        d = 1 + a + y * y + 1.41645 * y ** 4
        dd = (1 + 2 * a + 4 * 1.41645 * a ** 3) / (d * d)
        return epsilon * 1.7159 * (2.0 / 3.0) * dd


class ActivationRectifiedTanh(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "rectifiedtanh", 0.0)
        if r is not None:
            return r
        return torch.clamp(torch.tanh(x), min=0)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "rectifiedtanh", 0.0)
        if r is not None:
            return r
        t = torch.tanh(z)
        return torch.where(z > 0, epsilon * (1 - t * t), torch.zeros_like(epsilon))


class ActivationSoftPlus(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "softplus", 0.0)
        if r is not None:
            return r
        return torch.nn.functional.softplus(x)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "softplus", 0.0)
        if r is not None:
            return r
        return epsilon * torch.sigmoid(z)


class ActivationSoftSign(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "softsign", 0.0)
        if r is not None:
            return r
        return x / (1 + torch.abs(x))

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "softsign", 0.0)
        if r is not None:
            return r
        d = 1 + torch.abs(z)
        return epsilon / (d * d)


class ActivationCube(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "cube", 0.0)
        if r is not None:
            return r
        return x * x * x

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "cube", 0.0)
        if r is not None:
            return r
        return epsilon * 3 * z * z


class ActivationSwish(IActivation):
    def getActivation(self, x, training=False):
        r = _kf(x, "swish", 0.0)
        if r is not None:
            return r
        return x * torch.sigmoid(x)

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "swish", 0.0)
        if r is not None:
            return r
        s = torch.sigmoid(z)
        return epsilon * (s + z * s * (1 - s))


class ActivationGELU(IActivation):
    """GELU (tanh approximation) — beyond the reference snapshot, needed for the BERT config."""
    FIELDS = {"precise": False}

    def getActivation(self, x, training=False):
        r = _kf(x, "gelu" if self.precise else "gelu_tanh")
        if r is not None:
            return r
        return torch.nn.functional.gelu(x, approximate="none" if self.precise else "tanh")

    def backprop(self, z, epsilon):
        r = _kb(z, epsilon, "gelu" if self.precise else "gelu_tanh")
        if r is not None:
            return r
        if self.precise:
            cdf = 0.5 * (1 + torch.erf(z / math.sqrt(2)))
            pdf = torch.exp(-0.5 * z * z) / math.sqrt(2 * math.pi)
            return epsilon * (cdf + z * pdf)
        c = math.sqrt(2 / math.pi)
        inner = c * (z + 0.044715 * z ** 3)
        t = torch.tanh(inner)
        return epsilon * (0.5 * (1 + t) + 0.5 * z * (1 - t * t) * c * (1 + 3 * 0.044715 * z * z))


class ActivationSoftmax(IActivation):
    """Row softmax over dimension 1 (reference: ND4J OldSoftMax along dim 1)."""

    def getActivation(self, x, training=False):
        return torch.softmax(_acc(x), dim=1).to(x.dtype)

    def backprop(self, z, epsilon):
        s = torch.softmax(_acc(z), dim=1)
        e = _acc(epsilon)
        return (s * (e - (e * s).sum(dim=1, keepdim=True))).to(epsilon.dtype)


@register_enum
class Activation(Enum):
    CUBE = "CUBE"
    ELU = "ELU"
    HARDSIGMOID = "HARDSIGMOID"
    HARDTANH = "HARDTANH"
    IDENTITY = "IDENTITY"
    LEAKYRELU = "LEAKYRELU"
    RATIONALTANH = "RATIONALTANH"
    RELU = "RELU"
    RELU6 = "RELU6"
    RRELU = "RRELU"
    SIGMOID = "SIGMOID"
    SOFTMAX = "SOFTMAX"
    SOFTPLUS = "SOFTPLUS"
    SOFTSIGN = "SOFTSIGN"
    TANH = "TANH"
    RECTIFIEDTANH = "RECTIFIEDTANH"
    SELU = "SELU"
    SWISH = "SWISH"
    GELU = "GELU"

    def getActivationFunction(self):
        return _ACT_MAP[self]()

    @staticmethod
    def fromString(s):
        return Activation[s.upper()]


_ACT_MAP = {
    Activation.CUBE: ActivationCube, Activation.ELU: ActivationELU,
    Activation.HARDSIGMOID: ActivationHardSigmoid, Activation.HARDTANH: ActivationHardTanH,
    Activation.IDENTITY: ActivationIdentity, Activation.LEAKYRELU: ActivationLReLU,
    Activation.RATIONALTANH: ActivationRationalTanh, Activation.RELU: ActivationReLU,
    Activation.RELU6: ActivationReLU6, Activation.RRELU: ActivationRReLU,
    Activation.SIGMOID: ActivationSigmoid, Activation.SOFTMAX: ActivationSoftmax,
    Activation.SOFTPLUS: ActivationSoftPlus, Activation.SOFTSIGN: ActivationSoftSign,
    Activation.TANH: ActivationTanH, Activation.RECTIFIEDTANH: ActivationRectifiedTanh,
    Activation.SELU: ActivationSELU, Activation.SWISH: ActivationSwish, Activation.GELU: ActivationGELU,
}


def to_activation(a):
    """Accept an Activation enum, an IActivation instance or a name string."""
    if a is None or isinstance(a, IActivation):
        return a
    if isinstance(a, Activation):
        return a.getActivationFunction()
    if isinstance(a, str):
        return Activation.fromString(a).getActivationFunction()
    raise TypeError(f"Cannot convert {a!r} to an activation")
