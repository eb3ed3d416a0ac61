"""Loss functions (ND4J ILossFunction equivalents).

Contract (reference nn/layers/BaseOutputLayer.java:82-92,147-178):
  * ``computeScoreArray(labels, preOut, activationFn, mask)`` -> per-example score [mb]
  * ``computeScore(..., average)`` -> sum over examples (divided by mb when ``average``)
  * ``computeGradient(labels, preOut, activationFn, mask)`` -> dL/dpreOut, **per example, not divided
    by the minibatch size** (the updater divides by the batch size afterwards, reference
    nn/updater/BaseMultiLayerUpdater.java:296-308).
MCXENT / NLL with a softmax activation and XENT with sigmoid use the fused ``output - labels``
gradient, and on the GPU the fused softmax-cross-entropy HIP kernel (``ops.softmax_xent``).
"""
from enum import Enum

import torch

from .activations import ActivationSigmoid, ActivationSoftmax, IActivation, to_activation
from .base import Config, register_enum
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


def _apply_mask(arr, mask):
    if mask is None:
        return arr
    m = mask.to(arr.dtype)
    if m.dim() == 1 or (m.dim() == 2 and m.shape[1] == 1 and arr.shape[1] != 1):
        m = m.reshape(-1, *([1] * (arr.dim() - 1)))
    return arr * m


class ILossFunction(Config):
    FIELDS = {"weights": None}

    def _w(self, ref):
        if self.weights is None:
            return None
        w = self.weights
        if not torch.is_tensor(w):
            w = torch.tensor(w)
        return w.to(ref.device, ref.dtype).reshape(1, -1)

    def scoreArray(self, labels, output):
        """Per-element score (pre-sum) from the activated output."""
        raise NotImplementedError

    def gradOutput(self, labels, output):
        """dL/d(output) (pre activation-backprop)."""
        raise NotImplementedError

    def computeScoreArray(self, labels, preOutput, activationFn, mask=None):
        act = to_activation(activationFn)
        out = act.getActivation(_acc(preOutput), False)
        s = self.scoreArray(_acc(labels), out)
        w = self._w(s)
        if w is not None:
            s = s * w
        s = _apply_mask(s, mask)
        return s.reshape(s.shape[0], -1).sum(dim=1)

    def computeScore(self, labels, preOutput, activationFn, mask=None, average=True):
        s = self.computeScoreArray(labels, preOutput, activationFn, mask).sum()
        if average:
            s = s / preOutput.shape[0]
        return s

    def computeGradient(self, labels, preOutput, activationFn, mask=None):
        act = to_activation(activationFn)
        z = _acc(preOutput)
        out = act.getActivation(z, True)
        g = self.gradOutput(_acc(labels), out)
        w = self._w(g)
        if w is not None:
            g = g * w
        if mask is not None and tuple(mask.shape) == tuple(g.shape):
            # per-output masking: dL/da is masked BEFORE the activation backprop as well — for softmax dL/dz_i
            # depends on every dL/da_j, so a masked label would otherwise still steer the unmasked outputs
            # (the ND4J loss functions' per-output masking rule)
            g = _apply_mask(g, mask)
        g = act.backprop(z, g)
        g = _apply_mask(g, mask)
        return g.to(preOutput.dtype)

    def computeGradientAndScore(self, labels, preOutput, activationFn, mask=None, average=True):
        return (self.computeScore(labels, preOutput, activationFn, mask, average),
                self.computeGradient(labels, preOutput, activationFn, mask))

    def name(self):
        return type(self).__name__


class LossL2(ILossFunction):
    def scoreArray(self, labels, output):
        d = output - labels
        return d * d

    def gradOutput(self, labels, output):
        return 2 * (output - labels)


class LossMSE(LossL2):
    def scoreArray(self, labels, output):
        return super().scoreArray(labels, output) / labels.shape[1]

    def gradOutput(self, labels, output):
        return super().gradOutput(labels, output) / labels.shape[1]


class LossL1(ILossFunction):
    def scoreArray(self, labels, output):
        return torch.abs(output - labels)

    def gradOutput(self, labels, output):
        return torch.sign(output - labels)


class LossMAE(LossL1):
    def scoreArray(self, labels, output):
        return super().scoreArray(labels, output) / labels.shape[1]

    def gradOutput(self, labels, output):
        return super().gradOutput(labels, output) / labels.shape[1]


class LossMCXENT(ILossFunction):
    FIELDS = {"softmaxClipEps": 1e-10}

    def _clip(self, out):
        e = self.softmaxClipEps
        return torch.clamp(out, e, 1 - e) if e and e > 0 else out

    def scoreArray(self, labels, output):
        return -labels * torch.log(self._clip(output))

    def gradOutput(self, labels, output):
        return -labels / self._clip(output)

    def computeScoreArray(self, labels, preOutput, activationFn, mask=None):
        act = to_activation(activationFn)
        if isinstance(act, ActivationSoftmax) and self.weights is None:
            # log-softmax is numerically exact; clip only matters at saturation
            logp = torch.log_softmax(_acc(preOutput), dim=1)
            if self.softmaxClipEps:
                logp = torch.clamp(logp, min=torch.log(torch.tensor(self.softmaxClipEps)).item())
            s = _apply_mask(-_acc(labels) * logp, mask)
            return s.sum(dim=1)
        return super().computeScoreArray(labels, preOutput, activationFn, mask)

    def computeGradient(self, labels, preOutput, activationFn, mask=None):
        act = to_activation(activationFn)
        if isinstance(act, ActivationSoftmax):
            out = torch.softmax(_acc(preOutput), dim=1)
            lab = _acc(labels)
            w = self._w(out)
            if w is None:
                g = out - lab
            else:
                # d/dz of -sum_j w_j y_j log s_j = s * sum_j(w_j y_j) - w*y
                wy = lab * w
                g = out * wy.sum(dim=1, keepdim=True) - wy
            return _apply_mask(g, mask).to(preOutput.dtype)
        return super().computeGradient(labels, preOutput, activationFn, mask)


class LossNegativeLogLikelihood(LossMCXENT):
    pass


class LossBinaryXENT(ILossFunction):
    FIELDS = {"clipEps": 1e-5}

    def scoreArray(self, labels, output):
        o = torch.clamp(output, self.clipEps, 1 - self.clipEps)
        return -(labels * torch.log(o) + (1 - labels) * torch.log(1 - o))

    def gradOutput(self, labels, output):
        o = torch.clamp(output, self.clipEps, 1 - self.clipEps)
        return -(labels / o - (1 - labels) / (1 - o))

    def computeGradient(self, labels, preOutput, activationFn, mask=None):
        act = to_activation(activationFn)
        if isinstance(act, ActivationSigmoid) and self.weights is None:
            g = torch.sigmoid(_acc(preOutput)) - _acc(labels)
            return _apply_mask(g, mask).to(preOutput.dtype)
        return super().computeGradient(labels, preOutput, activationFn, mask)


class LossHinge(ILossFunction):
    def scoreArray(self, labels, output):
        return torch.clamp(1 - labels * output, min=0)

    def gradOutput(self, labels, output):
        return torch.where(1 - labels * output > 0, -labels, torch.zeros_like(labels))


class LossSquaredHinge(ILossFunction):
    def scoreArray(self, labels, output):
        h = torch.clamp(1 - labels * output, min=0)
        return h * h

    def gradOutput(self, labels, output):
        h = 1 - labels * output
        return torch.where(h > 0, -2 * labels * h, torch.zeros_like(labels))


class LossKLD(ILossFunction):
    def scoreArray(self, labels, output):
        o = torch.clamp(output, 1e-10, 1)
        lab = torch.clamp(labels, 1e-10, 1)
        return labels * torch.log(lab / o)

    def gradOutput(self, labels, output):
        return -labels / torch.clamp(output, 1e-10, 1)


class LossMAPE(ILossFunction):
    def scoreArray(self, labels, output):
        return torch.abs((labels - output) / labels) * 100.0 / labels.shape[1]

    def gradOutput(self, labels, output):
        return torch.sign(output - labels) / torch.abs(labels) * 100.0 / labels.shape[1]


class LossMSLE(ILossFunction):
    def scoreArray(self, labels, output):
        d = torch.log((output + 1) / (labels + 1))
        return d * d / labels.shape[1]

    def gradOutput(self, labels, output):
        return 2.0 / labels.shape[1] * torch.log((output + 1) / (labels + 1)) / (output + 1)


class LossPoisson(ILossFunction):
    def scoreArray(self, labels, output):
        return output - labels * torch.log(torch.clamp(output, min=1e-10))

    def gradOutput(self, labels, output):
        return 1 - labels / torch.clamp(output, min=1e-10)


class LossCosineProximity(ILossFunction):
    def scoreArray(self, labels, output):
        n = labels.norm(dim=1, keepdim=True) * output.norm(dim=1, keepdim=True)
        return -(labels * output) / torch.clamp(n, min=1e-12)

    def gradOutput(self, labels, output):
        yn = labels.norm(dim=1, keepdim=True).clamp(min=1e-12)
        on = output.norm(dim=1, keepdim=True).clamp(min=1e-12)
        dot = (labels * output).sum(dim=1, keepdim=True)
        return -(labels / (yn * on) - dot * output / (yn * on ** 3))


class LossWasserstein(ILossFunction):
    def scoreArray(self, labels, output):
        return labels * output / labels.shape[1]

    def gradOutput(self, labels, output):
        return labels / labels.shape[1]


@register_enum
class LossFunction(Enum):
    MSE = "MSE"
    L1 = "L1"
    XENT = "XENT"
    MCXENT = "MCXENT"
    SQUARED_LOSS = "SQUARED_LOSS"
    RECONSTRUCTION_CROSSENTROPY = "RECONSTRUCTION_CROSSENTROPY"
    NEGATIVELOGLIKELIHOOD = "NEGATIVELOGLIKELIHOOD"
    COSINE_PROXIMITY = "COSINE_PROXIMITY"
    HINGE = "HINGE"
    SQUARED_HINGE = "SQUARED_HINGE"
    KL_DIVERGENCE = "KL_DIVERGENCE"
    MEAN_ABSOLUTE_ERROR = "MEAN_ABSOLUTE_ERROR"
    L2 = "L2"
    MEAN_ABSOLUTE_PERCENTAGE_ERROR = "MEAN_ABSOLUTE_PERCENTAGE_ERROR"
    MEAN_SQUARED_LOGARITHMIC_ERROR = "MEAN_SQUARED_LOGARITHMIC_ERROR"
    POISSON = "POISSON"
    WASSERSTEIN = "WASSERSTEIN"

    def getILossFunction(self):
        return _LOSS_MAP[self]()


class LossFunctions:
    """Namespace matching ``org.nd4j.linalg.lossfunctions.LossFunctions``."""
    LossFunction = LossFunction


_LOSS_MAP = {
    LossFunction.MSE: LossMSE, LossFunction.L1: LossL1, LossFunction.XENT: LossBinaryXENT,
    LossFunction.MCXENT: LossMCXENT, LossFunction.SQUARED_LOSS: LossL2,
    LossFunction.RECONSTRUCTION_CROSSENTROPY: LossBinaryXENT,
    LossFunction.NEGATIVELOGLIKELIHOOD: LossNegativeLogLikelihood,
    LossFunction.COSINE_PROXIMITY: LossCosineProximity, LossFunction.HINGE: LossHinge,
    LossFunction.SQUARED_HINGE: LossSquaredHinge, LossFunction.KL_DIVERGENCE: LossKLD,
    LossFunction.MEAN_ABSOLUTE_ERROR: LossMAE, LossFunction.L2: LossL2,
    LossFunction.MEAN_ABSOLUTE_PERCENTAGE_ERROR: LossMAPE,
    LossFunction.MEAN_SQUARED_LOGARITHMIC_ERROR: LossMSLE, LossFunction.POISSON: LossPoisson,
    LossFunction.WASSERSTEIN: LossWasserstein,
}


def to_loss(x):
    if x is None or isinstance(x, ILossFunction):
        return x
    if isinstance(x, LossFunction):
        return x.getILossFunction()
    if isinstance(x, str):
        return LossFunction[x.upper()].getILossFunction()
    raise TypeError(f"Cannot convert {x!r} to a loss function")
