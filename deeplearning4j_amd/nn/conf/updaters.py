"""Updater configurations (ND4J IUpdater) + learning-rate schedules + reference update math.

Update formulas are exactly the ones asserted by the reference's TestUpdaters
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/updater/TestUpdaters.java):
  Sgd :506, Nesterovs :418-419, Adam :197-218, AdaMax :350-371, Nadam :279-292, RmsProp :471-472,
  AdaGrad :163, AdaDelta :109-120.
State layout inside one flat updater-state block of n params (checkpoint-relevant):
  Adam/AdaMax/Nadam: [m(n) | v(n)], AdaDelta: [msg(n) | msdx(n)], Nesterovs: [v], RmsProp: [s],
  AdaGrad: [h], Sgd/NoOp: [].

``apply_reference`` is the plain torch implementation (CPU path and the numerics oracle for the
fused HIP updater kernel ``ops.fused_update``).
"""
import math
from enum import Enum

import torch

from .base import Config, register_enum


# ----------------------------------------------------------------------------------- schedules
@register_enum
class ScheduleType(Enum):
    ITERATION = "ITERATION"
    EPOCH = "EPOCH"


class ISchedule(Config):
    FIELDS = {"scheduleType": ScheduleType.ITERATION}
    _POSITIONAL = None      # reference constructor order; default (scheduleType, *this class's FIELDS)

    def __init__(self, *args, **kw):
        if args:
            names = self._POSITIONAL or ("scheduleType",) + tuple(type(self).__dict__.get("FIELDS", {}))
            if len(args) > len(names):
                raise TypeError(f"{type(self).__name__} takes at most {len(names)} positional arguments {names}")
            for n, a in zip(names, args):
                kw[n] = a
        super().__init__(**kw)

    def _t(self, iteration, epoch):
        return iteration if self.scheduleType == ScheduleType.ITERATION else epoch

    def valueAt(self, iteration, epoch):
        raise NotImplementedError


class FixedSchedule(ISchedule):
    FIELDS = {"value": 0.0}
    _POSITIONAL = ("value",)

    def valueAt(self, iteration, epoch):
        return self.value


class ExponentialSchedule(ISchedule):
    FIELDS = {"initialValue": 0.1, "gamma": 0.99}

    def valueAt(self, iteration, epoch):
        return self.initialValue * self.gamma ** self._t(iteration, epoch)


class InverseSchedule(ISchedule):
    FIELDS = {"initialValue": 0.1, "gamma": 0.1, "power": 1.0}

    def valueAt(self, iteration, epoch):
        return self.initialValue / (1 + self.gamma * self._t(iteration, epoch)) ** self.power


class PolySchedule(ISchedule):
    FIELDS = {"initialValue": 0.1, "power": 1.0, "maxIter": 1000}

    def valueAt(self, iteration, epoch):
        return self.initialValue * (1 + self._t(iteration, epoch) / self.maxIter) ** self.power


class SigmoidSchedule(ISchedule):
    FIELDS = {"initialValue": 0.1, "gamma": 0.1, "stepSize": 100}

    def valueAt(self, iteration, epoch):
        return self.initialValue / (1 + math.exp(-self.gamma * (self._t(iteration, epoch) - self.stepSize)))


class StepSchedule(ISchedule):
    FIELDS = {"initialValue": 0.1, "decayRate": 0.5, "step": 100.0}

    def valueAt(self, iteration, epoch):
        return self.initialValue * self.decayRate ** math.floor(self._t(iteration, epoch) / self.step)


class MapSchedule(ISchedule):
    FIELDS = {"values": None}

    class Builder:
        """MapSchedule.Builder(ScheduleType).add(i, v)...build() (reference MapSchedule.Builder)."""

        def __init__(self, scheduleType):
            self._t, self._v = scheduleType, {}

        def add(self, position, value):
            self._v[int(position)] = value
            return self

        def build(self):
            if 0 not in self._v:
                raise ValueError("MapSchedule needs a value for position 0")
            return MapSchedule(self._t, dict(self._v))

    def valueAt(self, iteration, epoch):
        t = self._t(iteration, epoch)
        keys = sorted(int(k) for k in self.values)
        v = self.values[keys[0]] if keys[0] in self.values else self.values[str(keys[0])]
        for k in keys:
            if k <= t:
                v = self.values[k] if k in self.values else self.values[str(k)]
        return v


def _val(x, iteration, epoch):
    return x.valueAt(iteration, epoch) if isinstance(x, ISchedule) else x


# ------------------------------------------------------------------------------------ updaters
class IUpdater(Config):
    """Base updater config. ``stateSize(n)`` is the number of state scalars for n params."""
    STATE_MULT = 0
    HAS_LR = True

    def stateSize(self, n):
        return self.STATE_MULT * n

    def getLearningRate(self, iteration=0, epoch=0):
        lr = getattr(self, "learningRate", None)
        sched = getattr(self, "learningRateSchedule", None)
        if sched is not None:
            return sched.valueAt(iteration, epoch)
        return lr

    def setLrAndSchedule(self, lr, schedule):
        if hasattr(self, "learningRate"):
            self.learningRate = lr
            self.learningRateSchedule = schedule

    def hyper(self, iteration, epoch):
        """Hyperparameters for the fused kernel: dict of floats at this iteration."""
        return {}

    def apply_reference(self, g, state, iteration, epoch):
        """In-place: g <- update. ``state`` is this block's flat state slice.
        A user updater written against the reference API (``instantiate(viewArray, initialize)`` returning a
        GradientUpdater with ``applyUpdater(gradient, iteration, epoch)``) runs through that."""
        inst = getattr(self, "instantiate", None)
        if inst is None:
            raise NotImplementedError(f"{type(self).__name__}: neither apply_reference nor instantiate is defined")
        gu = inst(state if state.numel() else None, False)
        gu.applyUpdater(g, iteration, epoch)

    def kernel_supported(self):
        """True when the fused HIP updater kernel implements this updater (the built-in ND4J updaters)."""
        return type(self) in UPDATER_OPCODES


class NoOp(IUpdater):
    """ND4J NoOpUpdater: leaves the gradient unchanged (update == gradient). Layers that must not move
    (FrozenLayer, BN running stats) zero their gradient views instead."""
    HAS_LR = False

    def apply_reference(self, g, state, iteration, epoch):
        pass


class Sgd(IUpdater):
    FIELDS = {"learningRate": 1e-3, "learningRateSchedule": None}

    @classmethod
    def _builder_positional(cls, kw, *args):
        kw["learningRate"] = args[0]

    def __init__(self, learningRate=1e-3, **kw):
        if isinstance(learningRate, ISchedule):
            kw["learningRateSchedule"] = learningRate
            learningRate = float("nan")
        super().__init__(learningRate=learningRate, **kw)

    def apply_reference(self, g, state, iteration, epoch):
        g.mul_(self.getLearningRate(iteration, epoch))


class Nesterovs(IUpdater):
    FIELDS = {"learningRate": 0.1, "learningRateSchedule": None, "momentum": 0.9, "momentumSchedule": None}
    STATE_MULT = 1
    DEFAULT_NESTEROV_MOMENTUM = 0.9
    DEFAULT_NESTEROV_LEARNING_RATE = 0.1

    def getMomentumISchedule(self):
        return self.momentumSchedule

    def __init__(self, learningRate=0.1, momentum=0.9, **kw):
        if isinstance(learningRate, ISchedule):
            kw["learningRateSchedule"] = learningRate
            learningRate = float("nan")
        if isinstance(momentum, ISchedule):
            kw["momentumSchedule"] = momentum
            momentum = float("nan")
        super().__init__(learningRate=learningRate, momentum=momentum, **kw)

    def getMomentum(self, iteration=0, epoch=0):
        return self.momentumSchedule.valueAt(iteration, epoch) if self.momentumSchedule else self.momentum

    def apply_reference(self, g, state, iteration, epoch):
        mu = self.getMomentum(iteration, epoch)
        lr = self.getLearningRate(iteration, epoch)
        v_prev = state.clone()
        state.mul_(mu).sub_(g * lr)                  # v = mu*v - lr*g
        g.copy_(v_prev * mu - state * (1 + mu))      # u = mu*v_prev - (1+mu)*v


class Adam(IUpdater):
    FIELDS = {"learningRate": 1e-3, "learningRateSchedule": None, "beta1": 0.9, "beta2": 0.999,
              "epsilon": 1e-8}
    STATE_MULT = 2
    DEFAULT_ADAM_LEARNING_RATE, DEFAULT_ADAM_BETA1_MEAN_DECAY = 1e-3, 0.9
    DEFAULT_ADAM_BETA2_VAR_DECAY, DEFAULT_ADAM_EPSILON = 0.999, 1e-8

    def __init__(self, learningRate=1e-3, beta1=0.9, beta2=0.999, epsilon=1e-8, **kw):
        if isinstance(learningRate, ISchedule):
            kw["learningRateSchedule"] = learningRate
            learningRate = float("nan")
        super().__init__(learningRate=learningRate, beta1=beta1, beta2=beta2, epsilon=epsilon, **kw)

    def alpha_t(self, iteration, epoch):
        lr = self.getLearningRate(iteration, epoch)
        t = iteration + 1
        b1t = 1 - self.beta1 ** t
        b2t = 1 - self.beta2 ** t
        a = lr * math.sqrt(b2t) / b1t
        return self.epsilon if a == 0.0 else a

    def apply_reference(self, g, state, iteration, epoch):
        n = g.numel()
        m, v = state[:n], state[n:2 * n]
        m.mul_(self.beta1).add_(g * (1 - self.beta1))
        v.mul_(self.beta2).add_(g * g * (1 - self.beta2))
        a = self.alpha_t(iteration, epoch)
        g.copy_(m * a / (torch.sqrt(v) + self.epsilon))


class AdaMax(Adam):
    def apply_reference(self, g, state, iteration, epoch):
        n = g.numel()
        m, u = state[:n], state[n:2 * n]
        m.mul_(self.beta1).add_(g * (1 - self.beta1))
        torch.maximum(u * self.beta2, torch.abs(g), out=u)
        lr = self.getLearningRate(iteration, epoch)
        b1t = 1 - self.beta1 ** (iteration + 1)
        a = lr / b1t if b1t != 0 else self.epsilon
        g.copy_(m * a / (u + self.epsilon))


class Nadam(Adam):
    def apply_reference(self, g, state, iteration, epoch):
        n = g.numel()
        m, v = state[:n], state[n:2 * n]
        lr = self.getLearningRate(iteration, epoch)
        b1t = 1 - self.beta1 ** (iteration + 1)
        one_minus_b1_g = g * (1 - self.beta1)
        m.mul_(self.beta1).add_(one_minus_b1_g)
        v.mul_(self.beta2).add_(g * g * (1 - self.beta2))
        bias_m = m * self.beta1 / b1t
        second = one_minus_b1_g / b1t
        g.copy_((bias_m + second) * lr / (torch.sqrt(v) + self.epsilon))


class AdaGrad(IUpdater):
    FIELDS = {"learningRate": 1e-1, "learningRateSchedule": None, "epsilon": 1e-6}
    STATE_MULT = 1

    def __init__(self, learningRate=1e-1, epsilon=1e-6, **kw):
        if isinstance(learningRate, ISchedule):
            kw["learningRateSchedule"] = learningRate
            learningRate = float("nan")
        super().__init__(learningRate=learningRate, epsilon=epsilon, **kw)

    def apply_reference(self, g, state, iteration, epoch):
        state.add_(g * g)
        g.mul_(self.getLearningRate(iteration, epoch)).div_(torch.sqrt(state + self.epsilon))


class AdaDelta(IUpdater):
    FIELDS = {"rho": 0.95, "epsilon": 1e-6}
    STATE_MULT = 2
    HAS_LR = False
    DEFAULT_ADADELTA_RHO, DEFAULT_ADADELTA_EPSILON = 0.95, 1e-6

    def __init__(self, rho=0.95, epsilon=1e-6, **kw):
        super().__init__(rho=rho, epsilon=epsilon, **kw)

    def apply_reference(self, g, state, iteration, epoch):
        n = g.numel()
        msg, msdx = state[:n], state[n:2 * n]
        msg.mul_(self.rho).add_(g * g * (1 - self.rho))
        dx = torch.sqrt(msdx + self.epsilon) / torch.sqrt(msg + self.epsilon) * g
        msdx.mul_(self.rho).add_(dx * dx * (1 - self.rho))
        g.copy_(dx)


class RmsProp(IUpdater):
    FIELDS = {"learningRate": 1e-1, "learningRateSchedule": None, "rmsDecay": 0.95, "epsilon": 1e-8}
    STATE_MULT = 1
    DEFAULT_RMSPROP_LEARNING_RATE, DEFAULT_RMSPROP_RMSDECAY, DEFAULT_RMSPROP_EPSILON = 1e-1, 0.95, 1e-8

    def __init__(self, learningRate=1e-1, rmsDecay=0.95, epsilon=1e-8, **kw):
        if isinstance(learningRate, ISchedule):
            kw["learningRateSchedule"] = learningRate
            learningRate = float("nan")
        super().__init__(learningRate=learningRate, rmsDecay=rmsDecay, epsilon=epsilon, **kw)

    def apply_reference(self, g, state, iteration, epoch):
        state.mul_(self.rmsDecay).add_(g * g * (1 - self.rmsDecay))
        g.mul_(self.getLearningRate(iteration, epoch)).div_(torch.sqrt(state + self.epsilon))


# Kernel op codes shared with csrc/updater.hip (keep in sync).
UPDATER_OPCODES = {NoOp: 0, Sgd: 1, Nesterovs: 2, Adam: 3, AdaMax: 4, Nadam: 5, AdaGrad: 6,
                   AdaDelta: 7, RmsProp: 8}


def kernel_params(u, iteration, epoch):
    """(opcode, p0..p3) scalars for the fused HIP updater kernel."""
    t = type(u)
    op = UPDATER_OPCODES[t]
    if t is NoOp:
        return op, 0.0, 0.0, 0.0, 0.0
    if t is Sgd:
        return op, u.getLearningRate(iteration, epoch), 0.0, 0.0, 0.0
    if t is Nesterovs:
        return op, u.getLearningRate(iteration, epoch), u.getMomentum(iteration, epoch), 0.0, 0.0
    if t is Adam:
        return op, u.alpha_t(iteration, epoch), u.beta1, u.beta2, u.epsilon
    if t is AdaMax:
        b1t = 1 - u.beta1 ** (iteration + 1)
        return op, u.getLearningRate(iteration, epoch) / b1t, u.beta1, u.beta2, u.epsilon
    if t is Nadam:
        b1t = 1 - u.beta1 ** (iteration + 1)
        return op, u.getLearningRate(iteration, epoch) / b1t, u.beta1, u.beta2, u.epsilon
    if t is AdaGrad:
        return op, u.getLearningRate(iteration, epoch), u.epsilon, 0.0, 0.0
    if t is AdaDelta:
        return op, u.rho, u.epsilon, 0.0, 0.0
    if t is RmsProp:
        return op, u.getLearningRate(iteration, epoch), u.rmsDecay, u.epsilon, 0.0
    raise TypeError(f"No fused kernel for updater {t.__name__}")


def to_updater(u):
    from .enums import Updater
    if u is None or isinstance(u, IUpdater):
        return u
    if isinstance(u, Updater):
        return u.getIUpdaterWithDefaultConfig()
    if isinstance(u, str):
        return Updater[u.upper()].getIUpdaterWithDefaultConfig()
    raise TypeError(f"Cannot convert {u!r} to an IUpdater")
