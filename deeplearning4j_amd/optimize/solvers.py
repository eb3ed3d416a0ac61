"""Optimizers beyond plain SGD: line gradient descent, nonlinear conjugate gradient (Polak-Ribiere), L-BFGS,
with a backtracking (Armijo) line search; step functions and termination conditions.

Reference: optimize/Solver.java:50-84, optimize/solvers/{BaseOptimizer,LineGradientDescent,ConjugateGradient,
LBFGS,BackTrackLineSearch,StochasticGradientDescent}.java, optimize/stepfunctions/*, optimize/terminations/*.
Semantics kept: the search direction is the POST-updater gradient (BaseOptimizer.gradientAndScore applies the
configured updater, l1/l2 and the minibatch division to the raw gradient before the line search), the step
function applies ``params -= step * direction`` (NegativeDefaultStepFunction), and an optimizer iteration fires
the listeners' iterationDone and increments the model's iteration count.

MI355X notes: every vector op here is one fused device op over the flat [P] parameter/gradient buffers, and
the line search evaluates the score with forward passes only (no backward) until a step is accepted.
"""
import logging

import torch

from ..exceptions import UnsupportedOperationException

log = logging.getLogger("deeplearning4j_amd")


# ------------------------------------------------------------------------------------------ step functions
class StepFunction:
    def step(self, params, direction, step=1.0):
        raise NotImplementedError


class DefaultStepFunction(StepFunction):
    def step(self, params, direction, step=1.0):
        params.add_(direction, alpha=step)


class NegativeDefaultStepFunction(StepFunction):
    def step(self, params, direction, step=1.0):
        params.sub_(direction, alpha=step)


class GradientStepFunction(StepFunction):
    def step(self, params, direction, step=1.0):
        params.add_(direction)


class NegativeGradientStepFunction(StepFunction):
    def step(self, params, direction, step=1.0):
        params.sub_(direction)


# ------------------------------------------------------------------------------------------ terminations
class TerminationCondition:
    def terminate(self, cost, oldCost, otherParams=()):
        raise NotImplementedError


class EpsTermination(TerminationCondition):
    """|cost - oldCost| < tolerance * max(|cost|, |oldCost|, eps) (terminations/EpsTermination.java)."""

    def __init__(self, eps=1e-4, tolerance=2.220446049250313e-16):
        self.eps, self.tolerance = eps, tolerance

    def terminate(self, cost, oldCost, otherParams=()):
        if cost == 0 and oldCost == 0:
            return False
        return 2.0 * abs(oldCost - cost) <= self.tolerance * (abs(oldCost) + abs(cost) + self.eps)


class Norm2Termination(TerminationCondition):
    def __init__(self, gradientTolerance=1e-3):
        self.gradientTolerance = gradientTolerance

    def terminate(self, cost, oldCost, otherParams=()):
        g = otherParams[0] if otherParams else None
        return g is not None and float(torch.linalg.vector_norm(g.float())) < self.gradientTolerance


class ZeroDirection(TerminationCondition):
    def terminate(self, cost, oldCost, otherParams=()):
        g = otherParams[0] if otherParams else None
        return g is not None and float(g.abs().sum()) == 0.0


# ------------------------------------------------------------------------------------------ line search
class BackTrackLineSearch:
    """Backtracking line search with the Armijo test (BackTrackLineSearch.java:62-340): start at step 1 and shrink
    (quadratic-interpolation guess clamped to [0.1, 0.5] x step) until the sufficient-decrease condition
    f(x - s*d) <= f(x) - c * s * <g, d> holds, at most ``maxIterations`` evaluations; the best step seen is returned
    otherwise (0.0 when no step improved). A step function that ADDS the direction (DefaultStepFunction /
    GradientStepFunction) makes it a maximisation, as in the reference: sufficient increase
    f(x + s*d) >= f(x) - c * s * <g, d>.

    Constructors as the reference: ``BackTrackLineSearch(model, optimizer)``, ``(model, stepFunction, optimizer)``,
    or ``(model, score_fn, stepFunction, maxIterations)`` (score_fn: the objective at the model's current
    parameters; by default the model's score on its current input / labels)."""

    def __init__(self, model, score_fn=None, stepFunction=None, maxIterations=None, c1=1e-4):
        optimizer = None
        if isinstance(score_fn, StepFunction):
            score_fn, stepFunction, optimizer = None, score_fn, stepFunction
        elif isinstance(score_fn, BaseOptimizer):
            score_fn, optimizer = None, score_fn
        if isinstance(stepFunction, BaseOptimizer):
            optimizer, stepFunction = stepFunction, None
        self.model = model
        self.score_fn = score_fn or self._model_score
        self.optimizer = optimizer
        self.stepFunction = stepFunction or NegativeDefaultStepFunction()
        if maxIterations is None:
            g = getattr(getattr(model, "conf", None), "globalConf", None) or {}
            maxIterations = g.get("maxNumLineSearchIterations", 5)
        self.maxIterations, self.c1 = max(1, int(maxIterations)), c1

    def _model_score(self):
        m = self.model
        if self.optimizer is not None and self.optimizer._batch is not None:
            return self.optimizer._score_only()
        return float(m._score_batch(m.input, m.labels, getattr(m, "mask", None), getattr(m, "labelsMask", None)))

    def minimizes(self):
        return isinstance(self.stepFunction, (NegativeDefaultStepFunction, NegativeGradientStepFunction))

    def optimize(self, params, gradient, direction, f0=None):
        if f0 is None:
            f0 = float(self.model.score())
        minimize = self.minimizes()
        slope = float(torch.dot(gradient.reshape(-1).double(), direction.reshape(-1).double()))
        if minimize and slope <= 0:
            return 0.0
        x0 = params.clone()
        step = 1.0
        best_step, best_f = 0.0, f0
        for _ in range(self.maxIterations):
            params.copy_(x0)
            self.stepFunction.step(params, direction, step)
            self.model._params_changed()
            f = self.score_fn()
            if (f < best_f) if minimize else (f > best_f):
                best_step, best_f = step, f
            if minimize and f <= f0 - self.c1 * step * slope:
                break
            if not minimize and f >= f0 - self.c1 * step * abs(slope):
                best_step = step
                break
            # quadratic model through f0, slope, f(step) (of -f when maximising)
            df = (f - f0) if minimize else (f0 - f)
            denom = 2.0 * (df + abs(slope) * step)
            nxt = abs(slope) * step * step / denom if denom > 0 else step * 0.5
            step = min(max(nxt, 0.1 * step), 0.5 * step)
        params.copy_(x0)
        self.model._params_changed()
        return best_step


# ------------------------------------------------------------------------------------------ optimizers
def _batch_size(x):
    """Minibatch size of an input (array, or list of arrays for a graph); 1 for a model with no input — a cost
    function optimized directly (the reference's Model.computeGradientAndScore() with no DataSet)."""
    if hasattr(x, "shape"):
        return x.shape[0]
    if isinstance(x, (list, tuple)) and x and hasattr(x[0], "shape"):
        return x[0].shape[0]
    return 1


class BaseOptimizer:
    def __init__(self, model, stepFunction=None, terminationConditions=None, maxLineSearchIterations=None):
        self.model = model
        g = model.conf.globalConf if hasattr(model.conf, "globalConf") else {}
        self.stepFunction = stepFunction or NegativeDefaultStepFunction()
        self.terminationConditions = terminationConditions if terminationConditions is not None else \
            [ZeroDirection(), EpsTermination()]
        n = maxLineSearchIterations or g.get("maxNumLineSearchIterations", 5)
        self.lineMaximizer = BackTrackLineSearch(model, self._score_only, self.stepFunction, n)
        self.searchState = {}
        self.score = float("nan")
        self.oldScore = float("nan")
        self._batch = None

    # the model computes loss + gradient on the current batch, then the configured updater turns the raw
    # gradient into the update direction (without stepping the parameters)
    def gradientAndScore(self):
        m = self.model
        self.oldScore = self.score
        x, y, fm, lm = self._batch
        m.computeGradientAndScore(x, y, fm, lm)
        for l in m.listeners:
            if hasattr(l, "onGradientCalculation"):
                l.onGradientCalculation(m)
        self.score = float(m.score())
        p = m.flattenedParams
        keep = p.clone()
        m.updater.update(p, m.flattenedGradients, m.conf.iterationCount, m.conf.epochCount, _batch_size(x), None)
        p.copy_(keep)
        m._params_changed()
        return m.flattenedGradients.clone(), self.score

    def _score_only(self):
        x, y, fm, lm = self._batch
        return float(self.model._score_batch(x, y, fm, lm))

    def setupSearchState(self, g):
        self.searchState["gradient"] = g
        self.searchState["params"] = self.model.flattenedParams

    def preProcessLine(self):
        self.searchState["searchDirection"] = self.searchState["gradient"].clone()

    def postStep(self, g):
        pass

    def optimize(self, x, y, fmask=None, lmask=None):
        self._batch = (x, y, fmask, lmask)
        m = self.model
        g, f = self.gradientAndScore()
        if "gradient" not in self.searchState:
            self.setupSearchState(g)
        else:
            self.searchState["gradient"] = g
        self.preProcessLine()
        d = self.searchState["searchDirection"]
        params = m.flattenedParams
        step = self.lineMaximizer.optimize(params, g, d, f)
        if step != 0.0:
            self.stepFunction.step(params, d, step)
            m._params_changed()
        else:
            log.debug("Step size returned by line search is 0.0.")
        g2, _ = self.gradientAndScore()
        self.postStep(g2)
        m._iteration_done()
        for c in self.terminationConditions:
            if c.terminate(self.score, self.oldScore, (g2,)):
                log.debug("Hit termination condition %s", type(c).__name__)
                return False
        return True


class LineGradientDescent(BaseOptimizer):
    def postStep(self, g):
        self.searchState["gradient"] = g


class ConjugateGradient(BaseOptimizer):
    """Nonlinear CG with the Polak-Ribiere+ beta (ConjugateGradient.java)."""

    def preProcessLine(self):
        if "searchDirection" not in self.searchState:
            self.searchState["searchDirection"] = self.searchState["gradient"].clone()

    def postStep(self, g):
        g_last = self.searchState["gradient"]
        d_last = self.searchState["searchDirection"]
        dgg = float(torch.dot((g - g_last).double(), g.double()))
        gg = float(torch.dot(g_last.double(), g_last.double()))
        gamma = max(dgg / gg, 0.0) if gg > 0 else 0.0
        self.searchState["searchDirection"] = d_last.mul_(gamma).add_(g)
        self.searchState["gradient"] = g


class LBFGS(BaseOptimizer):
    """Limited-memory BFGS, two-loop recursion over the last m (s, y) pairs (LBFGS.java, m = 4)."""

    def __init__(self, model, m=4, **kw):
        super().__init__(model, **kw)
        self.m = m

    def setupSearchState(self, g):
        super().setupSearchState(g)
        self.searchState.update(s=[], y=[], rho=[], oldparams=self.model.flattenedParams.clone())

    def preProcessLine(self):
        if "searchDirection" not in self.searchState:
            self.searchState["searchDirection"] = self.searchState["gradient"].clone()

    def postStep(self, g):
        st = self.searchState
        p = self.model.flattenedParams
        s_k = p - st["oldparams"]
        y_k = g - st["gradient"]
        sy = float(torch.dot(s_k.double(), y_k.double()))
        yy = float(torch.dot(y_k.double(), y_k.double()))
        if sy > 1e-10:                # curvature condition; otherwise keep the old pairs
            st["s"].insert(0, s_k)
            st["y"].insert(0, y_k)
            st["rho"].insert(0, 1.0 / sy)
            del st["s"][self.m:], st["y"][self.m:], st["rho"][self.m:]
        q = g.clone()
        alpha = []
        for s_i, y_i, r_i in zip(st["s"], st["y"], st["rho"]):
            a = r_i * float(torch.dot(s_i.double(), q.double()))
            alpha.append(a)
            q.add_(y_i, alpha=-a)
        if st["s"]:
            q.mul_(sy / yy if sy > 1e-10 and yy > 0 else 1.0)
        for (s_i, y_i, r_i), a in zip(reversed(list(zip(st["s"], st["y"], st["rho"]))), reversed(alpha)):
            b = r_i * float(torch.dot(y_i.double(), q.double()))
            q.add_(s_i, alpha=a - b)
        st["searchDirection"] = q
        st["oldparams"] = p.clone()
        st["gradient"] = g


class StochasticGradientDescent:
    """The plain update path (StochasticGradientDescent.java:58-98) is the network's own fused fit step."""

    def __init__(self, model, **kw):
        self.model = model

    def optimize(self, x, y, fmask=None, lmask=None):
        self.model._fit_batch_sgd(x, y, fmask, lmask)
        return True


class Solver:
    """Builds the optimizer for a model's OptimizationAlgorithm (Solver.java:50-84)."""

    def __init__(self, model):
        self.model = model
        self._opt = None

    def getOptimizer(self):
        if self._opt is None:
            from ..nn.conf.enums import OptimizationAlgorithm as OA
            algo = OA.of(self.model.conf.globalConf.get("optimizationAlgo", OA.STOCHASTIC_GRADIENT_DESCENT))
            sf = self.model.conf.globalConf.get("stepFunction")
            kw = {"stepFunction": _step_function(sf)} if sf is not None else {}
            if algo == OA.HESSIAN_FREE:
                raise UnsupportedOperationException(
                    "HESSIAN_FREE optimisation is deprecated in the reference and has no solver "
                    "(OptimizationAlgorithm.java:27); use LBFGS or CONJUGATE_GRADIENT")
            cls = {OA.STOCHASTIC_GRADIENT_DESCENT: StochasticGradientDescent,
                   OA.LINE_GRADIENT_DESCENT: LineGradientDescent, OA.CONJUGATE_GRADIENT: ConjugateGradient,
                   OA.LBFGS: LBFGS}[algo]
            self._opt = cls(self.model, **kw)
        return self._opt

    def optimize(self, x, y, fmask=None, lmask=None):
        return self.getOptimizer().optimize(x, y, fmask, lmask)


def _step_function(sf):
    if isinstance(sf, StepFunction):
        return sf
    name = str(getattr(sf, "value", sf)).upper()
    return {"DEFAULT": DefaultStepFunction(), "NEGATIVE_DEFAULT": NegativeDefaultStepFunction(),
            "GRADIENT": GradientStepFunction(), "NEGATIVE_GRADIENT": NegativeGradientStepFunction()
            }.get(name, NegativeDefaultStepFunction())
