"""GradientCheckUtil: central-difference numerical gradients vs backprop, in double precision.

Reference: NN:gradientcheck/GradientCheckUtil.java:109-314 (MLN), :331 (CG), :512 (single layer).
As in the reference, the backprop gradient is taken *after* the updater with an identity update
(SGD lr=1 / NoOp) and the minibatch division, i.e. g_check = (g + l2*p + l1*sign(p)) / mb, which is
exactly d(score)/dp with score = (sum loss + L1 + L2) / mb.
"""
import torch

from .datasets.dataset import DataSet, MultiDataSet


def _check_net(net):
    if net.flattenedParams.dtype != torch.float64:
        raise ValueError("Gradient checks require DataType.DOUBLE networks (dataType(DataType.DOUBLE))")


def _analytic(net):
    g = net.flattenedGradients.clone()
    p = net.flattenedParams
    for seg in net.updater.plan.segments:
        sl = slice(seg.p_off, seg.p_off + seg.n)
        if seg.l2 > 0:
            g[sl] += seg.l2 * p[sl]
        if seg.l1 > 0:
            g[sl] += seg.l1 * torch.sign(p[sl])
    return g


def _clip_off(net):
    from .nn.conf.losses import LossMCXENT
    layers = net.layers if hasattr(net, "layers") else net.getLayers()
    for l in layers:
        lf = getattr(l.conf, "lossFn", None)
        if isinstance(lf, LossMCXENT):
            lf.softmaxClipEps = 0.0


def checkGradients(net, epsilon=1e-6, maxRelError=1e-3, minAbsoluteError=1e-8, print_results=False,
                   exitOnFirstError=False, input=None, labels=None, inputMask=None, labelMask=None,
                   subset=None, seed=12345):
    """MultiLayerNetwork or ComputationGraph. ``input``/``labels`` may be lists for graphs.
    ``subset``: if set, check at most that many randomly chosen parameters (large nets)."""
    _check_net(net)
    _clip_off(net)
    is_graph = hasattr(net, "topo")
    if is_graph:
        xs = input if isinstance(input, (list, tuple)) else [input]
        ys = labels if isinstance(labels, (list, tuple)) else [labels]
        fm = inputMask if inputMask is None or isinstance(inputMask, (list, tuple)) else [inputMask]
        lm = labelMask if labelMask is None or isinstance(labelMask, (list, tuple)) else [labelMask]
        mb = xs[0].shape[0]

        def score():
            return float(net.computeGradientAndScore(xs, ys, fm, lm))
    else:
        mb = input.shape[0]

        def score():
            return float(net.computeGradientAndScore(input, labels, inputMask, labelMask))

    score()
    div = mb if net.conf.globalConf.get("miniBatch", True) else 1
    analytic = _analytic(net) / div
    params = net.flattenedParams
    n = params.numel()
    idx = range(n)
    if subset is not None and subset < n:
        g = torch.Generator().manual_seed(seed)
        idx = sorted(torch.randperm(n, generator=g)[:subset].tolist())
    total_fail = 0
    worst = 0.0
    names = _param_names(net)
    with torch.no_grad():
        for i in idx:
            orig = params[i].item()
            params[i] = orig + epsilon
            sp = score()
            params[i] = orig - epsilon
            sm = score()
            params[i] = orig
            num = (sp - sm) / (2 * epsilon)
            an = analytic[i].item()
            denom = abs(an) + abs(num)
            rel = 0.0 if denom == 0 else abs(an - num) / denom
            if rel > maxRelError and abs(an - num) > minAbsoluteError:
                total_fail += 1
                if print_results:
                    print(f"Param {i} ({names.get(i, '?')}) FAILED: grad={an}, numerical={num}, relError={rel}")
                if exitOnFirstError:
                    return False
            worst = max(worst, rel if abs(an - num) > minAbsoluteError else 0.0)
    score()   # restore state
    if print_results:
        print(f"GradientCheck: {len(list(idx)) if not isinstance(idx, range) else n} params, {total_fail} failed, "
              f"max rel error {worst:.3e}")
    return total_fail == 0


def _param_names(net):
    out = {}
    for idx, name, impl, off in net._layer_offsets:
        o = off
        for spec in impl.conf.param_specs():
            for k in range(spec.numel):
                out[o + k] = f"{name}_{spec.key}[{k}]"
            o += spec.numel
    return out


class GradientCheckUtil:
    checkGradients = staticmethod(checkGradients)


_ = (DataSet, MultiDataSet)
