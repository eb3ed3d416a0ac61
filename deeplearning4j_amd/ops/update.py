"""Fused multi-tensor updater: ONE kernel launch updates the whole flat parameter vector.

Implements, per parameter segment, the reference's update order (BaseMultiLayerUpdater.java:223-309,
UpdaterBlock.java:142-193, StochasticGradientDescent.java:78):
    u = Updater(g)                 (Sgd / Nesterovs / Adam / AdaMax / Nadam / AdaGrad / AdaDelta / RmsProp)
    u += l2 * p + l1 * sign(p)     (post-apply regularisation)
    u /= minibatch                 (if miniBatch)
    p -= u                         (NegativeGradientStepFunction)
and optionally writes a bf16 shadow of p for the reduced-precision compute path, so the master
weights are read and written once per step.

Updater state layout follows UpdaterBlock: one contiguous state slice per *block* ([m(nb)|v(nb)] for
Adam over the block's nb params), so a segment addresses state at block_off + offset_in_block.
"""
import torch

from ..nn.conf.updaters import kernel_params
from .dispatch import use_native


class Segment:
    __slots__ = ("p_off", "n", "st_off", "in_block", "block_n", "updater", "l1", "l2", "block_id")

    def __init__(self, p_off, n, st_off, in_block, block_n, updater, l1, l2, block_id):
        self.p_off, self.n, self.st_off, self.in_block, self.block_n = p_off, n, st_off, in_block, block_n
        self.updater, self.l1, self.l2, self.block_id = updater, l1, l2, block_id


class UpdatePlan:
    """Static description of all blocks/segments of a network's flat vectors."""

    def __init__(self, segments, blocks):
        self.segments = segments
        self.blocks = blocks          # list of (p_start, p_end, st_off, updater)
        self._dev_table = {}

    def table(self, device, iteration, epoch, batch_div):
        """float64 table [nseg, 12] for the HIP kernel:
        p_off, n, st_off, in_block, block_n, opcode, h0..h3, l1, l2 (batch_div passed separately)."""
        rows = []
        for s in self.segments:
            op, h0, h1, h2, h3 = kernel_params(s.updater, iteration, epoch)
            rows.append([s.p_off, s.n, s.st_off, s.in_block, s.block_n, op, h0, h1, h2, h3, s.l1, s.l2])
        return torch.tensor(rows, dtype=torch.float64)


def fused_update(plan, params, grad, state, iteration, epoch, batch_size, mini_batch=True, shadow=None,
                 write_update=True, reg_out=None):
    """params/grad/state: flat 1-D fp32 (or fp64) tensors. shadow: optional bf16 flat copy of params.
    reg_out: optional zeroed 1-element tensor that receives sum(l1*|p| + 0.5*l2*p^2) of the pre-update
    params (the score's regularisation term) — computed inside the same kernel pass on GPU."""
    div = float(batch_size) if mini_batch else 1.0
    if use_native(params, "update") and params.dtype == torch.float32:
        from . import native
        if native.fused_update(plan, params, grad, state, iteration, epoch, div, shadow, write_update, reg_out):
            return
    with torch.no_grad():
        if reg_out is not None:
            r = torch.zeros((), dtype=params.dtype, device=params.device)
            for s in plan.segments:
                if s.l1 > 0 or s.l2 > 0:
                    p = params[s.p_off:s.p_off + s.n]
                    r = r + s.l1 * p.abs().sum() + 0.5 * s.l2 * (p * p).sum()
            reg_out.fill_(r.item() if reg_out.device.type == "cpu" else 0.0)
            if reg_out.device.type != "cpu":
                reg_out.copy_(r.reshape(reg_out.shape))
        for (p0, p1, st_off, upd) in plan.blocks:
            if p1 <= p0:
                continue
            g = grad[p0:p1]
            ssz = upd.stateSize(p1 - p0)
            upd.apply_reference(g, state[st_off:st_off + ssz], iteration, epoch)
        for s in plan.segments:
            if s.l2 > 0 or s.l1 > 0:
                g = grad[s.p_off:s.p_off + s.n]
                p = params[s.p_off:s.p_off + s.n]
                if s.l2 > 0:
                    g.add_(p * s.l2)
                if s.l1 > 0:
                    g.add_(torch.sign(p) * s.l1)
        if div != 1.0:
            grad.div_(div)
        params.sub_(grad)
        if shadow is not None:
            shadow.copy_(params)
