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


# gradient normalization modes of a segment (kernel codes, csrc/updater.hip SegDesc.gn_mode)
GN_NONE, GN_RENORM_LAYER, GN_RENORM_PARAM, GN_CLIP_ELEM, GN_CLIP_L2_LAYER, GN_CLIP_L2_PARAM = range(6)


class Segment:
    __slots__ = ("p_off", "n", "st_off", "in_block", "block_n", "updater", "l1", "l2", "block_id", "gn_mode",
                 "gn_thr", "gn_group")

    def __init__(self, p_off, n, st_off, in_block, block_n, updater, l1, l2, block_id, gn_mode=GN_NONE, gn_thr=1.0,
                 gn_group=None):
        self.p_off, self.n, self.st_off, self.in_block, self.block_n = p_off, n, st_off, in_block, block_n
        self.updater, self.l1, self.l2, self.block_id = updater, l1, l2, block_id
        # gn_group: segments sharing a norm (one layer for the *PerLayer modes); None = the segment alone
        self.gn_mode, self.gn_thr, self.gn_group = gn_mode, gn_thr, gn_group


def pre_apply(plan, grad):
    """Gradient normalization / clipping of the flat gradient (reference BaseMultiLayerUpdater.java:322-382) — the
    host-side path; on the GPU the fused updater applies it inside its kernel pass."""
    groups = {}
    for i, sg in enumerate(plan.segments):
        if sg.gn_mode != GN_NONE:
            groups.setdefault(sg.gn_group if sg.gn_group is not None else ("seg", i), []).append(sg)
    with torch.no_grad():
        for segs in groups.values():
            views = [grad[sg.p_off:sg.p_off + sg.n] for sg in segs]
            mode, thr = segs[0].gn_mode, segs[0].gn_thr
            if mode == GN_CLIP_ELEM:
                for v in views:
                    v.clamp_(-thr, thr)
                continue
            nrm = torch.sqrt(sum((v.double() ** 2).sum() for v in views)).to(grad.dtype)
            scale = 1.0 / nrm if mode in (GN_RENORM_LAYER, GN_RENORM_PARAM) else torch.clamp(thr / nrm, max=1.0)
            for v in views:
                v.mul_(scale)


def has_gn(plan):
    return any(sg.gn_mode != GN_NONE for sg in plan.segments)


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
    reg_out: optional 1-element tensor overwritten with sum(l1*|p| + 0.5*l2*p^2) of the pre-update
    params (the score's regularisation term) — computed inside the same kernel pass on GPU."""
    div = float(batch_size) if mini_batch else 1.0
    custom = [b[3] for b in plan.blocks if not b[3].kernel_supported()]
    if use_native(params, "update") and params.dtype == torch.float32:
        if not custom:
            from . import native
            if native.fused_update(plan, params, grad, state, iteration, epoch, div, shadow, write_update,
                                   reg_out):
                return
        elif params.is_cuda:
            from . import fallback
            fallback.record("update", f"user updater {type(custom[0]).__name__}: per-block reference update")
    if has_gn(plan):
        pre_apply(plan, grad)
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
