"""Fused softmax + cross-entropy (MCXENT / NLL) forward+backward.

Reference: LossMCXENT with softmax (gradient = softmax(z) - labels, score = -sum y*log(clip(p)))
called from BaseOutputLayer.java:82-92,173. One HIP kernel (``csrc/softmax_xent.hip``) does the row
max, exp-sum, per-row score and the gradient in a single pass over the logits (row per wavefront).
"""
import math

import torch

from .dispatch import use_native
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


def softmax_xent(logits, labels, mask=None, clip_eps=1e-10):
    """Returns (per_example_score [mb] fp32, dL/dz same dtype as logits, probabilities fp32 or None)."""
    if use_native(logits, "softmax_xent") and logits.dim() == 2:
        from . import native
        per_row = mask is not None and mask.numel() == logits.shape[0]
        if mask is None or per_row:            # per-time-step masks of RNN outputs: rows scaled in the kernel
            r = native.softmax_xent(logits, labels, clip_eps, row_mask=mask if per_row else None)
            if r is not None:
                return r
    from .fallback import note
    note(logits, "softmax_xent", f"{logits.dtype} mask={mask is not None}")
    z = _acc(logits)
    logp = torch.log_softmax(z, dim=1)
    if clip_eps:
        logp_c = torch.clamp(logp, min=math.log(clip_eps), max=math.log1p(-clip_eps))
    else:
        logp_c = logp
    lab = _acc(labels)
    s = -(lab * logp_c)
    p = torch.exp(logp)
    g = p - lab
    if mask is not None:
        m = _acc(mask).reshape(-1, 1) if mask.dim() == 1 or mask.shape[1] == 1 else _acc(mask)
        s = s * m
        g = g * m
    return s.sum(dim=1), g.to(logits.dtype), p
