"""Phase-split strided bwd-data plan (ops/conv_native._phase_plan): every phase, run as a stride-1 correlation of dY
with its flipped sub-kernel under the plan's pad, reproduces torch's strided conv input gradient (CPU, fp64)."""
import itertools

import pytest
import torch
import torch.nn.functional as F

from deeplearning4j_amd.ops.conv_native import _phase_plan


def _phase_dx(dy, w, H, W, stride, pad4):
    N, K, OH, OW = dy.shape
    _, C, R, S = w.shape
    plan = _phase_plan(H, W, OH, OW, R, S, stride, pad4, (1, 1))
    assert plan is not None
    flip = w.flip(2, 3).permute(1, 2, 3, 0)                          # [C, R, S, K], as the kernel layout
    dx = torch.zeros(N, C, H, W, dtype=dy.dtype)
    for (i0h, i0w, Rf, Sf, Hf, Wf, u0h, u0w, pth, ptw) in plan:
        if Rf == 0 or Sf == 0:
            continue
        sub = flip[:, u0h::stride[0], u0w::stride[1], :][:, :Rf, :Sf, :]      # [C, Rf, Sf, K]
        wk = sub.permute(0, 3, 1, 2)                                       # [C(out), K(in), Rf, Sf]
        # forward conv over dY: out[j] = sum_t dy[j - pth + t] * sub[t], explicit output size Hf x Wf
        xp = F.pad(dy, (ptw, Sf + Wf, pth, Rf + Hf))
        o = F.conv2d(xp, wk)[:, :, :Hf, :Wf]
        dx[:, :, i0h::stride[0], i0w::stride[1]] = o
    return dx


@pytest.mark.parametrize("R,S,stride,pad,H", [(3, 3, 2, 1, 56), (3, 3, 2, 1, 55), (3, 3, 2, 0, 29), (1, 1, 2, 0, 28),
                                              (5, 5, 2, 2, 17), (3, 3, 3, 0, 20), (7, 7, 2, 3, 30), (2, 2, 2, 0, 16),
                                              (3, 1, 2, 1, 12)])
def test_phase_split_matches_strided_conv_grad(R, S, stride, pad, H):
    torch.manual_seed(0)
    N, C, K = 2, 5, 4
    W = H + 1
    pw = pad if S > 1 else 0
    x = torch.randn(N, C, H, W, dtype=torch.float64, requires_grad=True)
    w = torch.randn(K, C, R, S, dtype=torch.float64)
    y = F.conv2d(x, w, stride=stride, padding=(pad, pw))
    dy = torch.randn_like(y)
    (want,) = torch.autograd.grad(y, x, dy)
    got = _phase_dx(dy, w, H, W, (stride, stride), (pad, pad, pw, pw))
    assert torch.allclose(got, want, atol=1e-10), (got - want).abs().max()


def test_phase_plan_covers_every_input_position_once():
    for H, R, s, p in itertools.product((7, 8, 55, 56), (1, 2, 3, 5), (2, 3), (0, 1, 2)):
        if p > R - 1:
            continue
        OH = (H + 2 * p - R) // s + 1
        plan = _phase_plan(H, H, OH, OH, R, R, (s, s), (p, p, p, p), (1, 1))
        if plan is None:
            continue
        seen = torch.zeros(H, H, dtype=torch.int32)
        for (i0h, i0w, *_r) in plan:
            seen[i0h::s, i0w::s] += 1
        assert bool((seen == 1).all())


def test_phase_plan_declines_negative_pads():
    # 3x3 stride 3 pad 1: phase 0 would read dY one row past its window start (negative pad) -> zero-interleave path
    assert _phase_plan(20, 20, 7, 7, 3, 3, (3, 3), (1, 1, 1, 1), (1, 1)) is None
