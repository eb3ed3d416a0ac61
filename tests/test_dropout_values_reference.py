"""Dropout implementations' values, after the reference's conf/dropout/TestDropout
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/dropout/TestDropout.java:178-290): inverted Dropout(p)
leaves 0 or 1/p (a fixed p and a MapSchedule that switches p from 0.5 to 0.1 at iteration 5); GaussianDropout(0.1)
multiplies by N(1, sqrt(0.1/0.9)); GaussianNoise(0.1) adds N(0, 0.1); AlphaDropout(p) keeps a*x + b or sets
a*alpha' + b with the SELU constants, a and b as in the paper. The input is never modified. CPU."""
import math

import pytest
import torch

import deeplearning4j_amd as D


def test_dropout_values_fixed_and_scheduled():
    torch.manual_seed(12345)
    x = torch.ones(10, 10, dtype=torch.float64)
    d = D.Dropout(0.5)
    out = d.applyDropout(x.clone(), 0, 0, False)
    zeros, twos = int((out == 0).sum()), int((out == 2).sum())
    assert zeros + twos == 100 and 25 <= zeros <= 75 and 25 <= twos <= 75
    d = D.Dropout(D.MapSchedule.Builder(D.ScheduleType.ITERATION).add(0, 0.5).add(5, 0.1).build())
    for i in range(10):
        inp = x.clone()
        out = d.applyDropout(inp, i, 0, False)
        assert torch.equal(inp, x)
        zeros = int((out == 0).sum())
        if i < 5:
            twos = int((out == 2).sum())
            assert zeros + twos == 100 and 25 <= zeros <= 75, i
        else:
            tens = int(torch.isclose(out, torch.full_like(out, 10.0)).sum())
            assert zeros + tens == 100 and zeros >= 80 and tens <= 20, i


def test_gaussian_dropout_and_noise_values():
    torch.manual_seed(12345)
    x = torch.ones(50, 50, dtype=torch.float64)
    out = D.GaussianDropout(0.1).applyDropout(x.clone(), 0, 0, False)
    assert abs(float(out.mean()) - 1.0) < 0.05
    assert abs(float(out.std()) - math.sqrt(0.1 / 0.9)) < 0.02
    out = D.GaussianNoise(0.1).applyDropout(x.clone(), 0, 0, False)
    assert abs(float(out.mean()) - 1.0) < 0.05
    assert abs(float(out.std()) - 0.1) < 0.01


def test_alpha_dropout_values():
    torch.manual_seed(12345)
    p = 0.4
    alpha, lam = 1.6732632423543772, 1.0507009873554804
    ap = -lam * alpha
    a = 1.0 / math.sqrt(p + ap * ap * p * (1 - p))
    b = -1.0 / math.sqrt(p + ap * ap * p * (1 - p)) * (1 - p) * ap
    d = D.AlphaDropout(p)
    assert d.a(p) == pytest.approx(a, abs=1e-6)
    assert d.b(p) == pytest.approx(b, abs=1e-6)
    out = d.applyDropout(torch.ones(10, 10, dtype=torch.float64), 0, 0, False).reshape(-1)
    dropped = int((out - (a * ap + b)).abs().lt(1e-6).sum())
    kept = int((out - (a + b)).abs().lt(1e-6).sum())
    assert dropped + kept == 100 and 25 <= dropped <= 75 and 25 <= kept <= 75
