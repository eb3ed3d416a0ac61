"""Updater math pinned to the reference's TestUpdaters hand calculations (host reference path)."""
import pytest
import torch

import _updater_ref as R


@pytest.mark.parametrize("kind", sorted(R.CASES))
def test_updater_matches_reference_formulas(kind):
    actual, exp = R.run_network_updates(kind, "cpu")
    for a, e in zip(actual, exp):
        assert torch.allclose(a, e, rtol=1e-5, atol=1e-7), (kind, (a - e).abs().max())
