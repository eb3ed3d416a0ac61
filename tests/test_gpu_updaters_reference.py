"""The fused HIP updater kernel (csrc/updater.hip) against the reference's TestUpdaters hand calculations."""
import pytest
import torch

import _updater_ref as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", sorted(R.CASES))
def test_fused_updater_matches_reference_formulas(kind):
    actual, exp = R.run_network_updates(kind, "cuda")
    for a, e in zip(actual, exp):
        assert torch.allclose(a, e, rtol=2e-5, atol=1e-7), (kind, (a - e).abs().max())
