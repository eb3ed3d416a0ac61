"""Distribution JSON, after the reference's TestDistributionDeserializer
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/distribution/serde/TestDistributionDeserializer.java):
Normal, Uniform, Gaussian and Binomial distributions round-trip through JSON unchanged, and read back through the
reference's getters. CPU."""
import pytest

import deeplearning4j_amd as D
from deeplearning4j_amd.nn.conf.base import Config


@pytest.mark.parametrize("d", [D.NormalDistribution(3, 0.5), D.UniformDistribution(-2, 1),
                               D.GaussianDistribution(2, 1.0), D.BinomialDistribution(10, 0.3)],
                         ids=lambda d: type(d).__name__)
def test_distribution_round_trip(d):
    back = Config.fromJson(d.toJson())
    assert type(back) is type(d) and back == d


def test_distribution_getters():
    n = Config.fromJson(D.NormalDistribution(0.1, 1.2).toJson())
    assert n.getMean() == pytest.approx(0.1) and n.getStd() == pytest.approx(1.2)
    u = Config.fromJson(D.UniformDistribution(-1.1, 2.2).toJson())
    assert u.getLower() == pytest.approx(-1.1) and u.getUpper() == pytest.approx(2.2)
