"""The device categorical draw (np8_pick_batch: np8_assign's pick_step) against the oracle's reservoir, bit
for bit, on the golden weight vectors of tests/golden/pick_freq.json (the reference's own
random_weighted_pick frequencies, dim1algebra.hpp:2078-2104) and on random ones; and the device draws'
frequencies against the reference's table (chi-square)."""
import json
import os

import numpy as np
import pytest
from scipy import stats

import oracle as O

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pick_freq.json")))["cases"]


@pytest.fixture(scope="module")
def smp():
    from noparama_amd import NealAlgorithm8

    s = NealAlgorithm8(2, seed=1, device=0)
    yield s
    s.close()


@pytest.mark.parametrize("name", sorted(GOLD))
def test_device_pick_equals_oracle_on_golden_vectors(smp, name):
    c = GOLD[name]
    lw = np.asarray(c["lw"])
    u = np.random.Generator(np.random.PCG64(c["seed"])).random(c["n_draws"])
    dev = smp.pick_batch(lw, u)
    assert np.array_equal(dev, O.pick_reservoir_batch(lw, u))
    # and the device's frequencies against the reference function's own table (same uniforms)
    mine = np.bincount(dev, minlength=lw.size)
    ref = np.asarray(c["counts_shifted"])
    tab = np.vstack([mine, ref])
    tab = tab[:, tab.sum(axis=0) >= 10]
    if tab.shape[1] > 1:
        assert stats.chi2_contingency(tab).pvalue > 1e-4, (name, tab)


def test_device_pick_equals_oracle_random_vectors(smp):
    rng = np.random.default_rng(11)
    for n in (1, 2, 3, 7, 64, 67, 300):
        lw = rng.normal(0.0, rng.choice([0.5, 5.0, 60.0]), n)
        lw[0] = rng.choice([lw[0], -1e300])
        u = rng.random(4096)
        assert np.array_equal(smp.pick_batch(lw, u), O.pick_reservoir_batch(lw, u)), n
