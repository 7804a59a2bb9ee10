"""The chain's categorical draw against the reference's own, in distribution.

The reference picks with `algebra::random_weighted_pick` (/root/reference/include/helper/dim1algebra.hpp:
2078-2104): an inverse CDF over linear weights with one double uniform.  The specification's pick
(DESIGN.md "Pick"; oracle `pick_step`, device `np8::pick_step`) is a one-pass single-uniform reservoir over
log-weights with the -80 skip rule.  tests/golden/pick_freq.json holds frequency tables of the reference
function itself (compiled from its header, tests/golden/make_pick_freq.py) on fixed weight vectors:
near-threshold (-79/-81), widely spread, all-far (underflow), singleton-own and single-candidate cases.

CPU: the oracle's reservoir, fed independent uniforms, must reproduce the reference's frequencies (chi-square
homogeneity test, and goodness of fit against the exact probabilities); the oracle's inverse-CDF restatement
fed the golden uniforms reproduces the reference's counts exactly.  GPU: the device pick equals the
oracle's reservoir bit for bit on the same (weights, uniform) pairs (tests/test_gpu_pick.py).
"""
import json
import os

import numpy as np
import pytest
from scipy import stats

import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pick_freq.json")
CASES = json.load(open(GOLD))["cases"]
ALPHA = 1e-4  # significance of the chi-square tests (9 cases x 2 tests)


def golden_uniforms(case):
    return np.random.Generator(np.random.PCG64(case["seed"])).random(case["n_draws"])


def pooled(expected, *observed, min_exp=5.0):
    """Cells with expected count below min_exp merged into one (chi-square validity)."""
    big = expected >= min_exp
    out = [np.append(o[big], o[~big].sum()) for o in (expected,) + observed]
    if out[0][-1] < min_exp:  # the pooled cell itself too small: drop it
        out = [o[:-1] for o in out]
    return out


@pytest.mark.parametrize("name", sorted(CASES))
def test_invcdf_restatement_reproduces_reference_counts(name):
    c = CASES[name]
    lw = np.asarray(c["lw"])
    w = np.exp(lw - lw.max())
    got = np.zeros(lw.size, dtype=np.int64)
    for u in golden_uniforms(c):
        got[O.weighted_pick_ref(w, u)] += 1
    assert got.tolist() == c["counts_shifted"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_reservoir_matches_reference_in_distribution(name):
    c = CASES[name]
    lw = np.asarray(c["lw"])
    n = c["n_draws"]
    u = np.random.Generator(np.random.PCG64(c["seed"] + 777)).random(n)  # independent of the golden draws
    picks = O.pick_reservoir_batch(lw, u)
    mine = np.bincount(picks, minlength=lw.size).astype(np.float64)
    ref = np.asarray(c["counts_shifted"], dtype=np.float64)
    p = np.asarray(c["p"])
    # candidates the skip rule drops have probability below e^-80 relative to the maximum: the reference
    # never draws them either
    skip = lw < lw.max() - 80.0
    assert mine[skip].sum() == 0 and ref[skip].sum() == 0
    if (p > 0).sum() <= 1 or mine.size == 1:
        assert mine.sum() == n and np.array_equal(mine > 0, ref > 0)
        return
    # goodness of fit of both samplers against the exact probabilities
    for obs in (mine, ref):
        e, o = pooled(p * n, obs)
        if e.size > 1:
            assert stats.chisquare(o, e * (o.sum() / e.sum())).pvalue > ALPHA, (name, o, e)
    # homogeneity of the two samples (2 x k contingency table)
    e, a, b = pooled(p * n, mine, ref)
    if e.size > 1:
        tab = np.vstack([a, b])
        tab = tab[:, tab.sum(axis=0) > 0]
        if tab.shape[1] > 1:
            assert stats.chi2_contingency(tab).pvalue > ALPHA, (name, tab)


def test_underflow_case_documents_the_reference_fallback():
    """All linear weights underflow: the reference's raw form returns index 0 every time (a zero cumulative
    sum, lower_bound of 0); the log-space pick draws by relative weight -- the documented deviation
    (DESIGN.md "Pick")."""
    c = CASES["all_far"]
    assert c["counts_raw"][0] == c["n_draws"]
    lw = np.asarray(c["lw"])
    picks = O.pick_reservoir_batch(lw, golden_uniforms(c))
    mine = np.bincount(picks, minlength=lw.size)
    assert abs(mine[2] / c["n_draws"] - c["p"][2]) < 0.01 and mine[0] < c["n_draws"]


def test_reservoir_single_candidate_and_singleton_own():
    assert (O.pick_reservoir_batch(np.array([-3.0]), np.linspace(0.01, 0.99, 50)) == 0).all()
    lw = np.array([-1e300, -2.0, -1.0, -3.0])  # a singleton's own cluster: weight 0, never kept
    picks = O.pick_reservoir_batch(lw, np.random.default_rng(5).random(20000))
    assert (picks != 0).all()
