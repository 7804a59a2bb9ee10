"""GPU: the per-sweep launch reductions are transparent to the chain (DESIGN.md §5 "Fewer launches per sweep").

* the folded max-likelihood check (np8_assign_fast sums the items' log-likelihoods, finalize decides the snapshot,
  the next assign copies it) against the separate np8_loglik / np8_loglik_reduce / np8_snapshot kernels
  (NP8_NO_LLFOLD=1), and against the oracle;
* the conditional candidate lists (finalize keeps the last build while the counts stay within kListSlack) against a
  rebuild after every step (NP8_LISTS_ALWAYS=1).

Labels, counts, K and the snapshot bit-exact; the log-likelihoods within 1e-11 relative (summation order).
The runs mix eager sweeps with 20-sweep graph replays, start from the reference's initialisation (new-cluster
requests accepted and rejected: the requests' dll terms) and from the warm state, and read the snapshot at
points where a copy is still pending (np8_snapshot_flush)."""
import os

import numpy as np
import pytest

import oracle as O
from noparama_amd import NealAlgorithm8, datasets

pytestmark = pytest.mark.gpu


def make(env, D, seed, **kw):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return NealAlgorithm8(D, seed=seed, device=0, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def same(a, b, which, ll=True):
    sa, sb = a.state(which), b.state(which)
    assert sa["K"] == sb["K"]
    assert np.array_equal(sa["z"], sb["z"])
    assert np.array_equal(sa["counts"], sb["counts"])
    np.testing.assert_array_equal(sa["mu"], sb["mu"])
    if ll:
        ta, tb = a.stats(), b.stats()
        np.testing.assert_allclose(ta["best_loglik"], tb["best_loglik"], rtol=1e-11)


@pytest.mark.parametrize("start", ["init_random", "warm"])
def test_fold_and_conditional_lists_transparent(start):
    X, zt, mu, sig = datasets.config_c3(N=60_000)
    runs = [make({}, 8, 5),
            make({"NP8_NO_LLFOLD": "1", "NP8_LISTS_ALWAYS": "1"}, 8, 5),
            make({"NP8_LISTS_ALWAYS": "1"}, 8, 5)]
    for s in runs:
        s.set_data(X)
        if start == "warm":
            s.set_state(zt, mu, sig)
        else:
            s.init_random(20)
    # eager sweeps, a read with a possibly pending snapshot (after sweep 5, a check), graph replays, eager again
    for n in (6, 1, 20, 3, 20, 7):
        for s in runs:
            s.sweep(n)
        for s in runs[1:]:
            same(runs[0], s, 0)
            same(runs[0], s, 1)
    st = [s.stats() for s in runs]
    assert st[0]["folded_checks"] == 12 and st[0]["tail_steps"] > 0  # the paths under test did run
    assert st[1]["folded_checks"] == 0 and st[1]["tail_steps"] == 0
    assert st[2]["folded_checks"] == 12 and st[2]["tail_steps"] == 0
    if start == "warm":  # a fixed point: the lists of the gathering sweeps are never rebuilt in between
        assert st[0]["tail_list_builds"] == 0


def test_fold_against_oracle_cold_start():
    """N = 20k from init_random: 46 sweeps (graph replays included) bit-exact against the oracle, snapshot too."""
    X, _, _, _ = datasets.config_c3(N=20_000)
    g = NealAlgorithm8(8, seed=3, device=0)
    o = O.Chain(8, seed=3, kcap=g.kcap)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    for n in (5, 1, 20, 20):
        g.sweep(n)
        o.sweep(n)
        sa, sb = g.state(0), o.state(0)
        assert np.array_equal(sa["z"], sb["z"])
        ba, bb = g.state(1), o.state(1)
        assert np.array_equal(ba["z"], bb["z"])
        assert np.array_equal(ba["counts"], bb["counts"])
        np.testing.assert_allclose(g.stats()["best_loglik"], o.best_loglik(), rtol=1e-11)


@pytest.mark.parametrize("D", [40, 64])
def test_wide_fold_transparent(D):
    """The wide path's folded check (the default: np8_assign_wide sums the items' log-likelihoods per wave,
    np8_ll_fix_wide moves the accepted requesters) against the separate np8_loglik_wide_mfma pass (NP8_WIDE_LLFOLD=0): labels,
    counts and the snapshot bit-exact, the best log-likelihood within 1e-11 relative, through eager sweeps and a
    graph replay from init_random (new clusters every early sweep)."""
    X, _, _, _ = datasets.mixture(12_000, D, 12, 1.0, 5.0, seed=9)
    kw = dict(prior="niw", contraction="f32", mu0=np.full(D, 6.0), kappa=0.01, nu=D + 2.0, Lambda=np.eye(D))
    runs = [make({}, D, 13, **kw), make({"NP8_WIDE_LLFOLD": "0"}, D, 13, **kw)]
    for s in runs:
        s.set_data(X)
        s.init_random(20)
    for n in (6, 1, 20, 3):
        for s in runs:
            s.sweep(n)
        same(runs[0], runs[1], 0)
        same(runs[0], runs[1], 1)
    assert runs[0].stats()["folded_checks"] > 0 and runs[1].stats()["folded_checks"] == 0
