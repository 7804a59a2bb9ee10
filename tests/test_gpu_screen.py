"""The auxiliary screen near v = 0 (DESIGN.md "Auxiliary screen"; np8_kernels.hip aux_screen_ub).

The reference's G0 draws v ~ N(D, nu) (include/statistics/invwishart.h:30-31) and scales the covariance by v^2,
so |v| near 0 gives a tiny covariance and ill-conditioned ny/|v|, -D log|v| terms.  The screen is disabled only
below |v| = 0.02.  Here nu is large against D so that a few percent of all auxiliaries fall in |v| in
[0.02, 0.25], the items sit near mu0 (small ny, so those auxiliaries are competitive), and the only existing
cluster is a poor fit (the running maximum stays low).  In count mode (set_timing(counters=True)) the kernel
evaluates every screened auxiliary exactly and counts lanes where the screen skipped one that pick_step would
not have skipped: there must be none, and the chain must equal the oracle's (which has no screen).
"""
import numpy as np
import pytest

import oracle as O
from noparama_amd import NealAlgorithm8

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D,nu", [(2, 4.0), (3, 6.0), (8, 16.0)])
def test_screen_has_no_violations_near_v_zero(D, nu):
    rng = np.random.default_rng(D)
    N = 200_000
    mu0 = np.full(D, 6.0)
    X = mu0 + 0.02 * rng.normal(size=(N, D))
    z = np.zeros(N, np.int32)
    mu = (mu0 + 3.0)[None]
    sig = np.eye(D)[None] * 4.0
    kw = dict(seed=70 + D, kcap=4096, mu0=mu0, kappa=1.0 / 500, nu=nu, Lambda=0.01 * np.eye(D))
    g = NealAlgorithm8(D, device=0, **kw)
    o = O.Chain(D, **kw)
    O.set_threads(16)
    try:
        g.set_timing(True, counters=True)
        for c in (g, o):
            c.set_data(X)
            c.set_state(z, mu, sig)
        s0 = g.stats()
        for _ in range(2):
            g.sweep(1)
            o.sweep(1)
            sg, so = g.state(params=False), o.state()
            assert sg["K"] == so["K"] and np.array_equal(sg["z"], so["z"])
        s1 = g.stats()
        assert s1["screen_violations"] - s0["screen_violations"] == 0
        if D <= 3:
            assert s1["new_clusters"] > 0  # auxiliaries were picked: the screened region mattered
        # the regime is populated: a few percent of G0 draws have |v| < 1/4 (P(|D + nu g| < 1/4))
        from math import erf, sqrt
        p = 0.5 * (erf((0.25 - D) / nu / sqrt(2)) - erf((-0.25 - D) / nu / sqrt(2)))
        assert p * N * 3 > 1000
    finally:
        O.set_threads(1)
        g.close()


@pytest.mark.parametrize("D,M,nu", [(3, 3, 4.0), (5, 3, 4.0), (8, 1, 4.0), (8, 3, 4.0), (8, 4, 16.0), (16, 3, 4.0),
                                    (16, 2, 40.0)])
def test_level0_bound_holds(D, M, nu):
    """Level 0 of the auxiliary screen (round 6, np8_kernels.hip aux_screen0_ub): from the item's prefix call alone,
    an upper bound of every auxiliary's exact log-likelihood -- for items near mu0 (where it must give way: +inf or a
    large bound), at the C3 scale of distances and far beyond, and for nu large against D (|v| reaching 0).  Each bound
    (without the caller's 1e-4 |threshold| term) lies above the exact value np8_loglik_matrix computes; at the C3
    distances it clears most auxiliaries by far more than the skip threshold."""
    rng = np.random.default_rng(100 + D + M)
    n = 6000
    mu0 = np.full(D, 6.0)
    scale = np.concatenate([np.full(n // 6, 0.01), np.full(n // 6, 0.3), np.full(n // 6, 3.0), np.full(n // 6, 12.0),
                            np.full(n // 6, 40.0), np.full(n - 5 * (n // 6), 400.0)])
    X = mu0 + scale[:, None] * rng.normal(size=(n, D))
    z = np.zeros(n, np.int32)
    g = NealAlgorithm8(D, M=M, seed=5 + D, device=0, kappa=1.0 / 500, nu=nu, mu0=mu0, Lambda=0.01 * np.eye(D))
    try:
        g.set_data(X)
        g.set_state(z, mu0[None] + 1.0, np.eye(D)[None])
        idx = np.arange(n)
        for _ in range(2):  # two epochs: fresh draws
            ll = g.loglik_matrix(idx)[:, -M:]
            ub = g.aux_bounds(idx)
            assert np.all(np.isfinite(ll))
            bad = ll > ub
            assert not bad.any(), (ll[bad][:5], ub[bad][:5])
            g.sweep(1)
        if D > 8:  # no prefixes above D = 8 (np8_device.h kPreMaxD): no level-0 bound, the round-5 screen instead
            assert np.all(np.isinf(ub))
        elif D == 8 and nu == 4.0:  # the C3-like regime (|x - mu0| ~ 12-40): the bound sits far below the own cluster
            far = (scale >= 12.0) & (scale <= 40.0)
            assert np.mean(ub[far] < -200.0) > 0.9
    finally:
        g.close()
