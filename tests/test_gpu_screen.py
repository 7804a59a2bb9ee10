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
