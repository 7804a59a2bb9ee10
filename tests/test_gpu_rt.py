"""The fp64 contraction above D = 16 (and at (D, M) pairs without a templated instance): np8_rt.hip's kernels with D
and M at run time, against the oracle's F64 path (oracle/np8_oracle.c: the same packed sym(Sigma^{-1}) form with D at
run time) -- labels, counts and K bit for bit, log-likelihoods to 1e-12 -- and against the per-call general-inverse
formula (np8o_loglik_matrix_ref: LU log-determinant and solve, the reference's multivariatenormal.cpp:84-92) to
1e-10.  The reference's data_t has any length (include/np_data.h:9)."""
import os
import sys

import numpy as np
import pytest

from noparama_amd import NealAlgorithm8, datasets

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle as O  # noqa: E402  (test infrastructure: the checker)

pytestmark = pytest.mark.gpu

LL_RTOL = 1e-12  # device vs oracle, the same operations in the same order (differences: libm vs device exp/log)
REF_RTOL = 1e-10  # device vs the general-inverse formula (another arithmetic)


def pair(D, seed, M=3, kcap=512, **kw):
    return (NealAlgorithm8(D, M=M, seed=seed, kcap=kcap, device=0, **kw),
            O.Chain(D, M=M, seed=seed, kcap=kcap, **kw))


def same_state(g, o):
    sg, so = g.state(), o.state()
    assert sg["K"] == so["K"]
    assert np.array_equal(sg["z"], so["z"])
    assert np.array_equal(sg["counts"], so["counts"])
    np.testing.assert_allclose(sg["mu"], so["mu"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(sg["sigma"], so["sigma"], rtol=1e-13, atol=1e-15)


def spd(D, K, seed):
    """K random SPD covariances (not isotropic: the packed quadratic form, not iso |d|^2)."""
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(K, D, D)) / np.sqrt(D)
    return 0.3 * np.einsum("kab,kcb->kac", A, A) + 0.2 * np.eye(D)[None]


@pytest.mark.parametrize("D,N", [(20, 6000), (32, 4000), (64, 2500), (100, 1200)])
def test_fp64_above_16_bit_exact(D, N):
    """Warm start with non-isotropic covariances, then the reference's initialisation (init_random(20)): the runtime-D
    kernels follow the oracle bit for bit (new clusters from the auxiliaries' (v, mu), candidate lists, radii)."""
    X, z, mu, _ = datasets.mixture(N, D, 6, 0.6, 6.0, seed=D)
    sig = spd(D, 6, D)
    g, o = pair(D, 500 + D)
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, mu, sig)
    g.sweep(3)
    o.sweep(3)
    same_state(g, o)
    idx = np.arange(24)
    lg, lo = g.loglik_matrix(idx), o.loglik_matrix(idx)
    np.testing.assert_allclose(lg, lo, rtol=LL_RTOL, atol=1e-12)
    np.testing.assert_allclose(lg, o.loglik_matrix(idx, ref=True), rtol=REF_RTOL, atol=1e-9)
    for c in (g, o):
        c.init_random(20)
    g.sweep(12)
    o.sweep(12)
    same_state(g, o)
    assert g.stats()["new_clusters"] > 0
    assert [g.stats()["new_clusters"], g.stats()["rejected_requests"]] == list(o.request_stats)
    np.testing.assert_allclose(g.loglik_matrix(idx), o.loglik_matrix(idx), rtol=LL_RTOL, atol=1e-12)


def test_fp64_rt_non_isotropic_base_measure_and_sequential():
    """D = 24 with a non-isotropic Lambda (every G0 draw a full packed form) in the data-parallel sweep and in the
    reference's sequential sweep (chunk = 1), and D = 12 with M = 2 (a pair without a templated instance)."""
    D, N = 24, 1500
    X, z, mu, _ = datasets.mixture(N, D, 5, 0.6, 6.0, seed=3)
    rng = np.random.default_rng(4)
    B = rng.normal(size=(D, D)) / D
    Lam = 0.01 * (np.eye(D) + B @ B.T)
    for chunk in (0, 1):
        g, o = pair(D, 71, Lambda=Lam, chunk=chunk)
        for c in (g, o):
            c.set_data(X)
            c.init_random(10)
        g.sweep(4)
        o.sweep(4)
        same_state(g, o)
    X2, z2, mu2, sig2 = datasets.mixture(4000, 12, 6, 0.6, 6.0, seed=12)
    g, o = pair(12, 90, M=2)
    for c in (g, o):
        c.set_data(X2)
        c.init_random(20)
    g.sweep(10)
    o.sweep(10)
    same_state(g, o)


def test_fp64_rt_max_likelihood_check():
    """The max-likelihood check (np8_loglik_rt) at D = 40: the best labelling and its log-likelihood match the
    oracle's."""
    D, N = 40, 3000
    X, z, mu, sig = datasets.mixture(N, D, 6, 0.6, 6.0, seed=40)
    g, o = pair(D, 640)
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    g.sweep(10)
    o.sweep(10)
    same_state(g, o)
    np.testing.assert_allclose(g.stats()["best_loglik"], o.best_loglik(), rtol=1e-11)
    bg, bo = g.state(which=1), o.state(which=1)
    assert np.array_equal(bg["z"], bo["z"])


@pytest.mark.parametrize("D", [8, 12, 24])
def test_non_isotropic_rows_pruned_bit_exact(D):
    """Rows that are not isotropic (full covariances; a non-isotropic Lambda, so every G0 draw too) are left out of
    the candidate lists by the slots' precision eigenvalue bounds (prune_row, round 6) -- on the templated path's
    general kernel (D = 8, 12) and on the run-time-D one (D = 24): labels, counts and K bit-exact against the oracle,
    which walks every row."""
    N = 12000
    X, z, mu, _ = datasets.mixture(N, D, 8, 0.6, 8.0, seed=100 + D)
    sig = spd(D, 8, 7 + D)
    rng = np.random.default_rng(5)
    B = rng.normal(size=(D, D)) / D
    g, o = pair(D, 800 + D, Lambda=0.01 * (np.eye(D) + B @ B.T))
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, mu, sig)
    g.sweep(12)
    o.sweep(12)
    same_state(g, o)
    for c in (g, o):
        c.init_random(20)
    g.sweep(12)
    o.sweep(12)
    same_state(g, o)
