"""GPU parity of the Jain-Neal split-merge sweep (np8_sm_sweep, noparama_amd/csrc/np8_sm.hip) against
the oracle's np8o_sm_sweep on identical inputs: labels, counts, parameters and the attempt outcome
counts bit for bit.  The device evaluates attempts in speculative batches against the batch-start
state and applies the first acceptance; the oracle runs them one by one -- equal results show the
batching changes nothing.
"""
import numpy as np
import pytest

import oracle as O
from noparama_amd import JainNealAlgorithm, NealAlgorithm8, NP8Error, datasets

pytestmark = pytest.mark.gpu

OUT_KEYS = ("skipped", "split_rejected", "merge_rejected", "split_accepted", "merge_accepted", "split_no_slot")


def pair(D, seed, kcap=256, **kw):
    return (JainNealAlgorithm(D, seed=seed, kcap=kcap, device=0, **kw), O.Chain(D, seed=seed, kcap=kcap, **kw))


def assert_same(g, o):
    sg, so = g.state(), o.state()
    assert sg["K"] == so["K"]
    assert np.array_equal(sg["z"], so["z"])
    assert np.array_equal(sg["counts"], so["counts"])
    assert np.array_equal(sg["mu"], so["mu"])
    assert np.array_equal(sg["sigma"], so["sigma"])
    st = g.sm_stats()
    assert [st[k] for k in OUT_KEYS] == o.sm_stats.tolist()


@pytest.mark.parametrize("D,N", [(2, 600), (3, 900)])
def test_random_start_parity(D, N):
    X, _, _, _ = datasets.mixture(N, D, 4, 0.3, 6.0, seed=11)
    g, o = pair(D, seed=3)
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    for s in range(4):
        g.sweep(1)
        o.sm_sweep(1)
        assert_same(g, o)
    assert o.sm_stats[4] > 0  # merges happened


def test_twogaussians_parity():
    X, gt = datasets.twogaussians()
    kw = dict(mu0=np.array([6.0, 6.0]), kappa=1.0 / 500, nu=4.0, Lambda=0.01 * np.eye(2))
    g, o = pair(2, seed=9, **kw)
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    g.sweep(10)
    o.sm_sweep(10)
    assert_same(g, o)
    assert g.stats()["best_loglik"] == pytest.approx(o.best_loglik(), rel=1e-12)


@pytest.mark.parametrize("D", [8, 16])
def test_warm_start_splits(D):
    """A warm state with a few wide clusters: the split moves (new G0 clusters, SAMS allocation over
    thousands of members in LDS chunks) are exercised; Lambda small so G0 draws are plausible."""
    N = 6000 if D == 8 else 3000
    X, gt, mu, sig = datasets.mixture(N, D, 6, 0.8, 8.0, seed=21)
    zr = (gt // 2).astype(np.int32)  # 3 clusters, each the union of two true components
    mu3 = np.stack([X[zr == k].mean(axis=0) for k in range(3)])
    sig3 = np.stack([np.cov(X[zr == k].T) + 0.1 * np.eye(D) for k in range(3)])
    kw = dict(mu0=X.mean(axis=0), kappa=0.05, nu=0.5, Lambda=(1.0 / D) * np.eye(D))
    g, o = pair(D, seed=5, **kw)
    for c in (g, o):
        c.set_data(X)
        c.set_state(zr, mu3, sig3)
    g.sweep(2)
    o.sm_sweep(2)
    assert_same(g, o)


def test_mixed_with_gibbs_and_mh():
    """Split-merge sweeps interleaved with Gibbs sweeps (and the mh_g0 parameter step): both paths
    read and write the same device state."""
    X, _, _, _ = datasets.mixture(800, 2, 4, 0.3, 6.0, seed=11)
    g, o = pair(2, seed=13, param_update="mh_g0")
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    for s in range(3):
        g.sweep(1)
        o.sm_sweep(1)
        g.sweep_gibbs(1)
        o.sweep(1)
        assert_same(g, o)


def test_rejects_unsupported():
    X, _, _, _ = datasets.mixture(200, 4, 2, 0.3, 6.0, seed=1)
    g = NealAlgorithm8(4, seed=1, kcap=64, device=0, prior="niw", mu0=np.zeros(4), kappa=0.1, nu=6.0,
                       Lambda=np.eye(4))
    g.set_data(X)
    g.init_random(5)
    with pytest.raises(NP8Error):
        g.sm_sweep(1)


@pytest.mark.parametrize("D", [2, 4])
def test_far_cluster_splits(D):
    """One cluster of 3000 items whose mean is far from all of them: splits with thousands of moved
    members (three LDS chunks) are accepted and merged back."""
    rng = np.random.default_rng(0)
    N = 3000
    X = np.concatenate([rng.normal(size=(N // 2, D)) * 0.5 + 3, rng.normal(size=(N // 2, D)) * 0.5 - 3])
    z = np.zeros(N, np.int32)
    kw = dict(mu0=np.zeros(D), kappa=0.2, nu=0.5, Lambda=0.25 * np.eye(D))
    g, o = pair(D, seed=1, kcap=64, **kw)
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, np.full((1, D), 50.0), np.eye(D)[None])
    g.sweep(2)
    o.sm_sweep(2)
    assert_same(g, o)
    assert o.sm_stats[3] >= 2


def test_kcap_saturation_parity():
    """kcap = the live clusters: accepted splits find no free slot (outcome 5) until merges free one."""
    X, _, _, _ = datasets.mixture(600, 2, 4, 0.3, 6.0, seed=11)
    g, o = pair(2, seed=21, kcap=20)
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    for s in range(3):
        g.sweep(1)
        o.sm_sweep(1)
        assert_same(g, o)
