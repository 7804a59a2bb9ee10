"""GPU parity of the triadic split-merge sweep (np8_tri_sweep, noparama_amd/csrc/np8_sm.hip) against the
oracle's np8o_tri_sweep: labels, counts, parameters and the outcome counts of every move kind, bit for
bit (speculative batches on the device, one attempt at a time in the oracle).
"""
import numpy as np
import pytest

import oracle as O
from noparama_amd import NP8Error, TriadicAlgorithm, datasets

pytestmark = pytest.mark.gpu

KEYS = ("skipped", "dyadic_merge_rejected", "dyadic_merge_accepted", "dyadic_split_rejected",
        "dyadic_split_accepted", "triadic_merge_rejected", "triadic_merge_accepted", "triadic_split_rejected",
        "triadic_split_accepted", "split_no_slot")


def pair(D, seed, kcap=256, **kw):
    return (TriadicAlgorithm(D, seed=seed, kcap=kcap, device=0, **kw), O.Chain(D, seed=seed, kcap=kcap, **kw))


def assert_same(g, o):
    sg, so = g.state(), o.state()
    assert sg["K"] == so["K"]
    assert np.array_equal(sg["z"], so["z"])
    assert np.array_equal(sg["counts"], so["counts"])
    assert np.array_equal(sg["mu"], so["mu"])
    assert np.array_equal(sg["sigma"], so["sigma"])
    st = g.tri_stats()
    assert [st[k] for k in KEYS] == o.tri_stats.tolist()


@pytest.mark.parametrize("D,N", [(2, 600), (3, 500), (8, 400)])
def test_random_start_parity(D, N):
    X, _, _, _ = datasets.mixture(N, D, 4, 0.3, 6.0, seed=11)
    g, o = pair(D, seed=3)
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    for s in range(4):
        g.sweep(1)
        o.tri_sweep(1)
        assert_same(g, o)
    st = o.tri_stats
    assert st[2] > 0 and st[6] > 0 and st[8] > 0  # dyadic merges, triadic merges and splits accepted


def test_twogaussians_parity():
    X, gt = datasets.twogaussians()
    kw = dict(mu0=np.array([6.0, 6.0]), kappa=1.0 / 500, nu=4.0, Lambda=0.01 * np.eye(2))
    g, o = pair(2, seed=9, **kw)
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    g.sweep(20)
    o.tri_sweep(20)
    assert_same(g, o)


def test_large_clusters_parity():
    """Members walked in several 64-lane steps and across three source clusters (far means so the
    moves are accepted)."""
    rng = np.random.default_rng(0)
    N, D = 3000, 2
    X = np.concatenate([rng.normal(size=(N // 2, D)) * 0.5 + 3, rng.normal(size=(N // 2, D)) * 0.5 - 3])
    z = (np.arange(N) % 3).astype(np.int32)
    kw = dict(mu0=np.zeros(D), kappa=0.2, nu=0.5, Lambda=0.25 * np.eye(D))
    g, o = pair(D, seed=1, kcap=64, **kw)
    mus = np.array([[40.0, 40.0], [-40.0, 40.0], [0.0, -40.0]])
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, mus, np.stack([np.eye(D)] * 3))
    g.sweep(2)
    o.tri_sweep(2)
    assert_same(g, o)


def test_mixed_with_gibbs():
    X, _, _, _ = datasets.mixture(500, 2, 4, 0.3, 6.0, seed=11)
    g, o = pair(2, seed=13, param_update="mh_g0")
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    for s in range(2):
        g.sweep(1)
        o.tri_sweep(1)
        g.sweep_gibbs(1)
        o.sweep(1)
        assert_same(g, o)


def test_rejects_niw():
    X, _, _, _ = datasets.mixture(200, 4, 2, 0.3, 6.0, seed=1)
    g = TriadicAlgorithm(4, seed=1, kcap=64, device=0, prior="niw", mu0=np.zeros(4), kappa=0.1, nu=6.0,
                         Lambda=np.eye(4))
    g.set_data(X)
    g.init_random(5)
    with pytest.raises(NP8Error):
        g.sweep(1)


def test_kcap_saturation_parity():
    X, _, _, _ = datasets.mixture(500, 2, 4, 0.3, 6.0, seed=11)
    g, o = pair(2, seed=21, kcap=20)
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    for s in range(3):
        g.sweep(1)
        o.tri_sweep(1)
        assert_same(g, o)


def test_merge_bound_warm_state_parity(monkeypatch):
    """Well-separated warm state (C3's shape, smaller): the triadic merges are rejected by the merge bound
    (np8_tri_bound / tri_merge_bound_rejects) without their walk.  Same chain as the oracle and as the
    device with the bound off (NP8_TRI_BOUND=0), bit for bit, outcome counts included."""
    N, D, K = 6000, 8, 8
    X, z, mu, sig = datasets.mixture(N, D, K, 0.8, 20.0, seed=5)
    g, o = pair(D, seed=17, kcap=64)
    monkeypatch.setenv("NP8_TRI_BOUND", "0")
    g_off = TriadicAlgorithm(D, seed=17, kcap=64, device=0)
    monkeypatch.delenv("NP8_TRI_BOUND")
    for c in (g, o, g_off):
        c.set_data(X)
        c.set_state(z, mu, sig)
    g.sweep(2)
    g_off.sweep(2)
    o.tri_sweep(2)
    assert_same(g, o)
    assert_same(g_off, o)
    assert o.tri_stats[5] > 500  # triadic merges rejected: the bound's case
