"""Triadic split-merge oracle (src/np_triadic_algorithm.cpp restated as np8o_tri_sweep):
invariants, determinism, every move kind firing, and the behaviour the reference's README promises
for `-a triadic` on twogaussians (README.rst:53-55: purity "should be almost 1").  No reference
fixture pins the chain (the reference is unseeded and unbuildable here)."""
import numpy as np

import oracle as O
from noparama_amd import datasets


def chain(D=2, N=400, seed=3, K=20):
    X, gt, _, _ = datasets.mixture(N, D, 4, 0.3, 6.0, seed=11)
    c = O.Chain(D, seed=seed, kcap=256)
    c.set_data(X)
    c.init_random(K)
    return c, X, gt


def test_invariants_and_stats():
    c, X, _ = chain()
    for s in range(3):
        c.tri_sweep(1)
        st = c.state()
        assert st["counts"].sum() == X.shape[0]
        assert np.array_equal(np.bincount(st["z"], minlength=st["K"]), st["counts"])
        assert (st["counts"] > 0).all()
        assert c.tri_stats.sum() == (s + 1) * X.shape[0]


def test_every_move_kind_and_determinism():
    a, _, _ = chain(seed=5)
    b, _, _ = chain(seed=5)
    a.tri_sweep(4)
    b.tri_sweep(4)
    assert np.array_equal(a.state()["z"], b.state()["z"])
    st = a.tri_stats
    assert np.array_equal(st, b.tri_stats)
    for k in (1, 2, 5, 6, 7, 8):  # dyadic merges, triadic merges and splits, rejected and accepted
        assert st[k] > 0, st


def test_twogaussians_purity():
    X, gt = datasets.twogaussians()
    c = O.Chain(2, seed=9, kcap=64, mu0=np.array([6.0, 6.0]), kappa=1.0 / 500, nu=4.0, Lambda=0.01 * np.eye(2))
    c.set_data(X)
    c.init_random(20)
    c.tri_sweep(30)
    z = c.state()["z"]
    purity = sum(np.bincount(gt[z == k]).max() for k in np.unique(z)) / len(z)
    assert purity > 0.9
