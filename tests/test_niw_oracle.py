"""NIW prior in the CPU oracle (DESIGN.md "Priors").

The reference's NIW update is a stub (include/statistics/normalinvwishart.h:66-75) and its G0 never
draws a full inverse Wishart, so no reference fixture pins this extension: it is pinned by exact
identities and by its distribution ("parity unpinned" against the reference, checked against the
mathematics instead):
  * the item-frame auxiliary likelihood equals the general-inverse likelihood of the fully built
    auxiliary draw (multivariatenormal.cpp:106-136 restated) -- the derivation, exactly;
  * the specification's Marsaglia-Tsang gamma is Gamma(alpha) (KS against scipy);
  * G0, auxiliary and posterior draws have the Normal-Inverse-Wishart moments.
"""
import numpy as np
import pytest
from scipy import stats

import oracle as O


def spd(rng, D, scale=1.0):
    A = rng.normal(size=(D, D))
    return scale * (A @ A.T / D + 0.5 * np.eye(D))


@pytest.mark.parametrize("alpha", [1.0, 1.5, 4.0, 33.0, 2000.0])
def test_gamma_mt_distribution(alpha):
    g = np.array([O.gamma_mt(7, i, 3, 8, 0, alpha) for i in range(6000)])
    assert stats.kstest(g, stats.gamma(alpha).cdf).pvalue > 1e-3
    assert abs(g.mean() - alpha) < 5 * np.sqrt(alpha / g.size)


@pytest.mark.parametrize("D", [1, 2, 3, 5, 8, 16, 64])
def test_aux_item_frame_equals_full_draw(D):
    rng = np.random.default_rng(D)
    mu0 = rng.normal(size=D)
    ch = O.Chain(D, mu0=mu0, kappa=0.05, nu=D + 3.0, Lambda=spd(rng, D), seed=5, kcap=64, prior="niw",
                 param_update="niw_conjugate")
    ch.set_data(mu0 + 2.0 * rng.normal(size=(40, D)))
    ch.init_random(5)
    idx = np.arange(8)
    fast, ref = ch.loglik_matrix(idx), ch.loglik_matrix(idx, ref=True)
    np.testing.assert_allclose(fast, ref, rtol=1e-11, atol=1e-11)


def test_g0_and_aux_moments():
    rng = np.random.default_rng(2)
    D, k0, nu0 = 3, 0.5, 13.0
    Psi, mu0 = spd(rng, D, 3.0), np.array([1.0, -2.0, 0.5])
    ES = Psi / (nu0 - D - 1)
    ch = O.Chain(D, mu0=mu0, kappa=k0, nu=nu0, Lambda=Psi, seed=9, kcap=64, prior="niw")
    ch.set_data(mu0 + 3.0 * rng.normal(size=(1500, D)))
    ch.init_random(3)
    mus, sgs = zip(*[ch.aux_params(i) for i in range(1500)])
    mus, sgs = np.concatenate(mus), np.concatenate(sgs)
    assert np.abs(sgs.mean(0) - ES).max() < 0.03 * np.abs(ES).max()
    assert np.abs(np.cov(mus.T) - ES / k0).max() < 0.05 * np.abs(ES / k0).max()
    z = (mus.mean(0) - mu0) / np.sqrt(np.diag(ES) / k0 / len(mus))
    assert np.all(np.abs(z) < 4.5)
    pm, ps = zip(*[ch.niw_draw(i, 77, 3) for i in range(4000)])
    pm, ps = np.array(pm), np.array(ps)
    assert np.abs(ps.mean(0) - ES).max() < 0.03 * np.abs(ES).max()
    assert np.abs(np.cov(pm.T) - ES / k0).max() < 0.05 * np.abs(ES / k0).max()


def test_posterior_moments():
    rng = np.random.default_rng(4)
    D, k0, nu0, n = 3, 0.5, 7.0, 50
    Psi, mu0 = spd(rng, D, 2.0), np.zeros(D)
    ch = O.Chain(D, mu0=mu0, kappa=k0, nu=nu0, Lambda=Psi, seed=9, kcap=8, prior="niw", param_update="niw_conjugate")
    Y = rng.normal(size=(n, D)) @ np.diag([1.0, 2.0, 0.5]) + 3.0
    anchor = np.array([2.5, 3.2, 2.9])
    d = Y - anchor
    st = np.concatenate([d.sum(0), [(d[:, a] * d[:, b]).sum() for a in range(D) for b in range(a, D)]])
    xb = Y.mean(0)
    kn, nun = k0 + n, nu0 + n
    mun = (k0 * mu0 + n * xb) / kn
    Psin = Psi + (Y - xb).T @ (Y - xb) + k0 * n / kn * np.outer(xb - mu0, xb - mu0)
    qm, qs = zip(*[ch.niw_draw(i, 78, 5, n, st, anchor) for i in range(4000)])
    qm, qs = np.array(qm), np.array(qs)
    EP = Psin / (nun - D - 1)
    assert np.abs(qs.mean(0) - EP).max() < 0.02 * np.abs(EP).max()
    assert np.all(np.abs(qm.mean(0) - mun) < 4.5 * np.sqrt(np.diag(EP) / kn / 4000))


def test_niw_conjugate_chain_recovers_mixture():
    rng = np.random.default_rng(3)
    D, K, N = 8, 6, 3000
    cent = rng.uniform(-10, 10, size=(K, D))
    lab = rng.integers(0, K, N)
    X = cent[lab] + rng.normal(size=(N, D))
    ch = O.Chain(D, mu0=np.zeros(D), kappa=0.01, nu=D + 2.0, Lambda=np.eye(D), seed=1, kcap=256, prior="niw",
                 param_update="niw_conjugate")
    ch.set_data(X)
    ch.init_random(20)
    ch.sweep(30)
    m = O.similarity(lab, ch.state()["z"])
    assert m["purity"] > 0.99 and m["adjusted_rand_index"] > 0.95


def test_invalid_combinations_rejected():
    with pytest.raises(ValueError):
        O.Chain(3, prior="niw", nu=3.5, Lambda=np.eye(3))  # nu0 < D + 1
    with pytest.raises(ValueError):
        O.Chain(3, prior="reference", param_update="niw_conjugate")
    with pytest.raises(ValueError):
        O.Chain(3, prior="niw", nu=6.0, Lambda=np.eye(3), param_update="mh_g0")
