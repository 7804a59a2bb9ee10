"""The cluster-parameter update (mh_g0) of the oracle, pinned against a direct restatement of the
reference's UpdateClusters::update (src/np_update_clusters.cpp:71-142): likelihoods summed item by
item with numpy (multivariatenormal.cpp:138-146 -> scipy-free logpdf), proposals drawn from G0 with
the same Philox streams, acceptance u < exp(LL' - LL).  CPU only."""
import numpy as np
import pytest

import oracle as O

STREAM_PARAM, STREAM_PARAM_U = 5, 6


def _logpdf_sum(X, mu, S):
    D = X.shape[1]
    d = X - mu
    sign, logdet = np.linalg.slogdet(S)
    assert sign > 0
    q = np.einsum("ia,ab,ib->i", d, np.linalg.inv(S), d)
    return float(np.sum(-0.5 * q - 0.5 * (D * np.log(2 * np.pi) + logdet)))


def _proposal(seed, slot, t, step, D, mu0, kappa, nu, Lam):
    Q = (D + 4) // 4  # Philox calls per G0 draw (normal_quad)
    g = [O.normal(seed, slot, t, STREAM_PARAM, 4 * step * Q + k) for k in range(D + 1)]
    v = D + nu * g[0]
    L = np.linalg.cholesky(Lam)
    mu = mu0 + abs(v) / np.sqrt(kappa) * (L.T @ np.array(g[1:]))
    return mu, v * v * (L.T @ L)


def _problem(seed=5, D=2, K=3, n=60):
    rng = np.random.default_rng(seed)
    centers = 6.0 + rng.uniform(-3, 3, size=(K, D))
    z = np.repeat(np.arange(K), n).astype(np.int32)
    X = centers[z] + 0.3 * rng.standard_normal((K * n, D))
    # poor starting parameters: shifted means, wide covariances
    mu = centers + 1.0
    sig = np.stack([4.0 * np.eye(D)] * K)
    return X, z, mu, sig


def test_suffstats_about_slot_means():
    X, z, mu, sig = _problem(D=3, K=4, n=50)
    c = O.Chain(3, seed=1, kcap=16)
    c.set_data(X)
    c.set_state(z, mu, sig)
    st = c.suffstats()
    iu = np.triu_indices(3)
    for k in range(4):
        d = X[z == k] - mu[k]
        np.testing.assert_allclose(st[k, :3], d.sum(0), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(st[k, 3:], (d.T @ d)[iu], rtol=1e-12, atol=1e-12)
    assert np.all(st[4:] == 0)


@pytest.mark.parametrize("D,steps,n", [(2, 300, 60), (3, 3000, 5)])
def test_mh_g0_matches_direct_restatement(D, steps, n):
    seed = 12
    X, z, mu, sig = _problem(seed=D, D=D, n=n)
    mu0, kappa, nu, Lam = np.full(D, 6.0), 1.0 / 500, 4.0, 0.01 * np.eye(D)
    c = O.Chain(D, seed=seed, kcap=8, param_update="mh_g0", mh_steps=steps)
    c.set_data(X)
    c.set_state(z, mu, sig)
    acc = c.param_update(c.suffstats())
    got = c.state()
    # direct restatement, cluster by cluster (clusters are independent; the epoch is 0)
    n_acc = 0
    for k in range(mu.shape[0]):
        Xk = X[z == k]
        cur_mu, cur_S = mu[k], sig[k]
        LL = _logpdf_sum(Xk, cur_mu, cur_S)
        for s in range(steps):
            pm, pS = _proposal(seed, k, 0, s, D, mu0, kappa, nu, Lam)
            LLp = _logpdf_sum(Xk, pm, pS)
            u = O.uniform(seed, k, 0, STREAM_PARAM_U, s)
            if LL == 0.0 or u < np.exp(LLp - LL):
                cur_mu, cur_S, LL = pm, pS, LLp
                n_acc += 1
        np.testing.assert_allclose(got["mu"][k], cur_mu, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(got["sigma"][k], cur_S, rtol=1e-12, atol=1e-14)
    assert acc == n_acc and acc > 0


def test_mh_g0_chain_improves_the_fit():
    X, z, mu, sig = _problem(seed=3)
    c = O.Chain(2, seed=4, kcap=64, param_update="mh_g0")
    c.set_data(X)
    c.set_state(z, mu, sig)
    L0 = c.total_loglik()
    c.sweep(30)
    assert c.mh_accepted > 0
    assert c.total_loglik() > L0 + 100.0
    # frozen parameters stay put (the reference's effective behaviour)
    f = O.Chain(2, seed=4, kcap=64)
    f.set_data(X)
    f.set_state(z, mu, sig)
    f.sweep(3)
    assert f.mh_accepted == 0
    np.testing.assert_array_equal(f.state()["mu"][:3], mu)
