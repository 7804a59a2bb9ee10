"""The plug-in keeps the caller's membertrix coherent (VERDICT r01 "boundary"): the reference's MCMC::run loop
(src/np_mcmc.cpp:109-175) driven from the host exactly as the reference structures it --

    for t in 0..T-1:
        if t % 10 == 0: membertrix.relabel()                      (:111-114)
        update_cluster_population.update(membertrix, ids)         (:146-164)
        update_clusters.update(membertrix)                        (:170)
        if t % 5 == 0: considerMaxLikelihood()  on the membertrix (:172-174, 187-203)

-- with NealAlgorithm8.update patching the membertrix in place from the device's change log (np8_changes:
moved items, created / removed / updated clusters) and the cluster-parameter update ending the sweep on the
device (np8_end_sweep) and patched in the same way.  After every update the membertrix must equal
np8_get_state (labels up to the naming of clusters, counts, mu, Sigma bit for bit); the host-side
considerMaxLikelihood over the membertrix must agree with the device's total log-likelihood, and its
best labelling with the device's snapshot (np8_get_state(which = 1))."""
import os

import numpy as np
import pytest

from noparama_amd import NealAlgorithm8, datasets, membertrix

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def mvn_logpdf(X, mu, S):
    """log N(x | mu, S) per row (S as the reference uses it: inverse and determinant of S as given)."""
    D = X.shape[1]
    Si = np.linalg.inv(S)
    d = X - mu
    q = np.einsum("na,ab,nb->n", d, Si, d)
    return -0.5 * (D * np.log(2 * np.pi) + np.log(np.linalg.det(S)) + q)


def consider_max_likelihood(trix, X):
    """MCMC::considerMaxLikelihood (np_mcmc.cpp:187-203) on the host membertrix."""
    tot = 0.0
    for cid, (mu, S) in trix.getClusters().items():
        tot += mvn_logpdf(X[trix.z == cid], mu, S).sum()
    return tot


def canonical(z, cnt, mu, sg):
    """Clusters renamed in order of their first item (cluster ids are names: the membertrix numbers them by
    creation and relabel(), the device by slot)."""
    labs, first = np.unique(z, return_index=True)
    perm = labs[np.argsort(first)]
    lut = np.empty(int(z.max()) + 1, dtype=np.int64)
    lut[perm] = np.arange(perm.size)
    return lut[z], np.asarray(cnt)[perm], np.asarray(mu)[perm], np.asarray(sg)[perm]


def assert_coherent(trix, smp):
    st = smp.state()
    z, cnt, mu, sg = canonical(*trix.dense())
    zd, cntd, mud, sgd = canonical(st["z"], st["counts"], st["mu"], st["sigma"])
    assert st["K"] == cnt.size
    assert np.array_equal(z, zd), "labels differ"
    assert np.array_equal(cnt, cntd)
    assert np.array_equal(mu, mud) and np.array_equal(sg, sgd), "parameters differ"


@pytest.mark.parametrize("chunk,param_update", [(0, "frozen"), (0, "mh_g0"), (7, "frozen"), (1, "mh_g0")])
def test_reference_mcmc_loop_keeps_membertrix_coherent(chunk, param_update):
    X, _ = datasets.read_data(os.path.join(HERE, "golden", "twogaussians.data"))
    N, T = X.shape[0], 30
    smp = NealAlgorithm8(2, seed=17, chunk=chunk, kcap=256, device=0, param_update=param_update)
    try:
        smp.set_data(X)
        smp.init_random(20)
        trix = membertrix(N)
        best, best_z = -np.inf, None
        rng = np.random.default_rng(3)
        for t in range(T):
            if t % 10 == 0:
                trix.relabel()
            smp.update(trix, rng.permutation(N))  # population update + patch
            assert_coherent(trix, smp)
            smp.end_sweep()  # UpdateClusters::update (np_mcmc.cpp:170) on the device, then patched
            smp.patch(trix)
            assert_coherent(trix, smp)
            if t % 5 == 0:
                L = consider_max_likelihood(trix, X)
                assert abs(L - smp.stats()["last_loglik"]) <= 1e-9 * abs(L), (L, smp.stats()["last_loglik"])
                if L > best:
                    best, best_z = L, trix.dense()[0]
        snap = smp.state(which=1, params=False)
        assert np.array_equal(canonical(snap["z"], snap["counts"], snap["counts"], snap["counts"])[0],
                              canonical(best_z, best_z, best_z, best_z)[0])
        assert abs(smp.stats()["best_loglik"] - best) <= 1e-9 * abs(best)
    finally:
        smp.close()


def test_single_item_updates_patch_membertrix():
    """The reference's per-item call (data_ids of size 1, np_mcmc.cpp:161): each update patches the
    membertrix with that item's move and the cluster it created or emptied."""
    X, _ = datasets.read_data(os.path.join(HERE, "golden", "twogaussians.data"))
    smp = NealAlgorithm8(2, seed=23, kcap=256, device=0)
    try:
        smp.set_data(X)
        smp.init_random(20)
        trix = membertrix(X.shape[0])
        smp.patch(trix)
        for i in np.random.default_rng(9).permutation(X.shape[0])[:60]:
            smp.update(trix, [int(i)])
            assert_coherent(trix, smp)
    finally:
        smp.close()


def test_patch_after_new_data_reloads_membertrix():
    """np8_set_data drops the device change log; the next update() must reload the whole state
    into the membertrix (first contact) instead of failing on change tracking being off."""
    X, _ = datasets.read_data(os.path.join(HERE, "golden", "twogaussians.data"))
    smp = NealAlgorithm8(2, seed=31, kcap=256, device=0)
    try:
        smp.set_data(X)
        smp.init_random(20)
        trix = membertrix(X.shape[0])
        smp.update(trix, np.arange(X.shape[0]))
        assert_coherent(trix, smp)
        smp.set_data(X[::-1].copy())  # new items
        smp.init_random(10)
        smp.update(trix, np.arange(X.shape[0]))
        assert_coherent(trix, smp)
    finally:
        smp.close()
