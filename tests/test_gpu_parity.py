"""GPU parity: the HIP path (libnp8.so via the C ABI) against the CPU oracle on identical inputs.

Integer outputs (labels, cluster counts, K) must be bit-exact; log-likelihoods within 1e-12
relative (fp64, DESIGN.md "Tolerances").  Mirrors the reference's own checks where they exist:
test/test_mvn_likelihood.cpp (KAT) and test/test_membertrix.cpp (auto-remove of emptied clusters).
"""
import numpy as np
import pytest

import oracle as O
from noparama_amd import NP8Error, NealAlgorithm8, datasets

pytestmark = pytest.mark.gpu

LL_RTOL = 1e-12


def pair(D, seed, chunk=0, kcap=2048, **kw):
    return (NealAlgorithm8(D, seed=seed, chunk=chunk, kcap=kcap, device=0, **kw),
            O.Chain(D, seed=seed, chunk=chunk, kcap=kcap, **kw))


def assert_same_state(a, b, which=0):
    sa, sb = a.state(which), b.state(which)
    assert sa["K"] == sb["K"]
    assert np.array_equal(sa["z"], sb["z"])
    assert np.array_equal(sa["counts"], sb["counts"])
    np.testing.assert_allclose(sa["mu"], sb["mu"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(sa["sigma"], sb["sigma"], rtol=1e-13, atol=1e-15)


def test_kat_likelihood_through_abi():
    """test/test_mvn_likelihood.cpp:18-33: mu=(1,1), Sigma=[[2,0],[1,2]] (non-symmetric), x=(1,2)."""
    g = NealAlgorithm8(2, seed=0, device=0)
    g.set_data(np.array([[1.0, 2.0], [1.0, 2.0]]))
    g.set_state(np.zeros(2, np.int32), np.array([[1.0, 1.0]]), np.array([[[2.0, 0.0], [1.0, 2.0]]]))
    ll = g.loglik_matrix(np.array([0, 1]))[:, 0]
    p = np.exp(ll)
    assert abs(p[0] - 0.061974) < 1e-5
    assert abs(p[0] * p[1] - 0.0038409) < 1e-6  # probability(dataset) = product (:41-44)
    np.testing.assert_allclose(ll[0], np.log(O.mvn_probability_ref([1, 2], [1, 1], [[2, 0], [1, 2]])),
                               rtol=1e-14)


@pytest.mark.parametrize("sweeps", [1, 4])
def test_twogaussians_sync_bit_exact(sweeps):
    X, _ = datasets.twogaussians()
    g, o = pair(2, 11)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    assert_same_state(g, o)
    g.sweep(sweeps)
    o.sweep(sweeps)
    assert_same_state(g, o)


@pytest.mark.parametrize("chunk", [1, 7, 64])
def test_chunked_sweeps_bit_exact(chunk):
    """chunk = 1 is the reference's sequential sweep (np_mcmc.cpp:146-164)."""
    X, _ = datasets.twogaussians(3)
    g, o = pair(2, 5, chunk=chunk)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    g.sweep(3)
    o.sweep(3)
    assert_same_state(g, o)


def test_update_points_explicit_order():
    X, _ = datasets.twogaussians(4)
    g, o = pair(2, 9)
    order = np.random.default_rng(1).permutation(200)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
        s.update_points(order)
        s.end_sweep()
        s.update_points(order[::-1].copy())
    assert_same_state(g, o)


def test_loglik_matrix_vs_oracle_and_reference_formula():
    X, _, mu, sig = datasets.mixture(3000, 8, 16, 0.8, 20.0, seed=3)
    g, o = pair(8, 21)
    z = np.random.default_rng(0).integers(0, 16, size=3000).astype(np.int32)
    for s in (g, o):
        s.set_data(X)
        s.set_state(z, mu, sig)
    idx = np.arange(0, 3000, 7)
    a = g.loglik_matrix(idx)
    b = o.loglik_matrix(idx)
    ref = o.loglik_matrix(idx, ref=True)  # multivariatenormal.cpp:124-135 with LU inverse per call
    np.testing.assert_allclose(a, b, rtol=LL_RTOL, atol=1e-12)
    np.testing.assert_allclose(a, ref, rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("D,K,s,r", [(2, 10, 0.3, 15.0), (8, 64, 0.8, 20.0), (3, 5, 0.5, 5.0), (16, 8, 1.0, 10.0)])
def test_warm_state_sweeps_bit_exact(D, K, s, r):
    X, z, mu, sig = datasets.mixture(20000, D, K, s, r, seed=D)
    g, o = pair(D, 100 + D)
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, mu, sig)
    g.sweep(3)
    o.sweep(3)
    assert_same_state(g, o)
    np.testing.assert_allclose(g.total_loglik(), o.total_loglik(), rtol=1e-11)


def test_sorted_layout_many_resorts_bit_exact():
    """Synchronous sweeps run on a label-sorted copy of the data, re-sorted every few sweeps; from a
    random start items move a lot, so the layout is stale most of the time.  Results must not care."""
    X, _, _, _ = datasets.mixture(6000, 3, 12, 0.5, 5.0, seed=12)
    g, o = pair(3, 41, kcap=4096)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    for _ in range(4):
        g.sweep(3)
        o.sweep(3)
        assert_same_state(g, o)
    # a per-item step in between invalidates the sorted copy
    g.update_points(np.arange(0, 6000, 13))
    o.update_points(np.arange(0, 6000, 13))
    g.sweep(2)
    o.sweep(2)
    assert_same_state(g, o)


def test_max_likelihood_snapshot():
    X, _ = datasets.twogaussians(8)
    g, o = pair(2, 13)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    g.sweep(16)
    o.sweep(16)
    assert_same_state(g, o, which=1)
    np.testing.assert_allclose(g.stats()["best_loglik"], o.best_loglik(), rtol=1e-12)


def test_singleton_cluster_auto_removed():
    """test/test_membertrix.cpp:16-93 analogue: emptied clusters disappear from the live table."""
    X = np.array([[0.0, 0.0], [0.1, 0.0], [50.0, 50.0]])
    g, o = pair(2, 1)
    mu = np.array([[0.0, 0.0], [50.0, 50.0], [-30.0, 8.0]])
    sig = np.stack([np.eye(2) * 0.5] * 3)
    z = np.array([0, 2, 1], np.int32)  # item 1 alone in a far cluster
    for s in (g, o):
        s.set_data(X)
        s.set_state(z, mu, sig)
        s.sweep(1)
    assert_same_state(g, o)
    assert g.state()["K"] <= 3


def test_errors_are_reported():
    g = NealAlgorithm8(2, seed=0, device=0)
    with pytest.raises(NP8Error):
        g.sweep(1)  # no data / state
    g.set_data(np.zeros((4, 2)))
    with pytest.raises(NP8Error):
        g.set_state(np.array([0, 0, 0, 5], np.int32), np.zeros((1, 2)), np.eye(2)[None])
    with pytest.raises(NP8Error):
        g.set_state(np.zeros(4, np.int32), np.zeros((1, 2)), np.zeros((1, 2, 2)))  # det = 0
    NealAlgorithm8(17, seed=0, device=0).close()  # fp64 above D = 16: the run-time-D kernels (np8_rt.hip)
    with pytest.raises(NP8Error):
        NealAlgorithm8(129, seed=0, device=0)  # at most kMaxD = 128
    with pytest.raises(NP8Error):  # the run-time-D path: reference prior, frozen parameters
        NealAlgorithm8(17, seed=0, device=0, prior="niw", nu=20.0)
    with pytest.raises(NP8Error):
        NealAlgorithm8(5, M=2, seed=0, device=0)  # D <= 8 outside {1, 2, 3, 4, 8} runs M = 3 (the reference's)


def test_partial_accept_at_kcap_matches_oracle():
    """More new-cluster requests than free slots (a huge alpha makes most items ask for a new
    cluster): the requests of lowest scan position fill the free slots, the rest are deferred."""
    X, _ = datasets.twogaussians(5)
    g, o = pair(2, 17, kcap=24, alpha=1e6)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    g.sweep(2)
    assert o.sweep(2) == 0
    assert_same_state(g, o)
    st = g.stats()
    assert st["rejected_requests"] > 0
    assert [st["new_clusters"], st["rejected_requests"]] == list(o.request_stats)


@pytest.mark.parametrize("D,N,req_max", [(2, 100_000, 0), (8, 100_000, 0), (8, 100_000, 300)])
def test_cold_start_from_init_random_bit_exact(D, N, req_max):
    """the reference's initialisation (np_mcmc.cpp:49-92, K=20 random G0 clusters) at
    N = 1e5 sends thousands of new-cluster requests in the first sweep; round 1 rejected them all
    (K stuck at 20).  Now: partial acceptance in scan order, bit-exact against the oracle."""
    X = (datasets.config_c2(N=N) if D == 2 else datasets.config_c3(N=N))[0]
    O.set_threads(8)
    g, o = pair(D, 23, req_max=req_max)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    for t in range(3):
        g.sweep(1)
        assert o.sweep(1) == 0
        sg, so = g.state(params=False), o.state()
        assert sg["K"] == so["K"], (t, sg["K"], so["K"])
        assert np.array_equal(sg["z"], so["z"]), t
        assert np.array_equal(sg["counts"], so["counts"])
    st = g.stats()
    assert [st["new_clusters"], st["rejected_requests"]] == list(o.request_stats)
    assert st["rejected_requests"] > 0 and g.K > 20
    assert_same_state(g, o)


def test_update_points_repeated_visits_bit_exact():
    """repeated np8_update_points without np8_end_sweep draws afresh at every visit (item key
    index | visit << 32), identically on the device and in the oracle, and does not cycle."""
    X, _ = datasets.twogaussians()
    g, o = pair(2, 29, kcap=256)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    ids = np.arange(X.shape[0], dtype=np.int64)
    seen = set()
    for k in range(6):
        sub = ids if k % 2 == 0 else ids[::-3]
        g.update_points(sub)
        o.update_points(sub)
        assert_same_state(g, o)
        seen.add(g.state()["z"].tobytes())
    assert len(seen) >= 4  # the chain moves (a deterministic 2-cycle would give at most 2)


@pytest.mark.parametrize("req_max", [0, 40])
def test_host_exchange_two_ranks_equals_one(req_max):
    """The multi-GPU protocol (exchange record, rank-ordered requests) with two contexts on one GPU
    and a host all-gather: identical to the single-rank sweep.  req_max = 40: most requests of the
    first sweeps are deferred, and each rank's record carries only its 40 lowest-position requests
    (np8_req_select)."""
    X, _, mu, sig = datasets.mixture(5000, 8, 12, 0.8, 6.0, seed=9)
    z = np.random.default_rng(2).integers(0, 12, size=5000).astype(np.int32)
    one = NealAlgorithm8(8, seed=77, device=0, req_max=req_max)
    one.set_data(X)
    one.init_random(12)
    one.sweep(3)
    if req_max:
        assert one.stats()["rejected_requests"] > 0
    half = 2600
    ranks = [NealAlgorithm8(8, seed=77, device=0, req_max=req_max) for _ in range(2)]
    for r, c in enumerate(ranks):
        c.comm_init(None, r, 2)
        lo, hi = (0, half) if r == 0 else (half, 5000)
        c.set_data(X[lo:hi], offset=lo, n_global=5000)
        c.init_random(12)
    for _ in range(3):
        recs = np.concatenate([c.step_local() for c in ranks])
        for c in ranks:
            c.step_merge(recs, 2)
            c.end_sweep()
    s1 = one.state()
    z2 = np.concatenate([c.state()["z"] for c in ranks])
    assert np.array_equal(s1["z"], z2)
    for c in ranks:
        st = c.state()
        assert st["K"] == s1["K"]
        assert np.array_equal(st["counts"], s1["counts"])
    del z, mu, sig


@pytest.mark.parametrize("param_update", ["frozen", "mh_g0"])
def test_host_exchange_substeps_equals_oracle(param_update):
    """the host-exchange transport (MPI/gloo) with S = 4 sub-steps runs S record exchanges
    (np8_step_local / np8_step_merge) per sweep and then ends the sweep; ending it earlier is an error.
    Two ranks on one GPU against the oracle's single chain, bit-exact."""
    X, _, mu, sig = datasets.mixture(6000, 8, 12, 0.8, 6.0, seed=19)
    N, S = X.shape[0], 4
    o = O.Chain(8, seed=55, kcap=512, substeps=S, param_update=param_update)
    o.set_data(X)
    o.init_random(12)
    o.sweep(3)
    ranks = [NealAlgorithm8(8, seed=55, kcap=512, device=0, substeps=S, param_update=param_update)
             for _ in range(2)]
    bounds = [(0, 2900), (2900, N)]
    for r, c in enumerate(ranks):
        c.comm_init(None, r, 2)
        c.set_data(X[bounds[r][0]:bounds[r][1]], offset=bounds[r][0], n_global=N)
        c.init_random(12)
    for sweep in range(3):
        for s in range(S):
            recs = np.concatenate([c.step_local() for c in ranks])
            for c in ranks:
                c.step_merge(recs, 2)
            if sweep == 0 and s == 0:
                with pytest.raises(NP8Error):
                    ranks[0].end_sweep()  # three sub-steps still to go
        if param_update == "frozen":
            for c in ranks:
                c.end_sweep()
        else:
            st = sum(c.param_stats_local() for c in ranks)
            for c in ranks:
                c.end_sweep_stats(st)
    so = o.state()
    z2 = np.concatenate([c.state()["z"] for c in ranks])
    assert np.array_equal(so["z"], z2)
    for c in ranks:
        st = c.state()
        assert st["K"] == so["K"] and np.array_equal(st["counts"], so["counts"])
        np.testing.assert_allclose(st["mu"], so["mu"], rtol=1e-13, atol=1e-13)
    for c in ranks:
        c.close()


# ---- cluster-parameter update (mh_g0, UpdateClusters as intended) ------------------------------------
# The statistics are fp64 sums whose order differs between the device (wave reduction + atomics) and
# the oracle (item order); decisions u < exp(LL' - LL) can only differ when the two sides fall within
# ~1e-12 of each other, so the chains are compared bit-for-bit.
def _mh_pair(D, seed, **kw):
    return pair(D, seed, param_update="mh_g0", **kw)


@pytest.mark.parametrize("chunk", [0, 16])
def test_mh_g0_twogaussians_bit_exact(chunk):
    X, _ = datasets.twogaussians(6)
    g, o = _mh_pair(2, 21, chunk=chunk)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    for _ in range(3):
        g.sweep(2)
        o.sweep(2)
        assert_same_state(g, o)
    assert g.stats()["mh_accepted"] == o.mh_accepted > 0


@pytest.mark.parametrize("D,K", [(2, 6), (8, 16), (16, 4)])
def test_mh_g0_warm_bit_exact(D, K):
    """Poor starting parameters (wide covariances) so that proposals are accepted."""
    X, z, mu, sig = datasets.mixture(20000, D, K, 0.3, 4.0, seed=D)
    sig = sig * 9.0
    g, o = _mh_pair(D, 300 + D, mh_steps=40)
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, mu, sig)
    for _ in range(2):
        g.sweep(2)
        o.sweep(2)
        assert_same_state(g, o)
    assert g.stats()["mh_accepted"] == o.mh_accepted
    np.testing.assert_allclose(g.total_loglik(), o.total_loglik(), rtol=1e-11)


def test_sweep_graph_replay_bit_exact():
    """Runs of >= 20 synchronous sweeps are replayed from a captured hipGraph (epoch, re-sort and
    max-likelihood cadence read on the device); results must equal the oracle's sweep by sweep."""
    X, z, mu, sig = datasets.mixture(6000, 3, 10, 0.5, 6.0, seed=4)
    g, o = pair(3, 77, kcap=4096)
    for c in (g, o):
        c.set_data(X)
        c.init_random(20)
    for n in (3, 20, 41, 7, 20):  # eager, graph at any phase, graph+eager, re-capture at a new phase
        g.sweep(n)
        o.sweep(n)
        assert_same_state(g, o)
        assert_same_state(g, o, which=1)
    assert g.stats()["epoch"] == o.epoch
    # a new state resets the device epoch; the cached graph must follow
    for c in (g, o):
        c.set_state(z, mu, sig)
    g.sweep(25)
    o.sweep(25)
    assert_same_state(g, o)
    np.testing.assert_allclose(g.stats()["best_loglik"], o.best_loglik(), rtol=1e-11)


def test_sweep_graph_mh_g0_bit_exact():
    X, z, mu, sig = datasets.mixture(20000, 2, 6, 0.3, 4.0, seed=9)
    g, o = _mh_pair(2, 55)
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, mu, sig * 9.0)
    g.sweep(45)
    o.sweep(45)
    assert_same_state(g, o)
    assert g.stats()["mh_accepted"] == o.mh_accepted


@pytest.mark.parametrize("S", [2, 8])
def test_substeps_twogaussians_bit_exact(S):
    """The data-parallel sweep in S synchronous sub-steps (np8_config.substeps, DESIGN.md "Sub-steps"):
    sub-step s = the items with substep_of(seed, i, S) == s, a contiguous range of the layout sorted by
    (sub-step, slot).  From the reference's init, eager sweeps then a graph replay, bit-exact."""
    X, _ = datasets.twogaussians()
    g, o = pair(2, 31, kcap=512, substeps=S)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    for n in (3, 20, 5):
        g.sweep(n)
        o.sweep(n)
        assert_same_state(g, o)
        assert_same_state(g, o, which=1)


def test_substeps_auto_resolves_by_data_size():
    """substeps = "auto" (NP8_SUBSTEPS_AUTO, include/np8.h): 16 sub-steps on twogaussians (N = 200, where one step
    over-splits), the same chain as an explicit 16 and as the oracle's; one step above 8192 items."""
    X, _ = datasets.twogaussians()
    g, o = pair(2, 33, kcap=512, substeps=16)
    from noparama_amd import NealAlgorithm8

    a = NealAlgorithm8(2, seed=33, kcap=512, device=0, substeps="auto")
    try:
        for s in (g, o, a):
            s.set_data(X)
            s.init_random(20)
        assert a.substeps == 16 and a.stats()["substeps"] == 16
        for s in (g, o, a):
            s.sweep(12)
        assert_same_state(g, o)
        assert np.array_equal(a.state()["z"], g.state()["z"])
        a.set_data(datasets.mixture(8193, 2, 4, 0.5, 8.0, seed=1)[0])
        assert a.substeps == 1 and a.stats()["substeps"] == 1
    finally:
        a.close()


@pytest.mark.parametrize("S,param_update", [(4, "frozen"), (8, "frozen"), (8, "mh_g0")])
def test_substeps_warm_c3_shape_bit_exact(S, param_update):
    """C3's shape (D = 8, K = 64) from the warm state with candidate pruning across sub-steps (lists
    rebuilt after every sub-step from the last sweep's radii) and the 20-sweep graph."""
    X, z, mu, sig = datasets.mixture(20000, 8, 64, 0.8, 20.0, seed=8)
    g, o = pair(8, 108, substeps=S, param_update=param_update)
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, mu, sig if param_update == "frozen" else sig * 4.0)
    for n in (2, 21):
        g.sweep(n)
        o.sweep(n)
        assert_same_state(g, o)
    np.testing.assert_allclose(g.total_loglik(), o.total_loglik(), rtol=1e-11)


def test_substeps_cold_start_bit_exact():
    X = datasets.config_c3(N=100_000)[0]
    O.set_threads(8)
    g, o = pair(8, 29, substeps=8)
    for s in (g, o):
        s.set_data(X)
        s.init_random(20)
    for _ in range(3):
        g.sweep(1)
        o.sweep(1)
        sg, so = g.state(params=False), o.state()
        assert sg["K"] == so["K"] and np.array_equal(sg["z"], so["z"])
    assert [g.stats()["new_clusters"], g.stats()["rejected_requests"]] == list(o.request_stats)


@pytest.mark.parametrize("D", [5, 6, 7, 9, 12, 15])
def test_every_dimension_up_to_16_bit_exact(D):
    """Any D from 1 to 16 on the fp64 path (the reference's data_t has any length, np_data.h:9): warm and
    random starts, mh_g0 and a split-merge sweep, bit-exact against the oracle."""
    X, z, mu, sig = datasets.mixture(6000, D, 6, 0.6, 6.0, seed=D)
    g, o = pair(D, 300 + D, kcap=512)
    for c in (g, o):
        c.set_data(X)
        c.set_state(z, mu, sig)
    g.sweep(3)
    o.sweep(3)
    assert_same_state(g, o)
    for c in (g, o):
        c.init_random(20)
    g.sweep(22)
    o.sweep(22)
    assert_same_state(g, o)
    np.testing.assert_allclose(g.loglik_matrix(np.arange(32)), o.loglik_matrix(np.arange(32)), rtol=LL_RTOL,
                               atol=1e-12)
    gm, om = pair(D, 400 + D, kcap=512, param_update="mh_g0")
    for c in (gm, om):
        c.set_data(X)
        c.set_state(z, mu, sig * 2.0)
    gm.sweep(4)
    om.sweep(4)
    assert_same_state(gm, om)
