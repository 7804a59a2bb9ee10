"""Pins the CPU oracle (oracle/np8_oracle.c) before it is trusted as the GPU's checker: every check
compares it with values produced by something else -- the reference's own KAT and its own
random_weighted_pick, numpy/LAPACK, sklearn, Random123 known answers, and distributional facts of
the base measure.  CPU only."""
import json
import math
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_philox_known_answers():
    for k in json.load(open(os.path.join(GOLD, "philox_kat.json"))):
        assert O.philox4x32_10(k["ctr"], k["key"]) == k["out"]


def test_reference_likelihood_kat():
    """test/test_mvn_likelihood.cpp:30-44 (the reference asserts are one-sided; we check both sides)."""
    p = O.mvn_probability_ref([1, 2], [1, 1], [[2, 0], [1, 2]])
    assert abs(p - 0.061974) < 1e-5
    assert abs(p * p - 0.0038409) < 1e-6
    # a Cholesky of the lower triangle would give 0.065841 and fail the KAT
    assert abs(p - 0.065841) > 1e-3
    lp = O.mvn_logprobability_ref([1, 2], [1, 1], [[2, 0], [1, 2]])
    assert abs(lp - math.log(p)) < 1e-14


def test_loglik_cases_vs_numpy():
    z = np.load(os.path.join(GOLD, "ll_cases.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in z.files if k.startswith("D")})
    assert len(keys) == 12
    for key in keys:
        X, mu, S, ll = z[key + "_X"], z[key + "_mu"], z[key + "_S"], z[key + "_ll"]
        got = np.array([O.mvn_logprobability_ref(x, mu, S) for x in X])
        np.testing.assert_allclose(got, ll, rtol=1e-11, atol=1e-10, err_msg=key)


def test_loglik_table_form_vs_numpy():
    """The chain's table form (packed symmetric precision + LU log-det) against numpy."""
    z = np.load(os.path.join(GOLD, "ll_cases.npz"))
    for D in (2, 3, 8, 16):
        for kind in ("spd", "iso", "nonsym"):
            key = f"D{D}_{kind}"
            X, mu, S, ll = z[key + "_X"], z[key + "_mu"], z[key + "_S"], z[key + "_ll"]
            c = O.Chain(D, seed=0, kcap=8)
            c.set_data(X)
            c.set_state(np.zeros(len(X), np.int32), mu[None], S[None])
            got = c.loglik_matrix(np.arange(len(X)))[:, 0]
            np.testing.assert_allclose(got, ll, rtol=1e-11, atol=1e-10, err_msg=key)


def test_weighted_pick_matches_reference_fixtures():
    """Indices produced by the reference's own dim1algebra.hpp (oracle/_ref), committed as fixtures."""
    cases = json.load(open(os.path.join(GOLD, "pick_ref.json")))
    assert len(cases) == 400
    for c in cases:
        assert O.weighted_pick_ref(np.array(c["w"]), c["u"]) == c["index"]


def test_weighted_pick_matches_live_reference_header():
    R = O.ref_harness()
    if R is None:
        pytest.skip("oracle/_ref not built (reference tree absent on this machine)")
    rng = np.random.default_rng(5)
    for _ in range(300):
        w = rng.exponential(size=int(rng.integers(1, 40)))
        u = float(np.floor(rng.random() * 2**53) / 2**53)
        assert O.weighted_pick_ref(w, u) == R.np8ref_weighted_pick(w.ctypes.data, w.size, u)


def test_metrics_vs_sklearn():
    for c in json.load(open(os.path.join(GOLD, "metrics.json"))):
        m = O.similarity(c["truth"], c["result"])
        assert abs(m["purity"] - c["purity"]) < 1e-12
        assert abs(m["rand_index"] - c["rand_index"]) < 1e-12
        if not math.isnan(m["adjusted_rand_index"]):
            assert abs(m["adjusted_rand_index"] - c["ari"]) < 1e-10


def test_metrics_no_int32_overflow():
    """the reference's int a,b,c overflow past a few hundred items; ours do not."""
    n = 200_000
    truth = np.repeat([0, 1], n // 2).astype(np.int32)
    m = O.similarity(truth, truth)
    assert m["purity"] == 1.0 and m["rand_index"] == 1.0 and abs(m["adjusted_rand_index"] - 1.0) < 1e-12


def test_lu_inverse_vs_numpy():
    import ctypes as C

    rng = np.random.default_rng(3)
    for D in (1, 2, 5, 8, 16):
        A = rng.normal(size=(D, D)) + D * np.eye(D)
        inv = np.zeros((D, D))
        det = C.c_double(0)
        O.lib().np8o_lu_inverse_det(A.ctypes.data, D, inv.ctypes.data, C.byref(det))
        np.testing.assert_allclose(inv, np.linalg.inv(A), rtol=1e-11, atol=1e-12)
        assert abs(det.value - np.linalg.det(A)) < 1e-9 * abs(np.linalg.det(A))


def test_spec_math_accuracy():
    """exp_le0 / log_pos / sincos_2pi (DESIGN.md "Math") against numpy over their domains."""
    import ctypes as C

    L = O.lib()
    L.np8o_exp_le0.argtypes = [C.c_double]
    L.np8o_exp_le0.restype = C.c_double
    L.np8o_log_pos.argtypes = [C.c_double]
    L.np8o_log_pos.restype = C.c_double
    L.np8o_sincos_2pi.argtypes = [C.c_double, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(11)
    xs = -rng.random(20000) * 740.0
    ex = np.array([L.np8o_exp_le0(float(x)) for x in xs])
    np.testing.assert_allclose(ex, np.exp(xs), rtol=4e-16 * 4, atol=0)
    assert L.np8o_exp_le0(float("-inf")) == 0.0 and L.np8o_exp_le0(0.0) == 1.0
    us = (np.floor(rng.random(20000) * 2**53) + 1) * 2.0**-53
    lg = np.array([L.np8o_log_pos(float(u)) for u in us])
    np.testing.assert_allclose(lg, np.log(us), rtol=5e-16, atol=0)
    sn, cs = C.c_double(), C.c_double()
    err = 0.0
    for t in us[:5000]:
        L.np8o_sincos_2pi(float(t), C.byref(sn), C.byref(cs))
        err = max(err, abs(sn.value - np.sin(2 * np.pi * t)), abs(cs.value - np.cos(2 * np.pi * t)))
    assert err < 1e-15


def test_uniforms_open_interval_and_normals_moments():
    us = np.array([O.uniform(1, i, 0, 2, 0) for i in range(20000)])
    assert us.min() > 0.0 and us.max() < 1.0
    assert abs(us.mean() - 0.5) < 0.01
    g = np.array([O.normal(3, i, 5, 1, n) for i in range(5000) for n in range(4)])
    assert abs(g.mean()) < 0.03 and abs(g.std() - 1.0) < 0.03
    # Gaussian tails: kurtosis 3
    assert abs(np.mean(g**4) / np.mean(g**2) ** 2 - 3.0) < 0.15


def test_base_measure_moments():
    """G0 (normalinvwishart.h:44-64, invwishart.h:30-43): v ~ N(D, nu^2), Sigma = v^2 L^T L,
    mu - mu0 ~ N(0, Sigma/kappa)."""
    D, nu, kappa = 2, 4.0, 1.0 / 500
    c = O.Chain(D, seed=42, nu=nu, kappa=kappa, kcap=8)
    c.set_data(np.zeros((20000, D)))
    c.set_state(np.zeros(20000, np.int32), np.zeros((1, D)), np.eye(D)[None])
    v2, std = [], []
    for i in range(20000):
        mu, S = c.aux_params(i)
        for m in range(3):
            vv = S[m, 0, 0] / 0.01
            v2.append(vv)
            assert abs(S[m, 0, 1]) < 1e-300 and abs(S[m, 1, 1] - S[m, 0, 0]) < 1e-15 * S[m, 0, 0]
            std.append((mu[m] - 6.0) / np.sqrt(S[m, 0, 0] / kappa))
    v2 = np.array(v2)
    std = np.concatenate(std)
    assert abs(v2.mean() - (D * D + nu * nu)) < 0.03 * (D * D + nu * nu)  # E[v^2] = D^2 + nu^2
    assert abs(std.mean()) < 0.01 and abs(std.std() - 1.0) < 0.01


def test_scan_order_is_a_permutation():
    for N in (1, 2, 3, 17, 200, 1000, 4097):
        p = [O.perm(9, 3, N, i) for i in range(N)]
        assert sorted(p) == list(range(N))
    a = [O.perm(9, 3, 200, i) for i in range(200)]
    b = [O.perm(9, 4, 200, i) for i in range(200)]
    assert a != b  # fresh order every sweep (np_mcmc.cpp:120-125)


def test_twogaussians_fixture_matches_recipe():
    from noparama_amd import datasets

    X, lab = datasets.read_data(os.path.join(GOLD, "twogaussians.data"))
    assert X.shape == (200, 2) and np.array_equal(np.bincount(lab), [100, 100])
    assert np.allclose(X[:100].mean(0), 0.0, atol=0.35) and np.allclose(X[100:].mean(0), 5.0, atol=0.35)
    X2, lab2 = datasets.twogaussians()
    np.testing.assert_allclose(X, X2, rtol=0, atol=1e-15)


def test_parallel_sync_step_is_deterministic():
    """The cpu_par baseline (OpenMP over the items of a synchronous step) equals the 1-thread run."""
    from noparama_amd import datasets

    X, z, mu, sig = datasets.mixture(3000, 3, 8, 0.5, 6.0, seed=3)
    out = []
    for threads in (1, 4):
        O.set_threads(threads)
        c = O.Chain(3, seed=8, kcap=1024)
        c.set_data(X)
        c.init_random(20)
        c.sweep(3)
        out.append(c.state())
    O.set_threads(1)
    assert out[0]["K"] == out[1]["K"] and np.array_equal(out[0]["z"], out[1]["z"])
    np.testing.assert_array_equal(out[0]["mu"], out[1]["mu"])
