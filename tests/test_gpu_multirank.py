"""Multi-rank protocol on one GPU (two contexts, host all-gather / all-reduce; DESIGN.md "Multi-GPU"):
the NIW prior, the niw_conjugate update and the wide path sharded over two ranks must reproduce the
single-rank sweep.  Labels, counts and K are compared exactly; with a parameter update the per-cluster
statistics are summed in another order (two partial sums), so parameters agree to ~1e-13 relative.
The RCCL transport runs the same records (tests/test_gpu_rccl.py; the driver's 8-GPU runs)."""
import numpy as np
import pytest

from noparama_amd import NealAlgorithm8

pytestmark = pytest.mark.gpu


def mixture(D, N, K, seed):
    rng = np.random.default_rng(seed)
    cent = rng.uniform(-5, 5, size=(K, D))
    z = rng.integers(0, K, N)
    return cent[z] + rng.normal(size=(N, D)), z.astype(np.int32), cent


def niw(D, seed):
    return dict(mu0=np.zeros(D), kappa=0.05, nu=D + 2.0, Lambda=0.5 * np.eye(D), seed=seed, prior="niw")


def run_sharded(make, X, z, mu, sig, sweeps, world=2, with_stats=False, compact=False, log=None, init=None):
    """compact: each step exchanges the compact records (np8_step_local_compact); a step where some rank's requests
    do not fit halts on every rank (np8_step_merge_compact) and is resumed with the full records (np8_step_resume,
    np8_step_merge).  log: per step, the ranks' request counts and the halt flags."""
    N = X.shape[0]
    ranks = [make() for _ in range(world)]
    counts = None if init else np.bincount(z, minlength=mu.shape[0])
    for r, c in enumerate(ranks):
        lo, hi = (N * r) // world, (N * (r + 1)) // world
        c.comm_init(None, r, world)
        c.set_data(X[lo:hi], offset=lo, n_global=N)
        if init:  # init_random(init): the global counts without communication
            c.init_random(init)
        else:
            c.set_state(z[lo:hi], mu, sig, counts=counts)
    for _ in range(sweeps):
        if compact:
            assert all(c.compact_record_bytes() > 0 for c in ranks)
            crecs = [c.step_local_compact() for c in ranks]
            halted = [c.step_merge_compact(np.concatenate(crecs), world) for c in ranks]
            if log is not None:
                log.append(([int(cr[:4].view(np.int32)[0]) for cr in crecs], halted))
            assert len(set(halted)) == 1  # the halt decision is alike on every rank
            if halted[0]:
                recs = np.concatenate([c.step_resume() for c in ranks])
                for c in ranks:
                    c.step_merge(recs, world)
        else:
            recs = np.concatenate([c.step_local() for c in ranks])
            for c in ranks:
                c.step_merge(recs, world)
        if with_stats:
            summed = sum(c.param_stats_local() for c in ranks)
            for c in ranks:
                c.end_sweep_stats(summed)
        else:
            for c in ranks:
                c.end_sweep()
    return ranks


def compare(one, ranks, exact_params):
    s1 = one.state()
    z2 = np.concatenate([c.state()["z"] for c in ranks])
    assert np.array_equal(s1["z"], z2)
    for c in ranks:
        st = c.state()
        assert st["K"] == s1["K"]
        assert np.array_equal(st["counts"], s1["counts"])
        if exact_params:
            assert np.array_equal(st["mu"], s1["mu"]) and np.array_equal(st["sigma"], s1["sigma"])
        else:
            np.testing.assert_allclose(st["mu"], s1["mu"], rtol=1e-11, atol=1e-11)
            np.testing.assert_allclose(st["sigma"], s1["sigma"], rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("D,contraction", [(8, "f64"), (64, "f32")])
def test_two_ranks_niw_frozen(D, contraction):
    X, z, cent = mixture(D, 3000, 8, D)
    sig = np.repeat(np.eye(D)[None], 8, axis=0)
    zr = np.random.default_rng(3).integers(0, 8, 3000).astype(np.int32)  # poor start: many moves, new clusters
    make = lambda: NealAlgorithm8(D, contraction=contraction, kcap=512, device=0, **niw(D, 5))  # noqa: E731
    one = make()
    one.set_data(X)
    one.set_state(zr, cent, sig)
    one.sweep(3)
    compare(one, run_sharded(make, X, zr, cent, sig, 3), exact_params=True)


def test_two_ranks_wide_reference_prior():
    D = 32
    X, z, cent = mixture(D, 2500, 6, 1)
    sig = np.repeat(np.eye(D)[None], 6, axis=0)
    kw = dict(mu0=np.zeros(D), kappa=0.02, nu=4.0, Lambda=np.eye(D) / D**2, seed=8)
    make = lambda: NealAlgorithm8(D, contraction="f32", kcap=512, device=0, **kw)  # noqa: E731
    zr = np.random.default_rng(4).integers(0, 6, 2500).astype(np.int32)
    one = make()
    one.set_data(X)
    one.set_state(zr, cent, sig)
    one.sweep(3)
    compare(one, run_sharded(make, X, zr, cent, sig, 3), exact_params=True)


@pytest.mark.parametrize("D,contraction", [(8, "f64"), (64, "f32")])
def test_two_ranks_niw_conjugate_stats_exchange(D, contraction):
    X, z, cent = mixture(D, 3000, 6, 10 + D)
    sig = np.repeat(np.eye(D)[None] * 2.0, 6, axis=0)
    make = lambda: NealAlgorithm8(D, contraction=contraction, kcap=512, device=0,  # noqa: E731
                                  param_update="niw_conjugate", **niw(D, 9))
    one = make()
    one.set_data(X)
    one.set_state(z, cent + 0.2, sig)
    one.sweep(3)
    compare(one, run_sharded(make, X, z, cent + 0.2, sig, 3, with_stats=True), exact_params=False)


def test_two_ranks_mh_g0_stats_exchange():
    D = 2
    X, z, cent = mixture(D, 4000, 5, 3)
    sig = np.repeat(np.eye(D)[None] * 9.0, 5, axis=0)
    make = lambda: NealAlgorithm8(D, kcap=512, device=0, param_update="mh_g0", seed=12)  # noqa: E731
    one = make()
    one.set_data(X)
    one.set_state(z, cent, sig)
    one.sweep(3)
    compare(one, run_sharded(make, X, z, cent, sig, 3, with_stats=True), exact_params=False)


@pytest.mark.parametrize("update,cap", [("niw_conjugate", 1), ("niw_conjugate", 32), ("frozen", 1)])
def test_two_ranks_c5_shaped_compact_records(monkeypatch, update, cap):
    """C5's sharded path (the NIW prior, the wide fp32-MFMA contraction, niw_conjugate, D = 64, N = 1e5) with the
    compact records over the host transport at world 2, capacity 1 and 32, from the reference's initialisation
    (init_random(20): the first steps carry hundreds of new-cluster requests per rank, later ones a few): a step where
    some rank's requests overflow halts on every rank and is resumed with the full records.  Labels, counts and K
    equal one rank's, parameters to the statistics' summation order (the full-record test above).  Frozen: the G0
    draws stay, items keep taking auxiliaries, and steps overflow on one rank only."""
    monkeypatch.setenv("NP8_COMPACT_REQ", str(cap))
    D, N, K, SW = 64, 100_000, 16, 5
    X, _, _ = mixture(D, N, K, 77)
    make = lambda: NealAlgorithm8(D, contraction="f32", kcap=2048, device=0,  # noqa: E731
                                  param_update=update, **niw(D, 21))
    one = make()
    one.set_data(X)
    one.init_random(20)
    one.sweep(SW)
    log = []
    ranks = run_sharded(make, X, None, None, None, SW, with_stats=update != "frozen", compact=True, log=log, init=20)
    compare(one, ranks, exact_params=update == "frozen")
    halts = [h[0] for _, h in log]
    assert ranks[0].stats()["compact_halts"] == sum(halts)
    over = [[n > cap for n in nreq] for nreq, _ in log]
    assert [any(o) for o in over] == halts  # halted exactly where some rank's requests overflowed
    print(f"cap {cap}: requests per step and rank {[n for n, _ in log]}")
    assert halts[0]  # the first step overflows
