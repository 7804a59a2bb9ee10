"""The RCCL exchange path on one GPU: a one-rank communicator (np8_comm_init with world = 1) sends every
step's record through ncclAllGather, the max-likelihood sum and the parameter statistics through
ncclAllReduce, and runs of 20 sweeps replay a hipGraph with those collectives captured -- the code the
driver's multi-GPU runs execute on each rank.  Results must equal the oracle bit for bit."""
import numpy as np
import pytest

import oracle as O
from noparama_amd import NealAlgorithm8, comm_unique_id, datasets

pytestmark = pytest.mark.gpu


def assert_same(g, o, which=0):
    a, b = g.state(which), o.state(which)
    assert a["K"] == b["K"] and np.array_equal(a["z"], b["z"]) and np.array_equal(a["counts"], b["counts"])
    np.testing.assert_allclose(a["mu"], b["mu"], rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("param_update,substeps", [("frozen", 1), ("mh_g0", 1), ("frozen", 4)])
def test_one_rank_rccl_sweeps_and_graph_bit_exact(param_update, substeps):
    X, z, mu, sig = datasets.mixture(20000, 8, 24, 0.8, 12.0, seed=3)
    g = NealAlgorithm8(8, seed=71, kcap=1024, device=0, param_update=param_update, substeps=substeps)
    o = O.Chain(8, seed=71, kcap=1024, param_update=param_update, substeps=substeps)
    try:
        g.comm_init(comm_unique_id(), 0, 1)
        for c in (g, o):
            c.set_data(X)
            c.init_random(20)
        for n in (3, 20, 22):  # eager, one graph replay, graph + eager
            g.sweep(n)
            o.sweep(n)
            assert_same(g, o)
            assert_same(g, o, which=1)
        np.testing.assert_allclose(g.stats()["best_loglik"], o.best_loglik(), rtol=1e-11)
        if param_update == "mh_g0":
            assert g.stats()["mh_accepted"] == o.mh_accepted
    finally:
        g.close()


@pytest.mark.parametrize("ccap", ["1", "4"])
def test_compact_exchange_halts_resume_bit_exact(monkeypatch, ccap):
    """Compact records too small for the cold start's requests: steps of the replayed graphs halt on the
    device, the host resumes each from the step's captured host state with the full records -- and the chain is the
    oracle's bit for bit, labels, counts, snapshot and best log-likelihood; later replays return to compact records
    once a replay's requests fit them."""
    monkeypatch.setenv("NP8_COMPACT_REQ", ccap)
    X, z, mu, sig = datasets.mixture(20000, 8, 24, 0.8, 12.0, seed=3)
    g = NealAlgorithm8(8, seed=72, kcap=1024, device=0)
    o = O.Chain(8, seed=72, kcap=1024)
    try:
        g.comm_init(comm_unique_id(), 0, 1)
        for c in (g, o):
            c.set_data(X)
            c.init_random(20)
        for n in (20, 3, 40, 20, 60):
            g.sweep(n)
            o.sweep(n)
            assert_same(g, o)
            assert_same(g, o, which=1)
        np.testing.assert_allclose(g.stats()["best_loglik"], o.best_loglik(), rtol=1e-11)
        if ccap == "1":  # (the replays' steps carry up to a few requests: one fits only some of them)
            assert g.stats()["compact_halts"] > 0
    finally:
        g.close()


def test_compact_exchange_warm_state_no_halt():
    """The C3-like warm state (few requests per step) never halts the compact records at the default capacity."""
    X, z, mu, sig = datasets.mixture(100000, 8, 64, 0.8, 20.0, seed=4)
    z = z.astype(np.int32)
    rng = np.random.default_rng(5)
    idx = rng.choice(z.size, z.size // 50, replace=False)
    z[idx] = rng.integers(0, mu.shape[0], size=idx.size)
    g = NealAlgorithm8(8, seed=73, device=0)
    o = O.Chain(8, seed=73)
    try:
        g.comm_init(comm_unique_id(), 0, 1)
        for c in (g, o):
            c.set_data(X)
            c.set_state(z, mu, sig)
        g.sweep(40)
        o.sweep(40)
        assert_same(g, o)
        assert_same(g, o, which=1)
        assert g.stats()["compact_halts"] == 0
    finally:
        g.close()
