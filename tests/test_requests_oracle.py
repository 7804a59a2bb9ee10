"""New-cluster requests and per-visit randomness of the specification (DESIGN.md "Finalize",
"Randomness"), on the CPU oracle.

* A synchronous step accepts the A = min(req_max, free slots, requests) requests of lowest scan
  position; the free slots are counted after the step's moves, with every requester still in its old
  slot; the other requesters keep their cluster until their next update.  This replaces round 1's
  all-or-none rejection, under which a sweep from the reference's initialisation (np_mcmc.cpp:49-92,
  K=20 random G0 clusters) could not start at N = 1e5.
* Item keys: the k-th visit of an item within one epoch draws with Philox item key index | k << 32, so
  np8_update_points called repeatedly without np8_end_sweep gets fresh auxiliaries and pick uniforms
  (visit 0 is what every sweep uses).
"""
import numpy as np

import oracle as O
from noparama_amd import datasets


def _fresh(X, **kw):
    c = O.Chain(X.shape[1], seed=5, **kw)
    c.set_data(X)
    c.init_random(20)
    return c


def test_partial_accept_lowest_positions_first():
    X, _, _, _ = datasets.config_c2(N=20_000)
    probe = _fresh(X, kcap=2048, req_max=100)
    z0 = probe.state()["z"].copy()
    delta, rp, ri, rm, rz, n = probe.assign_range(0, X.shape[0])
    assert n > 100  # far more requests than req_max
    probe.finalize(delta, rp, ri, rm, rz, n_req=n)
    st = probe.state()
    order = np.argsort(rp)
    acc, dfr = ri[order[:100]], ri[order[100:]]
    K0 = int(z0.max()) + 1
    # accepted requesters sit in new clusters (labels are dense in slot order: new slots come after the
    # K0 initial ones, in position order); deferred requesters kept their label
    assert np.array_equal(st["z"][acc], K0 + np.arange(100))
    assert np.array_equal(st["z"][dfr], z0[dfr])
    assert st["K"] == K0 + 100
    assert list(probe.request_stats) == [100, n - 100]
    # the same through a whole sweep
    c = _fresh(X, kcap=2048, req_max=100)
    assert c.sweep(1) == 0
    assert list(c.request_stats) == [100, n - 100]


def test_free_slots_bound_acceptance():
    """kcap saturation: no more new clusters than free slots (counted before requesters leave)."""
    X, _ = datasets.twogaussians(5)
    c = O.Chain(2, seed=17, kcap=24, alpha=1e6)
    c.set_data(X)
    c.init_random(20)
    assert c.sweep(1) == 0
    acc, dfr = c.request_stats
    assert dfr > 0 and 0 < acc <= 24  # bounded by the free slots left after the moves of the step
    assert c.K <= 24
    for _ in range(3):
        assert c.sweep(1) == 0
        assert c.K <= 24
    st = c.state()
    assert st["counts"].sum() == X.shape[0] and (st["counts"] > 0).all()


def test_cold_start_c3_shape_progresses():
    """From init_random(20) at D = 8 the sweep creates clusters and moves on (round 1: K stuck at 20)."""
    X, z, _, _ = datasets.config_c3(N=50_000)
    O.set_threads(8)
    c = _fresh(X, kcap=2048)
    Ks = []
    for _ in range(4):
        assert c.sweep(1) == 0
        Ks.append(c.K)
    assert Ks[0] > 20 + 500
    assert Ks[-1] < Ks[0]  # spurious singletons are absorbed
    s = O.similarity(z, c.state()["z"])
    assert s["purity"] > 0.5


def test_update_points_fresh_draws_per_visit():
    """repeated np8_update_points over all items without np8_end_sweep must not cycle."""
    X, _ = datasets.twogaussians()
    c = _fresh(X, kcap=256)
    seen = set()
    ids = np.arange(X.shape[0])
    for _ in range(60):
        c.update_points(ids)
        seen.add(c.state()["z"].tobytes())
    assert c.epoch == 0
    assert len(seen) >= 55  # a deterministic cycle would revisit after a handful of calls


def test_update_points_first_visit_is_the_sweep():
    """Visit 0 draws exactly what the sequential sweep draws: update_points over the sweep's scan order
    plus end_sweep equals one chunk=1 sweep."""
    X, _ = datasets.twogaussians()
    a = _fresh(X, kcap=256, chunk=1)
    b = _fresh(X, kcap=256, chunk=1)
    N = X.shape[0]
    for t in range(3):
        order = np.array([O.perm(5, t, N, p) for p in range(N)], dtype=np.int64)
        a.update_points(order)
        a.end_sweep()
        b.sweep(1)
        assert np.array_equal(a.state()["z"], b.state()["z"])
