"""SURVEY.md 5 auxiliary rows on the GPU: exact checkpoint / resume (a resumed chain equals the uninterrupted
one bit for bit) and the debug invariant check (labels, counts, K, candidate table)."""
import os

import numpy as np
import pytest

from noparama_amd import NP8Error, NealAlgorithm8, datasets

pytestmark = pytest.mark.gpu


def state_of(s):
    st = s.state()
    best = s.state(which=1)
    return st, best, s.stats()


@pytest.mark.parametrize("param_update,substeps", [("frozen", 1), ("mh_g0", 1), ("frozen", 4)])
def test_resumed_chain_equals_uninterrupted(param_update, substeps):
    X = datasets.config_c3(N=30000)[0]
    kw = dict(seed=91, kcap=1024, device=0, param_update=param_update, substeps=substeps)
    a = NealAlgorithm8(8, **kw)
    b = NealAlgorithm8(8, **kw)
    try:
        a.set_data(X)
        a.init_random(20)  # a cold start: clusters keep appearing and emptying after the checkpoint
        a.sweep(7)
        ck = a.checkpoint()
        a.sweep(26)  # a graph replay and eager sweeps
        b.set_data(X)
        b.restore(ck)
        b.sweep(26)
        sa, ba, ta = state_of(a)
        sb, bb, tb = state_of(b)
        for x, y in ((sa, sb), (ba, bb)):
            assert x["K"] == y["K"] and np.array_equal(x["z"], y["z"]) and np.array_equal(x["counts"], y["counts"])
            assert np.array_equal(x["mu"], y["mu"]) and np.array_equal(x["sigma"], y["sigma"])
        for k in ("epoch", "new_clusters", "rejected_requests", "best_loglik", "mh_accepted"):
            assert ta[k] == tb[k], k
        assert a.check_invariants().tolist() == [0, 0, 0, X.shape[0]]
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("other", [dict(seed=2), dict(param_update="mh_g0"), dict(alpha=2.0), dict(kappa=0.01),
                                   dict(req_max=64), dict(mh_steps=5), dict(chunk=100), "data"])
def test_restore_rejects_other_configuration(other):
    """a checkpoint names its configuration (parameter update, MH steps, req_max, chunk, the
    hyper-parameters) and its data (a hash of the items np8_set_data received); restoring it into anything
    else fails instead of silently continuing as another chain."""
    X = datasets.config_c3(N=5000)[0]
    base = dict(seed=1, kcap=512, device=0)
    a = NealAlgorithm8(8, **base)
    b = NealAlgorithm8(8, **{**base, **(other if isinstance(other, dict) else {})})
    try:
        a.set_data(X)
        a.init_random(20)
        ck = a.checkpoint()
        if other == "data":
            X2 = X.copy()
            X2[1234, 3] += 1e-9
            b.set_data(X2)
        else:
            b.set_data(X)
        with pytest.raises(NP8Error):
            b.restore(ck)
    finally:
        a.close()
        b.close()


def test_invariant_check_flags_inconsistent_counts():
    X, z, mu, sig = datasets.mixture(4000, 2, 4, 0.3, 5.0, seed=2)
    s = NealAlgorithm8(2, seed=3, kcap=256, device=0)
    try:
        s.set_data(X)
        s.set_state(z, mu, sig)
        assert s.check_invariants().tolist() == [0, 0, 0, 4000]
        s.set_state(z, mu, sig, counts=np.bincount(z) + 1)  # counts that disagree with the labels
        out = s.check_invariants(raise_on_violation=False)
        assert out[0] & 2 and out[0] & 4 and out[3] == 4004
    finally:
        s.close()


def test_invariants_every_sweep_under_the_debug_flag(monkeypatch):
    monkeypatch.setenv("NP8_DEBUG_INVARIANTS", "1")
    X = datasets.config_c3(N=20000)[0]
    s = NealAlgorithm8(8, seed=5, kcap=1024, device=0)
    try:
        s.set_data(X)
        s.init_random(20)
        s.sweep(25)  # np8_sync reports a violation raised on the device
        assert s.stats()["K"] > 20
    finally:
        s.close()
