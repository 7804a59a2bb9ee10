"""GPU: the two-kernel step (np8_assign_fast for the lanes it can finish, np8_assign_queue for the lanes it defers)
against the oracle and against the one-kernel forms, in the states where the split is mixed inside a wave.

* isotropic Lambda (every G0 draw isotropic) with anisotropic per-slot Sigma uploaded by set_state: lanes whose own
  row or a walked row is anisotropic are deferred, the others finish in the fast kernel -- within one wave when some
  lanes walk their pruned list and others (outside the list's radius) the whole table;
* a diagonal but anisotropic Lambda (the base measure's whitening diagonal, gp_iso = 0): every G0 draw anisotropic.

Labels, counts, K and the snapshot bit-exact against the oracle, and against NP8_NO_FAST=1 (np8_assign alone) and
NP8_QUEUE=1 (the queue launch kept although no lane could defer)."""
import os

import numpy as np
import pytest

import oracle as O
from noparama_amd import NealAlgorithm8, datasets

pytestmark = pytest.mark.gpu


def make(env, **kw):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return NealAlgorithm8(8, device=0, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def mixed_state(N=30_000, K=12, seed=4):
    """C3-style data with half of the clusters anisotropic (diag(s^2 r), r in [0.4, 2.5]) and 25% of the labels
    scrambled, so that many items move and walk."""
    rng = np.random.default_rng(seed)
    D = 8
    mu = 6.0 + rng.uniform(-12, 12, size=(K, D))
    sig = np.empty((K, D, D))
    for k in range(K):
        r = np.ones(D) if k < K // 2 else rng.uniform(0.4, 2.5, size=D)
        sig[k] = np.diag(0.8 ** 2 * r)
    zt = rng.integers(0, K, size=N)
    X = mu[zt] + rng.normal(size=(N, D)) * np.sqrt(np.einsum("kaa->ka", sig)[zt])
    z = zt.copy()
    idx = rng.choice(N, N // 4, replace=False)
    z[idx] = rng.integers(0, K, size=idx.size)
    return X, z.astype(np.int32), mu, sig


def same(a, b, which=0):
    sa, sb = a.state(which), b.state(which)
    assert sa["K"] == sb["K"]
    assert np.array_equal(sa["z"], sb["z"])
    assert np.array_equal(sa["counts"], sb["counts"])
    np.testing.assert_allclose(sa["mu"], sb["mu"], rtol=1e-13, atol=1e-13)


def test_anisotropic_slots_isotropic_lambda():
    X, z, mu, sig = mixed_state()
    runs = [make({}, seed=8), make({"NP8_NO_FAST": "1"}, seed=8), make({"NP8_QUEUE": "1"}, seed=8)]
    o = O.Chain(8, seed=8, kcap=runs[0].kcap)
    for s in runs + [o]:
        s.set_data(X)
        s.set_state(z, mu, sig)
    for n in (3, 20, 4):  # eager, a graph replay (gathering sweeps: lists), eager
        for s in runs + [o]:
            s.sweep(n)
        for s in runs:
            same(s, o)
            same(s, o, which=1)


def test_diagonal_anisotropic_lambda_every_row_deferred():
    X, _, _, _ = mixed_state(N=20_000)
    lam = np.diag(0.01 * np.array([1.0, 2.0, 0.5, 1.5, 0.8, 1.2, 3.0, 0.6]))
    runs = [make({}, seed=9, Lambda=lam), make({"NP8_NO_FAST": "1"}, seed=9, Lambda=lam)]
    o = O.Chain(8, seed=9, kcap=runs[0].kcap, Lambda=lam)
    for s in runs + [o]:
        s.set_data(X)
        s.init_random(20)
    for n in (2, 20, 3):
        for s in runs + [o]:
            s.sweep(n)
        for s in runs:
            same(s, o)
            same(s, o, which=1)


def test_c3_generator_fast_vs_one_kernel():
    """The benchmark's own generator and warm state, scrambled: the fast kernel (queue left out, every row
    isotropic) against np8_assign alone and against the fast kernel with the queue launch forced."""
    X, zt, mu, sig = datasets.config_c3(N=100_000)
    z = zt.astype(np.int32).copy()
    rng = np.random.default_rng(6)
    idx = rng.choice(z.size, z.size // 10, replace=False)
    z[idx] = rng.integers(0, mu.shape[0], size=idx.size)
    runs = [make({}, seed=12), make({"NP8_NO_FAST": "1"}, seed=12), make({"NP8_QUEUE": "1"}, seed=12)]
    for s in runs:
        s.set_data(X)
        s.set_state(z, mu, sig)
    for n in (2, 20, 5):
        for s in runs:
            s.sweep(n)
        for s in runs[1:]:
            same(runs[0], s)
            same(runs[0], s, which=1)
