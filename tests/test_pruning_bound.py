"""The candidate-pruning bound of np8_prune (DESIGN.md "Pruning"), checked on oracle states: every
row the bound leaves out of cluster k0's list must be skipped by pick_step for every item of k0
(log-weight at least kSkip = 80 below the item's own).  CPU only; the GPU parity tests then check that the
pruned sweep equals the oracle's unpruned one bit for bit."""
import numpy as np
import pytest

import oracle as O
from noparama_amd import datasets

SKIP, MARGIN = 80.0, 2.0


def _violations(chain, X, D):
    st = chain.state()
    z, K, mu, sig, cnt = st["z"], st["K"], st["mu"], st["sigma"], st["counts"]
    prec = np.linalg.inv(sig)
    pruned = bad = 0
    for k0 in range(K):
        iso0 = prec[k0][0, 0]
        if cnt[k0] <= 1 or not np.array_equal(prec[k0], iso0 * np.eye(D)):
            continue
        d0 = X[z == k0] - mu[k0]
        R2 = (d0 ** 2).sum(1).max()
        c0 = -0.5 * (D * np.log(2 * np.pi) - np.linalg.slogdet(prec[k0])[1])
        base0 = c0 + np.log(cnt[k0] - 1)
        lw_own = base0 - 0.5 * iso0 * (d0 ** 2).sum(1)
        for j in range(K):
            isoj = prec[j][0, 0]
            if j == k0 or not np.array_equal(prec[j], isoj * np.eye(D)):
                continue
            delta = np.sqrt(((mu[j] - mu[k0]) ** 2).sum()) - np.sqrt(R2)
            if delta <= 0:
                continue
            cj = -0.5 * (D * np.log(2 * np.pi) - np.linalg.slogdet(prec[j])[1]) + np.log(cnt[j])
            U = (cj - base0) - 0.5 * isoj * delta ** 2 + 0.5 * iso0 * R2
            if U <= -SKIP - MARGIN:
                pruned += 1
                lw_j = cj - 0.5 * isoj * ((X[z == k0] - mu[j]) ** 2).sum(1)
                bad += int((lw_j - lw_own).max() > -SKIP)
    return pruned, bad


@pytest.mark.parametrize("D,K,N,s,r,init", [(3, 10, 3000, 0.5, 8.0, True), (8, 24, 6000, 0.5, 8.0, False),
                                            (2, 12, 4000, 0.3, 15.0, False)])
def test_pruned_rows_are_always_skipped(D, K, N, s, r, init):
    X, z, mu, sig = datasets.mixture(N, D, K, s, r, seed=D)
    c = O.Chain(D, seed=5 + D, kcap=4096)
    c.set_data(X)
    if init:
        c.init_random(20)
    else:
        c.set_state(z, mu, sig)
    total = 0
    for _ in range(4):
        c.sweep(1)
        pruned, bad = _violations(c, X, D)
        assert bad == 0
        total += pruned
    assert total > 0  # the bound does prune on these states
