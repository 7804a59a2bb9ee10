"""Clustering metrics of the Python host mirror: the reference's clustering_performance
(src/clustering_performance.cpp:14-82) -- contingency matrix with the ground truth as rows
(calculateContingencyMatrix :14-36), purity (:52), Rand index (:65) and adjusted Rand index (:75) --
in int64 counts instead of the reference's int32 (which overflow past a few hundred items).
Same arithmetic as the C++ mirror (host/np_host.cpp clustering_performance::calculate).  Where the reference returns
early and leaves the index unset (clustering_performance.cpp:70-73, and S == 0), both mirrors report NaN: that is
their own convention for the reference's early return, not a value the reference computes (no reference fixture
pins it).
"""
from __future__ import annotations

import numpy as np


def contingency(truth, result):
    t = np.asarray(truth, dtype=np.int64)
    r = np.asarray(result, dtype=np.int64)
    if t.shape != r.shape or t.size == 0:
        raise ValueError("contingency: labellings of equal, non-zero length required")
    _, ti = np.unique(t, return_inverse=True)
    _, ri = np.unique(r, return_inverse=True)
    F = np.zeros((ti.max() + 1, ri.max() + 1), dtype=np.int64)
    np.add.at(F, (ti, ri), 1)
    return F


def similarity(truth, result):
    """{"purity", "rand_index", "adjusted_rand_index"} of result against truth."""
    F = contingency(truth, result)
    N = int(F.sum())

    def pairs(v):
        v = v.astype(np.int64)
        return int(((v * v - v) // 2).sum())

    a, b, c = pairs(F.ravel()), pairs(F.sum(axis=1)), pairs(F.sum(axis=0))
    purity = int(F.max(axis=0).sum()) / N
    S = (float(N) * N - N) / 2.0
    ri = ari = float("nan")
    if S:
        ri = (2 * a - b - c) / S + 1.0
        bc_S, bpc_2 = float(b) * float(c) / S, (b + c) / 2.0
        if bc_S != bpc_2:
            ari = (a - bc_S) / (bpc_2 - bc_S)
    return {"purity": purity, "rand_index": ri, "adjusted_rand_index": ari}
