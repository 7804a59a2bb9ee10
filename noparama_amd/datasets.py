"""Synthetic inputs (there is no network: the reference's twogaussians.data lives in another repo).

twogaussians: regenerated per the reference recipe /root/reference/scripts/generate.m:1-17 -- 100
points from N((0,0), I) labelled 0 and 100 from N((5,5), I) labelled 1, "x y label" rows.

mixture: the benchmark workloads of SURVEY.md 8(d): K components, mu_k = 6 + U[-r, r]^D,
Sigma_k = s^2 I, equal weights, labels kept as ground truth.
"""
from __future__ import annotations

import numpy as np


def twogaussians(seed: int = 20261015):
    rng = np.random.default_rng(seed)
    y0 = rng.normal(size=(100, 2))
    y1 = rng.normal(size=(100, 2)) + 5.0
    X = np.concatenate([y0, y1])
    labels = np.concatenate([np.zeros(100, dtype=np.int32), np.ones(100, dtype=np.int32)])
    return X, labels


def write_data(path, X, labels):
    """The reference's text format: 'a b c' per line (src/np_main.cpp:72-101)."""
    with open(path, "w") as f:
        for x, c in zip(X, labels):
            f.write(" ".join(f"{v:.17g}" for v in x) + f" {int(c)}\n")


def read_data(path, D=None):
    """Reader of the reference format, generalised to D value columns + one label column
    (src/np_main.cpp:57-148 hard-codes 2 columns in clustering mode).  A path ending in ".f64" is
    the binary form: raw float64 rows [N][D+1] (D required), memory-mapped."""
    if str(path).endswith(".f64"):
        if D is None:
            raise ValueError("read_data: D is required for .f64 files")
        A = np.memmap(path, dtype="<f8", mode="r").reshape(-1, D + 1)
        return np.ascontiguousarray(A[:, :D]), A[:, D].astype(np.int32)
    rows = [list(map(float, ln.split())) for ln in open(path) if ln.strip()]
    A = np.asarray(rows, dtype=np.float64)
    if D is None:
        D = A.shape[1] - 1
    return np.ascontiguousarray(A[:, :D]), A[:, D].astype(np.int32)


def write_data_f64(path, X, labels):
    """Binary form of the data file: little-endian float64 rows (x_1 .. x_D, label)."""
    A = np.concatenate([np.asarray(X, dtype="<f8"), np.asarray(labels, dtype="<f8")[:, None]], axis=1)
    A.tofile(path)


def mixture(N: int, D: int, K: int, s: float, r: float, seed: int = 20261015):
    """Returns X [N,D], ground-truth labels, component means [K,D] and covariances [K,D,D]."""
    rng = np.random.default_rng(seed)
    mu = 6.0 + rng.uniform(-r, r, size=(K, D))
    z = rng.integers(0, K, size=N).astype(np.int32)
    X = mu[z] + s * rng.normal(size=(N, D))
    sigma = np.broadcast_to((s * s) * np.eye(D), (K, D, D)).copy()
    return np.ascontiguousarray(X), z, mu, sigma


# SURVEY.md 8(d) workloads
def config_c2(N=100_000, seed=20261015):
    return mixture(N, 2, 10, 0.3, 15.0, seed)


def config_c3(N=1_000_000, seed=20261015):
    return mixture(N, 8, 64, 0.8, 20.0, seed)
