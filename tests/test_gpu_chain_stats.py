"""The GPU chain against the reference's sequential sampler, in distribution (config C1).

The reference is unseeded (src/np_main.cpp:180), so its chain can only be matched in distribution.
tests/golden/twogaussians_seq_stats.json holds 40 seeds of the reference's algorithm run by the oracle:
chunk = 1 (the exact sequential sweep of np_mcmc.cpp:146-164) with pick = "invcdf" (the reference's own
random_weighted_pick over linear weights, dim1algebra.hpp:2078-2104) -- nothing of the GPU's specification
(reservoir pick, synchronous steps) is in it.  On twogaussians, T = 1000, the reference settings:

  * the GPU's sequential sweep (chunk = 1: the reference's algorithm, the device's reservoir pick), 20 seeds:
    purity, ARI and K of the max-likelihood labelling within SURVEY.md 8(d)'s tolerances (|d mean purity|
    <= 0.02, |d mean ARI| <= 0.05), and those of the max-likelihood labelling and of the last state within
    3.5 standard errors of the golden means (Welch);
  * the GPU's data-parallel sweep (chunk = N, the benchmarked path), 40 seeds: the max-likelihood
    labelling (results.score.txt, np_main.cpp:492-497) within SURVEY.md's tolerances.  Its deviation in K
    and in the last state's ARI (a synchronous step is not an exact Gibbs step) is printed, and recorded
    in DESIGN.md.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from noparama_amd import datasets

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "twogaussians_seq_stats.json")))
T = GOLD["T"]
FIELDS = ("purity", "ari", "K")


def golden(tag):
    return {f: np.array([v[tag][f] for v in GOLD["seeds"].values()], dtype=np.float64) for f in FIELDS}


def gpu_run(seed, chunk):
    from noparama_amd import NealAlgorithm8

    X, lab = datasets.read_data(os.path.join(HERE, "golden", "twogaussians.data"))
    s = NealAlgorithm8(2, seed=seed, kcap=GOLD["kcap"], chunk=chunk, device=0)
    try:
        s.set_data(X)
        s.init_random(GOLD["K_init"])
        s.sweep(T)
        out = {}
        for which, tag in ((1, "maxlik"), (0, "last")):
            st = s.state(which=which, params=False)
            m = O.similarity(lab, st["z"])
            out[tag] = {"purity": m["purity"], "ari": m["adjusted_rand_index"], "K": st["K"]}
        return out
    finally:
        s.close()


def compare(runs, tag, welch=True, tol=True):
    g = golden(tag)
    report = {}
    for f in FIELDS:
        a = g[f][~np.isnan(g[f])]
        b = np.array([r[tag][f] for r in runs], dtype=np.float64)
        b = b[~np.isnan(b)]
        se = np.sqrt(a.var(ddof=1) / a.size + b.var(ddof=1) / b.size) + 1e-12
        report[f] = (a.mean(), b.mean(), (b.mean() - a.mean()) / se)
    print(tag, {f: tuple(round(float(x), 4) for x in v) for f, v in report.items()})
    if tol:
        assert abs(report["purity"][1] - report["purity"][0]) <= 0.02, report
        assert abs(report["ari"][1] - report["ari"][0]) <= 0.05, report
    if welch:
        for f in FIELDS:
            assert abs(report[f][2]) <= 3.5, (tag, f, report[f])
    return report


@pytest.mark.timeout(900)
def test_sequential_gpu_chain_matches_reference_sampler():
    runs = [gpu_run(20000 + s, chunk=1) for s in range(20)]
    compare(runs, "maxlik")
    # the last state's ARI spreads widely (sd ~0.15 over seeds): at 20 seeds SURVEY's absolute 0.05 is
    # 1.4 standard errors of the difference, so the last state is held to the Welch bound only
    compare(runs, "last", tol=False)


@pytest.mark.timeout(300)
def test_data_parallel_gpu_chain_scores_like_reference_sampler():
    runs = [gpu_run(30000 + s, chunk=0) for s in range(40)]
    compare(runs, "maxlik", welch=False)
    g, b = golden("last"), np.array([[r["last"]["ari"], r["last"]["K"]] for r in runs])
    print("data-parallel last state: ARI %.4f vs %.4f, K %.2f vs %.2f (reference sequential)"
          % (np.nanmean(b[:, 0]), np.nanmean(g["ari"]), b[:, 1].mean(), g["K"].mean()))
