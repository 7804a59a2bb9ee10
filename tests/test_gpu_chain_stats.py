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
  * the GPU's data-parallel sweep in 16 synchronous sub-steps, 40 seeds: the same bounds as the sequential
    sweep.  With one step per sweep (every item against the sweep-start state) the chain over-splits small
    data; that deviation is printed and recorded in DESIGN.md "Sub-steps".
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


def gpu_run(seed, chunk, substeps=1):
    from noparama_amd import NealAlgorithm8

    X, lab = datasets.read_data(os.path.join(HERE, "golden", "twogaussians.data"))
    s = NealAlgorithm8(2, seed=seed, kcap=GOLD["kcap"], chunk=chunk, device=0, substeps=substeps)
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
    """The data-parallel sweep in 16 synchronous sub-steps (DESIGN.md "Sub-steps"; 12 items per sub-step on
    twogaussians): within SURVEY's tolerances and 3.5 standard errors of the sequential sampler.  Run as
    substeps = "auto", the host driver's default (16 sub-steps up to 8192 items, include/np8.h)."""
    runs = [gpu_run(30000 + s, chunk=0, substeps="auto") for s in range(40)]
    compare(runs, "maxlik")
    compare(runs, "last", tol=False)


@pytest.mark.timeout(300)
def test_one_step_sweep_deviation_is_recorded():
    """One synchronous step per sweep (substeps = 1: every item against the sweep-start state, the fastest
    form) over-splits small data: more clusters than the sequential sampler (200 oracle seeds: K 15.6 vs 12.5,
    max-likelihood ARI 0.251 vs 0.300, DESIGN.md "Sub-steps").  Recorded, not held to the tolerance."""
    runs = [gpu_run(40000 + s, chunk=0) for s in range(40)]
    g = golden("maxlik")
    K = np.mean([r["maxlik"]["K"] for r in runs])
    ari = np.nanmean([r["maxlik"]["ari"] for r in runs])
    print(f"one-step sweep: maxlik K {K:.2f} vs {g['K'].mean():.2f}, ARI {ari:.4f} vs {np.nanmean(g['ari']):.4f}")
    assert np.mean([r["maxlik"]["purity"] for r in runs]) > 0.99
    assert K > g["K"].mean()  # the documented direction of the deviation


def scale_run(X, lab, seed, S, T=300):
    from noparama_amd import NealAlgorithm8, metrics

    s = NealAlgorithm8(X.shape[1], seed=seed, device=0, substeps=S, kcap=1024)
    try:
        s.set_data(X)
        s.init_random(20)
        s.sweep(T)
        st = s.state(which=1, params=False)
        m = metrics.similarity(lab, st["z"])
        return m["purity"], m["adjusted_rand_index"], st["K"]
    finally:
        s.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("N,seeds", [(100_000, 4), (1_000_000, 2)])
def test_one_step_sweep_matches_substeps_at_north_star_scale(N, seeds):
    """the benchmarked sampler (one synchronous step per sweep, S = 1) against S = 16 on the C3
    generator's data (64 components, D = 8) from the reference's initialisation (init_random(20),
    np_mcmc.cpp:49-92), 300 sweeps: the max-likelihood labelling's purity and ARI against the generator's
    labels within SURVEY.md 8(d)'s tolerances (|d mean purity| <= 0.02, |d mean ARI| <= 0.05).  Unlike
    twogaussians (N = 200, where S = 1 over-splits), at this scale the synchronous step scores like the
    sub-stepped one (tools/chain_quality.py: N = 1e6, 3 seeds: ARI 0.912 for S = 1, 0.911 for S = 8)."""
    X, lab = datasets.config_c3(N=N)[:2]
    res = {S: np.array([scale_run(X, lab, 500 + r, S) for r in range(seeds)]) for S in (1, 16)}
    m1, m16 = res[1].mean(axis=0), res[16].mean(axis=0)
    print(f"N={N}: S=1 purity {m1[0]:.4f} ARI {m1[1]:.4f} K {m1[2]:.1f}; "
          f"S=16 purity {m16[0]:.4f} ARI {m16[1]:.4f} K {m16[2]:.1f}")
    assert abs(m1[0] - m16[0]) <= 0.02
    assert abs(m1[1] - m16[1]) <= 0.05
    assert m1[0] > 0.95 and m1[1] > 0.8  # and both find the components
