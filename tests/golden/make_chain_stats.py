"""Generates tests/golden/twogaussians_seq_stats.json: scores of the reference's sequential sampler on C1.

C1: twogaussians (tests/golden/twogaussians.data, N = 200, D = 2), the reference settings
(alpha 1, M 3, K_init 20, mu0 (6,6), kappa 1/500, nu 4, Lambda 0.01 I), T = 1000 sweeps.  The chain is the
oracle at chunk = 1 -- the reference's exact sequential sweep (np_mcmc.cpp:146-164) -- with pick = "invcdf",
the reference's own categorical draw (random_weighted_pick, dim1algebra.hpp:2078-2104, over the linear
weights), so nothing of the specification's reservoir pick is in it.  Per seed: purity, Rand index, ARI
of the max-likelihood labelling (results.score.txt, np_main.cpp:492-497) and of the last state
(snapshot.score.txt), and K of both.

tests/test_gpu_chain_stats.py compares the GPU's data-parallel sweep with these in distribution;
tests/test_chain_statistics.py re-runs a few seeds to pin the file to the oracle.

usage: python tests/golden/make_chain_stats.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import oracle as O  # noqa: E402
from noparama_amd import datasets  # noqa: E402

T = 1000
SEEDS = range(40)


def run(seed, chunk=1, pick="invcdf", T=T):
    X, lab = datasets.read_data(os.path.join(HERE, "twogaussians.data"))
    c = O.Chain(2, seed=seed, chunk=chunk, kcap=1024, pick=pick)
    c.set_data(X)
    c.init_random(20)
    assert c.sweep(T) == 0
    out = {}
    for which, tag in ((1, "maxlik"), (0, "last")):
        st = c.state(which=which)
        m = O.similarity(lab, st["z"])
        out[tag] = {"purity": m["purity"], "rand_index": m["rand_index"], "ari": m["adjusted_rand_index"], "K": st["K"]}
    return out


def main():
    res = {"chain": "oracle chunk=1 (sequential sweep), pick=invcdf (the reference's random_weighted_pick)",
           "data": "tests/golden/twogaussians.data", "T": T, "K_init": 20, "kcap": 1024,
           "seeds": {str(s): run(s) for s in SEEDS}}
    with open(os.path.join(HERE, "twogaussians_seq_stats.json"), "w") as f:
        json.dump(res, f, indent=0)


if __name__ == "__main__":
    main()
