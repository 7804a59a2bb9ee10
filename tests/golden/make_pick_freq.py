"""Generates tests/golden/pick_freq.json: frequency tables of the reference's own categorical draw.

The draw is `algebra::random_weighted_pick` (/root/reference/include/helper/dim1algebra.hpp:2078-2104),
compiled from the reference header in place by oracle/Makefile into oracle/_ref/libnp8ref.so (test
infrastructure; nothing of the header is copied).  For each fixed log-weight vector below it is fed
n_draws uniforms u_k from numpy's PCG64(seed) (`random()`, 53-bit), with

  * "shifted": the linear weights exp(lw - max lw) -- what a point update's weights are up to a common
    factor, the form the specification's log-space pick is equal in distribution to;
  * "raw": the linear weights exp(lw) as the reference's NealAlgorithm8 forms them
    (np_neal_algorithm8.cpp:107,118: probability() * count, alpha / M); they underflow when every candidate is far,
    and the reference then returns index 0 (lower_bound of 0 in a zero cumulative sum).

Stored per case: lw, seed, n_draws, the two count vectors and the exact probabilities.  The tests
(tests/test_pick_distribution.py) check the oracle's reservoir pick against these tables by chi-square
with independent uniforms, and the device pick (np8_pick_batch) bit for bit against the oracle.

usage: python tests/golden/make_pick_freq.py   (needs oracle/_ref, i.e. /root/reference, at build time)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

N_DRAWS = 200_000


def cases():
    rng = np.random.default_rng(20261016)
    out = {
        # the item's own cluster alone (no other live cluster, every auxiliary skipped)
        "single": [-3.0],
        "two_equal": [0.0, 0.0],
        # own cluster first, then clusters and auxiliaries of mixed weight
        "spread": [0.0, -1.0, -2.0, -5.0, -10.0, 1.5, -0.3],
        # around the skip threshold (-80 relative to the running maximum): -79 is evaluated, -81 skipped
        "near_threshold": [0.0, -79.0, -81.0, -0.5, -80.0],
        # the running maximum moves up through the list (the reservoir's d > 0 branch every step)
        "increasing": [-10.0, -8.0, -6.0, -4.0, -2.0, 0.0],
        # a singleton's own cluster has weight 0 (the finite -1e300 of the specification)
        "singleton_own": [-1e300, -2.0, -1.0, -3.0],
        # widely spread log-weights (sd 20): most candidates are negligible, a few compete
        "wide64": list(np.round(rng.normal(0.0, 20.0, 64), 6)),
        # many candidates of similar weight (the C3 regime inside a cluster's neighbourhood)
        "flat200": list(np.round(rng.normal(0.0, 1.0, 200), 6)),
        # every linear weight underflows (an item far from everything): only the shifted form is a
        # distribution; the reference's raw form returns index 0
        "all_far": [-900.0, -905.0, -899.5, -950.0],
    }
    return out


def main():
    ref = O.ref_harness()
    if ref is None:
        raise SystemExit("oracle/_ref/libnp8ref.so is not built (needs /root/reference)")
    res = {"source": "algebra::random_weighted_pick, /root/reference/include/helper/dim1algebra.hpp:2078-2104 "
                     "(oracle/_ref/libnp8ref.so)",
           "uniforms": "numpy.random.Generator(PCG64(seed)).random(n_draws)", "cases": {}}
    for k, (name, lw) in enumerate(cases().items()):
        lw = np.asarray(lw, dtype=np.float64)
        seed = 1000 + k
        u = np.random.Generator(np.random.PCG64(seed)).random(N_DRAWS)
        ws = np.exp(lw - lw.max())
        wr = np.exp(lw)
        cs = np.zeros(lw.size, dtype=np.int64)
        cr = np.zeros(lw.size, dtype=np.int64)
        for uk in u:
            cs[ref.np8ref_weighted_pick(ws.ctypes.data, lw.size, float(uk))] += 1
            cr[ref.np8ref_weighted_pick(wr.ctypes.data, lw.size, float(uk))] += 1
        res["cases"][name] = {"lw": lw.tolist(), "seed": seed, "n_draws": N_DRAWS, "counts_shifted": cs.tolist(),
                              "counts_raw": cr.tolist(), "p": (ws / ws.sum()).tolist()}
        print(name, cs[:8], cr[:8])
    with open(os.path.join(HERE, "pick_freq.json"), "w") as f:
        json.dump(res, f, indent=0)


if __name__ == "__main__":
    main()
