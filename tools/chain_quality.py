"""Chain quality of the data-parallel sweep at the north-star scale: from the reference's
initialisation (init_random(20), np_mcmc.cpp:49-92) on the C3 generator's data, T sweeps for each number
of synchronous sub-steps S; per 10 sweeps K, and at the end purity / RI / ARI of the max-likelihood and the
last labelling against the generator's labels (noparama_amd.metrics = clustering_performance.cpp:38-82).

  python tools/chain_quality.py --n 1000000 --substeps 1,2,4,16 --seeds 3 --sweeps 300 --out gpurun_out/cq.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from noparama_amd import NealAlgorithm8, datasets, metrics  # noqa: E402


def run(X, lab, seed, S, T, every=10, alpha=1.0):
    # the sort of the sub-step layout holds substeps * kcap <= 16384 bins (np8_create)
    s = NealAlgorithm8(X.shape[1], seed=seed, device=0, substeps=S, alpha=alpha, kcap=min(2048, 16384 // S))
    try:
        s.set_data(X)
        s.init_random(20)
        Ks, t0 = [], time.perf_counter()
        for _ in range(T // every):
            s.sweep(every)
            Ks.append(s.K)
        el = time.perf_counter() - t0
        out = {"K_every_%d" % every: Ks, "seconds": el, "sweeps_per_s": T / el}
        for which, tag in ((1, "maxlik"), (0, "last")):
            st = s.state(which=which, params=False)
            m = metrics.similarity(lab, st["z"])
            out[tag] = {"K": st["K"], "purity": m["purity"], "rand_index": m["rand_index"],
                        "ari": m["adjusted_rand_index"]}
        st = s.stats()
        out["new_clusters"], out["deferred_requests"] = st["new_clusters"], st["rejected_requests"]
        return out
    finally:
        s.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--substeps", default="1,2,4,16")
    ap.add_argument("--seeds", type=int, default=3)
    ap.add_argument("--sweeps", type=int, default=300)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    X, lab = datasets.config_c3(N=a.n)[:2]
    res = {"n": a.n, "sweeps": a.sweeps, "init": "init_random(20)", "runs": {}}
    for S in map(int, a.substeps.split(",")):
        rows = [run(X, lab, 1000 + r, S, a.sweeps) for r in range(a.seeds)]
        res["runs"][f"S={S}"] = rows
        summ = {t: {f: float(np.mean([r[t][f] for r in rows])) for f in ("K", "purity", "ari")}
                for t in ("maxlik", "last")}
        res.setdefault("summary", {})[f"S={S}"] = summ
        print(f"N={a.n} S={S}: {json.dumps(summ)} "
              f"{np.mean([r['sweeps_per_s'] for r in rows]):.0f} sweeps/s", flush=True)
        if a.out:
            json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
