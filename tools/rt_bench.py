"""Sweep time of the run-time-D fp64 path (np8_rt.hip) on a warm mixture state: python tools/rt_bench.py D N K [sweeps]
(synthetic data, reference prior, isotropic and non-isotropic covariances; one JSON line per case)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))
from noparama_amd import NealAlgorithm8, datasets  # noqa: E402

D, N, K = (int(a) for a in sys.argv[1:4])
S = int(sys.argv[4]) if len(sys.argv) > 4 else 20
X, z, mu, sig = datasets.mixture(N, D, K, 0.6, 6.0, seed=D)
rng = np.random.default_rng(1)
A = rng.normal(size=(K, D, D)) / np.sqrt(D)
for kind, sg in (("isotropic", sig), ("full", 0.3 * np.einsum("kab,kcb->kac", A, A) + 0.2 * np.eye(D)[None])):
    g = NealAlgorithm8(D, seed=7, kcap=512, device=0)
    g.set_data(X)
    g.set_state(z, mu, sg)
    g.sweep(5)
    g.sync()
    t = time.perf_counter()
    g.sweep(S)
    g.sync()
    dt = (time.perf_counter() - t) / S
    print(json.dumps({"path": "np8_rt (fp64, D at run time)", "D": D, "N": N, "K": g.K, "covariances": kind,
                      "ms_per_sweep": round(dt * 1e3, 3), "sweeps_per_s": round(1 / dt, 1)}), flush=True)
    g.close()
