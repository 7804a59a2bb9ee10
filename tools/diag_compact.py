"""Diagnostic: the one-rank RCCL chain against the oracle sweep by sweep from init_random (which sweep first differs),
with and without a communicator.  usage: python tools/diag_compact.py <seed> [comm 0/1] [sweeps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from noparama_amd import NealAlgorithm8, comm_unique_id, datasets  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 72
comm = int(sys.argv[2]) if len(sys.argv) > 2 else 1
T = int(sys.argv[3]) if len(sys.argv) > 3 else 20
X, z, mu, sig = datasets.mixture(20000, 8, 24, 0.8, 12.0, seed=3)
g = NealAlgorithm8(8, seed=seed, kcap=1024, device=0)
o = O.Chain(8, seed=seed, kcap=1024)
if comm:
    g.comm_init(comm_unique_id(), 0, 1)
for c in (g, o):
    c.set_data(X)
    c.init_random(20)
for t in range(T):
    g.sweep(1)
    o.sweep(1)
    a, b = g.state(0), o.state(0)
    same = a["K"] == b["K"] and np.array_equal(a["z"], b["z"])
    print(t, "K", a["K"], b["K"], "same" if same else "DIFF", "nz_diff", int((a["z"] != b["z"]).sum()) if a["z"].shape == b["z"].shape else -1,
          "rej", g.stats()["rejected_requests"], flush=True)
    if not same:
        break
