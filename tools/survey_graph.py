"""bench.py's survey_state leg for a kernel trace or a finalize-phase probe: C3 data (N = 1e6, D = 8, 64 clusters),
z = the generator's labels, theta = 64 G0 draws, frozen parameters; 10 eager sweeps, 20 more (graph capture), then
100 sweeps in 20-sweep graph replays (rocprofv3 --kernel-trace around this script; tools/trace_tail.py keeps the replays' kernels).  Prints
the requests accepted / rejected per timed sweep.
usage: python tools/survey_graph.py [N=1000000]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from noparama_amd import NealAlgorithm8, datasets  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
X, z, mu, sig = datasets.mixture(N, 8, 64, 0.8, 20.0, seed=20261015)
s = NealAlgorithm8(8, seed=20261015 + 2, device=0)
s.set_data(X)
s.init_random(int(z.max()) + 1)
st = s.state(params=True)
s.set_state(z.astype(np.int32), st["mu"], st["sigma"])
for _ in range(10):
    s.sweep(1)
s.sync()
s.sweep(20)  # (captures the 20-sweep graph)
s.sync()
a = s.stats()
t0 = time.perf_counter()
s.sweep(100)
s.sync()
dt = time.perf_counter() - t0
b = s.stats()
print("K", s.K, "ms/sweep %.4f" % (dt * 10.0),
      " ".join("%s %.2f" % (k, (b[k] - a[k]) / 100.0) for k in ("new_clusters", "rejected_requests", "existing_picks")))
