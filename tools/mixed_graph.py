"""The bench's mixed leg for a kernel trace: C3 data, init_random(20), 50 sweeps one by one, then 40 in 20-sweep graph
replays (rocprofv3 --kernel-trace around this script; tools/trace_tail.py keeps the replays' kernels).
usage: python tools/mixed_graph.py [N=1000000]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from noparama_amd import NealAlgorithm8, datasets  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
X, z, mu, sig = datasets.config_c3(N=N)
s = NealAlgorithm8(8, seed=20261016, device=0)
s.set_data(X)
s.init_random(20)
for t in range(50):
    s.sweep(1)
s.sync()
s.sweep(40)
s.sync()
print("K", s.K)
