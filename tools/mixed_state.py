"""The regime the reference's own start reaches: C3 data, init_random(20), then sweeps one by
one; for profiling the assign kernel there (rocprofv3 --pmc / --kernel-trace around this script).
usage: python tools/mixed_state.py [sweeps=80] [N=1000000]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from noparama_amd import NealAlgorithm8, datasets  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 80
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
X, z, mu, sig = datasets.config_c3(N=N)
s = NealAlgorithm8(8, seed=20261016, device=0)
s.set_data(X)
s.init_random(20)
for t in range(T):
    s.sweep(1)
print("K", s.K, "sweeps", T)
