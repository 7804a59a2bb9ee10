"""Per-wave phase timestamps of np8_assign_fast (experiment build: tools/build_variant.sh clk -DNP8_EXP_CLOCKS,
run with NP8_LIB_OVERRIDE=noparama_amd/lib/exp/clk.so): the C3 warm state, 25 sweeps, then the stamps of the
last assign launch -- phase durations (each stamp waits for the loads issued before it), wave latency, and
how the waves' start times spread over the launch."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from noparama_amd import NealAlgorithm8, datasets  # noqa: E402
from noparama_amd import np8 as _np8  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
mode = sys.argv[2] if len(sys.argv) > 2 else "warm"  # warm: the C3 state; mixed: sweep 60 after init_random(20); mixedg: graphs
X, z, mu, sig = datasets.config_c3(N=N)
s = NealAlgorithm8(8, seed=20261015, device=0)
s.set_data(X)
if mode == "mixed":
    s.init_random(20)
    s.sweep(61)
elif mode == "mixedg":  # the bench's mixed leg: 50 sweeps one by one, then graph replays (the last launch's stamps)
    s.init_random(20)
    for _ in range(50):
        s.sweep(1)
    s.sweep(40)
else:
    s.set_state(z, mu, sig)
    s.sweep(25)
nw = (N + 63) // 64
buf = np.zeros(nw * 8, dtype=np.uint64)
lib = _np8.lib()
lib.np8_exp_clocks.argtypes = [C.c_void_p, C.c_int64]
assert lib.np8_exp_clocks(buf.ctypes.data, buf.size) == 0
info = buf.reshape(nw, 8)[:, 7].copy()  # the walk's shape per wave (np8_kernels.hip NP8_CLK_INFO)
T = buf.reshape(nw, 8).astype(np.float64) * 10.0  # ns (100 MHz)
T = T[:, :7]
ok = (T > 0).all(axis=1)
T = T[ok]
t0 = T[:, 0].min()
ph = np.diff(T, axis=1)
names = ["loads x/zs/ids", "own row", "lists/table", "ny + screen L1", "aux L2/exact", "pick end/writes"]
out = {"N": N, "mode": mode, "K": s.K, "waves": int(ok.sum()), "launch_span_us": (T[:, 6].max() - t0) / 1e3,
       "wave_latency_us_mean": float((T[:, 6] - T[:, 0]).mean() / 1e3),
       "phase_us_mean": {n: float(ph[:, k].mean() / 1e3) for k, n in enumerate(names)},
       "phase_us_p90": {n: float(np.percentile(ph[:, k], 90) / 1e3) for k, n in enumerate(names)},
       "start_us_percentiles": {q: float((np.percentile(T[:, 0], q) - t0) / 1e3) for q in (0, 10, 50, 90, 100)}}
iv = info[ok]
own, grp, tab, rows = iv & 0xFF, (iv >> 8) & 0xFF, (iv >> 16) & 1, iv >> 20
lat = T[:, 6] - T[:, 0]
out["walk_shape"] = {"own_passes_mean": float(own.mean()), "own_passes_hist": np.bincount(np.minimum(own, 16)).tolist(),
                     "list_groups_hist": np.bincount(np.minimum(grp, 8)).tolist(), "table_walk_frac": float(tab.mean()),
                     "listed_rows_mean": float(rows.mean()),
                     "latency_us_by_own_passes": {int(k): float(lat[own == k].mean() / 1e3) for k in np.unique(np.minimum(own, 8))},
                     "latency_us_table_walk": float(lat[tab == 1].mean() / 1e3) if tab.any() else None}
print(json.dumps(out, indent=1))
