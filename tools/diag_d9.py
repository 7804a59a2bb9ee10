"""Diagnostic (round 6): tests/test_gpu_parity.py::test_every_dimension_up_to_16_bit_exact[9]'s chain, one sweep per
call (no graphs) with the debug invariants checked after every sweep and the labels compared with the oracle's, so that
the first corrupted or diverging sweep is named before anything reads through it.  usage: python tools/diag_d9.py D"""
import os
import sys

os.environ.setdefault("NP8_NO_GRAPH", "1")
os.environ.setdefault("NP8_DEBUG_INVARIANTS", "1")
_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "oracle"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from noparama_amd import NealAlgorithm8, datasets  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 9
X, z, mu, sig = datasets.mixture(6000, D, 6, 0.6, 6.0, seed=D)
g = NealAlgorithm8(D, seed=300 + D, kcap=512, device=0)
o = O.Chain(D, seed=300 + D, kcap=512)
for c in (g, o):
    c.set_data(X)
    c.set_state(z, mu, sig)


def checks():
    """NP8_CHECKED builds: the first failed index check (line, value, lo, hi) and the count of failures."""
    import ctypes
    from noparama_amd import np8 as _np8
    L = _np8.lib()
    if not hasattr(L, "np8_exp_checks"):
        return None
    out = (ctypes.c_int * 8)()
    L.np8_exp_checks(out)
    return list(out)[:5]


def check(tag):
    try:
        g.sync()
    finally:
        c0 = checks()
        if c0 and c0[4]:
            print(f"{tag}: FAILED CHECK line {c0[0]} value {c0[1]} not in [{c0[2]}, {c0[3]}) x{c0[4]}", flush=True)
    inv = g.check_invariants() if hasattr(g, "check_invariants") else None
    a, b = g.state(params=False), o.state()
    same = a["K"] == b["K"] and np.array_equal(a["z"], b["z"])
    print(f"{tag}: K gpu {a['K']} oracle {b['K']} labels equal {same} inv {inv}", flush=True)
    if not same:
        sys.exit(3)


for s in range(3):
    g.sweep(1, sync=False)
    o.sweep(1)
    check(f"warm {s}")
for c in (g, o):
    c.init_random(20)
check("init")
for s in range(22):
    g.sweep(1, sync=False)
    o.sweep(1)
    check(f"cold {s}")
print("DIAG_OK")
