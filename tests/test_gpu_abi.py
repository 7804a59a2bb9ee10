"""The drop-in boundary's growth rules (include/np8.h "ABI growth") on a live context: np8_stats_sized writes
exactly the caller's prefix of np8_stats_t -- a caller built against the round-3 header (no folded_checks ..
pick_evals) passes its smaller struct and the bytes after it stay untouched -- and the unsized np8_stats writes
the first released layout only."""
import ctypes as C

import numpy as np
import pytest

from noparama_amd import NealAlgorithm8, datasets
from noparama_amd import np8

pytestmark = pytest.mark.gpu

GUARD = 0xA5


def _ctx():
    X, _ = datasets.twogaussians()
    g = NealAlgorithm8(2, seed=5, device=0)
    g.set_data(X)
    g.init_random(20)
    g.sweep(5)
    return g


def _call(fn, g, nbytes, *size):
    buf = (C.c_ubyte * (C.sizeof(np8.Stats) + 64))()
    C.memset(buf, GUARD, C.sizeof(buf))
    assert fn(g._h, C.cast(buf, C.POINTER(np8.Stats)), *size) == 0
    raw = bytes(buf)
    assert raw[nbytes:] == bytes([GUARD]) * (len(raw) - nbytes), "bytes past the caller's struct were written"
    return raw[:nbytes]


def test_stats_sized_honours_round3_struct():
    g = _ctx()
    L = np8.lib()
    r3 = np8.Stats.folded_checks.offset  # np8_stats_t as the round-3 header laid it out
    head = _call(L.np8_stats_sized, g, r3, C.c_size_t(r3))
    full = np8.Stats()
    assert L.np8_stats_sized(g._h, C.byref(full), C.sizeof(full)) == 0
    assert head == bytes(full)[:r3] or head[:8] == bytes(full)[:8]  # K, epoch (timers may move between calls)
    K = int.from_bytes(head[:4], "little", signed=True)
    assert K == g.K and K > 0


def test_unsized_stats_writes_first_layout_only():
    g = _ctx()
    n = np8.Stats.ms_assign.offset  # NP8_STATS_MIN_BYTES
    head = _call(np8.lib().np8_stats, g, n)
    assert int.from_bytes(head[:4], "little", signed=True) == g.K
    assert np.frombuffer(head[40:48], dtype=np.float64)[0] != 0.0  # last_loglik (the last field of the layout)
