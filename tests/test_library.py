"""CPU checks of the product library without compute: libnp8.so loads, exports exactly the C ABI that
include/np8.h declares, rejects bad configurations cleanly, and the host mirror behaves."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import noparama_amd
from noparama_amd import np8

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    L = noparama_amd.lib()
    declared = noparama_amd.header_symbols()
    assert len(declared) == 45
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", np8.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = sorted({ln.split()[-1] for ln in out.splitlines() if " T np8_" in ln})
    assert exported == declared


def test_library_is_gfx950_code_object():
    blob = open(np8.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"np8_assign" in blob and b"np8_finalize" in blob


def test_create_rejects_bad_configuration_without_crashing():
    L = noparama_amd.lib()
    mu0 = np.zeros(5)
    lam = np.eye(5)
    cfg = np8._Config()
    cfg.D, cfg.M, cfg.alpha = 5, 2, 1.0  # (D, M) = (5, 2) has no kernel instantiation
    cfg.mu0 = mu0.ctypes.data_as(C.POINTER(C.c_double))
    cfg.Lambda = lam.ctypes.data_as(C.POINTER(C.c_double))
    cfg.kappa, cfg.nu, cfg.kcap, cfg.device = 0.002, 4.0, 16, -1
    h = C.c_void_p()
    assert L.np8_create(C.byref(h), C.byref(cfg)) == np8.NP8_ERR_ARG
    cfg.D, cfg.M = 2, 3
    lam2 = -np.eye(2)  # not SPD
    cfg.Lambda = lam2.ctypes.data_as(C.POINTER(C.c_double))
    assert L.np8_create(C.byref(h), C.byref(cfg)) == np8.NP8_ERR_ARG
    assert L.np8_create(None, C.byref(cfg)) == np8.NP8_ERR_ARG
    assert L.np8_sweep(None, 1) == np8.NP8_ERR_ARG
    assert L.np8_destroy(None) == 0


def test_no_gpu_means_loud_failure():
    """Without a device the product must fail (no silent CPU fallback)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(np8.NP8Error):
        noparama_amd.NealAlgorithm8(2, device=0)


def test_header_matches_python_mirror_of_config():
    txt = open(np8.HEADER_PATH).read()
    for field, _ in np8._Config._fields_:
        assert field in txt
    for field, _ in np8.Stats._fields_:
        assert field in txt


def test_membertrix_host_view():
    m = noparama_amd.membertrix()
    m.load({"z": np.array([0, 1, 1, 2]), "counts": np.array([1, 2, 1])})
    assert m.count() == 4 and m.count(1) == 2 and m.getClusterId(2) == 1 and m.getClusterCount() == 3


def test_membertrix_mirror_follows_reference_semantics():
    """test/test_membertrix.cpp:16-93 analogue: addCluster ids in order, assign / retract with auto-remove,
    error on double assignment, cleanup of empty clusters, relabel to 0..K-1 in ascending id order."""
    m = noparama_amd.membertrix(5)
    a, b, c = (m.addCluster((np.zeros(2), np.eye(2))) for _ in range(3))
    assert (a, b, c) == (0, 1, 2)
    m.assign(a, 0)
    m.assign(c, 1)
    m.assign(c, 2)
    try:
        m.assign(b, 0)
        raise AssertionError("double assignment accepted")
    except ValueError:
        pass
    assert m.cleanup() == 1 and m.getClusterCount() == 2  # b never got an item
    m.retract(0)  # a empties and is auto-removed (membertrix.cpp:200-203)
    assert a not in m.getClusters() and m.getClusterCount() == 1
    m.assign(c, 0)
    m.relabel()
    assert m.getClusters().keys() == {0} and m.getClusterId(1) == 0 and m.count(0) == 3
    assert m.relabels_since(0) == [(1, {c: 0})]


_GUARD_SCRIPT = r"""
import ctypes as C, mmap, sys
import numpy as np
from noparama_amd import np8
L = np8.lib()
# two pages, the second PROT_NONE: a config prefix of `size` bytes ends exactly at the guard page, so any read past
# the caller's struct faults
libc = C.CDLL(None)
libc.mmap.restype = C.c_void_p
libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
libc.mprotect.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
pg = mmap.PAGESIZE
base = libc.mmap(None, 2 * pg, 3, 0x22, -1, 0)  # PROT_READ|PROT_WRITE, MAP_PRIVATE|MAP_ANONYMOUS
assert libc.mprotect(C.c_void_p(base + pg), pg, 0) == 0
size = int(sys.argv[1])
mu0, lam = np.zeros(2), np.eye(2)
cfg = np8._Config()
cfg.D, cfg.M, cfg.alpha = 2, 3, 1.0
cfg.mu0 = mu0.ctypes.data_as(C.POINTER(C.c_double))
cfg.Lambda = lam.ctypes.data_as(C.POINTER(C.c_double))
cfg.kappa, cfg.nu, cfg.kcap, cfg.device = 0.002, 4.0, 16, -1
C.memmove(base + pg - size, C.byref(cfg), size)
h = C.c_void_p()
r = L.np8_create_sized(C.byref(h), C.cast(C.c_void_p(base + pg - size), C.POINTER(np8._Config)), size)
if r == 0:
    L.np8_destroy(h)
print("RC", r)
"""


def test_create_sized_reads_only_the_callers_prefix():
    """np8_create_sized must not read past the configuration the caller allocated: the first released layout
    (NP8_CONFIG_MIN_BYTES = D .. device) placed against a PROT_NONE page creates (or fails for want of a GPU)
    without a fault; a prefix shorter than that is rejected."""
    min_bytes = np8._Config.param_update.offset
    for size in (min_bytes, C.sizeof(np8._Config)):
        out = subprocess.run(["python3", "-c", _GUARD_SCRIPT, str(size)], capture_output=True, text=True, cwd=ROOT,
                             timeout=300)
        assert out.returncode == 0, out.stderr[-2000:]
        rc = int(out.stdout.split("RC")[-1])
        assert rc in (0, np8.NP8_ERR_HIP), rc
    out = subprocess.run(["python3", "-c", _GUARD_SCRIPT, str(min_bytes - 8)], capture_output=True, text=True,
                         cwd=ROOT, timeout=300)
    assert out.returncode == 0 and int(out.stdout.split("RC")[-1]) == np8.NP8_ERR_ARG


def test_stats_sized_rejects_short_buffers_without_a_context():
    L = noparama_amd.lib()
    s = np8.Stats()
    assert L.np8_stats_sized(None, C.byref(s), C.sizeof(s)) == np8.NP8_ERR_ARG
    assert L.np8_stats(None, C.byref(s)) == np8.NP8_ERR_ARG
