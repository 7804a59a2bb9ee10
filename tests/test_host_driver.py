"""The C++ host mirror (host/): the reference's CLI contract and an end-to-end Neal-8 run through
MCMC -> NealAlgorithm8Hip -> C ABI on the GPU (config C1: twogaussians, T=1000)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "host", "build", "np8_noparama")
DATA = os.path.join(ROOT, "tests", "golden", "twogaussians.data")


def run(args, **kw):
    return subprocess.run([EXE] + args, capture_output=True, text=True, timeout=600, **kw)


def test_cli_contract_without_gpu(tmp_path):
    assert os.path.exists(EXE), "host driver not built (__graft_entry__.build())"
    assert run([]).returncode == 1  # usage (np_main.cpp:216-218)
    assert run(["-d", DATA, "-a", "triadic"]).returncode == 1  # unknown algorithm (np_main.cpp:231-233)
    assert run(["-d", DATA, "-a", "algorithm8", "-c", "regression", "-w", str(tmp_path / "w")]).returncode == 107
    existing = tmp_path / "exists"
    existing.mkdir()
    assert run(["-d", DATA, "-a", "algorithm8", "-w", str(existing) + "/"]).returncode == 106  # np_main.cpp:273-276
    empty = tmp_path / "empty.data"
    empty.write_text("")
    assert run(["-d", str(empty), "-a", "algorithm8", "-w", str(tmp_path / "w2")]).returncode == 7


@pytest.mark.gpu
def test_twogaussians_t1000_end_to_end(tmp_path):
    ws = str(tmp_path / "ws") + "/"
    r = run(["-d", DATA, "-a", "algorithm8", "-T", "1000", "-c", "clustering", "-s", "5", "-w", ws])
    assert r.returncode == 0, r.stderr + r.stdout
    score = open(os.path.join(ws, "5", "results.score.txt")).read()
    vals = dict(ln.split(": ") for ln in score.strip().splitlines())
    assert set(vals) == {"Purity", "Rand Index", "Adjusted Rand Index"}
    assert float(vals["Purity"]) > 0.95  # README.rst:53-55 "should be almost 1"
    assert float(vals["Adjusted Rand Index"]) > 0.0
    assert os.path.exists(os.path.join(ws, "5", "snapshot.score.txt"))
