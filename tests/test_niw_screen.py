"""Level 0 of the NIW auxiliary screen (noparama_amd/csrc/np8_device.h niw_aux_all_below, DESIGN.md §5 "Auxiliary
screen"): wherever it skips all of an item's auxiliaries at once, the level-1 screen skips each of them for every
draw tried (tests/native/niw_screen_check.hip, host code built with hipcc; no GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_level0_screen_implies_level1(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = str(tmp_path / "niw_screen_check")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "noparama_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "niw_screen_check.hip"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
