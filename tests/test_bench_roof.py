"""bench.py's roofline selection: the binding roof is whichever of executed flops / compute
peak and algorithmic bytes / HBM peak is the larger fraction; no GPU needed."""
import bench


def test_hbm_roof_when_pruning_leaves_little_compute():
    # C3-like: 72 MB per launch, 45 us, 0.6 TF executed of 78.6
    r = bench.binding_roof(0.6e12 * 45e-6, 72e6, 0.045, 78.6, "np8_assign")
    assert r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert abs(r["achieved"] - 72e6 / 45e-6 / 1e9) < 1e-6
    assert abs(r["frac"] - r["achieved"] / bench.HBM_PEAK_GBS) < 1e-12
    assert r["algorithmic_bytes_per_launch"] == 72e6


def test_compute_roof_when_executed_flops_dominate():
    # C5-like: 8.2 TF executed of 157.3 against 264 MB in 1.78 ms
    r = bench.binding_roof(8.2e12 * 1.78e-3, 264e6, 1.78, 157.3, "np8_assign_wide")
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s"
    assert abs(r["achieved"] - 8.2) < 1e-9 and abs(r["frac"] - 8.2 / 157.3) < 1e-12


def test_no_counters_reports_hbm():
    r = bench.binding_roof(None, 1e6, 0.01, 78.6, "np8_assign")
    assert r["bound"] == "hbm" and r["frac"] > 0
    assert bench.binding_roof(None, 1e6, 0.0, 78.6, "np8_assign")["achieved"] == 0.0


def test_weak_scaling_flag(monkeypatch):
    """--weak keeps --n items per rank (bench.py main multiplies by the ranks); the default is C4's strong scaling."""
    monkeypatch.setattr("sys.argv", ["bench.py", "--gpus", "2", "--weak", "--n", "1000"])
    a = bench.parse()
    assert a.weak and a.n == 1000 and a.gpus == 2
    monkeypatch.setattr("sys.argv", ["bench.py"])
    assert not bench.parse().weak
