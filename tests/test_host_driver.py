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
    assert run(["-d", DATA, "-a", "algorithm2"]).returncode == 1  # unknown algorithm (np_main.cpp:231-233)
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
    run_dir = os.path.join(ws, "LATEST")  # np_results.cpp:53-63
    score = open(os.path.join(run_dir, "results.score.txt")).read()
    vals = dict(ln.split(": ") for ln in score.strip().splitlines())
    assert set(vals) == {"Purity", "Rand Index", "Adjusted Rand Index"}
    assert float(vals["Purity"]) > 0.95  # README.rst:53-55 "should be almost 1"
    assert float(vals["Adjusted Rand Index"]) > 0.0
    for base in ("snapshot", "results"):
        assert os.path.exists(os.path.join(run_dir, base + ".score.txt"))
        K = int(open(os.path.join(run_dir, base + ".txt")).read().split("# rows: ")[1].split()[0])
        sizes = [len(open(os.path.join(run_dir, f"{base}{k}.txt")).read().splitlines()) for k in range(K)]
        assert sum(sizes) == 200 and min(sizes) > 0  # every item in exactly one cluster file


def test_results_files_in_reference_format(tmp_path):
    """np_results.cpp:39-196: per-cluster item files, Octave mu/sigma, scores, LATEST symlink."""
    exe = os.path.join(ROOT, "host", "build", "results_selftest")
    ws = str(tmp_path) + "/"
    r = subprocess.run([exe, ws], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = os.path.join(ws, "20261015_12:00")
    assert os.path.realpath(os.path.join(ws, "LATEST")) == os.path.realpath(d)
    assert open(os.path.join(d, "results0.txt")).read() == "1.5 2.25 \n1 2 \n1.25 2.5 \n"
    assert open(os.path.join(d, "results1.txt")).read() == "-3 0.5 \n-2.5 0.75 \n"
    assert open(os.path.join(d, "results.txt")).read() == (
        "# name: mu\n# type: matrix\n# rows: 2\n# columns: 2\n 1.25 2.25\n -2.75 0.625\n\n\n"
        "# name: sigma\n# type: matrix\n# ndims: 3\n 2 2 2\n 0.1 0 \n0 0.2\n 0.3 0.01 \n0.01 0.4\n")
    assert open(os.path.join(d, "results.score.txt")).read() == (
        "Purity: 1\nRand Index: 1\nAdjusted Rand Index: 1\n")


def test_product_metrics_match_sklearn_goldens(tmp_path):
    """the product's clustering_performance::calculate (host/np_host.cpp, which writes
    results.score.txt; reference src/clustering_performance.cpp:38-82 with int64 counts instead of its
    int32 ones) against sklearn's adjusted_rand_score / rand_score and a numpy purity
    (tests/golden/metrics.json), plus one case past the reference's int32 overflow (N = 200 000)."""
    import json
    import math

    import numpy as np

    exe = os.path.join(ROOT, "host", "build", "results_selftest")
    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "metrics.json")))
    big = np.repeat([0, 1, 2, 3], 50_000)
    big_res = big.copy()
    big_res[::7] = (big_res[::7] + 1) % 4
    p = tmp_path / "pairs.txt"
    with open(p, "w") as f:
        for c in cases:
            f.write(" ".join(map(str, c["truth"])) + "\n" + " ".join(map(str, c["result"])) + "\n")
        f.write(" ".join(map(str, big)) + "\n" + " ".join(map(str, big_res)) + "\n")
    r = subprocess.run([exe, "--metrics", str(p)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rows = [list(map(float, ln.split())) for ln in r.stdout.strip().splitlines()]
    assert len(rows) == len(cases) + 1
    for c, (pur, ri, ari) in zip(cases, rows):
        assert abs(pur - c["purity"]) <= 1e-12
        assert abs(ri - c["rand_index"]) <= 1e-12
        if math.isnan(ari):
            # the reference's formula is 0/0 (both labellings one cluster, or both all singletons):
            # clustering_performance.cpp:75 divides anyway (NaN); sklearn defines that case as 1.0
            assert c["ari"] == 1.0 and (len(set(c["truth"])) in (1, len(c["truth"])))
        else:
            assert abs(ari - c["ari"]) <= 1e-12, (ari, c["ari"])
    # the large case against the int64 formula computed here (sklearn's own formula, in Python ints)
    F = np.zeros((4, 4), dtype=object)
    np.add.at(F, (big, big_res), 1)
    comb = lambda v: v * (v - 1) // 2  # noqa: E731
    a = sum(comb(int(v)) for v in F.ravel())
    b = sum(comb(int(v)) for v in F.sum(axis=1))
    c_ = sum(comb(int(v)) for v in F.sum(axis=0))
    S = comb(big.size)
    exp_ari = (a - b * c_ / S) / ((b + c_) / 2 - b * c_ / S)
    assert abs(rows[-1][0] - sum(F.max(axis=0)) / big.size) <= 1e-12
    assert abs(rows[-1][1] - ((2 * a - b - c_) / S + 1)) <= 1e-12
    assert abs(rows[-1][2] - exp_ari) <= 1e-12


def test_f64_data_roundtrip(tmp_path):
    from noparama_amd import datasets

    X, z = datasets.twogaussians()
    p = str(tmp_path / "tg.f64")
    datasets.write_data_f64(p, X, z)
    X2, z2 = datasets.read_data(p, D=2)
    assert (X2 == X).all() and (z2 == z).all()


@pytest.mark.gpu
def test_binary_data_and_subsample(tmp_path):
    """np_main.cpp:283-295: a random subset of -n items (the reference's default is 200 of the file)."""
    from noparama_amd import datasets

    X, z = datasets.twogaussians()
    data = str(tmp_path / "tg.f64")
    datasets.write_data_f64(data, X, z)
    ws = str(tmp_path / "ws") + "/"
    r = run(["-d", data, "-a", "algorithm8", "-T", "200", "-s", "3", "-n", "120", "-w", ws])
    assert r.returncode == 0, r.stderr + r.stdout
    run_dir = os.path.join(ws, "LATEST")
    K = int(open(os.path.join(run_dir, "snapshot.txt")).read().split("# rows: ")[1].split()[0])
    n = sum(len(open(os.path.join(run_dir, f"snapshot{k}.txt")).read().splitlines()) for k in range(K))
    assert n == 120


@pytest.mark.gpu
def test_twogaussians_niw_conjugate_end_to_end(tmp_path):
    """The C++ driver with the NIW prior and the conjugate cluster update (-u niw_conjugate)."""
    ws = str(tmp_path / "ws") + "/"
    r = run(["-d", DATA, "-a", "algorithm8", "-T", "300", "-s", "3", "-u", "niw_conjugate", "-w", ws])
    assert r.returncode == 0, r.stderr + r.stdout
    score = open(os.path.join(ws, "LATEST", "results.score.txt")).read()
    vals = dict(ln.split(": ") for ln in score.strip().splitlines())
    assert float(vals["Purity"]) > 0.95


def test_cli_rejects_bad_prior_and_contraction(tmp_path):
    assert run(["-d", DATA, "-a", "algorithm8", "-p", "dirichlet", "-w", str(tmp_path / "a")]).returncode == 1
    assert run(["-d", DATA, "-a", "algorithm8", "-x", "bf16", "-w", str(tmp_path / "b")]).returncode == 1


@pytest.mark.gpu
def test_jain_neal_split_end_to_end(tmp_path):
    """`-a jain_neal_split` (np_main.cpp:440-445): the split-merge population update through the same
    MCMC driver; results written in the reference's layout and statistics printed."""
    ws = str(tmp_path / "ws") + "/"
    r = run(["-d", DATA, "-a", "jain_neal_split", "-T", "200", "-c", "clustering", "-s", "5", "-w", ws])
    assert r.returncode == 0, r.stderr + r.stdout
    assert "# of merge attempts" in r.stdout
    score = open(os.path.join(ws, "LATEST", "results.score.txt")).read()
    vals = dict(ln.split(": ") for ln in score.strip().splitlines())
    assert 0.5 <= float(vals["Purity"]) <= 1.0


@pytest.mark.gpu
def test_triadic_end_to_end(tmp_path):
    """`-a triadic` (np_main.cpp:447-455): the triadic split-merge update through the MCMC driver."""
    ws = str(tmp_path / "ws") + "/"
    r = run(["-d", DATA, "-a", "triadic", "-T", "200", "-c", "clustering", "-s", "5", "-w", ws])
    assert r.returncode == 0, r.stderr + r.stdout
    assert "split (2 -> 3) attempts" in r.stdout
    score = open(os.path.join(ws, "LATEST", "results.score.txt")).read()
    vals = dict(ln.split(": ") for ln in score.strip().splitlines())
    assert float(vals["Purity"]) > 0.9  # the proper SAMS weights find the two components


@pytest.mark.gpu
@pytest.mark.parametrize("algo,extra", [("algorithm8", []), ("algorithm8", ["-u", "mh_g0"]),
                                        ("algorithm8", ["-C", "1"]), ("jain_neal_split", []), ("triadic", [])])
def test_membertrix_coherent_through_reference_loop(tmp_path, algo, extra):
    """MCMC::run in the reference's structure (np_mcmc.cpp:109-175: relabel every 10 sweeps, update of all
    items, UpdateClusters, considerMaxLikelihood every 5 sweeps on the membertrix) with -V: after every
    population update and every cluster update the host membertrix -- patched from np8_changes -- equals
    np8_get_state, and the host's max-likelihood clone equals the device snapshot.  -j writes one JSON
    line per sweep."""
    import json

    ws = str(tmp_path / "ws") + "/"
    jl = str(tmp_path / "sweeps.jsonl")
    r = run(["-d", DATA, "-a", algo, "-T", "60", "-s", "11", "-V", "-j", jl, "-w", ws] + extra)
    assert r.returncode == 0, r.stderr + r.stdout
    recs = [json.loads(ln) for ln in open(jl)]
    assert [x["sweep"] for x in recs] == list(range(60))
    assert all(x["K"] >= 1 for x in recs) and all("loglik" in x for x in recs[::5])
