"""Measures BASELINE.json's configurations on one MI355X (run on the GPU box from the repo root):
C1 twogaussians T=1000 (GPU synchronous and exact sequential sweeps vs the CPU oracle: purity / RI /
ARI of the max-likelihood labelling over seeds, wall time), C2 and C3 through bench.py, C3 with
N = 8e6 (512 MB, past the 256 MB Infinity Cache) and C3 with the mh_g0 parameter update.
Writes gpurun_out/measure.json."""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def c1(seeds_gpu=20, seeds_seq=3, T=1000, substeps=16):
    import oracle as O
    from noparama_amd import NealAlgorithm8, datasets

    X, lab = datasets.read_data(os.path.join(ROOT, "tests", "golden", "twogaussians.data"))
    rows = {}
    for name, chunk, seeds, S in (("gpu_sync", 0, seeds_gpu, 1), (f"gpu_sync_substeps{substeps}", 0, seeds_gpu, substeps),
                                  ("gpu_sequential", 1, seeds_seq, 1)):
        res, t0 = [], time.perf_counter()
        for s in range(seeds):
            g = NealAlgorithm8(2, seed=s, chunk=chunk, kcap=1024, device=0, substeps=S)
            g.set_data(X)
            g.init_random(20)
            g.sweep(T)
            st = g.state(1)
            m = O.similarity(lab, st["z"])
            res.append((m["purity"], m["rand_index"], m["adjusted_rand_index"], st["K"]))
            g.close()
        el = (time.perf_counter() - t0) / seeds
        a = np.array(res)
        rows[name] = {"seeds": seeds, "purity": a[:, 0].mean(), "rand_index": a[:, 1].mean(),
                      "ari": float(np.nanmean(a[:, 2])), "K": a[:, 3].mean(), "seconds_per_run": el}
    res, t0 = [], time.perf_counter()
    for s in range(seeds_seq):
        c = O.Chain(2, seed=s, chunk=1, kcap=1024)
        c.set_data(X)
        c.init_random(20)
        c.sweep(T)
        st = c.state(1)
        m = O.similarity(lab, st["z"])
        res.append((m["purity"], m["rand_index"], m["adjusted_rand_index"], st["K"]))
    a = np.array(res)
    rows["cpu_oracle_sequential_1core"] = {"seeds": seeds_seq, "purity": a[:, 0].mean(),
                                           "rand_index": a[:, 1].mean(), "ari": float(np.nanmean(a[:, 2])),
                                           "K": a[:, 3].mean(),
                                           "seconds_per_run": (time.perf_counter() - t0) / seeds_seq}
    return rows


def bench(args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                         timeout=900)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    return json.loads(line[-1]) if line else {"error": out.stderr[-2000:]}


def main():
    out = {}
    out["C1"] = c1()
    print(json.dumps(out["C1"]), flush=True)
    out["C2"] = bench(["--config", "C2", "--n", "100000", "--d", "2", "--k", "10", "--cpu-seconds", "8"])
    print(json.dumps(out["C2"]), flush=True)
    out["C3"] = bench(["--cpu-seconds", "12"])
    print(json.dumps(out["C3"]), flush=True)
    out["C3_8e6"] = bench(["--config", "C3-8e6", "--n", "8000000", "--steps", "40", "--cpu-seconds", "0"])
    print(json.dumps(out["C3_8e6"]), flush=True)
    out["C3_mh_g0"] = bench(["--config", "C3-mh_g0", "--param-update", "mh_g0", "--cpu-seconds", "0"])
    print(json.dumps(out["C3_mh_g0"]), flush=True)
    for S, extra in ((8, []), (16, ["--kcap", "1024"])):
        out[f"C3_substeps{S}"] = bench(["--config", f"C3-S{S}", "--substeps", str(S), "--cpu-seconds", "0",
                                        "--cold-sweeps", "0"] + extra)
        print(json.dumps(out[f"C3_substeps{S}"]), flush=True)
    out["C3_rccl_one_rank"] = bench(["--config", "C3-rccl1", "--exchange", "rccl", "--cpu-seconds", "0",
                                     "--cold-sweeps", "0"])
    print(json.dumps(out["C3_rccl_one_rank"]), flush=True)
    out["C5"] = bench(["--config", "C5", "--steps", "20", "--warmup", "5", "--cpu-seconds", "0"])
    print(json.dumps(out["C5"]), flush=True)
    out["C5_niw_conjugate"] = bench(["--config", "C5", "--param-update", "niw_conjugate", "--steps", "20",
                                     "--warmup", "5", "--cpu-seconds", "0"])
    print(json.dumps(out["C5_niw_conjugate"]), flush=True)
    out["C3_jain_neal"] = bench(["--sampler", "jain_neal", "--steps", "10", "--warmup", "2", "--cpu-seconds", "0"])
    print(json.dumps(out["C3_jain_neal"]), flush=True)
    out["C3_triadic"] = bench(["--sampler", "triadic", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0"])
    print(json.dumps(out["C3_triadic"]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "measure.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
