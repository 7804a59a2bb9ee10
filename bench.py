"""Benchmark: Gibbs sweeps/sec of the Neal-8 sweep (BASELINE.json metric) on MI355X.

Workload: N = 1e6 items, D = 8, 64 components (sd 0.8, means 6 + U[-20,20]^8),
M = 3, fp64, reference hyper-parameters (alpha 1, mu0 = 6, kappa 1/500, nu 4, Lambda 0.01 I),
warm state (labels = ground truth, cluster parameters = the generating ones), frozen cluster
parameters (the reference's effective behaviour).  One step = one full sweep:
N point updates (np8_assign) + cluster bookkeeping (np8_finalize) + the max-likelihood check every
5th sweep, exactly as np8_sweep runs it.  Inputs are resident in HBM before the timed region.

--config C5 (BASELINE.json configs[4]): N = 1e6, D = 64, 256 components (sd 1,
means 6 + U[-5,5]^64), a proper Normal-Inverse-Wishart prior (mu0 = 6, kappa0 = 0.01, nu0 = D + 2,
Psi0 = I, so E[Sigma] = I), items in fp32 and the cluster likelihoods on the fp32 matrix cores
(np8_assign_wide); roofline against the fp32 MFMA peak.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): the N items are
sharded contiguously over ranks (strong scaling, total N fixed as in config C4); one RCCL
all-gather of the exchange record per sweep.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (= FP64 matrix) peak, vendor spec
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X FP32 matrix peak (MI355X_MICROARCH.md: 155 measured)
HBM_PEAK_GBS = 8000.0
# committed rocprofv3 PMC summaries of the assign kernels (HBM bytes per launch, tools/prof*.sh)
C3_TRAFFIC = "traffic_r06_final_c3.json"
C5_TRAFFIC = "traffic_r06_final_c5.json"
C5_CONJ_TRAFFIC = "traffic_r06_final_c5conj.json"  # PMC pass of the niw_conjugate C5 sweep (its assign reads more candidate rows than the frozen one)
MIXED_TRAFFIC = "traffic_r06_final_mixed.json"  # PMC pass of the mixed regime (tools/prof_mixed.sh, tools/summarize_profile.py)


def binding_roof(exec_flops, abytes, ms, peak_tflops, kname):
    """The roof that binds the kernel as it runs: its executed flops (device counters, after
    exact pruning) against the compute peak, or its algorithmic bytes (item row + label per item) against
    HBM -- whichever fraction is larger.  Without executed counts the HBM roof is reported."""
    hbm_gbs = abytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    exec_tf = exec_flops / (ms * 1e-3) / 1e12 if (exec_flops is not None and ms > 0) else None
    if exec_tf is not None and exec_tf / peak_tflops > hbm_gbs / HBM_PEAK_GBS:
        return {"bound": "mfma", "achieved": exec_tf, "peak": peak_tflops, "unit": "TFLOP/s",
                "frac": exec_tf / peak_tflops,
                "note": f"kernel {kname}: executed flops (device counters, after exact pruning) / launch time"}
    return {"bound": "hbm", "achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_gbs / HBM_PEAK_GBS,
            "algorithmic_bytes_per_launch": abytes,
            "note": f"kernel {kname}: algorithmic bytes (item row + label per item) / launch time; the "
                    "executed flops after exact pruning are a smaller fraction of the compute peak"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=None, help="default: 8 (C3) / 64 (C5)")
    ap.add_argument("--k", type=int, default=None, help="default: 64 (C3) / 256 (C5)")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--kcap", type=int, default=0, help="cluster capacity (0: the library default)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "rccl"],
                    help="rccl: with one GPU too, exchange the step records through a one-rank RCCL communicator "
                         "(the multi-GPU code path, collectives captured in the sweep graph)")
    ap.add_argument("--substeps", type=int, default=1,
                    help="the data-parallel sweep as S synchronous sub-steps (np8_config.substeps)")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: --n items PER RANK (total n x ranks); value = whole-job item updates/s / n, "
                         "i.e. sweeps/s of an n-item data set (C4 as written is strong: total n fixed)")
    ap.add_argument("--config", default="C3", help="config tag for the JSON line (BASELINE.json configs)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--cold-sweeps", type=int, default=20,
                    help="cold leg: sweeps from the reference's initialisation (init_random(20)), 0 = skip")
    ap.add_argument("--no-c5", dest="c5_sub", action="store_false",
                    help="skip the C5 sub-record of the default (C3) run")
    ap.add_argument("--traffic-json", default=None,
                    help="HBM bytes per assign launch from the committed PMC profile of this config")
    ap.add_argument("--sampler", default="neal8", choices=["neal8", "jain_neal", "triadic"],
                    help="jain_neal / triadic: split-merge sweeps (np8_sm_sweep / np8_tri_sweep, one rank) "
                         "instead of the Gibbs sweep")
    ap.add_argument("--param-update", default="frozen", choices=["frozen", "mh_g0", "niw_conjugate"],
                    help="cluster-parameter update after every sweep (frozen = the reference's effective one)")
    a = ap.parse_args()
    c5 = a.config.upper() == "C5"
    a.d = a.d if a.d is not None else (64 if c5 else 8)
    a.k = a.k if a.k is not None else (256 if c5 else 64)
    if a.traffic_json is None:
        name = (C5_CONJ_TRAFFIC if a.param_update == "niw_conjugate" else C5_TRAFFIC) if c5 else C3_TRAFFIC
        a.traffic_json = os.path.join(ROOT, "profiles", name) if name else None
    return a


def n_label(n):
    """1e6 for powers of ten (BASELINE.json's spelling), the plain count otherwise (125000, not '1e5')."""
    e = len(str(n)) - 1
    return f"1e{e}" if n == 10 ** e else str(n)


def workload(args):
    """Data, warm state and sampler options of the configuration."""
    from noparama_amd import datasets

    N, D, K = args.n, args.d, args.k
    if args.config.upper() == "C5":
        X, z, mu, sig = datasets.mixture(N, D, K, 1.0, 5.0, seed=args.seed)
        opts = dict(prior="niw", contraction="f32", kcap=512, mu0=np.full(D, 6.0), kappa=0.01, nu=D + 2.0,
                    Lambda=np.eye(D))
        return X, z, mu, sig, opts
    s, r = (0.3, 15.0) if D == 2 else (0.8, 20.0)
    X, z, mu, sig = datasets.mixture(N, D, K, s, r, seed=args.seed)
    opts = {"kcap": args.kcap} if args.kcap else {}
    if args.substeps > 1:
        opts["substeps"] = args.substeps
    return X, z, mu, sig, opts


def main():
    args = parse()
    if args.sampler in ("jain_neal", "triadic"):
        return main_sm(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = max(world, 1)

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")  # host barrier + timing max; the sweep itself uses RCCL
    # one GPU per rank on the scaling node; rehearsals with more ranks than GPUs share devices
    local_rank = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local_rank)

    from noparama_amd import NealAlgorithm8, comm_unique_id

    n_rank = args.n
    if args.weak:  # every rank keeps n items: the data set grows with the ranks
        args.n = n_rank * world
    N, D, K = args.n, args.d, args.k
    X, z, mu, sig, opts = workload(args)
    wide = opts.get("contraction") == "f32"
    lo = (N * rank) // world
    hi = (N * (rank + 1)) // world

    smp = NealAlgorithm8(D, seed=args.seed, device=local_rank, param_update=args.param_update, **opts)
    transport = "local"
    if world > 1:
        from noparama_amd import NP8Error

        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        # the multi-GPU configuration is the RCCL-over-xGMI exchange: with one GPU per rank, an RCCL failure
        # is an error, not a silent fall-back.  Only rehearsals with more ranks than GPUs (RCCL refuses
        # two ranks on one device) move the same record over gloo, and say so in "exchange".
        rehearsal = world > torch.cuda.device_count()
        try:
            smp.comm_init(uid[0], rank, world)
            ok = True
        except NP8Error as e:
            if not rehearsal:
                raise
            print(f"rank {rank}: RCCL unavailable ({e}); rehearsal exchanging records over gloo", file=sys.stderr)
            ok = False
        flags = [None] * world
        dist.all_gather_object(flags, ok)
        transport = "rccl" if all(flags) else "gloo"
        if transport == "gloo":
            smp.close()
            smp = NealAlgorithm8(D, seed=args.seed, device=local_rank, param_update=args.param_update, **opts)
            smp.comm_init(None, rank, world)
    if world == 1 and args.exchange == "rccl":
        smp.comm_init(comm_unique_id(), 0, 1)
        transport = "rccl"
    smp.set_data(X[lo:hi], offset=lo, n_global=N)
    if transport == "gloo":
        smp.set_state(z[lo:hi], mu, sig, counts=np.bincount(z, minlength=mu.shape[0]))
    else:
        smp.set_state(z[lo:hi], mu, sig)

    def sweeps(n, sync=True):
        if transport != "gloo":
            smp.sweep(n, sync=sync)
            return
        for _ in range(n):  # fallback transport: the exchange record through host memory
            for _ in range(smp.substeps):  # one record exchange per synchronous sub-step, then the sweep's end
                rec = torch.from_numpy(smp.step_local())
                out = [torch.zeros_like(rec) for _ in range(world)]
                dist.all_gather(out, rec)
                smp.step_merge(np.concatenate([o.numpy() for o in out]), world)
            if args.param_update == "frozen":
                smp.end_sweep()
            else:  # the per-cluster statistics summed over ranks on the host transport
                st = torch.from_numpy(smp.param_stats_local())
                dist.all_reduce(st)
                smp.end_sweep_stats(st.numpy())

    m = measure(smp, sweeps, args.steps, args.warmup, transport != "gloo", dist, torch, hi - lo, D, wide,
                max(args.substeps, 1), args.traffic_json)
    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            cpu = cpu_baseline(X, z, mu, sig, D, args.seed, args.cpu_seconds, opts)
        out = {
            "metric": f"Gibbs sweeps/sec (Neal-8, N={n_label(n_rank if args.weak else N)} D={D})",
            "value": args.steps / m["dt"] * (N / n_rank if args.weak else 1.0),
            "unit": "sweeps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": m["dt"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "f32-mfma contraction, f64 draws" if wide else "f64",
            "data": "synthetic",
            "config": {
                "workload": f"{args.config}: N={N} D={D} K~{K} M=3 mixture, warm state (theta = the generating "
                            "parameters, z = the ground truth), "
                            + ("NIW prior, fp32 items + fp32 MFMA contraction, " if wide else "")
                            + {"frozen": "frozen cluster parameters",
                               "mh_g0": "mh_g0 cluster-parameter update (20 MH steps/cluster/sweep)",
                               "niw_conjugate": "niw_conjugate cluster-parameter update"}[args.param_update],
                "N": N, "D": D, "K_final": m["K_final"], "parallelism": f"data-sharded x{world}",
                "substeps": args.substeps,
                "exchange": transport,
                "weak": ({"items_per_rank": n_rank, "items_total": N, "data_sweeps_per_s": args.steps / m["dt"],
                          "value": "whole-job item updates per second / items_per_rank"} if args.weak else None),
                "param_update": args.param_update,
                "params_ms_per_timed_sweep": m["params_ms"],
                "sweep_graphs": os.environ.get("NP8_NO_GRAPH") is None,
            },
            "roofline": m["roofline"],
            "cpu_baseline": cpu,
        }
        if world == 1 and not wide and args.cold_sweeps > 0:
            smp.close()
            out["cold_start"] = cold_start(args, X, z, D, opts, local_rank, torch)
            out["survey_state"] = survey_state(args, X, z, D, opts, local_rank, torch)
        if world == 1 and not wide and args.c5_sub:
            smp.close()
            del X, z, mu, sig
            out["c5"] = c5_record(args, local_rank, torch)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def measure(smp, sweeps, steps, warmup, graphs, dist, torch, n_loc, D, wide, S, traffic_json):
    """The timed region (barrier + synchronize on both sides, max over ranks) and the roofline of the
    dominant kernel.  The timed region replays the sweeps with device timing off (no event nodes in the graph,
    no event bookkeeping on the host) and checks the chain's error flags (np8_sync, a device-to-host read) after
    the clock stops; the assign launch time comes from a separate replay of one 20-sweep graph with every
    assign bracketed by event nodes (NP8_TIMING_ALL_ASSIGNS; VERDICT r2: not a single sample)."""
    smp.set_timing(False)
    sweeps(warmup)  # includes np8_sync
    if graphs:
        smp.prepare_sweeps(steps)  # captures and uploads the graph of the timed sweeps (outside the clock)
    torch.cuda.synchronize()
    st0 = smp.stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sweeps(steps, sync=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    smp.sync()  # (the chain's error flags: raises if a kernel reported one)
    if os.environ.get("NP8_BENCH_PHASES"):  # (experiment: host time to submit, and the whole region)
        print(f"timed region: submit {(t1 - t0) * 1e6:.1f} us, total {dt * 1e6:.1f} us", file=sys.stderr)
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    smp.set_timing(True)
    st1 = smp.stats()
    Kfinal = st1["K"]
    n_in = st1["n_timed_assign"] - st0["n_timed_assign"]  # (0: no timing in the timed region)
    ms_in = (st1["ms_assign"] - st0["ms_assign"]) / n_in if n_in > 0 else None
    ms_assign, n_launch, src = ms_in or 0.0, n_in, "timed region"
    if graphs or ms_in is None:  # every assign of one 20-sweep replay (after the timed region, untimed for the headline)
        smp.set_timing(True, all_assigns=True)
        a0 = smp.stats()
        sweeps(20)
        a1 = smp.stats()
        smp.set_timing(True)
        if a1["n_timed_assign"] > a0["n_timed_assign"]:
            n_launch = a1["n_timed_assign"] - a0["n_timed_assign"]
            ms_assign = (a1["ms_assign"] - a0["ms_assign"]) / n_launch
            src = "every assign launch of one 20-sweep graph replay after the timed region"
    # executed-work counters over separate (untimed) sweeps: they add scalar loads and atomics per wave
    cnt_sweeps = 20 if graphs else 0
    if cnt_sweeps:
        smp.set_timing(True, counters=True)
        sc0 = smp.stats()
        sweeps(cnt_sweeps)
        sc1 = smp.stats()
        smp.set_timing(True)
    Kc = Kfinal + smp.M
    # items of one assign launch: with S sub-steps a sweep makes S launches over ~N/S items each (ADVICE r2:
    # per-launch bytes/flops, not per-sweep)
    n_items = n_loc / S
    # N (K+M) (D^2 + 2D + 4) for the fp64 table form (packed P: D(D+1)/2 multiply-adds
    # plus d = x - mu and the weight).  Wide path: the triangular factor form y = A (x - mu), |y|^2:
    # D subtractions + D(D+1)/2 multiply-adds + D squares-and-adds = D^2 + 4D per item and candidate
    # (SURVEY.md's 2D^2 + 4D counts a full D x D contraction, which the kernel does not perform).
    flops = float(n_items) * Kc * ((D * D + 4 * D) if wide else (D * D + 2 * D + 4))
    # what the matrix cores execute on the wide path: 16-row tiles of the triangular A, 2 flops per MAC
    mac_tiles = sum(16 * (D - 16 * t) for t in range(D // 16))
    mfma_flops = float(n_items) * Kc * 2 * mac_tiles if wide else None
    achieved = flops / (ms_assign * 1e-3) / 1e12 if ms_assign > 0 else 0.0
    peak = FP32_MFMA_PEAK_TFLOPS if wide else FP64_PEAK_TFLOPS
    xbytes = 4 * D if wide else 8 * D
    # executed work: quadratic forms the kernel evaluated (device counters), at their real cost
    # (isotropic rows: D subtractions + D multiply-adds + scale, weight = 3D + 3 flops)
    nq = (sc1["n_quad"] - sc0["n_quad"]) / cnt_sweeps / S if cnt_sweeps else 0.0  # per launch
    nq_iso = (sc1["n_quad_iso"] - sc0["n_quad_iso"]) / cnt_sweeps / S if cnt_sweeps else 0.0
    if wide:  # item-row contractions on the matrix cores (pruned rows skipped), at the MACs of the 16-row tiles
        exec_flops = nq * 2 * mac_tiles if cnt_sweeps else None
    else:
        exec_flops = ((nq - nq_iso) * (D * D + 2 * D + 4) + nq_iso * (3 * D + 3)) if cnt_sweeps else None
    traffic = traffic_src = None
    if traffic_json and os.path.exists(traffic_json):
        try:
            tj = json.load(open(traffic_json))
            traffic = tj.get("assign_bytes_per_launch")
            traffic_src = f"{os.path.relpath(traffic_json, ROOT)} (rocprofv3 PMC pass, {tj.get('commit', 'commit n/a')})"
        except Exception:
            traffic = None
    abytes = float(n_items) * (xbytes + 8)
    binding = binding_roof(exec_flops, abytes, ms_assign, peak, "np8_assign_wide" if wide else "np8_assign")
    roof = {
        **binding,
        "traffic": traffic,
        "traffic_over_algorithmic": (traffic / abytes) if traffic else None,
        # the unpruned table form's flops over the launch time: an algorithmic-equivalent rate, not
        # work the kernel performs (exact pruning skips almost every candidate row), so it can pass 1
        "algorithmic_equivalent": {"achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak},
        "assign_ms_per_launch": ms_assign,
        "assign_ms_source": src,
        "assign_launches_timed": n_launch,
        "assign_ms_timed_region": ms_in,
        "assign_launches_timed_region": n_in,
        # wide path: the matrix-core work of every row, as if none were pruned
        "mfma_unpruned_tflops": (mfma_flops / (ms_assign * 1e-3) / 1e12) if (wide and ms_assign > 0) else None,
        "algorithmic_flops_per_launch": flops,
        "traffic_source": traffic_src,
        "executed": None if not cnt_sweeps else {
            "note": ("what np8_assign_wide executed: item-row contractions on the matrix cores after exact "
                     "candidate pruning (device counters over 20 untimed sweeps), at the MACs of the 16-row "
                     "tiles, over the launch time" if wide else
                     "what np8_assign executed: quadratic forms after exact candidate pruning "
                     "(device counters over 20 untimed sweeps after the timed ones), at their real "
                     "cost, over the launch time; the M auxiliary G0 draws per item (Philox, "
                     "Box-Muller, chi^2 logs) are not flops of this count"),
            "quad_forms_per_item": nq / max(n_items, 1),
            "aux_exact_per_item": (sc1["aux_exact_lanes"] - sc0["aux_exact_lanes"]) / cnt_sweeps / max(n_loc, 1),
            "aux_exact_wave_frac": (sc1["aux_exact_waves"] - sc0["aux_exact_waves"]) / cnt_sweeps
            / max(((n_loc + 63) // 64) * smp.M, 1),
            "aux_screen_violations": sc1["screen_violations"] - sc0["screen_violations"],
            # how the candidate walk went (DESIGN.md 4 "Candidate pruning"): lanes on the whole table, waves
            # that paid the table loop for at least one lane, waves of more own rows than the list walk takes
            "full_walk_lane_frac": (sc1["full_walk_lanes"] - sc0["full_walk_lanes"]) / cnt_sweeps / max(n_loc, 1),
            "full_walk_wave_frac": (sc1["full_walk_waves"] - sc0["full_walk_waves"]) / cnt_sweeps
            / max((n_loc + 63) // 64, 1),
            "many_group_wave_frac": (sc1["many_group_waves"] - sc0["many_group_waves"]) / cnt_sweeps
            / max((n_loc + 63) // 64, 1),
            "list_entries_per_item": (sc1["list_entries"] - sc0["list_entries"]) / cnt_sweeps / max(n_loc, 1),
            "pick_evals_per_item": (sc1["pick_evals"] - sc0["pick_evals"]) / cnt_sweeps / max(n_loc, 1),
            "iso_fraction": nq_iso / max(nq, 1),
            "tflops": exec_flops / (ms_assign * 1e-3) / 1e12 if ms_assign > 0 else None,
            "frac_of_peak": exec_flops / (ms_assign * 1e-3) / 1e12 / peak if ms_assign > 0 else None,
        },
        "hbm_frac_algorithmic": abytes / (ms_assign * 1e-3) / 1e9 / HBM_PEAK_GBS if ms_assign > 0 else None,
    }
    params_ms = ((st1["ms_params"] - st0["ms_params"]) / (st1["n_timed_params"] - st0["n_timed_params"])
                 if st1["n_timed_params"] > st0["n_timed_params"] else None)
    return {"dt": dt, "K_final": Kfinal, "roofline": roof, "params_ms": params_ms}


def cold_start(args, X, labels, D, opts, device, torch):
    """The reference's flow from its initialisation (np_mcmc.cpp:49-92: K = 20 random G0 clusters, uniform
    labels), on the same data:
      * sweeps 0 .. cold_sweeps-1 one by one (K read back after each: one host round trip per sweep), with
        the new-cluster requests accepted and deferred;
      * "mixed": sweeps 50 .. 149 timed as the warm leg is (graph replay, no per-sweep sync), with the
        assign kernel's roofline: the regime the reference's own start reaches;
      * "quality": at sweep 300, K and the purity / ARI of the max-likelihood and last labellings against
        the generator's labels (noparama_amd.metrics = clustering_performance.cpp:38-82), for this sampler
        and for the same chain in 16 synchronous sub-steps."""
    from noparama_amd import NealAlgorithm8, metrics

    smp = NealAlgorithm8(D, seed=args.seed + 1, device=device, param_update=args.param_update, **opts)
    smp.set_data(X)
    smp.init_random(20)
    per, Ks, acc, dfr = [], [], [], []
    s0 = smp.stats()
    for _ in range(args.cold_sweeps):
        t0 = time.perf_counter()
        smp.sweep(1)  # synchronous
        per.append((time.perf_counter() - t0) * 1e3)
        s1 = smp.stats()
        Ks.append(s1["K"])
        acc.append(s1["new_clusters"] - s0["new_clusters"])
        dfr.append(s1["rejected_requests"] - s0["rejected_requests"])
        s0 = s1
    tot = sum(per) * 1e-3
    out = {"sweeps": args.cold_sweeps, "value": args.cold_sweeps / tot, "unit": "sweeps/s",
           "ms_per_sweep": [round(v, 3) for v in per], "K_per_sweep": Ks,
           "new_clusters_per_sweep": acc, "deferred_requests_per_sweep": dfr,
           "req_max": smp.req_max, "init": "init_random(20) (np_mcmc.cpp:49-92)"}
    if args.cold_sweeps < 50:
        smp.sweep(50 - args.cold_sweeps)
    K50 = smp.K
    m = measure(smp, lambda n, sync=True: smp.sweep(n, sync=sync), 100, 0, True, None, torch, X.shape[0], D,
                False, 1, os.path.join(ROOT, "profiles", MIXED_TRAFFIC))
    out["mixed"] = {"sweeps": "50..149 (then 20 + 20 untimed for the launch times and counters)",
                    "value": 100 / m["dt"], "unit": "sweeps/s", "ms_per_sweep": m["dt"] / 100 * 1e3,
                    "K_at_50": K50, "K_final": m["K_final"], "roofline": m["roofline"]}
    smp.sweep(300 - 190)
    out["quality"] = {"sweeps": 300, "this_sampler": chain_quality(smp, labels),
                      "substeps_16": None}
    smp.close()
    s16 = NealAlgorithm8(D, seed=args.seed + 1, device=device, param_update=args.param_update, substeps=16,
                         kcap=1024)
    s16.set_data(X)
    s16.init_random(20)
    s16.sweep(300)
    out["quality"]["substeps_16"] = chain_quality(s16, labels)
    out["quality"]["note"] = ("S = 16 runs with kcap 1024 (the sub-step sort holds substeps x kcap <= 16384 bins); "
                              "tolerance SURVEY.md 8(d): |d purity| <= 0.02, |d ARI| <= 0.05")
    s16.close()
    return out


def survey_state(args, X, labels, D, opts, device, torch):
    """SURVEY.md 8(d)'s C3 start: z = the generator's labels, theta_k = G0 draws (64 of them, np8_init_random's),
    frozen parameters; sweeps 0 .. 9 one by one, then sweeps 10 .. 109 timed as the warm leg is (graph replays), with
    K per sweep over the eager ones and at the end.  Unlike the headline's warm state (theta = the generating
    parameters, a fixed point of the chain) the items leave their badly placed clusters: the regime of the mixed leg."""
    from noparama_amd import NealAlgorithm8

    smp = NealAlgorithm8(D, seed=args.seed + 2, device=device, param_update=args.param_update, **opts)
    smp.set_data(X)
    smp.init_random(int(labels.max()) + 1)  # (the G0 draws; its uniform labels are replaced next)
    st = smp.state(params=True)
    smp.set_state(labels.astype(np.int32), st["mu"], st["sigma"])
    Ks, per = [], []
    for _ in range(10):
        t0 = time.perf_counter()
        smp.sweep(1)
        per.append((time.perf_counter() - t0) * 1e3)
        Ks.append(smp.K)
    m = measure(smp, lambda n, sync=True: smp.sweep(n, sync=sync), 100, 0, True, None, torch, X.shape[0], D,
                False, 1, os.path.join(ROOT, "profiles", MIXED_TRAFFIC))
    out = {"start": "z = generator labels, theta_k = 64 G0 draws (SURVEY.md 8(d) C3 input)",
           "eager_ms_per_sweep_0_9": [round(v, 3) for v in per], "K_per_sweep_0_9": Ks,
           "sweeps": "10..109 (graph replays)", "value": 100 / m["dt"], "unit": "sweeps/s",
           "ms_per_sweep": m["dt"] / 100 * 1e3, "K_final": m["K_final"],
           "assign_ms_per_launch": m["roofline"].get("assign_ms_per_launch")}
    smp.close()
    return out


def chain_quality(smp, labels):
    from noparama_amd import metrics

    res = {}
    for which, tag in ((1, "maxlik"), (0, "last")):
        st = smp.state(which=which, params=False)
        mm = metrics.similarity(labels, st["z"])
        res[tag] = {"K": st["K"], "purity": mm["purity"], "rand_index": mm["rand_index"],
                    "ari": mm["adjusted_rand_index"]}
    return res


def c5_traffic(pu):
    """The PMC traffic file of the C5 sweep with cluster-parameter update pu (None: not profiled)."""
    name = C5_TRAFFIC if pu == "frozen" else C5_CONJ_TRAFFIC
    return os.path.join(ROOT, "profiles", name) if name else None


def c5_record(args, device, torch):
    """Config C5 (N = 1e6, D = 64, K = 256, NIW prior, fp32 MFMA contraction) timed inside the default run
    (VERDICT r2 #7): frozen and niw_conjugate sweeps/s with the roofline of np8_assign_wide."""
    import argparse as _ap

    from noparama_amd import NealAlgorithm8

    a = _ap.Namespace(**{**vars(args), "config": "C5", "d": 64, "k": 256, "substeps": 1})
    X, z, mu, sig, opts = workload(a)
    out = {"workload": "C5: N=1000000 D=64 K~256 M=3 mixture, warm state (theta = the generating parameters, "
                       "z = the ground truth), NIW prior, fp32 items + fp32 MFMA contraction"}
    for pu, steps in (("frozen", 40), ("niw_conjugate", 20)):
        smp = NealAlgorithm8(64, seed=args.seed, device=device, param_update=pu, **opts)
        smp.set_data(X)
        smp.set_state(z, mu, sig)
        m = measure(smp, lambda n, sync=True: smp.sweep(n, sync=sync), steps, 5, True, None, torch, X.shape[0],
                    64, True, 1, c5_traffic(pu))
        out[pu] = {"value": steps / m["dt"], "unit": "sweeps/s", "steps": steps, "ms_per_step": m["dt"] / steps * 1e3,
                   "K_final": m["K_final"], "params_ms_per_timed_sweep": m["params_ms"], "roofline": m["roofline"]}
        smp.close()
    return out


def main_sm(args):
    """Split-merge sweeps/sec (np8_sm_sweep: N Jain-Neal attempts + the end-of-sweep step per sweep) on
    the C2/C3 workload and warm state, one GPU.  Roofline of the state rebuild (np8_sm_own/np8_sm_cross:
    N (K + 1) fp64 likelihoods per launch, the sampler's compute-bound part); the attempt batches are
    latency-bound (the sequential SAMS allocation of a split, one lane per attempt)."""
    import torch

    from noparama_amd import JainNealAlgorithm, TriadicAlgorithm

    tri = args.sampler == "triadic"
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--sampler jain_neal/triadic runs on one rank")
    torch.cuda.set_device(0)
    N, D, K = args.n, args.d, args.k
    X, z, mu, sig, opts = workload(args)
    if any(k != "kcap" for k in opts):
        raise SystemExit("--sampler jain_neal/triadic: reference prior, fp64 configurations only")
    cls = TriadicAlgorithm if tri else JainNealAlgorithm
    smp = cls(D, seed=args.seed, device=0, param_update=args.param_update, kcap=opts.get("kcap", max(256, 4 * K)))
    outcomes = smp.tri_stats if tri else smp.sm_stats
    smp.set_data(X)
    smp.set_state(z, mu, sig)
    smp.sweep(args.warmup)
    smp.set_timing(True)
    st0, o0 = smp.stats(), outcomes()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    smp.sweep(args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st1, o1 = smp.stats(), outcomes()
    d = {k: o1[k] - o0[k] for k in o1}
    nm = st1["n_timed_sm_members"] - st0["n_timed_sm_members"]
    ne = st1["n_timed_sm_eval"] - st0["n_timed_sm_eval"]
    ms_m = (st1["ms_sm_members"] - st0["ms_sm_members"]) / max(nm, 1)
    ms_e = (st1["ms_sm_eval"] - st0["ms_sm_eval"]) / max(ne, 1)
    Kf = st1["K"]
    flops = float(N) * (Kf + 1) * (D * D + 2 * D + 4)  # cross matrix + own likelihoods per rebuild
    achieved = flops / (ms_m * 1e-3) / 1e12 if ms_m > 0 else 0.0
    cpu = cpu_baseline_sm(X, z, mu, sig, D, args.seed, args.cpu_seconds, tri) if args.cpu_seconds > 0 else None
    name = "triadic" if tri else "Jain-Neal"
    out = {
        "metric": f"split-merge sweeps/sec ({name}, N={n_label(N)} attempts/sweep, D={D})",
        "value": args.steps / dt,
        "unit": "sweeps/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "replicas only",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"{args.config}: N={N} D={D} K~{K} mixture, warm state (theta = the generating parameters, "
                        f"z = the ground truth), {name} split-merge "
                        f"(sams_prior, reference rules), {args.param_update} cluster parameters",
            "N": N, "D": D, "K_final": Kf, "attempt_outcomes": d,
            "state_rebuilds": nm, "attempt_batches": ne,
            "ms_per_rebuild": ms_m, "ms_per_batch": ms_e,
        },
        "roofline": {
            "bound": "mfma",
            "note": "fp64 compute roof of the state rebuild (np8_sm_own + np8_sm_cross); attempt batches "
                    "(np8_sm_eval) are latency-bound by the sequential SAMS allocation",
            "achieved": achieved,
            "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS,
            "traffic": None,
            "algorithmic_flops_per_launch": flops,
        },
        "cpu_baseline": cpu,
    }
    print(json.dumps(out))


def cpu_baseline_sm(X, z, mu, sig, D, seed, budget_s, tri=False):
    """The oracle's sequential split-merge attempts (np8o_sm_attempts / np8o_tri_attempts, one core) on
    the same data and state: the first attempts of one sweep, doubling until the budget, extrapolated
    to N attempts."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test infrastructure: timed as the CPU baseline only

    c = O.Chain(D, seed=seed, kcap=4096)
    c.set_data(X)
    c.set_state(z, mu, sig)
    N = X.shape[0]
    done, a, t0 = 0, 64, time.perf_counter()
    while time.perf_counter() - t0 < budget_s and done < N:
        b = min(N, done + a)
        (c.tri_attempts if tri else c.sm_attempts)(done, b)
        done, a = b, 2 * a
    el = time.perf_counter() - t0
    return {"value": done / el / N, "unit": "sweeps/s", "cores": 1, "kind": "port",
            "sample": f"the first {done} of the N={N} split-merge attempts of one sweep in {el:.1f}s on 1 core, "
                      f"extrapolated"}


def cpu_baseline(X, z, mu, sig, D, seed, budget_s, opts):
    """The oracle's sequential sweep (chunk = 1: the reference's algorithm, single thread) on the same
    workload and state, timed on a bounded prefix of one sweep, extrapolated to sweeps/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test infrastructure: timed as the CPU baseline only

    kc = opts.get("kcap", 2048)
    # the reference computes in fp64: the CPU legs use the fp64 table form (contraction f64)
    okw = {k: v for k, v in opts.items() if k not in ("kcap", "contraction")}
    c = O.Chain(D, seed=seed, chunk=1, kcap=kc, **okw)
    c.set_data(X)
    c.set_state(z, mu, sig)
    done, t0 = 0, time.perf_counter()
    batch = 10000 if D <= 16 else 64
    while time.perf_counter() - t0 < budget_s and done < X.shape[0]:
        c.update_points(np.arange(done, min(done + batch, X.shape[0]), dtype=np.int64))
        done = min(done + batch, X.shape[0])
    el = time.perf_counter() - t0
    rate = done / el
    out = {
        "value": rate / X.shape[0],
        "unit": "sweeps/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{done} sequential point-updates (chunk=1) of one N={X.shape[0]} sweep in {el:.1f}s "
                  f"on 1 core, extrapolated: {rate:.0f} point-updates/s",
    }
    # cpu_par: the same synchronous sweep the GPU runs, OpenMP over the items, on the
    # host cores this process may use (the box's share, not the whole machine)
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    O.set_threads(threads)
    cp = O.Chain(D, seed=seed, chunk=0, kcap=kc, **okw)
    cp.set_data(X)
    cp.set_state(z, mu, sig)
    N = X.shape[0]
    t0 = time.perf_counter()
    cp.assign_range(0, min(N, 2048), req_cap=4096)  # probe: how many items fit the budget
    el = time.perf_counter() - t0
    if el * N / min(N, 2048) < budget_s:  # whole synchronous sweeps
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s / 2 or n == 0:
            cp.sweep(1)
            n += 1
        el2 = time.perf_counter() - t0
        par = {"value": n / el2, "sample": f"{n} full synchronous sweeps (chunk=N, the GPU's algorithm) in "
                                           f"{el2:.1f}s on {threads} threads"}
    else:  # a prefix of one synchronous sweep's assignments, extrapolated
        m = int(min(N, max(2048, 2048 * (budget_s / 2) / max(el, 1e-6))))
        t0 = time.perf_counter()
        cp.assign_range(0, m, req_cap=65536)
        el2 = time.perf_counter() - t0
        par = {"value": m / el2 / N, "sample": f"{m} of the {N} point updates of one synchronous sweep "
                                                f"(chunk=N, the GPU's algorithm) in {el2:.1f}s on {threads} "
                                                f"threads, extrapolated"}
    O.set_threads(1)
    out["parallel"] = {"value": par["value"], "unit": "sweeps/s", "cores": threads, "kind": "port",
                       "sample": par["sample"]}
    return out


if __name__ == "__main__":
    main()
