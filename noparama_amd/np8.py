"""ctypes binding of libnp8.so (include/np8.h) and the host-side mirror of noparama's sampler API.

`NealAlgorithm8` mirrors the reference plug-in (include/np_neal_algorithm8.h:52-73 on
include/np_update_cluster_population.h:13-44): the same constructor parameters (likelihood =
multivariate normal of dimension D, nonparametrics = DP(alpha) with the NIW-like base measure of
src/np_main.cpp:365-372) and `update(membertrix, data_ids)`/`printStatistics()`.  Sweep-granular
entry points (`sweep`) are the MI355X path; `update` with a single id is the reference's exact
per-point granularity.  There is no CPU fallback: if the HIP library is missing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NP8_LIB_OVERRIDE") or os.path.join(_HERE, "lib", "libnp8.so")  # override: A/B experiments
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "np8.h")

NP8_OK = 0
NP8_ERR_ARG = -1
NP8_ERR_SIGMA = -2
NP8_ERR_RANGE = -3
NP8_ERR_CAPACITY = -4
NP8_ERR_STATE = -5
NP8_ERR_HIP = -6
NP8_ERR_COMM = -7
NP8_REQ_MAX = 4096
NP8_REQ_DEFAULT = 1024
NP8_SUBSTEPS_AUTO = -1  # np8_config.substeps: chosen by np8_set_data from n_global (include/np8.h)

_ERRNAMES = {
    NP8_ERR_ARG: "NP8_ERR_ARG",
    NP8_ERR_SIGMA: "NP8_ERR_SIGMA",
    NP8_ERR_RANGE: "NP8_ERR_RANGE",
    NP8_ERR_CAPACITY: "NP8_ERR_CAPACITY",
    NP8_ERR_STATE: "NP8_ERR_STATE",
    NP8_ERR_HIP: "NP8_ERR_HIP",
    NP8_ERR_COMM: "NP8_ERR_COMM",
}


class NP8Error(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class _ChangesT(C.Structure):
    _fields_ = [("n_moved", C.c_int64), ("n_created", C.c_int32), ("n_removed", C.c_int32),
                ("n_updated", C.c_int32), ("pad", C.c_int32)]


class _Config(C.Structure):
    _fields_ = [
        ("D", C.c_int32),
        ("M", C.c_int32),
        ("alpha", C.c_double),
        ("mu0", C.POINTER(C.c_double)),
        ("kappa", C.c_double),
        ("nu", C.c_double),
        ("Lambda", C.POINTER(C.c_double)),
        ("seed", C.c_uint64),
        ("kcap", C.c_int32),
        ("chunk", C.c_int64),
        ("device", C.c_int32),
        ("param_update", C.c_int32),
        ("mh_steps", C.c_int32),
        ("prior", C.c_int32),
        ("contraction", C.c_int32),
        ("req_max", C.c_int32),
        ("substeps", C.c_int32),
    ]


PARAM_UPDATE = {"frozen": 0, "mh_g0": 1, "niw_conjugate": 2}  # NP8_PARAM_* (include/np8.h)
PRIOR = {"reference": 0, "niw": 1}  # NP8_PRIOR_*
CONTRACTION = {"f64": 0, "f32": 1}  # NP8_CONTRACT_*: "f32" = the fp32 MFMA wide path (D in {32, 48, 64})


class Stats(C.Structure):
    _fields_ = [
        ("K", C.c_int32),
        ("epoch", C.c_uint32),
        ("new_clusters", C.c_int64),
        ("existing_picks", C.c_int64),
        ("rejected_requests", C.c_int64),
        ("best_loglik", C.c_double),
        ("last_loglik", C.c_double),
        ("ms_assign", C.c_double),
        ("ms_finalize", C.c_double),
        ("ms_loglik", C.c_double),
        ("mh_accepted", C.c_int64),
        ("ms_params", C.c_double),
        ("n_timed_assign", C.c_int64),
        ("n_timed_finalize", C.c_int64),
        ("n_timed_loglik", C.c_int64),
        ("n_timed_params", C.c_int64),
        ("ms_sm_members", C.c_double),
        ("ms_sm_eval", C.c_double),
        ("n_timed_sm_members", C.c_int64),
        ("n_timed_sm_eval", C.c_int64),
        ("n_quad", C.c_int64),
        ("n_quad_iso", C.c_int64),
        ("screen_violations", C.c_int64),
        ("aux_exact_lanes", C.c_int64),
        ("aux_exact_waves", C.c_int64),
        ("full_walk_lanes", C.c_int64),
        ("full_walk_waves", C.c_int64),
        ("many_group_waves", C.c_int64),
        ("list_entries", C.c_int64),
        ("folded_checks", C.c_int64),
        ("tail_list_builds", C.c_int64),
        ("tail_steps", C.c_int64),
        ("pick_evals", C.c_int64),
        ("compact_halts", C.c_int64),
        ("substeps", C.c_int64),
    ]


_lib = None


def header_symbols():
    """Entry points declared in include/np8.h."""
    txt = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char \*)\s*(np8_\w+)\s*\(", txt, re.M)))


def lib():
    """Load the in-tree HIP library.  Raises (no fallback) when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libnp8.so not built ({LIB_PATH}); run __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, d = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    P = C.POINTER
    sig = {
        "np8_create": ([P(vp), P(_Config)], i32),
        "np8_create_sized": ([P(vp), P(_Config), C.c_size_t], i32),
        "np8_destroy": ([vp], i32),
        "np8_last_error": ([vp], C.c_char_p),
        "np8_set_data": ([vp, vp, i64, i32, i64, i64], i32),
        "np8_set_state": ([vp, vp, i32, vp, vp], i32),
        "np8_set_state_counts": ([vp, vp, i32, vp, vp, vp], i32),
        "np8_init_random": ([vp, i32], i32),
        "np8_sweep": ([vp, i32], i32),
        "np8_prepare_sweeps": ([vp, i32], i32),
        "np8_update_points": ([vp, vp, i64], i32),
        "np8_end_sweep": ([vp], i32),
        "np8_population_sweep": ([vp], i32),
        "np8_checkpoint_bytes": ([vp], i64),
        "np8_checkpoint": ([vp, vp, i64], i32),
        "np8_restore": ([vp, vp, i64], i32),
        "np8_check_invariants": ([vp, vp], i32),
        "np8_track_changes": ([vp, i32], i32),
        "np8_changes": ([vp, i64, vp, vp, vp, vp, vp, vp, vp, vp], i32),
        "np8_sync": ([vp], i32),
        "np8_get_state": ([vp, i32, vp, vp, vp, vp, vp], i32),
        "np8_loglik_matrix": ([vp, vp, i64, vp], i32),
        "np8_aux_bounds": ([vp, vp, i64, vp], i32),
        "np8_total_loglik": ([vp, P(d)], i32),
        "np8_pick_batch": ([vp, vp, i32, vp, i64, vp], i32),
        "np8_stats": ([vp, P(Stats)], i32),
        "np8_stats_sized": ([vp, P(Stats), C.c_size_t], i32),
        "np8_set_timing": ([vp, i32], i32),
        "np8_set_stream": ([vp, vp], i32),
        "np8_comm_unique_id": ([vp], i32),
        "np8_comm_init": ([vp, vp, i32, i32], i32),
        "np8_record_bytes": ([vp], i64),
        "np8_step_local": ([vp, vp], i32),
        "np8_step_merge": ([vp, vp, i32], i32),
        "np8_compact_record_bytes": ([vp], i64),
        "np8_step_local_compact": ([vp, vp], i32),
        "np8_step_merge_compact": ([vp, vp, i32, P(i32)], i32),
        "np8_step_resume": ([vp, vp], i32),
        "np8_param_stats_bytes": ([vp], i64),
        "np8_param_stats_local": ([vp, vp], i32),
        "np8_end_sweep_stats": ([vp, vp], i32),
        "np8_sm_sweep": ([vp, i32], i32),
        "np8_sm_stats": ([vp, vp], i32),
        "np8_tri_sweep": ([vp, i32], i32),
        "np8_tri_stats": ([vp, vp], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def comm_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    r = lib().np8_comm_unique_id(buf)
    if r:
        raise NP8Error(r, "ncclGetUniqueId failed")
    return bytes(buf)


class NealAlgorithm8:
    """Neal Algorithm 8 on one MI355X (or one shard of a multi-GPU run).

    Parameters follow the reference wiring (src/np_main.cpp:164,365-372,433-438): D (likelihood
    dimension), M auxiliaries (np_neal_algorithm8.cpp:33), alpha (Suffies_Dirichlet), and the base
    measure mu0, kappa, nu, Lambda.  `chunk` = points per synchronous step (0: whole sweep).
    `param_update`: "frozen" (the reference's effective behaviour), "mh_g0" (UpdateClusters as
    intended: `mh_steps` G0-proposal MH steps per cluster after every sweep, np_update_clusters.cpp) or
    "niw_conjugate" (prior="niw": exact posterior draw per cluster, normalinvwishart.h:66-75).
    `req_max`: new clusters one synchronous step may create (0: NP8_REQ_DEFAULT); requests beyond it
    or beyond the free slots are deferred to the item's next update (lowest scan positions first).
    `prior`: "reference" (the reference's G0 as it draws) or "niw" (a proper Normal-Inverse-Wishart with
    kappa0 = kappa, nu0 = nu >= D + 1, Psi0 = Lambda).  `contraction`: "f64" (any D <= 128; above 16 the
    run-time-D kernels of np8_rt.hip: reference prior, frozen parameters) or "f32" (16 < D <= 80: items in fp32,
    cluster likelihoods on the fp32 matrix cores; config C5).
    `substeps`: the data-parallel sweep (chunk 0) as S synchronous sub-steps over a fixed hash partition of
    the items (DESIGN.md "Sub-steps"); 1 = one step against the sweep-start state; "auto" = 16 sub-steps for
    data sets of at most 8192 items (where one step over-splits), else one (resolved by set_data).
    """

    def __init__(self, D, M=3, alpha=1.0, mu0=None, kappa=1.0 / 500, nu=4.0, Lambda=None, seed=0, kcap=None,
                 chunk=0, device=-1, param_update="frozen", mh_steps=20, prior="reference", contraction="f64",
                 req_max=0, substeps=1):
        if kcap is None:  # the library's default: 512 on the wide path (kcap^2 x D offset table), else 2048
            kcap = 512 if contraction == "f32" else 2048
        self.D, self.M, self.kcap = int(D), int(M), int(kcap)
        self._mu0 = np.ascontiguousarray(np.full(D, 6.0) if mu0 is None else mu0, dtype=np.float64)
        self._Lam = np.ascontiguousarray(0.01 * np.eye(D) if Lambda is None else Lambda, dtype=np.float64)
        cfg = _Config()
        cfg.D, cfg.M, cfg.alpha = self.D, self.M, float(alpha)
        cfg.mu0 = self._mu0.ctypes.data_as(C.POINTER(C.c_double))
        cfg.kappa, cfg.nu = float(kappa), float(nu)
        cfg.Lambda = self._Lam.ctypes.data_as(C.POINTER(C.c_double))
        cfg.seed, cfg.kcap, cfg.chunk, cfg.device = int(seed), int(kcap), int(chunk), int(device)
        if param_update not in PARAM_UPDATE:
            raise ValueError(f"param_update must be one of {sorted(PARAM_UPDATE)}")
        cfg.param_update, cfg.mh_steps = PARAM_UPDATE[param_update], int(mh_steps)
        if prior not in PRIOR:
            raise ValueError(f"prior must be one of {sorted(PRIOR)}")
        cfg.prior = PRIOR[prior]
        if contraction not in CONTRACTION:
            raise ValueError(f"contraction must be one of {sorted(CONTRACTION)}")
        cfg.contraction = CONTRACTION[contraction]
        cfg.req_max = int(req_max)
        self.req_max = int(req_max) or NP8_REQ_DEFAULT
        auto = isinstance(substeps, str)
        if auto and substeps != "auto":
            raise ValueError('substeps must be an int or "auto"')
        cfg.substeps = NP8_SUBSTEPS_AUTO if auto else int(substeps)
        self.substeps = 1 if auto else max(int(substeps), 1)  # ("auto": set_data resolves it)
        self._substeps_auto = auto
        h = C.c_void_p()
        r = lib().np8_create_sized(C.byref(h), C.byref(cfg), C.sizeof(cfg))
        if r:
            raise NP8Error(r, "np8_create failed (unsupported D/M, bad base measure or no HIP device)")
        self._h = h
        self.N = 0
        self._statistics_new = 0

    # -- plumbing ------------------------------------------------------------------------------
    def _check(self, r):
        if r:
            raise NP8Error(r, lib().np8_last_error(self._h).decode())

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            lib().np8_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- state ---------------------------------------------------------------------------------
    def set_data(self, X, offset=0, n_global=None):
        X = np.ascontiguousarray(X, dtype=np.float64)
        if X.ndim != 2 or X.shape[1] != self.D:
            raise ValueError("X must be [n, D]")
        self.N = X.shape[0]
        # np8_set_data drops the device change log: the next patch() reloads the whole state
        self._tracked, self._slot_id = None, {}
        self._check(lib().np8_set_data(self._h, _p(X), self.N, self.D, int(offset),
                                       int(self.N if n_global is None else n_global)))
        if self._substeps_auto:
            self.substeps = int(self.stats()["substeps"])

    def set_state(self, z, mu, sigma, counts=None):
        """Labels of this shard; counts = global cluster sizes (host-exchange runs), else derived."""
        z = np.ascontiguousarray(z, dtype=np.int32)
        mu = np.ascontiguousarray(mu, dtype=np.float64)
        sigma = np.ascontiguousarray(sigma, dtype=np.float64)
        if counts is None:
            self._check(lib().np8_set_state(self._h, _p(z), mu.shape[0], _p(mu), _p(sigma)))
        else:
            cnt = np.ascontiguousarray(counts, dtype=np.int64)
            self._check(lib().np8_set_state_counts(self._h, _p(z), mu.shape[0], _p(mu), _p(sigma), _p(cnt)))

    def init_random(self, K=20):
        self._check(lib().np8_init_random(self._h, int(K)))

    def sweep(self, n=1, sync=True):
        self._check(lib().np8_sweep(self._h, int(n)))
        if sync:
            self.sync()

    def sync(self):
        self._check(lib().np8_sync(self._h))

    def prepare_sweeps(self, n):
        """Capture/upload the sweep graph the next sweep(n) replays (no sweep runs)."""
        self._check(lib().np8_prepare_sweeps(self._h, int(n)))

    def sm_sweep(self, n=1):
        """n Jain-Neal split-merge sweeps (np8_sm_sweep): N split/merge attempts each, then the
        end-of-sweep step.  Synchronous."""
        self._check(lib().np8_sm_sweep(self._h, int(n)))

    def sm_stats(self):
        """Cumulative split-merge outcomes: skipped, split_rejected, merge_rejected, split_accepted,
        merge_accepted, split_no_slot (np8_sm_stats)."""
        out = np.zeros(6, dtype=np.int64)
        self._check(lib().np8_sm_stats(self._h, _p(out)))
        return dict(zip(("skipped", "split_rejected", "merge_rejected", "split_accepted", "merge_accepted",
                         "split_no_slot"), (int(v) for v in out)))

    def update_points(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        self._check(lib().np8_update_points(self._h, _p(ids), ids.size))

    def end_sweep(self):
        self._check(lib().np8_end_sweep(self._h))

    def state(self, which=0, params=True):
        z = np.zeros(max(self.N, 1), dtype=np.int32)
        K = C.c_int32(0)
        mu = np.zeros((self.kcap, self.D))
        sg = np.zeros((self.kcap, self.D, self.D))
        cnt = np.zeros(self.kcap, dtype=np.int64)
        if params:
            self._check(lib().np8_get_state(self._h, int(which), _p(z), C.byref(K), _p(mu), _p(sg), _p(cnt)))
        else:
            self._check(lib().np8_get_state(self._h, int(which), _p(z), C.byref(K), None, None, _p(cnt)))
        k = K.value
        return {"z": z[: self.N], "K": k, "mu": mu[:k], "sigma": sg[:k], "counts": cnt[:k]}

    def stats(self):
        s = Stats()
        self._check(lib().np8_stats_sized(self._h, C.byref(s), C.sizeof(s)))
        return {f: getattr(s, f) for f, _ in Stats._fields_}

    @property
    def K(self):
        return self.stats()["K"]

    def aux_bounds(self, idx):
        """Debug: the level-0 screen's upper bound of each listed item's M auxiliary log-likelihoods (n x M)."""
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        out = np.zeros((idx.size, self.M))
        self._check(lib().np8_aux_bounds(self._h, _p(idx), idx.size, _p(out)))
        return out

    def loglik_matrix(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        K = self.K
        out = np.zeros((idx.size, K + self.M))
        self._check(lib().np8_loglik_matrix(self._h, _p(idx), idx.size, _p(out)))
        return out

    def pick_batch(self, lw, u):
        """Parity/debug: the sweep's categorical draw over log-weights lw (candidate 0 = the own cluster),
        one draw per uniform in u (np8_pick_batch)."""
        lw = np.ascontiguousarray(lw, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.zeros(u.size, dtype=np.int32)
        self._check(lib().np8_pick_batch(self._h, _p(lw), lw.size, _p(u), u.size, _p(out)))
        return out

    def total_loglik(self):
        v = C.c_double(0.0)
        self._check(lib().np8_total_loglik(self._h, C.byref(v)))
        return v.value

    def set_timing(self, on=True, counters=False, all_assigns=False):
        """on: device-event timing; counters: the assign kernel's executed-work counters (n_quad);
        all_assigns: a replayed sweep graph times every assign launch (default: one per replay)."""
        self._check(lib().np8_set_timing(self._h, (1 if on else 0) | (2 if counters else 0) | (4 if all_assigns else 0)))

    # -- multi-rank ----------------------------------------------------------------------------
    def comm_init(self, uid, rank, world):
        if uid is None:
            self._check(lib().np8_comm_init(self._h, None, int(rank), int(world)))
        else:
            buf = (C.c_uint8 * 128).from_buffer_copy(uid)
            self._check(lib().np8_comm_init(self._h, buf, int(rank), int(world)))

    def record_bytes(self):
        return int(lib().np8_record_bytes(self._h))

    def step_local(self):
        rec = np.zeros(self.record_bytes(), dtype=np.uint8)
        self._check(lib().np8_step_local(self._h, _p(rec)))
        return rec

    def step_merge(self, records, world):
        records = np.ascontiguousarray(records, dtype=np.uint8)
        self._check(lib().np8_step_merge(self._h, _p(records), int(world)))

    def compact_record_bytes(self):
        """Bytes of this rank's compact record (0: the step cannot use compact records; use step_local)."""
        return int(lib().np8_compact_record_bytes(self._h))

    def step_local_compact(self):
        rec = np.zeros(self.compact_record_bytes(), dtype=np.uint8)
        self._check(lib().np8_step_local_compact(self._h, _p(rec)))
        return rec

    def step_merge_compact(self, records, world):
        """Applies the gathered compact records; True when the step halted (some rank's requests did not fit):
        every rank then calls step_resume and exchanges the full records (step_merge)."""
        records = np.ascontiguousarray(records, dtype=np.uint8)
        halted = C.c_int32(0)
        self._check(lib().np8_step_merge_compact(self._h, _p(records), int(world), C.byref(halted)))
        return bool(halted.value)

    def step_resume(self):
        rec = np.zeros(self.record_bytes(), dtype=np.uint8)
        self._check(lib().np8_step_resume(self._h, _p(rec)))
        return rec

    def exchange_step(self, all_gather, world, compact=True):
        """One synchronous step over the caller's transport: all_gather(np.uint8 array) -> the ranks' arrays
        concatenated in rank order.  compact: the compact records with the halt-and-resume rule;
        returns True when this step halted and was resumed with the full records."""
        if compact and self.compact_record_bytes() > 0:
            if not self.step_merge_compact(all_gather(self.step_local_compact()), world):
                return False
            self.step_merge(all_gather(self.step_resume()), world)
            return True
        self.step_merge(all_gather(self.step_local()), world)
        return False

    def param_stats_local(self):
        """This rank's per-cluster statistics (host exchange of the parameter update)."""
        out = np.zeros(int(lib().np8_param_stats_bytes(self._h)) // 8)
        self._check(lib().np8_param_stats_local(self._h, _p(out)))
        return out

    def end_sweep_stats(self, summed):
        """End the sweep with the statistics summed over ranks (parameter update, bookkeeping)."""
        summed = np.ascontiguousarray(summed, dtype=np.float64)
        self._check(lib().np8_end_sweep_stats(self._h, _p(summed)))

    def checkpoint(self):
        """The complete chain state as bytes (np8_checkpoint); restore() continues it bit for bit."""
        n = int(lib().np8_checkpoint_bytes(self._h))
        buf = np.zeros(n, dtype=np.uint8)
        self._check(lib().np8_checkpoint(self._h, _p(buf), n))
        return buf.tobytes()

    def restore(self, ckpt):
        """Continue the chain of a checkpoint (same configuration, seed and data: set_data first)."""
        buf = np.frombuffer(ckpt, dtype=np.uint8).copy()
        self._check(lib().np8_restore(self._h, _p(buf), buf.size))

    def check_invariants(self, raise_on_violation=True):
        """Debug invariants (np8_check_invariants): [violated bits, bad labels, slots with a wrong count,
        sum of counts]."""
        out = np.zeros(4, dtype=np.int64)
        r = lib().np8_check_invariants(self._h, _p(out))
        if r and raise_on_violation:
            self._check(r)
        return out

    def population_sweep(self):
        """The population update of one sweep without the end-of-sweep step (np8_population_sweep)."""
        self._check(lib().np8_population_sweep(self._h))

    def track_changes(self, mode="now"):
        """Start (mode "now" / "empty") or stop (None) the membership change log (np8_track_changes)."""
        self._check(lib().np8_track_changes(self._h, {None: 0, "now": 1, "empty": 2}[mode]))

    def changes(self):
        """What changed since the last call (np8_changes): moved items and their new slots, created /
        removed / updated slots, and the parameters of the created and updated ones."""
        cs = _ChangesT()
        kc, D = self.kcap, self.D
        cr, rm, up = (np.zeros(kc, dtype=np.int32) for _ in range(3))
        mu, sg = np.zeros((kc, D)), np.zeros((kc, D, D))
        cap = max(self.N, 1)
        item, slot = np.zeros(cap, dtype=np.int64), np.zeros(cap, dtype=np.int32)
        self._check(lib().np8_changes(self._h, cap, _p(item), _p(slot), _p(cr), _p(rm), _p(up), _p(mu), _p(sg),
                                      C.byref(cs)))
        nc, nu = cs.n_created, cs.n_updated
        return {"item": item[:cs.n_moved].copy(), "slot": slot[:cs.n_moved].copy(), "created": cr[:nc].copy(),
                "removed": rm[:cs.n_removed].copy(), "updated": up[:nu].copy(), "mu": mu[:nc + nu].copy(),
                "sigma": sg[:nc + nu].copy()}

    # -- reference plug-in interface (np_update_cluster_population.h:35-43) --------------------
    def update(self, cluster_matrix, data_ids):
        """UpdateClusterPopulation::update: the population update of the listed items, then the caller's
        membertrix patched in place with what changed (O(changes), np8_changes), as the reference's
        update mutates it (retract / addCluster / assign, np_neal_algorithm8.cpp:62-64,139-157).
        A full permutation of the items is one population sweep (np8_population_sweep: data-parallel
        steps of `chunk` items); anything else runs the exact sequential steps of NealAlgorithm8::update.
        The end-of-sweep step (UpdateClusters, the max-likelihood check) stays with the caller."""
        ids = np.asarray(data_ids, dtype=np.int64).reshape(-1)
        if ids.size == self.N and self.N > 0 and np.array_equal(np.sort(ids), np.arange(self.N)):
            self.population_sweep()
        else:
            self.update_points(ids)
        if cluster_matrix is not None:
            self.patch(cluster_matrix)

    def patch(self, cluster_matrix):
        """Bring cluster_matrix (a membertrix this sampler keeps coherent) up to the device state."""
        if getattr(self, "_tracked", None) is not cluster_matrix:  # first contact: the whole state
            self.track_changes("empty")
            self._tracked, self._slot_id, self._gen = cluster_matrix, {}, cluster_matrix.generation
            cluster_matrix.clear_clusters()
        for g, remap in cluster_matrix.relabels_since(self._gen):  # ids renamed by relabel() meanwhile
            self._slot_id = {s: remap[i] for s, i in self._slot_id.items()}
            self._gen = g
        ch = self.changes()
        nc = ch["created"].size
        for q, s in enumerate(ch["created"]):
            self._slot_id[int(s)] = cluster_matrix.addCluster((ch["mu"][q].copy(), ch["sigma"][q].copy()))
        for q, s in enumerate(ch["updated"]):
            cluster_matrix.setCluster(self._slot_id[int(s)], (ch["mu"][nc + q].copy(), ch["sigma"][nc + q].copy()))
        for i, s in zip(ch["item"], ch["slot"]):
            if cluster_matrix.assigned(int(i)):
                cluster_matrix.retract(int(i), auto_remove=False)
            cluster_matrix.assign(self._slot_id[int(s)], int(i))
        for s in ch["removed"]:
            cluster_matrix.remove(self._slot_id.pop(int(s)))

    def printStatistics(self):
        s = self.stats()
        print("Statistics:")
        print(f" # of new cluster events accepted: {s['new_clusters']}")
        print(f" # of deferred new-cluster requests: {s['rejected_requests']}")


class JainNealAlgorithm(NealAlgorithm8):
    """The reference's split-merge population update (class JainNealAlgorithm,
    include/np_jain_neal_algorithm.h:52-98; `-a jain_neal_split`) on the same device context: one
    sweep = N split/merge attempts on the item pairs of two scan permutations (np_mcmc.cpp:117-164),
    then the end-of-sweep parameter step and max-likelihood check.  Reference prior, fp64 contraction,
    one rank.  The Gibbs sweep of the base class stays available (sweep_gibbs)."""

    def sweep(self, n=1, sync=True):
        self.sm_sweep(n)

    def sweep_gibbs(self, n=1, sync=True):
        NealAlgorithm8.sweep(self, n, sync)

    def update(self, cluster_matrix, data_ids):
        """UpdateClusterPopulation::update at sweep granularity: data_ids must be a permutation of all
        items (the pairs of one sweep come from the library's own permutations).  The reference's
        per-pair call (np_jain_neal_algorithm.cpp:424) has no sweep-parallel form."""
        ids = np.asarray(data_ids, dtype=np.int64).reshape(-1)
        if not (ids.size == self.N and np.array_equal(np.sort(ids), np.arange(self.N))):
            raise ValueError("JainNealAlgorithm.update: pass a permutation of all items (one split-merge sweep)")
        self.sm_sweep(1)
        if cluster_matrix is not None:
            self.patch(cluster_matrix)

    def printStatistics(self):
        s = self.sm_stats()
        print("Statistics:")
        print(f" # of merge attempts: {s['merge_accepted'] + s['merge_rejected']}")
        print(f"   o of accepted merge cluster events: {s['merge_accepted']}")
        print(f" # of split attempts: {s['split_accepted'] + s['split_rejected'] + s['split_no_slot']}")
        print(f"   o of accepted split cluster events: {s['split_accepted']}")


class TriadicAlgorithm(NealAlgorithm8):
    """The reference's triadic split-merge population update (class TriadicAlgorithm,
    src/np_triadic_algorithm.cpp; `-a triadic`): one sweep = N attempts on the item triples of three
    scan permutations (dyadic 1 <-> 2 and triadic 2 <-> 3 split/merge moves), then the end-of-sweep
    step.  Reference prior, fp64 contraction, one rank."""

    def sweep(self, n=1, sync=True):
        self._check(lib().np8_tri_sweep(self._h, int(n)))

    def sweep_gibbs(self, n=1, sync=True):
        NealAlgorithm8.sweep(self, n, sync)

    def tri_stats(self):
        out = np.zeros(10, dtype=np.int64)
        self._check(lib().np8_tri_stats(self._h, _p(out)))
        keys = ("skipped", "dyadic_merge_rejected", "dyadic_merge_accepted", "dyadic_split_rejected",
                "dyadic_split_accepted", "triadic_merge_rejected", "triadic_merge_accepted",
                "triadic_split_rejected", "triadic_split_accepted", "split_no_slot")
        return dict(zip(keys, (int(v) for v in out)))

    def update(self, cluster_matrix, data_ids):
        """Sweep granularity (a permutation of all items), as JainNealAlgorithm.update."""
        ids = np.asarray(data_ids, dtype=np.int64).reshape(-1)
        if not (ids.size == self.N and np.array_equal(np.sort(ids), np.arange(self.N))):
            raise ValueError("TriadicAlgorithm.update: pass a permutation of all items (one split-merge sweep)")
        self.sweep(1)
        if cluster_matrix is not None:
            self.patch(cluster_matrix)

    def printStatistics(self):
        s = self.tri_stats()
        print("Statistics:")
        for kind in ("dyadic_merge", "dyadic_split", "triadic_merge", "triadic_split"):
            print(f" # of {kind.replace('_', ' ')} attempts: {s[kind + '_accepted'] + s[kind + '_rejected']}")
            print(f"   o of accepted cluster events: {s[kind + '_accepted']}")


class membertrix:
    """Host mirror of the reference's membership state (include/membertrix.h:52-313, src/membertrix.cpp):
    labels per item and a map cluster id -> parameters (mu, Sigma) instead of the dense N x C bool matrix
    (membertrix.h:30).  Cluster ids come from addCluster in increasing order (the reference appends a
    column, membertrix.cpp:87-100); relabel() renames the live clusters 0..K-1 in ascending id order (the
    copy constructor's renumbering, membertrix.cpp:34-55) and records the renaming so that a sampler
    patching this membertrix can follow it (relabels_since)."""

    def __init__(self, n_items=0):
        self.z = np.full(int(n_items), -1, dtype=np.int64)
        self.clusters = {}
        self.counts = {}
        self._next = 0
        self.generation = 0
        self._relabels = []

    def addData(self, n=1):
        first = self.z.size
        self.z = np.concatenate([self.z, np.full(int(n), -1, dtype=np.int64)])
        return first

    def clear_clusters(self):
        self.z[:] = -1
        self.clusters, self.counts = {}, {}

    def addCluster(self, cluster):
        cid = self._next
        self._next += 1
        self.clusters[cid] = cluster
        self.counts[cid] = 0
        return cid

    def getCluster(self, cluster_id):
        return self.clusters[cluster_id]

    def setCluster(self, cluster_id, cluster):
        self.clusters[cluster_id] = cluster

    def assign(self, cluster_id, data_id):
        if self.z[data_id] >= 0:
            raise ValueError("already assigned")  # error_already_assigned
        self.z[data_id] = cluster_id
        self.counts[cluster_id] += 1

    def assigned(self, data_id):
        return bool(self.z[data_id] >= 0)

    def retract(self, data_id, auto_remove=True):
        c = int(self.z[data_id])
        if c < 0:
            raise ValueError("assignment absent")
        self.z[data_id] = -1
        self.counts[c] -= 1
        if auto_remove and self.counts[c] == 0:  # membertrix.cpp:200-203
            self.remove(c)

    def remove(self, cluster_id):
        if self.counts.get(cluster_id, 0) != 0:
            raise ValueError("assignment remaining")
        self.clusters.pop(cluster_id, None)
        self.counts.pop(cluster_id, None)

    def cleanup(self):
        empty = [c for c, n in self.counts.items() if n == 0]
        for c in empty:
            self.remove(c)
        return len(empty)

    def relabel(self):
        remap = {c: k for k, c in enumerate(sorted(c for c, n in self.counts.items() if n > 0))}
        self.clusters = {remap[c]: v for c, v in self.clusters.items() if c in remap}
        self.counts = {remap[c]: n for c, n in self.counts.items() if c in remap}
        lut = np.full(self._next + 1, -1, dtype=np.int64)
        for c, k in remap.items():
            lut[c] = k
        self.z = np.where(self.z >= 0, lut[np.maximum(self.z, 0)], -1)
        self._next = len(remap)
        self.generation += 1
        self._relabels.append((self.generation, remap))

    def relabels_since(self, generation):
        return [(g, m) for g, m in self._relabels if g > generation]

    def count(self, cluster_id=None):
        return int(self.z.size if cluster_id is None else self.counts.get(cluster_id, 0))

    def getClusterId(self, data_id):
        return int(self.z[data_id])

    def getClusters(self):
        return self.clusters

    def getClusterCount(self):
        return len(self.clusters)

    def dense(self):
        """(labels 0..K-1 in ascending id order, counts, mu [K, D], Sigma [K, D, D]) -- np8_get_state's form."""
        ids = sorted(self.clusters)
        lut = {c: k for k, c in enumerate(ids)}
        z = np.array([lut[int(c)] for c in self.z], dtype=np.int32)
        mu = np.array([self.clusters[c][0] for c in ids])
        sg = np.array([self.clusters[c][1] for c in ids])
        return z, np.array([self.counts[c] for c in ids], dtype=np.int64), mu, sg

    def load(self, st):
        """Replace the whole state by a dense one (labels 0..K-1, counts; parameters if present)."""
        K = int(st["K"]) if "K" in st else len(st["counts"])
        self.clusters = {k: (st["mu"][k] if "mu" in st else None, st["sigma"][k] if "sigma" in st else None)
                         for k in range(K)}
        self.counts = {k: int(st["counts"][k]) for k in range(K)}
        self.z = np.asarray(st["z"], dtype=np.int64).copy()
        self._next = K
