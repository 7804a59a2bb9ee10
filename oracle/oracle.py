"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (np8_oracle.c) and of the reference
header harness (_ref/libnp8ref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker or the timed CPU baseline.  The product path (noparama_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libnp8oracle.so")
_REF = os.path.join(_HERE, "_ref", "libnp8ref.so")

NP8O_DMAX = 128


class _Config(C.Structure):
    _fields_ = [
        ("D", C.c_int32),
        ("M", C.c_int32),
        ("alpha", C.c_double),
        ("mu0", C.c_double * NP8O_DMAX),
        ("kappa", C.c_double),
        ("nu", C.c_double),
        ("Lambda", C.c_double * (NP8O_DMAX * NP8O_DMAX)),
        ("seed", C.c_uint64),
        ("kcap", C.c_int32),
        ("chunk", C.c_int64),
        ("param_update", C.c_int32),
        ("mh_steps", C.c_int32),
        ("prior", C.c_int32),
        ("contraction", C.c_int32),
        ("req_max", C.c_int32),
        ("pick", C.c_int32),
        ("substeps", C.c_int32),
    ]


PARAM_UPDATE = {"frozen": 0, "mh_g0": 1, "niw_conjugate": 2}
PRIOR = {"reference": 0, "niw": 1}
CONTRACTION = {"f64": 0, "f32": 1}
PICK = {"reservoir": 0, "invcdf": 1}


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        P = C.POINTER
        d, i32, i64, u32, u64 = C.c_double, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
        vp = C.c_void_p
        L.np8o_philox4x32_10.argtypes = [P(u32), P(u32), P(u32)]
        L.np8o_u01.argtypes = [u32, u32]
        L.np8o_u01.restype = d
        L.np8o_normal.argtypes = [u64, u64, u32, u32, u32]
        L.np8o_normal.restype = d
        L.np8o_uniform.argtypes = [u64, u64, u32, u32, u32]
        L.np8o_uniform.restype = d
        L.np8o_perm.argtypes = [u64, u32, u32, u32]
        L.np8o_perm.restype = u32
        L.np8o_mvn_probability_ref.argtypes = [vp, vp, vp, C.c_int]
        L.np8o_mvn_probability_ref.restype = d
        L.np8o_mvn_logprobability_ref.argtypes = [vp, vp, vp, C.c_int]
        L.np8o_mvn_logprobability_ref.restype = d
        L.np8o_weighted_pick_ref.argtypes = [vp, i64, d]
        L.np8o_weighted_pick_ref.restype = i64
        L.np8o_pick_reservoir.argtypes = [vp, i64, d]
        L.np8o_pick_reservoir.restype = i64
        L.np8o_pick_reservoir_batch.argtypes = [vp, i64, vp, i64, vp]
        L.np8o_substep_of.argtypes = [u64, i64, u32]
        L.np8o_substep_of.restype = u32
        L.np8o_lu_inverse_det.argtypes = [vp, C.c_int, vp, vp]
        L.np8o_similarity.argtypes = [vp, vp, i64, vp]
        L.np8o_create.argtypes = [P(_Config)]
        L.np8o_create.restype = vp
        L.np8o_destroy.argtypes = [vp]
        L.np8o_set_data.argtypes = [vp, vp, i64]
        L.np8o_set_state.argtypes = [vp, vp, i32, vp, vp]
        L.np8o_init_random.argtypes = [vp, i32]
        L.np8o_sweep.argtypes = [vp, i32]
        L.np8o_update_points.argtypes = [vp, vp, i64]
        L.np8o_get_state.argtypes = [vp, i32, vp, vp, vp, vp, vp]
        L.np8o_num_clusters.argtypes = [vp]
        L.np8o_num_clusters.restype = i32
        L.np8o_epoch.argtypes = [vp]
        L.np8o_epoch.restype = u32
        L.np8o_best_loglik.argtypes = [vp]
        L.np8o_best_loglik.restype = d
        L.np8o_total_loglik.argtypes = [vp]
        L.np8o_total_loglik.restype = d
        L.np8o_loglik_matrix.argtypes = [vp, vp, i64, vp]
        L.np8o_loglik_matrix_ref.argtypes = [vp, vp, i64, vp]
        L.np8o_aux_params.argtypes = [vp, i64, vp, vp]
        L.np8o_assign_range.argtypes = [vp, i64, i64, vp, vp, vp, vp, vp, i32, vp]
        L.np8o_finalize.argtypes = [vp, vp, vp, vp, vp, vp, i32, i64, i64]
        L.np8o_end_sweep.argtypes = [vp]
        L.np8o_suffstats.argtypes = [vp, vp]
        L.np8o_param_update.argtypes = [vp, vp]
        L.np8o_param_update.restype = i64
        L.np8o_mh_accepted.argtypes = [vp]
        L.np8o_mh_accepted.restype = i64
        L.np8o_set_threads.argtypes = [C.c_int]
        L.np8o_gamma_mt.argtypes = [u64, u64, u32, u32, u32, d]
        L.np8o_gamma_mt.restype = d
        L.np8o_niw_draw.argtypes = [vp, u64, u32, u32, i64, vp, vp, vp, vp]
        L.np8o_sm_sweep.argtypes = [vp, i32]
        L.np8o_sm_get_stats.argtypes = [vp, vp]
        L.np8o_sm_attempts.argtypes = [vp, i64, i64]
        L.np8o_tri_sweep.argtypes = [vp, i32]
        L.np8o_tri_attempts.argtypes = [vp, i64, i64]
        L.np8o_tri_get_stats.argtypes = [vp, vp]
        L.np8o_lgamma_int.argtypes = [i64]
        L.np8o_lgamma_int.restype = d
        L.np8o_canon_sum.argtypes = [vp, i64]
        L.np8o_canon_sum.restype = d
        L.np8o_request_stats.argtypes = [vp, vp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


# ---- primitives ---------------------------------------------------------------------------------
def philox4x32_10(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().np8o_philox4x32_10(c, k, o)
    return [int(v) for v in o]


def normal(seed, i, t, stream, n):
    return lib().np8o_normal(seed, i, t, stream, n)


def uniform(seed, i, t, stream, n):
    return lib().np8o_uniform(seed, i, t, stream, n)


def perm(seed, t, N, p):
    return lib().np8o_perm(seed, t, N, p)


def gamma_mt(seed, i, t, stream, call0, alpha):
    """The specification's Marsaglia-Tsang Gamma(alpha, 1) draw (NIW prior)."""
    return lib().np8o_gamma_mt(seed, i, t, stream, call0, alpha)


def mvn_probability_ref(x, mu, sigma):
    x, mu, sigma = (np.ascontiguousarray(a, dtype=np.float64) for a in (x, mu, sigma))
    return lib().np8o_mvn_probability_ref(_p(x), _p(mu), _p(sigma), x.size)


def mvn_logprobability_ref(x, mu, sigma):
    x, mu, sigma = (np.ascontiguousarray(a, dtype=np.float64) for a in (x, mu, sigma))
    return lib().np8o_mvn_logprobability_ref(_p(x), _p(mu), _p(sigma), x.size)


def lgamma_int(n):
    return lib().np8o_lgamma_int(int(n))


def canon_sum(v):
    v = np.ascontiguousarray(v, dtype=np.float64)
    return lib().np8o_canon_sum(_p(v), v.size)


def weighted_pick_ref(w, u):
    w = np.ascontiguousarray(w, dtype=np.float64)
    return int(lib().np8o_weighted_pick_ref(_p(w), w.size, float(u)))


def pick_reservoir(lw, u):
    """The specification's reservoir pick over log-weights lw (candidate 0 first) with uniform u."""
    lw = np.ascontiguousarray(lw, dtype=np.float64)
    return int(lib().np8o_pick_reservoir(_p(lw), lw.size, float(u)))


def pick_reservoir_batch(lw, u):
    """pick_reservoir(lw, u_k) for every uniform u_k (int32 array)."""
    lw = np.ascontiguousarray(lw, dtype=np.float64)
    u = np.ascontiguousarray(u, dtype=np.float64)
    out = np.zeros(u.size, dtype=np.int32)
    lib().np8o_pick_reservoir_batch(_p(lw), lw.size, _p(u), u.size, _p(out))
    return out


def substep_of(seed, i, S):
    return lib().np8o_substep_of(seed, i, S)


def set_threads(n):
    """OpenMP threads of the oracle's synchronous step (the cpu_par baseline); results unchanged."""
    lib().np8o_set_threads(int(n))


def similarity(truth, result):
    t = np.ascontiguousarray(truth, dtype=np.int32)
    r = np.ascontiguousarray(result, dtype=np.int32)
    out = np.zeros(3)
    lib().np8o_similarity(_p(t), _p(r), t.size, _p(out))
    return {"purity": out[0], "rand_index": out[1], "adjusted_rand_index": out[2]}


def ref_harness():
    """The reference's own random_weighted_pick (oracle/_ref), or None when not built."""
    if not os.path.exists(_REF):
        return None
    L = C.CDLL(_REF)
    L.np8ref_weighted_pick.argtypes = [C.c_void_p, C.c_int64, C.c_double]
    L.np8ref_weighted_pick.restype = C.c_int64
    return L


# ---- chain --------------------------------------------------------------------------------------
class Chain:
    """The oracle chain (np8o_ctx).  Same constructor parameters as noparama_amd.NealAlgorithm8."""

    def __init__(self, D, M=3, alpha=1.0, mu0=None, kappa=1.0 / 500, nu=4.0, Lambda=None, seed=0,
                 kcap=4096, chunk=0, param_update="frozen", mh_steps=20, prior="reference", contraction="f64",
                 req_max=0, pick="reservoir", substeps=1):
        cfg = _Config()
        cfg.substeps = substeps
        cfg.req_max = req_max
        cfg.pick = PICK[pick]
        cfg.contraction = CONTRACTION[contraction]
        cfg.param_update = PARAM_UPDATE[param_update]
        cfg.prior = PRIOR[prior]
        cfg.mh_steps = mh_steps
        cfg.D, cfg.M, cfg.alpha = D, M, alpha
        mu0 = np.full(D, 6.0) if mu0 is None else np.asarray(mu0, dtype=np.float64)
        Lam = 0.01 * np.eye(D) if Lambda is None else np.asarray(Lambda, dtype=np.float64)
        for a in range(D):
            cfg.mu0[a] = mu0[a]
        flat = Lam.reshape(-1)
        for k in range(D * D):
            cfg.Lambda[k] = flat[k]
        cfg.kappa, cfg.nu, cfg.seed, cfg.kcap, cfg.chunk = kappa, nu, seed, kcap, chunk
        self.D, self.M, self.kcap = D, M, kcap
        self._h = lib().np8o_create(C.byref(cfg))
        if not self._h:
            raise ValueError("oracle: invalid configuration")
        self.N = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().np8o_destroy(h)
            self._h = None

    def set_data(self, X):
        X = np.ascontiguousarray(X, dtype=np.float64)
        assert X.ndim == 2 and X.shape[1] == self.D
        self.N = X.shape[0]
        lib().np8o_set_data(self._h, _p(X), self.N)

    def set_state(self, z, mu, sigma):
        z = np.ascontiguousarray(z, dtype=np.int32)
        mu = np.ascontiguousarray(mu, dtype=np.float64)
        sigma = np.ascontiguousarray(sigma, dtype=np.float64)
        r = lib().np8o_set_state(self._h, _p(z), mu.shape[0], _p(mu), _p(sigma))
        if r:
            raise ValueError(f"oracle set_state: {r}")

    def init_random(self, K=20):
        r = lib().np8o_init_random(self._h, K)
        if r:
            raise ValueError(f"oracle init_random: {r}")

    def sweep(self, n=1):
        return lib().np8o_sweep(self._h, n)

    def sm_sweep(self, n=1):
        """n Jain-Neal split-merge sweeps (N attempts each, then the end-of-sweep step)."""
        r = lib().np8o_sm_sweep(self._h, n)
        if r:
            raise ValueError(f"oracle sm_sweep: {r}")

    def sm_attempts(self, a0, a1):
        """Attempts [a0, a1) of the current split-merge sweep (no end-of-sweep step)."""
        r = lib().np8o_sm_attempts(self._h, int(a0), int(a1))
        if r:
            raise ValueError(f"oracle sm_attempts: {r}")

    def tri_sweep(self, n=1):
        """n triadic split-merge sweeps (N attempts on item triples each, then the end-of-sweep step)."""
        r = lib().np8o_tri_sweep(self._h, n)
        if r:
            raise ValueError(f"oracle tri_sweep: {r}")

    def tri_attempts(self, a0, a1):
        r = lib().np8o_tri_attempts(self._h, int(a0), int(a1))
        if r:
            raise ValueError(f"oracle tri_attempts: {r}")

    @property
    def tri_stats(self):
        """[skipped, dyadic merge rej/acc, dyadic split rej/acc, triadic merge rej/acc,
        triadic split rej/acc, split without a free slot]"""
        out = np.zeros(10, dtype=np.int64)
        lib().np8o_tri_get_stats(self._h, _p(out))
        return out

    @property
    def sm_stats(self):
        """[skipped, split rejected, merge rejected, split accepted, merge accepted, split at kcap]"""
        out = np.zeros(6, dtype=np.int64)
        lib().np8o_sm_get_stats(self._h, _p(out))
        return out

    def update_points(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        return lib().np8o_update_points(self._h, _p(ids), ids.size)

    def end_sweep(self):
        lib().np8o_end_sweep(self._h)

    @property
    def K(self):
        return lib().np8o_num_clusters(self._h)

    @property
    def request_stats(self):
        """[accepted new-cluster requests, requests deferred (not accepted)], cumulative."""
        out = np.zeros(2, dtype=np.int64)
        lib().np8o_request_stats(self._h, _p(out))
        return out

    @property
    def mh_accepted(self):
        return lib().np8o_mh_accepted(self._h)

    def suffstats(self):
        """Per-slot [kcap, D + D(D+1)/2] statistics about each slot's mean (np8o_suffstats)."""
        out = np.zeros((self.kcap, self.D + self.D * (self.D + 1) // 2))
        lib().np8o_suffstats(self._h, _p(out))
        return out

    def param_update(self, stats):
        stats = np.ascontiguousarray(stats, dtype=np.float64)
        return lib().np8o_param_update(self._h, _p(stats))

    @property
    def epoch(self):
        return lib().np8o_epoch(self._h)

    def best_loglik(self):
        return lib().np8o_best_loglik(self._h)

    def total_loglik(self):
        return lib().np8o_total_loglik(self._h)

    def state(self, which=0, params=True):
        z = np.zeros(max(self.N, 1), dtype=np.int32)
        K = C.c_int32(0)
        mu = np.zeros((self.kcap, self.D))
        sg = np.zeros((self.kcap, self.D, self.D))
        cnt = np.zeros(self.kcap, dtype=np.int64)
        r = lib().np8o_get_state(self._h, which, _p(z), C.byref(K), _p(mu), _p(sg), _p(cnt))
        if r:
            raise ValueError(f"oracle get_state: {r}")
        k = K.value
        return {"z": z[: self.N], "K": k, "mu": mu[:k], "sigma": sg[:k], "counts": cnt[:k]}

    def loglik_matrix(self, idx, ref=False):
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        out = np.zeros((idx.size, self.K + self.M))
        f = lib().np8o_loglik_matrix_ref if ref else lib().np8o_loglik_matrix
        r = f(self._h, _p(idx), idx.size, _p(out))
        if r:
            raise ValueError(f"oracle loglik_matrix: {r}")
        return out

    def niw_draw(self, i, t, stream, n=0, stats=None, anchor=None):
        """NIW posterior draw of n items with statistics (np8o_suffstats layout) about anchor; the
        prior draw for n = 0.  Returns (mu, Sigma); does not change the chain."""
        mu = np.zeros(self.D)
        sg = np.zeros((self.D, self.D))
        st = None if stats is None else np.ascontiguousarray(stats, dtype=np.float64)
        an = None if anchor is None else np.ascontiguousarray(anchor, dtype=np.float64)
        r = lib().np8o_niw_draw(self._h, int(i), int(t), int(stream), int(n), None if st is None else _p(st),
                                None if an is None else _p(an), _p(mu), _p(sg))
        if r:
            raise ValueError(f"oracle niw_draw: {r}")
        return mu, sg

    def aux_params(self, i):
        mu = np.zeros((self.M, self.D))
        sg = np.zeros((self.M, self.D, self.D))
        lib().np8o_aux_params(self._h, int(i), _p(mu), _p(sg))
        return mu, sg

    # sharded protocol (gloo tests)
    def assign_range(self, p0, p1, req_cap=65536):
        delta = np.zeros(self.kcap, dtype=np.int32)
        rp = np.zeros(req_cap, dtype=np.int64)
        ri = np.zeros(req_cap, dtype=np.int64)
        rm = np.zeros(req_cap, dtype=np.int32)
        rz = np.zeros(req_cap, dtype=np.int32)
        n = C.c_int32(0)
        r = lib().np8o_assign_range(self._h, p0, p1, _p(delta), _p(rp), _p(ri), _p(rm), _p(rz), req_cap,
                                    C.byref(n))
        if r:
            raise ValueError(f"oracle assign_range: {r}")
        k = min(n.value, req_cap)
        return delta, rp[:k].copy(), ri[:k].copy(), rm[:k].copy(), rz[:k].copy(), n.value

    def finalize(self, delta, rp, ri, rm, rz, n_req=None, owner_lo=0, owner_hi=-1):
        delta = np.ascontiguousarray(delta, dtype=np.int32)
        rp = np.ascontiguousarray(rp, dtype=np.int64)
        ri = np.ascontiguousarray(ri, dtype=np.int64)
        rm = np.ascontiguousarray(rm, dtype=np.int32)
        rz = np.ascontiguousarray(rz, dtype=np.int32)
        n = rp.size if n_req is None else n_req
        return lib().np8o_finalize(self._h, _p(delta), _p(rp), _p(ri), _p(rm), _p(rz), n, owner_lo, owner_hi)
