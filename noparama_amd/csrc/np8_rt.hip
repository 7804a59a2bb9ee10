// np8_rt.hip -- the fp64 sweep at any (D, M) the templated kernels are not instantiated for: 16 < D <= kMaxD with the
// reference's arithmetic (contraction F64), and the (D, M) pairs of 8 < D <= 16 without an instance.  The same
// operations in the same order as np8_assign / np8_loglik / np8_loglik_matrix_kernel (and oracle/np8_oracle.c's F64
// contraction, which has D at run time): the packed upper triangle of sym(Sigma^{-1}) with pre-doubled off-diagonals
// (isotropic rows: iso |x - mu|^2), the auxiliaries drawn exactly (aux_core_rt: no prefix words above kPreMaxD), the
// reservoir pick, candidate lists, radii, requests with their (v, mu) payload -- with D and M at run time.
// (src/np_neal_algorithm8.cpp:49-167 for every item; src/statistics/multivariatenormal.cpp:84-92: the dynamic-size
// fp64 likelihood, include/np_data.h:9.)
//
// One lane per item, one-wave workgroups: the lane's item row lives in LDS ([D][64] doubles, dynamic), read back at
// each use (a wave-uniform candidate row's fields come through the scalar cache).  No auxiliary screen: every lane
// draws its M auxiliaries exactly (aux_core_rt: (D - 1) / 2 + 2 Philox calls each).
#include "np8_kernels.h"

#include <hip/hip_runtime.h>

using namespace np8;

namespace {

__device__ __forceinline__ int64_t rt_position_to_local(const AssignArgs &A, int64_t p) {
    if (A.order) return A.order[p];
    if (A.use_perm) return (int64_t)perm_apply(A.perm, (uint32_t)p);
    return p;
}

// ll = c - q/2 of the candidate row at e for the item whose coordinate a is xa(a): cand_ll's operations with D at
// run time (d_a = x_a - e_a is recomputed at each use: the same bits).
template <class XA>
__device__ __forceinline__ double cand_ll_rt(const double *__restrict__ e, int D, XA xa) {
    const int DP = D * (D + 1) / 2;
    const double iso = e[D + DP + kFieldIso];
    double q;
    if (iso > 0.0) {
        const double d0 = xa(0) - e[0];
        double s = d0 * d0;
        for (int a = 1; a < D; ++a) {
            const double d = xa(a) - e[a];
            s = fma(d, d, s);
        }
        q = s * iso;
    } else {
        const double *P = e + D;
        q = 0.0;
        int k = 0;
        for (int a = 0; a < D; ++a) {
            const double da = xa(a) - e[a];
            double t = P[k++] * da;
            int b = a + 1;
            for (; b + 8 <= D; b += 8, k += 8) {  // eight terms' operands loaded together, then their fmas in order
                double pv[8], dv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    pv[u] = P[k + u];
                    dv[u] = xa(b + u) - e[b + u];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) t = fma(pv[u], dv[u], t);
            }
            for (; b < D; ++b) t = fma(P[k++], xa(b) - e[b], t);
            q = fma(t, da, q);
        }
    }
    return fma(-0.5, q, e[D + DP + kFieldC]);
}

// |y0|, y0 = U^T (x - mu0) (whiten + norm_of: the fma chains in ascending order); y0 stored when y0 != nullptr
template <class XA>
__device__ __forceinline__ double item_norm_rt(const double *__restrict__ hyp, int D, XA xa, double *y0) {
    const double *U = hyp + D;
    double n2 = 0.0;
    int k = 0;
    for (int a = 0; a < D; ++a) {
        double t0 = U[k++] * (xa(a) - hyp[a]);
        for (int b = a + 1; b < D; ++b) t0 = fma(U[k++], xa(b) - hyp[b], t0);
        if (y0) y0[a] = t0;
        n2 = fma(t0, t0, n2);
    }
    return sqrt(n2);
}

// ll of auxiliary m (reference prior): aux_core + aux_loglik with D at run time
__device__ __forceinline__ double aux_ll_rt(const double *__restrict__ hyp, int D, int M, double ny, uint64_t seed,
                                            uint64_t ig, uint32_t t, int m) {
    const int DP = D * (D + 1) / 2;
    double v, xpar, chi2;
    aux_core_rt(seed, ig, t, m, M, D, hyp[D + DP + 3], v, xpar, chi2);
    return aux_loglik(ny, v, xpar, chi2, D, hyp[D + DP + 1], hyp[D + DP]);
}

// (v, mu) of the picked auxiliary m: aux_params with D at run time (np8_frame_slots' frame_to_vmu from y0 in hand)
__device__ void aux_params_rt(const double *__restrict__ hyp, int D, int M, const double *y0, double ny, uint64_t seed,
                              uint64_t ig, uint32_t t, int m, double *vmu) {
    const int DP = D * (D + 1) / 2;
    double xi[kMaxD];
    double v, xpar, chi2;
    aux_core_rt(seed, ig, t, m, M, D, hyp[D + DP + 3], v, xpar, chi2);
    aux_xi<kMaxD>(seed, ig, t, m, D, y0, ny, xpar, chi2, xi);
    const double sc = fabs(v) * hyp[D + DP + 1];
    const double *LT = hyp + D + DP + 4;
    vmu[0] = v;
    int k = 0;
    for (int a = 0; a < D; ++a) {
        double t0 = LT[k++] * xi[a];
        for (int b = a + 1; b < D; ++b) t0 = fma(LT[k++], xi[b], t0);
        vmu[1 + a] = fma(sc, t0, hyp[a]);
    }
}

__device__ __forceinline__ void ensure_u_rt(PickState &st, double lw, uint64_t seed, uint64_t ig, uint32_t t) {
    const bool need = st.u < 0.0 && lw - st.T > -kSkip;
    if (__ballot(need)) {
        if (st.u < 0.0) st.u = uniform(seed, ig, t, kStreamPick, 0);
    }
}

}  // namespace

// np8_assign's step for one lane per item of [p0, p1) with D = A.dim, M = A.naux at run time (reference prior).
__global__ __launch_bounds__(64) void np8_assign_rt(AssignArgs A) {
    extern __shared__ double xs_rt[];  // [D][64]: the lanes' item rows
    const int D = A.dim, M = A.naux, DP = D * (D + 1) / 2, CS = cand_stride(D), F = D + DP;
    const int lane = threadIdx.x & 63;
    const int64_t p = A.p0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= A.p1) return;  // (the range's last wave: its active lanes only, below)
    const bool sorted = A.sorted != 0;
    int32_t *__restrict__ zs = A.zs[0];
    const int32_t *__restrict__ ids = A.ids[0];
    const int64_t lk = sorted ? (int64_t)ids[p] : rt_position_to_local(A, p);
    const int64_t il = key_item(lk);
    const int64_t xr = sorted ? p : il;
    const uint64_t ig = (uint64_t)(A.offset + lk);
    const double *__restrict__ X = sorted ? A.Xs[0] : A.X;
    const double *__restrict__ cand = A.cand;
    const double *__restrict__ hyp = A.hyp;
    const uint32_t t = A.ctl->t_base + A.t;
    for (int a = 0; a < D; ++a) xs_rt[a * 64 + lane] = X[(int64_t)a * A.n_loc + xr];  // (each lane its own column)
    auto xa = [&](int a) { return xs_rt[a * 64 + lane]; };
    const int32_t zi = sorted ? zs[p] : A.z[il];
    const int32_t jo = A.dense_of[zi];
    PickState st;
    {
        // the own row: one pass per distinct own row of the wave (wave-uniform rows)
        uint64_t pend = __ballot(1);
        while (pend) {
            const int32_t j = __builtin_amdgcn_readlane(jo, __ffsll((unsigned long long)pend) - 1);
            if (jo == j) {
                const double *eo = cand + (int64_t)j * CS;
                st.T = cand_ll_rt(eo, D, xa) + eo[F + kFieldLogn1];
            }
            pend &= ~__ballot(jo == j);
        }
        st.S = 1.0;
        st.u = -1.0;
        st.pick = jo;
    }
    const double zslot = (double)zi;
    const int K = A.ctl->K;
    int32_t pslot = zi;
    int ngroups = 0;
    for (uint64_t pend = __ballot(1); pend && ngroups <= A.max_groups; ++ngroups)
        pend &= ~__ballot(jo == __builtin_amdgcn_readlane(jo, __ffsll((unsigned long long)pend) - 1));
    bool full = true;
    if (A.use_lists && A.ctl->lists_ok && ngroups <= A.max_groups) {
        uint64_t pend = __ballot(1);
        while (pend) {
            const int32_t j0 = __builtin_amdgcn_readlane(jo, __ffsll((unsigned long long)pend) - 1);
            pend &= ~__ballot(jo == j0);
            if (jo == j0) {
                // the list holds for items within the radius it was built for
                const double *e0 = cand + (int64_t)j0 * CS;
                double d2 = 0.0;
                for (int a = 0; a < D; ++a) {
                    const double dd = xa(a) - e0[a];
                    d2 = fma(dd, dd, d2);
                }
                full = !(d2 <= A.plr2[j0]);
                if (!full) {
                    const int32_t nl = A.plen[j0];
                    const int32_t *__restrict__ lst = A.plist + (int64_t)j0 * A.ls;
                    for (int q = 0; q < nl; ++q) {
                        const int j = lst[q];
                        const double *e = cand + (int64_t)j * CS;
                        const double lw = cand_ll_rt(e, D, xa) + e[F + kFieldLogn];
                        ensure_u_rt(st, lw, A.seed, ig, t);
                        pick_step(st, lw, j);
                        pslot = (st.pick == j) ? (int32_t)e[F + kFieldSlot] : pslot;
                    }
                }
            }
        }
    }
    if (full) {  // wave-uniform row loop over the lanes that need it
        for (int j = 0; j < K; ++j) {
            const double *e = cand + (int64_t)j * CS;
            const double lw = cand_ll_rt(e, D, xa) + e[F + kFieldLogn];
            if (e[F + kFieldSlot] != zslot) {
                ensure_u_rt(st, lw, A.seed, ig, t);
                pick_step(st, lw, j);
                pslot = (st.pick == j) ? (int32_t)e[F + kFieldSlot] : pslot;
            }
        }
    }
    const double ny = item_norm_rt(hyp, D, xa, nullptr);
    {
        const double logam = hyp[D + DP + 2];
        for (int m = 0; m < M; ++m) {
            const double lw = aux_ll_rt(hyp, D, M, ny, A.seed, ig, t, m) + logam;
            ensure_u_rt(st, lw, A.seed, ig, t);
            pick_step(st, lw, K + m);
        }
    }

    int32_t *delta = reinterpret_cast<int32_t *>(A.rec + kRecHeaderBytes);
    const int32_t snew = (st.pick < K) ? pslot : -1;
    if (A.collect_r2) {  // the radius of the item's cluster for the next sweep's lists (np8_assign's rule)
        const int32_t tr = (st.pick < K) ? st.pick : jo;
        const int32_t ts = (st.pick < K) ? snew : zi;
        const double *e = cand + (int64_t)tr * CS;
        double d2 = 0.0;
        for (int a = 0; a < D; ++a) {
            const double dd = xa(a) - e[a];
            d2 = fma(dd, dd, d2);
        }
        const int32_t t0 = __builtin_amdgcn_readfirstlane(ts);
        const bool one = __ballot(1) == ~0ull && __ballot(ts != t0) == 0;
        if (one) {
            for (int o = 32; o > 0; o >>= 1) d2 = fmax(d2, __shfl_xor(d2, o));
        } else {
            wave_max_by_key(reinterpret_cast<unsigned long long *>(A.r2 + A.kcap), ts, d2, true);
        }
        if (lane == (__ffsll((unsigned long long)__ballot(1)) - 1)) {  // the wave's record
            WaveR2 w;
            w.d2 = one ? d2 : 0.0;
            w.slot = one ? t0 : -1;
            w.pad = 0;
            A.wr2[(p - A.p0) >> 6] = w;
        }
    }
    const uint64_t mv = __ballot(snew != zi);
    if (mv && lane == (__ffsll((unsigned long long)__ballot(1)) - 1))
        atomicAdd(reinterpret_cast<unsigned long long *>(&A.ctl->moved), (unsigned long long)__popcll(mv));
    const bool mover = st.pick < K && snew != zi;
    wave_add_by_key(delta, zi, -1, mover);
    wave_add_by_key(delta, snew, 1, mover);
    const int qreq = wave_append(A.nreq, st.pick >= K);  // (requests are accepted by scan position, not arrival)
    if (st.pick < K) {
        if (snew != zi) {
            A.z[il] = snew;
            if (sorted) zs[p] = snew;
        }
    } else {
        const int q = qreq;
        if (q < A.req_cap) {  // always: the area holds every item of the step
            Request r;
            r.pos = sorted ? (int64_t)ig : A.offset + p;  // synchronous sweep: scan position = item index
            r.i = (int64_t)ig;
            r.m = st.pick - K;
            r.zold = zi;
            r.lpos = sorted ? (int32_t)p : -1;
            r.pad = 0;
            r.dll.lo = 0ull;
            r.dll.hi = 0;
            A.req[q] = r;
            double y0[kMaxD];
            const double nyr = item_norm_rt(hyp, D, xa, y0);
            aux_params_rt(hyp, D, M, y0, nyr, A.seed, ig, t, st.pick - K, A.vmu + (int64_t)q * (D + 1));
        }
    }
}

// Max-likelihood partials: one lane per item, its own row's ll (np8_loglik's operations), block sums in order.
__global__ __launch_bounds__(256) void np8_loglik_rt(LoglikArgs A, int D) {
    const int DP = D * (D + 1) / 2, CS = cand_stride(D);
    __shared__ double red[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double ll = 0.0;
    if (i < A.n_loc) {
        const double *X = A.X;
        const int64_t n = A.n_loc;
        ll = cand_ll_rt(A.cand + (int64_t)A.dense_of[A.z[i]] * CS, D, [&](int a) { return X[(int64_t)a * n + i]; });
    }
    (void)DP;
    red[threadIdx.x] = ll;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) A.partial[blockIdx.x] = red[0];
}

// Parity/debug: out[r (K + M) + j] = ll of item idx[r] under row j, then its M auxiliaries (reference prior).
__global__ __launch_bounds__(256) void np8_loglik_matrix_rt(AssignArgs A, const int64_t *__restrict__ idx, int64_t n,
                                                            double *__restrict__ out) {
    const int D = A.dim, M = A.naux, CS = cand_stride(D);
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t il = idx[r];
    const uint64_t ig = (uint64_t)(A.offset + il);
    const double *X = A.X;
    const int64_t nl = A.n_loc;
    auto xa = [&](int a) { return X[(int64_t)a * nl + il]; };
    const int K = A.ctl->K;
    for (int j = 0; j < K; ++j) out[r * (K + M) + j] = cand_ll_rt(A.cand + (int64_t)j * CS, D, xa);
    const double ny = item_norm_rt(A.hyp, D, xa, nullptr);
    const uint32_t t = A.ctl->t_base + A.t;
    for (int m = 0; m < M; ++m) out[r * (K + M) + K + m] = aux_ll_rt(A.hyp, D, M, ny, A.seed, ig, t, m);
}

hipError_t np8_launch_assign_rt(const AssignArgs &A0, int D, int M, hipStream_t s) {
    const int64_t n = A0.p1 - A0.p0;
    if (n <= 0) return hipSuccess;
    if (D < 1 || D > kMaxD || M < 1 || M > kMaxM) return hipErrorInvalidValue;
    AssignArgs A = A0;
    A.dim = D;
    A.naux = M;
    hipLaunchKernelGGL(np8_assign_rt, dim3((unsigned)((n + 63) / 64)), dim3(64), sizeof(double) * 64 * (size_t)D, s, A);
    return hipGetLastError();
}

hipError_t np8_launch_loglik_rt(const LoglikArgs &A, int D, hipStream_t s) {
    const int64_t nb = (A.n_loc + 255) / 256;
    if (nb <= 0) return hipSuccess;
    hipLaunchKernelGGL(np8_loglik_rt, dim3((unsigned)nb), dim3(256), 0, s, A, D);
    return hipGetLastError();
}

hipError_t np8_launch_loglik_matrix_rt(const AssignArgs &A0, int D, int M, const int64_t *idx, int64_t n, double *out,
                                       hipStream_t s) {
    if (n <= 0) return hipSuccess;
    AssignArgs A = A0;
    A.dim = D;
    A.naux = M;
    hipLaunchKernelGGL(np8_loglik_matrix_rt, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, idx, n, out);
    return hipGetLastError();
}
