// np8_wide.hip -- the wide path (DESIGN.md "Wide path"; BASELINE.json config C5): D in {32, 64}, items
// held in fp32, cluster likelihoods through fp32 MFMA (v_mfma_f32_32x32x2_f32, exact k-ordered fmaf
// chains), everything else (auxiliary draws, the categorical pick, counts) in fp64 as on the narrow path.
//
//   np8_wide_rows     per slot whose parameters changed: R = chol_upper(sym Sigma^{-1}) (fp64, in LDS),
//                     A = fp32(R) in natural and MFMA-fragment order, muf = fp32(mu)
//   np8_wide_gtab     g[sj][sk] = A_j (muf_j - muf_k) for every live pair touching a changed slot: the
//                     offset of candidate j in the frame of an item's own cluster k
//   np8_wide_clean    clears the change flags
//   np8_assign_wide   one wave per 64 items (one lane per item for the fp64 parts): per candidate row
//                     the 64 x D x D contraction y = A_j (x - muf_k) - g_jk on the matrix cores,
//                     q = |y|^2 in fp64, then the same single-uniform reservoir pick as np8_assign
//                     (src/np_neal_algorithm8.cpp:49-167 for every item of the wave)
//   np8_loglik_wide / np8_loglik_matrix_wide   the same arithmetic on the vector ALU (bit-identical:
//                     an MFMA is an fmaf chain) for the max-likelihood sum and the parity debug entry
//
// The contraction is specified in oracle/np8_oracle.h (NP8O_CONTRACT_F32) so that the CPU oracle
// reproduces it bit for bit.  A is upper triangular: rows 32..63 skip the k-steps of columns 0..31.
#include "np8_kernels.h"

#include <hip/hip_runtime.h>

using namespace np8;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int D>
struct Wide {
    static constexpr int MT = D / 32;  // 32-row tiles of A
    static constexpr int S = D / 2;    // k-steps of the 32x32x2 MFMA
    static constexpr int S4 = S / 4;   // float4 groups of k-steps per lane
    static constexpr int DP = D * (D + 1) / 2;
    static constexpr int CS = (D + DP + 5 + 1) & ~1;
    static constexpr int F = D + DP;
};

__device__ __forceinline__ int64_t wpos_to_local(const AssignArgs &A, int64_t p) {
    if (A.order) return A.order[p];
    if (A.use_perm) return (int64_t)perm_apply(A.perm, (uint32_t)p);
    return p;
}

// |U^T (x - mu0)| with U^T packed upper in hyp (the item frame of the auxiliary draws): the loop order
// of whiten() + norm_of(); the whitened vector itself is never stored.
template <int D>
__device__ __forceinline__ double wide_whiten_norm(const double *__restrict__ hyp, const float (&xf)[D]) {
    const double *U = hyp + D;
    double dx[D];
#pragma unroll
    for (int a = 0; a < D; ++a) dx[a] = (double)xf[a] - hyp[a];
    double n2 = 0.0;
    int k = 0;
#pragma unroll
    for (int a = 0; a < D; ++a) {  // fully unrolled: register operands, U through the scalar cache
        double t0 = U[k++] * dx[a];
#pragma unroll
        for (int b = a + 1; b < D; ++b) t0 = fma(U[k++], dx[b], t0);
        n2 = fma(t0, t0, n2);
    }
    return sqrt(n2);
}

// The request payload of the wide path: (|y0|, y0) with y0 = U^T (x - mu0), read from global memory.
template <int D>
__device__ void wide_frame_payload(const double *__restrict__ hyp, const float *__restrict__ X, int64_t n, int64_t xr,
                                   double *vmu) {
    const double *U = hyp + D;
    double n2 = 0.0;
    int k = 0;
    for (int a = 0; a < D; ++a) {
        double t0 = U[k++] * ((double)X[(int64_t)a * n + xr] - hyp[a]);
        for (int b = a + 1; b < D; ++b) t0 = fma(U[k++], (double)X[(int64_t)b * n + xr] - hyp[b], t0);
        vmu[1 + a] = t0;
        n2 = fma(t0, t0, n2);
    }
    vmu[0] = sqrt(n2);
}

template <int D, int PRIOR>
__device__ __forceinline__ double wide_aux_ll(const double *__restrict__ hyp, double ny, uint64_t seed, uint64_t ig,
                                              uint32_t t, int m) {
    constexpr int DP = D * (D + 1) / 2;
    const double caux = hyp[D + DP], rsk = hyp[D + DP + 1], nu = hyp[D + DP + 3];
    if constexpr (PRIOR == kPriorNiw) {
        double sumlog, b00, chi, z1;
        niw_aux_core(seed, ig, t, m, D, nu, sumlog, b00, chi, z1);
        return niw_aux_loglik(ny, sumlog, b00, chi, z1, rsk, caux);
    } else {
        double v, xpar, chi2;
        aux_core(seed, ig, t, m, D, nu, v, xpar, chi2);
        return aux_loglik(ny, v, xpar, chi2, D, rsk, caux);
    }
}

// q for the lane's item (item index = lane) against slot sj: the 64 items' x~ fragments are in xb,
// their own slots in zc (items col and 32 + col).
template <int D>
__device__ __forceinline__ double wide_pass(const AssignArgs &A, int sj, const float (&xb)[2][D / 2],
                                            const int32_t (&zc)[2], int lane) {
    using W = Wide<D>;
    const int h = lane >> 5;
    f32x16 acc[W::MT][2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const float *gp = A.gtab + ((int64_t)sj * A.kcap + zc[nt]) * D;
#pragma unroll
        for (int mt = 0; mt < W::MT; ++mt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 v = *reinterpret_cast<const float4 *>(gp + mt * 32 + 8 * g + 4 * h);
                acc[mt][nt][4 * g + 0] = -v.x;
                acc[mt][nt][4 * g + 1] = -v.y;
                acc[mt][nt][4 * g + 2] = -v.z;
                acc[mt][nt][4 * g + 3] = -v.w;
            }
    }
    const float *wf = A.wfrag + (int64_t)sj * (W::MT * W::S * 64);
#pragma unroll
    for (int mt = 0; mt < W::MT; ++mt)
#pragma unroll
        for (int s4 = mt * 4; s4 < W::S4; ++s4) {  // A upper triangular: tile mt starts at column 32 mt
            const float4 a4 = *reinterpret_cast<const float4 *>(wf + ((mt * W::S4 + s4) * 64 + lane) * 4);
            const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc[mt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], xb[0][s4 * 4 + e], acc[mt][0], 0, 0, 0);
                acc[mt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], xb[1][s4 * 4 + e], acc[mt][1], 0, 0, 0);
            }
        }
    double sh[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        double s = 0.0;
#pragma unroll
        for (int mt = 0; mt < W::MT; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const double v = (double)acc[mt][nt][r];
                s = fma(v, v, s);
            }
        sh[nt] = s;
    }
    const double recv = __shfl_xor(h ? sh[0] : sh[1], 32);
    return h ? recv + sh[1] : sh[0] + recv;  // s_0 + s_1 for item `lane`
}

}  // namespace

// ---- table maintenance ---------------------------------------------------------------------------
// One block per slot (grid kcap): the slots flagged in wdirty get their factor and fp32 mean.
__global__ __launch_bounds__(256) void np8_wide_rows(WideArgs W) {
    const int s = blockIdx.x;
    if (!W.dirty[s] || W.cnt[s] <= 0) return;
    const int D = W.D, DP = D * (D + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) double R[];
    const double *Pp = W.slot_P + (int64_t)s * DP;
    for (int k = threadIdx.x; k < D * D; k += blockDim.x) R[k] = 0.0;
    __shared__ int ok_s;
    __syncthreads();
    for (int j = 0; j < D; ++j) {
        if (threadIdx.x == 0) {
            double v = Pp[j * D - (j * (j - 1)) / 2];
            for (int k = 0; k < j; ++k) v = fma(-R[k * D + j], R[k * D + j], v);
            ok_s = v > 0.0;
            if (!(v > 0.0)) atomicOr(&W.ctl->err, kErrSigma);
            R[j * D + j] = (v > 0.0) ? sqrt(v) : 1e-300;
        }
        __syncthreads();
        if (ok_s)
            for (int i = j + 1 + threadIdx.x; i < D; i += blockDim.x) {
                double w = 0.5 * Pp[j * D - (j * (j - 1)) / 2 + (i - j)];
                for (int k = 0; k < j; ++k) w = fma(-R[k * D + j], R[k * D + i], w);
                R[j * D + i] = w / R[j * D + j];
            }
        __syncthreads();
    }
    float *An = W.wA + (int64_t)s * D * D;
    for (int k = threadIdx.x; k < D * D; k += blockDim.x) An[k] = (float)R[k];
    // fragment order [mt][s4][lane][e]: lane l, k-step s = 4 s4 + e holds A[32 mt + (l & 31)][2 s + (l >> 5)]
    const int MT = D / 32, S4 = D / 8;
    float *Af = W.wfrag + (int64_t)s * D * D;
    for (int k = threadIdx.x; k < D * D; k += blockDim.x) {
        const int e = k & 3, l = (k >> 2) & 63, rest = k >> 8;
        const int s4 = rest % S4, mt = rest / S4;
        (void)MT;
        const int ks = 4 * s4 + e;
        Af[k] = (float)R[(32 * mt + (l & 31)) * D + 2 * ks + (l >> 5)];
    }
    for (int a = threadIdx.x; a < D; a += blockDim.x) W.wmu[(int64_t)s * D + a] = (float)W.slot_mu[(int64_t)s * D + a];
}

// g[sj][sk][a] = fmaf chain over b >= a of A_j[a][b] (muf_j[b] - muf_k[b]) (zero terms b < a skipped:
// fmaf(0, x, v) == v).  Grid (kcap, kcap / 4): block (sj, 4 sk), one wave per sk, lane = row a.
__global__ __launch_bounds__(256) void np8_wide_gtab(WideArgs W) {
    const int sj = blockIdx.x, sk = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (sk >= W.kcap || W.cnt[sj] <= 0 || W.cnt[sk] <= 0 || !(W.dirty[sj] || W.dirty[sk])) return;
    const int D = W.D, a = threadIdx.x & 63;
    if (a >= D) return;
    const float *Aj = W.wA + (int64_t)sj * D * D + (int64_t)a * D;
    const float *mj = W.wmu + (int64_t)sj * D, *mk = W.wmu + (int64_t)sk * D;
    float g = 0.0f;
    for (int b = a; b < D; ++b) g = fmaf(Aj[b], mj[b] - mk[b], g);
    W.gtab[((int64_t)sj * W.kcap + sk) * D + a] = g;
}

__global__ void np8_wide_clean(WideArgs W) {
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < W.kcap; s += gridDim.x * blockDim.x) W.dirty[s] = 0;
}

// ---- the sweep kernel -----------------------------------------------------------------------------
template <int D, int M, int PRIOR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void np8_assign_wide(AssignArgs A) {
    using W = Wide<D>;
    constexpr int CS = W::CS, F = W::F;
    const int lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
    const int64_t pw = A.p0 + (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
    if (pw >= A.p1) return;  // wave-uniform
    const int64_t p = pw + lane;
    const bool valid = p < A.p1;
    const bool sorted = A.sorted != 0;
    const int cur = sorted ? A.ctl->cur : 0;
    int32_t *__restrict__ zs = cur ? A.zs[1] : A.zs[0];
    const int32_t *__restrict__ ids = cur ? A.ids[1] : A.ids[0];
    const float *__restrict__ X = reinterpret_cast<const float *>(sorted ? (cur ? A.Xs[1] : A.Xs[0]) : A.X);
    const double *__restrict__ cand = A.cand;
    const double *__restrict__ hyp = A.hyp;
    const uint32_t t = A.ctl->t_base + A.t;
    const int64_t n = A.n_loc;

    // the lane's own item
    const int64_t pc = valid ? p : pw;
    const int64_t il = sorted ? (int64_t)ids[pc] : wpos_to_local(A, pc);
    const int64_t xr = sorted ? pc : il;
    const uint64_t ig = (uint64_t)(A.offset + il);
    const int32_t zi = sorted ? zs[pc] : A.z[il];
    const int32_t jo = A.dense_of[zi];

    // auxiliaries first (fp64, per lane): only |U^T (x - mu0)| of the item is needed
    double lwa[M];
    {
        float xf[D];
#pragma unroll
        for (int a = 0; a < D; ++a) xf[a] = X[(int64_t)a * n + xr];
        const double ny = wide_whiten_norm<D>(hyp, xf);
        const double logam = hyp[D + W::DP + 2];
#pragma unroll 1
        for (int m = 0; m < M; ++m) lwa[m] = wide_aux_ll<D, PRIOR>(hyp, ny, A.seed, ig, t, m) + logam;
    }

    // MFMA operand B: x~ = x - muf(own) of items col and 32 + col, dims 2 s + h
    float xb[2][W::S];
    int32_t zc[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        int64_t pq = pw + nt * 32 + col;
        if (pq >= A.p1) pq = pw;  // padding column: any valid item, result unused
        const int64_t iq = sorted ? (int64_t)ids[pq] : wpos_to_local(A, pq);
        const int64_t xq = sorted ? pq : iq;
        zc[nt] = sorted ? zs[pq] : A.z[iq];
        const float *mk = A.wmu + (int64_t)zc[nt] * D;
#pragma unroll
        for (int s = 0; s < W::S; ++s) xb[nt][s] = X[(int64_t)(2 * s + h) * n + xq] - mk[2 * s + h];
    }

    // own clusters first (weight n_k - 1), one pass per distinct own slot of the wave
    PickState st;
    st.T = 0.0;
    st.S = 1.0;
    st.u = uniform(A.seed, ig, t, kStreamPick, 0);
    st.pick = jo;
    uint64_t pend = __ballot(valid);
    while (pend) {
        const int lead = __ffsll((unsigned long long)pend) - 1;
        const int32_t sj = __shfl(zi, lead);
        const double q = wide_pass<D>(A, sj, xb, zc, lane);
        const bool mine = valid && zi == sj;
        if (mine) {
            const double *e = cand + (int64_t)jo * CS;
            st.T = fma(-0.5, q, e[F + kFieldC]) + e[F + kFieldLogn1];
        }
        pend &= ~__ballot(mine);
    }
    const int K = A.ctl->K;
    const int32_t z0 = __builtin_amdgcn_readfirstlane(zi);
    const bool homog = __ballot(valid && zi != z0) == 0;
    for (int j = 0; j < K; ++j) {
        const double *e = cand + (int64_t)j * CS;  // wave-uniform: scalar loads
        const int32_t sj = (int32_t)e[F + kFieldSlot];
        if (homog && sj == z0) continue;
        const double q = wide_pass<D>(A, sj, xb, zc, lane);
        if (sj != zi) pick_step(st, fma(-0.5, q, e[F + kFieldC]) + e[F + kFieldLogn], j);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) pick_step(st, lwa[m], K + m);
    if (!valid) return;

    RecHeader *hdr = reinterpret_cast<RecHeader *>(A.rec);
    int32_t *delta = reinterpret_cast<int32_t *>(A.rec + kRecHeaderBytes);
    const int32_t snew = (st.pick < K) ? (int32_t)cand[(int64_t)st.pick * CS + F + kFieldSlot] : -1;
    const uint64_t mv = __ballot(snew != zi);
    if (mv && lane == (__ffsll((unsigned long long)__ballot(1)) - 1))
        atomicAdd(reinterpret_cast<unsigned long long *>(&A.ctl->moved), (unsigned long long)__popcll(mv));
    if (st.pick < K) {
        if (snew != zi) {
            atomicSub(delta + zi, 1);
            atomicAdd(delta + snew, 1);
            A.z[il] = snew;
            if (sorted) zs[pc] = snew;
        }
    } else {
        const int q = atomicAdd(&hdr->nreq, 1);
        if (q < A.rec_cap) {
            Request *req = reinterpret_cast<Request *>(A.rec + kRecHeaderBytes + (int64_t)A.kcap * 4);
            Request r;
            r.pos = sorted ? (int64_t)ig : A.offset + p;
            r.i = (int64_t)ig;
            r.m = st.pick - K;
            r.zold = zi;
            r.lpos = sorted ? (int32_t)pc : -1;
            r.pad = 0;
            req[q] = r;
            double *vmu = reinterpret_cast<double *>(A.rec + record_vmu_offset(A.kcap, A.rec_cap)) + (int64_t)q * (D + 1);
            wide_frame_payload<D>(hyp, X, n, xr, vmu);
        }
    }
}

// ---- max likelihood and parity ---------------------------------------------------------------------
// q of item x (fp32 values) against slot sj in the frame of its own slot sk, on the vector ALU:
// the same fmaf chains (zero terms of the triangular A skipped) and the same fp64 summation order.
template <int D>
__device__ double wide_q_valu(const WideArgs &W, const float *__restrict__ X, int64_t n, int64_t xr, int sk, int sj) {
    const float *Aj = W.wA + (int64_t)sj * D * D;
    const float *mk = W.wmu + (int64_t)sk * D;
    const float *g = W.gtab + ((int64_t)sj * W.kcap + sk) * D;
    float xt[D];
#pragma unroll
    for (int b = 0; b < D; ++b) xt[b] = X[(int64_t)b * n + xr] - mk[b];
    double s[2] = {0.0, 0.0};
#pragma unroll
    for (int mt = 0; mt < D / 32; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int a = 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * hh;
                float v = -g[a];
                for (int b = a; b < D; ++b) v = fmaf(Aj[(int64_t)a * D + b], xt[b], v);
                const double dv = (double)v;
                s[hh] = fma(dv, dv, s[hh]);
            }
    return s[0] + s[1];
}

template <int D>
__global__ __launch_bounds__(256) void np8_loglik_wide(LoglikArgs L, WideArgs W) {
    constexpr int CS = Wide<D>::CS, F = Wide<D>::F;
    __shared__ double red[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double ll = 0.0;
    if (i < L.n_loc) {
        const int32_t s = L.z[i];
        const double *e = L.cand + (int64_t)L.dense_of[s] * CS;
        ll = fma(-0.5, wide_q_valu<D>(W, reinterpret_cast<const float *>(L.X), L.n_loc, i, s, s), e[F + kFieldC]);
    }
    red[threadIdx.x] = ll;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) L.partial[blockIdx.x] = red[0];
}

template <int D, int M, int PRIOR>
__global__ __launch_bounds__(64) void np8_loglik_matrix_wide(AssignArgs A, WideArgs W, const int64_t *__restrict__ idx,
                                                             int64_t n, double *__restrict__ out) {
    constexpr int CS = Wide<D>::CS, F = Wide<D>::F;
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t il = idx[r];
    const float *X = reinterpret_cast<const float *>(A.X);
    const int K = A.ctl->K;
    const int32_t sk = A.z[il];
    for (int j = 0; j < K; ++j) {
        const double *e = A.cand + (int64_t)j * CS;
        out[r * (K + M) + j] = fma(-0.5, wide_q_valu<D>(W, X, A.n_loc, il, sk, (int)e[F + kFieldSlot]), e[F + kFieldC]);
    }
    float xf[D];
    for (int a = 0; a < D; ++a) xf[a] = X[(int64_t)a * A.n_loc + il];
    const double ny = wide_whiten_norm<D>(A.hyp, xf);
    const uint32_t t = A.ctl->t_base + A.t;
    for (int m = 0; m < M; ++m) out[r * (K + M) + K + m] = wide_aux_ll<D, PRIOR>(A.hyp, ny, A.seed, (uint64_t)(A.offset + il), t, m);
}

// ---- dispatch ----------------------------------------------------------------------------------------
#define NP8_WIDE_FOR_EACH(X) X(32, 3) X(64, 3)

bool np8_wide_supported(int D, int M) {
#define X(d, m) \
    if (D == d && M == m) return true;
    NP8_WIDE_FOR_EACH(X)
#undef X
    return false;
}

hipError_t np8_launch_assign_wide(const AssignArgs &A, int D, int M, int prior, hipStream_t s) {
    const int64_t n = A.p1 - A.p0;
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
#define X(d, m)                                                                                 \
    if (D == d && M == m) {                                                                     \
        if (prior == kPriorNiw)                                                                 \
            hipLaunchKernelGGL((np8_assign_wide<d, m, kPriorNiw>), grid, block, 0, s, A);       \
        else                                                                                    \
            hipLaunchKernelGGL((np8_assign_wide<d, m, kPriorReference>), grid, block, 0, s, A); \
        return hipGetLastError();                                                               \
    }
    NP8_WIDE_FOR_EACH(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_loglik_matrix_wide(const AssignArgs &A, const WideArgs &W, int D, int M, int prior,
                                         const int64_t *idx, int64_t n, double *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 63) / 64)), block(64);
#define X(d, m)                                                                                                    \
    if (D == d && M == m) {                                                                                        \
        if (prior == kPriorNiw)                                                                                    \
            hipLaunchKernelGGL((np8_loglik_matrix_wide<d, m, kPriorNiw>), grid, block, 0, s, A, W, idx, n, out);   \
        else                                                                                                       \
            hipLaunchKernelGGL((np8_loglik_matrix_wide<d, m, kPriorReference>), grid, block, 0, s, A, W, idx, n, \
                               out);                                                                               \
        return hipGetLastError();                                                                                  \
    }
    NP8_WIDE_FOR_EACH(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_loglik_wide(const LoglikArgs &L, const WideArgs &W, int D, hipStream_t s) {
    const int64_t nb = (L.n_loc + 255) / 256;
    if (nb <= 0) return hipSuccess;
    if (D == 32)
        hipLaunchKernelGGL((np8_loglik_wide<32>), dim3((unsigned)nb), dim3(256), 0, s, L, W);
    else if (D == 64)
        hipLaunchKernelGGL((np8_loglik_wide<64>), dim3((unsigned)nb), dim3(256), 0, s, L, W);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t np8_launch_wide_refresh(const WideArgs &W, hipStream_t s) {
    hipLaunchKernelGGL(np8_wide_rows, dim3((unsigned)W.kcap), dim3(256), sizeof(double) * W.D * W.D, s, W);
    hipLaunchKernelGGL(np8_wide_gtab, dim3((unsigned)W.kcap, (unsigned)((W.kcap + 3) / 4)), dim3(256), 0, s, W);
    hipLaunchKernelGGL(np8_wide_clean, dim3((unsigned)((W.kcap + 255) / 256)), dim3(256), 0, s, W);
    return hipGetLastError();
}
