// np8_wide.hip -- the wide path (DESIGN.md "Wide path"; BASELINE.json config C5): 16 < D <= 80 (kernels instantiated
// for DT = D rounded up to 16 in {32, 48, 64, 80}; item rows, factors and means beyond D are zero), items
// held in fp32, cluster likelihoods through fp32 MFMA (v_mfma_f32_16x16x4_f32, exact k-ordered fmaf
// chains), everything else (auxiliary draws, the categorical pick, counts) in fp64 as on the narrow path.
//
//   np8_wide_rows     per slot whose parameters changed: R = chol_upper(sym Sigma^{-1}) (fp64, in LDS),
//                     A = fp32(R) in natural and MFMA-fragment order, muf = fp32(mu) (natural and
//                     fragment order); clears the change flags
//   np8_assign_wide   4 waves x 64 items per block (one lane per item for the fp64 parts): per candidate
//                     row the 64 x D x D contraction y = A_j (x - muf_j) on the matrix cores, q = |y|^2 in
//                     fp64, then the single-uniform reservoir pick of np8_assign (src/np_neal_algorithm8.cpp:
//                     49-167 for every item); the candidate rows stream through a double-buffered LDS stage
//                     shared by the block's waves
//   np8_loglik_wide / np8_loglik_matrix_wide   the same arithmetic on the vector ALU (bit-identical:
//                     an MFMA is an fmaf chain) for the max-likelihood sum and the parity debug entry
//
// The contraction is specified in oracle/np8_oracle.h (NP8O_CONTRACT_F32) so that the CPU oracle
// reproduces it bit for bit.  A is upper triangular: 16-row tile mt skips the k-steps of columns < 16 mt
// (2560 instead of 4096 multiply-adds per item and candidate at D = 64).
#include "np8_kernels.h"

#include <hip/hip_runtime.h>

using namespace np8;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int D>
struct Wide {
    static constexpr int MT = D / 16;  // 16-row tiles of A (and 16-item column tiles: 4 per wave)
    static constexpr int S = D / 4;    // k-steps of the 16x16x4 MFMA
    static constexpr int S4 = S / 4;   // float4 groups of k-steps per lane
    static constexpr int DP = D * (D + 1) / 2;
    static constexpr int CS = (D + DP + 5 + 1) & ~1;
    static constexpr int F = D + DP;
    // used fragment chunks (1 KB = one float4 per lane): (mt, s4) with s4 >= mt, compact order
    static constexpr int NCH = MT * (MT + 1) / 2;
    static constexpr int ROW = NCH * 256 + D;  // floats per candidate row: chunks | muf transposed
    static __host__ __device__ constexpr int chunk(int mt, int s4) { return mt * S4 - (mt * (mt - 1)) / 2 + (s4 - mt); }
};

__device__ __forceinline__ int64_t wpos_to_local(const AssignArgs &A, int64_t p) {
    if (A.order) return A.order[p];
    if (A.use_perm) return (int64_t)perm_apply(A.perm, (uint32_t)p);
    return p;
}

// |U^T (x - mu0)| with U^T packed upper in hyp (the item frame of the auxiliary draws): the loop order
// of whiten() + norm_of(); the whitened vector itself is never stored.
// uw: mu0 and U^T packed for DT (AssignArgs::uw; zero beyond D, as the item rows): the extra terms are exact zeros,
// fma(0, 0, t) = t, so the norm is the one over the data's D dims.
template <int DT>
__device__ __forceinline__ double wide_whiten_norm(const double *__restrict__ uw, const float (&xf)[DT]) {
    const double *U = uw + DT;
    double dx[DT];
#pragma unroll
    for (int a = 0; a < DT; ++a) dx[a] = (double)xf[a] - uw[a];
    double n2 = 0.0;
    int k = 0;
#pragma unroll
    for (int a = 0; a < DT; ++a) {  // fully unrolled: register operands, U through the scalar cache
        double t0 = U[k++] * dx[a];
#pragma unroll
        for (int b = a + 1; b < DT; ++b) t0 = fma(U[k++], dx[b], t0);
        n2 = fma(t0, t0, n2);
    }
    return sqrt(n2);
}

// The request payload of the wide path: (|y0|, y0) with y0 = U^T (x - mu0), read from global memory.
__device__ void wide_frame_payload(const double *__restrict__ hyp, int D, const float *__restrict__ X, int64_t n,
                                   int64_t xr, double *vmu) {
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

template <int PRIOR>
__device__ __forceinline__ double wide_aux_ll(const double *__restrict__ hyp, int D, double ny, uint64_t seed,
                                              uint64_t ig, uint32_t t, int m, int M) {
    const int DP = D * (D + 1) / 2;
    const double caux = hyp[D + DP], rsk = hyp[D + DP + 1], nu = hyp[D + DP + 3];
    if constexpr (PRIOR == kPriorNiw) {
        double sumlog, b00, chi, z1;
        niw_aux_core(seed, ig, t, m, D, nu, sumlog, b00, chi, z1);
        return niw_aux_loglik(ny, sumlog, b00, chi, z1, rsk, caux);
    } else {
        double v, xpar, chi2;
        aux_core_rt(seed, ig, t, m, M, D, nu, v, xpar, chi2);
        return aux_loglik(ny, v, xpar, chi2, D, rsk, caux);
    }
}

// q for the lane's item (item index = lane) against a candidate row staged at `row` (A fragments,
// then muf transposed: row[D*D + g*S + s] = muf[4 s + g]); xb holds the raw items of the wave's four
// 16-item column tiles (lane l: item 16 nt + (l & 15), dims 4 s + (l >> 4)).
// Column tile nt, row tile mt: lane group g = l >> 4 holds rows 16 mt + 4 g + r (r = 0..3) of item
// 16 nt + (l & 15); s_g = fp32 fmaf chain of y^2 over (mt, r); q = (s_0 + s_1) + (s_2 + s_3) in fp32.
template <int D>
__device__ __forceinline__ double wide_pass(const float *row, const float (&xb)[4][D / 4], int lane) {
    using W = Wide<D>;
    const int g = lane >> 4;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    // row tiles one after another (mt outer): four live accumulators (one per column tile) instead of
    // MT x 4; each accumulator still receives its k-steps in ascending order, and the squares enter the
    // fmaf chains s_g in (mt, r) order as before -- the same arithmetic, 48 fewer registers at D = 64
    float sacc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const float *mut = row + W::NCH * 256 + g * W::S;
#pragma unroll
    for (int mt = 0; mt < W::MT; ++mt) {
        f32x4 acc[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[nt] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s4 = mt; s4 < W::S4; ++s4) {  // A upper triangular: columns < 16 mt of row tile mt are zero
            const float4 m4 = *reinterpret_cast<const float4 *>(mut + 4 * s4);
            const float mv[4] = {m4.x, m4.y, m4.z, m4.w};
            const float4 a4 = *reinterpret_cast<const float4 *>(row + (W::chunk(mt, s4) * 64 + lane) * 4);
            const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
                    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], xb[nt][4 * s4 + e] - mv[e], acc[nt], 0, 0, 0);
        }
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) sacc[nt] = fmaf(acc[nt][r], acc[nt][r], sacc[nt]);
    }
    const float sp[4] = {sacc[0], sacc[1], sacc[2], sacc[3]};
    // 4 x 4 transpose across the lane groups (lane group g, register k) -> (group k's partial of
    // column tile g): the half exchanges of permlane32_swap then permlane16_swap
    const auto r02 = __builtin_amdgcn_permlane32_swap(__float_as_uint(sp[0]), __float_as_uint(sp[2]), false, false);
    const auto r13 = __builtin_amdgcn_permlane32_swap(__float_as_uint(sp[1]), __float_as_uint(sp[3]), false, false);
    const auto r01 = __builtin_amdgcn_permlane16_swap(r02[0], r13[0], false, false);
    const auto r23 = __builtin_amdgcn_permlane16_swap(r02[1], r13[1], false, false);
    const float q = (__uint_as_float(r01[0]) + __uint_as_float(r01[1])) +
                    (__uint_as_float(r23[0]) + __uint_as_float(r23[1]));
    (void)g;
    return (double)q;
}

// The block's 256 threads copy one candidate row (A fragments + transposed muf of slot sj) from HBM
// straight into an LDS stage (global_load_lds_dwordx4, no registers): wave w moves the 1 KB chunks
// w, w + 4, ... of the A fragments, wave 0's first D/4 lanes the muf part.  The LDS image equals the
// HBM row (lane-linear 16-byte pieces).  Landed once the block passes a __syncthreads().
template <int D>
__device__ __forceinline__ void row_glds(const float *__restrict__ wfrag, int sj, float *dst) {
    constexpr int NCH = Wide<D>::NCH;
    const float4 *src = reinterpret_cast<const float4 *>(wfrag + (int64_t)sj * Wide<D>::ROW);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < (NCH + 3) / 4; ++k) {
        const int c = w + 4 * k;  // wave-uniform
        if (c < NCH)
            __builtin_amdgcn_global_load_lds((const void *)(src + 64 * c + lane),
                                             (__attribute__((address_space(3))) void *)(dst + 256 * c), 16, 0, 0);
    }
    if (w == 3 && lane < D / 4)  // the wave with the fewest chunks
        __builtin_amdgcn_global_load_lds((const void *)(src + 64 * NCH + lane),
                                         (__attribute__((address_space(3))) void *)(dst + 256 * NCH), 16, 0, 0);
}

}  // namespace

// Fx through a lane shuffle (four 32-bit pieces)
__device__ __forceinline__ Fx wfx_shfl_xor(Fx a, int o) {
    const uint32_t l0 = (uint32_t)__shfl_xor((int)(uint32_t)a.lo, o), l1 = (uint32_t)__shfl_xor((int)(uint32_t)(a.lo >> 32), o);
    const uint32_t h0 = (uint32_t)__shfl_xor((int)(uint32_t)(uint64_t)a.hi, o),
                   h1 = (uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)a.hi >> 32), o);
    Fx r;
    r.lo = ((uint64_t)l1 << 32) | l0;
    r.hi = (int64_t)(((uint64_t)h1 << 32) | h0);
    return r;
}

// ---- table maintenance ---------------------------------------------------------------------------
constexpr int kLamRounds = 5;  // eigenvalue-bound rounds of three concurrent Cholesky tests: 4^5 = 1024 steps
#ifndef NP8_LAM_REL_WIDTH
#define NP8_LAM_REL_WIDTH 0.05  // 2%: C5 niw_conjugate 638 vs 675 sweeps/s, the bound 3% looser at most, contractions unchanged
#endif
constexpr double kLamRelWidth = NP8_LAM_REL_WIDTH;  // ... or fewer, once the bracket [lo, hi] is within 5% of hi

// One block of four waves per slot (grid kcap): the slots flagged in wdirty get their factor, its eigenvalue bound
// and their fp32 mean.  The factor and the eigenvalue bound's Cholesky tests run blocked, right-looking, 16 columns
// per panel: one wave factors a panel with its 16 rows in registers (lane = column, pivots and row entries by
// readlane), then all 256 threads apply the panel's 16 updates to the rows below, each element's fma chain in
// ascending column order -- the operations of the unblocked form (and of the oracle) in their order, with two
// workgroup barriers per panel instead of two per column.  Waves 0..3 factor panels of four matrices at once: P
// (wave 0) and P - beta_q I for the three betas of an eigenvalue round (waves 1-3).
// LDS: four [D][D + 1] double matrices (133 KB at D = 64): the factor's work matrix (R in place), three tests.
constexpr int kPanel = 16;
// Cholesky tests np8_wide_rows runs beside the factor: three, or two when four D x (D + 1) doubles exceed the LDS.
__host__ __device__ constexpr int wide_rows_tests(int D) { return D <= 64 ? 3 : 2; }

// Panel p of matrix M (rows c0 .. c0 + 15, columns c0 .. D - 1) on one wave, lane = column (and lane + 64 above
// D = 64: a second register set).  Factor form (test = false): row jj of R = row jj / sqrt(pivot); a non-positive pivot
// is replaced by 1e-300 and its column skips every update (np8_wide_rows' error path), bit q of *skip.  Test form: the
// row is kept unscaled, rk[j] = 1 / sqrt(pivot) scales both factors of each update; a non-positive pivot ends the test
// (*fail).  Each column's chain is the same whichever register set holds it.
__device__ __forceinline__ void panel_factor(double *M, int LD, int D, int c0, bool test, double *rk, int *skip,
                                             int *fail) {
    const int lane = threadIdx.x & 63, l2 = lane + 64;
    const bool two = D > 64;
    double w[kPanel], u[kPanel];
#pragma unroll
    for (int i = 0; i < kPanel; ++i) {
        w[i] = (lane < D && c0 + i < D) ? M[(c0 + i) * LD + lane] : 0.0;
        u[i] = (two && l2 < D && c0 + i < D) ? M[(c0 + i) * LD + l2] : 0.0;
    }
    // element (row j of the panel, column c), c wave-uniform
    auto col = [&](double wj, double uj, int c) { return c < 64 ? __shfl(wj, c) : __shfl(uj, c - 64); };
    int sk = 0, fl = 0;
#pragma unroll
    for (int j = 0; j < kPanel; ++j) {
        const int jj = c0 + j;
        if (jj >= D) break;  // (the last panel of a D that is not a multiple of 16)
        const double v = col(w[j], u[j], jj);  // the pivot (row jj, column jj)
        if (test) {
            if (!(v > 0.0) || fl) {
                fl = 1;
                continue;
            }
            const double r = 1.0 / sqrt(v);
            if (lane == 0) rk[j] = r;
            const double rowj = w[j] * r, rowj2 = u[j] * r;  // C[jj][l] r
#pragma unroll
            for (int i = j + 1; i < kPanel; ++i) {
                const double ci = col(w[j], u[j], c0 + i) * r;  // C[jj][ii] r
                if (lane >= c0 + i) w[i] = fma(-ci, rowj, w[i]);
                if (two && l2 >= c0 + i) u[i] = fma(-ci, rowj2, u[i]);
            }
        } else {
            const bool ok = v > 0.0;
            const double dj = ok ? sqrt(v) : 1e-300;
            if (!ok) sk |= 1 << j;
            if (lane == jj) w[j] = dj;
            if (lane > jj) w[j] = ok ? w[j] / dj : 0.0;  // row jj of R (zero after a failed pivot)
            if (two) {
                if (l2 == jj) u[j] = dj;
                if (l2 > jj) u[j] = ok ? u[j] / dj : 0.0;
            }
            if (ok) {
#pragma unroll
                for (int i = j + 1; i < kPanel; ++i) {
                    const double rji = col(w[j], u[j], c0 + i);  // R[jj][ii]
                    if (lane >= c0 + i) w[i] = fma(-rji, w[j], w[i]);
                    if (two && l2 >= c0 + i) u[i] = fma(-rji, u[j], u[i]);
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < kPanel; ++i) {
        if (lane < D && lane >= c0 + i && c0 + i < D) M[(c0 + i) * LD + lane] = w[i];
        if (two && l2 < D && l2 >= c0 + i && c0 + i < D) M[(c0 + i) * LD + l2] = u[i];
    }
    if (lane == 0) {
        *skip = sk;
        *fail = fl;
    }
}

// The panel's 16 updates to element (ii, l), ii >= c0 + 16, l >= ii, in ascending column order; all threads.
__device__ __forceinline__ void panel_trailing(double *M, int LD, int D, int c0, bool test, const double *rk, int skip) {
    const int rows = D - (c0 + kPanel);
    for (int e = threadIdx.x; e < rows * D; e += blockDim.x) {
        const int ii = c0 + kPanel + e / D, l = e - (e / D) * D;
        if (l < ii) continue;
        double acc = M[ii * LD + l];
#pragma unroll
        for (int j = 0; j < kPanel; ++j) {
            const int k = c0 + j;
            if (test)
                acc = fma(-(M[k * LD + ii] * rk[j]), M[k * LD + l] * rk[j], acc);
            else if (!((skip >> j) & 1))
                acc = fma(-M[k * LD + ii], M[k * LD + l], acc);
        }
        M[ii * LD + l] = acc;
    }
}

#ifdef NP8_EXP_WIDE_TIMING  // experiment: phase cycle counts of np8_wide_rows, blocks 0 and 1, printed
#define WR_T(k) \
    if (threadIdx.x == 0 && (k) < 16) tph[k] = (long long)__builtin_amdgcn_s_memtime();
#else
#define WR_T(k)
#endif
__device__ void wide_rows_slot(const WideArgs &W, const int s) {
#ifdef NP8_EXP_WIDE_TIMING
    long long tph[16];
    for (int k = 0; k < 16; ++k) tph[k] = 0;
    int nrd = 0;
#endif
    WR_T(0)
    if (W.cnt[s] <= 0) return;  // block-uniform
    const int D = W.D, LD = D + 1, tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nq = wide_rows_tests(D);  // concurrent Cholesky tests: three, two above D = 64 (LDS)
    extern __shared__ __attribute__((aligned(16))) double smr[];
    double *Wk = smr, *C0 = Wk + D * LD;  // C0 + q * D * LD: test matrix q; R = the upper triangle of Wk at the end
    const double *Pp = W.slot_P + (int64_t)s * (D * (D + 1) / 2);
    auto pget = [&](int a, int b) {  // sym(P) upper element, a <= b (the packed P' doubles off-diagonals)
        const double v = Pp[a * D - (a * (a - 1)) / 2 + (b - a)];
        return (a == b) ? v : 0.5 * v;
    };
    __shared__ double dmin;
    __shared__ double rk_s[4][kPanel];
    __shared__ int skip_s[4], fail_s[4];
    if (tid == 0) dmin = 1e300;
    __syncthreads();
    for (int k = tid; k < D * D; k += blockDim.x) {
        const int a = k / D, b = k - a * D;
        const double v = (b >= a) ? pget(a, b) : 0.0;
        Wk[a * LD + b] = v;
        if (a == b && W.lam_lo) atomicMin(reinterpret_cast<unsigned long long *>(&dmin), (unsigned long long)__double_as_longlong(v));
    }
    __syncthreads();
    // candidate pruning: lam_lo <= the smallest eigenvalue of P, by Cholesky tests of P - beta I (positive definite
    // <=> lambda_min(P) > beta) on [0, min_i P_ii]: each round tests three betas at once (quarter points; the first
    // round brackets the slot's last bound); the first round runs beside the factor
    const bool lam = W.lam_lo != nullptr;
    double lo = 0.0, hi = lam ? dmin : 0.0;
    const double prev = lam ? W.lam_lo[s] / 0.99 : 0.0;
    const bool warm = prev > 0.0 && prev < hi;
    bool factor = true;  // the first pass also factors P
    int err = 0;
    WR_T(1)
    for (int rd = 0; rd < (lam ? kLamRounds : 1); ++rd) {  // block-uniform
        const bool tests = lam && hi > lo;
        double beta[3] = {0.0, 0.0, 0.0};
        if (tests) {
            if (rd == 0 && warm) {
                beta[0] = 0.93 * prev;
                beta[1] = 0.98 * prev;
                beta[2] = fmin(1.02 * prev, 0.5 * (prev + hi));
                if (nq == 2) beta[1] = beta[2];
            } else {
#pragma unroll
                for (int q = 0; q < 3; ++q) beta[q] = lo + (hi - lo) * ((double)(q + 1) / (nq + 1));
            }
            for (int k = tid; k < nq * D * D; k += blockDim.x) {
                const int q = k / (D * D), kk = k - q * D * D, a = kk / D, b = kk - a * D;
                if (b >= a) C0[q * D * LD + a * LD + b] = (a == b) ? pget(a, a) - beta[q] : pget(a, b);
            }
            if (tid < 4) fail_s[tid] = (tid < 3 && tid >= nq) ? 1 : 0;  // (a test not run: "not positive definite")
            __syncthreads();
        }
        if (!factor && !tests) break;
        for (int p = 0; p * kPanel < D; ++p) {
            const int c0 = p * kPanel;
            // panel steps: wave 0 the factor (first pass), wave q + 1 test q (a failed test stops)
            if (wv == 0 && factor) {
                panel_factor(Wk, LD, D, c0, false, nullptr, &skip_s[0], &fail_s[3]);
            } else if (wv > 0 && wv <= nq && tests && !fail_s[wv - 1]) {
                int dummy;
                panel_factor(C0 + (wv - 1) * D * LD, LD, D, c0, true, rk_s[wv], &dummy, &fail_s[wv - 1]);
            }
            __syncthreads();
            if (factor) {
                err |= skip_s[0];
                panel_trailing(Wk, LD, D, c0, false, nullptr, skip_s[0]);
            }
            if (tests)
                for (int q = 0; q < nq; ++q)
                    if (!fail_s[q]) panel_trailing(C0 + q * D * LD, LD, D, c0, true, rk_s[q + 1], 0);
            __syncthreads();
        }
        if (factor && err && tid == 0) atomicOr(&W.ctl->err, kErrSigma);
        factor = false;
#ifdef NP8_EXP_WIDE_TIMING
        ++nrd;
        WR_T(1 + nrd)
#endif
        if (!tests) break;
        // positive definiteness is monotone in beta: the largest positive definite beta is the new lower end
        const int pd = (!fail_s[0]) | ((!fail_s[1]) << 1) | ((!fail_s[2]) << 2);
        const int top = (pd & 4) ? 3 : (pd & 2) ? 2 : (pd & 1) ? 1 : 0;
        if (top > 0) lo = beta[top - 1];
        if (top < nq) hi = beta[top];
        __syncthreads();  // (fail_s read by every thread before the next round resets it)
        if (hi - lo <= kLamRelWidth * hi) break;  // block-uniform
    }
    // 1% for the fp32 factor and the fp32 contraction, and the Cholesky's own rounding
    if (lam && tid == 0) W.lam_lo[s] = 0.99 * lo;
    const int DT = W.DT, NCH = (DT / 16) * (DT / 16 + 1) / 2;
    wide_write_rows(D, DT, Wk, LD, W.slot_mu + (int64_t)s * D, W.wA + (int64_t)s * DT * DT,
                    W.wfrag + (int64_t)s * (NCH * 256 + DT), W.wmu + (int64_t)s * DT);
#ifdef NP8_EXP_WIDE_TIMING
    WR_T(15)
    if (tid == 0 && s < 3)
        printf("wide_rows s=%d rounds %d load %lld r1 %lld r2 %lld r3 %lld r4 %lld r5 %lld out %lld total %lld\n", s, nrd,
               tph[1] - tph[0], tph[2] - tph[1], nrd > 1 ? tph[3] - tph[2] : 0, nrd > 2 ? tph[4] - tph[3] : 0,
               nrd > 3 ? tph[5] - tph[4] : 0, nrd > 4 ? tph[6] - tph[5] : 0, tph[15] - tph[1 + nrd], tph[15] - tph[0]);
#endif
}

// The slots flagged in wdirty, each by one block in turn (a grid of at most one block per CU: the factor's LDS
// allows one per CU anyway, and a sweep that changed no slot costs one round of blocks instead of kcap / 256); the
// flags are cleared as they are taken.
constexpr int kWideRowsBlocks = 256;
__global__ __launch_bounds__(256) void np8_wide_rows(WideArgs W) {
    for (int s = blockIdx.x; s < W.kcap; s += gridDim.x) {
        if (!W.dirty[s]) continue;  // block-uniform
        __syncthreads();            // every thread has read the flag; the previous slot's LDS reads are done
        if (threadIdx.x == 0) W.dirty[s] = 0;
        wide_rows_slot(W, s);
    }
}

// Candidate pruning (DESIGN.md "Wide path"): distances between the fp32 means of the dense rows, in fp64,
// wdist[j0 * kcap + j].  One block per row j0 (a grid of kcap; rows >= K exit).  The means are read four at a
// time over all DT dims (zero beyond D: fma(0, 0, d2) = d2), every load of a row before the chain.
__global__ __launch_bounds__(256) void np8_wide_dist(WideArgs W) {
    const int K = W.ctl->K, j0 = blockIdx.x;
    if (j0 >= K) return;
    const int D = W.D, DP = D * (D + 1) / 2, CS = cand_stride(D), DT = W.DT;
    const int s0 = (int)W.cand[(int64_t)j0 * CS + D + DP + kFieldSlot];
    const float4 *m0 = reinterpret_cast<const float4 *>(W.wmu + (int64_t)s0 * DT);
    for (int j = threadIdx.x; j < K; j += blockDim.x) {
        const int sj = (int)W.cand[(int64_t)j * CS + D + DP + kFieldSlot];
        const float4 *mj = reinterpret_cast<const float4 *>(W.wmu + (int64_t)sj * DT);
        double d2 = 0.0;
        for (int a0 = 0; a0 < DT / 4; a0 += 4) {  // (DT / 4 is a multiple of 4)
            float4 v[4], u[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[q] = mj[a0 + q];
                u[q] = m0[a0 + q];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double d0 = (double)v[q].x - (double)u[q].x, d1 = (double)v[q].y - (double)u[q].y;
                const double e0 = (double)v[q].z - (double)u[q].z, e1 = (double)v[q].w - (double)u[q].w;
                d2 = fma(d0, d0, d2);
                d2 = fma(d1, d1, d2);
                d2 = fma(e0, e0, d2);
                d2 = fma(e1, e1, d2);
            }
        }
        W.wdist[(int64_t)j0 * W.kcap + j] = sqrt(d2);  // the distance itself: no square root per lane and row
    }
}

// ---- the sweep kernel -----------------------------------------------------------------------------
// Dynamic LDS: two candidate-row stages of Wide<D>::ROW floats (33 KB at D = 64).
// LL: a max-likelihood check sweep with the sum folded in (frozen parameters, one rank): each wave stores the exact sum
// of its items' log-likelihoods under their new labels in llpart (a requester under its old slot: np8_ll_fix_wide moves
// the accepted ones once their slots exist) -- np8_loglik_wide_mfma's values, the own and walked rows' q being the
// same contractions.
// (the assign's late-used arguments: np8_late_arg, as np8_assign_fast's NP8_LATE)
#ifdef NP8_EXP_EARLY_ARGS
#define NP8_WLATE(f) (A.f)
#else
#define NP8_WLATE(f) np8_late_arg<decltype(AssignArgs::f)>(offsetof(AssignArgs, f))
#endif
template <int DT, int M, int PRIOR, bool LL, bool EXACT>
#ifndef NP8_WIDE_WAVES
#define NP8_WIDE_WAVES 2
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NP8_WIDE_WAVES, NP8_WIDE_WAVES))) void np8_assign_wide(AssignArgs A) {
    using W = Wide<DT>;
    // the data's D (hyp, cand, records): EXACT = D is DT itself, a constant of the instance -- the pruning distance,
    // the auxiliaries' D chi^2 draws and every table offset fold (a runtime D cost C5's assign 235 -> 338 us)
    const int D = EXACT ? DT : A.dim, DP = D * (D + 1) / 2, CS = cand_stride(D), F = D + DP;
    extern __shared__ __attribute__((aligned(16))) float stage[];
    const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
    const int64_t pw = A.p0 + (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
    const bool wave_live = pw < A.p1;  // waves past the end still take part in the block's staging
    const int64_t p = pw + lane;
    const bool valid = p < A.p1;
    const bool sorted = A.sorted != 0;
    constexpr int cur = 0;  // the label-sorted layout is always buffer 0 (buffer 1: the re-sort's scratch)
    int32_t *__restrict__ zs = cur ? A.zs[1] : A.zs[0];
    const int32_t *__restrict__ ids = cur ? A.ids[1] : A.ids[0];
    const float *__restrict__ X = reinterpret_cast<const float *>(sorted ? (cur ? A.Xs[1] : A.Xs[0]) : A.X);
    const double *__restrict__ cand = A.cand;
    const double *__restrict__ hyp = A.hyp;
    const uint32_t t = A.ctl->t_base + A.t;
    const int64_t n = A.n_loc;
    const int K = A.ctl->K;

    // the lane's own item (lanes past the end of the range mirror the wave's first item)
    const int64_t pc = valid ? p : (wave_live ? pw : A.p0);
    const int64_t lk = sorted ? (int64_t)ids[pc] : wpos_to_local(A, pc);
    const int64_t il = key_item(lk);
    const int64_t xr = sorted ? pc : il;
    const uint64_t ig = (uint64_t)(A.offset + lk);  // item key: global index | visit << 32
    const int32_t zi = sorted ? zs[pc] : A.z[il];
    const int32_t jo = A.dense_of[zi];

    // the item's frame for the auxiliaries (|U^T (x - mu0)|) and |x|^2 (the exact distance screen): per item, once
    // per data set (np8_wide_frame, the kFrameRows rows after the item's DT rows) -- a general U^T's D (D + 1) / 2
    // products per lane stay out of the sweep
    const uint32_t *fr = reinterpret_cast<const uint32_t *>(X) + (int64_t)DT * n + xr;
    const double ny = __hiloint2double((int)fr[n], (int)fr[0]), x2 = __hiloint2double((int)fr[3 * n], (int)fr[2 * n]);
    double rown = 0.0;  // |x - muf_own| (candidate pruning)
    if (A.wdist) {
        const float *mo = A.wmu + (int64_t)zi * DT;
        double d2 = 0.0;
#pragma unroll 16
        for (int a = 0; a < D; ++a) {
            const double dd = (double)X[(int64_t)a * n + xr] - (double)mo[a];
            d2 = fma(dd, dd, d2);
        }
        rown = sqrt(d2);
    }

    // MFMA operand B: raw items 16 nt + col of the wave, dims 4 s + g
    float xb[4][W::S];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        int64_t pq = pw + nt * 16 + col;
        if (pq >= A.p1) pq = pc;  // padding column: any valid item, result unused
        const int64_t xq = sorted ? pq : key_item(wpos_to_local(A, pq));
#pragma unroll
        for (int st = 0; st < W::S; ++st) xb[nt][st] = X[(int64_t)(4 * st + g) * n + xq];
    }

    // own clusters first (weight n_k - 1): one pass per distinct own slot of the wave, rows read
    // straight from HBM (L2)
    PickState st;
    st.T = 0.0;
    st.S = 1.0;
    st.u = uniform(A.seed, ig, t, kStreamPick, 0);
    st.pick = jo;
    double ll_own = 0.0, llp = 0.0;  // (LL) ll under the own row and under the row picked so far
    uint64_t pend = wave_live ? __ballot(valid) : 0ull;
    int own_passes = 0;  // executed-work counters (count_eval): the own-row passes of this wave
    while (pend) {
        ++own_passes;
        const int lead = __ffsll((unsigned long long)pend) - 1;
        const int32_t sj = __shfl(zi, lead);
        const double q = wide_pass<DT>(A.wfrag + (int64_t)sj * W::ROW, xb, lane);
        const bool mine = valid && zi == sj;
        if (mine) {
            const double *e = cand + (int64_t)jo * CS;
            const double llo = fma(-0.5, q, e[F + kFieldC]);
            st.T = llo + e[F + kFieldLogn1];
            if (LL) ll_own = llp = llo;
        }
        pend &= ~__ballot(mine);
    }

    // the auxiliaries (fp64, per lane), after the own row: with the NIW prior each is screened against
    // T_own - kSkip (the pick's T only grows), so most of them skip their D chi^2 draws
    double lwa[M];
    {
        const double logam = hyp[D + DP + 2];
        bool all_below = false;  // (level 0: no auxiliary of this item can reach the skip threshold, whatever its draws)
        if constexpr (PRIOR == kPriorNiw)
            all_below = niw_aux_all_below(ny, hyp[D + DP + 3], hyp[D + DP + 1], hyp[D + DP],
                                          hyp[D + DP + 4 + DP], st.T - kSkip - logam);
#pragma unroll
        for (int k = 0; k < M; ++k) lwa[k] = kZeroLogWeight + logam;
#pragma unroll 1
        for (int m = 0; m < (all_below ? 0 : M); ++m) {
            double v;
            if constexpr (PRIOR == kPriorNiw) {
                const double caux = hyp[D + DP], rsk = hyp[D + DP + 1], nu = hyp[D + DP + 3];
                const double smax = hyp[D + DP + 4 + DP];
                v = niw_aux_ll_screened(A.seed, ig, t, m, D, nu, ny, rsk, caux, smax, st.T - kSkip - logam) + logam;
            } else {
                v = wide_aux_ll<PRIOR>(hyp, D, ny, A.seed, ig, t, m, M) + logam;
            }
#pragma unroll
            for (int k = 0; k < M; ++k) lwa[k] = (k == m) ? v : lwa[k];  // no dynamic register index
        }
    }

    // candidate pruning: a row is evaluated for the block when one of its items may pick it.  For lane x
    // with running maximum T >= lw_own(x): lw_j(x) <= c_j + log n_j - lam_j (|mu_j - mu_own| - |x - mu_own|)^2 / 2
    // (triangle inequality, lam_j <= the smallest eigenvalue of row j's precision); a row below T - 80 - 2
    // (and a relative margin) for every lane is one its pick_step would skip -- results unchanged.
    // kMaskWords: up to 64 * 8 = 512 rows (kcap of the wide path).  The rows' scalars (slot, c + log n, lam / 2) are
    // staged in LDS once per block, and the rows each stage keeps are compacted into a list (no bit scans per row).
    constexpr int kMaskWords = 8, kRowsMax = 64 * kMaskWords;
    __shared__ unsigned long long rmask[kMaskWords], rmask2[kMaskWords];
    __shared__ int32_t rslot[kRowsMax];
    __shared__ double rbase[kRowsMax], rlamh[kRowsMax];
    __shared__ int16_t rlist[2][kRowsMax];
    __shared__ int rlist_n[2];
    const bool prune = A.wdist != nullptr && K <= kRowsMax;
    // the rows set in mask m, ascending, into list (all threads; a barrier before the list is read)
    auto compact = [&](const unsigned long long *m, int16_t *list, int *cnt) {
        for (int j = threadIdx.x; j < K; j += blockDim.x) {
            const int w = j >> 6, bit = j & 63;
            const unsigned long long mw = m[w];
            if ((mw >> bit) & 1ull) {
                int pos = __popcll(mw & ((1ull << bit) - 1ull));
                for (int v = 0; v < w; ++v) pos += __popcll(m[v]);
                list[pos] = (int16_t)j;
            }
        }
        if (threadIdx.x == 0) {
            int c = 0;
            for (int v = 0; v < kMaskWords; ++v) c += __popcll(m[v]);
            *cnt = c;
        }
    };
    if (prune) {
        for (int j = threadIdx.x; j < K; j += blockDim.x) {
            const double *e = cand + (int64_t)j * CS;
            const int32_t sj = (int32_t)e[F + kFieldSlot];
            rslot[j] = sj;
            rbase[j] = e[F + kFieldC] + e[F + kFieldLogn];
            rlamh[j] = 0.5 * A.lam_lo[sj];
        }
        if (threadIdx.x < kMaskWords) rmask[threadIdx.x] = rmask2[threadIdx.x] = 0ull;
        __syncthreads();
        // per distinct own row of the wave (one in the label-sorted layout): the group's largest radius and
        // smallest running maximum bound every lane of the group at once (U grows with |x - mu_own| and falls
        // with T), then lane l decides rows l, l + 64, ... -- ceil(K/64) bounds per group instead of K per lane
        uint64_t pend = wave_live ? __ballot(valid) : 0ull;
        while (pend) {
            const int lead = __ffsll((unsigned long long)pend) - 1;
            const int32_t zg = __shfl(zi, lead);
            const int32_t jg = __shfl(jo, lead);
            const bool in = valid && zi == zg;
            double rmax = in ? rown : 0.0, tmin = in ? st.T : 1e300;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                rmax = fmax(rmax, __shfl_xor(rmax, o));
                tmin = fmin(tmin, __shfl_xor(tmin, o));
            }
            pend &= ~__ballot(in);
            for (int jb = 0; jb < K; jb += 64) {
                const int j = jb + lane;
                bool need = false;
                if (j < K && rslot[j] != zg) {
                    const double base = rbase[j];
                    const double gap = fmax(A.wdist[(int64_t)jg * A.kcap + j] - rmax, 0.0);
                    const double far = rlamh[j] * gap * gap;
                    const double U = base - far - tmin;
                    need = !(U <= -kSkip - 2.0 - 1e-9 * (fabs(base) + fabs(tmin) + far));
                }
                const uint64_t b = __ballot(need);
                if (b != 0ull && lane == 0) atomicOr(&rmask[jb >> 6], b);
            }
        }
        __syncthreads();
        compact(rmask, rlist[0], &rlist_n[0]);
        __syncthreads();
    }
    // The exact-distance screen of the rows the mask kept (DESIGN.md §5 "Wide-path pruning"): per item and row,
    // lw_j(x) <= c_j + log n_j - lam_j |x - muf_j|^2 / 2 with the distance itself, |x|^2 + |muf_j|^2 - 2 x.muf_j,
    // the dot products of 16 rows and the wave's 64 items on the matrix cores (D/4 MFMAs per item tile and 16
    // rows, against 2.5 D^2/16... for a contraction), lowered by a rigorous margin for their fp32 rounding
    // (|error| <= 64 u sum |x_a mu_a| <= 4e-6 (|x|^2 + |muf|^2)); the triangle inequality of the mask loses
    // most of it at D = 64 (x - mu_own is nearly orthogonal to mu_j - mu_own).  A row survives when a lane of
    // the block may not skip it; results are unchanged.  The next batch's means are loaded while this one's
    // MFMAs run.
    // h16 (DT <= 64, items with |x|^2 <= kScreen16X2, np8_set_data): the dot products in fp16, v_mfma_f32_16x16x32_f16, S / 8
    // MFMAs per item tile and 16 rows instead of S.  Rigorous margin: rounding x and muf to fp16 (relative 2^-11,
    // absolute 2^-14 with subnormals flushed) and summing the exact products in fp32 errs by <= 2^-10 sum |x_a muf_a| +
    // 2^-14 (sum |x_a| + sum |muf_a|) + 2^-17 sq <= 9.8e-4 sq + 2.5e-4 (D <= 64, sq = |x|^2 + |muf|^2), so
    // d^2 >= sq - 2 x.muf - (2e-3 sq + 1e-3); a pair with sq > 1e8 (fp16 overflow possible) is not screened.
    if (prune) {
        const int n1 = rlist_n[0];
        const bool h16 = DT <= 64 && A.screen16;
        if (wave_live && n1 > 0) {
            using W2 = Wide<DT>;
            const double Tl = valid ? st.T : 1e300;
            // a pair (row j, item i) stays skippable when U = base_j - lam_j/2 d^2 - T_i <= -kSkip - 2 - 1e-9 (|base_j| +
            // |T_i| + lam_j/2 d^2), d^2 = max(sq - 2 x.muf - (mA sq + mB), 0), evaluated as
            // fma(lam_j/2 (1 - 1e-9), d^2, Tm_i) >= base_j + 1e-9 |base_j| with Tm_i = T_i - kSkip - 2 - 1e-9 |T_i| and
            // sq (1 - mA) - mB = x2m_i + m2m_j: the same inequality, its per-item and per-row terms formed once (the
            // rounding of the regrouping is far inside the 1e-9 slack); lanes past the end (T = 1e300) never keep a row
            const double mA = h16 ? 2e-3 : 1e-5, mB = h16 ? 1e-3 : 0.0;
            double Tm[4], x2m[4];
            int32_t zit[4];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const double Ti = __shfl(Tl, 16 * nt + col);
                Tm[nt] = Ti - kSkip - 2.0 - 1e-9 * fabs(Ti);
                x2m[nt] = __shfl(x2, 16 * nt + col) * (1.0 - mA);
                zit[nt] = __shfl(zi, 16 * nt + col);
            }
            // A operand: lane (g, col) holds muf[4 s + g] of row list[b0 + col] (the transposed mean of its row)
            auto load_means = [&](int b0, float (&am)[W2::S]) {
                if (b0 + col < n1) {
                    const float *mt = A.wfrag + (int64_t)rslot[rlist[0][b0 + col]] * W2::ROW + W2::NCH * 256 + g * W2::S;
#pragma unroll
                    for (int s4 = 0; s4 < W2::S / 4; ++s4) {
                        const float4 v = *reinterpret_cast<const float4 *>(mt + 4 * s4);
                        am[4 * s4] = v.x;
                        am[4 * s4 + 1] = v.y;
                        am[4 * s4 + 2] = v.z;
                        am[4 * s4 + 3] = v.w;
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < W2::S; ++s) am[s] = 0.0f;
                }
            };
            float am[W2::S];
            load_means(0, am);
            for (int b0 = 0; b0 < n1; b0 += 16) {  // block-uniform: 16 kept rows at a time
                float amn[W2::S];
                if (b0 + 16 < n1) load_means(b0 + 16, amn);
                double m2p = 0.0;
#pragma unroll
                for (int s = 0; s < W2::S; ++s) m2p = fma((double)am[s], (double)am[s], m2p);
                double m2 = m2p + __shfl_xor(m2p, 16);
                m2 += __shfl_xor(m2, 32);  // |muf|^2 of row list[b0 + col], on the four lanes of column col
                typedef float f32x4 __attribute__((ext_vector_type(4)));
                f32x4 acc[4];
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[nt] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
                if (h16) {  // fp16 operands, 32 dims per MFMA (the same dims of a lane in A and B: any k order will do)
                    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
                    constexpr int HC = (W2::S + 7) / 8;
#pragma unroll
                    for (int hc = 0; hc < HC; ++hc) {
                        h8 ah;
#pragma unroll
                        for (int e = 0; e < 8; ++e) ah[e] = (8 * hc + e < W2::S) ? (_Float16)am[(8 * hc + e) % W2::S] : (_Float16)0.0f;
#pragma unroll
                        for (int nt = 0; nt < 4; ++nt) {
                            h8 bh;
#pragma unroll
                            for (int e = 0; e < 8; ++e)
                                bh[e] = (8 * hc + e < W2::S) ? (_Float16)xb[nt][(8 * hc + e) % W2::S] : (_Float16)0.0f;
                            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[nt], 0, 0, 0);
                        }
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < W2::S; ++s)
#pragma unroll
                        for (int nt = 0; nt < 4; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(am[s], xb[nt][s], acc[nt], 0, 0, 0);
                }
                // output (nt, r) of lane (g, col): row list[b0 + 4 g + r], item 16 nt + col
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int li = b0 + 4 * g + r;
                    const int jr = (li < n1) ? (int)rlist[0][li] : K;
                    const double m2r = __shfl(m2, 4 * g + r);
                    bool nr = false;
                    if (jr < K) {
                        const int32_t sjr = rslot[jr];
                        const double base = rbase[jr];
                        const double Bp = base + 1e-9 * fabs(base), lamp = rlamh[jr] * (1.0 - 1e-9);
                        const double m2m = fma(m2r, 1.0 - mA, -mB);
                        // fp16: |x|^2 <= 4096, so sq > 1e8 (overflow possible) implies |muf|^2 > 5e7: not screened
                        const bool rowbig = h16 && !(m2r <= 5e7);
#pragma unroll
                        for (int nt = 0; nt < 4; ++nt) {
                            if (sjr != zit[nt]) {
                                const double d2 = fmax(fma(-2.0, (double)acc[nt][r], x2m[nt] + m2m), 0.0);
                                nr = nr || rowbig || !(fma(lamp, d2, Tm[nt]) >= Bp);
                            }
                        }
                    }
                    const uint64_t b = __ballot(nr);
                    // rows 4 g' + r: lanes 16 g' .. 16 g' + 15
#pragma unroll
                    for (int gg = 0; gg < 4; ++gg) {
                        const int row = __builtin_amdgcn_readlane(jr, 16 * gg);
                        if (lane == 0 && ((b >> (16 * gg)) & 0xFFFFull) != 0ull && row < K)
                            atomicOr(&rmask2[row >> 6], 1ull << (row & 63));
                    }
                }
                if (b0 + 16 < n1) {
#pragma unroll
                    for (int s = 0; s < W2::S; ++s) am[s] = amn[s];
                }
            }
        }
        __syncthreads();
        compact(rmask2, rlist[1], &rlist_n[1]);
        __syncthreads();
    }
    // the rows to evaluate (block-uniform): the screen's list, or every row
    const int nrows = prune ? rlist_n[1] : K;
    auto row_at = [&](int i) -> int { return prune ? (int)rlist[1][i] : i; };

    // the evaluated candidates in ascending order, block-uniform: the next one is copied into the other
    // stage while the MFMAs of this one run; one barrier per row
    int buf = 0, rows_done = 0;
    if (nrows > 0) row_glds<DT>(A.wfrag, (int)cand[(int64_t)row_at(0) * CS + F + kFieldSlot], stage);
    __syncthreads();
    for (int i = 0; i < nrows; ++i) {
        const int j = row_at(i);
        const double *e = cand + (int64_t)j * CS;  // block-uniform: scalar loads
        const int32_t sj = (int32_t)e[F + kFieldSlot];
        if (i + 1 < nrows)
            row_glds<DT>(A.wfrag, (int)cand[(int64_t)row_at(i + 1) * CS + F + kFieldSlot], stage + (buf ^ 1) * W::ROW);
        const float *row = stage + buf * W::ROW;
        if (wave_live) {
            const double q = wide_pass<DT>(row, xb, lane);
            if (sj != zi) {
                const double llj = fma(-0.5, q, e[F + kFieldC]);
                pick_step(st, llj + e[F + kFieldLogn], j);
                if (LL) llp = (st.pick == j) ? llj : llp;
            }
        }
        __syncthreads();  // the next row has landed (vmcnt(0)); this row's stage may be overwritten
        buf ^= 1;
        ++rows_done;
    }
    if (NP8_WLATE(count_eval) && wave_live) {  // item-row contractions this wave executed (own passes + evaluated rows)
        const unsigned long long items = (unsigned long long)__popcll(__ballot(valid));
        if (lane == 0) {
            unsigned long long *ec = NP8_WLATE(evalc) + 2 * ((blockIdx.x * 4 + (threadIdx.x >> 6)) % kEvalSlots);
            atomicAdd(ec, items * (unsigned long long)(rows_done + own_passes));
#ifdef NP8_EXP_WIDE_ROWS  // experiment: per wave, the rows the triangle mask kept and the rows the exact screen kept
            if (prune) {
                atomicAdd(ec + 6 * kEvalSlots, (unsigned long long)rlist_n[0]);
                atomicAdd(ec + 4 * kEvalSlots + 1, (unsigned long long)rlist_n[1]);
            }
#endif
        }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) pick_step(st, lwa[m], K + m);
    if constexpr (LL) {  // the wave's exact sum (every lane of a live wave takes part; lanes past the end add 0)
        Fx v = {0ull, 0};
        if (valid) v = fx_of(st.pick >= K ? ll_own : llp);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = fx_add(v, wfx_shfl_xor(v, o));
        if (wave_live && lane == 0) NP8_WLATE(llpart)[(pw - NP8_WLATE(p0)) >> 6] = v;
    }
    if (!valid) return;

    int32_t *delta = reinterpret_cast<int32_t *>(NP8_WLATE(rec) + kRecHeaderBytes);
    const int32_t snew = (st.pick < K) ? (int32_t)cand[(int64_t)st.pick * CS + F + kFieldSlot] : -1;
    const uint64_t mv = __ballot(snew != zi);
    if (mv && lane == (__ffsll((unsigned long long)__ballot(1)) - 1))
        atomicAdd(reinterpret_cast<unsigned long long *>(&NP8_WLATE(ctl)->moved), (unsigned long long)__popcll(mv));
    const bool mover = st.pick < K && snew != zi;
    wave_add_by_key(delta, zi, -1, mover);
    wave_add_by_key(delta, snew, 1, mover);
    const int qreq = wave_append(NP8_WLATE(nreq), st.pick >= K);  // (requests are accepted by scan position, not arrival)
    if (st.pick < K) {
        if (snew != zi) {
            NP8_WLATE(z)[il] = snew;
            if (sorted) zs[pc] = snew;
        }
    } else {
        const int q = qreq;
        if (q < NP8_WLATE(req_cap)) {  // always: the area holds every item of the step
            Request r;
            r.pos = sorted ? (int64_t)ig : NP8_WLATE(offset) + p;
            r.i = (int64_t)ig;
            r.m = st.pick - K;
            r.zold = zi;
            r.lpos = sorted ? (int32_t)pc : -1;
            r.pad = 0;
            r.dll.lo = 0ull;
            r.dll.hi = 0;
            NP8_WLATE(req)[q] = r;
            double *vmu = NP8_WLATE(vmu) + (int64_t)q * (D + 1);
            wide_frame_payload(hyp, D, X, n, xr, vmu);
            if (q < NP8_WLATE(ccap)) {  // compact exchange (np8_step_local_compact): the first ccap requests in the compact record
                NP8_WLATE(creq)[q] = r;
                for (int a = 0; a <= D; ++a) NP8_WLATE(cvmu)[(int64_t)q * (D + 1) + a] = vmu[a];
            }
        }
    }
}

// ---- max likelihood and parity ---------------------------------------------------------------------
// q of item x (fp32 values) against slot sj on the vector ALU: the same fmaf chains (zero terms of the
// triangular A skipped) and the same fp64 summation order as wide_pass.
template <int DT>
__device__ double wide_q_valu(const WideArgs &W, const float *__restrict__ X, int64_t n, int64_t xr, int sj) {
    const float *Aj = W.wA + (int64_t)sj * DT * DT;
    const float *mj = W.wmu + (int64_t)sj * DT;
    float xt[DT];
#pragma unroll
    for (int b = 0; b < DT; ++b) xt[b] = X[(int64_t)b * n + xr] - mj[b];
    float sg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int mt = 0; mt < DT / 16; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const int a = 16 * mt + 4 * gg + r;
                float v = 0.0f;
                for (int b = a; b < DT; ++b) v = fmaf(Aj[(int64_t)a * DT + b], xt[b], v);
                sg[gg] = fmaf(v, v, sg[gg]);
            }
    return (double)((sg[0] + sg[1]) + (sg[2] + sg[3]));
}

template <int DT>
__global__ __launch_bounds__(256) void np8_loglik_wide(LoglikArgs L, WideArgs W) {
    const int CS = cand_stride(W.D), F = W.D + W.D * (W.D + 1) / 2;
    __shared__ double red[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double ll = 0.0;
    if (i < L.n_loc) {
        const int32_t s = L.z[i];
        const double *e = L.cand + (int64_t)L.dense_of[s] * CS;
        ll = fma(-0.5, wide_q_valu<DT>(W, reinterpret_cast<const float *>(L.X), L.n_loc, i, s), e[F + kFieldC]);
    }
    red[threadIdx.x] = ll;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) L.partial[blockIdx.x] = red[0];
}

template <int DT, int M, int PRIOR>
__global__ __launch_bounds__(64) void np8_loglik_matrix_wide(AssignArgs A, WideArgs W, const int64_t *__restrict__ idx,
                                                             int64_t n, double *__restrict__ out) {
    const int D = W.D, CS = cand_stride(D), F = D + D * (D + 1) / 2;
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t il = idx[r];
    const float *X = reinterpret_cast<const float *>(A.X);
    const int K = A.ctl->K;
    for (int j = 0; j < K; ++j) {
        const double *e = A.cand + (int64_t)j * CS;
        out[r * (K + M) + j] = fma(-0.5, wide_q_valu<DT>(W, X, A.n_loc, il, (int)e[F + kFieldSlot]), e[F + kFieldC]);
    }
    float xf[DT];
#pragma unroll
    for (int a = 0; a < DT; ++a) xf[a] = X[(int64_t)a * A.n_loc + il];
    const double ny = wide_whiten_norm<DT>(A.uw, xf);
    const uint32_t t = A.ctl->t_base + A.t;
    for (int m = 0; m < M; ++m)
        out[r * (K + M) + K + m] = wide_aux_ll<PRIOR>(A.hyp, D, ny, A.seed, (uint64_t)(A.offset + il), t, m, M);
}

// ---- max likelihood on the matrix cores -------------------------------------------------------------
// sum_i ll(x_i | theta_{z_i}) (MCMC::considerMaxLikelihood, np_mcmc.cpp:187-203): the own-cluster passes
// of np8_assign_wide (one MFMA pass per distinct own slot of a wave; one on the label-sorted layout),
// a fixed-order block reduction into partial[block] (reduced by np8_loglik_reduce).
template <int DT>
// Three waves per SIMD (159 VGPRs, no spills; 180 and two waves without the attribute, four spill): C5 niw_conjugate
// 1 753-1 755 -> 1 759-1 765 sweeps/s, A/B on one box (profiles/r06/ab_llw3).
#ifndef NP8_LLW_WAVES
#define NP8_LLW_WAVES 3
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NP8_LLW_WAVES))) void np8_loglik_wide_mfma(
    AssignArgs A, double *__restrict__ partial) {
    using W = Wide<DT>;
    const int CS = cand_stride(A.dim), F = A.dim + A.dim * (A.dim + 1) / 2;
    __shared__ double red[256];
    const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
    const int64_t pw = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
    const int64_t p = pw + lane;
    const bool valid = p < A.n_loc;
    const bool sorted = A.sorted != 0;
    constexpr int cur = 0;  // the label-sorted layout is always buffer 0 (buffer 1: the re-sort's scratch)
    const int32_t *__restrict__ zs = cur ? A.zs[1] : A.zs[0];
    const float *__restrict__ X = reinterpret_cast<const float *>(sorted ? (cur ? A.Xs[1] : A.Xs[0]) : A.X);
    const int64_t n = A.n_loc;
    double ll = 0.0;
    if (pw < n) {  // wave-uniform
        const int64_t pc = valid ? p : pw;
        const int32_t zi = sorted ? zs[pc] : A.z[pc];
        float xb[4][W::S];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            int64_t pq = pw + nt * 16 + col;
            if (pq >= n) pq = pc;
#pragma unroll
            for (int st = 0; st < W::S; ++st) xb[nt][st] = X[(int64_t)(4 * st + g) * n + pq];
        }
        uint64_t pend = __ballot(valid);
        while (pend) {
            const int32_t sj = __shfl(zi, __ffsll((unsigned long long)pend) - 1);
            const double q = wide_pass<DT>(A.wfrag + (int64_t)sj * W::ROW, xb, lane);
            const bool mine = valid && zi == sj;
            if (mine) ll = fma(-0.5, q, A.cand[(int64_t)A.dense_of[sj] * CS + F + kFieldC]);
            pend &= ~__ballot(mine);
        }
    }
    red[threadIdx.x] = ll;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

hipError_t np8_launch_loglik_wide_mfma(const AssignArgs &A, int D, double *partial, hipStream_t s) {
    const int64_t nb = (A.n_loc + 255) / 256;
    if (nb <= 0) return hipSuccess;
    const int DT = wide_dt(D);
    if (DT == 32)
        hipLaunchKernelGGL((np8_loglik_wide_mfma<32>), dim3((unsigned)nb), dim3(256), 0, s, A, partial);
    else if (DT == 48)
        hipLaunchKernelGGL((np8_loglik_wide_mfma<48>), dim3((unsigned)nb), dim3(256), 0, s, A, partial);
    else if (DT == 64)
        hipLaunchKernelGGL((np8_loglik_wide_mfma<64>), dim3((unsigned)nb), dim3(256), 0, s, A, partial);
    else if (DT == 80)
        hipLaunchKernelGGL((np8_loglik_wide_mfma<80>), dim3((unsigned)nb), dim3(256), 0, s, A, partial);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// The folded check's last part on the wide path (np8_finalize with FinArgs::ll_defer left the assign's sum in
// ctl->L_fx): every accepted requester's ll moves from its old slot to its new one -- both the VALU form of the
// contraction (bit-identical to the MFMA passes), on its position of the label-sorted layout -- then L and the snapshot
// decision of np8_finalize's check.  One workgroup.
template <int DT>
__global__ __launch_bounds__(256) void np8_ll_fix_wide(WideArgs W, const float *__restrict__ Xs, int64_t n,
                                                       const double *__restrict__ slot_c, const int64_t *__restrict__ pend,
                                                       const int64_t *__restrict__ pend_ll, double *best, int32_t *have_best,
                                                       int par, Ctl *ctl) {
    __shared__ Fx part[256];
    const int np = ctl->n_pend;
    Fx v = {0ull, 0};
    for (int q = threadIdx.x; q < np; q += blockDim.x) {
        const int s_new = (int)pend[4 * (int64_t)q + 3], s_old = (int)pend_ll[2 * (int64_t)q];
        const int64_t lp = pend_ll[2 * (int64_t)q + 1];
        const double lo = fma(-0.5, wide_q_valu<DT>(W, Xs, n, lp, s_old), slot_c[s_old]);
        const double ln = fma(-0.5, wide_q_valu<DT>(W, Xs, n, lp, s_new), slot_c[s_new]);
        v = fx_add(v, fx_add(fx_of(ln), fx_neg(fx_of(lo))));
    }
    part[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        Fx S;
        S.lo = ctl->L_fx_lo;
        S.hi = ctl->L_fx_hi;
        for (int k = 0; k < (int)blockDim.x; ++k) S = fx_add(S, part[k]);  // (exact: any order)
        const double L = fx_to_double(S);
        ctl->L = L;
        ctl->L_local = L;
        const double b = best[par];
        const bool better = L > b;
        best[par ^ 1] = better ? L : b;
        if (better) *have_best = 1;
        ctl->snap_pend = better ? 1 : 0;
    }
}

hipError_t np8_launch_ll_fix_wide(const WideArgs &W, const float *Xs, int64_t n, const double *cand,
                                  const int32_t *dense_of, const double *slot_c, const int64_t *pend, const int64_t *pend_ll,
                                  double *best, int32_t *have_best, int par, Ctl *ctl, hipStream_t s) {
    (void)cand;
    (void)dense_of;
    const int DT = W.DT;
#define NP8_FIX(d)                                                                                                 \
    if (DT == d) {                                                                                                 \
        hipLaunchKernelGGL((np8_ll_fix_wide<d>), dim3(1), dim3(256), 0, s, W, Xs, n, slot_c, pend, pend_ll, best,  \
                           have_best, par, ctl);                                                                   \
        return hipGetLastError();                                                                                  \
    }
    NP8_FIX(32)
    NP8_FIX(48)
    NP8_FIX(64)
    NP8_FIX(80)
#undef NP8_FIX
    return hipErrorInvalidValue;
}

// ---- sufficient statistics on the fp64 matrix cores (niw_conjugate on the wide path) -------------------
// Per slot: s1 = sum d, S = sum d d^T (packed upper) with d = x - mu_slot in fp64 (the layout of
// np8_suffstats / np8o_suffstats).  One wave walks 64 kSuffChunks consecutive positions of the (label-sorted)
// layout in chunks of 32 items; each chunk is staged in LDS (coalesced row reads: one load instruction moves
// 128 B of dim a and 128 B of dim a + D/2), then for the slot run being accumulated S += D^T D on
// v_mfma_f64_16x16x4_f64 (items = the k dimension: 4 per MFMA, 8 steps per chunk, the 16x16 tiles ti <= tj of S),
// items of other slots masked to 0.  Sums stay in registers while the slot does not change and are committed
// as a run record (ParamArgs::part, reduced in record order by np8_niw_post) or with fp64 atomics.
// Registers: the next chunk's 32 floats per lane in flight while this one is contracted, the accumulators in
// AGPRs, one MFMA step's operands at a time -- two waves per SIMD (round 3: 472 registers, one wave).
#ifndef NP8_SUFF_CHUNKS
#define NP8_SUFF_CHUNKS 8
#endif
constexpr int kSuffChunks = NP8_SUFF_CHUNKS;  // (64-item units per wave)

// BUF: item rows through a buffer descriptor (32-bit offsets: D n 4 < 2^31 bytes), two VGPRs of addressing instead
// of one 64-bit address per row.
// DT: the items' rows (D rounded up to 16, rows >= D zero); statistics and run records in the DT layout, acc in the
// data's D layout (its packed upper triangle: entries with a row or column >= D are the zero rows, left out).
template <int DT, bool BUF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void np8_suffstats_wide(ParamArgs P) {
    constexpr int D = DT;  // (the tile structure; P.D is the data's)
    constexpr int T = D / 16, NT = T * (T + 1) / 2, H = D / 2;
    const int Dd = P.D, W = Dd + Dd * (Dd + 1) / 2;
    constexpr int CI = 32;           // items per chunk
    constexpr int PS = 2 * CI + 2;   // floats per dim pair (a, a + H): conflict-free column reads
    constexpr int NCH = 2 * kSuffChunks;
    typedef double f64x4 __attribute__((ext_vector_type(4)));
    __shared__ float tile[4][H * PS];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4, col = lane & 15;
    const bool sorted = P.sorted != 0;
    constexpr int cur = 0;  // the label-sorted layout is always buffer 0 (buffer 1: the re-sort's scratch)
    const float *__restrict__ X = reinterpret_cast<const float *>(sorted ? (cur ? P.Xs[1] : P.Xs[0]) : P.X);
    const int32_t *__restrict__ z = sorted ? (cur ? P.zs[1] : P.zs[0]) : P.z;
    const int64_t n = P.n_loc;
    const int64_t wid = (int64_t)blockIdx.x * 4 + wv;
    const int64_t base = wid * (int64_t)(CI * NCH);
    int nrun = 0;  // run records this wave wrote
    auto close_records = [&]() {  // the unused run records of this wave
        if (P.part && lane < kSuffRuns && lane >= nrun) P.part_slot[wid * kSuffRuns + lane] = -1;
    };
    if (base >= n) {  // wave-uniform; no block barrier below
        close_records();
        return;
    }
    float *tl = tile[wv];
    f64x4 acc[NT];
    double s1[T];
    int32_t cs = -1;        // slot being accumulated
    double anc[T];          // its mean, dims 16 t + col
    auto reset = [&]() {
#pragma unroll
        for (int q = 0; q < NT; ++q) acc[q] = (f64x4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int t = 0; t < T; ++t) s1[t] = 0.0;
    };
    auto commit = [&]() {
        // the lane's index made opaque here: its address arithmetic stays in this (rare) path instead of being
        // hoisted out of the chunk loop and held in registers across it
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int g = ln >> 4, col = ln & 15;
        if (P.part && nrun < kSuffRuns) {  // a run record: the raw accumulators, then s1 (dims 16 t + col)
            constexpr int RS = NT * 4 * 64 + T * 16;
            double *rec = P.part + (wid * kSuffRuns + nrun) * RS;
#pragma unroll
            for (int q = 0; q < NT; ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) rec[(q * 4 + r) * 64 + ln] = acc[q][r];
#pragma unroll
            for (int t = 0; t < T; ++t) {
                double v = s1[t];
                v += __shfl_xor(v, 16);
                v += __shfl_xor(v, 32);
                if (g == 0) rec[NT * 4 * 64 + t * 16 + col] = v;
            }
            if (ln == 0) P.part_slot[wid * kSuffRuns + nrun] = cs;
            ++nrun;
            return;
        }
        double *dst = P.acc + (int64_t)cs * W;
        int q = 0;
#pragma unroll
        for (int ti = 0; ti < T; ++ti)
#pragma unroll
            for (int tj = ti; tj < T; ++tj, ++q)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int a = 16 * ti + g + 4 * r, b = 16 * tj + col;  // f64 MFMA layout
                    if (a <= b && b < Dd) unsafeAtomicAdd(dst + Dd + a * Dd - (a * (a - 1)) / 2 + (b - a), acc[q][r]);
                }
#pragma unroll
        for (int t = 0; t < T; ++t) {
            double v = s1[t];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (g == 0 && 16 * t + col < Dd) unsafeAtomicAdd(dst + 16 * t + col, v);
        }
    };
    reset();
    // LDS word of (dim, item): pair a = dim mod H, half dim / H
    auto lds_at = [&](int dim, int it) { return (dim % H) * PS + (dim / H) * CI + it; };
    // software-pipelined: chunk c + 1's item rows (lane: item lane & 31 of dims a + H (lane >> 5)) and labels are
    // in flight while chunk c (LDS) is contracted
    float xn[H];
    int32_t zn;
    const uint64_t xa = reinterpret_cast<uint64_t>(X);
    const uint32_t xlo = __builtin_amdgcn_readfirstlane((uint32_t)xa), xhi = __builtin_amdgcn_readfirstlane((uint32_t)(xa >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>(((uint64_t)xhi << 32) | xlo), 0, __builtin_amdgcn_readfirstlane((int)(BUF ? n * D * 4 : 0)),
        0x00020000);
    auto fetch = [&](int c) {
        const int64_t p = base + CI * c + (lane & 31);
        const bool valid = p < n && lane < CI;
        zn = valid ? z[p] : -1;
        const int64_t pr = (p < n) ? p : 0;  // (rows past the end: any in-bounds word, masked by its label)
        if constexpr (BUF) {
            const int vo = (int)(((int64_t)(lane >> 5) * H * n + pr) * 4);
            const int n4 = (int)(n * 4);
#pragma unroll
            for (int a = 0; a < H; ++a) xn[a] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, a * n4, 0));
        } else {
            const float *src = X + (int64_t)(lane >> 5) * H * n + pr;
#pragma unroll
            for (int a = 0; a < H; ++a) xn[a] = src[(int64_t)a * n];
        }
    };
    fetch(0);
    for (int c = 0; c < NCH; ++c) {
        const int64_t p0 = base + CI * c;
        if (p0 >= n) break;
        const int32_t zl = zn;  // labels of the chunk's items (lanes 0..31; -1 past the end)
#pragma unroll
        for (int a = 0; a < H; ++a) tl[a * PS + lane] = xn[a];
        __builtin_amdgcn_wave_barrier();
        if (c + 1 < NCH) fetch(c + 1);
        uint64_t pend = __ballot(zl >= 0);
        while (pend) {
            const int32_t sl = __shfl(zl, __ffsll((unsigned long long)pend) - 1);
            if (sl != cs) {
                if (cs >= 0) commit();
                reset();
                cs = sl;
#pragma unroll
                for (int t = 0; t < T; ++t) anc[t] = (16 * t + col < Dd) ? P.slot_mu[(int64_t)cs * Dd + 16 * t + col] : 0.0;
            }
            pend &= ~__ballot(zl == sl);
#pragma unroll 2
            for (int st = 0; st < CI / 4; ++st) {
                const int it = 4 * st + g;  // item of this k-step held by the lane
                const bool in = __shfl(zl, it) == sl;
                double dv[T];
#pragma unroll
                for (int t = 0; t < T; ++t) dv[t] = in ? (double)tl[lds_at(16 * t + col, it)] - anc[t] : 0.0;
#pragma unroll
                for (int t = 0; t < T; ++t) s1[t] += dv[t];
                int q = 0;
#pragma unroll
                for (int ti = 0; ti < T; ++ti)
#pragma unroll
                    for (int tj = ti; tj < T; ++tj, ++q)
                        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(dv[ti], dv[tj], acc[q], 0, 0, 0);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (cs >= 0) commit();
    close_records();
}

// Waves of an np8_suffstats_wide launch over n items, and the doubles of one run record at D (ParamArgs::part).
int64_t np8_suffstats_wide_waves(int64_t n) { return 4 * ((n + 4 * 64 * kSuffChunks - 1) / (4 * 64 * kSuffChunks)); }  // (64 kSuffChunks items per wave)
int64_t np8_suffstats_wide_record(int D) {
    const int T = wide_dt(D) / 16;
    return (int64_t)(T * (T + 1) / 2) * 4 * 64 + T * 16;
}

hipError_t np8_launch_suffstats_wide(const ParamArgs &P, hipStream_t s) {
    const int64_t per_block = 4 * 64 * kSuffChunks;
    const int64_t nb = (P.n_loc + per_block - 1) / per_block;
    if (nb <= 0) return hipSuccess;
    const bool buf = P.n_loc * P.DT * 4 < ((int64_t)1 << 31);
#define NP8_SUFF_LAUNCH(DD)                                                                                   \
    if (P.DT == DD) {                                                                                         \
        if (buf)                                                                                              \
            hipLaunchKernelGGL((np8_suffstats_wide<DD, true>), dim3((unsigned)nb), dim3(256), 0, s, P);       \
        else                                                                                                  \
            hipLaunchKernelGGL((np8_suffstats_wide<DD, false>), dim3((unsigned)nb), dim3(256), 0, s, P);      \
        return hipGetLastError();                                                                             \
    }
    NP8_SUFF_LAUNCH(32)
    NP8_SUFF_LAUNCH(48)
    NP8_SUFF_LAUNCH(64)
    NP8_SUFF_LAUNCH(80)
#undef NP8_SUFF_LAUNCH
    return hipErrorInvalidValue;
}

// ---- dispatch ----------------------------------------------------------------------------------------
// tile dimensions DT (D rounded up to 16) the kernels are instantiated for, with M
#define NP8_WIDE_FOR_EACH(X) X(32, 3) X(48, 3) X(64, 3) X(80, 3)

bool np8_wide_supported(int D, int M) {
    if (D <= 16) return false;  // (the fp64 path)
    const int DT = wide_dt(D);
#define X(d, m) \
    if (DT == d && M == m) return true;
    NP8_WIDE_FOR_EACH(X)
#undef X
    return false;
}

hipError_t np8_launch_assign_wide(const AssignArgs &A, int D, int M, int prior, hipStream_t s) {
    const int64_t n = A.p1 - A.p0;
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    const int DT = wide_dt(D);
    const bool exact = D == DT;  // (D a multiple of 16: the instances with a constant D)
#define AW(d, m, prior_, ll_, ex_) hipLaunchKernelGGL((np8_assign_wide<d, m, prior_, ll_, ex_>), grid, block, lds, s, A)
#define AWP(d, m, prior_)                                                                                    \
    {                                                                                                        \
        if (A.ll_on)                                                                                         \
            { if (exact) AW(d, m, prior_, true, true); else AW(d, m, prior_, true, false); }                 \
        else                                                                                                 \
            { if (exact) AW(d, m, prior_, false, true); else AW(d, m, prior_, false, false); }               \
    }
#define X(d, m)                                                                                              \
    if (DT == d && M == m) {                                                                                 \
        const size_t lds = 2 * sizeof(float) * Wide<d>::ROW;                                                 \
        if (prior == kPriorNiw) AWP(d, m, kPriorNiw) else AWP(d, m, kPriorReference)                         \
        return hipGetLastError();                                                                            \
    }
    NP8_WIDE_FOR_EACH(X)
#undef X
#undef AWP
#undef AW
    return hipErrorInvalidValue;
}

// The per-item frame of the wide assign (kFrameRows): |U^T (x - mu0)| (wide_whiten_norm, the fully unrolled triangular
// product) and |x|^2, one thread per item, once per data set, into the four 32-bit rows after the item's DT rows.
template <int DT>
__global__ __launch_bounds__(256) void np8_wide_frame(float *__restrict__ X, int64_t n, const double *__restrict__ uw) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float xf[DT];
#pragma unroll
    for (int a = 0; a < DT; ++a) xf[a] = X[(int64_t)a * n + i];  // (rows >= D: zeros)
    const double ny = wide_whiten_norm<DT>(uw, xf);
    double x2 = 0.0;
#pragma unroll
    for (int a = 0; a < DT; ++a) x2 = fma((double)xf[a], (double)xf[a], x2);  // (rows >= D: + 0)
    uint32_t *fr = reinterpret_cast<uint32_t *>(X) + (int64_t)DT * n + i;
    fr[0] = (uint32_t)__double2loint(ny);
    fr[n] = (uint32_t)__double2hiint(ny);
    fr[2 * n] = (uint32_t)__double2loint(x2);
    fr[3 * n] = (uint32_t)__double2hiint(x2);
}

hipError_t np8_launch_wide_frame(float *X, int64_t n, const double *uw, int DT, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
#define X(d, m)                                                                                     \
    if (DT == d) {                                                                                  \
        hipLaunchKernelGGL((np8_wide_frame<d>), grid, block, 0, s, X, n, uw);                       \
        return hipGetLastError();                                                                   \
    }
    NP8_WIDE_FOR_EACH(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_loglik_matrix_wide(const AssignArgs &A, const WideArgs &W, int D, int M, int prior,
                                         const int64_t *idx, int64_t n, double *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 63) / 64)), block(64);
    const int DT = wide_dt(D);
#define X(d, m)                                                                                                    \
    if (DT == d && M == m) {                                                                                       \
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
    const int DT = wide_dt(D);
    if (DT == 32)
        hipLaunchKernelGGL((np8_loglik_wide<32>), dim3((unsigned)nb), dim3(256), 0, s, L, W);
    else if (DT == 48)
        hipLaunchKernelGGL((np8_loglik_wide<48>), dim3((unsigned)nb), dim3(256), 0, s, L, W);
    else if (DT == 64)
        hipLaunchKernelGGL((np8_loglik_wide<64>), dim3((unsigned)nb), dim3(256), 0, s, L, W);
    else if (DT == 80)
        hipLaunchKernelGGL((np8_loglik_wide<80>), dim3((unsigned)nb), dim3(256), 0, s, L, W);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t np8_launch_wide_dist(const WideArgs &W, hipStream_t s) {
    hipLaunchKernelGGL(np8_wide_dist, dim3((unsigned)W.kcap), dim3(256), 0, s, W);
    return hipGetLastError();
}

hipError_t np8_launch_wide_refresh(const WideArgs &W, hipStream_t s) {
    // the factor's matrix and the tests': 133 KB at D = 64, 156 KB at D = 80 (two tests)
    const size_t lds = (1 + wide_rows_tests(W.D)) * sizeof(double) * W.D * (W.D + 1);
    static bool allowed = false;  // (set before the first launch, which is not inside a graph capture)
    if (!allowed) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&np8_wide_rows),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)(3 * sizeof(double) * 80 * 81));
        if (e != hipSuccess) return e;
        allowed = true;
    }
    hipLaunchKernelGGL(np8_wide_rows, dim3((unsigned)std::min(W.kcap, kWideRowsBlocks)), dim3(256), lds, s, W);
    return hipGetLastError();
}
