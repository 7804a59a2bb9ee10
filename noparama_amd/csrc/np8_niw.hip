// np8_niw.hip -- gfx950 kernels of the NIW prior (DESIGN.md "Priors").
//
//   np8_niw_post        one workgroup per live slot: the slot's (mu, Sigma) drawn from its exact
//                       Normal-Inverse-Wishart posterior given the sufficient statistics np8_suffstats
//                       summed (param_update = NIW_CONJUGATE; the update the reference stubs with
//                       assert(false), include/statistics/normalinvwishart.h:66-75).  With no items it
//                       is a draw from G0 itself (np8_init_random under the NIW prior,
//                       np_init_clusters.cpp:24-40).
//   np8_niw_aux_slots   one workgroup per accepted new-cluster request: the full (mu, Sigma) of the
//                       picked auxiliary, whose likelihood np8_assign evaluated in the item's frame
//                       (membertrix::addCluster with the auxiliary's theta, np_neal_algorithm8.cpp:140-153).
//
// Both are O(D^3) dense linear algebra on LDS-resident D x D matrices (D <= 64: at most four 32 KB
// matrices).  Every output element is one sequential loop in the order oracle/np8_oracle.c
// (niw_draw_impl, niw_aux_slot) writes it; threads own output elements, so results are bit-identical
// to the oracle.  Sequential recurrences (triangular solves) run one thread per right-hand side.
#include "np8_kernels.h"

#include <hip/hip_runtime.h>

using namespace np8;

namespace {

constexpr int kNiwThreads = 256;
// np8_niw_post's workgroup: its MFMA tiles, trailing updates and record sums spread over blockDim.x / 64 waves, the
// serial panels stay on waves 0-2.  512 (two waves per SIMD, 251 VGPRs): C5 niw_conjugate 1 706 -> 1 745 sweeps/s
// against 256, A/B on one box (profiles/r06/ab_niw512); 1 024 would leave 128 registers per lane.
#ifndef NP8_NIW_POST_THREADS
#define NP8_NIW_POST_THREADS 512
#endif
constexpr int kNiwPostThreads = NP8_NIW_POST_THREADS;

#ifdef NP8_EXP_NIW_TIMING  // experiment: phase cycle counts of np8_niw_post, block 0, printed
#define NIW_T(k) \
    if (threadIdx.x == 0) tph[k] = (long long)__builtin_amdgcn_s_memtime();
#define NIW_SYNC() __syncthreads();
#else
#define NIW_T(k)
#define NIW_SYNC()
#endif

__device__ __forceinline__ int pix(int D, int a, int b) { return a * D - (a * (a - 1)) / 2 + (b - a); }

// (a, b), a > b, of the e-th strictly-lower element in row-major order (e = a(a-1)/2 + b).
__device__ __forceinline__ void lower_index(int e, int &a, int &b) {
    int r = (int)((1.0 + sqrt(1.0 + 8.0 * (double)e)) * 0.5);
    while (r * (r - 1) / 2 > e) --r;
    while ((r + 1) * r / 2 <= e) ++r;
    a = r;
    b = e - r * (r - 1) / 2;
}

__device__ __forceinline__ void zero_block(double *p, int n) {
    for (int k = threadIdx.x; k < n; k += blockDim.x) p[k] = 0.0;
}

// P' = packed sym(F F^T), off-diagonals doubled, into the slot table and its candidate row.  Returns
// the candidate table's isotropy value: P'_00 when P' is a multiple of I, else 0 (block-uniform).
__device__ double write_pprime(int D, int LD, const double *F, double *slotP, double *candP) {
    bool iso = true;
    double p00 = 0.0;  // the same chain as element (0, 0) below
    #pragma unroll 8
    for (int k = 0; k < D; ++k) p00 = fma(F[k], F[k], p00);
    for (int e = threadIdx.x; e < D * D; e += blockDim.x) {
        const int a = e / D, b = e - a * D;
        if (b < a) continue;
        double s = 0.0;
        #pragma unroll 8
        for (int k = 0; k < D; ++k) s = fma(F[a * LD + k], F[b * LD + k], s);
        const double v = (a == b) ? s : 2.0 * s;
        slotP[pix(D, a, b)] = v;
        if (candP) candP[pix(D, a, b)] = v;
        iso = iso && ((a == b) ? v == p00 : v == 0.0);
    }
    return __syncthreads_and(iso ? 1 : 0) ? p00 : 0.0;
}

// Sigma = T^T T, B T = Rhs (B lower triangular).  T by right-looking forward substitution: row k is final
// once divided by B_kk, then it updates every later row -- element (a, j) receives fma(-B_ak, T_kj, .) for
// k = 0, ..., a - 1 in order from Rhs_aj, as the oracle's loop does.  Sigma in 2 x 2 blocks per thread (half
// the LDS reads), each element one k-ordered chain.
__device__ void write_sigma(int D, int LD, const double *B, const double *Rhs, bool rhs_transposed, double *T, double *Sigma) {
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 x 16 threads (no index division)
    for (int a = ty; a < D; a += 16)
        for (int j = tx; j < D; j += 16) T[a * LD + j] = rhs_transposed ? Rhs[j * LD + a] : Rhs[a * LD + j];
    __syncthreads();
    for (int k = 0; k < D; ++k) {
        const double bkk = B[k * LD + k];
        for (int j = threadIdx.x; j < D; j += blockDim.x) T[k * LD + j] = T[k * LD + j] / bkk;
        __syncthreads();
        for (int a = k + 1 + ty; a < D; a += 16)
            for (int j = tx; j < D; j += 16) T[a * LD + j] = fma(-B[a * LD + k], T[k * LD + j], T[a * LD + j]);
        __syncthreads();
    }
    const int H = (D + 1) / 2;  // 2 x 2 blocks (D even on every instantiated path; odd D: edge guarded)
    for (int e = threadIdx.x; e < 16 * H; e += blockDim.x) {  // b-block e & 15 (+16 ...), a-block e >> 4
      for (int bb = e & 15; bb < H; bb += 16) {
        const int a = 2 * (e >> 4), b = 2 * bb;
        const bool a1 = a + 1 < D, b1 = b + 1 < D;
        double s00 = 0.0, s01 = 0.0, s10 = 0.0, s11 = 0.0;
        #pragma unroll 4
        for (int k = 0; k < D; ++k) {
            const double ta0 = T[k * LD + a], ta1 = a1 ? T[k * LD + a + 1] : 0.0;
            const double tb0 = T[k * LD + b], tb1 = b1 ? T[k * LD + b + 1] : 0.0;
            s00 = fma(ta0, tb0, s00);
            s01 = fma(ta0, tb1, s01);
            s10 = fma(ta1, tb0, s10);
            s11 = fma(ta1, tb1, s11);
        }
        Sigma[a * D + b] = s00;
        if (b1) Sigma[a * D + b + 1] = s01;
        if (a1) Sigma[(a + 1) * D + b] = s10;
        if (a1 && b1) Sigma[(a + 1) * D + b + 1] = s11;
      }
    }
}

// Sigma = T^T T in 2 x 2 blocks per thread (half the LDS reads), each element one k-ordered chain (write_sigma's
// second half, for a T already formed).
// T lower triangular: the terms k < max(a, b) are products with a zero (fma(0, t, +0) = +0 keeps the chain's bits)
// and are skipped.  Sl (or null): Sigma also into LDS (leading dimension LD).
__device__ __forceinline__ void sigma_from_t(int D, int LD, const double *T, double *Sigma, double *Sl = nullptr) {
    const int H = (D + 1) / 2;
    for (int e = threadIdx.x; e < 16 * H; e += blockDim.x) {
      for (int bb = e & 15; bb < H; bb += 16) {
        const int a = 2 * (e >> 4), b = 2 * bb;
        const bool a1 = a + 1 < D, b1 = b + 1 < D;
        double s00 = 0.0, s01 = 0.0, s10 = 0.0, s11 = 0.0;
        #pragma unroll 4
        for (int k = (a > b ? a : b); k < D; ++k) {
            const double ta0 = T[k * LD + a], ta1 = a1 ? T[k * LD + a + 1] : 0.0;
            const double tb0 = T[k * LD + b], tb1 = b1 ? T[k * LD + b + 1] : 0.0;
            s00 = fma(ta0, tb0, s00);
            s01 = fma(ta0, tb1, s01);
            s10 = fma(ta1, tb0, s10);
            s11 = fma(ta1, tb1, s11);
        }
        Sigma[a * D + b] = s00;
        if (b1) Sigma[a * D + b + 1] = s01;
        if (a1) Sigma[(a + 1) * D + b] = s10;
        if (a1 && b1) Sigma[(a + 1) * D + b + 1] = s11;
        if (Sl) {
            Sl[a * LD + b] = s00;
            if (b1) Sl[a * LD + b + 1] = s01;
            if (a1) Sl[(a + 1) * LD + b] = s10;
            if (a1 && b1) Sl[(a + 1) * LD + b + 1] = s11;
        }
      }
    }
}

// Y = X X (X symmetric, D a multiple of 4) in 4 x 4 register blocks per thread.  Y is symmetric too (bit for bit:
// element (j, i) is element (i, j)'s chain with the factors of each fma swapped), so only the blocks bi <= bj are
// computed and each is stored twice.
__device__ __forceinline__ void sym_square(int D, int LD, const double *X, double *Y) {
    const int nb = D / 4;
    for (int e = threadIdx.x; e < nb * (nb + 1) / 2; e += blockDim.x) {
        int bi = 0, rem = e;  // (bi, bj), bi <= bj: row-major over the upper block triangle
        while (rem >= nb - bi) {
            rem -= nb - bi;
            ++bi;
        }
        const int bj = bi + rem;
        double acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
#pragma unroll 4
        for (int k = 0; k < D; ++k) {
            double a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a[i] = X[(4 * bi + i) * LD + k];  // (row 4 bi + i = column, X symmetric)
                b[i] = X[k * LD + 4 * bj + i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], b[j], acc[i][j]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                Y[(4 * bi + i) * LD + 4 * bj + j] = acc[i][j];
                Y[(4 * bj + j) * LD + 4 * bi + i] = acc[i][j];
            }
    }
}

// Largest |row sum| of X (four threads per row, then the rows' sums in one wave; rs: D doubles of scratch).
// Block-uniform result (a bound's norm: no bit-exact order needed).
__device__ __forceinline__ double max_abs_row_sum(int D, int LD, const double *X, double *rs) {
    for (int t = threadIdx.x; t < 4 * D; t += blockDim.x) {
        const int a = t >> 2, part = t & 3;
        double v = 0.0;
        for (int b = part; b < D; b += 4) v += fabs(X[a * LD + b]);
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        if (part == 0) rs[a] = v;
    }
    __syncthreads();
    __shared__ double m_s;
    if (threadIdx.x < 64) {
        double m = 0.0;
        for (int a = threadIdx.x; a < D; a += 64) m = fmax(m, rs[a]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
        if (threadIdx.x == 0) m_s = m;
    }
    __syncthreads();
    return m_s;
}

// P' = packed sym(R^T R) for R upper (element (a, b), a <= b: sum_{k <= a} R_ka R_kb, k ascending from 0), off-diagonals
// doubled, into the slot table and its candidate row; returns the candidate table's isotropy value (write_pprime).
__device__ __forceinline__ double write_pprime_r(int D, int LD, const double *R, double *slotP, double *candP) {
    bool iso = true;
    const double p00 = fma(R[0], R[0], 0.0);  // element (0, 0)
    for (int e = threadIdx.x; e < D * D; e += blockDim.x) {
        const int a = e / D, b = e - a * D;
        if (b < a) continue;
        double s = 0.0;
        #pragma unroll 8
        for (int k = 0; k <= a; ++k) s = fma(R[k * LD + a], R[k * LD + b], s);
        const double v = (a == b) ? s : 2.0 * s;
        slotP[pix(D, a, b)] = v;
        if (candP) candP[pix(D, a, b)] = v;
        iso = iso && ((a == b) ? v == p00 : v == 0.0);
    }
    return __syncthreads_and(iso ? 1 : 0) ? p00 : 0.0;
}

constexpr int kPanelN = 16;

// ---- dense products on the fp64 matrix cores (round 5) ---------------------------------------------------------
// v_mfma_f64_16x16x4_f64 is a k-ordered fma chain (tools/mfma_f64_exact.hip measures it on the device): each output
// element receives fma(a_k, b_k, .) for k = k0, k0 + 1, ... in order, one rounding per product -- the chains the VALU
// loops above run.  Terms outside an element's own k range have a zero factor (the triangular operands), and
// fma(0, t, +0) = +0 / fma(x, 0, v) = v leave the chain's bits alone, so a whole 16 x 16 tile takes one k range.
typedef double f64x4 __attribute__((ext_vector_type(4)));

// One 16 x 16 tile (one wave): acc(i, j) = acc0(i, j) + sum_k a_at(i, k) b_at(k, j) over k = k0 .. k1 - 1 (k1 - k0 a
// multiple of 4; accessors return 0 outside the matrices); element r of lane l is (row (l >> 4) + 4 r, column l & 15).
// (chunked below: one LDS round trip per 16 k instead of one per k-step)
// M[o] when ok, else 0 -- the load made at offset 0 instead, so that it is unconditional (a guarded LDS load became a
// branch around every operand of the tiles)
__device__ __forceinline__ double lds_or0(const double *M, int o, bool ok) {
    const double v = M[ok ? o : 0];
    return ok ? v : 0.0;
}
// EX: D a multiple of 16, every index the tiles form is inside the matrix -- a plain load, nothing to mask (the select
// after a masked load pins its wait next to it)
template <bool EX>
__device__ __forceinline__ double lds_at(const double *M, int o, bool ok) {
    if constexpr (EX) {
        (void)ok;
        return M[o];
    } else {
        return lds_or0(M, o, ok);
    }
}
// NC chunks of 16 k with every operand read before the first MFMA (one LDS wait per tile)
template <int NC, class FA, class FB>
__device__ __forceinline__ f64x4 mfma_run(f64x4 acc, FA a_at, FB b_at, int k0) {
    const int lane = threadIdx.x & 63, il = lane & 15, kl = lane >> 4;
    double a[4 * NC], b[4 * NC];
#pragma unroll
    for (int q = 0; q < 4 * NC; ++q) {
        a[q] = a_at(il, k0 + 4 * q + kl);
        b[q] = b_at(k0 + 4 * q + kl, il);
    }
#pragma unroll
    for (int q = 0; q < 4 * NC; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[q], acc, 0, 0, 0);
    return acc;
}

template <class FA, class FB>
__device__ __forceinline__ f64x4 mfma_tile_acc(f64x4 acc, FA a_at, FB b_at, int k0, int k1) {
    switch ((k1 - k0 + 15) >> 4) {  // (wave-uniform) up to D = 80: the whole range's operands first
        case 1: return mfma_run<1>(acc, a_at, b_at, k0);
        case 2: return mfma_run<2>(acc, a_at, b_at, k0);
        case 3: return mfma_run<3>(acc, a_at, b_at, k0);
        case 4: return mfma_run<4>(acc, a_at, b_at, k0);
        case 5: return mfma_run<5>(acc, a_at, b_at, k0);
        default: break;
    }
    // chunks of 16 k (4 steps): the next chunk's operands are read while this chunk's MFMAs run (one wait per chunk,
    // not per step: per-step waits made a 64 x 64 product ~15k cycles, the loads-first form ~6k).  A chunk that runs
    // past k1 takes terms the accessors return as exact zeros (triangular operands, or masked past D), which leave the
    // chain's bits alone.
    const int lane = threadIdx.x & 63, il = lane & 15, kl = lane >> 4;
    const int nch = (k1 - k0 + 15) >> 4;  // (wave-uniform)
    double a[4], b[4];
    if (nch > 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a[q] = a_at(il, k0 + 4 * q + kl);
            b[q] = b_at(k0 + 4 * q + kl, il);
        }
    }
    for (int c = 0; c < nch; ++c) {
        double an[4], bn[4];
        if (c + 1 < nch) {
            const int kb = k0 + 16 * (c + 1);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                an[q] = a_at(il, kb + 4 * q + kl);
                bn[q] = b_at(kb + 4 * q + kl, il);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[q], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a[q] = an[q];
            b[q] = bn[q];
        }
    }
    return acc;
}
template <class FA, class FB>
__device__ __forceinline__ f64x4 mfma_tile(FA a_at, FB b_at, int k0, int k1) {
    return mfma_tile_acc((f64x4){0.0, 0.0, 0.0, 0.0}, a_at, b_at, k0, k1);
}

// Sigma = T^T T (T lower): tiles ti <= tj, element (a, b) = sum over k from 16 tj (below max(a, b) a factor is zero) of
// T_ka T_kb, mirrored -- sigma_from_t's chains (its element (b, a) is the same chain with each fma's factors swapped).
template <bool EX>
__device__ __forceinline__ void sigma_from_t_mfma(int D, int LD, const double *T, double *Sigma, double *Sl) {
    const int nt = (D + 15) / 16, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = __builtin_amdgcn_readfirstlane(blockDim.x >> 6), lane = threadIdx.x & 63;
    const int k1 = (D + 3) & ~3;
    for (int tt = wv; tt < nt * (nt + 1) / 2; tt += nw) {
        int ti = 0, rem = tt;
        while (rem >= nt - ti) {
            rem -= nt - ti;
            ++ti;
        }
        const int tj = ti + rem;
        const f64x4 acc = mfma_tile([&](int i, int k) { return lds_at<EX>(T, k * LD + 16 * ti + i, k < D && 16 * ti + i < D); },
                                    [&](int k, int j) { return lds_at<EX>(T, k * LD + 16 * tj + j, k < D && 16 * tj + j < D); },
                                    16 * tj, k1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int a = 16 * ti + (lane >> 4) + 4 * r, b = 16 * tj + (lane & 15);
            if (a < D && b < D) {
                Sigma[a * D + b] = acc[r];
                Sigma[b * D + a] = acc[r];
                if (Sl) {
                    Sl[a * LD + b] = acc[r];
                    Sl[b * LD + a] = acc[r];
                }
            }
        }
    }
}

// R = B^T U^{-1} (upper): R_ab = sum_{k = a..b} B_ka M[D-1-k][D-1-b] (M = Lr^{-1} lower, B lower), 0 below the diagonal.
template <bool EX>
__device__ __forceinline__ void r_from_b_mfma(int D, int LD, const double *B, const double *M, double *R) {
    const int nt = (D + 15) / 16, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = __builtin_amdgcn_readfirstlane(blockDim.x >> 6), lane = threadIdx.x & 63;
    for (int e = threadIdx.x; e < D * D; e += blockDim.x) {  // the lower triangle (tiles below the diagonal included)
        const int a = e / D, b = e - a * D;
        if (b < a) R[a * LD + b] = 0.0;
    }
    for (int tt = wv; tt < nt * (nt + 1) / 2; tt += nw) {
        int ti = 0, rem = tt;
        while (rem >= nt - ti) {
            rem -= nt - ti;
            ++ti;
        }
        const int tj = ti + rem;
        const int k1 = min((D + 3) & ~3, 16 * tj + 16);
        const f64x4 acc = mfma_tile(
            [&](int i, int k) { return lds_at<EX>(B, k * LD + 16 * ti + i, k < D && 16 * ti + i < D); },
            [&](int k, int j) { return lds_at<EX>(M, (D - 1 - k) * LD + (D - 1 - (16 * tj + j)), k < D && 16 * tj + j < D); },
            16 * ti, k1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int a = 16 * ti + (lane >> 4) + 4 * r, b = 16 * tj + (lane & 15);
            if (a < D && b < D && b >= a) R[a * LD + b] = acc[r];
        }
    }
}

// P' = packed sym(R^T R) (R upper): element (a, b), a <= b, = sum_{k = 0..a} R_ka R_kb, off-diagonals doubled, into the
// slot table and its candidate row; returns the isotropy value (write_pprime_r's).
template <bool EX>
__device__ __forceinline__ double write_pprime_r_mfma(int D, int LD, const double *R, double *slotP, double *candP) {
    const int nt = (D + 15) / 16, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = __builtin_amdgcn_readfirstlane(blockDim.x >> 6), lane = threadIdx.x & 63;
    const double p00 = fma(R[0], R[0], 0.0);
    bool iso = true;
    for (int tt = wv; tt < nt * (nt + 1) / 2; tt += nw) {
        int ti = 0, rem = tt;
        while (rem >= nt - ti) {
            rem -= nt - ti;
            ++ti;
        }
        const int tj = ti + rem;
        const int k1 = min((D + 3) & ~3, 16 * ti + 16);
        const f64x4 acc = mfma_tile([&](int i, int k) { return lds_at<EX>(R, k * LD + 16 * ti + i, k < D && 16 * ti + i < D); },
                                    [&](int k, int j) { return lds_at<EX>(R, k * LD + 16 * tj + j, k < D && 16 * tj + j < D); },
                                    0, k1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int a = 16 * ti + (lane >> 4) + 4 * r, b = 16 * tj + (lane & 15);
            if (a < D && b < D && b >= a) {
                const double v = (a == b) ? acc[r] : 2.0 * acc[r];
                slotP[pix(D, a, b)] = v;
                if (candP) candP[pix(D, a, b)] = v;
                iso = iso && ((a == b) ? v == p00 : v == 0.0);
            }
        }
    }
    return __syncthreads_and(iso ? 1 : 0) ? p00 : 0.0;
}

// Y = X X (X symmetric) for the eigenvalue bound (a bound, not a bit-exact quantity).  Y is symmetric: the tiles
// ti <= tj are computed (nt (nt + 1) / 2 of nt^2) and each is stored twice; the k-steps past D are never loaded.  The f64
// matrix core is the bound here (~64 cycles per 16x16x4 step on gfx950, the fp64 VALU rate), so fewer tiles is the lever.
template <bool EX>
__device__ __forceinline__ void sym_square_mfma(int D, int LD, const double *X, double *Y) {
    const int nt = (D + 15) / 16, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nw = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
    for (int tt = wv; tt < nt * (nt + 1) / 2; tt += nw) {
        int ti = 0, rem = tt;  // (ti, tj), ti <= tj, row-major over the upper tile triangle
        while (rem >= nt - ti) {
            rem -= nt - ti;
            ++ti;
        }
        const int tj = ti + rem;
        // A(i, k) = X[16 ti + i][k] read as X[k][16 ti + i] (X symmetric): consecutive lanes, consecutive words -- the
        // row-wise read put four lanes on each bank pair
        const f64x4 c = mfma_tile([&](int i, int k) { return lds_at<EX>(X, k * LD + 16 * ti + i, k < D && 16 * ti + i < D); },
                                  [&](int k, int j) { return lds_at<EX>(X, k * LD + 16 * tj + j, k < D && 16 * tj + j < D); },
                                  0, D);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int a = 16 * ti + (lane >> 4) + 4 * r, b = 16 * tj + (lane & 15);
            if (a < D && b < D) {
                Y[a * LD + b] = c[r];
                Y[b * LD + a] = c[r];
            }
        }
    }
}

// Squarings of Sigma / ||Sigma|| behind the wide path's eigenvalue bound (np8_niw_post): lambda_max <= g ||.^(2^k)||^(2^-k).
// A/B at C5 niw_conjugate, one box: k = 2: 1 157 sweeps/s, 3: 1 283, 4: 1 338 (each squaring ~10 us of np8_niw_post, a
// tighter bound fewer screen batches in np8_assign_wide).  Round 5 (a squaring ~5 us on the matrix cores): k = 4: 1 496,
// 5: 1 525, 6: 1 512.
#ifndef NP8_BOUND_SQUARINGS
#define NP8_BOUND_SQUARINGS 5
#endif
constexpr int kBoundSquarings = NP8_BOUND_SQUARINGS;

// Panel of 16 columns c0 .. c0 + 15 of the lower Cholesky factor of the symmetric matrix in L's lower triangle, on
// one wave (lane = row r, its 16 panel entries in registers): per column j the pivot, the scaled column, and the
// updates of the panel's later columns -- element (r, c) receives fma(-L_rj, L_cj, .) for j ascending, then the
// division by its pivot.  *skip != 0 if a pivot is not positive.
// Lane l's double (l wave-uniform) as two v_readlane: a scalar operand for the whole wave, no LDS round trip (the
// ds_bpermute of __shfl, waited on one by one, made each column of the panel ~1 500 cycles).
__device__ __forceinline__ double lane_d(double v, int l) {
    const int64_t b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFFll), l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}

// Column J of the panel and then the later ones, by template recursion: the indices into w[] are constants (a `#pragma
// unroll` the compiler declined left w[j] runtime-indexed -- v_cndmask selection trees, ~700 cycles per column)
template <int J>
__device__ __forceinline__ void panel_cols(double (&w)[kPanelN], int lane, int c0, int D, int &sk) {
    if constexpr (J < kPanelN) {
        const int jj = c0 + J;
        if (jj < D) {  // (wave-uniform: a last panel narrower than 16 when D is not a multiple of 16)
            const double v = lane_d(w[J], jj);  // the pivot L[jj][jj]
            const bool ok = v > 0.0;
            if (!ok) sk = 1;
            const double dj = ok ? sqrt(v) : 1e-300;
            const double q = w[J] / dj;
            w[J] = (lane == jj) ? dj : ((lane > jj) ? q : w[J]);  // column jj of L
#pragma unroll
            for (int i = J + 1; i < kPanelN; ++i) {
                const double lcj = lane_d(w[J], min(c0 + i, 63));  // L[c][jj], c = c0 + i
                if (lane >= c0 + i && c0 + i < D) w[i] = fma(-w[J], lcj, w[i]);
            }
        }
        panel_cols<J + 1>(w, lane, c0, D, sk);
    }
}

__device__ __forceinline__ void lower_panel_factor(double *L, int LD, int D, int c0, int *skip) {
    const int lane = threadIdx.x & 63;
    double w[kPanelN];
#pragma unroll
    for (int i = 0; i < kPanelN; ++i) w[i] = lds_or0(L, lane * LD + c0 + i, lane < D && c0 + i < D);
    int sk = 0;
    panel_cols<0>(w, lane, c0, D, sk);
#pragma unroll
    for (int i = 0; i < kPanelN; ++i)
        if (lane < D && c0 + i < D && lane >= c0 + i) L[lane * LD + c0 + i] = w[i];
    if (lane == 0) *skip = sk;
}

// The panel's 16 updates to element (r, c), r >= c >= c0 + 16, in ascending column order; all threads.  On the fp64
// matrix cores: tile (ti, tj), tj <= ti, of the trailing lower triangle starts from L's elements and takes the 16 terms
// fma(-L_rj, L_cj, .), j = c0 .. c0 + 15 ascending, as four k-ordered MFMA steps -- the VALU chain, bit for bit (the
// negated factor is exact).  valu: the per-element VALU loop.
template <bool EX>
__device__ __forceinline__ void lower_panel_trailing(double *L, int LD, int D, int c0, bool valu) {
    const int rows = D - (c0 + kPanelN);
    if (rows <= 0) return;  // (the last panel: nothing below it)
    if (!valu) {
        const int t0 = (c0 + kPanelN) / 16, nt = (D + 15) / 16, m = nt - t0;  // trailing tiles per side
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = __builtin_amdgcn_readfirstlane(blockDim.x >> 6), lane = threadIdx.x & 63;
        for (int tt = wv; tt < m * (m + 1) / 2; tt += nw) {
            int ti = 0, rem = tt;  // (ti, tj), tj <= ti, row-major over the lower tile triangle
            while (rem > ti) {
                rem -= ti + 1;
                ++ti;
            }
            const int r0 = 16 * (t0 + ti), q0 = 16 * (t0 + rem);
            f64x4 acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int a = r0 + (lane >> 4) + 4 * r, b = q0 + (lane & 15);
                acc[r] = (a < D && b < D && b <= a) ? L[a * LD + b] : 0.0;
            }
            acc = mfma_tile_acc(acc, [&](int i, int k) { return -lds_at<EX>(L, (r0 + i) * LD + c0 + k, r0 + i < D && k < kPanelN); },
                                [&](int k, int j) { return lds_at<EX>(L, (q0 + j) * LD + c0 + k, q0 + j < D && k < kPanelN); }, 0, kPanelN);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int a = r0 + (lane >> 4) + 4 * r, b = q0 + (lane & 15);
                if (a < D && b < D && b <= a) L[a * LD + b] = acc[r];
            }
        }
        return;
    }
    // only the trailing lower triangle (r >= c >= c0 + 16): e -> (r', c') row-major, r' = floor((sqrt(8e + 1) - 1) / 2)
    for (int e = threadIdx.x; e < rows * (rows + 1) / 2; e += blockDim.x) {
        int rr = (int)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
        while (rr * (rr + 1) / 2 > e) --rr;
        while ((rr + 1) * (rr + 2) / 2 <= e) ++rr;
        const int r = c0 + kPanelN + rr, c = c0 + kPanelN + (e - rr * (rr + 1) / 2);
        double acc = L[r * LD + c];
#pragma unroll
        for (int j = 0; j < kPanelN; ++j) acc = fma(-L[r * LD + c0 + j], L[c * LD + c0 + j], acc);  // (c0 + 16 <= c < D)
        L[r * LD + c] = acc;
    }
}

// Forward substitution panel (rows c0 .. c0 + 15) of X = G^{-1} X0 (G lower) on one wave (lane = column j, the 16
// rows in registers): row k divided by G_kk (inv: the lower inverse, columns j <= k only and 1 / G_kk on the
// diagonal), then the panel's later rows updated, fma(-G_rk, X_kj, .).
// Row I of a forward-substitution panel and then the later ones (template recursion, as panel_cols)
template <int I>
__device__ __forceinline__ void forward_rows(double (&w)[kPanelN], const double *G, int LD, int D, int c0, bool inv,
                                             int lane) {
    if constexpr (I < kPanelN) {
        const int k = c0 + I;
        if (k < D) {  // (wave-uniform)
            // the row's divisor and its multipliers in one round of (broadcast) LDS reads
            double g[kPanelN];
#pragma unroll
            for (int i2 = I; i2 < kPanelN; ++i2) g[i2] = lds_or0(G, (c0 + i2) * LD + k, c0 + i2 < D);
            const double gkk = g[I];
            const bool col = lane < D && (!inv || lane <= k);
            const double q = ((inv && lane == k) ? 1.0 : w[I]) / gkk;
            if (col) w[I] = q;
#pragma unroll
            for (int i2 = I + 1; i2 < kPanelN; ++i2)
                if (col && c0 + i2 < D) w[i2] = fma(-g[i2], w[I], w[i2]);
        }
        forward_rows<I + 1>(w, G, LD, D, c0, inv, lane);
    }
}

__device__ __forceinline__ void forward_panel(double *X, const double *G, int LD, int D, int c0, bool inv) {
    const int lane = threadIdx.x & 63;
    double w[kPanelN];
#pragma unroll
    for (int i = 0; i < kPanelN; ++i) w[i] = lds_or0(X, (c0 + i) * LD + lane, lane < D && c0 + i < D);
    forward_rows<0>(w, G, LD, D, c0, inv, lane);
#pragma unroll
    for (int i = 0; i < kPanelN; ++i)
        if (lane < D && c0 + i < D && (!inv || lane <= c0 + i)) X[(c0 + i) * LD + lane] = w[i];
}

// The panel's updates to rows r >= c0 + 16, fma(-G_rk, X_kj, .) for k = c0 .. c0 + 15 ascending (inv: k >= j only);
// all threads.
// lower: X0 (hence X) lower triangular -- elements j > r stay 0 and are skipped.
// On the matrix cores (!valu): tile (rows r0.., columns q0..) from X's elements plus the 16 terms as four k-ordered MFMA
// steps; the terms the VALU loop skips (inv: k < j; lower: X_kj = 0 for j > k) have X_kj = +0 and leave the chain alone
// (fma(-g, +0, v) = v for v != -0, and the chains never hold -0: they start from +0 or nonzero values).
template <bool EX>
__device__ __forceinline__ void forward_trailing(double *X, const double *G, int LD, int D, int c0, bool inv,
                                                 bool lower, bool valu) {
    const int rows = D - (c0 + kPanelN);
    // inv / lower: the columns right of the panel get nothing from it (X_kj = 0 for j > k, every panel row k < j), so
    // only columns 0 .. c0 + 15 are visited -- a quarter of the row's elements at the first panel
    const int W = (inv || lower) ? c0 + kPanelN : D;
    if (!valu) {
        if (rows <= 0) return;
        const int t0 = (c0 + kPanelN) / 16, nt = (D + 15) / 16, mr = nt - t0, mc = (W + 15) / 16;
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = __builtin_amdgcn_readfirstlane(blockDim.x >> 6), lane = threadIdx.x & 63;
        for (int tt = wv; tt < mr * mc; tt += nw) {
            const int r0 = 16 * (t0 + tt / mc), q0 = 16 * (tt % mc);
            f64x4 acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int a = r0 + (lane >> 4) + 4 * r, b = q0 + (lane & 15);
                acc[r] = (a < D && b < W) ? X[a * LD + b] : 0.0;
            }
            acc = mfma_tile_acc(acc, [&](int i, int k) { return -lds_at<EX>(G, (r0 + i) * LD + c0 + k, r0 + i < D && k < kPanelN); },
                                [&](int k, int j) { return lds_at<EX>(X, (c0 + k) * LD + q0 + j, q0 + j < W && k < kPanelN); }, 0, kPanelN);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int a = r0 + (lane >> 4) + 4 * r, b = q0 + (lane & 15);
                if (a < D && b < W) X[a * LD + b] = acc[r];
            }
        }
        return;
    }
    for (int e = threadIdx.x; e < rows * W; e += blockDim.x) {
        const int r = c0 + kPanelN + e / W, j = e - (e / W) * W;
        double acc = X[r * LD + j];
#pragma unroll
        for (int i = 0; i < kPanelN; ++i) {
            const int k = c0 + i;
            if (!inv || k >= j) acc = fma(-G[r * LD + k], X[k * LD + j], acc);
        }
        X[r * LD + j] = acc;
    }
}

__device__ __forceinline__ bool init_ok_records(const NiwArgs &A) { return A.init_k <= 0 && A.part_slot != nullptr; }

// Slot s's statistics from np8_suffstats_wide's run records (ParamArgs::part): the matching records are listed in
// record order (each thread scans a contiguous range of headers, an exclusive scan places its matches), then every
// thread sums its raw accumulator elements over the list in that order -- a fixed order, no atomics -- and adds
// them to what the atomic fallback left in acc.  S lands in L's lower triangle index-reversed (element
// (D - 1 - a, D - 1 - b) = S_ab, a <= b: where np8_niw_post forms J Psin J), s1 in s1.  Scratch: an int list of cap entries (Li's storage, unused until the factor exists).
// overlap(): block-wide work that needs none of the statistics (the NIW draws), run once while the first round of
// record loads is in flight (every thread calls it exactly once, no barrier inside).
template <class Overlap>
__device__ __forceinline__ void reduce_run_records(const NiwArgs &A, int s, const double *acc, double *L, int LD, double *s1, int *list,
                                   int cap, Overlap overlap) {
    // (the records' layout is np8_suffstats_wide's at DT: rows and columns >= D are the zero rows of the items)
    const int D = A.D, T = A.DT / 16, NT = T * (T + 1) / 2, RS = NT * 4 * 64 + T * 16;
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nt >> 6;
    __shared__ int woff[17];
    const int64_t per = (A.n_rec + nt - 1) / nt, h0 = (int64_t)tid * per, h1 = min(A.n_rec, h0 + per);
    // the thread's headers in batches of 8 independent loads, the matches as a bit mask (up to 64 headers per thread:
    // one scan of dependent loads per header cost ~25 us at C5)
    const bool fast = per <= 64;
    uint64_t mb = 0ull;
    int c = 0;
    if (fast) {
        for (int64_t hb = h0; hb < h1; hb += 8) {
            int32_t hv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) hv[i] = (hb + i < h1) ? A.part_slot[hb + i] : -1;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (hv[i] == s) mb |= 1ull << (hb + i - h0);
        }
        c = __popcll(mb);
    } else {
        for (int64_t h = h0; h < h1; ++h) c += (A.part_slot[h] == s);
    }
    int inc = c;  // block exclusive scan of the counts (thread order = record order)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
    }
    if (lane == 63) woff[wv] = inc;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
        for (int w = 0; w < nw; ++w) {
            const int x = woff[w];
            woff[w] = t;
            t += x;
        }
        woff[16] = t;
    }
    __syncthreads();
    int o = woff[wv] + inc - c;
    const int nm = woff[16];
    if (nm <= cap) {
        if (fast) {
            for (uint64_t m = mb; m; m &= m - 1ull) list[o++] = (int)(h0 + __ffsll((unsigned long long)m) - 1);
        } else {
            for (int64_t h = h0; h < h1; ++h)
                if (A.part_slot[h] == s) list[o++] = (int)h;
        }
    }
    __syncthreads();
    // this thread's elements e = tid + k nt (RS <= kRecE nt for D <= 64), two records per round of loads
    constexpr int kRecE = 12;
    double v[kRecE];
#pragma unroll
    for (int k = 0; k < kRecE; ++k) v[k] = 0.0;
    if (nm <= cap) {
        constexpr int kRecR = 4;  // records per round of loads (their sums still taken in record order; 8: no faster)
        for (int m = 0; m < nm; m += kRecR) {
            int64_t rr[kRecR];
#pragma unroll
            for (int q = 0; q < kRecR; ++q) rr[q] = (m + q < nm) ? (int64_t)list[m + q] * RS : -1;
            double a[kRecR][kRecE];
#pragma unroll
            for (int q = 0; q < kRecR; ++q)
#pragma unroll
                for (int k = 0; k < kRecE; ++k) {
                    const int e = tid + k * nt;
                    a[q][k] = (e < RS && rr[q] >= 0) ? A.part[rr[q] + e] : 0.0;
                }
            if (m == 0) overlap();  // (the first round's loads are in flight)
#pragma unroll
            for (int k = 0; k < kRecE; ++k)
#pragma unroll
                for (int q = 0; q < kRecR; ++q)
                    if (rr[q] >= 0) v[k] = v[k] + a[q][k];
        }
        if (nm == 0) overlap();
    } else {  // (more records than the scratch holds: every header in order)
        overlap();
        for (int64_t h = 0; h < A.n_rec; ++h)
            if (A.part_slot[h] == s)
#pragma unroll
                for (int k = 0; k < kRecE; ++k)
                    if (tid + k * nt < RS) v[k] = v[k] + A.part[h * RS + tid + k * nt];
    }
#pragma unroll
    for (int k = 0; k < kRecE; ++k) {
        const int e = tid + k * nt;
        if (e >= RS) continue;
        const double vk = v[k];
        if (e < NT * 256) {  // raw accumulator element (tile q, row group r, lane ln) -> (a, b)
            const int q = e >> 8, r = (e >> 6) & 3, ln = e & 63;
            int ti = 0, qq = q;
            while (qq >= T - ti) {
                qq -= T - ti;
                ++ti;
            }
            const int tj = ti + qq;
            const int a = 16 * ti + (ln >> 4) + 4 * r, b = 16 * tj + (ln & 15);
            if (a <= b && b < D) L[(D - 1 - a) * LD + (D - 1 - b)] = acc[D + pix(D, a, b)] + vk;
        } else {
            const int kk = e - NT * 256, dim = 16 * (kk >> 4) + (kk & 15);
            if (dim < D) s1[dim] = acc[dim] + vk;
        }
    }
}

// Scalars of slot s and of its candidate row (when it has one): c, isotropy, pruning radius unknown.
__device__ __forceinline__ void write_row_scalars(const NiwArgs &A, int s, int row, double c, double iso) {
    A.slot_c[s] = c;
    A.slot_iso[s] = iso;
    r2_unknown(A.r2, A.kcap, s);  // radius unknown: no pruning yet
    if (row >= 0) {
        double *e = A.cand + (int64_t)row * cand_stride(A.D) + A.D + A.D * (A.D + 1) / 2;
        e[kFieldC] = c;
        e[kFieldIso] = iso;
    }
}

}  // namespace

// LDS matrices use the leading dimension D + 1: row-strided reads by consecutive threads fall into
// different banks (a stride of D doubles put every lane of a wave on one bank).
size_t np8_niw_lds_bytes(int D) { return sizeof(double) * (4 * (size_t)D * (D + 1) + 10 * (size_t)D); }

// ---- posterior (and prior) draw -------------------------------------------------------------------
// Block b: init mode (A.init_k > 0) draws G0 sample b into slot init_map[b] on stream INIT_THETA;
// otherwise slot b's posterior on stream PARAM at the current epoch (oracle niw_draw_impl).
__global__ __launch_bounds__(kNiwPostThreads) void np8_niw_post(NiwArgs A) {
    const int D = A.D, W = D + D * (D + 1) / 2, LD = D + 1;
    const bool ex16 = D % 16 == 0;  // the MFMA tiles' instances without masking (lds_at)
    int s;
    int64_t n;
    uint64_t i;
    uint32_t t, stream;
    if (A.init_k > 0) {
        if ((int)blockIdx.x >= A.init_k) return;
        s = A.init_map[blockIdx.x];
        if (s < 0) return;
        n = 0;
        i = blockIdx.x;
        t = 0xFFFFFFFFu;
        stream = kStreamInitTheta;
    } else {
        s = blockIdx.x;
        n = A.cnt[s];
        if (n <= 0) return;
        i = (uint64_t)s;
        t = A.ctl->t_base + A.t;
        stream = kStreamParam;
    }
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *L = sm, *Li = L + D * LD, *B = Li + D * LD, *F = B + D * LD;
    double *xb = F + D * LD, *dm = xb + D, *mun = dm + D, *gv = mun + D, *z = gv + D, *y = z + D, *s1 = y + D,
           *anc = s1 + D;
    __shared__ double sh[4];
    __shared__ int bad;
    const int tid = threadIdx.x;
    const double *acc = A.acc + (int64_t)s * W;
    const double *S = acc + D;
    const double k0 = A.kappa0, nd = (double)n;
    const double kn = k0 + nd, nun = A.nu0 + nd;
    const double kf = (k0 * nd) / kn;
#ifdef NP8_EXP_NIW_TIMING
    long long tph[40] = {0};
#endif
    NIW_T(0)
    zero_block(L, 3 * D * LD);  // L, Li, B: upper triangles stay 0
    NIW_T(10)
    // the Bartlett draws and the normals (nothing of the statistics): with run records they run while the records'
    // first round of loads is in flight
    auto draws = [&]() {
        for (int a = tid; a < D; a += blockDim.x) {  // Bartlett diagonal
            const double g = chi2_mt(A.seed, i, t, stream, kNiwGammaCalls * (uint32_t)a, nun - a);
            gv[a] = g;
            B[a * LD + a] = sqrt(g);
        }
        // the normals by Philox call: one Box-Muller quad per call gives normals 4q .. 4q + 3 (normal_at's layout), so
        // each call is made once, not once per normal -- B's off-diagonals first, then z
        const int nb = D * (D - 1) / 2, nn = nb + D;
        for (int qd = tid; 4 * qd < nn; qd += blockDim.x) {
            double g[4];
            normal_quad(A.seed, i, t, stream, kNiwNormalCall0 + (uint32_t)qd, g);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = 4 * qd + k;
                if (e < nb) {
                    int a, b;
                    lower_index(e, a, b);
                    B[a * LD + b] = g[k];
                } else if (e < nn) {
                    z[e - nb] = g[k];
                }
            }
        }
    };
    const bool recs = A.part != nullptr && n > 0 && init_ok_records(A);
    if (recs) {  // the statistics from np8_suffstats_wide's run records: S into L's lower triangle, s1
        __syncthreads();
        reduce_run_records(A, s, acc, L, LD, s1, reinterpret_cast<int *>(Li), (int)(D * LD * 2), draws);
        __syncthreads();
        NIW_T(11)
    } else {
        __syncthreads();  // (zero_block's writes to B land first)
        draws();
    }
    for (int a = tid; a < D; a += blockDim.x) {
        anc[a] = (n > 0) ? A.slot_mu[(int64_t)s * D + a] : 0.0;
        if (!recs) s1[a] = (n > 0) ? acc[a] : 0.0;
        xb[a] = (n > 0) ? anc[a] + s1[a] / nd : A.mu0[a];
        dm[a] = xb[a] - A.mu0[a];
        mun[a] = fma(k0, A.mu0[a], nd * xb[a]) / kn;
    }
    if (tid == 0) bad = 0;
    __syncthreads();
    // J Psin J (J the index reversal) formed in LDS's lower triangle by all threads: element (r, j), r >= j, is
    // Psin[D-1-r][D-1-j] (the statistics and Psi0 come from HBM once); the Bartlett draws (they need nothing of
    // Psin) in the same phase
    auto psin = [&](int r, int j, double Srj) {  // element (r, j), r >= j
        const int ri = D - 1 - r, ji = D - 1 - j;  // ri <= ji
        const double sc = (n > 0) ? Srj - (s1[ri] * s1[ji]) / nd : 0.0;
        L[r * LD + j] = fma(kf, dm[ri] * dm[ji], A.Psi0[ri * D + ji] + sc);
    };
    if (recs) {  // (two loops: the statistics' source is LDS or HBM, and a select of the two pointers is a flat load)
        for (int e = tid; e < D * D; e += blockDim.x) {
            const int r = e / D, j = e - r * D;
            if (j <= r) psin(r, j, L[r * LD + j]);
        }
    } else {
        for (int e = tid; e < D * D; e += blockDim.x) {
            const int r = e / D, j = e - r * D;
            if (j <= r) psin(r, j, S[pix(D, D - 1 - r, D - 1 - j)]);
        }
    }
    __syncthreads();
    NIW_T(1)
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // (wave-uniform: SGPR loops and branches)
    // Lr = chol(J Psin J), blocked right-looking (panels of 16 columns: the panel factored by wave 0 in registers,
    // the rows below updated by every thread): element (r, c) receives fma(-L_rk, L_ck, .) for k = 0, 1, ... in
    // order, then the division by its pivot -- the operations of the oracle's left-looking loop, in its order, with
    // two barriers per panel.  U = J Lr J is upper with Psin = U U^T.  Wave 1 meanwhile: y = B^{-T} z / sqrt(kn).
    __shared__ int skip_s;
    // (the solve for y is serial in its 64 rows: 16 of them beside each panel's factor keep it off the critical path)
    double yv = 0.0;
    if (wv == 1) {
        const int ln = tid & 63;
        yv = (ln < D) ? z[ln] * (1.0 / sqrt(kn)) : 0.0;
    }
    for (int p = 0; p * kPanelN < D; ++p) {
        const int c0 = p * kPanelN;
        if (wv == 0) {
            lower_panel_factor(L, LD, D, c0, &skip_s);
        } else if (wv == 1) {
            const int ln = tid & 63;
            for (int k = D - 1 - c0; k >= 0 && k > D - 1 - c0 - kPanelN; --k) {
                const double yk = lane_d(yv, k) / B[k * LD + k];
                if (ln == k) y[k] = yk;
                if (ln < k) yv = fma(-B[k * LD + ln], yk, yv);
            }
        }
        __syncthreads();
        NIW_T(14 + p)
        if (skip_s) {  // block-uniform: not numerically positive definite
            if (tid == 0) bad = 1;
            break;
        }
        if (ex16)
            lower_panel_trailing<true>(L, LD, D, c0, A.valu);
        else
            lower_panel_trailing<false>(L, LD, D, c0, A.valu);
        __syncthreads();
        NIW_T(18 + p)
    }
    __syncthreads();
    NIW_T(2)
    if (bad) {  // block-uniform: not numerically positive definite, the slot keeps its parameters
        if (n > 0)
            for (int w = tid; w < W; w += blockDim.x) A.acc[(int64_t)s * W + w] = 0.0;
        return;
    }
    // M = Lr^{-1} (U^{-1} = J M J) and T = B^{-1} U^T (lower; into F's storage) as blocked forward substitutions:
    // row k final once divided by its diagonal, then it updates every later row -- element (r, j) receives
    // fma(-L_rk, M_kj, .) for k = j, ..., r - 1 (T: fma(-B_ak, T_kj, .) for k = 0, ..., a - 1) in order, as the
    // oracle's loops do; the two panels side by side (waves 0 and 1), the trailing rows by every thread.  Wave 2: the
    // new mean mun + U y.
    double *T = F;
    for (int e = tid; e < D * D; e += blockDim.x) {
        const int a = e / D, j = e - a * D;
        T[a * LD + j] = (j <= a) ? L[(D - 1 - j) * LD + (D - 1 - a)] : 0.0;  // U^T_aj = U_ja = Lr[D-1-j][D-1-a]
    }
    __syncthreads();
    for (int p = 0; p * kPanelN < D; ++p) {
        const int c0 = p * kPanelN;
        if (wv == 0) {
            forward_panel(Li, L, LD, D, c0, true);
        } else if (wv == 1) {
            forward_panel(T, B, LD, D, c0, false);
        } else if (wv == 2 && p == 0) {
            for (int a = tid - 128; a < D; a += 64) {
                double v = 0.0;  // (U y)_a = sum_{k >= a} Lr[D-1-a][D-1-k] y_k
#pragma unroll 8
                for (int k = a; k < D; ++k) v = fma(L[(D - 1 - a) * LD + (D - 1 - k)], y[k], v);
                mun[a] = mun[a] + v;  // (mun no longer needed: the new mean in its place)
            }
        }
        __syncthreads();
        NIW_T(22 + p)
        if (ex16) {
            forward_trailing<true>(Li, L, LD, D, c0, true, false, A.valu);
            forward_trailing<true>(T, B, LD, D, c0, false, true, A.valu);
        } else {
            forward_trailing<false>(Li, L, LD, D, c0, true, false, A.valu);
            forward_trailing<false>(T, B, LD, D, c0, false, true, A.valu);
        }
        __syncthreads();
        NIW_T(26 + p)
    }
    __syncthreads();
    NIW_T(3)
    const int row = A.write_cand ? A.dense_of[s] : -1;
    for (int a = tid; a < D; a += blockDim.x) {
        A.slot_mu[(int64_t)s * D + a] = mun[a];
        if (row >= 0) A.cand[(int64_t)row * cand_stride(D) + a] = mun[a];
    }
    // (L's diagonal leaves with its logarithms: L's storage takes Sigma next, for the eigenvalue bound)
    double *lg = xb, *rs = anc + D;
    for (int a = tid; a < D; a += blockDim.x) lg[a] = log_pos(L[a * LD + a]);
    if (tid == 0) {
        LogAcc la;
        for (int a = 0; a < D; ++a) la.add(gv[a], a, D - 1);
        sh[0] = la.sumlog;
    }
    __syncthreads();
    if (tid == 0) {
        double sl = 0.0;
        for (int a = 0; a < D; ++a) sl += lg[a];
        sh[1] = sl;
    }
    const bool bound = A.lam_lo != nullptr;
    if (A.valu) {
        sigma_from_t(D, LD, F, A.slot_sigma + (int64_t)s * D * D, bound ? L : nullptr);  // Sigma = T^T T
    } else {
        if (ex16)
            sigma_from_t_mfma<true>(D, LD, F, A.slot_sigma + (int64_t)s * D * D, bound ? L : nullptr);
        else
            sigma_from_t_mfma<false>(D, LD, F, A.slot_sigma + (int64_t)s * D * D, bound ? L : nullptr);
    }
    __syncthreads();
    NIW_T(4)
    // R = B^T U^{-1} (upper, into F's storage: T is dead): R_ab = sum_{k = a..b} B_ka M[D-1-k][D-1-b]
    if (A.valu) {
        for (int e = tid; e < D * D; e += blockDim.x) {
            const int a = e / D, b = e - a * D;
            double v = 0.0;
            if (b >= a) {
#pragma unroll 8
                for (int k = a; k <= b; ++k) v = fma(B[k * LD + a], Li[(D - 1 - k) * LD + (D - 1 - b)], v);
            }
            F[a * LD + b] = v;
        }
    } else {
        if (ex16)
            r_from_b_mfma<true>(D, LD, B, Li, F);
        else
            r_from_b_mfma<false>(D, LD, B, Li, F);
    }
    __syncthreads();
    NIW_T(5)
    const double iso = A.valu ? write_pprime_r(D, LD, F, A.slot_P + (int64_t)s * (D * (D + 1) / 2),
                                               row >= 0 ? A.cand + (int64_t)row * cand_stride(D) + D : nullptr)
                       : ex16 ? write_pprime_r_mfma<true>(D, LD, F, A.slot_P + (int64_t)s * (D * (D + 1) / 2),
                                                          row >= 0 ? A.cand + (int64_t)row * cand_stride(D) + D : nullptr)
                              : write_pprime_r_mfma<false>(D, LD, F, A.slot_P + (int64_t)s * (D * (D + 1) / 2),
                                                    row >= 0 ? A.cand + (int64_t)row * cand_stride(D) + D : nullptr);
    NIW_T(6)
    if (A.wA) {  // the wide path: the contraction rows from R itself, the eigenvalue bound from Sigma's row sums
        const int DT = A.DT, NCH = (DT / 16) * (DT / 16 + 1) / 2;
        wide_write_rows(D, DT, F, LD, mun, A.wA + (int64_t)s * DT * DT, A.wfrag + (int64_t)s * (NCH * 256 + DT),
                        A.wmu + (int64_t)s * DT);
    }
    if (bound) {
        // lambda_min(P) = 1 / lambda_max(Sigma), lambda_max(Sigma) = rho(Sigma) <= ||Sigma^n||^(1/n), n = 2^k (any
        // consistent norm; max |row sum| here) -- within a few % of lambda_max where the Gershgorin bound ||Sigma||
        // can be 40% above it.  Sigma is scaled by g = ||Sigma|| first (entries of (Sigma/g)^n stay in [0, 1], no
        // overflow, and ||(Sigma/g)^n|| >= D^(-n/2) >= 8^-32 at D = 64, k <= 5: no underflow); 1% for the fp32
        // factor, the fp32 contraction and the rounding.
        NIW_T(30)
        const double g = max_abs_row_sum(D, LD, L, rs);
        const double rg = (g > 0.0) ? 1.0 / g : 0.0;
        for (int e = tid; e < D * D; e += blockDim.x) {
            const int a = e / D, b = e - a * D;
            L[a * LD + b] *= rg;
        }
        __syncthreads();
        // kBoundSquarings squarings, (Sigma/g)^(2^k), through L -> B -> Li -> L ... (B and Li are free once R exists)
        // (unrolled: each buffer is a known LDS array, so the loads stay ds_read -- a runtime-indexed pointer table
        // made them flat loads, 2x slower)
        auto buf = [&](int k) -> double * { return k == 0 ? L : (k == 1 ? B : Li); };
        // (written out: a loop the compiler failed to unroll left buf() runtime-indexed -- flat loads)
        auto square = [&](const double *X, double *Y) {
            if (A.valu)
                sym_square(D, LD, X, Y);
            else if (ex16)
                sym_square_mfma<true>(D, LD, X, Y);
            else
                sym_square_mfma<false>(D, LD, X, Y);
            __syncthreads();
        };
        static_assert(kBoundSquarings >= 0 && kBoundSquarings <= 6, "squarings L -> B -> Li -> L ...");
        NIW_T(32)
        if (kBoundSquarings > 0) square(L, B);
        NIW_T(33)
        if (kBoundSquarings > 1) square(B, Li);
        NIW_T(34)
        if (kBoundSquarings > 2) square(Li, L);
        NIW_T(35)
        if (kBoundSquarings > 3) square(L, B);
        NIW_T(36)
        if (kBoundSquarings > 4) square(B, Li);
        if (kBoundSquarings > 5) square(Li, L);
        NIW_T(31)
        const double m = max_abs_row_sum(D, LD, buf(kBoundSquarings % 3), rs);
        if (tid == 0) {
            double root = m;
            for (int q = 0; q < kBoundSquarings; ++q) root = sqrt(root);
            const double lmax = g * root;
            A.lam_lo[s] = (lmax > 0.0 && lmax < 1e300) ? 0.99 / lmax : 0.0;
        }
    }
    NIW_T(7)
    NIW_T(8)
#ifdef NP8_EXP_NIW_TIMING
    if (tid == 0 && s < 2 && (t % 16) == 0)
        printf("niw_post s=%d t=%u n=%ld phases %lld %lld %lld %lld %lld %lld %lld %lld\n", s, t, (long)n, tph[1] - tph[0],
               tph[2] - tph[1], tph[3] - tph[2], tph[4] - tph[3], tph[5] - tph[4], tph[6] - tph[5], tph[7] - tph[6],
               tph[8] - tph[7]);
    if (tid == 0 && s < 1 && (t % 16) == 0) {
        printf("niw_post detail t=%u:", t);
        for (int k = 10; k < 37; ++k) printf(" %d:%lld", k, tph[k] ? tph[k] - tph[0] : -1ll);
        printf("\n");
    }
#endif
    if (tid == 0) write_row_scalars(A, s, row, fma(0.5, sh[0], fma(-0.5 * (double)D, kLog2Pi, -sh[1])), iso);
    if (n > 0)
        for (int w = tid; w < W; w += blockDim.x) A.acc[(int64_t)s * W + w] = 0.0;  // zero for the next sweep
}

// ---- picked auxiliaries -> slots (oracle niw_aux_slot) ------------------------------------------------
__global__ __launch_bounds__(kNiwThreads) void np8_niw_aux_slots(NiwArgs A) {
    const int D = A.D, LD = D + 1;
    const int npend = A.ctl->n_pend;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double *B = sm, *RB = B + D * LD, *F = RB + D * LD;
    double *gv = F + D * LD, *z = gv + D, *h = z + D, *cs = h + D, *y = cs + D, *ry = y + D, *eps = ry + D, *dt = eps + D;
    __shared__ double sh[8];
    const int tid = threadIdx.x;
    const uint32_t t = A.ctl->t_base + A.t;
    for (int p = blockIdx.x; p < npend; p += gridDim.x) {
        const int64_t *pe = A.pend + 4 * (int64_t)p;
        const double *vmu = reinterpret_cast<const double *>(A.recs + pe[0]);
        const uint64_t i = (uint64_t)pe[1];
        const int m = (int)pe[2], s = (int)pe[3];
        const uint32_t base = (uint32_t)m * kNiwAuxCalls;
        __syncthreads();  // LDS of the previous request fully consumed
        zero_block(B, D * LD);
        for (int a = tid; a < D; a += blockDim.x) dt[a] = vmu[1 + a];
        __syncthreads();
        for (int a = tid; a < D; a += blockDim.x) {
            const double g = chi2_mt(A.seed, i, t, kStreamAuxNiw, base + kNiwGammaCalls * (uint32_t)a, A.nu0 - a);
            gv[a] = g;
            B[a * LD + a] = sqrt(g);
        }
        if (tid == blockDim.x - 1) {
            sh[1] = niw_chi_perp(A.seed, i, t, kStreamAuxNiw, base, D);
            sh[2] = normal_at(A.seed, i, t, kStreamAuxNiw, base + kNiwAuxCalls - 1u, 0);
        }
        for (int e = tid; e < D * (D - 1) / 2; e += blockDim.x) {
            int a, b;
            lower_index(e, a, b);
            B[a * LD + b] = normal_at(A.seed, i, t, kStreamAuxDir, base, (uint32_t)e);
        }
        for (int j = tid; j + 1 < D; j += blockDim.x)
            z[1 + j] = normal_at(A.seed, i, t, kStreamAuxDir, base, (uint32_t)(D * (D - 1) / 2 + j));
        __syncthreads();
        if (tid == 0) {
            LogAcc la;
            for (int a = 0; a < D; ++a) la.add(gv[a], a, D - 1);
            sh[0] = la.sumlog;
            double w2 = 0.0;
            for (int j = 1; j < D; ++j) w2 = fma(z[j], z[j], w2);
            const double sc = (w2 > 0.0) ? sqrt(sh[1] / w2) : 0.0;
            for (int j = 1; j < D; ++j) z[j] *= sc;
            double n2 = 0.0;
            for (int a = 0; a < D; ++a) n2 = fma(dt[a], dt[a], n2);
            const double nd = sqrt(n2);
            double beta = 0.0, sig = 1.0;
            for (int a = 0; a < D; ++a) h[a] = 0.0;
            if (nd > 0.0) {
                for (int a = 0; a < D; ++a) h[a] = dt[a] / nd;
                const double sg = (h[0] >= 0.0) ? 1.0 : -1.0;
                h[0] = h[0] + sg;
                double hh = 0.0;
                for (int a = 0; a < D; ++a) hh = fma(h[a], h[a], hh);
                beta = 2.0 / hh;
                sig = -sg;
            }
            z[0] = sig * sh[2];
            sh[3] = beta;
        }
        __syncthreads();
        const double beta = sh[3];
        for (int b = tid; b < D; b += blockDim.x) {  // column sums h^T B
            double v = 0.0;
            #pragma unroll 8
            for (int k = b; k < D; ++k) v = fma(h[k], B[k * LD + b], v);
            cs[b] = v;
        }
        __syncthreads();
        for (int e = tid; e < D * D; e += blockDim.x) {
            const int a = e / D, b = e - a * D;
            RB[a * LD + b] = fma(-(beta * h[a]), cs[b], B[a * LD + b]);
        }
        __syncthreads();
        for (int e = tid; e < D * D; e += blockDim.x) {  // F = U RB
            const int a = e / D, b = e - a * D;
            double v = 0.0;
            #pragma unroll 8
            for (int k = 0; k <= a; ++k) v = fma(A.U[a * D + k], RB[k * LD + b], v);
            F[a * LD + b] = v;
        }
        __syncthreads();
        const int row = A.dense_of[s];
        const double iso = write_pprime(D, LD, F, A.slot_P + (int64_t)s * (D * (D + 1) / 2),
                                        row >= 0 ? A.cand + (int64_t)row * cand_stride(D) + D : nullptr);
        if (tid == 0) {  // mu = mu0 + U^{-T} R B^{-T} z / sqrt(kappa0)
            for (int a = D - 1; a >= 0; --a) {
                double v = z[a] * A.rsk;
                #pragma unroll 8
                for (int k = a + 1; k < D; ++k) v = fma(-B[k * LD + a], y[k], v);
                y[a] = v / B[a * LD + a];
            }
            double hy = 0.0;
            for (int k = 0; k < D; ++k) hy = fma(h[k], y[k], hy);
            for (int a = 0; a < D; ++a) ry[a] = fma(-(beta * h[a]), hy, y[a]);
            for (int a = D - 1; a >= 0; --a) {
                double v = ry[a];
                #pragma unroll 8
                for (int k = a + 1; k < D; ++k) v = fma(-A.U[k * D + a], eps[k], v);
                eps[a] = v / A.U[a * D + a];
            }
            for (int a = 0; a < D; ++a) {
                const double mm = A.mu0[a] + eps[a];
                A.slot_mu[(int64_t)s * D + a] = mm;
                if (row >= 0) A.cand[(int64_t)row * cand_stride(D) + a] = mm;
            }
        }
        for (int b = tid; b < D; b += blockDim.x) {  // R U^{-1}
            double v = 0.0;
            #pragma unroll 8
            for (int k = b; k < D; ++k) v = fma(h[k], A.Uinv[k * D + b], v);
            cs[b] = v;
        }
        __syncthreads();
        for (int e = tid; e < D * D; e += blockDim.x) {
            const int a = e / D, b = e - a * D;
            RB[a * LD + b] = fma(-(beta * h[a]), cs[b], A.Uinv[e]);
        }
        __syncthreads();
        write_sigma(D, LD, B, RB, false, F, A.slot_sigma + (int64_t)s * D * D);
        if (tid == 0) write_row_scalars(A, s, row, fma(0.5, sh[0], A.caux), iso);
    }
}

// Dynamic LDS above 64 KB (D > 44) must be allowed per kernel.
static hipError_t allow_lds(const void *fn, size_t bytes) {
    if (bytes <= 65536) return hipSuccess;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// Called once per context at creation (not inside a stream capture).
hipError_t np8_niw_prepare(int D) {
    const size_t lds = np8_niw_lds_bytes(D);
    hipError_t e = allow_lds(reinterpret_cast<const void *>(&np8_niw_post), lds);
    if (e == hipSuccess) e = allow_lds(reinterpret_cast<const void *>(&np8_niw_aux_slots), lds);
    return e;
}

hipError_t np8_launch_niw_post(const NiwArgs &A, int nblocks, hipStream_t s) {
    if (nblocks <= 0) return hipSuccess;
    const size_t lds = np8_niw_lds_bytes(A.D);
    hipLaunchKernelGGL(np8_niw_post, dim3((unsigned)nblocks), dim3(kNiwPostThreads), lds, s, A);
    return hipGetLastError();
}

hipError_t np8_launch_niw_aux_slots(const NiwArgs &A, hipStream_t s) {
    const size_t lds = np8_niw_lds_bytes(A.D);
    hipLaunchKernelGGL(np8_niw_aux_slots, dim3(64), dim3(kNiwThreads), lds, s, A);
    return hipGetLastError();
}
