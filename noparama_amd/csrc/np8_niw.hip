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
__global__ __launch_bounds__(kNiwThreads) void np8_niw_post(NiwArgs A) {
    const int D = A.D, W = D + D * (D + 1) / 2, LD = D + 1;
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
    long long tph[12];
#endif
    NIW_T(0)
    zero_block(L, 3 * D * LD);  // L, Li, B: upper triangles stay 0
    for (int a = tid; a < D; a += blockDim.x) {
        anc[a] = (n > 0) ? A.slot_mu[(int64_t)s * D + a] : 0.0;
        s1[a] = (n > 0) ? acc[a] : 0.0;
        xb[a] = (n > 0) ? anc[a] + s1[a] / nd : A.mu0[a];
        dm[a] = xb[a] - A.mu0[a];
        mun[a] = fma(k0, A.mu0[a], nd * xb[a]) / kn;
    }
    if (tid == 0) bad = 0;
    __syncthreads();
    // Psin's lower triangle formed in LDS by all threads (the statistics and Psi0 come from HBM once),
    // then the left-looking Cholesky in place: the diagonal of column j, then its rows below -- the
    // operations of the oracle's loop, in its order
    for (int e = tid; e < D * D; e += blockDim.x) {
        const int r = e / D, j = e - r * D;
        if (j > r) continue;
        const double sc = (n > 0) ? S[pix(D, j, r)] - (s1[r] * s1[j]) / nd : 0.0;
        L[r * LD + j] = fma(kf, dm[r] * dm[j], A.Psi0[r * D + j] + sc);
    }
    __syncthreads();
    NIW_T(1)
    // right-looking: per column the pivot and the scaled column, then the trailing update.  Element (r, c)
    // receives fma(-L_rk, L_ck, .) for k = 0, 1, ... in order, then the division by its pivot: the
    // operations of the oracle's left-looking loop, in its order.  (The pivot is read by every thread
    // and written back after the barrier.)
    for (int j = 0; j < D; ++j) {
        const double v = L[j * LD + j];  // fully updated (behind the barrier)
        if (!(v > 0.0)) {                // block-uniform
            if (tid == 0) bad = 1;
            break;
        }
        const double dj = sqrt(v);
        for (int r = j + 1 + tid; r < D; r += blockDim.x) L[r * LD + j] = L[r * LD + j] / dj;
        __syncthreads();
        if (tid == 0) L[j * LD + j] = dj;
        for (int r = j + 1 + (tid >> 4); r < D; r += 16)  // 16 x 16 threads over (r, c), no index division
            for (int c = j + 1 + (tid & 15); c <= r; c += 16) L[r * LD + c] = fma(-L[r * LD + j], L[c * LD + j], L[r * LD + c]);
        __syncthreads();
    }
    __syncthreads();
    NIW_T(2)
    if (bad) {  // block-uniform: not numerically positive definite, the slot keeps its parameters
        if (n > 0)
            for (int w = tid; w < W; w += blockDim.x) A.acc[(int64_t)s * W + w] = 0.0;
        return;
    }
    // Li = L^{-1} (lower), right-looking over rows: row k is final once its sums are divided by L_kk, then
    // it updates every later row -- element (r, j) receives fma(-L_rk, Li_kj, .) for k = j, ..., r - 1 in
    // order from 0, as the oracle's column loop does
    for (int k = 0; k < D; ++k) {
        const double lkk = L[k * LD + k];
        for (int j = tid; j <= k; j += blockDim.x) Li[k * LD + j] = (j == k) ? 1.0 / lkk : Li[k * LD + j] / lkk;
        __syncthreads();
        for (int r = k + 1 + (tid >> 4); r < D; r += 16)  // rows r > k, columns j <= k
            for (int j = tid & 15; j <= k; j += 16) Li[r * LD + j] = fma(-L[r * LD + k], Li[k * LD + j], Li[r * LD + j]);
        __syncthreads();
    }
    NIW_SYNC()
    NIW_T(3)
    for (int a = tid; a < D; a += blockDim.x) {  // Bartlett diagonal
        const double g = chi2_mt(A.seed, i, t, stream, kNiwGammaCalls * (uint32_t)a, nun - a);
        gv[a] = g;
        B[a * LD + a] = sqrt(g);
    }
    for (int e = tid; e < D * (D - 1) / 2; e += blockDim.x) {
        int a, b;
        lower_index(e, a, b);
        B[a * LD + b] = normal_at(A.seed, i, t, stream, kNiwNormalCall0, (uint32_t)e);
    }
    for (int j = tid; j < D; j += blockDim.x)
        z[j] = normal_at(A.seed, i, t, stream, kNiwNormalCall0, (uint32_t)(D * (D - 1) / 2 + j));
    __syncthreads();
    NIW_T(4)
    if (tid == 0) {
        LogAcc la;
        for (int a = 0; a < D; ++a) la.add(gv[a], a, D - 1);
        sh[0] = la.sumlog;
    }
    for (int e = tid; e < D * D; e += blockDim.x) {  // F = Li^T B
        const int a = e / D, b = e - a * D;
        double v = 0.0;
        #pragma unroll 8
        for (int k = (a > b ? a : b); k < D; ++k) v = fma(Li[k * LD + a], B[k * LD + b], v);
        F[a * LD + b] = v;
    }
    __syncthreads();
    NIW_T(5)
    const int row = A.write_cand ? A.dense_of[s] : -1;
    const double iso = write_pprime(D, LD, F, A.slot_P + (int64_t)s * (D * (D + 1) / 2),
                                    row >= 0 ? A.cand + (int64_t)row * cand_stride(D) + D : nullptr);
    NIW_T(6)
    if (tid < 64) {  // y = B^{-T} z / sqrt(kn): one wave, lane a holds y_a's sum; column k leaves it as k falls
        const double rskn = 1.0 / sqrt(kn);
        double v = (tid < D) ? z[tid] * rskn : 0.0;
        for (int k = D - 1; k >= 0; --k) {
            const double yk = __shfl(v, k) / B[k * LD + k];
            if (tid == k) y[k] = yk;
            if (tid < k) v = fma(-B[k * LD + tid], yk, v);
        }
    }
    __syncthreads();
    for (int a = tid; a < D; a += blockDim.x) {
        double v = 0.0;
        #pragma unroll 8
        for (int k = 0; k <= a; ++k) v = fma(L[a * LD + k], y[k], v);
        const double m = mun[a] + v;
        A.slot_mu[(int64_t)s * D + a] = m;
        if (row >= 0) A.cand[(int64_t)row * cand_stride(D) + a] = m;
    }
    NIW_SYNC()
    NIW_T(7)
    write_sigma(D, LD, B, L, true, F, A.slot_sigma + (int64_t)s * D * D);  // T = B^{-1} L^T
    NIW_SYNC()
    NIW_T(8)
#ifdef NP8_EXP_NIW_TIMING
    if (tid == 0 && s < 2 && (t % 16) == 0)
        printf("niw_post s=%d t=%u n=%ld phases %lld %lld %lld %lld %lld %lld %lld %lld\n", s, t, (long)n, tph[1] - tph[0],
               tph[2] - tph[1], tph[3] - tph[2], tph[4] - tph[3], tph[5] - tph[4], tph[6] - tph[5], tph[7] - tph[6],
               tph[8] - tph[7]);
#endif
    if (tid == 0) {
        double sl = 0.0;
        for (int a = 0; a < D; ++a) sl += log_pos(L[a * LD + a]);
        write_row_scalars(A, s, row, fma(0.5, sh[0], fma(-0.5 * (double)D, kLog2Pi, -sl)), iso);
    }
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
    hipLaunchKernelGGL(np8_niw_post, dim3((unsigned)nblocks), dim3(kNiwThreads), lds, s, A);
    return hipGetLastError();
}

hipError_t np8_launch_niw_aux_slots(const NiwArgs &A, hipStream_t s) {
    const size_t lds = np8_niw_lds_bytes(A.D);
    hipLaunchKernelGGL(np8_niw_aux_slots, dim3(64), dim3(kNiwThreads), lds, s, A);
    return hipGetLastError();
}
