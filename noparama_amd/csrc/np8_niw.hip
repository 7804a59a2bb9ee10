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

// Sigma = T^T T, B T = Rhs (B lower triangular): one thread per column of T, then per element.
__device__ void write_sigma(int D, int LD, const double *B, const double *Rhs, bool rhs_transposed, double *T, double *Sigma) {
    for (int j = threadIdx.x; j < D; j += blockDim.x)
        for (int a = 0; a < D; ++a) {
            double s = rhs_transposed ? Rhs[j * LD + a] : Rhs[a * LD + j];
            #pragma unroll 8
            for (int k = 0; k < a; ++k) s = fma(-B[a * LD + k], T[k * LD + j], s);
            T[a * LD + j] = s / B[a * LD + a];
        }
    __syncthreads();
    for (int e = threadIdx.x; e < D * D; e += blockDim.x) {
        const int a = e / D, b = e - a * D;
        double s = 0.0;
        #pragma unroll 8
        for (int k = 0; k < D; ++k) s = fma(T[k * LD + a], T[k * LD + b], s);
        Sigma[e] = s;
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
    for (int j = 0; j < D; ++j) {
        if (tid == 0) {
            double v = L[j * LD + j];
            #pragma unroll 8
            for (int k = 0; k < j; ++k) v = fma(-L[j * LD + k], L[j * LD + k], v);
            if (!(v > 0.0)) {
                bad = 1;
                v = 1.0;
            }
            L[j * LD + j] = sqrt(v);
        }
        __syncthreads();
        for (int r = j + 1 + tid; r < D; r += blockDim.x) {
            double v = L[r * LD + j];
            #pragma unroll 8
            for (int k = 0; k < j; ++k) v = fma(-L[r * LD + k], L[j * LD + k], v);
            L[r * LD + j] = v / L[j * LD + j];
        }
        __syncthreads();
    }
    if (bad) {  // block-uniform: not numerically positive definite, the slot keeps its parameters
        if (n > 0)
            for (int w = tid; w < W; w += blockDim.x) A.acc[(int64_t)s * W + w] = 0.0;
        return;
    }
    for (int j = tid; j < D; j += blockDim.x) {  // Li = L^{-1}, one column per thread
        Li[j * LD + j] = 1.0 / L[j * LD + j];
        for (int r = j + 1; r < D; ++r) {
            double v = 0.0;
            #pragma unroll 8
            for (int k = j; k < r; ++k) v = fma(-L[r * LD + k], Li[k * LD + j], v);
            Li[r * LD + j] = v / L[r * LD + r];
        }
    }
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
    const int row = A.write_cand ? A.dense_of[s] : -1;
    const double iso = write_pprime(D, LD, F, A.slot_P + (int64_t)s * (D * (D + 1) / 2),
                                    row >= 0 ? A.cand + (int64_t)row * cand_stride(D) + D : nullptr);
    if (tid == 0) {  // y = B^{-T} z / sqrt(kn)
        const double rskn = 1.0 / sqrt(kn);
        for (int a = D - 1; a >= 0; --a) {
            double v = z[a] * rskn;
            #pragma unroll 8
            for (int k = a + 1; k < D; ++k) v = fma(-B[k * LD + a], y[k], v);
            y[a] = v / B[a * LD + a];
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
    write_sigma(D, LD, B, L, true, F, A.slot_sigma + (int64_t)s * D * D);  // T = B^{-1} L^T
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
