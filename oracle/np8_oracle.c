/*
 * np8_oracle.c -- TEST INFRASTRUCTURE ONLY (see np8_oracle.h).  CPU restatement of noparama's
 * Neal-8 sweep.  Compiled with -O2 -ffp-contract=off so that every fused multiply-add is the
 * explicit fma() written here, exactly as in the HIP kernels (DESIGN.md "Chain specification").
 */
#include "np8_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define LOG2PI 1.8378770664093454835606594728112
#define TWO_PI 6.283185307179586476925286766559

/* ================================================================================================
 * Primitives
 * ============================================================================================== */

static inline uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

/* Philox4x32-10 (Salmon et al., SC'11; Random123 philox4x32round / philox4x32bumpkey). */
void np8o_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

/* Open-interval uniform from 64 random bits: an odd 53-bit integer times 2^-53, never 0 or 1. */
double np8o_u01(uint32_t hi, uint32_t lo) {
    uint64_t v = (((uint64_t)hi << 32) | lo) >> 11;
    v |= 1u;
    return (double)v * 0x1.0p-53;
}

/* (k + 1/2) 2^-32: 32-bit uniform on (0,1), exact (the Box-Muller inputs). */
static inline double u32_01(uint32_t k) { return fma((double)k, 0x1.0p-32, 0x1.0p-33); }

/* 1/y on the log's denominator range: minimax quadratic + three Newton steps (fma only). */
static inline double recip_logden(double y) {
    double r = fma(fma(0.11686276, y, -0.72244362), y, 1.47775548);
    for (int k = 0; k < 3; ++k) r = fma(r, fma(-y, r, 1.0), r);
    return r;
}

static void philox_call(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call, uint32_t out[4]) {
    uint32_t ctr[4] = {(uint32_t)i, (uint32_t)(i >> 32), t, (stream << 24) | (call & 0xFFFFFFu)};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    np8o_philox4x32_10(ctr, key, out);
}

/* ---- elementary functions of the specification (DESIGN.md "Math"): the same polynomials the HIP
 * code evaluates, so host and device agree to the bit. ------------------------------------------- */

/* exp(x) for x <= 0: Cody-Waite reduction by ln2, degree-13 Taylor on |r| <= ln2/2, ldexp. */
double np8o_exp_le0(double x) {
    x = fmax(x, -800.0);
    const double k = rint(x * 1.4426950408889634);
    double r = fma(-k, 0.6931471803691238, x);
    r = fma(-k, 1.9082149292705877e-10, r);
    static const double C[14] = {1.6059043836821613e-10, 2.08767569878681e-09, 2.505210838544172e-08,
                                 2.755731922398589e-07,  2.7557319223985893e-06, 2.48015873015873e-05,
                                 0.0001984126984126984,  0.001388888888888889,  0.008333333333333333,
                                 0.041666666666666664,   0.16666666666666666,   0.5,
                                 1.0,                    1.0};
    double p = C[0];
    for (int n = 1; n < 14; ++n) p = fma(p, r, C[n]);
    return ldexp(p, (int)k);
}

/* log(u), u > 0 normal: log1p(m-1) = 2 atanh((m-1)/(m+1)) with m in [1/sqrt2, sqrt2). */
double np8o_log_pos(double u) {
    int e;
    double m = frexp(u, &e);
    const int lo = m < 0.70710678118654757;
    m = lo ? m + m : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0;
    const double s = f * recip_logden(2.0 + f);
    const double s2 = s * s;
    static const double A[10] = {0.09523809523809523, 0.10526315789473684, 0.11764705882352941, 0.13333333333333333,
                                 0.15384615384615385, 0.18181818181818182, 0.2222222222222222,  0.2857142857142857,
                                 0.4,                 0.6666666666666666};
    double p = A[0];
    for (int n = 1; n < 10; ++n) p = fma(p, s2, A[n]);
    const double l1 = fma(s * s2, p, s + s);
    const double de = (double)e;
    return fma(de, 0.6931471803691238, fma(de, 1.9082149292705877e-10, l1));
}

/* (sin 2 pi t, cos 2 pi t), t in [0,1]: exact reduction to f in [-1/8,1/8] and Taylor polynomials. */
void np8o_sincos_2pi(double t, double *sn, double *cs) {
    const double q = rint(4.0 * t);
    const double f = t - 0.25 * q;
    const double f2 = f * f;
    static const double S[9] = {0.10422916220813984, -0.7181223017785006, 3.819952584848282,
                                -15.09464257682299,  42.058693944897655,  -76.70585975306139,
                                81.60524927607506,   -41.34170224039976,  6.283185307179586};
    static const double Cc[10] = {-0.03638284114254567, 0.28200596845579123, -1.714390711088672,
                                  7.903536371318469,    -26.4262567833744,   60.24464137187666,
                                  -85.45681720669373,   64.9393940226683,    -19.739208802178716,
                                  1.0};
    double ps = S[0];
    for (int n = 1; n < 9; ++n) ps = fma(ps, f2, S[n]);
    const double s0 = ps * f;
    double pc = Cc[0];
    for (int n = 1; n < 10; ++n) pc = fma(pc, f2, Cc[n]);
    const double c0 = pc;
    const int qi = ((int)q) & 3;
    const double a = (qi & 1) ? c0 : s0;
    const double b = (qi & 1) ? s0 : c0;
    *sn = (qi & 2) ? -a : a;
    *cs = ((qi + 1) & 2) ? -b : b;
}

/* Four normals from one Philox call: two Box-Muller pairs over 32-bit uniforms (words 0,1 and 2,3),
 * (r cos 2 pi u2, r sin 2 pi u2), r = sqrt(-2 log u1).  A draw of n normals uses calls
 * base .. base + ceil(n/4) - 1; normal k is g[k & 3] of call k >> 2. */
static void normal_quad(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call, double g[4]) {
    uint32_t o[4];
    philox_call(seed, i, t, stream, call, o);
    for (int h = 0; h < 2; ++h) {
        const double r = sqrt(-2.0 * np8o_log_pos(u32_01(o[2 * h])));
        double sn, cs;
        np8o_sincos_2pi(u32_01(o[2 * h + 1]), &sn, &cs);
        g[2 * h] = r * cs;
        g[2 * h + 1] = r * sn;
    }
}

/* Philox calls per G0 draw (D+1 normals). */
static inline int g0_calls(int D) { return (D + 4) / 4; }

double np8o_normal(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t n) {
    double g[4];
    normal_quad(seed, i, t, stream, n >> 2, g);
    return g[n & 3];
}

double np8o_uniform(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t n) {
    uint32_t o[4];
    philox_call(seed, i, t, stream, n, o);
    return np8o_u01(o[0], o[1]);
}

static inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

uint32_t np8o_substep_of(uint64_t seed, int64_t i, uint32_t S) {
    if (S <= 1) return 0;
    const uint32_t h = fmix32(fmix32((uint32_t)i ^ 0x5EB57E95u ^ (uint32_t)(seed >> 32)) ^ (uint32_t)seed);
    return (uint32_t)(((uint64_t)h * S) >> 32);
}

/* Scan order of a chunked sweep (replaces dim1algebra.hpp:2066-2073 random_order): a keyed 4-round
 * Feistel bijection on [0,2^b), cycle-walked into [0,N). */
uint32_t np8o_perm(uint64_t seed, uint32_t t, uint32_t N, uint32_t p) {
    if (N <= 1) return 0;
    int b = 0;
    while ((1ull << b) < (uint64_t)N) ++b;
    if (b < 2) b = 2;
    if (b & 1) ++b;
    const int h = b / 2;
    const uint32_t mask = (h >= 32) ? 0xFFFFFFFFu : ((1u << h) - 1u);
    uint32_t k[4];
    for (int r = 0; r < 4; ++r)
        k[r] = fmix32((uint32_t)seed ^ fmix32(t * 4u + (uint32_t)r + 0x9E3779B9u)) ^ (uint32_t)(seed >> 32);
    uint32_t x = p;
    do {
        uint32_t L = x >> h, R = x & mask;
        for (int r = 0; r < 4; ++r) {
            uint32_t nl = R;
            R = L ^ (fmix32(R ^ k[r]) & mask);
            L = nl;
        }
        x = (L << h) | R;
    } while (x >= N);
    return x;
}

/* ================================================================================================
 * Faithful reference restatements
 * ============================================================================================== */

/* LU with partial pivoting, row-major; Eigen's PartialPivLU is what MatrixXd::inverse() and
 * ::determinant() use for dynamic sizes (multivariatenormal.cpp:87,90). */
int np8o_lu_inverse_det(const double *A, int D, double *inv, double *det) {
    double LU[NP8O_DMAX * NP8O_DMAX];
    int perm[NP8O_DMAX];
    int sign = 1;
    memcpy(LU, A, sizeof(double) * D * D);
    for (int i = 0; i < D; ++i) perm[i] = i;
    for (int k = 0; k < D; ++k) {
        int p = k;
        double best = fabs(LU[k * D + k]);
        for (int i = k + 1; i < D; ++i)
            if (fabs(LU[i * D + k]) > best) {
                best = fabs(LU[i * D + k]);
                p = i;
            }
        if (best == 0.0) {
            if (det) *det = 0.0;
            return -1;
        }
        if (p != k) {
            for (int j = 0; j < D; ++j) {
                double tmp = LU[k * D + j];
                LU[k * D + j] = LU[p * D + j];
                LU[p * D + j] = tmp;
            }
            int tp = perm[k];
            perm[k] = perm[p];
            perm[p] = tp;
            sign = -sign;
        }
        for (int i = k + 1; i < D; ++i) {
            double f = LU[i * D + k] / LU[k * D + k];
            LU[i * D + k] = f;
            for (int j = k + 1; j < D; ++j) LU[i * D + j] = LU[i * D + j] - f * LU[k * D + j];
        }
    }
    if (det) {
        double d = (double)sign;
        for (int k = 0; k < D; ++k) d *= LU[k * D + k];
        *det = d;
    }
    if (inv) {
        /* Solve LU X = P I column by column. */
        for (int c = 0; c < D; ++c) {
            double y[NP8O_DMAX];
            for (int i = 0; i < D; ++i) {
                double s = (perm[i] == c) ? 1.0 : 0.0;
                for (int j = 0; j < i; ++j) s -= LU[i * D + j] * y[j];
                y[i] = s;
            }
            for (int i = D - 1; i >= 0; --i) {
                double s = y[i];
                for (int j = i + 1; j < D; ++j) s -= LU[i * D + j] * y[j];
                y[i] = s / LU[i * D + i];
            }
            for (int i = 0; i < D; ++i) inv[i * D + c] = y[i];
        }
    }
    return 0;
}

/* exponent = -0.5 * diff' * inverse * diff, evaluated left to right like Eigen's product chain. */
static double ref_exponent(const double *x, const double *mu, const double *inv, int D) {
    double d[NP8O_DMAX], r[NP8O_DMAX];
    for (int a = 0; a < D; ++a) d[a] = x[a] - mu[a];
    for (int b = 0; b < D; ++b) {
        double s = 0.0;
        for (int a = 0; a < D; ++a) s += (-0.5 * d[a]) * inv[a * D + b];
        r[b] = s;
    }
    double e = 0.0;
    for (int b = 0; b < D; ++b) e += r[b] * d[b];
    return e;
}

/* src/statistics/multivariatenormal.cpp:82-93 */
double np8o_mvn_probability_ref(const double *x, const double *mu, const double *Sigma, int D) {
    double inv[NP8O_DMAX * NP8O_DMAX], det;
    np8o_lu_inverse_det(Sigma, D, inv, &det);
    double exponent = ref_exponent(x, mu, inv, D);
    double constant = sqrt(pow(TWO_PI, D) * det);
    return exp(exponent) / constant;
}

/* src/statistics/multivariatenormal.cpp:124-135 */
double np8o_mvn_logprobability_ref(const double *x, const double *mu, const double *Sigma, int D) {
    double inv[NP8O_DMAX * NP8O_DMAX], det;
    np8o_lu_inverse_det(Sigma, D, inv, &det);
    double exponent = ref_exponent(x, mu, inv, D);
    double constant = sqrt(pow(TWO_PI, D) * det);
    return exponent - log(constant);
}

/* include/helper/dim1algebra.hpp:2078-2104: partial_sum, u*cumsum.back(), lower_bound. */
int64_t np8o_weighted_pick_ref(const double *w, int64_t n, double u) {
    if (n <= 0) return 0;
    double *cs = (double *)malloc(sizeof(double) * n);
    double acc = 0.0;
    for (int64_t j = 0; j < n; ++j) {
        acc += w[j];
        cs[j] = acc;
    }
    double target = u * cs[n - 1];
    int64_t lo = 0, len = n; /* std::lower_bound: first element not less than target */
    while (len > 0) {
        int64_t half = len / 2;
        if (cs[lo + half] < target) {
            lo += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    free(cs);
    return lo;
}

/* src/clustering_performance.cpp:14-82, with a,b,c,N in int64 (the reference's int overflows past
 * a few hundred points).  Degenerate ARI (reference returns early) -> NaN. */
void np8o_similarity(const int32_t *truth, const int32_t *result, int64_t n, double out[3]) {
    out[0] = out[1] = out[2] = NAN;
    if (n <= 0) return;
    int32_t ga = 0, gb = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (truth[i] > ga) ga = truth[i];
        if (result[i] > gb) gb = result[i];
    }
    int64_t A = (int64_t)ga + 1, B = (int64_t)gb + 1;
    int64_t *F = (int64_t *)calloc((size_t)(A * B), sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) F[(int64_t)truth[i] * B + result[i]] += 1;
    int64_t N = n;
    int64_t purity_sum = 0;
    for (int64_t c = 0; c < B; ++c) {
        int64_t m = 0;
        for (int64_t r = 0; r < A; ++r)
            if (F[r * B + c] > m) m = F[r * B + c];
        purity_sum += m;
    }
    out[0] = (double)purity_sum / (double)N;
    int64_t a = 0, b = 0, c = 0;
    for (int64_t r = 0; r < A; ++r) {
        int64_t rs = 0;
        for (int64_t cc = 0; cc < B; ++cc) {
            int64_t f = F[r * B + cc];
            a += (f * f - f) / 2;
            rs += f;
        }
        b += (rs * rs - rs) / 2;
    }
    for (int64_t cc = 0; cc < B; ++cc) {
        int64_t cs = 0;
        for (int64_t r = 0; r < A; ++r) cs += F[r * B + cc];
        c += (cs * cs - cs) / 2;
    }
    free(F);
    double S = ((double)N * (double)N - (double)N) / 2.0;
    if (S == 0.0) return;
    out[1] = (double)(2 * a - b - c) / S + 1.0;
    double bc_S = (double)b * (double)c / S;
    double bpc_2 = (double)(b + c) / 2.0;
    if (bc_S == bpc_2) return;
    out[2] = ((double)a - bc_S) / (bpc_2 - bc_S);
}

/* ================================================================================================
 * The chain
 * ============================================================================================== */

struct np8o_ctx {
    np8o_config cfg;
    int D, M, DP, kcap;
    /* G0 precomputes (DESIGN.md "G0"): L = chol(Lambda) lower. */
    double LT[NP8O_DMAX * NP8O_DMAX];    /* L^T (upper), row-major */
    double UinvT[NP8O_DMAX * NP8O_DMAX]; /* (L^T)^{-1} (upper) */
    double Gp[NP8O_DMAX * NP8O_DMAX];    /* (L^T L)^{-1}, off-diagonals doubled (upper used) */
    double LTL[NP8O_DMAX * NP8O_DMAX];   /* L^T L */
    double caux, rsk, logam;
    /* NIW prior: U = chol(Psi0^{-1}) (lower) and its inverse; UinvT then holds U^T and caux the NIW
     * constant -D/2 log 2pi + sum log U_aa (DESIGN.md "Priors") */
    double U[NP8O_DMAX * NP8O_DMAX], Uinv[NP8O_DMAX * NP8O_DMAX];
    /* F32 contraction: per slot A = fp32(chol_upper(sym P)) [kcap][D][D] and muf = fp32(mu) [kcap][D] */
    float *wA, *wmu;
    unsigned char *wdirty; /* slot parameters changed since its factor was computed */
    /* data */
    int64_t N;
    double *X; /* N x D row-major */
    int32_t *z;
    /* slots */
    double *slot_mu, *slot_P, *slot_c, *slot_sigma;
    int32_t *cnt;
    /* dense candidate table (ascending slot order) */
    int32_t K;
    int32_t *live, *dense_of;
    double *logn, *logn1, *iso;
    uint32_t t;
    /* max likelihood (np_mcmc.cpp:187-203) */
    double best_L;
    int have_best;
    int32_t *z_best, *cnt_best;
    double *mu_best, *sigma_best;
    /* scratch for the sequential driver */
    int32_t *delta;
    int64_t *rq_pos, *rq_i;
    int32_t *rq_m, *rq_zold;
    int64_t mh_accepted;
    int64_t n_new, n_deferred; /* accepted / not accepted new-cluster requests (cumulative) */
    int32_t req_max;
    /* per-item visits within the epoch (np8o_update_points): tag = epoch + 1, count */
    uint32_t *vis_tag, *vis_n;
    int64_t *sub_items, *sub_start; /* items of each data-parallel sub-step (ascending), CSR */
    /* split-merge (np8o_sm_sweep): member lists, per-member scratch, outcome counts */
    int64_t *sm_off, *sm_cur, *sm_mem;
    double *sm_v0, *sm_v1;
    unsigned char *sm_flag;
    int64_t sm_stats[6];
    double sm_log_alpha;
    int32_t *tri_asg; /* triadic: target of every member of the sources */
    int64_t tri_stats[10];
};

static int packed_index(int D, int a, int b) { /* upper triangle, row-major, a <= b */
    return a * D - (a * (a - 1)) / 2 + (b - a);
}

/* Host-side precomputes (the library's host code runs the same loops): Cholesky (lower) and the
 * inverse of a lower-triangular matrix. */
static int chol_lower(const double *A, int D, double *L) {
    memset(L, 0, sizeof(double) * D * D);
    for (int j = 0; j < D; ++j) {
        double s = A[j * D + j];
        for (int k = 0; k < j; ++k) s -= L[j * D + k] * L[j * D + k];
        if (!(s > 0.0)) return -1;
        L[j * D + j] = sqrt(s);
        for (int i = j + 1; i < D; ++i) {
            double v = A[i * D + j];
            for (int k = 0; k < j; ++k) v -= L[i * D + k] * L[j * D + k];
            L[i * D + j] = v / L[j * D + j];
        }
    }
    return 0;
}

static void inv_lower(const double *L, int D, double *Li) {
    memset(Li, 0, sizeof(double) * D * D);
    for (int j = 0; j < D; ++j) {
        Li[j * D + j] = 1.0 / L[j * D + j];
        for (int r = j + 1; r < D; ++r) {
            double s = 0.0;
            for (int k = j; k < r; ++k) s -= L[r * D + k] * Li[k * D + j];
            Li[r * D + j] = s / L[r * D + r];
        }
    }
}

/* NIW prior: U = chol(Psi0^{-1}) with Psi0^{-1} = Lp^{-T} Lp^{-1}, Lp = chol(Psi0). */
static int niw_prepare(np8o_ctx *c) {
    const int D = c->D;
    static double Lp[NP8O_DMAX * NP8O_DMAX], Li[NP8O_DMAX * NP8O_DMAX], Pi[NP8O_DMAX * NP8O_DMAX];
    if (chol_lower(c->cfg.Lambda, D, Lp) != 0) return -1;
    inv_lower(Lp, D, Li);
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) {
            double s = 0.0;
            for (int k = (a > b ? a : b); k < D; ++k) s += Li[k * D + a] * Li[k * D + b];
            Pi[a * D + b] = s;
        }
    if (chol_lower(Pi, D, c->U) != 0) return -1;
    inv_lower(c->U, D, c->Uinv);
    double sl = 0.0;
    for (int a = 0; a < D; ++a) sl += log(c->U[a * D + a]);
    c->caux = -0.5 * (double)D * LOG2PI + sl;
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) c->UinvT[a * D + b] = c->U[b * D + a];
    return 0;
}

np8o_ctx *np8o_create(const np8o_config *cfg) {
    if (cfg->D < 1 || cfg->D > NP8O_DMAX || cfg->M < 1 || cfg->M > NP8O_MMAX || cfg->kcap < 1) return NULL;
    if (cfg->pick != NP8O_PICK_RESERVOIR && (cfg->pick != NP8O_PICK_INVCDF || cfg->kcap > NP8O_KCAP_PICK)) return NULL;
    if (cfg->substeps < 0 || cfg->substeps > 64) return NULL;
    if (cfg->param_update < NP8O_PARAM_FROZEN || cfg->param_update > NP8O_PARAM_NIW_CONJUGATE || cfg->mh_steps < 0)
        return NULL;
    if (cfg->prior != NP8O_PRIOR_REFERENCE && cfg->prior != NP8O_PRIOR_NIW) return NULL;
    /* mh_g0 proposes from the reference's G0; the conjugate update needs the NIW prior; Bartlett's
     * chi^2(nu0 - a), a < D, need nu0 >= D + 1 for Marsaglia-Tsang's shape >= 1 */
    if ((cfg->prior == NP8O_PRIOR_NIW) != (cfg->param_update == NP8O_PARAM_NIW_CONJUGATE) &&
        !(cfg->prior == NP8O_PRIOR_NIW && cfg->param_update == NP8O_PARAM_FROZEN))
        return NULL;
    if (cfg->prior == NP8O_PRIOR_NIW && !(cfg->nu >= cfg->D + 1.0 && cfg->nu < 1e12)) return NULL;
    if (cfg->contraction != NP8O_CONTRACT_F64 &&
        !(cfg->contraction == NP8O_CONTRACT_F32 && cfg->D > 16 && cfg->D <= 80 &&
          cfg->param_update != NP8O_PARAM_MH_G0))
        return NULL;
    if (cfg->req_max < 0 || cfg->req_max > NP8O_REQMAX) return NULL;
    np8o_ctx *c = (np8o_ctx *)calloc(1, sizeof(np8o_ctx));
    c->cfg = *cfg;
    c->req_max = cfg->req_max > 0 ? cfg->req_max : NP8O_REQ_DEFAULT;
    const int D = cfg->D;
    c->D = D;
    c->M = cfg->M;
    c->DP = D * (D + 1) / 2;
    c->kcap = cfg->kcap;
    /* Cholesky of Lambda (invwishart.h:40 uses Lambda.llt().matrixL()). */
    double L[NP8O_DMAX * NP8O_DMAX];
    memset(L, 0, sizeof(L));
    for (int j = 0; j < D; ++j) {
        double s = cfg->Lambda[j * D + j];
        for (int k = 0; k < j; ++k) s -= L[j * D + k] * L[j * D + k];
        if (!(s > 0.0)) {
            free(c);
            return NULL;
        }
        L[j * D + j] = sqrt(s);
        for (int i = j + 1; i < D; ++i) {
            double v = cfg->Lambda[i * D + j];
            for (int k = 0; k < j; ++k) v -= L[i * D + k] * L[j * D + k];
            L[i * D + j] = v / L[j * D + j];
        }
    }
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) c->LT[a * D + b] = L[b * D + a];
    /* (L^T)^{-1}: invert the upper-triangular L^T by back substitution. */
    memset(c->UinvT, 0, sizeof(c->UinvT));
    for (int col = 0; col < D; ++col)
        for (int i = col; i >= 0; --i) {
            double s = (i == col) ? 1.0 : 0.0;
            for (int j = i + 1; j <= col; ++j) s -= c->LT[i * D + j] * c->UinvT[j * D + col];
            c->UinvT[i * D + col] = s / c->LT[i * D + i];
        }
    /* L^T L and its inverse (L^T L)^{-1} = UinvT * UinvT^T. */
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) {
            double s = 0.0, g = 0.0;
            for (int k = 0; k < D; ++k) {
                s += L[k * D + a] * L[k * D + b];
                g += c->UinvT[a * D + k] * c->UinvT[b * D + k];
            }
            c->LTL[a * D + b] = s;
            c->Gp[a * D + b] = (a == b) ? g : 2.0 * g;
        }
    double sumlog = 0.0;
    for (int a = 0; a < D; ++a) sumlog += log(L[a * D + a]);
    c->caux = -0.5 * (double)D * LOG2PI - sumlog;
    c->rsk = 1.0 / sqrt(cfg->kappa);
    c->logam = log(cfg->alpha / (double)cfg->M);
    if (cfg->prior == NP8O_PRIOR_NIW && niw_prepare(c) != 0) {
        free(c);
        return NULL;
    }
    const int K = c->kcap;
    c->slot_mu = (double *)calloc((size_t)K * D, sizeof(double));
    c->slot_P = (double *)calloc((size_t)K * c->DP, sizeof(double));
    c->slot_c = (double *)calloc((size_t)K, sizeof(double));
    c->slot_sigma = (double *)calloc((size_t)K * D * D, sizeof(double));
    c->cnt = (int32_t *)calloc((size_t)K, sizeof(int32_t));
    c->live = (int32_t *)calloc((size_t)K, sizeof(int32_t));
    c->logn = (double *)calloc((size_t)K, sizeof(double));
    c->logn1 = (double *)calloc((size_t)K, sizeof(double));
    c->iso = (double *)calloc((size_t)K, sizeof(double));
    c->dense_of = (int32_t *)calloc((size_t)K, sizeof(int32_t));
    c->cnt_best = (int32_t *)calloc((size_t)K, sizeof(int32_t));
    c->mu_best = (double *)calloc((size_t)K * D, sizeof(double));
    c->sigma_best = (double *)calloc((size_t)K * D * D, sizeof(double));
    c->delta = (int32_t *)calloc((size_t)K, sizeof(int32_t));
    c->sm_off = (int64_t *)calloc((size_t)K + 1, sizeof(int64_t));
    c->sm_cur = (int64_t *)calloc((size_t)K, sizeof(int64_t));
    c->sm_log_alpha = log(cfg->alpha);
    if (cfg->contraction == NP8O_CONTRACT_F32) {
        c->wA = (float *)calloc((size_t)K * D * D, sizeof(float));
        c->wmu = (float *)calloc((size_t)K * D, sizeof(float));
        c->wdirty = (unsigned char *)calloc((size_t)K, 1);
    }
    c->best_L = -INFINITY;
    return c;
}

void np8o_destroy(np8o_ctx *c) {
    if (!c) return;
    free(c->X);
    free(c->z);
    free(c->z_best);
    free(c->slot_mu);
    free(c->slot_P);
    free(c->slot_c);
    free(c->slot_sigma);
    free(c->cnt);
    free(c->live);
    free(c->logn);
    free(c->logn1);
    free(c->iso);
    free(c->dense_of);
    free(c->cnt_best);
    free(c->mu_best);
    free(c->sigma_best);
    free(c->delta);
    free(c->wA);
    free(c->wmu);
    free(c->wdirty);
    free(c->rq_pos);
    free(c->rq_i);
    free(c->rq_m);
    free(c->rq_zold);
    free(c->sm_off);
    free(c->sm_cur);
    free(c->sm_mem);
    free(c->sm_v0);
    free(c->sm_v1);
    free(c->sm_flag);
    free(c->tri_asg);
    free(c->sub_items);
    free(c->sub_start);
    free(c->vis_tag);
    free(c->vis_n);
    free(c);
}

int np8o_set_data(np8o_ctx *c, const double *X, int64_t N) {
    free(c->X);
    free(c->z);
    free(c->z_best);
    free(c->rq_pos);
    free(c->rq_i);
    free(c->rq_m);
    free(c->rq_zold);
    free(c->sm_mem);
    free(c->sm_v0);
    free(c->sm_v1);
    free(c->sm_flag);
    free(c->tri_asg);
    free(c->vis_tag);
    free(c->vis_n);
    free(c->sub_items);
    free(c->sub_start);
    {
        const uint32_t S = c->cfg.substeps > 1 ? (uint32_t)c->cfg.substeps : 1u;
        c->sub_items = (int64_t *)malloc(sizeof(int64_t) * (size_t)(N > 0 ? N : 1));
        c->sub_start = (int64_t *)calloc(S + 1, sizeof(int64_t));
        for (int64_t i = 0; i < N; ++i) c->sub_start[np8o_substep_of(c->cfg.seed, i, S) + 1] += 1;
        for (uint32_t k = 0; k < S; ++k) c->sub_start[k + 1] += c->sub_start[k];
        int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * S);
        for (uint32_t k = 0; k < S; ++k) fill[k] = c->sub_start[k];
        for (int64_t i = 0; i < N; ++i) c->sub_items[fill[np8o_substep_of(c->cfg.seed, i, S)]++] = i;
        free(fill);
    }
    c->vis_tag = (uint32_t *)calloc((size_t)(N > 0 ? N : 1), sizeof(uint32_t));
    c->vis_n = (uint32_t *)calloc((size_t)(N > 0 ? N : 1), sizeof(uint32_t));
    c->N = N;
    c->X = (double *)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1) * c->D);
    if (N > 0) memcpy(c->X, X, sizeof(double) * (size_t)N * c->D);
    if (c->cfg.contraction == NP8O_CONTRACT_F32) /* the items as the device holds them */
        for (int64_t k = 0; k < N * c->D; ++k) c->X[k] = (double)(float)c->X[k];
    c->z = (int32_t *)calloc((size_t)(N > 0 ? N : 1), sizeof(int32_t));
    c->z_best = (int32_t *)calloc((size_t)(N > 0 ? N : 1), sizeof(int32_t));
    c->rq_pos = (int64_t *)malloc(sizeof(int64_t) * (size_t)(N > 0 ? N : 1));
    c->rq_i = (int64_t *)malloc(sizeof(int64_t) * (size_t)(N > 0 ? N : 1));
    c->rq_m = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    c->rq_zold = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    c->sm_mem = (int64_t *)malloc(sizeof(int64_t) * (size_t)(N > 0 ? N : 1));
    c->sm_v0 = (double *)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
    c->sm_v1 = (double *)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
    c->sm_flag = (unsigned char *)malloc((size_t)(N > 0 ? N : 1));
    c->tri_asg = (int32_t *)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    return 0;
}

/* Table entry from an explicit covariance: P' = sym(LU-inverse) with doubled off-diagonals,
 * c = -0.5 (D log 2pi + log det). */
static int slot_from_sigma(np8o_ctx *c, int s, const double *mu, const double *Sigma) {
    const int D = c->D;
    double inv[NP8O_DMAX * NP8O_DMAX], det;
    if (np8o_lu_inverse_det(Sigma, D, inv, &det) != 0 || !(det > 0.0)) return -2;
    memcpy(c->slot_mu + (size_t)s * D, mu, sizeof(double) * D);
    memcpy(c->slot_sigma + (size_t)s * D * D, Sigma, sizeof(double) * D * D);
    double *P = c->slot_P + (size_t)s * c->DP;
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b)
            P[packed_index(D, a, b)] = (a == b) ? inv[a * D + a] : inv[a * D + b] + inv[b * D + a];
    c->slot_c[s] = -0.5 * ((double)D * LOG2PI + log(det));
    if (c->wdirty) c->wdirty[s] = 1;
    return 0;
}

/* G0 draw from scale normal g0 and xi (normalinvwishart.h:44-64, invwishart.h:34-46):
 * v = D + nu g0, Sigma = v^2 L^T L, mu = mu0 + (|v|/sqrt(kappa)) L^T xi. */
static void aux_from_normals(const np8o_ctx *c, double g0, const double *xi, double *v_out, double *mu) {
    const int D = c->D;
    double v = fma(c->cfg.nu, g0, (double)D);
    double s = fabs(v) * c->rsk;
    for (int a = 0; a < D; ++a) {
        double t = c->LT[a * D + a] * xi[a];
        for (int b = a + 1; b < D; ++b) t = fma(c->LT[a * D + b], xi[b], t);
        mu[a] = fma(s, t, c->cfg.mu0[a]);
    }
    *v_out = v;
}

static void slot_from_aux(np8o_ctx *c, int s, double v, const double *mu) {
    const int D = c->D;
    memcpy(c->slot_mu + (size_t)s * D, mu, sizeof(double) * D);
    double v2 = v * v;
    double *P = c->slot_P + (size_t)s * c->DP;
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) P[packed_index(D, a, b)] = c->Gp[a * D + b] / v2;
    c->slot_c[s] = fma(-(double)D, np8o_log_pos(fabs(v)), c->caux);
    if (c->wdirty) c->wdirty[s] = 1;
    double *S = c->slot_sigma + (size_t)s * D * D;
    for (int k = 0; k < D * D; ++k) S[k] = v2 * c->LTL[k];
}

/* ---- auxiliary draws in the item's frame (DESIGN.md "G0") ----------------------------------------
 * Auxiliary m of item i is theta = (v, mu0 + (|v|/sqrt kappa) L^T xi), xi ~ N(0, I_D).  With
 * y0 = (L^T)^{-1}(x - mu0) the likelihood needs only xi_par = xi . y0/|y0| ~ N(0,1) and
 * chi2 = |xi_perp|^2 ~ chi^2_{D-1}: |y0 - s xi|^2 = (|y0| - s xi_par)^2 + s^2 chi2.  Calls m*Qa .. of
 * stream AUX: call 0 words (0,1) -> Box-Muller (v-normal, xi_par) = (r cos, r sin), words 2,3 -> the
 * first two of the k = (D-1)/2 uniforms whose product gives chi^2_{2k} = -2 log(prod); call 1 (odd D-1
 * or k > 2): words (0,1) -> g_odd = r cos (chi2 += g_odd^2 for odd D-1), words 2,3 -> uniforms 2,3;
 * call 2+c: uniforms 4+4c .. 7+4c; logs over products of at most 16 uniforms.  Call 0 alone bounds the
 * log-likelihood from above (the device screens far auxiliaries with it; results unchanged).  A picked
 * auxiliary's xi = xi_par yhat + sqrt(chi2) w_perp/|w_perp|, w ~ N(0,I) on stream AUX_DIR. */
static inline int aux_calls(int D) {
    const int k = (D - 1) / 2;
    return 1 + ((((D - 1) & 1) || k > 2) ? 1 : 0) + (k > 4 ? (k - 1) / 4 : 0);
}
static inline int dir_calls(int D) { return (D + 3) / 4; }

/* The screen prefixes (round 6; noparama_amd/csrc/np8_device.h aux_pre_bits, DESIGN.md "Auxiliary screen"), D <= 8: call 0
 * of stream AUX_PRE (i = item key) holds the leading b bits of the first P = min(k, 3) chi^2 uniforms of every
 * auxiliary, b = min(16, floor(128 / (M P))); field f = m P + j is bits [b f, b f + b) of the call's four words
 * (word 0 = bits 0..31).  Chi^2 uniform j < P of auxiliary m takes the word (field << (32 - b)) | (its own word &
 * (2^(32 - b) - 1)).  (A restatement of the specification; the reference draws from an unseeded engine, so only
 * the distribution is the reference's: uniform 32-bit words, independent of the rest.) */
#define NP8O_PRE_MAX_D 8 /* prefixes for D <= 8 only (the device's kPreMaxD) */
static inline int aux_pre_n(int D) {
    const int k = (D - 1) / 2;
    return D > NP8O_PRE_MAX_D ? 0 : (k < 3 ? k : 3);
}
static inline int aux_pre_bits(int D, int M) {
    const int P = aux_pre_n(D);
    if (P <= 0 || M <= 0) return 0;
    const int b = 128 / (M * P);
    return b > 16 ? 16 : b;
}
static uint32_t aux_chi_word(const uint32_t pre[4], uint32_t w, int m, int j, int D, int M) {
    const int P = aux_pre_n(D), b = aux_pre_bits(D, M);
    if (j >= P || b <= 0) return w;
    const int lo = b * (m * P + j), wi = lo >> 5, sh = lo & 31;
    const uint64_t v = (((uint64_t)(wi < 3 ? pre[wi + 1] : 0u)) << 32 | pre[wi]) >> sh;
    const uint32_t field = (uint32_t)v & ((1u << b) - 1u);
    return (field << (32 - b)) | (w & ((1u << (32 - b)) - 1u));
}

static void aux_core(const np8o_ctx *c, uint64_t i, uint32_t t, int m, double *v, double *xpar, double *chi2) {
    const int D = c->D, Qa = aux_calls(D), k = (D - 1) / 2, odd = (D - 1) & 1;
    const uint32_t base = (uint32_t)(m * Qa);
    uint32_t w[4], w1[4] = {0u, 0u, 0u, 0u}, wc[4] = {0u, 0u, 0u, 0u}, pre[4] = {0u, 0u, 0u, 0u};
    if (aux_pre_n(D) > 0) philox_call(c->cfg.seed, i, t, NP8O_STREAM_AUX_PRE, 0u, pre);
    philox_call(c->cfg.seed, i, t, NP8O_STREAM_AUX, base, w);
    {
        const double r = sqrt(-2.0 * np8o_log_pos(u32_01(w[0])));
        double sn, cs;
        np8o_sincos_2pi(u32_01(w[1]), &sn, &cs);
        *v = fma(c->cfg.nu, r * cs, (double)D);
        *xpar = r * sn;
    }
    double godd = 0.0;
    if (odd || k > 2) {
        philox_call(c->cfg.seed, i, t, NP8O_STREAM_AUX, base + 1u, w1);
        if (odd) {
            const double r = sqrt(-2.0 * np8o_log_pos(u32_01(w1[0])));
            double sn, cs;
            np8o_sincos_2pi(u32_01(w1[1]), &sn, &cs);
            godd = r * cs;
        }
    }
    double c2 = 0.0, prod = 1.0;
    int in_chunk = 0;
    for (int j = 0; j < k; ++j) {
        uint32_t word;
        if (j < 2) {
            word = aux_chi_word(pre, w[2 + j], m, j, D, c->M);
        } else if (j < 4) {
            word = aux_chi_word(pre, w1[j], m, j, D, c->M);
        } else {
            if (((j - 4) & 3) == 0)
                philox_call(c->cfg.seed, i, t, NP8O_STREAM_AUX, base + 2u + (uint32_t)((j - 4) >> 2), wc);
            word = wc[(j - 4) & 3];
        }
        prod *= u32_01(word);
        if (++in_chunk == 16 || j == k - 1) {
            c2 = fma(-2.0, np8o_log_pos(prod), c2);
            prod = 1.0;
            in_chunk = 0;
        }
    }
    if (odd) c2 = fma(godd, godd, c2);
    *chi2 = c2;
}

static double aux_loglik(const np8o_ctx *c, double ny, double v, double xpar, double chi2) {
    const double s = fabs(v) * c->rsk;
    const double d = fma(-s, xpar, ny);
    const double r2 = fma(d, d, (s * s) * chi2);
    const double q = r2 / (v * v);
    const double cm = fma(-(double)c->D, np8o_log_pos(fabs(v)), c->caux);
    return fma(-0.5, q, cm);
}

/* y0 = (L^T)^{-1}(x - mu0) and |y0|. */
static double whiten(const np8o_ctx *c, const double *x, double *y0) {
    const int D = c->D;
    double dx[NP8O_DMAX];
    for (int a = 0; a < D; ++a) dx[a] = x[a] - c->cfg.mu0[a];
    for (int a = 0; a < D; ++a) {
        double t0 = c->UinvT[a * D + a] * dx[a];
        for (int b = a + 1; b < D; ++b) t0 = fma(c->UinvT[a * D + b], dx[b], t0);
        y0[a] = t0;
    }
    double n2 = 0.0;
    for (int a = 0; a < D; ++a) n2 = fma(y0[a], y0[a], n2);
    return sqrt(n2);
}

static void aux_xi(const np8o_ctx *c, uint64_t i, uint32_t t, int m, const double *y0, double ny, double xpar,
                   double chi2, double *xi) {
    const int D = c->D, Qd = dir_calls(D);
    double yh[NP8O_DMAX], w[NP8O_DMAX], g[4] = {0.0, 0.0, 0.0, 0.0};
    for (int a = 0; a < D; ++a) yh[a] = (ny > 0.0) ? y0[a] / ny : (a == 0 ? 1.0 : 0.0);
    for (int a = 0; a < D; ++a) {
        if ((a & 3) == 0) normal_quad(c->cfg.seed, i, t, NP8O_STREAM_AUX_DIR, (uint32_t)(m * Qd + (a >> 2)), g);
        w[a] = g[a & 3];
    }
    double dot = 0.0;
    for (int a = 0; a < D; ++a) dot = fma(w[a], yh[a], dot);
    double n2 = 0.0;
    for (int a = 0; a < D; ++a) {
        w[a] = fma(-dot, yh[a], w[a]);
        n2 = fma(w[a], w[a], n2);
    }
    const double np = sqrt(n2);
    const double sc = (np > 0.0) ? sqrt(chi2) / np : 0.0;
    for (int a = 0; a < D; ++a) xi[a] = fma(xpar, yh[a], sc * w[a]);
}

/* The M auxiliary draws of item key i (data row NP8O_ITEM(i)) at epoch t: v[m], mu[m*D..]. */
static void aux_draws(const np8o_ctx *c, uint64_t i, uint32_t t, double *v, double *mu /* M*D */) {
    double y0[NP8O_DMAX];
    const double ny = whiten(c, c->X + (size_t)NP8O_ITEM(i) * c->D, y0);
    for (int m = 0; m < c->M; ++m) {
        double xpar, chi2, xi[NP8O_DMAX];
        aux_core(c, i, t, m, v + m, &xpar, &chi2);
        aux_xi(c, i, t, m, y0, ny, xpar, chi2, xi);
        const int D = c->D;
        const double s = fabs(v[m]) * c->rsk;
        for (int a = 0; a < D; ++a) {
            double t0 = c->LT[a * D + a] * xi[a];
            for (int b = a + 1; b < D; ++b) t0 = fma(c->LT[a * D + b], xi[b], t0);
            mu[(size_t)m * D + a] = fma(s, t0, c->cfg.mu0[a]);
        }
    }
}

/* ================================================================================================
 * NIW prior (DESIGN.md "Priors").  A proper Normal-Inverse-
 * Wishart G0 -- Sigma ~ IW(Psi0, nu0), mu | Sigma ~ N(mu0, Sigma/kappa0) -- replacing the reference's
 * scale-only draw, and its conjugate posterior (the update the reference stubs with assert(false),
 * include/statistics/normalinvwishart.h:66-75).  Sampling follows the reference's two-stage
 * operator() (normalinvwishart.h:44-64: Sigma from the inverse Wishart, then mu from N(mu, Sigma/kappa));
 * the inverse Wishart is drawn through Bartlett's decomposition of the Wishart precision.
 * ============================================================================================== */
#define NIW_AUX_CALLS 8192u   /* Philox calls reserved per auxiliary m on streams AUX_NIW / AUX_DIR */
#define NIW_GAMMA_CALLS 64u   /* calls reserved per chi^2 draw (two Marsaglia-Tsang attempts per call) */
#define NIW_NORMAL_CALL0 8192u /* posterior draws: first call of the Bartlett off-diagonal and z normals */

/* Marsaglia & Tsang (2000), Gamma(alpha, 1) for alpha >= 1: per Philox call one Box-Muller pair
 * (words 0, 1) gives two attempts x, with 32-bit uniforms words 2, 3; accept d v, v = (1 + c x)^3, when
 * u < 1 - 0.0331 x^4 or log u < x^2/2 + d (1 - v + log v).  4096 calls at most (never reached: each
 * attempt is accepted with probability > 0.95), so every lane of a kernel terminates. */
double np8o_gamma_mt(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call0, double alpha) {
    const double d = alpha - 1.0 / 3.0;
    const double cc = 1.0 / sqrt(9.0 * d);
    for (uint32_t r = 0; r < 4096u; ++r) {
        uint32_t o[4];
        philox_call(seed, i, t, stream, call0 + r, o);
        const double rad = sqrt(-2.0 * np8o_log_pos(u32_01(o[0])));
        double sn, cs;
        np8o_sincos_2pi(u32_01(o[1]), &sn, &cs);
        for (int h = 0; h < 2; ++h) {
            const double x = rad * (h ? sn : cs);
            const double v1 = fma(cc, x, 1.0);
            if (v1 <= 0.0) continue;
            const double v = v1 * v1 * v1;
            const double u = u32_01(o[2 + h]);
            const double x2 = x * x;
            if (u < fma(-0.0331, x2 * x2, 1.0)) return d * v;
            if (np8o_log_pos(u) < fma(0.5, x2, d * ((1.0 - v) + np8o_log_pos(v)))) return d * v;
        }
    }
    return d;
}

/* chi^2 with dof degrees of freedom (dof >= 2) = 2 Gamma(dof/2). */
static inline double chi2_mt(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call0, double dof) {
    return 2.0 * np8o_gamma_mt(seed, i, t, stream, call0, 0.5 * dof);
}

/* Normal number n of stream (i, t) counted from call c0 (normal_quad layout). */
static inline double normal_at(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t c0, uint32_t n) {
    double g[4];
    normal_quad(seed, i, t, stream, c0 + (n >> 2), g);
    return g[n & 3];
}

/* chi^2_{D-1} of |z_perp|^2: a sum of D-1 squared normals (one call) for D <= 4, else Marsaglia-Tsang
 * at call base + 64 D. */
static double niw_chi_perp(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t base, int D) {
    const int k = D - 1;
    if (k <= 0) return 0.0;
    if (k <= 3) {
        double g[4];
        normal_quad(seed, i, t, stream, base + NIW_AUX_CALLS - 2u, g);
        double s = g[0] * g[0];
        for (int j = 1; j < k; ++j) s = fma(g[j], g[j], s);
        return s;
    }
    return chi2_mt(seed, i, t, stream, base + NIW_GAMMA_CALLS * (uint32_t)D, (double)k);
}

/* Running sum of logs of products of at most 16 chi^2 draws (their product cannot overflow). */
typedef struct {
    double prod, sumlog;
} logacc;

static inline void logacc_add(logacc *a, double g, int idx, int last) {
    a->prod *= g;
    if ((idx & 15) == 15 || idx == last) {
        a->sumlog += np8o_log_pos(a->prod);
        a->prod = 1.0;
    }
}

/* ---- auxiliary draws in the item's frame ------------------------------------------------------
 * Sigma^{-1} = U Omega U^T with U U^T = Psi0^{-1} (U = chol(Psi0^{-1}), lower) and Omega ~ W(I, nu0);
 * mu = mu0 + eps, U^T... Write Omega = R B B^T R with B Bartlett-lower (B_aa^2 ~ chi^2(nu0 - a),
 * B_ab ~ N(0,1) below) and R the reflection taking e1 to -+ dt/|dt|, dt = U^T (x - mu0): rotation
 * invariance of W(I, nu0) makes this a G0 draw whatever R is.  With F = U R B, Sigma^{-1} = F F^T and
 * mu = mu0 + F^{-T} z'/sqrt(kappa0), z' ~ N(0, I):
 *   F^T (x - mu) = (s |dt| B_00 - s z'_0/sqrt(kappa0), -z'_rest/sqrt(kappa0))          (s = +-1)
 *   ll = -D/2 log 2pi + sum log U_aa + 1/2 sum_a log B_aa^2 - q/2,
 *   q  = (|dt| B_00 - z_1/sqrt(kappa0))^2 + chi^2_{D-1}/kappa0.
 * So the likelihood needs the D diagonal chi^2 draws, z_1 and chi^2_{D-1} = |z_rest|^2: auxiliary m
 * draws them on stream AUX_NIW, calls base = m NIW_AUX_CALLS: chi^2(nu0 - a) from base + 64 a,
 * chi^2_{D-1} from niw_chi_perp, z_1 = normal 0 of call base + NIW_AUX_CALLS - 1.  Only a picked
 * auxiliary is built in full (niw_aux_slot): B's off-diagonals (normal a(a-1)/2 + b) and the direction
 * w of z_rest (normals D(D-1)/2 + j) on stream AUX_DIR from call base. */
static void niw_aux_core(const np8o_ctx *c, uint64_t i, uint32_t t, int m, double *sumlog, double *b00, double *chi,
                         double *z1) {
    const int D = c->D;
    const uint64_t seed = c->cfg.seed;
    const uint32_t base = (uint32_t)m * NIW_AUX_CALLS;
    logacc la = {1.0, 0.0};
    *b00 = 0.0;
    for (int a = 0; a < D; ++a) {
        const double g = chi2_mt(seed, i, t, NP8O_STREAM_AUX_NIW, base + NIW_GAMMA_CALLS * (uint32_t)a, c->cfg.nu - a);
        if (a == 0) *b00 = sqrt(g);
        logacc_add(&la, g, a, D - 1);
    }
    *sumlog = la.sumlog;
    *chi = niw_chi_perp(seed, i, t, NP8O_STREAM_AUX_NIW, base, D);
    *z1 = normal_at(seed, i, t, NP8O_STREAM_AUX_NIW, base + NIW_AUX_CALLS - 1u, 0);
}

static double niw_aux_loglik(const np8o_ctx *c, double nd, double sumlog, double b00, double chi, double z1) {
    const double e = fma(-z1, c->rsk, nd * b00);
    const double q = fma(e, e, chi * (c->rsk * c->rsk));
    return fma(-0.5, q, fma(0.5, sumlog, c->caux));
}

static inline int packed_ix(int D, int a, int b) { return a * D - (a * (a - 1)) / 2 + (b - a); }

/* Outputs shared by the NIW draws: mu, packed P' = sym(Sigma^{-1}) (off-diagonals doubled), Sigma, c. */
static void niw_outputs_from_F(int D, const double *F, double *Ppk) {
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) {
            double s = 0.0;
            for (int k = 0; k < D; ++k) s = fma(F[a * D + k], F[b * D + k], s);
            Ppk[packed_ix(D, a, b)] = (a == b) ? s : 2.0 * s;
        }
}

/* Sigma = T^T T with T lower-solved from B T = Rhs (B lower triangular, Rhs full). */
static void niw_sigma(int D, const double *B, const double *Rhs, double *T, double *Sigma) {
    for (int j = 0; j < D; ++j)
        for (int a = 0; a < D; ++a) {
            double s = Rhs[a * D + j];
            for (int k = 0; k < a; ++k) s = fma(-B[a * D + k], T[k * D + j], s);
            T[a * D + j] = s / B[a * D + a];
        }
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) {
            double s = 0.0;
            for (int k = 0; k < D; ++k) s = fma(T[k * D + a], T[k * D + b], s);
            Sigma[a * D + b] = s;
        }
}

/* The full parameters of auxiliary m of item i (dt = U^T (x - mu0)), exactly the draw whose
 * likelihood niw_aux_core/niw_aux_loglik evaluated. */
static void niw_aux_slot(const np8o_ctx *c, uint64_t i, uint32_t t, int m, const double *dt, double *mu, double *Ppk,
                         double *Sigma, double *cc) {
    const int D = c->D;
    const uint64_t seed = c->cfg.seed;
    const uint32_t base = (uint32_t)m * NIW_AUX_CALLS;
    static _Thread_local double B[NP8O_DMAX * NP8O_DMAX], RB[NP8O_DMAX * NP8O_DMAX], F[NP8O_DMAX * NP8O_DMAX],
        T[NP8O_DMAX * NP8O_DMAX];
    memset(B, 0, sizeof(double) * D * D);
    logacc la = {1.0, 0.0};
    for (int a = 0; a < D; ++a) {
        const double g = chi2_mt(seed, i, t, NP8O_STREAM_AUX_NIW, base + NIW_GAMMA_CALLS * (uint32_t)a, c->cfg.nu - a);
        B[a * D + a] = sqrt(g);
        logacc_add(&la, g, a, D - 1);
    }
    const double chi = niw_chi_perp(seed, i, t, NP8O_STREAM_AUX_NIW, base, D);
    const double z1 = normal_at(seed, i, t, NP8O_STREAM_AUX_NIW, base + NIW_AUX_CALLS - 1u, 0);
    for (int a = 1; a < D; ++a)
        for (int b = 0; b < a; ++b)
            B[a * D + b] = normal_at(seed, i, t, NP8O_STREAM_AUX_DIR, base, (uint32_t)(a * (a - 1) / 2 + b));
    double z[NP8O_DMAX], w2 = 0.0;
    const uint32_t nw0 = (uint32_t)(D * (D - 1) / 2);
    for (int j = 0; j + 1 < D; ++j) {
        z[1 + j] = normal_at(seed, i, t, NP8O_STREAM_AUX_DIR, base, nw0 + (uint32_t)j);
        w2 = fma(z[1 + j], z[1 + j], w2);
    }
    const double sc = (w2 > 0.0) ? sqrt(chi / w2) : 0.0;
    for (int j = 1; j < D; ++j) z[j] *= sc;
    /* Householder reflection R = I - beta h h^T, R dt = sig |dt| e1 */
    double n2 = 0.0;
    for (int a = 0; a < D; ++a) n2 = fma(dt[a], dt[a], n2);
    const double nd = sqrt(n2);
    double h[NP8O_DMAX] = {0.0}, beta = 0.0, sig = 1.0;
    if (nd > 0.0) {
        for (int a = 0; a < D; ++a) h[a] = dt[a] / nd;
        const double sg = (h[0] >= 0.0) ? 1.0 : -1.0;
        h[0] = h[0] + sg;
        double hh = 0.0;
        for (int a = 0; a < D; ++a) hh = fma(h[a], h[a], hh);
        beta = 2.0 / hh;
        sig = -sg;
    }
    z[0] = sig * z1;
    /* RB = B - beta h (h^T B);  F = U RB */
    for (int b = 0; b < D; ++b) {
        double cs = 0.0;
        for (int k = b; k < D; ++k) cs = fma(h[k], B[k * D + b], cs);
        for (int a = 0; a < D; ++a) RB[a * D + b] = fma(-(beta * h[a]), cs, B[a * D + b]);
    }
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) {
            double s = 0.0;
            for (int k = 0; k <= a; ++k) s = fma(c->U[a * D + k], RB[k * D + b], s);
            F[a * D + b] = s;
        }
    niw_outputs_from_F(D, F, Ppk);
    /* mu = mu0 + U^{-T} R B^{-T} z rsk */
    double y[NP8O_DMAX], ry[NP8O_DMAX], eps[NP8O_DMAX];
    for (int a = D - 1; a >= 0; --a) {
        double s = z[a] * c->rsk;
        for (int k = a + 1; k < D; ++k) s = fma(-B[k * D + a], y[k], s);
        y[a] = s / B[a * D + a];
    }
    double hy = 0.0;
    for (int k = 0; k < D; ++k) hy = fma(h[k], y[k], hy);
    for (int a = 0; a < D; ++a) ry[a] = fma(-(beta * h[a]), hy, y[a]);
    for (int a = D - 1; a >= 0; --a) {
        double s = ry[a];
        for (int k = a + 1; k < D; ++k) s = fma(-c->U[k * D + a], eps[k], s);
        eps[a] = s / c->U[a * D + a];
    }
    for (int a = 0; a < D; ++a) mu[a] = c->cfg.mu0[a] + eps[a];
    /* Sigma = T^T T, T = F^{-1} = B^{-1} (R U^{-1}) */
    for (int b = 0; b < D; ++b) {
        double cs = 0.0;
        for (int k = b; k < D; ++k) cs = fma(h[k], c->Uinv[k * D + b], cs);
        for (int a = 0; a < D; ++a) RB[a * D + b] = fma(-(beta * h[a]), cs, c->Uinv[a * D + b]);
    }
    niw_sigma(D, B, RB, T, Sigma);
    *cc = fma(0.5, la.sumlog, c->caux);
}

/* NIW(mu0, kappa0, nu0, Psi0) posterior of n items with statistics s1 = sum d, S = sum d d^T (packed
 * upper) about the anchor a (d = x - a), then a draw (Sigma, mu) from it (n = 0: the prior):
 *   kn = kappa0 + n, nun = nu0 + n, xb = a + s1/n, mun = (kappa0 mu0 + n xb)/kn,
 *   Psin = Psi0 + (S - s1 s1^T/n) + (kappa0 n/kn)(xb - mu0)(xb - mu0)^T;
 *   Psin = U U^T with U upper triangular: Lr = chol(J Psin J) (J the index reversal), U = J Lr J;
 *   R = B^T U^{-1} (upper; B Bartlett-lower with nun): Sigma^{-1} = R^T R = G B B^T G^T with G = U^{-T},
 *   G G^T = Psin^{-1}, so Sigma ~ IW(Psin, nun) -- and R, upper with a positive diagonal, IS the Cholesky
 *   factor of Sigma^{-1} that the fp32 contraction uses (no factorization of P afterwards);
 *   mu = mun + U B^{-T} z / sqrt(kn) (= mun + R^{-1} z / sqrt(kn)) ~ N(mun, Sigma/kn);
 *   Sigma = T^T T with T = B^{-1} U^T (lower);  c = -D/2 log 2pi - sum log U_aa + 1/2 sum log B_aa^2.
 * Every output element is one k-ascending fma chain from 0 (the device's order, np8_niw.hip np8_niw_post).
 * Draws of (i, t, stream): chi^2(nun - a) from call 64 a, then normals from call NIW_NORMAL_CALL0:
 * B_ab (a > b) is normal a(a-1)/2 + b, z_j is normal D(D-1)/2 + j.  Returns -1 (nothing written) if
 * Psin is not numerically positive definite.  Rout (D x D row-major, or NULL): R. */
static int niw_draw_impl(const np8o_ctx *c, uint64_t i, uint32_t t, uint32_t stream, int64_t n, const double *s1,
                         const double *S, const double *anchor, double *mu, double *Ppk, double *Sigma, double *cc,
                         double *Rout) {
    const int D = c->D;
    const uint64_t seed = c->cfg.seed;
    static _Thread_local double L[NP8O_DMAX * NP8O_DMAX], M[NP8O_DMAX * NP8O_DMAX], B[NP8O_DMAX * NP8O_DMAX],
        R[NP8O_DMAX * NP8O_DMAX], T[NP8O_DMAX * NP8O_DMAX], Ut[NP8O_DMAX * NP8O_DMAX];
    const double k0 = c->cfg.kappa, nd = (double)n;
    const double kn = k0 + nd, nun = c->cfg.nu + nd;
    const double kf = (k0 * nd) / kn;
    double xb[NP8O_DMAX], dm[NP8O_DMAX], mun[NP8O_DMAX];
    for (int a = 0; a < D; ++a) {
        xb[a] = (n > 0) ? anchor[a] + s1[a] / nd : c->cfg.mu0[a];
        dm[a] = xb[a] - c->cfg.mu0[a];
        mun[a] = fma(k0, c->cfg.mu0[a], nd * xb[a]) / kn;
    }
    /* Cholesky Lr of J Psin J (element (r, j), r >= j, is Psin[D-1-r][D-1-j]; formed on the fly) */
    memset(L, 0, sizeof(double) * D * D);
    for (int j = 0; j < D; ++j) {
        for (int r = j; r < D; ++r) {
            const int ri = D - 1 - r, ji = D - 1 - j; /* ri <= ji */
            const double sc = (n > 0) ? S[packed_ix(D, ri, ji)] - (s1[ri] * s1[ji]) / nd : 0.0;
            double v = fma(kf, dm[ri] * dm[ji], c->cfg.Lambda[ri * D + ji] + sc);
            for (int k = 0; k < j; ++k) v = fma(-L[r * D + k], L[j * D + k], v);
            if (r == j) {
                if (!(v > 0.0)) return -1;
                L[j * D + j] = sqrt(v);
            } else {
                L[r * D + j] = v / L[j * D + j];
            }
        }
    }
    /* M = Lr^{-1} (lower), forward substitution per column; U^{-1} = J M J */
    memset(M, 0, sizeof(double) * D * D);
    for (int j = 0; j < D; ++j) {
        M[j * D + j] = 1.0 / L[j * D + j];
        for (int r = j + 1; r < D; ++r) {
            double s = 0.0;
            for (int k = j; k < r; ++k) s = fma(-L[r * D + k], M[k * D + j], s);
            M[r * D + j] = s / L[r * D + r];
        }
    }
    memset(B, 0, sizeof(double) * D * D);
    logacc la = {1.0, 0.0};
    for (int a = 0; a < D; ++a) {
        const double g = chi2_mt(seed, i, t, stream, NIW_GAMMA_CALLS * (uint32_t)a, nun - a);
        B[a * D + a] = sqrt(g);
        logacc_add(&la, g, a, D - 1);
    }
    for (int a = 1; a < D; ++a)
        for (int b = 0; b < a; ++b)
            B[a * D + b] = normal_at(seed, i, t, stream, NIW_NORMAL_CALL0, (uint32_t)(a * (a - 1) / 2 + b));
    double z[NP8O_DMAX];
    for (int j = 0; j < D; ++j) z[j] = normal_at(seed, i, t, stream, NIW_NORMAL_CALL0, (uint32_t)(D * (D - 1) / 2 + j));
    /* R = B^T U^{-1}: R_ab = sum_{k = a..b} B_ka M[D-1-k][D-1-b] (a <= b) */
    memset(R, 0, sizeof(double) * D * D);
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) {
            double s = 0.0;
            for (int k = a; k <= b; ++k) s = fma(B[k * D + a], M[(D - 1 - k) * D + (D - 1 - b)], s);
            R[a * D + b] = s;
        }
    /* P' = packed sym(R^T R), off-diagonals doubled: element (a, b), a <= b = sum_{k <= a} R_ka R_kb */
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) {
            double s = 0.0;
            for (int k = 0; k <= a; ++k) s = fma(R[k * D + a], R[k * D + b], s);
            Ppk[packed_ix(D, a, b)] = (a == b) ? s : 2.0 * s;
        }
    /* mu = mun + U y, y = B^{-T} z / sqrt(kn): back substitution by columns, y_k = acc_k / B_kk for k = D-1, ..., 0,
     * each leaving fma(-B_ka, y_k, acc_a) in the sums of a < k (the device runs it on one wave, np8_niw.hip) */
    const double rskn = 1.0 / sqrt(kn);
    double y[NP8O_DMAX], acc[NP8O_DMAX];
    for (int a = 0; a < D; ++a) acc[a] = z[a] * rskn;
    for (int k = D - 1; k >= 0; --k) {
        y[k] = acc[k] / B[k * D + k];
        for (int a = 0; a < k; ++a) acc[a] = fma(-B[k * D + a], y[k], acc[a]);
    }
    for (int a = 0; a < D; ++a) {
        double s = 0.0; /* U_ak = Lr[D-1-a][D-1-k], k >= a */
        for (int k = a; k < D; ++k) s = fma(L[(D - 1 - a) * D + (D - 1 - k)], y[k], s);
        mu[a] = mun[a] + s;
    }
    /* Sigma = T^T T, T = B^{-1} U^T (U^T_aj = Lr[D-1-j][D-1-a], lower) */
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) Ut[a * D + b] = (b <= a) ? L[(D - 1 - b) * D + (D - 1 - a)] : 0.0;
    niw_sigma(D, B, Ut, T, Sigma);
    double sl = 0.0;
    for (int a = 0; a < D; ++a) sl += np8o_log_pos(L[a * D + a]);
    *cc = fma(0.5, la.sumlog, fma(-0.5 * (double)D, LOG2PI, -sl));
    if (Rout) memcpy(Rout, R, sizeof(double) * D * D);
    return 0;
}

/* The fp32 contraction rows of slot s from its factor R (R^T R = P): A = fp32(R) (transposed store), muf = fp32(mu). */
static void wide_rows_from_r(np8o_ctx *c, int s, const double *R) {
    const int D = c->D;
    float *At = c->wA + (size_t)s * D * D; /* transposed: At[b][a] = fp32(R[a][b]) */
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) At[b * D + a] = (b >= a) ? (float)R[a * D + b] : 0.0f;
    for (int a = 0; a < D; ++a) c->wmu[(size_t)s * D + a] = (float)c->slot_mu[(size_t)s * D + a];
}

/* Candidate table: live slots in ascending order, log n_k, log(n_k - 1) (weight 0 as the finite
 * NP8O_ZERO_LW), and the isotropy flag (off-diagonals of P' exactly 0, one common diagonal). */
#define NP8O_ZERO_LW (-1.0e300)
#define NP8O_SKIP 80.0 /* skip rule: relative weight below e^-80 (np8_device.h kSkip) */

/* Slot s from auxiliary m of item i (NIW prior). */
static void niw_slot_from_aux(np8o_ctx *c, int s, uint64_t i, uint32_t t, int m) {
    const int D = c->D;
    double dt[NP8O_DMAX];
    whiten(c, c->X + (size_t)NP8O_ITEM(i) * D, dt);
    niw_aux_slot(c, i, t, m, dt, c->slot_mu + (size_t)s * D, c->slot_P + (size_t)s * c->DP,
                 c->slot_sigma + (size_t)s * D * D, c->slot_c + s);
    if (c->wdirty) c->wdirty[s] = 1;
}

/* F32 contraction: A = fp32(R), R = chol_upper(sym Sigma^{-1}) (R^T R = P, fp64, R_jj first, then
 * row j of R left to right), and muf = fp32(mu).  A pivot <= 0 (not numerically positive definite)
 * leaves the rest of the row 0 and the pivot at 1e-300 (the device sets an error bit). */
static void wide_factor(np8o_ctx *c, int s) {
    const int D = c->D;
    const double *Pp = c->slot_P + (size_t)s * c->DP;
    double R[NP8O_DMAX * NP8O_DMAX];
    memset(R, 0, sizeof(double) * D * D);
    for (int j = 0; j < D; ++j) {
        double v = Pp[packed_index(D, j, j)];
        for (int k = 0; k < j; ++k) v = fma(-R[k * D + j], R[k * D + j], v);
        const int ok = v > 0.0;
        R[j * D + j] = ok ? sqrt(v) : 1e-300;
        for (int i = j + 1; i < D && ok; ++i) {
            double w = 0.5 * Pp[packed_index(D, j, i)];
            for (int k = 0; k < j; ++k) w = fma(-R[k * D + j], R[k * D + i], w);
            R[j * D + i] = w / R[j * D + j];
        }
    }
    wide_rows_from_r(c, s, R);
}

/* q of item x (fp32 values) for candidate slot sj (np8_oracle.h NP8O_CONTRACT_F32):
 * y_a = fmaf chain over b of A[a][b] (x_b - muf_b) from 0 (= v_mfma_f32_16x16x4_f32 in k order),
 * q = (s_0 + s_1) + (s_2 + s_3) in fp32, s_g = fp32 fmaf chain of y_a^2 over a = 16 mt + 4 g + r (mt outer,
 * r inner): the lane groups of the 16x16 accumulator layout; ll = c - q/2 in fp64. */
static double wide_q(const np8o_ctx *c, const double *x, int sj) {
    const int D = c->D;
    const float *At = c->wA + (size_t)sj * D * D, *mj = c->wmu + (size_t)sj * D;
    float xt[NP8O_DMAX], y[NP8O_DMAX];
    for (int b = 0; b < D; ++b) xt[b] = (float)x[b] - mj[b];
    /* R is upper triangular: A[a][b] = 0 for b < a, and fmaf(0, t, v) = v, so each row's chain starts at
     * b = a; the rows' chains run interleaved (b outer), each still in increasing b */
    for (int a = 0; a < D; ++a) y[a] = 0.0f;
    for (int b = 0; b < D; ++b) {
        const float t = xt[b];
        const float *col = At + (size_t)b * D;
        for (int a = 0; a <= b; ++a) y[a] = fmaf(col[a], t, y[a]);
    }
    /* any D: the device pads to DT = D rounded up to 16 with zero rows, whose squares are exact zeros */
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int g = 0; g < 4; ++g)
        for (int mt = 0; mt < (D + 15) / 16; ++mt)
            for (int r = 0; r < 4; ++r) {
                const int a = 16 * mt + 4 * g + r;
                if (a >= D) continue;
                const float v = y[a];
                s[g] = fmaf(v, v, s[g]);
            }
    return (double)((s[0] + s[1]) + (s[2] + s[3]));
}

static void rebuild_dense(np8o_ctx *c) {
    int K = 0;
    const int D = c->D;
    if (c->cfg.contraction == NP8O_CONTRACT_F32)
        for (int s = 0; s < c->kcap; ++s)
            if (c->cnt[s] > 0 && c->wdirty[s]) {
                wide_factor(c, s);
                c->wdirty[s] = 0;
            }
    for (int s = 0; s < c->kcap; ++s) {
        c->dense_of[s] = -1;
        if (c->cnt[s] > 0) {
            const double *P = c->slot_P + (size_t)s * c->DP;
            int iso = 1;
            for (int a = 0, q = 0; a < D; ++a)
                for (int b = a; b < D; ++b, ++q) iso = iso && ((a == b) ? (P[q] == P[0]) : (P[q] == 0.0));
            c->dense_of[s] = K;
            c->live[K] = s;
            c->logn[K] = np8o_log_pos((double)c->cnt[s]);
            c->logn1[K] = (c->cnt[s] > 1) ? np8o_log_pos((double)(c->cnt[s] - 1)) : NP8O_ZERO_LW;
            c->iso[K] = iso ? P[0] : 0.0;
            ++K;
        }
    }
    c->K = K;
}

int np8o_set_state(np8o_ctx *c, const int32_t *z, int32_t K, const double *mu, const double *Sigma) {
    if (K > c->kcap || K < 0) return -1;
    memset(c->cnt, 0, sizeof(int32_t) * c->kcap);
    for (int k = 0; k < K; ++k)
        if (slot_from_sigma(c, k, mu + (size_t)k * c->D, Sigma + (size_t)k * c->D * c->D) != 0) return -2;
    for (int64_t i = 0; i < c->N; ++i) {
        if (z[i] < 0 || z[i] >= K) return -3;
        c->z[i] = z[i];
        c->cnt[z[i]]++;
    }
    rebuild_dense(c);
    c->t = 0;
    c->have_best = 0;
    c->best_L = -INFINITY;
    return 0;
}

/* np_mcmc.cpp:49-92 + np_init_clusters.cpp:24-40: K_init G0 clusters, uniform assignment, cleanup. */
int np8o_init_random(np8o_ctx *c, int32_t K_init) {
    if (K_init < 1) return -1;
    const int D = c->D;
    if (K_init > c->kcap) return -1;
    double *mu = (double *)malloc(sizeof(double) * (size_t)K_init * D);
    double *vv = (double *)malloc(sizeof(double) * (size_t)K_init);
    int32_t *cntk = (int32_t *)calloc((size_t)K_init, sizeof(int32_t));
    const int niw = c->cfg.prior == NP8O_PRIOR_NIW;
    for (int k = 0; k < K_init && !niw; ++k) {
        double g[NP8O_DMAX + 4];
        for (int call = 0; call < g0_calls(D); ++call)
            normal_quad(c->cfg.seed, (uint64_t)k, 0xFFFFFFFFu, NP8O_STREAM_INIT_THETA, (uint32_t)call, g + 4 * call);
        aux_from_normals(c, g[0], g + 1, vv + k, mu + (size_t)k * D);
    }
    for (int64_t i = 0; i < c->N; ++i) {
        double u = np8o_uniform(c->cfg.seed, (uint64_t)i, 0xFFFFFFFFu, NP8O_STREAM_INIT_Z, 0);
        int k = (int)(u * (double)K_init);
        if (k >= K_init) k = K_init - 1;
        c->z[i] = k;
        cntk[k]++;
    }
    /* cleanup (membertrix.cpp:343-364): drop empty clusters, keep ascending order */
    int32_t *remap = (int32_t *)malloc(sizeof(int32_t) * (size_t)K_init);
    int s = 0;
    memset(c->cnt, 0, sizeof(int32_t) * c->kcap);
    for (int k = 0; k < K_init; ++k) {
        if (cntk[k] > 0) {
            remap[k] = s;
            if (c->wdirty) c->wdirty[s] = 1;
            if (niw) { /* G0 draw k: the NIW posterior of no items, stream INIT_THETA (i = k) */
                static _Thread_local double Rk[NP8O_DMAX * NP8O_DMAX];
                if (niw_draw_impl(c, (uint64_t)k, 0xFFFFFFFFu, NP8O_STREAM_INIT_THETA, 0, NULL, NULL, NULL,
                                  c->slot_mu + (size_t)s * D, c->slot_P + (size_t)s * c->DP,
                                  c->slot_sigma + (size_t)s * D * D, c->slot_c + s, Rk) == 0 && c->wdirty) {
                    wide_rows_from_r(c, s, Rk); /* the draw's own factor */
                    c->wdirty[s] = 0;
                }
            } else
                slot_from_aux(c, s, vv[k], mu + (size_t)k * D);
            c->cnt[s] = cntk[k];
            ++s;
        } else {
            remap[k] = -1;
        }
    }
    for (int64_t i = 0; i < c->N; ++i) c->z[i] = remap[c->z[i]];
    free(remap);
    free(mu);
    free(vv);
    free(cntk);
    rebuild_dense(c);
    c->t = 0;
    c->have_best = 0;
    c->best_L = -INFINITY;
    return 0;
}

static inline double quad_form(const np8o_ctx *c, const double *x, const double *mu, const double *P) {
    const int D = c->D;
    double d[NP8O_DMAX];
    for (int a = 0; a < D; ++a) d[a] = x[a] - mu[a];
    double q = 0.0;
    int k = 0;
    for (int a = 0; a < D; ++a) {
        double t = P[k++] * d[a];
        for (int b = a + 1; b < D; ++b) t = fma(P[k++], d[b], t);
        q = fma(t, d[a], q);
    }
    return q;
}

/* ll of point x under slot s, packed table form (the max-likelihood sum, np_mcmc.cpp:187-203). */
static inline double slot_ll(const np8o_ctx *c, const double *x, int s) {
    double q = quad_form(c, x, c->slot_mu + (size_t)s * c->D, c->slot_P + (size_t)s * c->DP);
    return fma(-0.5, q, c->slot_c[s]);
}

/* ll of point x (own row jo) under candidate row j (what the sweep uses): isotropic rows q = iso |d|^2;
 * F32 contraction: wide_q in the frame of the own cluster. */
static inline double cand_ll(const np8o_ctx *c, const double *x, int jo, int j) {
    const int s = c->live[j];
    (void)jo;
    if (c->cfg.contraction == NP8O_CONTRACT_F32) return fma(-0.5, wide_q(c, x, s), c->slot_c[s]);
    if (c->iso[j] > 0.0) {
        const int D = c->D;
        const double *mu = c->slot_mu + (size_t)s * D;
        double d0 = x[0] - mu[0];
        double acc = d0 * d0;
        for (int a = 1; a < D; ++a) {
            const double d = x[a] - mu[a];
            acc = fma(d, d, acc);
        }
        return fma(-0.5, acc * c->iso[j], c->slot_c[s]);
    }
    return slot_ll(c, x, s);
}

/* ll of point x under its M auxiliary draws, in the item's frame (DESIGN.md "G0"). */
static void aux_ll(const np8o_ctx *c, const double *x, uint64_t i, uint32_t t, double *ll /* M */) {
    double y0[NP8O_DMAX];
    const double ny = whiten(c, x, y0); /* NIW: dt = U^T (x - mu0) */
    if (c->cfg.prior == NP8O_PRIOR_NIW) {
        for (int m = 0; m < c->M; ++m) {
            double sumlog, b00, chi, z1;
            niw_aux_core(c, i, t, m, &sumlog, &b00, &chi, &z1);
            ll[m] = niw_aux_loglik(c, ny, sumlog, b00, chi, z1);
        }
        return;
    }
    for (int m = 0; m < c->M; ++m) {
        double v, xpar, chi2;
        aux_core(c, i, t, m, &v, &xpar, &chi2);
        ll[m] = aux_loglik(c, ny, v, xpar, chi2);
    }
}

/* ---- categorical draw: single-uniform weighted reservoir (DESIGN.md "Pick") ------------------
 * Equal in distribution to dim1algebra.hpp:2078-2104 (inverse CDF over the linear weights) but one
 * pass: state (T, S, u) with S = sum of exp(lw_j - T) so far and u ~ U(0,1) independent of the
 * current pick; candidate j replaces the pick with probability w_j / S_new and u is renormalised
 * into the chosen sub-interval.  A candidate with lw <= T - 80 (relative weight below 1.8e-35, beyond
 * the resolution of the reference's one double uniform) is skipped. */
typedef struct {
    double T, S, u;
    int32_t pick;
} pick_state;

static inline double clamp_u(double u) { return fmin(fmax(u, 0x1.0p-60), 0x1.fffffffffffffp-1); }

static inline void pick_step(pick_state *st, double lw, int32_t j) {
    const double d = lw - st->T;
    if (d <= -NP8O_SKIP) return;
    const int gt = d > 0.0;
    const double e = np8o_exp_le0(-fabs(d));
    const double a = gt ? 1.0 : e;
    const double S = gt ? fma(st->S, e, 1.0) : st->S + e;
    const double uS = st->u * S;
    const int take = uS < a;
    const double num = take ? uS : uS - a;
    const double den = take ? a : S - a;
    st->u = clamp_u(num / den);
    if (take) st->pick = j;
    if (gt) st->T = lw;
    st->S = S;
}

/* One Neal-8 step for point i against the frozen candidate table (np_neal_algorithm8.cpp:60-130).
 * Order of the draw: the item's own cluster first (weight n_k - 1; 0 for a singleton, whose cluster
 * the reference deletes on retract, membertrix.cpp:200-203), then every other live cluster in
 * ascending slot order (weight n_k), then the M auxiliaries (weight alpha/M).  Returns the candidate
 * row (< K existing, >= K auxiliary). */
int64_t np8o_pick_reservoir(const double *lw, int64_t n, double u) {
    if (n <= 0) return 0;
    pick_state st = {lw[0], 1.0, u, 0};
    for (int64_t j = 1; j < n; ++j) pick_step(&st, lw[j], (int32_t)j);
    return st.pick;
}

void np8o_pick_reservoir_batch(const double *lw, int64_t n, const double *u, int64_t n_draws, int32_t *out) {
    for (int64_t k = 0; k < n_draws; ++k) out[k] = (int32_t)np8o_pick_reservoir(lw, n, u[k]);
}

/* NP8O_PICK_INVCDF: the reference's inverse-CDF rule over exp(lw - max), candidates in the order
 * choose() visits them (own, other live slots ascending, auxiliaries); returns the candidate row. */
static int32_t choose_invcdf(const np8o_ctx *c, int64_t key, const double *x, int32_t jo) {
    const int K = c->K, M = c->M;
    double lw[NP8O_KCAP_PICK + NP8O_MMAX];
    int32_t row[NP8O_KCAP_PICK + NP8O_MMAX];
    int n = 0;
    lw[n] = cand_ll(c, x, jo, jo) + c->logn1[jo];
    row[n++] = jo;
    for (int j = 0; j < K; ++j) {
        if (j == jo) continue;
        lw[n] = cand_ll(c, x, jo, j) + c->logn[j];
        row[n++] = j;
    }
    double lla[NP8O_MMAX];
    aux_ll(c, x, (uint64_t)key, c->t, lla);
    for (int m = 0; m < M; ++m) {
        lw[n] = lla[m] + c->logam;
        row[n++] = K + m;
    }
    double mx = lw[0];
    for (int j = 1; j < n; ++j) mx = fmax(mx, lw[j]);
    double w[NP8O_KCAP_PICK + NP8O_MMAX];
    for (int j = 0; j < n; ++j) w[j] = exp(lw[j] - mx);
    const double u = np8o_uniform(c->cfg.seed, (uint64_t)key, c->t, NP8O_STREAM_PICK, 0);
    return row[np8o_weighted_pick_ref(w, n, u)];
}

static int32_t choose(const np8o_ctx *c, int64_t key, const double *x, int32_t zi) {
    const int K = c->K, M = c->M;
    const int jo = c->dense_of[zi];
    if (c->cfg.pick == NP8O_PICK_INVCDF) return choose_invcdf(c, key, x, jo);
    pick_state st;
    st.T = cand_ll(c, x, jo, jo) + c->logn1[jo];
    st.S = 1.0;
    st.u = np8o_uniform(c->cfg.seed, (uint64_t)key, c->t, NP8O_STREAM_PICK, 0);
    st.pick = jo;
    for (int j = 0; j < K; ++j) {
        if (j == jo) continue;
        pick_step(&st, cand_ll(c, x, jo, j) + c->logn[j], j);
    }
    double lla[NP8O_MMAX];
    aux_ll(c, x, (uint64_t)key, c->t, lla);
    for (int m = 0; m < M; ++m) pick_step(&st, lla[m] + c->logam, K + m);
    return st.pick;
}

static inline int64_t position_to_point(const np8o_ctx *c, int64_t p, int sync, const int64_t *order) {
    if (order) return order[p];
    if (sync) return p;
    return (int64_t)np8o_perm(c->cfg.seed, c->t, (uint32_t)c->N, (uint32_t)p);
}

static int assign_range_impl(np8o_ctx *c, int64_t p0, int64_t p1, int sync, const int64_t *order, int32_t *delta,
                             int64_t *req_pos, int64_t *req_i, int32_t *req_m, int32_t *req_zold, int32_t req_cap,
                             int32_t *n_req) {
    int32_t nr = 0;
    int err = 0;
    if (sync && p1 - p0 > 1) {
        /* synchronous step: items are independent given the frozen state, so the CPU-parallel
         * baseline (SURVEY.md 8(d) "cpu_par") runs them on all threads with identical results
         * (finalize orders requests by position) */
#pragma omp parallel for schedule(static)
        for (int64_t p = p0; p < p1; ++p) {
            const int64_t key = position_to_point(c, p, sync, order), i = NP8O_ITEM(key);
            const double *x = c->X + (size_t)i * c->D;
            const int32_t zi = c->z[i];
            const int32_t j = choose(c, key, x, zi);
            if (j < c->K) {
                const int32_t s = c->live[j];
                if (s != zi) {
#pragma omp atomic
                    delta[zi] -= 1;
#pragma omp atomic
                    delta[s] += 1;
                    c->z[i] = s;
                }
            } else {
                int32_t q;
#pragma omp atomic capture
                q = nr++;
                if (q < req_cap) {
                    req_pos[q] = p;
                    req_i[q] = key;
                    req_m[q] = j - c->K;
                    req_zold[q] = zi;
                }
            }
        }
        *n_req = nr;
        return err;
    }
    for (int64_t p = p0; p < p1; ++p) {
        const int64_t key = position_to_point(c, p, sync, order), i = NP8O_ITEM(key);
        const double *x = c->X + (size_t)i * c->D;
        int32_t zi = c->z[i];
        int32_t j = choose(c, key, x, zi);
        if (j < c->K) {
            int32_t s = c->live[j];
            if (s != zi) {
                delta[zi] -= 1;
                delta[s] += 1;
                c->z[i] = s;
            }
        } else {
            if (nr < req_cap) {
                req_pos[nr] = p;
                req_i[nr] = key;
                req_m[nr] = j - c->K;
                req_zold[nr] = zi;
            }
            ++nr; /* counted even past the capacity */
        }
    }
    *n_req = nr;
    return err;
}

int np8o_assign_range(np8o_ctx *c, int64_t p0, int64_t p1, int32_t *delta, int64_t *req_pos, int64_t *req_i,
                      int32_t *req_m, int32_t *req_zold, int32_t req_cap, int32_t *n_req) {
    int64_t chunk = c->cfg.chunk <= 0 ? c->N : c->cfg.chunk;
    return assign_range_impl(c, p0, p1, chunk >= c->N, NULL, delta, req_pos, req_i, req_m, req_zold, req_cap, n_req);
}

/* New-cluster requests (DESIGN.md "Finalize"): the deltas are applied first; the free slots are
 * counted then, with every requester still in its old slot; the A = min(req_max, free, n_req)
 * requests of lowest scan position are accepted and take the lowest free slots in ascending order
 * (position order); each accepted requester leaves its old slot (which may become free for the next
 * step); the remaining requesters keep their cluster -- their update is deferred to the next time they
 * are visited (the next step or sweep), like an item whose draw picked its own cluster. */
static int cmp_req(const void *a, const void *b) {
    const int64_t *x = (const int64_t *)a, *y = (const int64_t *)b;
    return (x[0] > y[0]) - (x[0] < y[0]);
}

int np8o_finalize(np8o_ctx *c, const int32_t *delta, const int64_t *req_pos, const int64_t *req_i,
                  const int32_t *req_m, const int32_t *req_zold, int32_t n_req, int64_t owner_lo, int64_t owner_hi) {
    const int D = c->D;
    for (int s = 0; s < c->kcap; ++s) c->cnt[s] += delta[s];
    int32_t nfree = 0;
    for (int s = 0; s < c->kcap; ++s) nfree += (c->cnt[s] == 0);
    int32_t A = n_req < c->req_max ? n_req : c->req_max;
    if (A > nfree) A = nfree;
    if (A > 0) {
        int64_t *ord = (int64_t *)malloc(sizeof(int64_t) * 2 * (size_t)n_req);
        for (int32_t q = 0; q < n_req; ++q) {
            ord[2 * q] = req_pos[q];
            ord[2 * q + 1] = q;
        }
        qsort(ord, (size_t)n_req, 2 * sizeof(int64_t), cmp_req);
        /* the free slots before any requester leaves (a slot emptied by a departure is free next step) */
        int32_t *freeslot = (int32_t *)malloc(sizeof(int32_t) * (size_t)A);
        for (int s = 0, f = 0; s < c->kcap && f < A; ++s)
            if (c->cnt[s] == 0) freeslot[f++] = s;
        for (int32_t q = 0; q < A; ++q) {
            const int s = freeslot[q];
            const int64_t r = ord[2 * q + 1];
            const int64_t key = req_i[r], i = NP8O_ITEM(key);
            if (c->cfg.prior == NP8O_PRIOR_NIW) {
                niw_slot_from_aux(c, s, (uint64_t)key, c->t, req_m[r]);
            } else {
                double vv[NP8O_MMAX], mm[NP8O_MMAX * NP8O_DMAX];
                aux_draws(c, (uint64_t)key, c->t, vv, mm);
                slot_from_aux(c, s, vv[req_m[r]], mm + (size_t)req_m[r] * D);
            }
            c->cnt[s] = 1;
            c->cnt[req_zold[r]] -= 1;
            if (owner_hi < 0 || (i >= owner_lo && i < owner_hi)) c->z[i] = s;
        }
        free(freeslot);
        free(ord);
    }
    c->n_new += A;
    c->n_deferred += n_req - A;
    rebuild_dense(c);
    return n_req - A;
}

double np8o_total_loglik(np8o_ctx *c) {
    double L = 0.0;
    for (int64_t i = 0; i < c->N; ++i) {
        const int jo = c->dense_of[c->z[i]];
        L += cand_ll(c, c->X + (size_t)i * c->D, jo, jo);
    }
    return L;
}

/* ---- cluster-parameter update (mh_g0) ---------------------------------------------------------
 * The reference's UpdateClusters::update (src/np_update_clusters.cpp:71-142, called once per sweep
 * from np_mcmc.cpp:170 with number_mh_steps = 20, :54) as it is meant to work -- in the reference
 * the accepted proposal is sliced away, so `frozen` is its effective behaviour.
 * Per live cluster and MH step: theta' ~ G0 (independence proposal, :33-59), accept if
 * u < exp(LL(theta') - LL(theta)) (:118-132; LL == 0 accepts, :114-117), LL = sum over the cluster's
 * items of log N(x | theta) (multivariatenormal.cpp:138-146), evaluated from statistics about the
 * anchor a = mu at the start of the update (d = x - a, s1 = sum d, S = sum d d^T):
 *   current:  LL = n c - tr(P' S)/2                                (P' = packed, off-diagonals doubled)
 *   proposal: LL' = n c' - (tr(G S) - 2 e^T G s1 + n e^T G e) / (2 v'^2),  e = mu' - a,
 *             G = (L^T L)^{-1}, c' = caux - D log|v'|               (Sigma' = v'^2 L^T L)
 * Randomness: proposal normals = Philox stream PARAM (i = slot, calls step*Q .. step*Q+Q-1, laid out
 * like an auxiliary draw), acceptance uniform = stream PARAM_U (i = slot, call = step). */
int np8o_suffstats(np8o_ctx *c, double *out) {
    const int D = c->D, W = D + c->DP;
    memset(out, 0, sizeof(double) * (size_t)c->kcap * W);
    for (int64_t i = 0; i < c->N; ++i) {
        const int s = c->z[i];
        const double *x = c->X + (size_t)i * D;
        const double *mu = c->slot_mu + (size_t)s * D;
        double *o = out + (size_t)s * W;
        double d[NP8O_DMAX];
        for (int a = 0; a < D; ++a) {
            d[a] = x[a] - mu[a];
            o[a] += d[a];
        }
        for (int a = 0, k = D; a < D; ++a)
            for (int b = a; b < D; ++b, ++k) o[k] += d[a] * d[b];
    }
    return 0;
}

/* log-likelihood of n items with statistics (s1, S) about anchor a under the G0 draw (v, mu'). */
static double mh_proposal_ll(const np8o_ctx *c, int64_t n, double trGS, const double *g1, const double *anchor,
                             double v, const double *mup) {
    const int D = c->D;
    double e[NP8O_DMAX], eg = 0.0, eGe = 0.0;
    for (int a = 0; a < D; ++a) {
        e[a] = mup[a] - anchor[a];
        eg = fma(e[a], g1[a], eg);
    }
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) eGe = fma(c->Gp[a * D + b], e[a] * e[b], eGe);
    const double tr = fma((double)n, eGe, fma(-2.0, eg, trGS));
    const double cp = fma(-(double)D, np8o_log_pos(fabs(v)), c->caux);
    return fma(-0.5, tr / (v * v), (double)n * cp);
}

static void mh_proposal(const np8o_ctx *c, int s, uint32_t t, int step, double *v, double *mup) {
    const int Q = g0_calls(c->D);
    double g[NP8O_DMAX + 4];
    for (int k = 0; k < Q; ++k)
        normal_quad(c->cfg.seed, (uint64_t)s, t, NP8O_STREAM_PARAM, (uint32_t)(step * Q + k), g + 4 * k);
    aux_from_normals(c, g[0], g + 1, v, mup);
}

/* NIW_CONJUGATE: every live slot's (mu, Sigma) drawn from its posterior (niw_draw_impl) given the
 * statistics about its current mean; draws on stream PARAM (i = slot) at the current epoch.  A slot
 * whose posterior scale is not numerically positive definite keeps its parameters. */
static int64_t niw_param_update(np8o_ctx *c, const double *stats) {
    const int D = c->D, W = D + c->DP;
    int64_t updated = 0;
    double anchor[NP8O_DMAX];
    for (int s = 0; s < c->kcap; ++s) {
        const int64_t n = c->cnt[s];
        if (n <= 0) continue;
        memcpy(anchor, c->slot_mu + (size_t)s * D, sizeof(double) * D);
        const double *s1 = stats + (size_t)s * W;
        static _Thread_local double Rs[NP8O_DMAX * NP8O_DMAX];
        if (niw_draw_impl(c, (uint64_t)s, c->t, NP8O_STREAM_PARAM, n, s1, s1 + D, anchor, c->slot_mu + (size_t)s * D,
                          c->slot_P + (size_t)s * c->DP, c->slot_sigma + (size_t)s * D * D, c->slot_c + s, Rs) == 0) {
            ++updated;
            if (c->wdirty) {
                wide_rows_from_r(c, s, Rs); /* the draw's own factor */
                c->wdirty[s] = 0;
            }
        }
    }
    rebuild_dense(c);
    return updated;
}

int np8o_niw_draw(np8o_ctx *c, uint64_t i, uint32_t t, uint32_t stream, int64_t n, const double *stats,
                  const double *anchor, double *mu, double *Sigma) {
    if (c->cfg.prior != NP8O_PRIOR_NIW) return -1;
    static double P[NP8O_DMAX * (NP8O_DMAX + 1) / 2];
    double cc;
    return niw_draw_impl(c, i, t, stream, n, stats, stats ? stats + c->D : NULL, anchor, mu, P, Sigma, &cc, NULL);
}

int64_t np8o_param_update(np8o_ctx *c, const double *stats) {
    if (c->cfg.param_update == NP8O_PARAM_NIW_CONJUGATE) return niw_param_update(c, stats);
    const int D = c->D, DP = c->DP, W = D + DP;
    const int steps = c->cfg.mh_steps > 0 ? c->cfg.mh_steps : 20;
    int64_t accepted = 0;
    for (int s = 0; s < c->kcap; ++s) {
        const int64_t n = c->cnt[s];
        if (n <= 0) continue;
        const double *s1 = stats + (size_t)s * W, *S = s1 + D;
        const double *P = c->slot_P + (size_t)s * DP;
        double anchor[NP8O_DMAX];
        memcpy(anchor, c->slot_mu + (size_t)s * D, sizeof(double) * D);
        double trPS = 0.0, trGS = 0.0, g1[NP8O_DMAX];
        for (int a = 0, k = 0; a < D; ++a)
            for (int b = a; b < D; ++b, ++k) {
                trPS = fma(P[k], S[k], trPS);
                trGS = fma(c->Gp[a * D + b], S[k], trGS);
            }
        for (int a = 0; a < D; ++a) {
            double acc = 0.0;
            for (int b = 0; b < D; ++b) acc = fma((a == b) ? c->Gp[a * D + b] : 0.5 * c->Gp[a * D + b], s1[b], acc);
            g1[a] = acc;
        }
        double LL = fma(-0.5, trPS, (double)n * c->slot_c[s]);
        int chosen = -1;
        for (int step = 0; step < steps; ++step) {
            double v, mup[NP8O_DMAX];
            mh_proposal(c, s, c->t, step, &v, mup);
            const double LLp = mh_proposal_ll(c, n, trGS, g1, anchor, v, mup);
            const double u = np8o_uniform(c->cfg.seed, (uint64_t)s, c->t, NP8O_STREAM_PARAM_U, (uint32_t)step);
            const double dl = LLp - LL;
            if (LL == 0.0 || dl >= 0.0 || u < np8o_exp_le0(dl)) {
                LL = LLp;
                chosen = step;
                ++accepted;
            }
        }
        if (chosen >= 0) {
            double v, mup[NP8O_DMAX];
            mh_proposal(c, s, c->t, chosen, &v, mup);
            slot_from_aux(c, s, v, mup);
        }
    }
    rebuild_dense(c);
    return accepted;
}

int np8o_end_sweep(np8o_ctx *c) {
    if (c->cfg.param_update != NP8O_PARAM_FROZEN && c->N > 0) {
        double *st = (double *)malloc(sizeof(double) * (size_t)c->kcap * (c->D + c->DP));
        np8o_suffstats(c, st);
        c->mh_accepted += np8o_param_update(c, st);
        free(st);
    }
    if (c->t % 5u == 0u) { /* np_mcmc.cpp:172-174 */
        double L = np8o_total_loglik(c);
        if (L > c->best_L) {
            c->best_L = L;
            c->have_best = 1;
            memcpy(c->z_best, c->z, sizeof(int32_t) * (size_t)c->N);
            memcpy(c->cnt_best, c->cnt, sizeof(int32_t) * c->kcap);
            memcpy(c->mu_best, c->slot_mu, sizeof(double) * (size_t)c->kcap * c->D);
            memcpy(c->sigma_best, c->slot_sigma, sizeof(double) * (size_t)c->kcap * c->D * c->D);
        }
    }
    c->t += 1u;
    return 0;
}

static int run_chunks(np8o_ctx *c, const int64_t *order, int64_t npos, int64_t chunk) {
    int err = 0;
    const int sync = (order == NULL) && (chunk >= c->N);
    for (int64_t p0 = 0; p0 < npos; p0 += chunk) {
        int64_t p1 = (p0 + chunk < npos) ? p0 + chunk : npos;
        memset(c->delta, 0, sizeof(int32_t) * c->kcap);
        int32_t nr = 0;
        int e1 = assign_range_impl(c, p0, p1, sync, order, c->delta, c->rq_pos, c->rq_i, c->rq_m, c->rq_zold,
                                   (int32_t)(p1 - p0), &nr);
        (void)np8o_finalize(c, c->delta, c->rq_pos, c->rq_i, c->rq_m, c->rq_zold, nr, 0, -1);
        if (e1) err = e1;
    }
    return err;
}

/* The data-parallel sweep in S sub-steps: one synchronous step per sub-step over its items (ascending;
 * scan position = rank in that list, so requests are accepted in ascending item order). */
static int run_substeps(np8o_ctx *c) {
    int err = 0;
    const int S = c->cfg.substeps > 1 ? c->cfg.substeps : 1;
    for (int k = 0; k < S; ++k) {
        const int64_t *items = c->sub_items + c->sub_start[k];
        const int64_t n = c->sub_start[k + 1] - c->sub_start[k];
        memset(c->delta, 0, sizeof(int32_t) * c->kcap);
        int32_t nr = 0;
        int e1 = assign_range_impl(c, 0, n, 1, items, c->delta, c->rq_pos, c->rq_i, c->rq_m, c->rq_zold,
                                   (int32_t)(n > 0 ? n : 1), &nr);
        (void)np8o_finalize(c, c->delta, c->rq_pos, c->rq_i, c->rq_m, c->rq_zold, nr, 0, -1);
        if (e1) err = e1;
    }
    return err;
}

int np8o_sweep(np8o_ctx *c, int32_t n) {
    int err = 0;
    int64_t chunk = c->cfg.chunk <= 0 ? c->N : c->cfg.chunk;
    if (chunk > c->N) chunk = c->N;
    for (int s = 0; s < n; ++s) {
        if (c->N > 0) {
            int e = (chunk >= c->N && c->cfg.substeps > 1) ? run_substeps(c) : run_chunks(c, NULL, c->N, chunk);
            if (e) err = e;
        }
        np8o_end_sweep(c);
    }
    return err;
}

int np8o_update_points(np8o_ctx *c, const int64_t *ids, int64_t n) {
    for (int64_t k = 0; k < n; ++k)
        if (ids[k] < 0 || ids[k] >= c->N) return -3;
    /* item keys: the k-th visit of an item within this epoch draws with visit index k */
    int64_t *keys = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t k = 0; k < n; ++k) {
        const int64_t i = ids[k];
        if (c->vis_tag[i] != c->t + 1u) {
            c->vis_tag[i] = c->t + 1u;
            c->vis_n[i] = 0;
        }
        keys[k] = i | ((int64_t)c->vis_n[i]++ << 32);
    }
    const int r = run_chunks(c, keys, n, 1);
    free(keys);
    return r;
}

void np8o_request_stats(np8o_ctx *c, int64_t out[2]) {
    out[0] = c->n_new;
    out[1] = c->n_deferred;
}

int np8o_get_state(np8o_ctx *c, int32_t which, int32_t *z, int32_t *K, double *mu, double *Sigma,
                   int64_t *counts) {
    const int D = c->D;
    const int32_t *zz = c->z, *cc = c->cnt;
    const double *mm = c->slot_mu, *ss = c->slot_sigma;
    if (which == 1) {
        if (!c->have_best) return -5;
        zz = c->z_best;
        cc = c->cnt_best;
        mm = c->mu_best;
        ss = c->sigma_best;
    }
    int32_t *lab = (int32_t *)malloc(sizeof(int32_t) * c->kcap);
    int k = 0;
    for (int s = 0; s < c->kcap; ++s) {
        if (cc[s] > 0) {
            lab[s] = k;
            if (mu) memcpy(mu + (size_t)k * D, mm + (size_t)s * D, sizeof(double) * D);
            if (Sigma) memcpy(Sigma + (size_t)k * D * D, ss + (size_t)s * D * D, sizeof(double) * D * D);
            if (counts) counts[k] = cc[s];
            ++k;
        } else {
            lab[s] = -1;
        }
    }
    if (K) *K = k;
    if (z)
        for (int64_t i = 0; i < c->N; ++i) z[i] = lab[zz[i]];
    free(lab);
    return 0;
}

int32_t np8o_num_clusters(np8o_ctx *c) { return c->K; }
uint32_t np8o_epoch(np8o_ctx *c) { return c->t; }
double np8o_best_loglik(np8o_ctx *c) { return c->best_L; }
int64_t np8o_mh_accepted(np8o_ctx *c) { return c->mh_accepted; }

void np8o_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
int32_t *np8o_z_ptr(np8o_ctx *c) { return c->z; }

int np8o_loglik_matrix(np8o_ctx *c, const int64_t *idx, int64_t n, double *out) {
    const int K = c->K, M = c->M;
    for (int64_t r = 0; r < n; ++r) {
        int64_t i = idx[r];
        if (i < 0 || i >= c->N) return -3;
        const double *x = c->X + (size_t)i * c->D;
        for (int j = 0; j < K; ++j) out[r * (K + M) + j] = cand_ll(c, x, c->dense_of[c->z[i]], j);
        aux_ll(c, x, (uint64_t)i, c->t, out + r * (K + M) + K);
    }
    return 0;
}

int np8o_aux_params(np8o_ctx *c, int64_t i, double *mu, double *Sigma) {
    const int D = c->D;
    if (c->cfg.prior == NP8O_PRIOR_NIW) {
        double dt[NP8O_DMAX], cc;
        static double P[NP8O_DMAX * (NP8O_DMAX + 1) / 2], Sg[NP8O_DMAX * NP8O_DMAX];
        whiten(c, c->X + (size_t)i * D, dt);
        for (int m = 0; m < c->M; ++m) {
            niw_aux_slot(c, (uint64_t)i, c->t, m, dt, mu + (size_t)m * D, P, Sg, &cc);
            if (Sigma) memcpy(Sigma + (size_t)m * D * D, Sg, sizeof(double) * D * D);
        }
        return 0;
    }
    double vv[NP8O_MMAX];
    aux_draws(c, (uint64_t)i, c->t, vv, mu);
    if (Sigma)
        for (int m = 0; m < c->M; ++m)
            for (int k = 0; k < D * D; ++k) Sigma[(size_t)m * D * D + k] = vv[m] * vv[m] * c->LTL[k];
    return 0;
}

int np8o_loglik_matrix_ref(np8o_ctx *c, const int64_t *idx, int64_t n, double *out) {
    const int K = c->K, M = c->M, D = c->D;
    double amu[NP8O_MMAX * NP8O_DMAX], asig[NP8O_MMAX * NP8O_DMAX * NP8O_DMAX];
    for (int64_t r = 0; r < n; ++r) {
        int64_t i = idx[r];
        if (i < 0 || i >= c->N) return -3;
        const double *x = c->X + (size_t)i * D;
        for (int j = 0; j < K; ++j) {
            int s = c->live[j];
            out[r * (K + M) + j] =
                np8o_mvn_logprobability_ref(x, c->slot_mu + (size_t)s * D, c->slot_sigma + (size_t)s * D * D, D);
        }
        np8o_aux_params(c, i, amu, asig);
        for (int m = 0; m < M; ++m)
            out[r * (K + M) + K + m] =
                np8o_mvn_logprobability_ref(x, amu + (size_t)m * D, asig + (size_t)m * D * D, D);
    }
    return 0;
}

/* ================================================================================================
 * Jain-Neal split-merge: src/np_jain_neal_algorithm.cpp driven by
 * src/np_mcmc.cpp:117-164 with subset_count = 2 (src/np_main.cpp:440-445).  One sweep = N attempts;
 * attempt a takes the pair (pi0(a), pi1(a)) of two independent scan permutations (np_mcmc.cpp:118-125,
 * 142-148; a pair with equal items is skipped, :153-156).  Same cluster: split (:251-351) with the
 * sams_prior allocation (:146-171); different clusters: merge of the first item's cluster into the
 * second's (:353-429).  The reference's own rules are kept (DESIGN.md "Split-merge"): the SAMS weights
 * are log-likelihood + count fed to the linear-weight pick (:157-168 with dim1algebra.hpp:2078-2104,
 * including lower_bound on a non-monotone cumulative sum), the proposal ratio is 0 (:57-59) and the
 * acceptance is exp(q + p + lratio) >= u (:306-316, :398-408).  Members are visited in ascending item
 * order (the reference shuffles them, :121; the data are permuted at load, np_main.cpp:283-295);
 * sums over members use canon_sum (256 lane-strided partials, then a pairwise tree) -- the order the
 * device reduces in.  The cluster log-likelihoods use the sweep's candidate form (isotropic rows by
 * the |d|^2 shortcut, others by the packed table form).
 * ============================================================================================== */
static const double kLgammaTab[33] = {
    0.0, /* unused: n >= 1 */
    0.0, 0.0, 0.693147180559945, 1.7917594692280554, 3.178053830347945, 4.787491742782047,
    6.579251212010102, 8.525161361065415, 10.604602902745249, 12.801827480081467, 15.104412573075514,
    17.502307845873887, 19.987214495661885, 22.55216385312342, 25.191221182738683, 27.89927138384089,
    30.671860106080672, 33.50507345013689, 36.39544520803305, 39.339884187199495, 42.335616460753485,
    45.38013889847691, 48.47118135183522, 51.60667556776438, 54.78472939811232, 58.00360522298052,
    61.26170176100201, 64.55753862700634, 67.88974313718153, 71.257038967168, 74.65823634883017,
    78.0922235533153};

/* log Gamma(n) for an integer n >= 1 (std::lgamma at np_jain_neal_algorithm.cpp:48): table to 32,
 * Stirling's series beyond (truncation error < 1e-17 relative for n > 32). */
double np8o_lgamma_int(int64_t n) {
    if (n <= 32) return kLgammaTab[n < 1 ? 1 : n];
    const double x = (double)n;
    const double r = 1.0 / x, r2 = r * r;
    const double s = r * (0.083333333333333333 - r2 * (0.0027777777777777778 - r2 * (0.00079365079365079365 - r2 * 0.00059523809523809524)));
    return ((x - 0.5) * np8o_log_pos(x) - x) + 0.91893853320467274178 + s;
}

/* Canonical sum of v[0..n) (only entries with keep[p] != 0 when keep is given): partial t sums
 * p = t, t+256, .. in ascending order, then partial[t] += partial[t+h] for h = 128, 64, .., 1. */
static double canon_sum(const double *v, const unsigned char *keep, int64_t n) {
    double part[256];
    for (int t = 0; t < 256; ++t) part[t] = 0.0;
    for (int64_t p = 0; p < n; ++p)
        if (!keep || keep[p]) part[p & 255] += v[p];
    for (int h = 128; h >= 1; h >>= 1)
        for (int t = 0; t < h; ++t) part[t] += part[t + h];
    return part[0];
}

double np8o_canon_sum(const double *v, int64_t n) { return canon_sum(v, NULL, n); }

static const uint64_t kSmPermKey[2] = {0x4A4E53504C495430ull, 0x4A4E53504C495431ull};

/* Members of every slot in ascending item order: mem[off[s] .. off[s+1]). */
static void sm_members(np8o_ctx *c) {
    int64_t *off = c->sm_off;
    for (int s = 0; s <= c->kcap; ++s) off[s] = 0;
    for (int64_t i = 0; i < c->N; ++i) off[c->z[i] + 1]++;
    for (int s = 0; s < c->kcap; ++s) off[s + 1] += off[s];
    int64_t *cur = c->sm_cur;
    for (int s = 0; s < c->kcap; ++s) cur[s] = off[s];
    for (int64_t i = 0; i < c->N; ++i) c->sm_mem[cur[c->z[i]]++] = i;
}

/* Cluster log-likelihood of the split-merge moves: the sweep's candidate form (cand_ll) -- the
 * isotropic shortcut for rows whose P' is a multiple of I, else the packed quadratic form. */
static double sm_iso_ll(const double *x, const double *mu, int D, double iso, double cc) {
    double d0 = x[0] - mu[0];
    double acc = d0 * d0;
    for (int a = 1; a < D; ++a) {
        const double d = x[a] - mu[a];
        acc = fma(d, d, acc);
    }
    return fma(-0.5, acc * iso, cc);
}

static double sm_slot_ll(const np8o_ctx *c, const double *x, int s) {
    const double iso = c->iso[c->dense_of[s]];
    if (iso > 0.0) return sm_iso_ll(x, c->slot_mu + (size_t)s * c->D, c->D, iso, c->slot_c[s]);
    return slot_ll(c, x, s);
}

/* Gp = (L^T L)^{-1} a multiple of I: its diagonal, else 0 (the new slots' isotropic factor). */
static double sm_gp_iso(const np8o_ctx *c) {
    const int D = c->D;
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b)
            if ((a == b) ? c->Gp[a * D + b] != c->Gp[0] : c->Gp[a * D + b] != 0.0) return 0.0;
    return c->Gp[0];
}

/* accept iff exp(x) >= u (x > 0: always) */
static int sm_accept(double x, double u) { return (x >= 0.0) || !(np8o_exp_le0(x) < u); }

/* The new cluster of a split attempt: a G0 draw on stream SM_THETA (i = attempt, t = epoch). */
static void sm_theta(const np8o_ctx *c, uint64_t a, double *v, double *mu) {
    double g[NP8O_DMAX + 4];
    for (int call = 0; call < g0_calls(c->D); ++call)
        normal_quad(c->cfg.seed, a, c->t, NP8O_STREAM_SM_THETA, (uint32_t)call, g + 4 * call);
    aux_from_normals(c, g[0], g + 1, v, mu);
}

/* One attempt.  Returns 0 skipped, 1 split rejected, 2 merge rejected, 3 split accepted,
 * 4 merge accepted, 5 split rejected for want of a free slot. */
static int sm_attempt(np8o_ctx *c, uint64_t a) {
    const int D = c->D;
    const uint32_t N = (uint32_t)c->N;
    const int64_t i = np8o_perm(c->cfg.seed ^ kSmPermKey[0], c->t, N, (uint32_t)a);
    const int64_t j = np8o_perm(c->cfg.seed ^ kSmPermKey[1], c->t, N, (uint32_t)a);
    if (i == j) return 0;
    const int ci = c->z[i], cj = c->z[j];
    const double u_acc = np8o_uniform(c->cfg.seed, a, c->t, NP8O_STREAM_SM_ACCEPT, 0);
    const int64_t *L = c->sm_mem + c->sm_off[ci];
    const int64_t n0 = c->sm_off[ci + 1] - c->sm_off[ci];
    double *own = c->sm_v0, *nw = c->sm_v1;
    if (ci != cj) { /* merge ci into cj */
        for (int64_t p = 0; p < n0; ++p) {
            const double *x = c->X + (size_t)L[p] * D;
            own[p] = sm_slot_ll(c, x, ci);
            nw[p] = sm_slot_ll(c, x, cj);
        }
        const double lsrc = canon_sum(own, NULL, n0), ldest = canon_sum(nw, NULL, n0);
        const int64_t n1 = c->cnt[cj];
        const double pr = c->sm_log_alpha + np8o_lgamma_int(n0) + np8o_lgamma_int(n1) - np8o_lgamma_int(n0 + n1);
        if (!sm_accept(-pr + (ldest - lsrc), u_acc)) return 2;
        for (int64_t p = 0; p < n0; ++p) c->z[L[p]] = cj;
        c->cnt[cj] += (int32_t)n0;
        c->cnt[ci] = 0;
        return 4;
    }
    /* split: the move set starts with i, the remaining set with j */
    double v, mu[NP8O_DMAX];
    sm_theta(c, a, &v, mu);
    double Pn[NP8O_DMAX * (NP8O_DMAX + 1) / 2];
    const double v2 = v * v;
    for (int q = 0, aa = 0; aa < D; ++aa)
        for (int b = aa; b < D; ++b, ++q) Pn[q] = c->Gp[aa * D + b] / v2;
    const double cn = fma(-(double)D, np8o_log_pos(fabs(v)), c->caux);
    const double gi = sm_gp_iso(c), isn = (gi > 0.0) ? gi / v2 : 0.0;
    unsigned char *mv = c->sm_flag;
    int64_t m = 1, r = 1;
    for (int64_t p = 0; p < n0; ++p) {
        const double *x = c->X + (size_t)L[p] * D;
        own[p] = sm_slot_ll(c, x, ci);
        nw[p] = (isn > 0.0) ? sm_iso_ll(x, mu, D, isn, cn) : fma(-0.5, quad_form(c, x, mu, Pn), cn);
        if (L[p] == i) {
            mv[p] = 1;
            continue;
        }
        if (L[p] == j) {
            mv[p] = 0;
            continue;
        }
        const double a0 = own[p] + (double)r, a1 = nw[p] + (double)m;
        const double tot = a0 + a1;
        const double w = np8o_uniform(c->cfg.seed, a, c->t, NP8O_STREAM_SM_ALLOC, (uint32_t)p) * tot;
        const int idx = (tot < w) ? 2 : ((a0 < w) ? 1 : 0); /* std::lower_bound over {a0, a0+a1} */
        mv[p] = (unsigned char)(idx != 0);
        if (idx != 0)
            ++m;
        else
            ++r;
    }
    const double lsrc = canon_sum(own, mv, n0), ldest = canon_sum(nw, mv, n0);
    const double pr = c->sm_log_alpha + np8o_lgamma_int(m) + np8o_lgamma_int(r) - np8o_lgamma_int(n0);
    if (!sm_accept(pr + (ldest - lsrc), u_acc)) return 1;
    int s = -1;
    for (int k = 0; k < c->kcap; ++k)
        if (c->cnt[k] == 0) {
            s = k;
            break;
        }
    if (s < 0) return 5;
    slot_from_aux(c, s, v, mu);
    for (int64_t p = 0; p < n0; ++p)
        if (mv[p]) c->z[L[p]] = s;
    c->cnt[ci] -= (int32_t)m;
    c->cnt[s] = (int32_t)m;
    return 3;
}

int np8o_sm_sweep(np8o_ctx *c, int32_t n) {
    if (c->cfg.prior != NP8O_PRIOR_REFERENCE || c->cfg.contraction != NP8O_CONTRACT_F64) return -1;
    for (int s = 0; s < n; ++s) {
        sm_members(c);
        for (int64_t a = 0; a < c->N; ++a) {
            const int o = sm_attempt(c, (uint64_t)a);
            c->sm_stats[o]++;
            if (o == 3 || o == 4) {
                rebuild_dense(c);
                sm_members(c);
            }
        }
        np8o_end_sweep(c);
    }
    return 0;
}

int np8o_sm_attempts(np8o_ctx *c, int64_t a0, int64_t a1) {
    if (c->cfg.prior != NP8O_PRIOR_REFERENCE || c->cfg.contraction != NP8O_CONTRACT_F64) return -1;
    sm_members(c);
    for (int64_t a = a0; a < a1 && a < c->N; ++a) {
        const int o = sm_attempt(c, (uint64_t)a);
        c->sm_stats[o]++;
        if (o == 3 || o == 4) {
            rebuild_dense(c);
            sm_members(c);
        }
    }
    return 0;
}

void np8o_sm_get_stats(np8o_ctx *c, int64_t out[6]) {
    for (int k = 0; k < 6; ++k) out[k] = c->sm_stats[k];
}

/* ================================================================================================
 * Triadic split-merge: src/np_triadic_algorithm.cpp driven by
 * src/np_mcmc.cpp:117-164 with subset_count = 3 (np_main.cpp:447-455).  Attempt a takes the items of
 * three independent scan permutations (skipped unless all distinct, np_mcmc.cpp:153-156) and a
 * uniform u_b (stream SM_ACCEPT, call 1; the reference's first draw in update(), :676):
 *   one cluster             -> dyadic split 1 -> 2 of it (:679-699), picks (p0, p2)
 *   else u_b < beta (0.5)   -> dyadic merge 2 -> 1 (:701-724): the pair left after duplicate_pick
 *                              (dim1algebra.hpp:2117-2137) removes one; all items go to the first's
 *   else two clusters       -> triadic split 2 -> 3 (:731-755), the duplicate moved last
 *   else three clusters     -> triadic merge 3 -> 2 (:757-775): clusters 0, 1 keep, 2 dissolves
 * A move reallocates every member of its source clusters (sams_prior, propose_split :208-296 and
 * propose_merge :135-206): pick q starts target q (q < Q), the other members -- those of the sources
 * in order, ascending item order within each (the reference shuffles them) -- go to target q with
 * weight p(x | theta_q) |target q| (linear probabilities as the reference; drawn here from
 * w_q = exp(lw_q - max lw), lw_q = ll_q + log|target q|, by one uniform over the cumulative sum --
 * the same pick without the reference's all-underflow fallback to index 0).  Acceptance
 * exp(rQ + rP + rR + rL) >= u (:414-425, :577-590) with rQ = 0 (sams_prior :100-102),
 * rP = +-(log alpha + sum lgamma(larger partition sizes) - sum lgamma(smaller)) (:78-94),
 * rR = log beta, -log(1-beta), -log beta, log(1-beta) for 1->2, 2->3, 2->1, 3->2 (:116-131),
 * rL = sum of the after-move log-likelihoods - sum of the before ones; sums over members of several
 * clusters are the sums, in source order, of per-source canon_sums.
 * ============================================================================================== */
static const uint64_t kTriPermKey[3] = {0x5452494144494330ull, 0x5452494144494331ull, 0x5452494144494332ull};
#define TRI_BETA 0.5

/* ll of x under target q: an existing slot, or the new cluster (mu, isotropic factor / packed P, c) */
typedef struct {
    int slot; /* -1: new cluster */
    const double *mu, *P;
    double iso, cc;
} tri_target;

static double tri_ll(const np8o_ctx *c, const double *x, const tri_target *tg) {
    if (tg->slot >= 0) return sm_slot_ll(c, x, tg->slot);
    if (tg->iso > 0.0) return sm_iso_ll(x, tg->mu, c->D, tg->iso, tg->cc);
    return fma(-0.5, quad_form(c, x, tg->mu, tg->P), tg->cc);
}

/* Reallocate the members of sources src[0..ns) over targets tg[0..Q) (picks[q] starts target q; the
 * other members in order by the max-shifted weighted pick).  asg[...] receives the target of every
 * member (concatenated source order); np[q] the target sizes; lp[q] the after-move log-likelihoods. */
static void tri_walk(np8o_ctx *c, uint64_t a, const int *src, int ns, const tri_target *tg, int Q,
                     const int64_t *picks, int32_t *asg, int64_t *np, double *lp) {
    const int D = c->D;
    for (int q = 0; q < Q; ++q) {
        np[q] = 1;
        lp[q] = 0.0;
    }
    int64_t rank = 0;
    double *v = c->sm_v0;
    for (int si = 0; si < ns; ++si) {
        const int64_t *L = c->sm_mem + c->sm_off[src[si]];
        const int64_t n = c->sm_off[src[si] + 1] - c->sm_off[src[si]];
        for (int64_t p = 0; p < n; ++p, ++rank) {
            const double *x = c->X + (size_t)L[p] * D;
            int pq = -1;
            for (int q = 0; q < Q; ++q)
                if (L[p] == picks[q]) pq = q;
            int32_t d;
            if (pq >= 0) {
                d = pq;
            } else {
                double lw[3], mx = -INFINITY;
                for (int q = 0; q < Q; ++q) {
                    lw[q] = tri_ll(c, x, tg + q) + np8o_log_pos((double)np[q]);
                    mx = fmax(mx, lw[q]);
                }
                double cum[3], tot = 0.0;
                for (int q = 0; q < Q; ++q) {
                    tot += np8o_exp_le0(lw[q] - mx);
                    cum[q] = tot;
                }
                const double w = np8o_uniform(c->cfg.seed, a, c->t, NP8O_STREAM_SM_ALLOC, (uint32_t)rank) * tot;
                d = Q - 1;
                for (int q = 0; q < Q; ++q)
                    if (cum[q] >= w) {
                        d = q;
                        break;
                    }
                np[d]++;
            }
            asg[rank] = d;
        }
    }
    /* per-source canonical sums of the after-move likelihoods */
    rank = 0;
    for (int si = 0; si < ns; ++si) {
        const int64_t *L = c->sm_mem + c->sm_off[src[si]];
        const int64_t n = c->sm_off[src[si] + 1] - c->sm_off[src[si]];
        for (int q = 0; q < Q; ++q) {
            for (int64_t p = 0; p < n; ++p) {
                c->sm_flag[p] = (unsigned char)(asg[rank + p] == q);
                v[p] = c->sm_flag[p] ? tri_ll(c, c->X + (size_t)L[p] * D, tg + q) : 0.0;
            }
            lp[q] += canon_sum(v, c->sm_flag, n);
        }
        rank += n;
    }
}

/* Before-move log-likelihood of source s: canon_sum of its members under its own parameters. */
static double tri_own(np8o_ctx *c, int s) {
    const int64_t *L = c->sm_mem + c->sm_off[s];
    const int64_t n = c->sm_off[s + 1] - c->sm_off[s];
    for (int64_t p = 0; p < n; ++p) c->sm_v0[p] = sm_slot_ll(c, c->X + (size_t)L[p] * c->D, s);
    return canon_sum(c->sm_v0, NULL, n);
}

/* first index whose cluster id repeats an earlier one; the last index when all differ */
static int tri_duplicate_pick(const int *ids, int n) {
    for (int i = 1; i < n; ++i)
        for (int j = 0; j < i; ++j)
            if (ids[j] == ids[i]) return i;
    return n - 1;
}

/* Outcomes: 0 skipped, 1/2 dyadic merge rejected/accepted, 3/4 dyadic split rejected/accepted,
 * 5/6 triadic merge rejected/accepted, 7/8 triadic split rejected/accepted, 9 split accepted by the
 * ratio but dropped for want of a free slot. */
static int tri_attempt(np8o_ctx *c, uint64_t a) {
    const int D = c->D;
    const uint32_t N = (uint32_t)c->N;
    int64_t pk[3];
    int cl[3];
    for (int r = 0; r < 3; ++r) pk[r] = np8o_perm(c->cfg.seed ^ kTriPermKey[r], c->t, N, (uint32_t)a);
    if (pk[0] == pk[1] || pk[0] == pk[2] || pk[1] == pk[2]) return 0;
    for (int r = 0; r < 3; ++r) cl[r] = c->z[pk[r]];
    const int uniq = 1 + (cl[1] != cl[0]) + (cl[2] != cl[0] && cl[2] != cl[1]);
    const double ub = np8o_uniform(c->cfg.seed, a, c->t, NP8O_STREAM_SM_ACCEPT, 1);
    const double u = np8o_uniform(c->cfg.seed, a, c->t, NP8O_STREAM_SM_ACCEPT, 0);
    int kind; /* 0 dyadic merge, 1 dyadic split, 2 triadic merge, 3 triadic split */
    if (uniq == 1) {
        kind = 1;
        pk[1] = pk[2]; /* duplicate_pick([c,c,c]) = 1 is removed */
        cl[1] = cl[2];
    } else if (ub < TRI_BETA) {
        kind = 0;
        const int rm = tri_duplicate_pick(cl, 3);
        for (int r = rm; r < 2; ++r) {
            pk[r] = pk[r + 1];
            cl[r] = cl[r + 1];
        }
    } else if (uniq == 2) {
        kind = 3;
        const int dp = tri_duplicate_pick(cl, 3);
        int64_t tp = pk[dp];
        pk[dp] = pk[2];
        pk[2] = tp;
        int tc = cl[dp];
        cl[dp] = cl[2];
        cl[2] = tc;
    } else {
        kind = 2;
    }
    const int split = (kind & 1);
    const int ns = (kind == 0) ? 2 : (kind == 1 ? 1 : (kind == 2 ? 3 : 2)); /* sources */
    const int Q = (kind == 0) ? 1 : (kind == 1 ? 2 : (kind == 2 ? 2 : 3));  /* targets */
    int src[3];
    for (int i = 0; i < ns; ++i) src[i] = cl[i];
    tri_target tg[3];
    double v = 0.0, mu[NP8O_DMAX], Pn[NP8O_DMAX * (NP8O_DMAX + 1) / 2];
    for (int q = 0; q < Q; ++q) {
        tg[q].slot = (split && q == Q - 1) ? -1 : cl[q];
        tg[q].mu = tg[q].P = NULL;
        tg[q].iso = tg[q].cc = 0.0;
    }
    if (split) {
        sm_theta(c, a, &v, mu);
        const double v2 = v * v;
        for (int q = 0, aa = 0; aa < D; ++aa)
            for (int b = aa; b < D; ++b, ++q) Pn[q] = c->Gp[aa * D + b] / v2;
        const double gi = sm_gp_iso(c);
        tg[Q - 1].mu = mu;
        tg[Q - 1].P = Pn;
        tg[Q - 1].iso = (gi > 0.0) ? gi / v2 : 0.0;
        tg[Q - 1].cc = fma(-(double)D, np8o_log_pos(fabs(v)), c->caux);
    }
    int64_t nsrc[3], np[3], ntot = 0;
    double ld[3], lp[3];
    for (int i = 0; i < ns; ++i) {
        nsrc[i] = c->sm_off[src[i] + 1] - c->sm_off[src[i]];
        ntot += nsrc[i];
        ld[i] = tri_own(c, src[i]);
    }
    int32_t *asg = c->tri_asg;
    tri_walk(c, a, src, ns, tg, Q, pk, asg, np, lp);
    /* rP (:78-94): more = the larger partition, less = the smaller */
    double frac = 0.0;
    if (split) {
        for (int q = 0; q < Q; ++q) frac += np8o_lgamma_int(np[q]);
        for (int i = 0; i < ns; ++i) frac -= np8o_lgamma_int(nsrc[i]);
    } else {
        for (int i = 0; i < ns; ++i) frac += np8o_lgamma_int(nsrc[i]);
        for (int q = 0; q < Q; ++q) frac -= np8o_lgamma_int(np[q]);
    }
    const double rP = split ? c->sm_log_alpha + frac : -(c->sm_log_alpha + frac);
    const double rR = (kind == 1) ? log(TRI_BETA) : (kind == 3) ? -log(1.0 - TRI_BETA)
                                                 : (kind == 0) ? -log(TRI_BETA) : log(1.0 - TRI_BETA);
    double rLd = 0.0, rLdp = 0.0;
    for (int i = 0; i < ns; ++i) rLd += ld[i];
    for (int q = 0; q < Q; ++q) rLdp += lp[q];
    const double x = ((0.0 + rP) + rR) + (rLdp - rLd);
    if (!sm_accept(x, u)) return 1 + 2 * kind;
    int snew = -1;
    if (split) {
        for (int k = 0; k < c->kcap; ++k)
            if (c->cnt[k] == 0) {
                snew = k;
                break;
            }
        if (snew < 0) return 9;
        slot_from_aux(c, snew, v, mu);
    }
    int64_t rank = 0;
    for (int i = 0; i < ns; ++i) {
        const int64_t *L = c->sm_mem + c->sm_off[src[i]];
        for (int64_t p = 0; p < nsrc[i]; ++p, ++rank) {
            const int d = asg[rank];
            c->z[L[p]] = (tg[d].slot >= 0) ? tg[d].slot : snew;
        }
    }
    for (int i = 0; i < ns; ++i) c->cnt[src[i]] = 0;
    for (int q = 0; q < Q; ++q) c->cnt[(tg[q].slot >= 0) ? tg[q].slot : snew] = (int32_t)np[q];
    return 2 + 2 * kind;
}

int np8o_tri_sweep(np8o_ctx *c, int32_t n) {
    if (c->cfg.prior != NP8O_PRIOR_REFERENCE || c->cfg.contraction != NP8O_CONTRACT_F64) return -1;
    for (int s = 0; s < n; ++s) {
        sm_members(c);
        for (int64_t a = 0; a < c->N; ++a) {
            const int o = tri_attempt(c, (uint64_t)a);
            c->tri_stats[o]++;
            if (o > 0 && o < 9 && (o & 1) == 0) {
                rebuild_dense(c);
                sm_members(c);
            }
        }
        np8o_end_sweep(c);
    }
    return 0;
}

int np8o_tri_attempts(np8o_ctx *c, int64_t a0, int64_t a1) {
    if (c->cfg.prior != NP8O_PRIOR_REFERENCE || c->cfg.contraction != NP8O_CONTRACT_F64) return -1;
    sm_members(c);
    for (int64_t a = a0; a < a1 && a < c->N; ++a) {
        const int o = tri_attempt(c, (uint64_t)a);
        c->tri_stats[o]++;
        if (o > 0 && o < 9 && (o & 1) == 0) {
            rebuild_dense(c);
            sm_members(c);
        }
    }
    return 0;
}

void np8o_tri_get_stats(np8o_ctx *c, int64_t out[10]) {
    for (int k = 0; k < 10; ++k) out[k] = c->tri_stats[k];
}
