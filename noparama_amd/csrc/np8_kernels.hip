// np8_kernels.hip -- gfx950 kernels of the Neal Algorithm 8 sweep.
//
//   np8_assign<D,M>   one lane per data item: fp64 log-likelihood against every live cluster (cluster
//                     table read through the scalar cache: wave-uniform addresses, SGPR operands) and
//                     against M auxiliary G0 draws generated in-register from Philox; block-reservoir
//                     categorical draw; writes the new label or a new-cluster request.
//                     Reference: src/np_neal_algorithm8.cpp:49-167 (one point), np_mcmc.cpp:146-164.
//   np8_finalize      one workgroup: applies count deltas of all ranks, turns new-cluster requests into
//                     clusters (membertrix::addCluster/assign, membertrix.cpp:87-164), frees empty ones
//                     (retract auto-remove, membertrix.cpp:200-203) and rebuilds the dense candidate table.
//   np8_loglik / np8_loglik_reduce / np8_snapshot
//                     MCMC::considerMaxLikelihood (np_mcmc.cpp:187-203): sum_i log p(x_i|theta_z_i),
//                     keep the labelling when it improves.
//   np8_loglik_matrix debug/parity: the assign kernel's log-likelihoods for chosen items.
#include "np8_kernels.h"

#include <hip/hip_runtime.h>

using namespace np8;

// Checked indices (debug builds only, -DNP8_CHECKED, tools/ab_build.sh): an index outside [lo, hi) is printed with its
// source line and replaced by lo, so that a bad state is named instead of faulting the GPU.
#ifdef NP8_CHECKED
__device__ int g_np8_chk[8];  // the first failed check: line, value, lo, hi (read by np8_exp_checks)
__device__ __noinline__ int64_t np8_chk(int64_t v, int64_t lo, int64_t hi, int line) {
    if (v < lo || v >= hi) {
        if (atomicCAS(&g_np8_chk[0], 0, line) == 0) {
            g_np8_chk[1] = (int)v;
            g_np8_chk[2] = (int)lo;
            g_np8_chk[3] = (int)hi;
        }
        atomicAdd(&g_np8_chk[4], 1);
        return lo;
    }
    return v;
}
extern "C" int np8_exp_checks(int *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_np8_chk), sizeof(int) * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#define NP8_CHK(v, lo, hi) np8_chk((int64_t)(v), (int64_t)(lo), (int64_t)(hi), __LINE__)
#else
#define NP8_CHK(v, lo, hi) (v)
#endif

namespace {

template <int D>
struct HypView {
    // hyp layout: mu0[D] | UinvT packed[DP] | caux | rsk | logam | nu | LT packed[DP]
    static constexpr int DP = D * (D + 1) / 2;
    static constexpr int kMu0 = 0;
    static constexpr int kUinvT = D;
    static constexpr int kCaux = D + DP;
    static constexpr int kRsk = kCaux + 1;
    static constexpr int kLogam = kCaux + 2;
    static constexpr int kNu = kCaux + 3;
    static constexpr int kLT = kCaux + 4;
    static constexpr int kSmax = kLT + DP;  // NIW screen: bound of the D-1 further log chi^2 draws
    static constexpr int kUdiag = kSmax + 1;  // the diagonal of UinvT again, contiguous (one scalar load round)
    // level 0 of the auxiliary screen (aux_screen0): 1/gamma, the |v| interval [v_lo, v_hi], c = rsk xmax
    static constexpr int kPre = kUdiag + D;
};

// ll = c - q/2 with q = d' P d.  Isotropic entries (iso > 0, a wave-uniform branch): q = iso * |d|^2;
// otherwise the packed upper triangle with pre-doubled off-diagonals.
template <int D>
__device__ __forceinline__ double cand_ll(const double *__restrict__ e, const double (&x)[D]) {
    constexpr int DP = D * (D + 1) / 2;
    double d[D];
#pragma unroll
    for (int a = 0; a < D; ++a) d[a] = x[a] - e[a];
    const double iso = e[D + DP + kFieldIso];
    double q;
    if (iso > 0.0) {
        double s = d[0] * d[0];
#pragma unroll
        for (int a = 1; a < D; ++a) s = fma(d[a], d[a], s);
        q = s * iso;
    } else {
        const double *P = e + D;
        q = 0.0;
        int k = 0;
#pragma unroll
        for (int a = 0; a < D; ++a) {
            double t = P[k++] * d[a];
#pragma unroll
            for (int b = a + 1; b < D; ++b) t = fma(P[k++], d[b], t);
            q = fma(t, d[a], q);
        }
    }
    return fma(-0.5, q, e[D + DP + kFieldC]);
}

// y0 = (L^T)^{-1} (x - mu0): the item in the whitened frame of the base measure.
template <int D>
__device__ __forceinline__ void whiten(const double *__restrict__ hyp, const double (&x)[D], double (&y0)[D]) {
    using H = HypView<D>;
    double dx[D];
#pragma unroll
    for (int a = 0; a < D; ++a) dx[a] = x[a] - hyp[H::kMu0 + a];
    const double *U = hyp + H::kUinvT;
    int k = 0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double t0 = U[k++] * dx[a];
#pragma unroll
        for (int b = a + 1; b < D; ++b) t0 = fma(U[k++], dx[b], t0);
        y0[a] = t0;
    }
}

// Log-likelihood of the item (whitened: ny = |y0|) under auxiliary G0 draw m of (item ig, epoch t),
// in the item's frame: (v, xi_par, chi2) from aux_core (normalinvwishart.h:44-64, invwishart.h:34-46,
// multivariatenormal.cpp:124-135; DESIGN.md "G0").
template <int D>
__device__ __forceinline__ double aux_ll(const double *__restrict__ hyp, double ny, uint64_t seed, uint64_t ig,
                                         uint32_t t, int m, int M) {
    using H = HypView<D>;
    double v, xpar, chi2;
    aux_core<D>(seed, ig, t, m, M, hyp[H::kNu], v, xpar, chi2);
    return aux_loglik(ny, v, xpar, chi2, D, hyp[H::kRsk], hyp[H::kCaux]);
}

// Log-likelihood of the item (whitened by U^T: nd = |U^T (x - mu0)|) under auxiliary m of the NIW prior.
template <int D>
__device__ __forceinline__ double niw_aux_ll(const double *__restrict__ hyp, double nd, uint64_t seed, uint64_t ig,
                                             uint32_t t, int m) {
    using H = HypView<D>;
    double sumlog, b00, chi, z1;
    niw_aux_core(seed, ig, t, m, D, hyp[H::kNu], sumlog, b00, chi, z1);
    return niw_aux_loglik(nd, sumlog, b00, chi, z1, hyp[H::kRsk], hyp[H::kCaux]);
}

// Screen of an auxiliary (DESIGN.md "Auxiliary screen"): an upper bound (plus its error margin) of the
// exact fp64 log-likelihood aux_core + aux_loglik computes.  From the words w of call 0: v and xi_par
// exactly, chi2 >= -2 log(u_0 u_1) (the other uniforms are <= 1, g_odd^2 >= 0) plus chi_extra, what the
// caller adds from call 1 (level 2), so
//   ll = caux - D log|v| - q/2,  q = (ny/|v| - rsk xi_par)^2 + rsk^2 chi2  >=  the same with chi2's bound.
// fp32 on the transcendental units (v_log_f32, v_sqrt_f32, v_cos_f32/v_sin_f32 in revolutions,
// v_rcp_f32); the margin covers those approximations with a factor of ten: |error of r cos, r sin| <=
// 4e-3 (3.5e-4 from rounding u0 to fp32 near 1), relative 1e-4 elsewhere, chi_extra_err for chi_extra.
// |v| enters only through the interval [av_lo, av_hi], which contains it whenever the error of g0 is within
// dg, so the bound stays valid for small |v|: ny/|v| and -D log|v| grow there, and the relative margin grows
// with them (qlb and D |log av_lo| are in err).  Returns +inf (no screen) when av_lo < 0.02, which keeps the
// interval away from 0; tests/test_gpu_screen.py drives many lanes into |v| in [0.02, 0.25] in count mode.
template <int D>
__device__ __forceinline__ float aux_screen_ub(const uint32_t (&w)[4], float chi_extra, float chi_extra_err, float ny,
                                               float nu, float rsk, float caux, float thr, bool with_thr = true) {
    constexpr float kLn2 = 0.693147180559945f;
    constexpr int k = (D - 1) / 2;
    const float u0 = fmaf((float)w[0], 0x1.0p-32f, 0x1.0p-33f);
    const float u1 = fmaf((float)w[1], 0x1.0p-32f, 0x1.0p-33f);
    const float r = __builtin_amdgcn_sqrtf(-2.0f * kLn2 * __builtin_amdgcn_logf(u0));
    const float g0 = r * __builtin_amdgcn_cosf(u1);
    const float xp = r * __builtin_amdgcn_sinf(u1);
    const float v = fmaf(nu, g0, (float)D);
    const float av = fabsf(v);
    float chi = chi_extra;
    if constexpr (k >= 2) {
        const float ua = fmaf((float)w[2], 0x1.0p-32f, 0x1.0p-33f), ub = fmaf((float)w[3], 0x1.0p-32f, 0x1.0p-33f);
        chi = fmaf(-2.0f * kLn2, __builtin_amdgcn_logf(ua * ub), chi);
    } else if constexpr (k == 1) {
        chi = fmaf(-2.0f * kLn2, __builtin_amdgcn_logf(fmaf((float)w[2], 0x1.0p-32f, 0x1.0p-33f)), chi);
    }
    // interval bounds: |v| in [av_lo, av_hi], xi_par in [xp - dg, xp + dg] (dg = 4e-3 covers r cos, r sin)
    constexpr float dg = 4e-3f;
    const float dv = nu * dg;
    const float av_lo = av - dv, av_hi = av + dv;
    const float a_lo = fmaf(-rsk, xp + dg, ny * __builtin_amdgcn_rcpf(av_hi));  // ny / |v| - rsk xi_par
    const float a_hi = fmaf(-rsk, xp - dg, ny * __builtin_amdgcn_rcpf(av_lo));
    const float amin = (a_lo > 0.0f) ? a_lo : ((a_hi < 0.0f) ? -a_hi : 0.0f);
    const float lnv = kLn2 * __builtin_amdgcn_logf(av_lo);  // -D log|v| <= -D log av_lo
    const float rsk2 = rsk * rsk;
    const float qlb = fmaf(amin, amin, rsk2 * fmaxf(chi - chi_extra_err, 0.0f));
    const float ub_ll = fmaf(-0.5f, qlb, caux - (float)D * lnv);
    // with_thr = false: the margin without the threshold's own term, which the caller adds once thr is known
    // (np8_assign_fast screens before its own row is loaded: ub + 1e-4 |thr| <= thr)
    const float err = 1.0f + 1e-4f * (qlb + fabsf(caux) + (float)D * fabsf(lnv) + (with_thr ? fabsf(thr) : 0.0f));
    return (av_lo >= 0.02f) ? ub_ll + err : __builtin_inff();
}

// Level 0 of the screen (round 6): an upper bound of auxiliary m's log-likelihood from the item's prefix call alone
// (aux_pre_call: the leading b bits of its first P chi^2 uniforms), the supremum over the draws of call 0 taken in
// closed form:
//   ll = caux - D log|v| - q/2,  q = (ny/|v| - rsk xi_par)^2 + rsk^2 chi2  <=  caux + S(ny) - rsk^2 chi2_lb / 2,
//   S(ny) = max over |v| in [v_lo, v_hi] of h(|v|),  h(a) = -D log a - (ny/a - c)_+^2 / 2,  c = rsk xmax,
// since |xi_par| <= r <= xmax = 6.77 for every Box-Muller pair of u32_01 uniforms (r <= sqrt(-2 log 2^-33) = 6.7638)
// and |v| = |D + nu g0| lies in [max(D - |nu| xmax, 0), D + |nu| xmax].  h rises up to a* = ny / gamma, gamma =
// (sqrt(c^2 + 4D) + c) / 2, and falls after it (a^3 h'(a) = -D a^2 - c ny a + ny^2 below ny/c, -D a^2 above), so
// S = h(clamp(a*, v_lo, v_hi)).  chi2 >= chi2_lb = -2 log prod_j (field_j + 1) 2^-b over the prefixed uniforms (each
// u32_01 word with that prefix is below (field + 1) 2^-b; the other uniforms are <= 1 and g_odd^2 >= 0).  In fp32 with
// the level-1 screen's margin (1 nat + 1e-4 of every term); S = +inf (no screen) when the interval reaches |v| = 0 at
// ny = 0.  Returns the bound without the threshold's own margin term, which the caller adds (as for level 1).
// s0: S(ny) (aux_screen0_s, once per item); k2 = rsk^2 / 2.
template <int D, int M>
__device__ __forceinline__ float aux_screen0_ub(const uint32_t (&pre)[4], int m, float s0, float s0_abs, float caux,
                                                float k2) {
    constexpr int P = D > kPreMaxD ? 0 : ((D - 1) / 2 < 3 ? (D - 1) / 2 : 3);  // (aux_pre_n)
    constexpr int b0 = P > 0 ? 128 / (M * P) : 0;
    constexpr int b = b0 > 16 ? 16 : b0;
    if constexpr (P == 0) {
        return __builtin_inff();
    } else {
        float prod = 1.0f;
#pragma unroll
        for (int j = 0; j < P; ++j) prod *= (float)(aux_pre_field(pre, m * P + j, b) + 1u);
        // chi2_lb = 2 ln2 (P b - log2 prod) >= 0 (each factor <= 2^b)
        const float chi = 2.0f * 0.693147180559945f * fmaxf((float)(P * b) - __builtin_amdgcn_logf(prod), 0.0f);
        const float ub = fmaf(-k2, chi, caux + s0);
        return ub + 1.0f + 1e-4f * (fabsf(caux) + s0_abs + k2 * chi);
    }
}

// S(ny) of aux_screen0_ub and the size of its terms (for the margin); +inf when no bound applies.
__device__ __forceinline__ float aux_screen0_s(float ny, float inv_gamma, float v_lo, float v_hi, float c, int D,
                                               float &s_abs) {
    const float a = fminf(fmaxf(ny * inv_gamma, v_lo), v_hi);
    const float tt = fmaxf(ny * __builtin_amdgcn_rcpf(a) - c, 0.0f);
    const float dl = (float)D * 0.693147180559945f * __builtin_amdgcn_logf(a);
    s_abs = fabsf(dl) + 0.5f * tt * tt;
    return (a > 0.0f) ? fmaf(-0.5f * tt, tt, -dl) : __builtin_inff();
}

// Level 2 of the screen from the words w1 of call 1: the further chi^2 terms it holds (uniforms 2, 3 and
// g_odd^2 for odd D - 1; exact chi2 for D <= 9) and their fp32 error.
template <int D>
__device__ __forceinline__ float aux_screen_chi1(const uint32_t (&w1)[4], float &err) {
    constexpr float kLn2 = 0.693147180559945f;
    constexpr int k = (D - 1) / 2;
    constexpr bool odd = ((D - 1) & 1) != 0;
    float chi = 0.0f;
    err = 0.0f;
    if constexpr (odd) {
        const float u0 = fmaf((float)w1[0], 0x1.0p-32f, 0x1.0p-33f);
        const float u1 = fmaf((float)w1[1], 0x1.0p-32f, 0x1.0p-33f);
        const float g = __builtin_amdgcn_sqrtf(-2.0f * kLn2 * __builtin_amdgcn_logf(u0)) * __builtin_amdgcn_cosf(u1);
        chi = g * g;
        err = fmaf(8e-3f, fabsf(g), 2e-5f) + 1e-4f * chi;
    }
    if constexpr (k >= 3) {
        float p = fmaf((float)w1[2], 0x1.0p-32f, 0x1.0p-33f);
        if constexpr (k >= 4) p *= fmaf((float)w1[3], 0x1.0p-32f, 0x1.0p-33f);
        const float c = -2.0f * kLn2 * __builtin_amdgcn_logf(p);
        chi += c;
        err += 1e-4f * c + 1e-6f;
    }
    return chi;
}

// call 0 / call 1 words of auxiliary m with its chi^2 prefixes in place (aux_chi_word): what the level-1 / level-2
// screens read; aux_core_w takes them as they are (combining a combined word again changes nothing)
template <int D, int M>
__device__ __forceinline__ void aux_words0(const uint32_t (&pre)[4], int m, uint32_t (&w)[4]) {
    if constexpr (D <= kPreMaxD) {
        w[2] = aux_chi_word(pre, w[2], m, 0, D, M);
        w[3] = aux_chi_word(pre, w[3], m, 1, D, M);
    }
}
template <int D, int M>
__device__ __forceinline__ void aux_words1(const uint32_t (&pre)[4], int m, uint32_t (&w1)[4]) {
    if constexpr (D <= kPreMaxD) w1[2] = aux_chi_word(pre, w1[2], m, 2, D, M);
}

template <int D, int PRIOR>
__device__ __forceinline__ double prior_aux_ll(const double *__restrict__ hyp, double ny, uint64_t seed, uint64_t ig,
                                               uint32_t t, int m, int M) {
    if constexpr (PRIOR == kPriorNiw)
        return niw_aux_ll<D>(hyp, ny, seed, ig, t, m);
    else
        return aux_ll<D>(hyp, ny, seed, ig, t, m, M);
}

// (v, mu) of a picked auxiliary: mu = mu0 + (|v|/sqrt kappa) L^T xi with xi from aux_xi.
template <int D>
__device__ __forceinline__ void aux_params(const double *__restrict__ hyp, const double (&y0)[D], double ny,
                                           uint64_t seed, uint64_t ig, uint32_t t, int m, int M, double *vmu) {
    using H = HypView<D>;
    double v, xpar, chi2, xi[D];
    aux_core<D>(seed, ig, t, m, M, hyp[H::kNu], v, xpar, chi2);
    aux_xi<D>(seed, ig, t, m, D, y0, ny, xpar, chi2, xi);
    const double sc = fabs(v) * hyp[H::kRsk];
    const double *LT = hyp + H::kLT;
    vmu[0] = v;
    int k = 0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double t0 = LT[k++] * xi[a];
#pragma unroll
        for (int b = a + 1; b < D; ++b) t0 = fma(LT[k++], xi[b], t0);
        vmu[1 + a] = fma(sc, t0, hyp[H::kMu0 + a]);
    }
}

template <int D>
__device__ __forceinline__ double norm_of(const double (&y0)[D]) {
    double n2 = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) n2 = fma(y0[a], y0[a], n2);
    return sqrt(n2);
}

// Scan position -> local item | visit << 32 (the visit is non-zero only for explicit orders).
// The pick's uniform (stream PICK, call 0) is drawn when a candidate first survives the skip rule: an
// item whose draw never leaves its own cluster does not need it (same value as drawing it up front).
// Wave-uniform branch: when any lane needs it, every lane without it draws it.
// (out of line: the Philox rounds would otherwise be inlined into every candidate loop, and their
// registers counted against the loops' live state)
__device__ __forceinline__ double pick_uniform(uint64_t seed, uint64_t ig, uint32_t t) {
    return uniform(seed, ig, t, kStreamPick, 0);
}

__device__ __forceinline__ void ensure_u(PickState &st, double lw, uint64_t seed, uint64_t ig, uint32_t t) {
    const bool need = st.u < 0.0 && lw - st.T > -kSkip;
    if (__ballot(need)) {
        if (st.u < 0.0) st.u = pick_uniform(seed, ig, t);
    }
}

// Own rows per wave up to which the lanes walk their rows' pruned lists group by group (np8_assign).
// (own rows per wave walked list by list: AssignArgs::max_groups, kMaxListGroups in np8_kernels.h)
// Own rows per wave whose row distances np8_assign_fast's walk screen stages (LDS: kScreenGroups x 64 floats).
constexpr int kScreenGroups = 4;

__device__ __forceinline__ int64_t position_to_local(const AssignArgs &A, int64_t p) {
    if (A.order) return A.order[p];
    if (A.use_perm) return (int64_t)perm_apply(A.perm, (uint32_t)p);
    return p;
}

// COUNT: the executed-work counters and the auxiliary screen's self-check (NP8_TIMING_COUNTERS), compiled
// into a separate instance so that the timed kernel carries none of their registers.
template <int D, int M, int PRIOR, bool COUNT>
#ifndef NP8_ASSIGN_WAVES
#define NP8_ASSIGN_WAVES 4
#endif
#ifndef NP8_ASSIGN_BLOCK
#define NP8_ASSIGN_BLOCK 64  // one wave per workgroup (256: 2% slower at C3)
#endif
#ifndef NP8_WALK_LDS
#define NP8_WALK_LDS 1  // np8_assign_fast's candidate walk broadcasts rows through LDS (0: v_readlane)
#endif
#if !NP8_WALK_LDS
#error "np8_assign_fast's walk screen stages its row distances beside the LDS rows"
#endif
#ifndef NP8_FAST_WAVES
#define NP8_FAST_WAVES 4  // 127 VGPRs, 30 dwords spilled on the rare paths (62 KB written per C3 launch); 5: 2-6% slower
#endif
#ifndef NP8_FAST_WAVES_LL
#define NP8_FAST_WAVES_LL NP8_FAST_WAVES  // the max-likelihood instance (every 5th sweep)
#endif
__device__ __forceinline__ void assign_item(const AssignArgs &A, const int64_t p, const int64_t qslot) {
    constexpr int DP = D * (D + 1) / 2;
    constexpr int CS = (D + DP + 5 + 1) & ~1;
    constexpr int F = D + DP;
    const bool sorted = A.sorted != 0;  // label-sorted layout: X and zs indexed by position
    // (ternaries, not A.zs[cur]: a runtime index into the argument struct would move it to scratch)
    constexpr int cur = 0;  // the label-sorted layout is always buffer 0 (buffer 1: the re-sort's scratch)
    int32_t *__restrict__ zs = cur ? A.zs[1] : A.zs[0];
    const int32_t *__restrict__ ids = cur ? A.ids[1] : A.ids[0];
    const int64_t lk = sorted ? (int64_t)ids[p] : position_to_local(A, p);
    const int64_t il = key_item(lk);
    const int64_t xr = sorted ? p : il;
    const uint64_t ig = (uint64_t)(A.offset + lk);  // item key: global index | visit << 32
    const double *__restrict__ X = sorted ? (cur ? A.Xs[1] : A.Xs[0]) : A.X;
    const double *__restrict__ cand = A.cand;
    const double *__restrict__ hyp = A.hyp;

    const uint32_t t = A.ctl->t_base + A.t;
    double x[D];
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = X[(int64_t)a * A.n_loc + xr];
    const int32_t zi = sorted ? zs[p] : A.z[il];

    // The item's own cluster enters the draw first (weight n_k - 1): its log-weight is a lower bound
    // of the final maximum, so every later candidate more than kSkip below it is skipped.
    // the own row: a scalar load when the wave's items share their slot (the label-sorted layout)
    const int32_t zf = __builtin_amdgcn_readfirstlane(zi);
    const int32_t jo = (__ballot(zi != zf) == 0ull) ? A.dense_of[zf] : A.dense_of[zi];
    PickState st;
    {
        // one pass per distinct own row of the wave (one in the label-sorted layout), the row read with
        // scalar loads: a per-lane row would hold all D + D(D+1)/2 of its doubles in vector registers
        uint64_t pend = __ballot(1);
        while (pend) {
            const int32_t j = __builtin_amdgcn_readlane(jo, __ffsll((unsigned long long)pend) - 1);
            const double *eo = cand + (int64_t)j * CS;
            const double lw = cand_ll<D>(eo, x) + eo[F + kFieldLogn1];
            if (jo == j) st.T = lw;
            pend &= ~__ballot(jo == j);
        }
        st.S = 1.0;
        st.u = -1.0;  // drawn when a candidate first survives the skip rule (ensure_u)
        st.pick = jo;
    }
    const double zslot = (double)zi;
    const int K = A.ctl->K;
    // with candidate lists (np8_prune), the lanes of each distinct own row of the wave walk that row's
    // pruned list (one group in the label-sorted layout, two or three at cluster boundaries): the rows
    // left out are those every such lane's pick_step skips anyway, and the order is ascending as in the
    // full walk.  Lists hold for every item of the row, whatever its wave (np8_prune: the radius covers
    // each item the last sweep left in the row).
    int32_t nq_lane = 0, niso_lane = 0, nlist_lane = 0;  // COUNT: quadratic forms this lane evaluated, list entries
    int32_t npick_lane = 0;  // COUNT: walked rows within kSkip of the running maximum (pick_step's exp and division)
    int32_t pslot = zi;                  // slot of the picked row (no reload of the row at the end)
    // (a wave of many own rows -- a stale layout, a cold start -- walks the table once instead)
    int ngroups = 0;
    for (uint64_t pend = __ballot(1); pend && ngroups <= A.max_groups; ++ngroups)
        pend &= ~__ballot(jo == __builtin_amdgcn_readlane(jo, __ffsll((unsigned long long)pend) - 1));
    bool full = true;  // this lane walks the whole table
    if (A.use_lists && A.ctl->lists_ok && ngroups <= A.max_groups) {
        uint64_t pend = __ballot(1);
        while (pend) {
            const int32_t j0 = __builtin_amdgcn_readlane(jo, __ffsll((unsigned long long)pend) - 1);
            pend &= ~__ballot(jo == j0);
            if (jo == j0) {
                // the list holds for items within the radius it was built for: a lane outside it (an item
                // that arrived since the radii were gathered) walks the whole table below
                const double *e0 = cand + (int64_t)j0 * CS;
                double d2 = 0.0;
#pragma unroll
                for (int a = 0; a < D; ++a) {
                    const double dd = x[a] - e0[a];
                    d2 = fma(dd, dd, d2);
                }
                full = !(d2 <= A.plr2[j0]);
                if (!full) {
#ifdef NP8_EXP_NO_WALK
                    const int32_t nl = COUNT ? A.plen[j0] : 0;
#else
                    const int32_t nl = A.plen[j0];
#endif
                    const int32_t *__restrict__ lst = A.plist + (int64_t)j0 * A.ls;
                    for (int q = 0; q < nl; ++q) {
                        const int j = lst[q];  // uniform across the group: scalar loads
                        const double *e = cand + (int64_t)j * CS;
                        const double lw = cand_ll<D>(e, x) + e[F + kFieldLogn];
#ifdef NP8_EXP_SKIPCOUNT  // (experiment: pick_evals counts the listed rows no walking lane of the group needs,
                          //  iso counts the group's listed rows, once per group)
                        if constexpr (COUNT) {
                            const uint64_t bn = __ballot(lw - st.T > -kSkip - 2.0);
                            const bool lead = (threadIdx.x & 63) == (__ffsll((unsigned long long)__ballot(1)) - 1);
                            npick_lane += (lead && bn == 0ull) ? 1 : 0;
                            niso_lane += lead ? 1 : 0;
                        }
#else
                        if constexpr (COUNT) npick_lane += (lw - st.T > -kSkip) ? 1 : 0;
#endif
                        ensure_u(st, lw, A.seed, ig, t);
                        pick_step(st, lw, j);
                        pslot = (st.pick == j) ? (int32_t)e[F + kFieldSlot] : pslot;
                        if constexpr (COUNT) {
                            nq_lane += 1;
                            nlist_lane += 1;
#ifndef NP8_EXP_SKIPCOUNT
                            niso_lane += (e[F + kFieldIso] > 0.0) ? 1 : 0;
#endif
                        }
                    }
                }
            }
        }
    }
    if constexpr (COUNT) {  // how the walk went (lanes on the whole table, waves paying the table loop)
        const uint64_t fb = __ballot(full);
        const int64_t nl_w = [&] {
            int64_t t = 0;
            for (uint64_t act = __ballot(1); act; act &= act - 1ull) t += __builtin_amdgcn_readlane(nlist_lane, __ffsll((unsigned long long)act) - 1);
            return t;
        }();
        if ((threadIdx.x & 63) == (__ffsll((unsigned long long)__ballot(1)) - 1)) {
            const int64_t w = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % kEvalSlots;
            unsigned long long *ec = A.evalc + 4 * kEvalSlots + 2 * w;
            atomicAdd(ec, (unsigned long long)__popcll(fb));
            atomicAdd(ec + 1, fb ? 1ull : 0ull);
            atomicAdd(ec + 2 * kEvalSlots, (ngroups > A.max_groups) ? 1ull : 0ull);
            atomicAdd(ec + 2 * kEvalSlots + 1, (unsigned long long)nl_w);
        }
    }
    if (full) {  // wave-uniform row loop (scalar loads) over the lanes that need it
        for (int j = 0; j < K; ++j) {
            const double *e = cand + (int64_t)j * CS;
            const double lw = cand_ll<D>(e, x) + e[F + kFieldLogn];
            if (e[F + kFieldSlot] != zslot) {
                if constexpr (COUNT) npick_lane += (lw - st.T > -kSkip) ? 1 : 0;
                ensure_u(st, lw, A.seed, ig, t);
                pick_step(st, lw, j);
                pslot = (st.pick == j) ? (int32_t)e[F + kFieldSlot] : pslot;
            }
            if constexpr (COUNT) {
                nq_lane += 1;
                niso_lane += (e[F + kFieldIso] > 0.0) ? 1 : 0;
            }
        }
    }
    if constexpr (COUNT) {  // the quadratic forms this wave executed (own row + walked rows)
        nq_lane += 1;
        niso_lane += (cand[(int64_t)jo * CS + F + kFieldIso] > 0.0) ? 1 : 0;
        int64_t nq = 0, niso = 0, npk = 0;
        const uint64_t lanes = __ballot(1);
        for (uint64_t act = lanes; act; act &= act - 1ull) {  // sums over the active lanes
            const int l = __ffsll((unsigned long long)act) - 1;
            nq += __builtin_amdgcn_readlane(nq_lane, l);
            niso += __builtin_amdgcn_readlane(niso_lane, l);
            npk += __builtin_amdgcn_readlane(npick_lane, l);
        }
        if ((threadIdx.x & 63) == (__ffsll((unsigned long long)lanes) - 1)) {
            unsigned long long *ec = A.evalc + 2 * ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % kEvalSlots);
            atomicAdd(ec, (unsigned long long)nq);
            atomicAdd(ec + 1, (unsigned long long)niso);
            atomicAdd(ec + 8 * kEvalSlots, (unsigned long long)npk);
        }
    }
    double ny;
    {
        double y0[D];
        whiten<D>(hyp, x, y0);
        ny = norm_of<D>(y0);
    }
    {
        const double logam = hyp[HypView<D>::kLogam];
        if constexpr (PRIOR == kPriorNiw) {
#pragma unroll 1
            for (int m = 0; m < M; ++m) {  // screened: T only grows, so a bound below T - kSkip now stays so
                using H = HypView<D>;
                const double lw = niw_aux_ll_screened(A.seed, ig, t, m, D, hyp[H::kNu], ny, hyp[H::kRsk], hyp[H::kCaux],
                                                      hyp[H::kSmax], st.T - kSkip - logam) + logam;
                ensure_u(st, lw, A.seed, ig, t);
                pick_step(st, lw, K + m);
            }
        } else {
            // the first Philox call of every auxiliary bounds its log-likelihood (aux_screen_ub); lanes
            // it cannot rule out take call 1 (level 2), and only the lanes still left finish the fp64
            // draw -- those whose auxiliary may come within kSkip of the running maximum
            using H = HypView<D>;
            const double nu = hyp[H::kNu], rsk = hyp[H::kRsk], caux = hyp[H::kCaux];
            const float thr = (float)(st.T - kSkip - logam);  // T only grows: conservative for every m
            const float nyf = (float)ny, nuf = (float)nu, rskf = (float)rsk, cauxf = (float)caux;
            constexpr int Qa = (1 + ((((D - 1) & 1) || (D - 1) / 2 > 2) ? 1 : 0) + ((D - 1) / 2 > 4 ? ((D - 1) / 2 - 1) / 4 : 0));
            constexpr bool has_call1 = Qa > 1;
            // level 1 for every auxiliary at once (M independent Philox chains): a bit per auxiliary the
            // screen cannot rule out
            uint32_t need = 0u;
            uint32_t pre[4] = {0u, 0u, 0u, 0u};
            if constexpr (D <= kPreMaxD && (D - 1) / 2 >= 1) aux_pre_call(A.seed, ig, t, pre);
#ifdef NP8_EXP_UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
            for (int m = 0; m < M; ++m) {
#ifdef NP8_EXP_NO_AUX
                if (!COUNT) break;
#endif
                uint32_t w[4];
                philox_call(A.seed, ig, t, kStreamAux, (uint32_t)(m * Qa), w);
                aux_words0<D, M>(pre, m, w);
                if (!(aux_screen_ub<D>(w, 0.0f, 0.0f, nyf, nuf, rskf, cauxf, thr) <= thr)) need |= 1u << m;
            }
            int64_t n_viol = 0, n_ex_lane = 0, n_ex_wave = 0;
#pragma unroll 1
            for (int m = 0; m < M; ++m) {
                bool skip = ((need >> m) & 1u) == 0u;
                if (!COUNT && __ballot(!skip) == 0ull) continue;  // wave-uniform: the common case
#ifdef NP8_EXP_NO_EXACT
                if (!COUNT) continue;
#endif
                uint32_t w0[4], w1[4] = {0u, 0u, 0u, 0u};
                philox_call(A.seed, ig, t, kStreamAux, (uint32_t)(m * Qa), w0);
                aux_words0<D, M>(pre, m, w0);
                const bool l2 = has_call1 && !skip;
                if (l2) {  // level 2: the chi^2 terms of call 1
                    philox_call(A.seed, ig, t, kStreamAux, (uint32_t)(m * Qa + 1), w1);
                    aux_words1<D, M>(pre, m, w1);
                    float e1;
                    const float c1 = aux_screen_chi1<D>(w1, e1);
                    skip = aux_screen_ub<D>(w0, c1, e1, nyf, nuf, rskf, cauxf, thr) <= thr;
                }
                if constexpr (COUNT) {
                    const uint64_t b = __ballot(!skip);
                    n_ex_lane += __popcll(b);
                    n_ex_wave += (b != 0ull) ? 1 : 0;
                }
                if (!skip || COUNT) {
                    double v, xpar, chi2;
                    aux_core_w<D>(A.seed, ig, t, m, nu, v, xpar, chi2, w0, l2, w1, pre, M);
                    const double lw = aux_loglik(ny, v, xpar, chi2, D, rsk, caux) + logam;
                    if (!skip) {
                        ensure_u(st, lw, A.seed, ig, t);
                        pick_step(st, lw, K + m);
                    } else if (lw - st.T > -kSkip) {
                        ++n_viol;  // debug count: a screened auxiliary pick_step would not have skipped
                    }
                }
            }
            if constexpr (COUNT) {
                const int nv = __popcll(__ballot(n_viol > 0));
                if ((threadIdx.x & 63) == (__ffsll((unsigned long long)__ballot(1)) - 1)) {
                    if (nv) atomicAdd(&A.ctl->n_screen_viol, (unsigned long long)nv);
                    unsigned long long *ec = A.evalc + 2 * kEvalSlots +
                                             2 * ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % kEvalSlots);
                    atomicAdd(ec, (unsigned long long)n_ex_lane);
                    atomicAdd(ec + 1, (unsigned long long)n_ex_wave);
                }
            }
        }
    }

    int32_t *delta = reinterpret_cast<int32_t *>(A.rec + kRecHeaderBytes);
    const int32_t snew = (st.pick < K) ? pslot : -1;
#ifdef NP8_EXP_NO_R2
    if (A.collect_r2 && COUNT) {
#else
    if (A.collect_r2) {
#endif
        // radius of the item's cluster for the next sweep's lists: its distance to the mean of the row
        // it joins (an item that asked for a new cluster counts for its old one, in case the request
        // is rejected; the new slot's radius is set to +inf by np8_finalize)
        const int32_t tr = (st.pick < K) ? st.pick : jo;
        const int32_t ts = (st.pick < K) ? snew : zi;
        const double *e = cand + (int64_t)tr * CS;
        double d2 = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const double dd = x[a] - e[a];
            d2 = fma(dd, dd, d2);
        }
        const int32_t t0 = __builtin_amdgcn_readfirstlane(ts);
        // full wave, one slot (queue mode: the wave's record belongs to np8_assign_fast, lanes go one by one)
        const bool one = !A.queue && __ballot(1) == ~0ull && __ballot(ts != t0) == 0;
        if (one) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) d2 = fmax(d2, __shfl_xor(d2, o));
        } else {
            wave_max_by_key(reinterpret_cast<unsigned long long *>(A.r2 + A.kcap), ts, d2, true);
        }
        if (!A.queue && (threadIdx.x & 63) == (__ffsll((unsigned long long)__ballot(1)) - 1)) {  // the wave's record
            WaveR2 w;
            w.d2 = one ? d2 : 0.0;
            w.slot = one ? t0 : -1;
            w.pad = 0;
            A.wr2[(p - A.p0) >> 6] = w;
        }
    }
    // items leaving their cluster, counted per wave (drives the re-sort of the layout)
    const uint64_t mv = __ballot(snew != zi);
#ifdef NP8_EXP_NO_MOVED
    if (COUNT)
#endif
    if (mv && (threadIdx.x & 63) == (__ffsll((unsigned long long)__ballot(1)) - 1))
        atomicAdd(reinterpret_cast<unsigned long long *>(&A.ctl->moved), (unsigned long long)__popcll(mv));
    const bool mover = st.pick < K && snew != zi;
    wave_add_by_key(delta, zi, -1, mover);
    wave_add_by_key(delta, snew, 1, mover);
    const int qreq = wave_append(A.nreq, st.pick >= K);  // (requests are accepted by scan position, not arrival)
    if (st.pick < K) {
        const int32_t s = snew;
        if (s != zi) {
            // the item's addresses again (a rare path): two 64-bit addresses kept live through the draw were
            // spilled to scratch for every item (19 of the 38 MB the C3 launch wrote)
            int64_t pq = A.queue ? qslot : (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
            asm volatile("" : "+v"(pq));
            pq = A.queue ? (int64_t)A.queue[pq] : A.p0 + pq;
            const int64_t lq = sorted ? (int64_t)__atomic_load_n(ids + pq, __ATOMIC_RELAXED) : position_to_local(A, pq);
            A.z[key_item(lq)] = s;
            if (sorted) zs[pq] = s;
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
            double *vmu = A.vmu + (int64_t)q * (D + 1);
            double y0[D];  // the item's frame again (not kept live through the draw: registers)
            whiten<D>(hyp, x, y0);
            if constexpr (PRIOR == kPriorNiw) {  // the item's frame; np8_niw_aux_slots builds the slot
                vmu[0] = ny;
#pragma unroll
                for (int a = 0; a < D; ++a) vmu[1 + a] = y0[a];
            } else {
                aux_params<D>(hyp, y0, ny, A.seed, ig, t, st.pick - K, M, vmu);
            }
        }
    }
}

// One lane per item of [p0, p1).
template <int D, int M, int PRIOR, bool COUNT>
__global__ __launch_bounds__(NP8_ASSIGN_BLOCK) __attribute__((amdgpu_waves_per_eu(NP8_ASSIGN_WAVES))) void np8_assign(AssignArgs A) {
    const int64_t p = A.p0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < A.p1) assign_item<D, M, PRIOR, COUNT>(A, p, -1);
}

// The lanes np8_assign_fast deferred: fast-kernel wave qlist[k] left qcount of them at queue[64 wave ..]; the
// grid walks the listed waves (the deferred lanes of one fast wave share its rows).  Rarely has work, so it
// takes the registers it wants (no spills) at fewer waves per SIMD.
template <int D, int M, int PRIOR, bool COUNT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void np8_assign_queue(AssignArgs A) {
    static_assert(NP8_ASSIGN_BLOCK == 64, "np8_assign_fast's waves are its workgroups");
    const int lane = threadIdx.x & 63;
    const int nw = (int)A.ctl->qwaves;
    for (int k = blockIdx.x; k < nw; k += gridDim.x) {
        const int64_t wv = A.qlist[k];
        const int cnt = A.qcount[wv];
        if (lane < cnt) assign_item<D, M, PRIOR, COUNT>(A, (int64_t)A.queue[wv * 64 + lane], wv * 64 + lane);
    }
}

// ---- experiment: per-wave phase timestamps of np8_assign_fast (built only with NP8_EXP_CLOCKS) -------
#ifdef NP8_EXP_CLOCKS
constexpr int64_t kClkWaves = 1 << 16;
__device__ unsigned long long g_np8_clk[kClkWaves * 8];
// every load issued so far has landed, then the 100 MHz real-time clock (10 ns)
#define NP8_CLK(k)                                                                                     \
    do {                                                                                               \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                    \
        const int64_t w_ = (p - A.p0) >> 6;                                                            \
        if (!COUNT && (threadIdx.x & 63) == 0 && w_ < kClkWaves)                                       \
            g_np8_clk[w_ * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                                \
    } while (0)
// slot 7: the wave's walk shape (own-row passes | list groups << 8 | table walk << 16 | listed rows walked << 20)
#define NP8_CLK_INFO(v)                                                                                \
    do {                                                                                               \
        const int64_t w_ = (p - A.p0) >> 6;                                                            \
        if (!COUNT && (threadIdx.x & 63) == 0 && w_ < kClkWaves) g_np8_clk[w_ * 8 + 7] = (v);          \
    } while (0)
#define NP8_CLK_ON 1
extern "C" int np8_exp_clocks(unsigned long long *out, int64_t n) {
    if (n > kClkWaves * 8) n = kClkWaves * 8;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_np8_clk), sizeof(unsigned long long) * n, 0, hipMemcpyDeviceToHost) ==
                   hipSuccess ? 0 : -1;
}
#else
#define NP8_CLK(k)
#define NP8_CLK_INFO(v)
#define NP8_CLK_ON 0
#endif

// ---- the data-parallel sweep's fast path -------------------------------------------------------------
// lane l's double (l wave-uniform), as two readlanes: an SGPR pair for the rest of the wave
[[maybe_unused]] __device__ __forceinline__ double readlane_d(double v, int l) {
    const int64_t b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFFll), l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}

// Fx through a lane shuffle / readlane (four 32-bit pieces)
__device__ __forceinline__ Fx fx_shfl_xor(Fx a, int o) {
    const uint32_t l0 = (uint32_t)__shfl_xor((int)(uint32_t)a.lo, o), l1 = (uint32_t)__shfl_xor((int)(uint32_t)(a.lo >> 32), o);
    const uint32_t h0 = (uint32_t)__shfl_xor((int)(uint32_t)(uint64_t)a.hi, o),
                   h1 = (uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)a.hi >> 32), o);
    Fx r;
    r.lo = ((uint64_t)l1 << 32) | l0;
    r.hi = (int64_t)(((uint64_t)h1 << 32) | h0);
    return r;
}

__device__ __forceinline__ Fx fx_readlane(Fx a, int l) {
    Fx r;
    r.lo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a.lo >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a.lo, l);
    r.hi = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)a.hi >> 32), l) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)a.hi, l));
    return r;
}

// np8_assign_fast<D,M>: the common case of np8_assign -- the reference prior with an isotropic Lambda (every
// G0 draw, and so every row, isotropic; the base measure's whitening diagonal), the label-sorted layout --
// with only the work almost every lane needs: the own row, the candidate list (or the table), the two
// levels of the auxiliary screen, the exact fp64 draw for the auxiliaries the screen cannot clear (an auxiliary
// may come within kSkip of the running maximum: 0.3% of (item, auxiliary) pairs at C3), the move and the
// new-cluster request with its payload.  Only a lane whose own row or a walked row is not isotropic is deferred:
// its position goes to a queue that np8_assign then runs in queue mode, from the start, with the full code.  A
// deferred lane writes nothing here, so every item's result is np8_assign's, bit for bit; when every live row is
// isotropic the host leaves the queue launch out (AssignArgs::no_queue; a deferred lane would set kErrQueue).
// LL: a max-likelihood check sweep with the sum folded in (AssignArgs::ll_on): each wave also stores the sum of its
// items' log-likelihoods under their new labels -- the values np8_loglik would compute after the step, operation for
// operation (the walk's quadratic forms are the table form's isotropic one) -- in a separate instance, so that the
// other sweeps carry none of its registers.
// A field of np8_assign_fast's argument (the kernel's only explicit argument: offset 0 of the kernarg segment) read where
// it is used: a scalar load behind an empty asm barrier on the segment pointer, so that it is neither hoisted into the
// entry block nor held (and spilled to VGPR lanes, a v_writelane/v_readlane pair each) across the kernel
#ifdef NP8_EXP_EARLY_ARGS  // (A/B: the compiler's own placement)
#define NP8_LATE(f) (A.f)
#else
#define NP8_LATE(f) np8_late_arg<decltype(AssignArgs::f)>(offsetof(AssignArgs, f))
#endif

template <int D, int M, int PRIOR, bool COUNT, bool LL>
__global__ __launch_bounds__(NP8_ASSIGN_BLOCK) __attribute__((amdgpu_waves_per_eu(LL ? NP8_FAST_WAVES_LL : NP8_FAST_WAVES))) void np8_assign_fast(AssignArgs A) {
    using H = HypView<D>;
    constexpr int DP = D * (D + 1) / 2;
    constexpr int CS = (D + DP + 5 + 1) & ~1;
    constexpr int F = D + DP;
    const int64_t p = A.p0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= A.p1) return;
    NP8_CLK(0);
    const int lane = threadIdx.x & 63;
    // the label-sorted layout is always buffer 0 (np8_sort_copyback): no load in front of the item loads
    int32_t *__restrict__ zs = A.zs[0];
    const int32_t *__restrict__ ids = A.ids[0];
    const double *__restrict__ X = A.Xs[0];
    const double *__restrict__ cand = A.cand;
    const double *__restrict__ hyp = A.hyp;
    const int32_t zi = (int32_t)NP8_CHK(zs[p], 0, A.kcap);
    const int32_t il = (int32_t)NP8_CHK(ids[p], 0, A.n_loc);
    const uint64_t ig = (uint64_t)(A.offset + il);
    const uint32_t t = A.ctl->t_base + A.t;
    double x[D];
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = X[(int64_t)a * A.n_loc + p];
    const int K = A.ctl->K;
    const int lists_ok = A.ctl->lists_ok;  // (the same round of scalar loads)
    if (A.compact && A.ctl->halt) return;  // a compact sweep graph halted at an earlier step: nothing until resolved
    // a max-likelihood snapshot the last check left pending: the labelling before this step is the one it keeps
    // (copied in position order -- coalesced; np8_best_unsort puts it in item order before a re-sort or a read)
    const int snap = (!LL && A.snap_on) ? A.ctl->snap_pend : 0;
    if (snap) {
        A.z_best[p] = zi;
        if (p == A.p0) A.ctl->best_sorted = 1;
    }
    NP8_CLK(1);
    bool defer = COUNT;  // counting runs: every lane takes np8_assign's counting instance
    [[maybe_unused]] unsigned long long clk_own = 1, clk_rows = 0;  // (NP8_EXP_CLOCKS: the walk's shape)
    PickState st;
    st.S = 1.0;
    st.u = -1.0;
    st.T = 0.0;
    double d2own = 0.0;  // |x - mu_own|^2: the own row's quadratic form and the list's radius check
    double ll_own = 0.0, llp = 0.0;  // (LL) ll under the own row and under the row picked so far
    int32_t jo = 0, nlist = 0;
    double r2list = 0.0;
    int32_t pslot = zi;
    // the wave's first own slot (usually its only one in the label-sorted layout): its row's scalars are requested
    // first, so that the auxiliaries' level-1 screen below runs while they are in flight
    // (read-only in this kernel: restrict lets the wave-uniform reads go through the scalar cache)
    const double *__restrict__ slot_mu = A.slot_mu, *__restrict__ slot_iso = A.slot_iso, *__restrict__ slot_c = A.slot_c,
                               *__restrict__ slot_logn1 = A.slot_logn1, *__restrict__ plr2_s = A.plr2_s;
    const int32_t *__restrict__ dense_of = A.dense_of, *__restrict__ plen_s = A.plen_s;
    const int32_t s_1 = __builtin_amdgcn_readfirstlane(zi);
    double mo_1[D];
#pragma unroll
    for (int a = 0; a < D; ++a) mo_1[a] = slot_mu[(int64_t)s_1 * D + a];
    const double iso_1 = slot_iso[s_1], cs_1 = slot_c[s_1], l1_1 = slot_logn1[s_1];
    const int32_t js_1 = dense_of[s_1], pl_1 = plen_s[s_1];
    const double pr_1 = plr2_s[s_1];
    // level 0 of the auxiliary screen while the own row's loads are in flight: every auxiliary's bound from the item's
    // prefix call (aux_screen0_ub), without the threshold (the running maximum), which is compared below.  |y0|^2 in
    // fp64 (its root in fp64 only where an auxiliary is drawn exactly, fp32 for the bounds)
    // (D > kPreMaxD: no prefixes; every auxiliary's bound from its call 0 up front, the round-5 form of the screen)
    constexpr bool kL0 = D <= kPreMaxD && (D - 1) / 2 >= 1;
    double n2 = 0.0;
    {
        const double *U = hyp + H::kUdiag;  // diagonal (launch condition): whiten() + norm_of() with zeros left out
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const double y = U[a] * (x[a] - hyp[H::kMu0 + a]);
            n2 = fma(y, y, n2);
        }
    }
    [[maybe_unused]] double ny = 0.0;
    [[maybe_unused]] float nyf = 0.0f;
    if constexpr (kL0)
        nyf = __builtin_amdgcn_sqrtf((float)n2);
    else
        ny = sqrt(n2);
    constexpr int Qa = (1 + ((((D - 1) & 1) || (D - 1) / 2 > 2) ? 1 : 0) + ((D - 1) / 2 > 4 ? ((D - 1) / 2 - 1) / 4 : 0));
    [[maybe_unused]] uint32_t pre[4];
    float ub0[M];
    if (!COUNT) {
        if constexpr (kL0) {
            aux_pre_call(A.seed, ig, t, pre);
            float s_abs;
            const float s0 = aux_screen0_s(nyf, (float)hyp[H::kPre], (float)hyp[H::kPre + 1], (float)hyp[H::kPre + 2],
                                           (float)hyp[H::kPre + 3], D, s_abs);
            const float rskf = (float)hyp[H::kRsk], cauxf = (float)hyp[H::kCaux];
#pragma unroll
            for (int m = 0; m < M; ++m) {
#ifdef NP8_EXP_NOAUXSCREEN  // (ablation timing only: no auxiliary is ever evaluated -- not the chain)
                ub0[m] = -__builtin_inff() + 0.0f * nyf;
#else
                ub0[m] = aux_screen0_ub<D, M>(pre, m, s0, s_abs, cauxf, 0.5f * rskf * rskf);
#endif
                asm volatile("" ::"v"(ub0[m]));  // computed here, while the own row's loads are in flight (not sunk)
            }
        } else {
            const float nyf1 = (float)ny, nuf = (float)hyp[H::kNu], rskf = (float)hyp[H::kRsk],
                        cauxf = (float)hyp[H::kCaux];
#pragma unroll
            for (int m = 0; m < M; ++m) {
                uint32_t w[4];
                philox_call(A.seed, ig, t, kStreamAux, (uint32_t)(m * Qa), w);
                ub0[m] = aux_screen_ub<D>(w, 0.0f, 0.0f, nyf1, nuf, rskf, cauxf, 0.0f, false);
                asm volatile("" ::"v"(ub0[m]));  // computed here, while the own row's loads are in flight (not sunk)
            }
        }
    }
    {
        // one pass per distinct own slot of the wave (one in the label-sorted layout); everything about the
        // own row is read by slot in one round of scalar loads: the parameters from the slot tables (the
        // candidate rows copy them), log(n - 1), the dense row and its candidate list's length and radius
        auto own = [&](int32_t s, const double (&mo)[D], double iso, double cs, double l1, int32_t js, int32_t pl,
                       double pr) {
            if (zi == s) {
                jo = js;
                nlist = pl;
                r2list = pr;
                if (iso > 0.0) {  // cand_ll's isotropic form, operation for operation
                    double s2 = (x[0] - mo[0]) * (x[0] - mo[0]);
#pragma unroll
                    for (int a = 1; a < D; ++a) s2 = fma(x[a] - mo[a], x[a] - mo[a], s2);
                    d2own = s2;
                    ll_own = fma(-0.5, s2 * iso, cs);
                    st.T = ll_own + l1;
                } else {
                    defer = true;
                }
            }
        };
        own(s_1, mo_1, iso_1, cs_1, l1_1, js_1, pl_1, pr_1);  // the first group, from the loads issued above
        // waves of several own slots (a layout gone stale between re-sorts, the range's edges): the other lanes gather
        // their rows' fields with vector loads, one round trip whatever the number of slots (a scalar round per slot
        // cost a stale wave ~2 us each)
        if (__ballot(zi != s_1)) {
            if (NP8_CLK_ON) clk_own = 1 + __popcll(__ballot(zi != s_1));
            if (zi != s_1) {
                double mo[D];
#pragma unroll
                for (int a = 0; a < D; ++a) mo[a] = slot_mu[(int64_t)zi * D + a];
                own(zi, mo, slot_iso[zi], slot_c[zi], slot_logn1[zi], (int32_t)NP8_CHK(dense_of[zi], 0, A.ctl->K),
                    plen_s[zi], plr2_s[zi]);
            }
        }
    }
    if (COUNT) defer = true;
    st.pick = jo;
    llp = ll_own;
    NP8_CLK(2);
    const double zslot = (double)zi;
    int ngroups = 0;
    for (uint64_t pend = __ballot(1); pend && ngroups <= A.max_groups; ++ngroups)
        pend &= ~__ballot(jo == __builtin_amdgcn_readlane(jo, __ffsll((unsigned long long)pend) - 1));
    bool full = !defer;  // this lane walks the whole table
    // rows row_of(0 .. n-1) (wave-uniform), for the lanes with `mine`: a wave's worth of rows per round of loads
    // (lane q: row q's fields, the wave's active lanes are 0 .. nact - 1 -- the last wave of the range is
    // partial), then broadcast row by row: no dependent load per row (the mixed regime walks ~9 rows per item,
    // a stale wave the whole table).  A row that is not isotropic defers the lane (np8_assign takes it).
    __shared__ float s_dist[kScreenGroups][64];  // the walk screen's row distances (below), per staged own row
#if NP8_WALK_LDS
    // the round's rows staged in LDS ([field][row], one-wave workgroups) and read back at a wave-uniform address
    // (a broadcast on the LDS pipe) instead of 2 v_readlane per double on the VALU
    static_assert(NP8_ASSIGN_BLOCK == 64, "the walk's LDS rows are per wave");
    __shared__ double s_row[D + 4][64];
    __shared__ int32_t s_j[64];
#define NP8_ROWF(v, f, k) s_row[f][k]
#define NP8_ROWJ(k) s_j[k]
#else
#define NP8_ROWF(v, f, k) readlane_d(v, k)
#define NP8_ROWJ(k) __builtin_amdgcn_readlane(jq, k)
#endif
    // The screen (AssignArgs::walk_screen): row j is left out for the wave when for every walking lane
    //   lw_j(x) = c_j + log n_j - iso_j |x - mu_j|^2 / 2 <= c_j + log n_j - iso_j gap^2 / 2,
    //   gap = max(|mu_j - mu_own| - |x - mu_own|, |x - mu_own| - |mu_j - mu_own|, 0)  (triangle inequality)
    // lies below the lane's running maximum T by kSkip + 2 nats (plus 1e-9 of the terms): the row's pick_step would
    // return at once and ensure_u draw nothing for every lane -- the row changes no result.  |mu_j - mu_own| comes
    // from the lists' build (pdist, every pair of dense rows, rounded down; 2^-21 relative up for the upper side),
    // staged per round for the first kScreenGroups own rows among the walking lanes (a list walk has one, a table walk
    // of a wave with several labels several); lanes of further own rows take gap = 0.  Valid while the lists are (the
    // same table).  Cost per row: the bound instead of the quadratic form and the pick.
    const bool screen = A.walk_screen != 0 && A.pdist != nullptr && A.use_lists && lists_ok;
    auto walk = [&](auto row_of, int n, bool mine, bool own_skip) {
        if (n <= 0) return;  // (wave-uniform: the warm state's lists are empty -- none of the set-up below)
        // the walking lanes' own rows (wave-uniform, first kScreenGroups) and this lane's index among them
        int32_t gid[kScreenGroups];
        int ng = 0, gi = -1;
        const double d_own = screen ? sqrt(d2own) : 0.0;
        if (screen) {
            uint64_t pg = __ballot(mine && !defer);
            for (; pg && ng < kScreenGroups; ++ng) {
                gid[ng] = __builtin_amdgcn_readlane(jo, __ffsll((unsigned long long)pg) - 1);
                if (jo == gid[ng]) gi = ng;
                pg &= ~__ballot(jo == gid[ng]);
            }
        }
        const int nact = __popcll(__ballot(1));
        for (int qb = 0; qb < n; qb += nact) {
            const int q = qb + lane;
            int32_t jq = 0;
            double fm[D], fiso = 0.0, fc = 0.0, fl = 0.0, fsl = 0.0;
            float fdist[kScreenGroups];
#pragma unroll
            for (int g = 0; g < kScreenGroups; ++g) fdist[g] = 0.0f;
#pragma unroll
            for (int a = 0; a < D; ++a) fm[a] = 0.0;
            if (q < n) {
                jq = row_of(q);
#pragma unroll
                for (int g = 0; g < kScreenGroups; ++g)
                    if (g < ng) fdist[g] = A.pdist[NP8_CHK((int64_t)gid[g] * A.ls + jq, 0, (int64_t)A.kcap * A.ls)];
                const double *e = cand + (int64_t)NP8_CHK(jq, 0, K) * CS;
#pragma unroll
                for (int a = 0; a < D; ++a) fm[a] = e[a];
                fiso = e[F + kFieldIso];
                fc = e[F + kFieldC];
                fl = e[F + kFieldLogn];
                fsl = e[F + kFieldSlot];
            }
#if NP8_WALK_LDS
            __syncthreads();  // (one wave) the previous round's reads are done
#pragma unroll
            for (int a = 0; a < D; ++a) s_row[a][lane] = fm[a];
            s_row[D][lane] = fiso;
            s_row[D + 1][lane] = fc;
            s_row[D + 2][lane] = fl;
            s_row[D + 3][lane] = fsl;
            s_j[lane] = jq;
#pragma unroll
            for (int g = 0; g < kScreenGroups; ++g) s_dist[g][lane] = fdist[g];
            __syncthreads();
#endif
            const int nb = min(nact, n - qb);
#if NP8_WALK_LDS && !defined(NP8_EXP_INLINE_PICK)
            // Two passes over the round's rows.  Pass 1 (every row): the quadratic form, and the rows the lane's
            // pick_step would not skip -- lw - T > -kSkip with T the running maximum, which only such rows raise --
            // appended to a per-lane buffer (ll, row index in the round).  Pass 2 (flush: a full buffer, the round's
            // end): pick_step over each lane's buffered rows in order.  The same steps on the same values as one
            // pass, but the wave runs the pick's exp and division for max-over-lanes of the buffered rows instead of
            // for every row that some lane needs (the mixed regime: ~19 listed rows per wave, ~1.35 picked per item).
            constexpr int kBuf = 4;
            double bl[kBuf];
            int bk[kBuf];
            int nbuf = 0;
            double Tc = st.T;  // the running maximum pick_step will have reached at this row
            auto flush = [&]() {
#pragma unroll
                for (int e = 0; e < kBuf; ++e) {
                    if (__ballot(e < nbuf) == 0ull) break;  // (wave-uniform)
                    if (e < nbuf) {
                        const double llj = bl[e];
                        const int kk = bk[e];
                        const double lw = llj + s_row[D + 2][kk];
                        const int j = s_j[kk];
                        ensure_u(st, lw, A.seed, ig, t);
                        pick_step(st, lw, j);
                        pslot = (st.pick == j) ? (int32_t)s_row[D + 3][kk] : pslot;
                        if (LL) llp = (st.pick == j) ? llj : llp;
                    }
                }
                nbuf = 0;
            };
            for (int k = 0; k < nb; ++k) {  // wave-uniform: the rows in order (ascending)
                const double iso = s_row[D][k];
                if (screen) {  // (wave-uniform)
                    bool need = mine && !defer;
                    if (need && iso > 0.0) {
                        const double base = s_row[D + 1][k] + s_row[D + 2][k];
                        const double dl = (gi >= 0) ? (double)s_dist[gi][k] : 0.0;
                        const double gap = (gi >= 0) ? fmax(fmax(dl - d_own, fma(-dl, 1.0 + 0x1p-21, d_own)), 0.0) : 0.0;
                        const double far = 0.5 * iso * gap * gap;
                        const double U = base - far - Tc;
                        need = !(U <= -kSkip - 2.0 - 1e-9 * (fabs(base) + fabs(Tc) + far));
                    }
                    if (__ballot(need) == 0ull) continue;
                }
                if (mine && !defer) {
                    if (!(iso > 0.0)) {
                        defer = true;
                    } else {
                        const double m0 = s_row[0][k];
                        double s2 = (x[0] - m0) * (x[0] - m0);
#pragma unroll
                        for (int a = 1; a < D; ++a) {
                            const double ma = s_row[a][k];
                            s2 = fma(x[a] - ma, x[a] - ma, s2);
                        }
                        const double llj = fma(-0.5, s2 * iso, s_row[D + 1][k]);
                        const double lw = llj + s_row[D + 2][k];
                        const double sl = s_row[D + 3][k];
                        if (!(own_skip && sl == zslot) && lw - Tc > -kSkip) {
#pragma unroll
                            for (int e = 0; e < kBuf; ++e)
                                if (nbuf == e) {
                                    bl[e] = llj;
                                    bk[e] = k;
                                }
                            ++nbuf;
                            Tc = fmax(Tc, lw);
                        }
                    }
                }
                if (__ballot(nbuf == kBuf)) flush();  // (wave-uniform)
            }
            flush();  // (the round's rows are still in LDS)
#else
            for (int k = 0; k < nb; ++k) {  // wave-uniform: the rows in order (ascending)
                const double iso = NP8_ROWF(fiso, D, k);
                if (screen) {  // (wave-uniform)
                    bool need = mine && !defer;
                    if (need && iso > 0.0) {
                        const double base = NP8_ROWF(fc, D + 1, k) + NP8_ROWF(fl, D + 2, k);
                        const double dl = (gi >= 0) ? (double)s_dist[gi][k] : 0.0;
                        const double gap = (gi >= 0) ? fmax(fmax(dl - d_own, fma(-dl, 1.0 + 0x1p-21, d_own)), 0.0) : 0.0;
                        const double far = 0.5 * iso * gap * gap;
                        const double U = base - far - st.T;
                        need = !(U <= -kSkip - 2.0 - 1e-9 * (fabs(base) + fabs(st.T) + far));
                    }
                    if (__ballot(need) == 0ull) continue;
                }
                if (mine && !defer) {
                    if (!(iso > 0.0)) {
                        defer = true;
                    } else {
                        const double m0 = NP8_ROWF(fm[0], 0, k);
                        double s2 = (x[0] - m0) * (x[0] - m0);
#pragma unroll
                        for (int a = 1; a < D; ++a) {
                            const double ma = NP8_ROWF(fm[a], a, k);
                            s2 = fma(x[a] - ma, x[a] - ma, s2);
                        }
                        const double llj = fma(-0.5, s2 * iso, NP8_ROWF(fc, D + 1, k));
                        const double lw = llj + NP8_ROWF(fl, D + 2, k);
                        const double sl = NP8_ROWF(fsl, D + 3, k);
                        if (!(own_skip && sl == zslot)) {
                            const int j = NP8_ROWJ(k);
                            ensure_u(st, lw, A.seed, ig, t);
                            pick_step(st, lw, j);
                            pslot = (st.pick == j) ? (int32_t)sl : pslot;
                            if (LL) llp = (st.pick == j) ? llj : llp;
                        }
                    }
                }
            }
#endif
        }
    };
    if (A.use_lists && lists_ok && ngroups <= A.max_groups) {  // wave-uniform
        uint64_t pend = __ballot(1);
        while (pend) {
            const int lead = __ffsll((unsigned long long)pend) - 1;
            const int32_t j0 = __builtin_amdgcn_readlane(jo, lead);
            const int32_t nl0 = __builtin_amdgcn_readlane(nlist, lead);
            const bool grp = jo == j0;
            pend &= ~__ballot(grp);
            bool mine = false;  // this lane walks the group's list
            if (grp && !defer) {
                full = !(d2own <= r2list);
                mine = !full;
            }
            if (__ballot(mine) == 0ull) continue;
            if (NP8_CLK_ON) clk_rows += (unsigned long long)nl0;
            walk([&](int q) { return A.plist[NP8_CHK((int64_t)j0 * A.ls + q, 0, (int64_t)A.kcap * A.ls)]; }, nl0, mine,
                 false);
        }
    }
    const bool table_walk = __ballot(full && !defer) != 0ull;
    if (table_walk)  // wave-uniform row loop over the lanes that need it
        walk([](int q) { return q; }, K, full && !defer, true);
    NP8_CLK_INFO(clk_own | ((unsigned long long)ngroups << 8) | ((unsigned long long)table_walk << 16) | (clk_rows << 20));
#undef NP8_ROWF
#undef NP8_ROWJ
    NP8_CLK(3);
    // the auxiliaries: the screen's three levels (0: the prefix call, above; 1: the auxiliary's call 0; 2: its call 1),
    // then the exact fp64 draw for the lanes none of them clears; a lane that picks an auxiliary makes a new-cluster
    // request (appended below)
    bool req = false;
    if (!defer) {
        const double logam = hyp[H::kLogam];
        const float thr = (float)(st.T - kSkip - logam);  // T only grows: conservative for every m
        const float nuf = (float)hyp[H::kNu], rskf = (float)hyp[H::kRsk], cauxf = (float)hyp[H::kCaux];
        constexpr bool has_call1 = Qa > 1;
        uint32_t need = 0u;
        const float thr_err = 1e-4f * fabsf(thr);
#pragma unroll
        for (int m = 0; m < M; ++m)
            if (!(ub0[m] + thr_err <= thr)) need |= 1u << m;
        NP8_CLK(4);
        if constexpr (kL0) {
#pragma unroll 1
            for (int m = 0; m < M; ++m) {
                bool skip = ((need >> m) & 1u) == 0u;
                if (__ballot(!skip) == 0ull) continue;  // wave-uniform: the common case
                uint32_t w0[4], w1[4] = {0u, 0u, 0u, 0u};
                philox_call(A.seed, ig, t, kStreamAux, (uint32_t)(m * Qa), w0);
                aux_words0<D, M>(pre, m, w0);
                if (!skip) skip = aux_screen_ub<D>(w0, 0.0f, 0.0f, nyf, nuf, rskf, cauxf, thr) <= thr;  // level 1
                if (__ballot(!skip) == 0ull) continue;
                const bool l2 = has_call1 && !skip;
                if (l2) {  // level 2: the chi^2 terms of call 1
                    philox_call(A.seed, ig, t, kStreamAux, (uint32_t)(m * Qa + 1), w1);
                    aux_words1<D, M>(pre, m, w1);
                    float e1;
                    const float c1 = aux_screen_chi1<D>(w1, e1);
                    skip = aux_screen_ub<D>(w0, c1, e1, nyf, nuf, rskf, cauxf, thr) <= thr;
                }
                if (!skip) {
                    double v, xpar, chi2;
                    aux_core_w<D>(A.seed, ig, t, m, hyp[H::kNu], v, xpar, chi2, w0, l2, w1, pre, M);
                    const double lw = aux_loglik(sqrt(n2), v, xpar, chi2, D, hyp[H::kRsk], hyp[H::kCaux]) + logam;
                    ensure_u(st, lw, A.seed, ig, t);
                    pick_step(st, lw, K + m);
                }
            }
        } else {  // (the round-5 loop: level 1 was computed up front for every lane)
            const uint32_t none[4] = {0u, 0u, 0u, 0u};
            const float nyf1 = (float)ny;
#pragma unroll 1
            for (int m = 0; m < M; ++m) {
                bool skip = ((need >> m) & 1u) == 0u;
                if (__ballot(!skip) == 0ull) continue;  // wave-uniform: the common case
                uint32_t w0[4], w1[4] = {0u, 0u, 0u, 0u};
                philox_call(A.seed, ig, t, kStreamAux, (uint32_t)(m * Qa), w0);
                const bool l2 = has_call1 && !skip;
                if (l2) {  // level 2: the chi^2 terms of call 1
                    philox_call(A.seed, ig, t, kStreamAux, (uint32_t)(m * Qa + 1), w1);
                    float e1;
                    const float c1 = aux_screen_chi1<D>(w1, e1);
                    skip = aux_screen_ub<D>(w0, c1, e1, nyf1, nuf, rskf, cauxf, thr) <= thr;
                }
                if (!skip) {
                    double v, xpar, chi2;
                    aux_core_w<D>(A.seed, ig, t, m, hyp[H::kNu], v, xpar, chi2, w0, l2, w1, none, M);
                    const double lw = aux_loglik(ny, v, xpar, chi2, D, hyp[H::kRsk], hyp[H::kCaux]) + logam;
                    ensure_u(st, lw, A.seed, ig, t);
                    pick_step(st, lw, K + m);
                }
            }
        }
        req = st.pick >= K;
    }
    NP8_CLK(5);
    // deferred lanes: positions into this wave's slots of the queue (compacted, no atomics), their count
    // for np8_assign's queue mode; nothing else is written for them
    const uint64_t db = __ballot(defer);
    if (db) {  // rare (rows that are not isotropic): the wave lists itself for np8_assign's queue mode
        if (NP8_LATE(no_queue)) {  // the host left the queue kernel out (every row isotropic): must not happen
            if (lane == (__ffsll((unsigned long long)db) - 1)) atomicOr(&NP8_LATE(ctl)->err, kErrQueue);
            return;
        }
        const int64_t wv = (p - NP8_LATE(p0)) >> 6;
        if (defer) NP8_LATE(queue_out)[wv * 64 + __popcll(db & ((1ull << lane) - 1ull))] = (int32_t)p;
        if (lane == (__ffsll((unsigned long long)db) - 1)) {
            NP8_LATE(qcount)[wv] = __popcll(db);
            NP8_LATE(qlist)[atomicAdd(&NP8_LATE(ctl)->qwaves, 1u)] = (int32_t)wv;
        }
    }
    const int32_t snew = req ? zi : pslot;  // a lane not deferred picked an existing row or stays (request)
    if (NP8_LATE(collect_r2)) {  // np8_assign's radius collection, over the lanes not deferred
        // (a requester counts for its old cluster, in case the request is rejected: np8_assign's rule)
        const int32_t tr = (defer || req) ? jo : st.pick;
        const double *e = cand + (int64_t)NP8_CHK(tr, 0, K) * CS;
        double d2 = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const double dd = x[a] - e[a];
            d2 = fma(dd, dd, d2);
        }
        // the lanes not deferred share one slot (the label-sorted layout): one record for the wave; deferred
        // lanes add theirs in np8_assign's queue mode
        const uint64_t kept = __ballot(!defer);
        const int32_t t0 = __shfl(snew, kept ? __ffsll((unsigned long long)kept) - 1 : 0);
        const bool one = kept != 0ull && __ballot(!defer && snew != t0) == 0;
        if (one) {
            d2 = defer ? 0.0 : d2;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) d2 = fmax(d2, __shfl_xor(d2, o));
        } else {
            wave_max_by_key(reinterpret_cast<unsigned long long *>(NP8_LATE(r2) + NP8_LATE(kcap)), (int32_t)NP8_CHK(snew, 0, NP8_LATE(kcap)), d2,
                            !defer);
        }
        if (lane == (__ffsll((unsigned long long)__ballot(1)) - 1)) {  // the wave's record
            WaveR2 wr;
            wr.d2 = one ? d2 : 0.0;
            wr.slot = one ? (int32_t)NP8_CHK(t0, 0, NP8_LATE(kcap)) : -1;
            wr.pad = 0;
            NP8_LATE(wr2)[(p - NP8_LATE(p0)) >> 6] = wr;
        }
    }
    const uint64_t mv = __ballot(!defer && snew != zi);
    if (mv && lane == (__ffsll((unsigned long long)__ballot(1)) - 1))
        atomicAdd(reinterpret_cast<unsigned long long *>(&NP8_LATE(ctl)->moved), (unsigned long long)__popcll(mv));
    {
        int32_t *delta = reinterpret_cast<int32_t *>(NP8_LATE(rec) + kRecHeaderBytes);
        const bool mover = !defer && snew != zi;
        wave_add_by_key(delta, zi, -1, mover);
        wave_add_by_key(delta, (int32_t)NP8_CHK(snew, 0, NP8_LATE(kcap)), 1, mover);
    }
    if (!defer && snew != zi) {
        NP8_LATE(z)[il] = snew;
        zs[p] = snew;
    }
    if constexpr (LL) {  // the wave's exact sum (a requester counts under its old slot)
        Fx v = fx_of(req ? ll_own : llp);
        const uint64_t act = __ballot(1);
        if (act == ~0ull) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v = fx_add(v, fx_shfl_xor(v, o));
        } else {  // the range's last, partial wave
            Fx s = {0ull, 0};
            for (uint64_t m = act; m; m &= m - 1ull) s = fx_add(s, fx_readlane(v, __ffsll((unsigned long long)m) - 1));
            v = s;
        }
        if (lane == __ffsll((unsigned long long)act) - 1) NP8_LATE(llpart)[(p - NP8_LATE(p0)) >> 6] = v;
    }
    const int qreq = wave_append(NP8_LATE(nreq), req);  // (requests are accepted by scan position, not arrival)
    if (req) {  // np8_assign's request with its payload, the auxiliary's (v, mu)
        const int q = (int)NP8_CHK(qreq, 0, NP8_LATE(req_cap));
        if (q < NP8_LATE(req_cap)) {  // always: the area holds every item of the step
            // the item key and epoch read again here (volatile: not kept live from the top of the kernel -- they
            // were spilled to scratch on every lane, 16 MB of writes per C3 launch, for this rare path)
            const uint64_t igr = (uint64_t)(NP8_LATE(offset) + reinterpret_cast<const volatile int32_t *>(ids)[p]);
            const uint32_t tr = reinterpret_cast<const volatile Ctl *>(NP8_LATE(ctl))->t_base + NP8_LATE(t);
            double *vm = NP8_LATE(vmu) + (int64_t)q * (D + 1);
            double y0[D];
            whiten<D>(hyp, x, y0);
            aux_params<D>(hyp, y0, kL0 ? norm_of<D>(y0) : ny, NP8_LATE(seed), igr, tr, st.pick - K, M, vm);
            Request r;
            r.pos = (int64_t)igr;  // synchronous sweep: scan position = item index
            r.i = (int64_t)igr;
            r.m = st.pick - K;
            r.zold = zi;
            r.lpos = (int32_t)p;
            r.pad = 0;
            r.dll.lo = 0ull;
            r.dll.hi = 0;
            if (LL) {  // ll under the slot np8_finalize would build from (v, mu) (write_new_slot), as np8_loglik evaluates it
                const double v = vm[0], v2 = v * v;
                const double iso_n = NP8_LATE(gp0) / v2, c_n = fma(-(double)D, log_pos(fabs(v)), hyp[H::kCaux]);
                double s2 = (x[0] - vm[1]) * (x[0] - vm[1]);
#pragma unroll
                for (int a = 1; a < D; ++a) s2 = fma(x[a] - vm[1 + a], x[a] - vm[1 + a], s2);
                r.dll = fx_add(fx_of(fma(-0.5, s2 * iso_n, c_n)), fx_neg(fx_of(ll_own)));
            }
            NP8_LATE(req)[q] = r;
            if (q < NP8_LATE(ccap)) {  // compact exchange: the record the ranks all-gather holds the first ccap requests too
                NP8_LATE(creq)[q] = r;
                for (int a = 0; a <= D; ++a) NP8_LATE(cvmu)[(int64_t)q * (D + 1) + a] = vm[a];
            }
        }
    }
    if (snap) {  // the rest of the pending snapshot: counts and parameters as the check's finalize left them
        const int64_t g = p - NP8_LATE(p0), ng = NP8_LATE(p1) - NP8_LATE(p0);
        for (int64_t k = g; k < NP8_LATE(kcap); k += ng) NP8_LATE(cnt_best)[k] = NP8_LATE(cnt)[k];
        for (int64_t k = g; k < (int64_t)NP8_LATE(kcap) * D; k += ng) NP8_LATE(mu_best)[k] = NP8_LATE(slot_mu)[k];
        for (int64_t k = g; k < (int64_t)NP8_LATE(kcap) * D * D; k += ng) NP8_LATE(sigma_best)[k] = NP8_LATE(slot_sigma)[k];
    }
    NP8_CLK(6);
}

// ---- label-sorted layout ------------------------------------------------------------------------------
// Counting sort by slot.  The order inside a cluster depends on atomic arrival, which changes no
// result: in the synchronous sweep every item's draw is a pure function of (state, item, epoch).
constexpr int kSortThreads = 1024, kSortItems = 4;  // 4096 items per block

// (never while a compact sweep graph is halted: the halted step's requests name positions of the current layout)
__device__ __forceinline__ bool sort_needed(const SortArgs &S) {
    return !S.ctl->halt && (S.force || S.ctl->moved * 32 > S.n);
}

// Sort key of position p: the slot, after the item's data-parallel sub-step (sub-steps are contiguous
// ranges of the layout, clusters contiguous inside each).  ids = null: p is the local item itself.
__device__ __forceinline__ int sort_key(const SortArgs &S, const int32_t *__restrict__ z, const int32_t *__restrict__ ids,
                                        int64_t p) {
    const int32_t slot = (int32_t)NP8_CHK(z[p], 0, S.kcap);
    if (S.nsub <= 1) return slot;
    const int64_t item = S.offset + (ids ? (int64_t)ids[p] : p);
    return (int)substep_of(S.seed, item, (uint32_t)S.nsub) * S.kcap + slot;
}

__global__ __launch_bounds__(kSortThreads) void np8_sort_hist(SortArgs S) {
    if (!sort_needed(S)) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int *lh = reinterpret_cast<int *>(smem);
    const int nb = S.kcap * S.nsub;
    const int32_t *z = S.force ? S.z : S.zs[0];
    const int32_t *ids = S.force ? nullptr : S.ids[0];
    for (int s = threadIdx.x; s < nb; s += kSortThreads) lh[s] = 0;
    __syncthreads();
    for (int k = 0; k < kSortItems; ++k) {
        const int64_t p = ((int64_t)blockIdx.x * kSortItems + k) * kSortThreads + threadIdx.x;
        if (p < S.n) atomicAdd(&lh[sort_key(S, z, ids, p)], 1);
    }
    __syncthreads();
    for (int s = threadIdx.x; s < nb; s += kSortThreads)
        if (lh[s]) atomicAdd(&S.hist[s], lh[s]);
}

__global__ __launch_bounds__(kSortThreads) void np8_sort_scatter(SortArgs S) {
    if (!S.ctl->do_sort) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nb = S.kcap * S.nsub;
    int *lh = reinterpret_cast<int *>(smem);
    int *lbase = lh + nb;
    // the current layout is always buffer 0 (kernels need not load which one): a rebuild from the item order
    // writes it directly, a re-sort goes 0 -> 1 and np8_sort_copyback copies it back
    const int src = 0, dst = S.force ? 0 : 1;
    const int32_t *z = S.force ? S.z : (src ? S.zs[1] : S.zs[0]);
    const int32_t *ids = S.force ? nullptr : (src ? S.ids[1] : S.ids[0]);
    const double *X = S.force ? S.X : (src ? S.Xs[1] : S.Xs[0]);
    int32_t *zo = dst ? S.zs[1] : S.zs[0];
    int32_t *ido = dst ? S.ids[1] : S.ids[0];
    double *Xo = dst ? S.Xs[1] : S.Xs[0];
    for (int s = threadIdx.x; s < nb; s += kSortThreads) lh[s] = 0;
    __syncthreads();
    int zp[kSortItems], rk[kSortItems];  // sort keys, ranks in the block
    for (int k = 0; k < kSortItems; ++k) {
        const int64_t p = ((int64_t)blockIdx.x * kSortItems + k) * kSortThreads + threadIdx.x;
        zp[k] = (p < S.n) ? sort_key(S, z, ids, p) : -1;
        rk[k] = (zp[k] >= 0) ? atomicAdd(&lh[zp[k]], 1) : 0;
    }
    __syncthreads();
    for (int s = threadIdx.x; s < nb; s += kSortThreads)
        if (lh[s]) lbase[s] = atomicAdd(&S.cursor[s], lh[s]);
    __syncthreads();
    for (int k = 0; k < kSortItems; ++k) {
        if (zp[k] < 0) continue;
        const int64_t p = ((int64_t)blockIdx.x * kSortItems + k) * kSortThreads + threadIdx.x;
        const int64_t q = (int64_t)S.off[zp[k]] + lbase[zp[k]] + rk[k];
        zo[q] = z[p];
        ido[q] = ids ? ids[p] : (int32_t)p;
        if (S.esz == 4) {  // wide path: fp32 items and the frame's words, copied as bits
            const uint32_t *Xf = reinterpret_cast<const uint32_t *>(X);
            uint32_t *Xfo = reinterpret_cast<uint32_t *>(Xo);
            for (int a = 0; a < S.D; ++a) Xfo[(int64_t)a * S.n + q] = Xf[(int64_t)a * S.n + p];
        } else {
            for (int a = 0; a < S.D; ++a) Xo[(int64_t)a * S.n + q] = X[(int64_t)a * S.n + p];
        }
    }
}

// A re-sort's result (buffer 1) back into buffer 0, the current layout.  16-byte pieces, grid-stride.
__global__ __launch_bounds__(256) void np8_sort_copyback(SortArgs S) {
    if (!S.ctl->do_sort || S.force) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto copy = [&](const void *src, void *dst, int64_t bytes) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        const int64_t n16 = bytes / 16;
        for (int64_t i = i0; i < n16; i += stride) d4[i] = s4[i];
        const unsigned char *sb = reinterpret_cast<const unsigned char *>(src);
        unsigned char *db = reinterpret_cast<unsigned char *>(dst);
        for (int64_t i = n16 * 16 + i0; i < bytes; i += stride) db[i] = sb[i];
    };
    copy(S.zs[1], S.zs[0], 4 * S.n);
    copy(S.ids[1], S.ids[0], 4 * S.n);
    copy(S.Xs[1], S.Xs[0], (int64_t)S.esz * S.D * S.n);
}

__global__ __launch_bounds__(1024) void np8_sort_scan(SortArgs S) {
    const bool need = sort_needed(S);
    __syncthreads();
    if (threadIdx.x == 0) {
        S.ctl->do_sort = need ? 1 : 0;
        if (need) {
            S.ctl->moved = 0;
            S.ctl->done_blocks = 0;
        }
    }
    if (!need) return;
    __shared__ int sh[32];
    const int nb = S.kcap * S.nsub;
    const int per = (nb + 1023) / 1024;
    const int s0 = min(nb, (int)threadIdx.x * per), s1 = min(nb, s0 + per);
    int v = 0;
    for (int s = s0; s < s1; ++s) v += S.hist[s];
    int tot;
    int base = 0;
    {
        // inclusive wave scan, then across waves
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        int inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const int n = __shfl_up(inc, o, 64);
            if (lane >= o) inc += n;
        }
        if (lane == 63) sh[wid] = inc;
        __syncthreads();
        if (wid == 0) {
            const int x = (lane < 16) ? sh[lane] : 0;
            int y = x;
            for (int o = 1; o < 64; o <<= 1) {
                const int n = __shfl_up(y, o, 64);
                if (lane >= o) y += n;
            }
            if (lane < 16) sh[lane] = y - x;
            if (lane == 15) sh[16] = y;
        }
        __syncthreads();
        base = sh[wid] + inc - v;
        tot = sh[16];
    }
    (void)tot;
    for (int s = s0; s < s1; ++s) {
        S.off[s] = base;
        base += S.hist[s];
        S.cursor[s] = 0;
        S.hist[s] = 0;  // ready for the next pass
    }
}

// ---- block-wide helpers (1024 threads) ------------------------------------------------------------
constexpr int kFinThreads = 1024;

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int n = __shfl_up(v, o, 64);
        if (lane >= o) v += n;
    }
    return v;
}

// Exclusive scan over the block; returns this thread's prefix, *total the block sum.
__device__ int block_excl_scan(int v, int *sh /* >= 16 ints */, int *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int inc = wave_incl_scan(v);
    __syncthreads();
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        const int x = (lane < nw) ? sh[lane] : 0;
        const int y = wave_incl_scan(x);
        if (lane < nw) sh[lane] = y - x;
        if (lane == nw - 1) sh[16] = y;
    }
    __syncthreads();
    const int r = sh[wid] + inc - v;
    *total = sh[16];
    __syncthreads();
    return r;
}

// Exact block sum of Fx values (every thread returns it).
__device__ Fx block_sum_fx(Fx v, Fx *sh /* >= 16 */) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t l0 = (uint32_t)__shfl_xor((int)(uint32_t)v.lo, o), l1 = (uint32_t)__shfl_xor((int)(uint32_t)(v.lo >> 32), o);
        const uint32_t h0 = (uint32_t)__shfl_xor((int)(uint32_t)(uint64_t)v.hi, o),
                       h1 = (uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)v.hi >> 32), o);
        Fx w;
        w.lo = ((uint64_t)l1 << 32) | l0;
        w.hi = (int64_t)(((uint64_t)h1 << 32) | h0);
        v = fx_add(v, w);
    }
    __syncthreads();
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    Fx t = sh[0];
    for (int w = 1; w < nw; ++w) t = fx_add(t, sh[w]);
    __syncthreads();
    return t;
}

// The folded max-likelihood check's per-rank sum of the assign's per-wave partials (exact).
__device__ Fx partials_sum(const Fx *__restrict__ part, int64_t n, Fx *sh) {
    Fx v = {0ull, 0};
    for (int64_t k = threadIdx.x; k < n; k += blockDim.x) v = fx_add(v, part[k]);
    return block_sum_fx(v, sh);
}

}  // namespace

// ---- candidate pruning ------------------------------------------------------------------------------
// v >= 0 as a float no larger than v (a distance the walk's screen may only underestimate)
__device__ __forceinline__ float f32_down(double v) {
    const float f = (float)v;
    return ((double)f > v) ? __int_as_float(__float_as_int(f) - 1) : f;
}

// For dense row k0 (mean mu0, radius R = max |x - mu0| over its items, collected by the sweep), row j
// can be left out of k0's list when no item of k0 can bring it within kSkip of its own log-weight:
//   lw_j(x) - lw_own(x) <= (c_j + log n_j) - (c_0 + log(n_0 - 1)) - iso_j (|mu_j - mu0| - R)^2 / 2
//                           + iso_0 R^2 / 2  =: U,
// using q_j(x) = iso_j |x - mu_j|^2 >= iso_j (|mu_j - mu0| - R)^2 (triangle inequality) and
// q_0(x) <= iso_0 R^2; T >= lw_own at every step of the pick.  Rows are left out only for U below
// -kSkip by a margin of 2 nats plus 1e-9 of the terms' magnitude (rounding of the kernel's own
// arithmetic is ~1e-15 relative).  Non-isotropic rows and singletons (own weight 0) keep every row.
// One wave builds one row's list (ascending j) and clears the row's radius for the next sweep.
constexpr int kPruneBlocks = 32;  // np8_prune grid: 128 rows per pass

// DT > 0: the dimension as a template constant (loops unrolled, the row loads issued together)
// R2of(slot): the squared radius of the slot's items that will walk the list.
template <int DT = 0, typename R2of>
__device__ void prune_row(const double *__restrict__ cand, R2of R2of_slot, int32_t *__restrict__ plist,
                          float *__restrict__ pdist, int32_t *__restrict__ plen, double *__restrict__ plr2, int32_t *__restrict__ plen_s,
                          double *__restrict__ plr2_s, int ls, int Drt, int K, int k0, double *__restrict__ lb, int kcap,
                          const double *__restrict__ lam) {
    const int D = DT > 0 ? DT : Drt;
    const int DP = D * (D + 1) / 2, CS = cand_stride(D), F = D + DP;
    const int lane = threadIdx.x & 63;
    const double *e0 = cand + (int64_t)k0 * CS;
    const int slot0 = (int)NP8_CHK((int)e0[F + kFieldSlot], 0, kcap);
    const double R2 = R2of_slot(slot0);
    const double iso0 = e0[F + kFieldIso];
    // (rows that are not isotropic, round 6: q_0(x) <= hi_0 |x - mu0|^2 and q_j(x) >= lo_j |x - mu_j|^2 with the slots'
    // precision eigenvalue bounds -- the same bound with iso replaced; isotropic rows exactly as before)
    const double hi0 = iso0 > 0.0 ? iso0 : (lam ? lam[kcap + slot0] : 0.0);
    const double base0 = e0[F + kFieldC] + e0[F + kFieldLogn1];
    const bool prunable = hi0 > 0.0 && R2 < 1e300 && base0 > -1e299;
    const double R = sqrt(R2);
    int count = 0;
    for (int jb = 0; jb < K; jb += 64) {
        const int j = jb + lane;
        bool keep = j < K && j != k0;
        if (j < K) {
            const double *ej = cand + (int64_t)j * CS;
            double dist2 = 0.0;
#pragma unroll
            for (int a = 0; a < (DT > 0 ? DT : 1); ++a) {  // DT: fully unrolled
                const double dd = ej[a] - e0[a];
                dist2 = fma(dd, dd, dist2);
            }
            for (int a = (DT > 0 ? DT : 1); a < D; ++a) {  // runtime D (only when DT == 0)
                const double dd = ej[a] - e0[a];
                dist2 = fma(dd, dd, dist2);
            }
            if (pdist) pdist[(int64_t)k0 * ls + j] = f32_down(sqrt(dist2));  // (every pair: the walk's screen)
            const double isoj = ej[F + kFieldIso];
            const double loj = isoj > 0.0 ? isoj : (lam ? lam[(int)NP8_CHK((int)ej[F + kFieldSlot], 0, kcap)] : 0.0);
            if (keep && prunable && loj > 0.0) {
                const double delta = sqrt(dist2) - R;
                if (delta > 0.0) {
                    const double wj = ej[F + kFieldC] + ej[F + kFieldLogn];
                    const double far = 0.5 * loj * delta * delta, near = 0.5 * hi0 * R2;
                    const double U = (wj - base0) - far + near;
                    const double mag = fabs(wj) + fabs(base0) + far + near;
                    keep = !(U <= -kSkip - 2.0 - kListSlack - 1e-9 * mag);
                }
            }
        }
        const uint64_t b = __ballot(keep);
        if (keep) plist[(int64_t)k0 * ls + count + __popcll(b & ((1ull << lane) - 1ull))] = j;
        count += __popcll(b);
    }
    if (lane == 0) {
        const double r2l = prunable ? R2 : __longlong_as_double(0x7FF0000000000000ll);  // +inf: every row is listed
        plen[k0] = count;
        plr2[k0] = r2l;
        plen_s[slot0] = count;
        plr2_s[slot0] = r2l;
        if (lb) {  // the counts' logs this list is exact for (within kListSlack / 2)
            lb[slot0] = e0[F + kFieldLogn];
            lb[kcap + slot0] = e0[F + kFieldLogn1];
        }
    }
}

// ---- finalize --------------------------------------------------------------------------------------
namespace {

__device__ __forceinline__ const RecHeader *rec_header(const FinArgs &F, int r) {
    return reinterpret_cast<const RecHeader *>(F.recs + (int64_t)r * F.rec_bytes);
}

__device__ __forceinline__ const int32_t *rec_delta(const FinArgs &F, int r) {
    return reinterpret_cast<const int32_t *>(F.recs + (int64_t)r * F.rec_bytes + kRecHeaderBytes);
}

__device__ __forceinline__ const Request *rec_reqs(const FinArgs &F, int r) {
    return reinterpret_cast<const Request *>(F.recs + (int64_t)r * F.rec_bytes + kRecHeaderBytes +
                                             (int64_t)F.kcap * 4);
}

// Global request q (ranks concatenated in rank order) -> its record entry.
__device__ const Request *request_at(const FinArgs &F, const int *base, int q) {
    int r = 0;
    while (r + 1 < F.world && q >= base[r + 1]) ++r;
    return rec_reqs(F, r) + (q - base[r]);
}

// ... and the (v, mu) its rank computed for it.
__device__ const double *request_vmu(const FinArgs &F, const int *base, int q) {
    int r = 0;
    while (r + 1 < F.world && q >= base[r + 1]) ++r;
    return reinterpret_cast<const double *>(F.recs + (int64_t)r * F.rec_bytes + record_vmu_offset(F.kcap, F.rec_cap)) +
           (int64_t)(q - base[r]) * (F.D + 1);
}

// Wide path, reference prior: (v, mu) of auxiliary m of item i from the item frame (|y0|, y0) its
// rank recorded -- aux_params of the narrow path with D at run time (any D of the wide path) and the frame read back
// instead of recomputed: the same operations in the same order.
__device__ void frame_to_vmu(const FinArgs &F, const double *frame, int64_t i, int m, double *vmu) {
    const int D = F.D, DP = D * (D + 1) / 2;
    const double *hyp = F.hyp;  // mu0 | UinvT packed | caux | rsk | logam | nu | LT packed (HypView)
    const uint32_t t = F.ctl->t_base + F.t;
    double y0[kMaxD], xi[kMaxD];
    for (int a = 0; a < D; ++a) y0[a] = frame[1 + a];
    double v, xpar, chi2;
    aux_core_rt(F.seed, (uint64_t)i, t, m, F.M, D, hyp[D + DP + 3], v, xpar, chi2);
    aux_xi<kMaxD>(F.seed, (uint64_t)i, t, m, D, y0, frame[0], xpar, chi2, xi);
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

}  // namespace

// ---- request selection ------------------------------------------------------------------------------
namespace {

// The k-th smallest (1 <= k <= n) of n distinct scan positions (all < 2^33) held by pos_at(q), q < n:
// three passes of an 11-bit radix histogram (2048 bins in LDS) over the entries that share the bits
// fixed so far.  One workgroup of kFinThreads; every thread returns the same value.
template <class PosAt>
__device__ int64_t select_kth_pos(PosAt pos_at, int n, int k, int *hist /* 2048 */, int *sh /* >= 20 */) {
    const int tid = threadIdx.x;
    int64_t prefix = 0;
    for (int pass = 0; pass < 3; ++pass) {
        const int shift = 22 - 11 * pass;  // bits [shift, shift + 11)
        const int64_t fixed = ~((1ll << (shift + 11)) - 1);
        for (int b = tid; b < 2048; b += kFinThreads) hist[b] = 0;
        __syncthreads();
        for (int q = tid; q < n; q += kFinThreads) {
            const int64_t pos = pos_at(q);
            if ((pos & fixed) == prefix) atomicAdd(&hist[(pos >> shift) & 2047], 1);
        }
        __syncthreads();
        const int h0 = hist[2 * tid], h1 = hist[2 * tid + 1];
        int tot;
        const int ex = block_excl_scan(h0 + h1, sh, &tot);
        if (ex < k && k <= ex + h0) {
            sh[18] = 2 * tid;
            sh[19] = k - ex;
        } else if (ex + h0 < k && k <= ex + h0 + h1) {
            sh[18] = 2 * tid + 1;
            sh[19] = k - ex - h0;
        }
        __syncthreads();
        prefix |= (int64_t)sh[18] << shift;
        k = sh[19];
        __syncthreads();
    }
    return prefix;
}

}  // namespace

// Several ranks: this rank's requests of the step (staging record, arrival order) -> the req_max of
// lowest scan position in the exchanged record (the only ones np8_finalize can accept from this rank,
// DESIGN.md "Finalize"); clears the staging count.  One workgroup; dynamic LDS: hist int[2048].
// (the body of np8_req_select, also run as the serial tail of np8_step_tail)
__device__ void req_select_block(const unsigned char *__restrict__ stage, int64_t stage_cap,
                                 unsigned char *__restrict__ rec, int64_t rec_cap, int kcap, int D, int req_max,
                                 const Fx *__restrict__ llpart, int64_t ll_n, int *hist /* LDS int[2048] */) {
    __shared__ int sh[32];
    __shared__ int s_cnt;
    __shared__ Fx shfx[16];
    // folded max-likelihood check: this rank's exact sum travels in the exchanged record's header
    Fx Lloc = {0ull, 0};
    if (llpart) Lloc = partials_sum(llpart, ll_n, shfx);
    RecHeader *sh_hdr = reinterpret_cast<RecHeader *>(const_cast<unsigned char *>(stage));
    const Request *sreq = reinterpret_cast<const Request *>(stage + kRecHeaderBytes + 4ll * kcap);
    const double *svmu = reinterpret_cast<const double *>(stage + record_vmu_offset(kcap, (int)stage_cap));
    Request *rreq = reinterpret_cast<Request *>(rec + kRecHeaderBytes + 4ll * kcap);
    double *rvmu = reinterpret_cast<double *>(rec + record_vmu_offset(kcap, (int)rec_cap));
    const int n = (int)min((int64_t)sh_hdr->nreq, stage_cap);
    const int k = min(n, req_max);
    int64_t T = INT64_MAX;
    if (n > k && k > 0) T = select_kth_pos([&](int q) { return sreq[q].pos; }, n, k, hist, sh);
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    for (int q = threadIdx.x; q < (k > 0 ? n : 0); q += kFinThreads) {
        const Request r = sreq[q];
        if (r.pos > T) continue;
        const int o = atomicAdd(&s_cnt, 1);
        rreq[o] = r;
        for (int a = 0; a <= D; ++a) rvmu[(int64_t)o * (D + 1) + a] = svmu[(int64_t)q * (D + 1) + a];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        reinterpret_cast<RecHeader *>(rec)->nreq = k;
        reinterpret_cast<RecHeader *>(rec)->nreq_all = n;
        if (llpart) reinterpret_cast<RecHeader *>(rec)->L_local = Lloc;
        sh_hdr->nreq = 0;
    }
}

// compact exchange, check sweeps: this rank's exact log-likelihood sum into the compact record's header (the full
// records get it from np8_req_select)
__global__ __launch_bounds__(kFinThreads) void np8_ll_header(const Ctl *__restrict__ ctl, const Fx *__restrict__ llpart,
                                                             int64_t ll_n, unsigned char *__restrict__ rec) {
    __shared__ Fx shfx[16];
    if (ctl->halt) return;
    const Fx L = partials_sum(llpart, ll_n, shfx);
    if (threadIdx.x == 0) reinterpret_cast<RecHeader *>(rec)->L_local = L;
}

__global__ __launch_bounds__(kFinThreads) void np8_req_select(const unsigned char *__restrict__ stage, int64_t stage_cap,
                                                              unsigned char *__restrict__ rec, int64_t rec_cap, int kcap,
                                                              int D, int req_max, const Fx *__restrict__ llpart,
                                                              int64_t ll_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    req_select_block(stage, stage_cap, rec, rec_cap, kcap, D, req_max, llpart, ll_n, reinterpret_cast<int *>(smem));
}

namespace {
__device__ int64_t request_pos(const FinArgs &F, const int *base, int q) { return request_at(F, base, q)->pos; }
}  // namespace

// One workgroup of 1024 threads.  Dynamic LDS: sort keys int64[kReqMax] | sort idx int[kReqMax] |
// free slots int[kReqMax] (first the selection histogram, int[2048]) | cnt int[kcap] | live int[kcap].
// New-cluster requests (DESIGN.md "Finalize"): the deltas are applied first and the free slots counted
// with every requester still in its old slot; the A = min(req_max, free, requests) requests of lowest
// scan position are accepted, in position order, into the lowest free slots in ascending order; each
// accepted requester leaves its old slot; the others keep their cluster (deferred to their next update).
#ifdef NP8_EXP_FIN_TIMING  // experiment: finalize_block phase clocks (thread 0), printed per call
#define FIN_T(k) \
    if (threadIdx.x == 0) ftm[k] = (long long)__builtin_amdgcn_s_memtime();
#else
#define FIN_T(k)
#endif
// (the body of np8_finalize, also run as the serial tail of np8_step_tail; smem: np8_finalize_lds_bytes)
// Returns (block-uniform) whether the candidate lists of the last build may be stale after this step: a slot changed
// liveness, requests were accepted, the rows were re-copied, or (slack_test) a live slot's log n or log(n - 1) moved
// more than kListSlack / 2 from the build's values.
__device__ int finalize_block(const FinArgs &F, unsigned char *smem) {
    int64_t *keys = reinterpret_cast<int64_t *>(smem);
    int *kidx = reinterpret_cast<int *>(smem + sizeof(int64_t) * kReqMax);
    int *freeslot = kidx + kReqMax;
    int *cnt_s = freeslot + kReqMax;
    int *live_s = cnt_s + F.kcap;
    __shared__ int sh[32];
    __shared__ int base[65];
    __shared__ int s_flags[4];  // nreq, gathered
    const int tid = threadIdx.x;
    const int kcap = F.kcap;
#ifdef NP8_EXP_FIN_TIMING
    long long ftm[12] = {0};
#endif
    FIN_T(0)
    const int D = F.D, DP = D * (D + 1) / 2, CS = cand_stride(D);
    const int per = (kcap + kFinThreads - 1) / kFinThreads;
    const int s0 = min(kcap, tid * per), s1 = min(kcap, s0 + per);
    // everything the common step (no request accepted) needs from global memory, loaded in one round:
    // old counts (liveness changes), deltas, and the table entries of this thread's first kFinPre slots
    constexpr int kFinPre = 2;
    int cold[kFinPre], d0[kFinPre], dof[kFinPre];
    double pc[kFinPre], piso[kFinPre], plb0[kFinPre], plb1[kFinPre];
    const int32_t *delta0 = rec_delta(F, 0);
#pragma unroll
    for (int q = 0; q < kFinPre; ++q) {
        const int s = s0 + q;
        const bool in = s < s1;
        cold[q] = in ? F.cnt[s] : 0;
        d0[q] = in ? delta0[s] : 0;  // rank 0's delta in the same round of loads (the single-rank step: all of them)
        dof[q] = in ? F.dense_of[s] : -1;
        pc[q] = in ? F.slot_c[s] : 0.0;
        piso[q] = in ? F.slot_iso[s] : 0.0;
        plb0[q] = (in && F.slack_test) ? F.lb[s] : 0.0;
        plb1[q] = (in && F.slack_test) ? F.lb[kcap + s] : 0.0;
    }
    const int cand_fresh = F.ctl->cand_fresh;
    const int nreq0 = rec_header(F, 0)->nreq;  // (same round: every thread, one address)
    if (F.compact && F.ctl->halt) return -1;   // (same round) a compact graph halted at an earlier step
    int nreq_all = min(nreq0, F.rec_cap);
    int peak = max(nreq0, rec_header(F, 0)->nreq_all), over = nreq0 > F.rec_cap;
    for (int r = 1; r < F.world; ++r) {
        const RecHeader *h = rec_header(F, r);
        nreq_all += min(h->nreq, F.rec_cap);
        peak = max(peak, max(h->nreq, h->nreq_all));
        over |= h->nreq > F.rec_cap;
    }
    if (F.compact && over) {  // block-uniform (every thread read the same headers; so does every rank)
        // some rank's requests did not fit its compact record: apply nothing, halt the graph (the host runs this step's
        // exchange with the full records, from the records and staging area left as they are)
        if (tid == 0) {
            F.ctl->halt = 1;
            F.ctl->halt_t = F.t;
            F.ctl->n_pend = 0;  // (the NIW / wide slot kernels after this finalize: no accepted request to build)
            if (F.mirror) {
                F.mirror[1] = (int32_t)F.t;
                F.mirror[0] = 1;
            }
        }
        return -1;
    }
    if (tid == 0 && peak > F.ctl->req_peak) F.ctl->req_peak = peak;
    // the folded check's partials (one rank), eight independent loads per round
    Fx llv = {0ull, 0};
    if (F.ll_on && !F.ll_rec) {
        const uint64_t *pp = reinterpret_cast<const uint64_t *>(F.llpart);
        for (int64_t b = tid; b < F.ll_n; b += 8 * kFinThreads) {
            uint64_t vl[8], vh[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t k = b + (int64_t)u * kFinThreads;
                const bool in = k < F.ll_n;
                vl[u] = in ? pp[2 * k] : 0ull;
                vh[u] = in ? pp[2 * k + 1] : 0ull;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                Fx w;
                w.lo = vl[u];
                w.hi = (int64_t)vh[u];
                llv = fx_add(llv, w);
            }
        }
    }
    FIN_T(1)

    // The steady step (no request, no slot changing liveness, rows current): the dense table keeps its rows, so only
    // the slots whose count moved get their count and logs rewritten (rows from the prefetched dense_of) -- no scan,
    // no table rebuild: one round of loads and a barrier or two.  Everything else takes the general path below.
    {
        int cnew[kFinPre], lch = 0;
#pragma unroll
        for (int q = 0; q < kFinPre; ++q) {
            const int s = s0 + q;
            int c = cold[q] + d0[q];
            if (s < s1)
                for (int r = 1; r < F.world; ++r) c += rec_delta(F, r)[s];
            cnew[q] = c;
            lch |= (s < s1) && ((c > 0) != (cold[q] > 0));
        }
        const int any_lch = __syncthreads_or(lch);
        FIN_T(2)
        if (!any_lch && nreq_all == 0 && cand_fresh && per <= kFinPre && !F.frame_payload) {  // block-uniform
            int viol = 0;
#pragma unroll
            for (int q = 0; q < kFinPre; ++q) {
                const int s = s0 + q;
                if (s < s1 && cnew[q] != cold[q]) {  // a live slot whose count moved (a dead one stays dead)
                    const int c = cnew[q];
                    F.cnt[s] = c;
                    const double l0 = log_pos((double)c), l1 = (c > 1) ? log_pos((double)(c - 1)) : kZeroLogWeight;
                    if (F.slack_test && !(fabs(l0 - plb0[q]) <= 0.5 * kListSlack && fabs(l1 - plb1[q]) <= 0.5 * kListSlack))
                        viol = 1;
                    double *e = F.cand + (int64_t)dof[q] * CS + D + DP;
                    e[kFieldLogn] = l0;
                    e[kFieldLogn1] = l1;
                    F.slot_logn1[s] = l1;
                }
            }
            const int stale_f = __syncthreads_or(viol);  // (unchanged slots passed the test at the last step)
            if (F.ll_on) {
                __shared__ Fx shfx_f[16];
                Fx S = block_sum_fx(llv, shfx_f);
                Fx Sloc = S;
                if (F.ll_rec)
                    for (int r = 0; r < F.world; ++r) S = fx_add(S, rec_header(F, r)->L_local);
                const double L = fx_to_double(S);
                if (tid == 0) {
                    F.ctl->L = L;
                    F.ctl->L_local = fx_to_double(F.ll_rec ? reinterpret_cast<const RecHeader *>(F.local_rec)->L_local : Sloc);
                    const double b = F.best[F.par];
                    const bool better = L > b;
                    F.best[F.par ^ 1] = better ? L : b;
                    if (better) *F.have_best = 1;
                    F.ctl->snap_pend = better ? 1 : 0;
                }
            } else if (F.snap_clear && tid == 0) {
                F.ctl->snap_pend = 0;
            }
            if (F.local_rec) {  // the local record's deltas (sparse when it is the record just read)
                int32_t *delta = reinterpret_cast<int32_t *>(F.local_rec + kRecHeaderBytes);
                if (F.local_rec == F.recs) {
#pragma unroll
                    for (int q = 0; q < kFinPre; ++q)
                        if (s0 + q < s1 && d0[q] != 0) delta[s0 + q] = 0;
                } else {
                    for (int s = tid; s < kcap; s += kFinThreads) delta[s] = 0;
                    if (tid == 0) reinterpret_cast<RecHeader *>(F.local_rec)->nreq = 0;
                }
            }
            if (tid == 0) {
                F.ctl->qwaves = 0;
                if (F.prior == kPriorNiw) F.ctl->n_pend = 0;
                if (F.moved_mirror) *F.moved_mirror = F.ctl->moved;
                if (F.mirror && F.peak_out) {  // (a replay's last step) the requests' peak over the replay, then anew
                    F.mirror[2] = max(F.ctl->req_peak, peak);
                    F.ctl->req_peak = 0;
                }
                if (F.advance) F.ctl->t_base += F.advance;
            }
            return stale_f;
        }
    }
    if (tid == 0) {
        int n = 0, nall = 0;
        for (int r = 0; r < F.world; ++r) {
            base[r] = n;
            const RecHeader *h = rec_header(F, r);
            const int nr = min(r == 0 ? nreq0 : h->nreq, F.rec_cap);
            n += nr;
            nall += max(nr, h->nreq_all);
        }
        base[F.world] = n;
        s_flags[0] = n;
        s_flags[1] = 0;
        s_flags[2] = nall;
    }
    // (slot s0 + q for q < kFinPre from the registers -- unrolled, static indices -- then any further ones)
#pragma unroll
    for (int q = 0; q < kFinPre; ++q) {
        const int s = s0 + q;
        if (s < s1) {
            int c = cold[q] + d0[q];
            for (int r = 1; r < F.world; ++r) c += rec_delta(F, r)[s];
            cnt_s[s] = c;
        }
    }
    for (int s = s0 + kFinPre; s < s1; ++s) {
        int c = F.cnt[s];
        for (int r = 0; r < F.world; ++r) c += rec_delta(F, r)[s];
        cnt_s[s] = c;
    }
    __syncthreads();
    FIN_T(3)
    const int nreq = s_flags[0];
    int nf = 0, nfree = 0, frank = 0;
    if (nreq > 0) {  // block-uniform: the free slots are only needed when there are requests
        for (int s = s0; s < s1; ++s) nf += (cnt_s[s] == 0);
        frank = block_excl_scan(nf, sh, &nfree);
    }
    const int A = min(min(nreq, F.req_max), nfree);  // accepted this step (block-uniform)
    FIN_T(4)
    if (tid == 0) {
        F.ctl->n_new += A;
        F.ctl->n_rejected += s_flags[2] - A;  // (every rank's requests, also those its selection did not send)
    }
    if (A > 0) {  // block-uniform
        // the A requests of lowest scan position: all of them, or those up to the A-th smallest
        const int64_t T = (nreq > A) ? select_kth_pos([&](int q) { return request_pos(F, base, q); }, nreq, A,
                                                      freeslot, sh)
                                     : INT64_MAX;
        for (int q = tid; q < nreq; q += kFinThreads) {
            const int64_t pos = request_pos(F, base, q);
            if (pos > T) continue;
            const int o = atomicAdd(&s_flags[1], 1);
            keys[o] = pos;
            kidx[o] = q;
        }
        __syncthreads();
        int n2 = 1;
        while (n2 < A) n2 <<= 1;
        for (int q = A + tid; q < n2; q += kFinThreads) {
            keys[q] = INT64_MAX;
            kidx[q] = -1;
        }
        for (int s = s0; s < s1; ++s)
            if (cnt_s[s] == 0) {
                if (frank < A) freeslot[frank] = s;
                ++frank;
            }
        __syncthreads();
        for (int k = 2; k <= n2; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int q = tid; q < n2; q += kFinThreads) {
                    const int l = q ^ j;
                    if (l > q) {
                        const bool up = ((q & k) == 0);
                        const int64_t a = keys[q], b = keys[l];
                        if ((a > b) == up) {
                            keys[q] = b;
                            keys[l] = a;
                            const int t = kidx[q];
                            kidx[q] = kidx[l];
                            kidx[l] = t;
                        }
                    }
                }
                __syncthreads();
            }
        }
        FIN_T(5)
        for (int q = tid; q < A; q += kFinThreads) {
            const Request r = *request_at(F, base, (int)NP8_CHK(kidx[q], 0, kReqMax * 64));
            const int s = (int)NP8_CHK(freeslot[q], 0, kcap);
            if (F.prior == kPriorNiw || F.frame_payload) {
                // built by np8_niw_aux_slots (NIW: O(D^3) per slot) or np8_frame_slots (the wide path's (v, mu)
                // from the item frame): registers this one workgroup cannot spare
                int64_t *pe = F.pend + 4 * (int64_t)q;
                pe[0] = reinterpret_cast<const unsigned char *>(request_vmu(F, base, kidx[q])) - F.recs;
                pe[1] = r.i;
                pe[2] = r.m;
                pe[3] = s;
            }  // (else: the slot's parameters below, spread over the workgroup)
            if (F.wdirty) F.wdirty[s] = 1;
            if (F.ll_on) llv = fx_add(llv, r.dll);  // (exact: any order)
            if (F.ll_defer) {  // (np8_ll_fix_wide: the requester's ll moves from its old slot to this one)
                F.pend_ll[2 * (int64_t)q] = r.zold;
                F.pend_ll[2 * (int64_t)q + 1] = r.lpos;
            }
            cnt_s[s] = 1;
            atomicSub(&cnt_s[NP8_CHK(r.zold, 0, kcap)], 1);  // a live slot (the requester is in it), never a free one
            const int64_t item = key_item(r.i);
            if (item >= F.offset && item < F.offset + F.n_loc) {
                F.z[item - F.offset] = s;
                if (F.zs[0] && r.lpos >= 0) F.zs[0][NP8_CHK(r.lpos, 0, F.n_loc)] = s;
            }
        }
        if (!(F.prior == kPriorNiw || F.frame_payload)) {  // block-uniform; kidx / freeslot final since the sort
            const int ne = new_slot_elems(D);
            for (int e = tid; e < A * ne; e += kFinThreads) {
                const int q = e / ne;
                write_new_slot_elem(F, request_vmu(F, base, kidx[q]), freeslot[q], e - q * ne);
            }
        }
    }
    __syncthreads();
    // write counts back and rebuild the dense candidate table in ascending slot order
    FIN_T(6)
    int nl = 0, lchange = 0;
#pragma unroll
    for (int q = 0; q < kFinPre; ++q) {
        const int s = s0 + q;
        if (s < s1) {
            nl += (cnt_s[s] > 0);
            lchange |= ((cnt_s[s] > 0) != (cold[q] > 0));  // a slot became live or empty
        }
    }
    for (int s = s0 + kFinPre; s < s1; ++s) {
        nl += (cnt_s[s] > 0);
        lchange |= ((cnt_s[s] > 0) != (F.cnt[s] > 0));
    }
    // the live rows keep their order and parameters unless a slot changed liveness, requests were
    // accepted or the state was uploaded: then mu/P' of every row are copied below
    const bool copy_rows = __syncthreads_or(lchange | (A > 0 ? 1 : 0) | (cand_fresh ? 0 : 1)) != 0;
    int nlive;
    int k = block_excl_scan(nl, sh, &nlive);
    // slot s -> its dense row, counts and the row's scalar fields (the prefetched entries unless this step
    // created slots, whose entries were written above)
    int viol = 0;
    auto write_slot = [&](int s, double cs, double iso, double lb0, double lb1) {
        const int c = cnt_s[s];
        F.cnt[s] = c;
        F.dense_of[s] = (c > 0) ? k : -1;
        if (c > 0) {
            double *e = F.cand + (int64_t)k * CS + D + DP;
            const double l1 = (c > 1) ? log_pos((double)(c - 1)) : kZeroLogWeight;
            const double l0 = log_pos((double)c);
            if (F.slack_test && !(fabs(l0 - lb0) <= 0.5 * kListSlack && fabs(l1 - lb1) <= 0.5 * kListSlack)) viol = 1;
            e[kFieldC] = cs;
            e[kFieldLogn] = l0;
            e[kFieldLogn1] = l1;
            F.slot_logn1[s] = l1;
            e[kFieldSlot] = (double)s;
            e[kFieldIso] = iso;
            live_s[k] = s;
            ++k;
        }
    };
#pragma unroll
    for (int q = 0; q < kFinPre; ++q) {
        const int s = s0 + q;
        if (s < s1) write_slot(s, A == 0 ? pc[q] : F.slot_c[s], A == 0 ? piso[q] : F.slot_iso[s], plb0[q], plb1[q]);
    }
    for (int s = s0 + kFinPre; s < s1; ++s)
        write_slot(s, F.slot_c[s], F.slot_iso[s], F.slack_test ? F.lb[s] : 0.0, F.slack_test ? F.lb[kcap + s] : 0.0);
    const int stale = __syncthreads_or(viol) != 0 || copy_rows;
    FIN_T(7)
    // mu and P' of every live row, all threads (not on the wide path: its kernels read the fp32 factor
    // rows of np8_wide_rows, and 4 MB of P' at D = 64 would keep this one workgroup busy for 0.3 ms)
    const int W = D + DP;
    for (int idx = tid; idx < ((F.frame_payload || !copy_rows) ? 0 : nlive * W); idx += kFinThreads) {
        const int r = idx / W, f = idx - r * W, s = live_s[r];
        F.cand[(int64_t)r * CS + f] = (f < D) ? F.slot_mu[(int64_t)s * D + f] : F.slot_P[(int64_t)s * DP + (f - D)];
    }
    FIN_T(8)
    if (tid == 0) {
        F.ctl->K = nlive;
        F.ctl->qwaves = 0;  // np8_assign_fast's deferred waves of this step are done
        F.ctl->cand_fresh = 1;
        F.ctl->n_pend = (F.prior == kPriorNiw || F.frame_payload) ? A : 0;
    }
    // folded max-likelihood check (np_mcmc.cpp:172-174, 187-203): L = the ranks' sums of the assign's per-item
    // log-likelihoods (requesters under their old slot) + the accepted requests' dll, in position order; the
    // labelling is snapshotted on improvement by the next np8_assign_fast (ctl->snap_pend)
    if (F.ll_on) {
        __shared__ Fx shfx[16];
        Fx S = block_sum_fx(llv, shfx);  // (one rank: partials + accepted requests' dll; sharded: the dll only)
        Fx Sloc = S;
        if (F.ll_rec)
            for (int r = 0; r < F.world; ++r) S = fx_add(S, rec_header(F, r)->L_local);
        const double L = fx_to_double(S);
        if (F.ll_defer) {
            if (tid == 0) {  // (np8_ll_fix_wide completes it and decides)
                F.ctl->L_fx_lo = S.lo;
                F.ctl->L_fx_hi = S.hi;
            }
        } else if (tid == 0) {
            F.ctl->L = L;
            F.ctl->L_local = fx_to_double(F.ll_rec ? reinterpret_cast<const RecHeader *>(F.local_rec)->L_local : Sloc);
            const double b = F.best[F.par];
            const bool better = L > b;
            F.best[F.par ^ 1] = better ? L : b;
            if (better) *F.have_best = 1;
            F.ctl->snap_pend = better ? 1 : 0;
        }
    } else if (F.snap_clear && tid == 0) {
        F.ctl->snap_pend = 0;
    }
    // clear the local record for the next step (all reads of it are behind the barriers above)
    if (F.local_rec) {
        int32_t *delta = reinterpret_cast<int32_t *>(F.local_rec + kRecHeaderBytes);
        for (int s = tid; s < kcap; s += kFinThreads) delta[s] = 0;
        if (tid == 0) reinterpret_cast<RecHeader *>(F.local_rec)->nreq = 0;
    }
    if (tid == 0) {
        if (F.moved_mirror) *F.moved_mirror = F.ctl->moved;  // (host-mapped: the host's lagged re-sort decision)
        if (F.mirror && F.peak_out) {
            F.mirror[2] = max(F.ctl->req_peak, peak);
            F.ctl->req_peak = 0;
        }
        if (F.advance) F.ctl->t_base += F.advance;  // nothing after this step reads t_base before the next replay
    }
#ifdef NP8_EXP_FIN_TIMING
    FIN_T(9)
    if (tid == 0)
        printf("fin nreq %d A %d nlive %d copy %d ph %lld %lld %lld %lld %lld %lld %lld %lld %lld\n", nreq, A, nlive,
               (int)copy_rows, ftm[1] - ftm[0], ftm[2] - ftm[1], ftm[3] - ftm[2], ftm[4] - ftm[3],
               ftm[5] ? ftm[5] - ftm[4] : 0ll, ftm[6] - (ftm[5] ? ftm[5] : ftm[4]), ftm[7] - ftm[6], ftm[8] - ftm[7],
               ftm[9] - ftm[8]);
#endif
    return stale;
}

__global__ __launch_bounds__(kFinThreads) void np8_finalize(FinArgs F) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    (void)finalize_block(F, smem);
}

// np8_prune's work for one workgroup of kFinThreads: every live row's list, after the radius buffers'
// bookkeeping.  Runs after finalize_block in the same workgroup (the table it reads is behind a barrier).  The
// rows' fields the bound needs are staged in LDS first (the finalize scratch, free by now; structure of arrays,
// lane j reads row j's), so one wave per row walks them without a dependent global load per row; the
// arithmetic is prune_row's, operation for operation.  Tables too large for the LDS take prune_row itself.
template <int D>
__device__ void prune_block(const PruneArgs &A, unsigned char *smem, size_t lds_bytes) {
    constexpr int DP = D * (D + 1) / 2, CS = (D + DP + 5 + 1) & ~1, F = D + DP;
    constexpr int RW = D + 7;  // mu[D] | c + log n | c + log(n - 1) | iso | R^2 | slot | log n | log(n - 1)
    __syncthreads();
    const int K = A.ctl->K;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), nwb = kFinThreads / 64;
    if (tid == 0) A.ctl->lists_ok = 1;
    const double *src = A.r2 + (A.gathered ? A.kcap : 0);
    auto R2of = [&](int slot) { return src[slot]; };
    if ((size_t)K * RW * sizeof(double) > lds_bytes) {
        for (int k0 = wid; k0 < K; k0 += nwb)  // wave-uniform
            prune_row<D>(A.cand, R2of, A.plist, A.pdist, A.plen, A.plr2, A.plen_s, A.plr2_s, A.ls, A.D, K, k0, A.lb, A.kcap, A.lam);
    } else {
        double *st = reinterpret_cast<double *>(smem);
        for (int idx = tid; idx < K * RW; idx += kFinThreads) {
            const int r = idx / RW, f = idx - r * RW;
            const double *e = A.cand + (int64_t)r * CS;
            double v;
            if (f < D)
                v = e[f];
            else if (f == D)
                v = e[F + kFieldC] + e[F + kFieldLogn];
            else if (f == D + 1)
                v = e[F + kFieldC] + e[F + kFieldLogn1];
            else if (f == D + 2)
                v = e[F + kFieldIso];
            else if (f == D + 3)
                v = src[(int)e[F + kFieldSlot]];
            else if (f == D + 4)
                v = e[F + kFieldSlot];
            else if (f == D + 5)
                v = e[F + kFieldLogn];
            else
                v = e[F + kFieldLogn1];
            st[f * K + r] = v;
        }
        __syncthreads();
        for (int k0 = wid; k0 < K; k0 += nwb) {  // wave-uniform: one row per wave
            const int slot0 = (int)st[(D + 4) * K + k0];
            const double R2 = st[(D + 3) * K + k0];
            const double iso0 = st[(D + 2) * K + k0];
            const double base0 = st[(D + 1) * K + k0];
            const bool prunable = iso0 > 0.0 && R2 < 1e300 && base0 > -1e299;
            const double R = sqrt(R2);
            int count = 0;
            for (int jb = 0; jb < K; jb += 64) {
                const int j = jb + lane;
                bool keep = j < K && j != k0;
                if (j < K) {
                    double dist2 = 0.0;
#pragma unroll
                    for (int a = 0; a < D; ++a) {
                        const double dd = st[a * K + j] - st[a * K + k0];
                        dist2 = fma(dd, dd, dist2);
                    }
                    if (A.pdist) A.pdist[(int64_t)k0 * A.ls + j] = f32_down(sqrt(dist2));
                    const double isoj = st[(D + 2) * K + j];
                    if (keep && prunable && isoj > 0.0) {
                        const double delta = sqrt(dist2) - R;
                        if (delta > 0.0) {
                            const double wj = st[D * K + j];
                            const double far = 0.5 * isoj * delta * delta, near = 0.5 * iso0 * R2;
                            const double U = (wj - base0) - far + near;
                            const double mag = fabs(wj) + fabs(base0) + far + near;
                            keep = !(U <= -kSkip - 2.0 - kListSlack - 1e-9 * mag);
                        }
                    }
                }
                const uint64_t b = __ballot(keep);
                if (keep) A.plist[(int64_t)k0 * A.ls + count + __popcll(b & ((1ull << lane) - 1ull))] = j;
                count += __popcll(b);
            }
            if (lane == 0) {
                const double r2l = prunable ? R2 : __longlong_as_double(0x7FF0000000000000ll);  // +inf: every row listed
                A.plen[k0] = count;
                A.plr2[k0] = r2l;
                A.plen_s[slot0] = count;
                A.plr2_s[slot0] = r2l;
                if (A.lb) {
                    A.lb[slot0] = st[(D + 5) * K + k0];
                    A.lb[A.kcap + slot0] = st[(D + 6) * K + k0];
                }
            }
        }
    }
    __syncthreads();  // the radius buffers' bookkeeping after every read of src
    if (A.gathered)
        for (int s = tid; s < A.kcap; s += kFinThreads) A.r2[s] = A.r2[A.kcap + s];
    if (A.clear_next)  // only the radii in use were read (not gathered)
        for (int s = tid; s < A.kcap; s += kFinThreads) A.r2[A.kcap + s] = 0.0;
}

namespace {

// The end of a synchronous step in one launch (DESIGN.md §5 "Fewer launches"): the lanes np8_assign_fast deferred
// (np8_assign_queue's work, T.queue), the step's radius records folded into the gathered radii (np8_fold_r2,
// T.fold), then -- in the one workgroup that finishes last (a release/acquire counter, no workgroup waits for
// another) -- the request selection of a sharded step (np8_req_select, T.select) or np8_finalize (T.fin) followed
// by the candidate lists (np8_prune, T.prune).  Each part does what its own kernel did, in the same order, so the
// chain is unchanged; the separate kernels remain for the other step kinds.
template <int D>
__global__ __launch_bounds__(kFinThreads) void np8_step_tail(AssignArgs A, FinArgs F, PruneArgs P, TailArgs T) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int s_last;
    const int lane = threadIdx.x & 63;
    if (T.fold) {  // np8_fold_r2, one record per thread (both it and the queue's lanes only raise the radii)
        unsigned long long *g = reinterpret_cast<unsigned long long *>(F.r2 + F.kcap);
        const int64_t nf = (T.fold_n + 63) & ~63ll;  // whole waves (the shuffles below)
        for (int64_t k = (int64_t)blockIdx.x * kFinThreads + threadIdx.x; k < nf; k += (int64_t)gridDim.x * kFinThreads) {
            WaveR2 r;
            r.slot = -1;
            r.d2 = 0.0;
            if (k < T.fold_n) r = A.wr2[k];
            unsigned long long m = r.slot >= 0 ? (unsigned long long)__double_as_longlong(r.d2) : 0ull;
            const int32_t s0 = __builtin_amdgcn_readfirstlane(r.slot);
            if (__ballot(r.slot >= 0 && r.slot != s0) == 0ull) {  // the wave's records are one slot: one atomic
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const unsigned long long v = __shfl_xor(m, o);
                    m = v > m ? v : m;
                }
                if (lane == 0 && s0 >= 0) atomicMax(g + s0, m);
            } else if (r.slot >= 0) {
                atomicMax(g + r.slot, m);
            }
        }
    }
    __syncthreads();  // this workgroup's records are folded
    if (gridDim.x > 1) {  // the workgroup that finishes last runs the serial part
        if (threadIdx.x == 0) {
            __threadfence();  // release this workgroup's writes (labels, records, radii) at device scope
            const unsigned prev = atomicAdd(&A.ctl->tail_done, 1u);
            s_last = prev == gridDim.x - 1;
            if (s_last) {
                __threadfence();  // acquire the other workgroups' writes
                A.ctl->tail_done = 0u;
            }
        }
        __syncthreads();
        if (!s_last) return;
        __threadfence();
    }
    if (T.select)
        req_select_block(T.stage, T.stage_cap, T.rec, T.rec_cap, F.kcap, D, F.req_max, nullptr, 0,
                         reinterpret_cast<int *>(smem));
    int stale = 1;
    if (T.fin) stale = finalize_block(F, smem);
    if (stale < 0) return;  // a halted compact graph: nothing applied, no lists
    if (T.prune == 1 || (T.prune == 2 && stale)) {
        prune_block<D>(P, smem, T.lds_bytes);
        if (T.prune == 2 && threadIdx.x == 0) P.ctl->list_builds += 1u;
    } else if (T.prune == 2) {  // the lists stay: only the radius buffers' bookkeeping (never a gathering step here)
        if (P.clear_next)
            for (int s = threadIdx.x; s < P.kcap; s += kFinThreads) P.r2[P.kcap + s] = 0.0;
    }
}

// Finalize and the candidate lists in one launch with the lists still built in parallel (DESIGN.md §5 "Fewer
// launches"): workgroup 0 runs np8_finalize's body, then releases a flag (agent scope); workgroups 1 .. nP wait
// for it (bounded spin: a workgroup that gives up sets kErrSpin and builds nothing) and build one list per wave,
// prune_row's arithmetic, as np8_prune's workgroups do.  Every workgroup is resident at once (nP <= 8 on 256
// CUs; workgroup 0 is dispatched first), so the wait always ends.  The last prune workgroup to finish resets the
// flag and the exit counter for the next launch.  Saves one dependent kernel dispatch per sweep.
constexpr int kFpPruneBlocks = 8;
template <int DT>
__global__ __launch_bounds__(kFinThreads) void np8_fin_prune(FinArgs F, PruneArgs P, int nP) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int s_ok;
    if (blockIdx.x == 0) {
        finalize_block(F, smem);
        __syncthreads();
        // np8_prune's first-workgroup duties: the radius buffers (the lists read the other half of r2) and lists_ok
        if (P.gathered)
            for (int s = threadIdx.x; s < P.kcap; s += kFinThreads) P.r2[s] = P.r2[P.kcap + s];
        if (P.clear_next)
            for (int s = threadIdx.x; s < P.kcap; s += kFinThreads) P.r2[P.kcap + s] = 0.0;
        if (threadIdx.x == 0) {
            P.ctl->lists_ok = 1;
            __threadfence();
            __hip_atomic_store(&F.ctl->fin_flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (threadIdx.x == 0) {
        int ok = 0;
        for (int it = 0; it < (1 << 22); ++it) {
            if (__hip_atomic_load(&F.ctl->fin_flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
                ok = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) {  // the lists this workgroup owes are not built: the assign must walk the whole table
            atomicOr(&F.ctl->err, kErrSpin);
            __hip_atomic_store(&P.ctl->lists_ok, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_ok = ok;
    }
    __syncthreads();
    __threadfence();  // every wave: acquire what workgroup 0 wrote (the table, K)
    if (s_ok) {
        const int K = __hip_atomic_load(&P.ctl->K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double *src = P.r2 + (P.gathered ? P.kcap : 0);
        auto R2of = [&](int slot) { return src[slot]; };
        constexpr int kWaves = kFinThreads / 64;
        for (int k0 = ((int)blockIdx.x - 1) * kWaves + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); k0 < K;
             k0 += nP * kWaves)  // wave-uniform (readfirstlane: SGPR loop)
            prune_row<DT>(P.cand, R2of, P.plist, P.pdist, P.plen, P.plr2, P.plen_s, P.plr2_s, P.ls, P.D, K, k0, P.lb, P.kcap, P.lam);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&F.ctl->prune_exit, 1u) == (unsigned)nP - 1u) {  // the last one: reset for the next launch
            atomicExch(&F.ctl->prune_exit, 0u);
            atomicExch(&F.ctl->fin_flag, 0u);
        }
    }
}

}  // namespace

// The wide path's new slots under the reference prior: (v, mu) of each accepted request from the item frame
// its rank recorded, then the slot (what np8_finalize did in place before: 2.7 KB of scratch per lane there).
// One thread per pending request (ctl->n_pend, listed by np8_finalize).
__global__ __launch_bounds__(64) void np8_frame_slots(FinArgs F) {
    const int n = F.ctl->n_pend;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
        const int64_t *pe = F.pend + 4 * (int64_t)q;
        const double *frame = reinterpret_cast<const double *>(F.recs + pe[0]);
        double vmu[kMaxD + 1];
        const int sl = (int)pe[3];
        frame_to_vmu(F, frame, pe[1], (int)pe[2], vmu);
        write_new_slot(F, vmu, sl);
        // np8_finalize built the slot's dense row before its parameters existed: its scalars now
        double *e = F.cand + (int64_t)F.dense_of[sl] * cand_stride(F.D) + F.D + F.D * (F.D + 1) / 2;
        e[kFieldC] = F.slot_c[sl];
        e[kFieldIso] = F.slot_iso[sl];
    }
}

hipError_t np8_launch_frame_slots(const FinArgs &F, hipStream_t s) {
    hipLaunchKernelGGL(np8_frame_slots, dim3(64), dim3(64), 0, s, F);
    return hipGetLastError();
}

// ---- max likelihood --------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void np8_loglik(LoglikArgs A) {
    constexpr int DP = D * (D + 1) / 2;
    constexpr int CS = (D + DP + 5 + 1) & ~1;
    __shared__ double red[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double ll = 0.0;
    if (i < A.n_loc) {
        double x[D];
#pragma unroll
        for (int a = 0; a < D; ++a) x[a] = A.X[(int64_t)a * A.n_loc + i];
        ll = cand_ll<D>(A.cand + (int64_t)A.dense_of[A.z[i]] * CS, x);
    }
    red[threadIdx.x] = ll;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) A.partial[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(1024) void np8_loglik_reduce(const double *__restrict__ partial, int64_t nb,
                                                          double *__restrict__ out, double *__restrict__ out2) {
    __shared__ double red[1024];
    double s = 0.0;
    for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) s = s + partial[b];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *out = red[0];
        if (out2) *out2 = red[0];  // one rank: the global sum too
    }
}

// Every block decides from (L, best[par]); block 0 publishes best[par^1].
__global__ __launch_bounds__(256) void np8_snapshot(SnapArgs A) {
    const double L = *A.L;
    const double best = A.best[A.par];
    const bool better = L > best;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.best[A.par ^ 1] = better ? L : best;
        if (better) *A.have_best = 1;
    }
    if (!better) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) A.ctl->best_sorted = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.n_loc; i += stride)
        A.z_best[i] = A.z[i];
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < A.kcap; k += stride) A.cnt_best[k] = A.cnt[k];
    const int64_t nm = (int64_t)A.kcap * A.D, ns = (int64_t)A.kcap * A.D * A.D;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nm; k += stride) A.mu_best[k] = A.slot_mu[k];
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < ns; k += stride)
        A.sigma_best[k] = A.slot_sigma[k];
}

// A snapshot the folded check left pending (ctl->snap_pend, consumed otherwise by the next np8_assign_fast): the
// labelling, counts and parameters as they stand; the host clears the flag behind this launch.
__global__ __launch_bounds__(256) void np8_snapshot_flush(SnapArgs A, const Ctl *__restrict__ ctl) {
    if (!ctl->snap_pend || ctl->halt) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x, g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0) A.ctl->best_sorted = 0;
    for (int64_t i = g; i < A.n_loc; i += stride) A.z_best[i] = A.z[i];
    for (int64_t k = g; k < A.kcap; k += stride) A.cnt_best[k] = A.cnt[k];
    const int64_t nm = (int64_t)A.kcap * A.D, ns = (int64_t)A.kcap * A.D * A.D;
    for (int64_t k = g; k < nm; k += stride) A.mu_best[k] = A.slot_mu[k];
    for (int64_t k = g; k < ns; k += stride) A.sigma_best[k] = A.slot_sigma[k];
}

// ---- cluster-parameter update (mh_g0) ------------------------------------------------------------------
// UpdateClusters::update (src/np_update_clusters.cpp:71-142) from sufficient statistics; formulas in
// oracle/np8_oracle.c (np8o_param_update) and DESIGN.md "Parameter update".

// Per-slot statistics about the slot mean.  One wave per block covers kSuffRows rows of 64
// consecutive positions (all loads issued up front).  For each distinct slot among its items -- one
// on the label-sorted layout, a few where items moved since the last re-sort -- every lane sums its
// items of that slot, the per-lane sums are transposed through LDS, lane c adds up component c and
// the wave issues ONE contiguous atomic wave-instruction.  (Float atomics run at the memory side at
// a fixed instruction rate, MI355X_MICROARCH.md "Global float atomics", so one-lane atomics per
// component were the first bottleneck; DPP/readlane reductions of 44 components the second.)
constexpr int kSuffRows = 4;

// Column sums of T[w][0..63] for w = lane (+64 q), then one atomic add per component into dst.
template <int W>
__device__ __forceinline__ void suff_commit(double (*T)[65], int lane, double *dst) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < (W + 63) / 64; ++q) {
        const int c = lane + 64 * q;
        if (c < W) {
            double r0 = 0.0, r1 = 0.0, r2 = 0.0, r3 = 0.0;
#pragma unroll 4
            for (int k = 0; k < 64; k += 4) {
                r0 += T[c][k];
                r1 += T[c][k + 1];
                r2 += T[c][k + 2];
                r3 += T[c][k + 3];
            }
            unsafeAtomicAdd(dst + c, (r0 + r1) + (r2 + r3));
        }
    }
    __syncthreads();
}

template <int D>
__global__ __launch_bounds__(64) void np8_suffstats(ParamArgs A) {
    constexpr int W = D + D * (D + 1) / 2;
    __shared__ double T[W][65];
    const int lane = threadIdx.x;
    const bool sorted = A.sorted != 0;
    constexpr int cur = 0;  // the label-sorted layout is always buffer 0 (buffer 1: the re-sort's scratch)
    const double *__restrict__ X = sorted ? (cur ? A.Xs[1] : A.Xs[0]) : A.X;
    const int32_t *__restrict__ z = sorted ? (cur ? A.zs[1] : A.zs[0]) : A.z;
    const int64_t n = A.n_loc;
    const int64_t base = (int64_t)blockIdx.x * (64 * kSuffRows) + lane;
    double x[kSuffRows][D];
    int32_t s[kSuffRows];
    uint64_t pend[kSuffRows];
#pragma unroll
    for (int j = 0; j < kSuffRows; ++j) {
        const int64_t p = base + 64 * j;
        const bool v = p < n;
        s[j] = v ? z[p] : -1;
#pragma unroll
        for (int a = 0; a < D; ++a) x[j][a] = v ? X[(int64_t)a * n + p] : 0.0;
        pend[j] = __ballot(v);
    }
    // one pass per distinct slot of the wave's items (one pass on the label-sorted layout, a few
    // where items moved since the last re-sort)
    for (;;) {
        int jr = -1;
#pragma unroll
        for (int j = kSuffRows - 1; j >= 0; --j)
            if (pend[j]) jr = j;
        if (jr < 0) break;
        uint64_t pm = pend[0];
        int32_t sr = s[0];
#pragma unroll
        for (int j = 1; j < kSuffRows; ++j) {
            pm = (jr == j) ? pend[j] : pm;
            sr = (jr == j) ? s[j] : sr;
        }
        const int32_t g = __shfl(sr, __ffsll((unsigned long long)pm) - 1);
        double mu[D];
#pragma unroll
        for (int a = 0; a < D; ++a) mu[a] = A.slot_mu[(int64_t)g * D + a];
        double acc[W];
#pragma unroll
        for (int w = 0; w < W; ++w) acc[w] = 0.0;
#pragma unroll
        for (int j = 0; j < kSuffRows; ++j) {
            const bool mine = s[j] == g;
            pend[j] &= ~__ballot(mine);
            double d[D];
#pragma unroll
            for (int a = 0; a < D; ++a) d[a] = mine ? x[j][a] - mu[a] : 0.0;
            int k = 0;
#pragma unroll
            for (int a = 0; a < D; ++a, ++k) acc[k] += d[a];
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int b = a; b < D; ++b, ++k) acc[k] = fma(d[a], d[b], acc[k]);
        }
#pragma unroll
        for (int w = 0; w < W; ++w) T[w][lane] = acc[w];
        suff_commit<W>(T, lane, A.acc + (int64_t)g * W);
    }
}

// G0 independence proposal `step` of slot s: the auxiliary-draw layout on stream PARAM.
template <int D>
__device__ __forceinline__ void mh_proposal(const ParamArgs &A, uint32_t t, int s, int step, double &v,
                                            double (&mup)[D]) {
    constexpr int Q = (D + 4) / 4;  // g0_calls(D)
    double gq[4] = {0.0, 0.0, 0.0, 0.0}, xi[D];
#pragma unroll
    for (int k = 0; k <= D; ++k) {
        if ((k & 3) == 0) normal_quad(A.seed, (uint64_t)s, t, kStreamParam, (uint32_t)(step * Q + (k >> 2)), gq);
        const double g = gq[k & 3];
        if (k == 0)
            v = fma(A.nu, g, (double)D);
        else
            xi[k - 1] = g;
    }
    const double sc = fabs(v) * A.rsk;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double t0 = A.LT[a * D + a] * xi[a];
#pragma unroll
        for (int b = a + 1; b < D; ++b) t0 = fma(A.LT[a * D + b], xi[b], t0);
        mup[a] = fma(sc, t0, A.mu0[a]);
    }
}

__device__ __forceinline__ int packed_ix(int D, int a, int b) { return a * D - (a * (a - 1)) / 2 + (b - a); }

// One wave per slot: the proposals of up to 64 MH steps are evaluated in parallel (their
// likelihoods do not depend on the chain), then lane 0 walks the accept/reject sequence.
template <int D>
__global__ __launch_bounds__(64) void np8_mh_g0(ParamArgs A) {
    constexpr int DP = D * (D + 1) / 2, W = D + DP;
    const int s = blockIdx.x;
    const int n = A.cnt[s];
    if (n <= 0) return;
    const int lane = threadIdx.x;
    const uint32_t t = A.ctl->t_base + A.t;
    __shared__ double st[W];
    __shared__ double llp[64], up[64];
    __shared__ double s_LL;
    __shared__ int s_chosen, s_nacc;
    for (int w = lane; w < W; w += 64) {
        st[w] = A.acc[(int64_t)s * W + w];
        A.acc[(int64_t)s * W + w] = 0.0;  // leaves the buffer zeroed for the next sweep
    }
    __syncthreads();
    const double *s1 = st, *S = st + D;
    const double *Pp = A.slot_P + (int64_t)s * DP;
    double anchor[D], g1[D];
#pragma unroll
    for (int a = 0; a < D; ++a) anchor[a] = A.slot_mu[(int64_t)s * D + a];
    double trPS = 0.0, trGS = 0.0;
#pragma unroll
    for (int k = 0; k < DP; ++k) {
        trPS = fma(Pp[k], S[k], trPS);
        trGS = fma(A.Gp[k], S[k], trGS);
    }
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double acc = 0.0;
#pragma unroll
        for (int b = 0; b < D; ++b) {
            const double G = (a == b) ? A.Gp[packed_ix(D, a, a)] : 0.5 * A.Gp[packed_ix(D, min(a, b), max(a, b))];
            acc = fma(G, s1[b], acc);
        }
        g1[a] = acc;
    }
    const double nd = (double)n;
    if (lane == 0) {
        s_LL = fma(-0.5, trPS, nd * A.slot_c[s]);
        s_chosen = -1;
        s_nacc = 0;
    }
    for (int b0 = 0; b0 < A.steps; b0 += 64) {
        const int step = b0 + lane;
        if (step < A.steps) {
            double v, mup[D];
            mh_proposal<D>(A, t, s, step, v, mup);
            double e[D], eg = 0.0, eGe = 0.0;
#pragma unroll
            for (int a = 0; a < D; ++a) {
                e[a] = mup[a] - anchor[a];
                eg = fma(e[a], g1[a], eg);
            }
            int k = 0;
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int b = a; b < D; ++b) eGe = fma(A.Gp[k++], e[a] * e[b], eGe);
            const double tr = fma(nd, eGe, fma(-2.0, eg, trGS));
            const double cp = fma(-(double)D, log_pos(fabs(v)), A.caux);
            llp[lane] = fma(-0.5, tr / (v * v), nd * cp);
            up[lane] = uniform(A.seed, (uint64_t)s, t, kStreamParamU, (uint32_t)step);
        }
        __syncthreads();
        if (lane == 0) {  // np_update_clusters.cpp:114-137
            double L = s_LL;
            int ch = s_chosen, na = s_nacc;
            const int nb = min(64, A.steps - b0);
            for (int q = 0; q < nb; ++q) {
                const double dl = llp[q] - L;
                if (L == 0.0 || dl >= 0.0 || up[q] < exp_le0(dl)) {
                    L = llp[q];
                    ch = b0 + q;
                    ++na;
                }
            }
            s_LL = L;
            s_chosen = ch;
            s_nacc = na;
        }
        __syncthreads();
    }
    const int ch = s_chosen;
    if (ch < 0) return;  // block-uniform
    double v, mup[D];
    mh_proposal<D>(A, t, s, ch, v, mup);
    const double v2 = v * v;
    const int CS = cand_stride(D);
    const int row = A.dense_of[s];
    double *crow = A.cand + (int64_t)row * CS;
    for (int k = lane; k < DP; k += 64) {
        const double val = A.Gp[k] / v2;
        A.slot_P[(int64_t)s * DP + k] = val;
        crow[D + k] = val;
    }
    for (int k = lane; k < D * D; k += 64) A.slot_sigma[(int64_t)s * D * D + k] = v2 * A.LTL[k];
    if (lane == 0) {
#pragma unroll
        for (int a = 0; a < D; ++a) {
            A.slot_mu[(int64_t)s * D + a] = mup[a];
            crow[a] = mup[a];
        }
        const double c = fma(-(double)D, log_pos(fabs(v)), A.caux);
        const double iso = (A.gp_iso > 0.0) ? A.Gp[0] / v2 : 0.0;
        A.slot_c[s] = c;
        A.slot_iso[s] = iso;
        r2_unknown(A.r2, A.kcap, s);  // the mean moved
        crow[D + DP + kFieldC] = c;
        crow[D + DP + kFieldIso] = iso;
        atomicAdd(reinterpret_cast<unsigned long long *>(&A.ctl->mh_accepted), (unsigned long long)s_nacc);
    }
}

// ---- parity/debug: log-likelihood matrix --------------------------------------------------------------
template <int D, int M, int PRIOR>
__global__ __launch_bounds__(256) void np8_loglik_matrix_kernel(AssignArgs A, const int64_t *__restrict__ idx,
                                                                int64_t n, double *__restrict__ out) {
    constexpr int DP = D * (D + 1) / 2;
    constexpr int CS = (D + DP + 5 + 1) & ~1;
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t il = idx[r];
    const uint64_t ig = (uint64_t)(A.offset + il);
    double x[D];
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = A.X[(int64_t)a * A.n_loc + il];
    const int K = A.ctl->K;
    for (int j = 0; j < K; ++j) out[r * (K + M) + j] = cand_ll<D>(A.cand + (int64_t)j * CS, x);
    double y0[D];
    whiten<D>(A.hyp, x, y0);
    const double ny = norm_of<D>(y0);
    const uint32_t t = A.ctl->t_base + A.t;
    for (int m = 0; m < M; ++m) out[r * (K + M) + K + m] = prior_aux_ll<D, PRIOR>(A.hyp, ny, A.seed, ig, t, m, M);
}

// debug: the level-0 auxiliary bound np8_assign_fast screens with (aux_screen0_ub, without the threshold's own
// margin term) for chosen items, out[r M + m]; tests/test_gpu_screen.py holds it above the exact log-likelihood
template <int D, int M>
__global__ __launch_bounds__(256) void np8_aux_bounds_kernel(AssignArgs A, const int64_t *__restrict__ idx, int64_t n,
                                                             double *__restrict__ out) {
    using H = HypView<D>;
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t il = idx[r];
    const uint64_t ig = (uint64_t)(A.offset + il);
    const double *hyp = A.hyp;
    double x[D], y0[D];
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = A.X[(int64_t)a * A.n_loc + il];
    whiten<D>(hyp, x, y0);
    double n2 = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) n2 = fma(y0[a], y0[a], n2);
    const float nyf = __builtin_amdgcn_sqrtf((float)n2);
    const uint32_t t = A.ctl->t_base + A.t;
    uint32_t pre[4];
    aux_pre_call(A.seed, ig, t, pre);
    float s_abs;
    const float s0 = aux_screen0_s(nyf, (float)hyp[H::kPre], (float)hyp[H::kPre + 1], (float)hyp[H::kPre + 2],
                                   (float)hyp[H::kPre + 3], D, s_abs);
    const float rskf = (float)hyp[H::kRsk], cauxf = (float)hyp[H::kCaux];
    for (int m = 0; m < M; ++m)
        out[r * M + m] = (double)aux_screen0_ub<D, M>(pre, m, s0, s_abs, cauxf, 0.5f * rskf * rskf);
}

// ---- dispatch ----------------------------------------------------------------------------------------
#if defined(NP8_EXP_ONLY_D9)  // (debug builds: the D = 9 instances only)
#define NP8_FOR_EACH_DM(X) X(9, 3)
#elif defined(NP8_EXP_ONLY_D8)  // (A/B experiment builds, tools/ab_build.sh: the C3 instances only, a fast compile)
#define NP8_FOR_EACH_DM(X) X(8, 3)
#else
#define NP8_FOR_EACH_DM(X) \
    X(1, 1) X(1, 2) X(1, 3) X(1, 4) X(2, 1) X(2, 2) X(2, 3) X(2, 4) X(3, 1) X(3, 2) X(3, 3) X(3, 4) X(4, 1) \
    X(4, 2) X(4, 3) X(4, 4) X(8, 1) X(8, 2) X(8, 3) X(8, 4) X(16, 1) X(16, 2) X(16, 3) X(16, 4)         \
    X(5, 3) X(6, 3) X(7, 3) X(9, 3) X(10, 3) X(11, 3) X(12, 3) X(13, 3) X(14, 3) X(15, 3)
#endif

bool np8_supported(int D, int M) {
#define X(d, m) \
    if (D == d && M == m) return true;
    NP8_FOR_EACH_DM(X)
#undef X
    return false;
}

hipError_t np8_launch_assign_fast(const AssignArgs &A, int D, int M, hipStream_t s) {
    const int64_t n = A.p1 - A.p0;
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + NP8_ASSIGN_BLOCK - 1) / NP8_ASSIGN_BLOCK)), block(NP8_ASSIGN_BLOCK);
#define X(d, m)                                                                                          \
    if (D == d && M == m) {                                                                              \
        if (A.count_eval)                                                                                \
            hipLaunchKernelGGL((np8_assign_fast<d, m, kPriorReference, true, false>), grid, block, 0, s, A); \
        else if (A.ll_on)                                                                                \
            hipLaunchKernelGGL((np8_assign_fast<d, m, kPriorReference, false, true>), grid, block, 0, s, A); \
        else                                                                                             \
            hipLaunchKernelGGL((np8_assign_fast<d, m, kPriorReference, false, false>), grid, block, 0, s, A); \
        return hipGetLastError();                                                                        \
    }
    NP8_FOR_EACH_DM(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_assign_queue(const AssignArgs &A, int D, int M, hipStream_t s) {
    const int64_t n = A.p1 - A.p0;
    if (n <= 0) return hipSuccess;
    // walks the listed waves with a grid of at most kQueueBlocks (usually a few waves have work)
    constexpr int64_t kQueueBlocks = 2048;
    int64_t nb = (n + 63) / 64;
    if (nb > kQueueBlocks) nb = kQueueBlocks;
    const dim3 grid((unsigned)nb), block(64);
#define X(d, m)                                                                                           \
    if (D == d && M == m) {                                                                               \
        if (A.count_eval)                                                                                 \
            hipLaunchKernelGGL((np8_assign_queue<d, m, kPriorReference, true>), grid, block, 0, s, A);    \
        else                                                                                              \
            hipLaunchKernelGGL((np8_assign_queue<d, m, kPriorReference, false>), grid, block, 0, s, A);   \
        return hipGetLastError();                                                                         \
    }
    NP8_FOR_EACH_DM(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_assign(const AssignArgs &A, int D, int M, int prior, hipStream_t s) {
    const int64_t n = A.p1 - A.p0;
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + NP8_ASSIGN_BLOCK - 1) / NP8_ASSIGN_BLOCK)), block(NP8_ASSIGN_BLOCK);
#define X(d, m)                                                                                        \
    if (D == d && M == m) {                                                                            \
        if (prior == kPriorNiw)                                                                        \
            hipLaunchKernelGGL((np8_assign<d, m, kPriorNiw, false>), grid, block, 0, s, A);             \
        else if (A.count_eval)                                                                         \
            hipLaunchKernelGGL((np8_assign<d, m, kPriorReference, true>), grid, block, 0, s, A);        \
        else                                                                                           \
            hipLaunchKernelGGL((np8_assign<d, m, kPriorReference, false>), grid, block, 0, s, A);       \
        return hipGetLastError();                                                                      \
    }
    NP8_FOR_EACH_DM(X)
#undef X
    if (prior == kPriorReference && np8_rt_supported(D, M, prior)) return np8_launch_assign_rt(A, D, M, s);
    return hipErrorInvalidValue;
}

bool np8_rt_supported(int D, int M, int prior) {
    return prior == kPriorReference && D > kPreMaxD && D <= kMaxD && M >= 1 && M <= kMaxM && !np8_supported(D, M);
}

// ---- pruning radii: the step's wave records into this sweep's buffer (DESIGN.md "Candidate pruning") ----
// One lane per record (the label-sorted layout makes runs of one slot); a wave whose 64
// records share one slot raises the slot's radius with one atomic, others lane by lane.  Many small waves:
// one workgroup reading all records (250 KB at C3) took 14 us, latency bound.
constexpr int kFoldPer = 1;

__global__ __launch_bounds__(256) void np8_fold_r2(const WaveR2 *__restrict__ wr2, int64_t n, double *r2, int kcap,
                                                   const Ctl *__restrict__ ctl) {
    if (ctl->halt) return;
    const int64_t k0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * kFoldPer;
    unsigned long long *cur = reinterpret_cast<unsigned long long *>(r2 + kcap);
    int32_t sl = -1;
    unsigned long long m = 0ull;
    bool one = true;  // this lane's records share slot sl (or it has none)
#pragma unroll
    for (int u = 0; u < kFoldPer; ++u) {
        if (k0 + u >= n) break;
        WaveR2 r = wr2[k0 + u];
        if (r.slot < 0) continue;
        r.slot = (int32_t)NP8_CHK(r.slot, 0, kcap);
        const unsigned long long b = (unsigned long long)__double_as_longlong(r.d2);
        if (sl < 0 || sl == r.slot) {
            sl = r.slot;
            m = b > m ? b : m;
        } else {
            one = false;
            atomicMax(cur + r.slot, b);
        }
    }
    const int32_t s0 = __builtin_amdgcn_readfirstlane(sl);
    if (__ballot(!one || (sl >= 0 && sl != s0)) == 0ull) {  // the wave's runs are one slot: one atomic
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long v = __shfl_xor(m, o);
            m = v > m ? v : m;
        }
        if ((threadIdx.x & 63) == 0 && s0 >= 0) atomicMax(cur + s0, m);
    } else if (sl >= 0) {
        atomicMax(cur + sl, m);
    }
}

hipError_t np8_launch_fold_r2(const WaveR2 *wr2, int64_t n, double *r2, int kcap, const Ctl *ctl, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t lanes = (n + kFoldPer - 1) / kFoldPer;
    hipLaunchKernelGGL(np8_fold_r2, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, wr2, n, r2, kcap, ctl);
    return hipGetLastError();
}

// ---- debug invariants (np8_check_invariants) -----------------------------------------------------------
__global__ __launch_bounds__(256) void np8_inv_items(const int32_t *__restrict__ z, int64_t n, const int32_t *__restrict__ cnt,
                                                     int kcap, int32_t *__restrict__ hist, unsigned long long *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t s = z[i];
    if (s < 0 || s >= kcap || cnt[s] <= 0) {
        atomicOr(out, 1ull);
        atomicAdd(out + 1, 1ull);
        return;
    }
    atomicAdd(hist + s, 1);
}

__global__ __launch_bounds__(1024) void np8_inv_slots(const int32_t *__restrict__ cnt, const int32_t *__restrict__ dense_of,
                                                      const double *__restrict__ cand, int CS, int D, int kcap,
                                                      int64_t n_global, int check_hist, int32_t *__restrict__ hist,
                                                      unsigned long long *out, Ctl *ctl) {
    __shared__ unsigned long long tot, live;
    __shared__ int bad;
    if (threadIdx.x == 0) {
        tot = live = 0ull;
        bad = 0;
    }
    __syncthreads();
    const int DP = D * (D + 1) / 2;
    for (int s = threadIdx.x; s < kcap; s += blockDim.x) {
        const int c = cnt[s];
        if (c > 0) {
            atomicAdd(&tot, (unsigned long long)c);
            atomicAdd(&live, 1ull);
            const int r = dense_of[s];  // the dense row of a live slot names the slot back
            if (r < 0 || (int)cand[(int64_t)r * CS + D + DP + kFieldSlot] != s) atomicOr(&bad, 8);
        } else if (dense_of[s] >= 0) {
            atomicOr(&bad, 8);
        }
        if (check_hist && hist[s] != (c > 0 ? c : 0)) {
            atomicOr(&bad, 2);
            atomicAdd(out + 2, 1ull);
        }
        hist[s] = 0;  // ready for the next check
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int b = bad;
        if ((int64_t)tot != n_global) b |= 4;
        if ((int64_t)live != ctl->K) b |= 8;
        out[3] = tot;
        if (b) atomicOr(out, (unsigned long long)b);
        if (b || out[0]) atomicOr(&ctl->err, kErrInvariant);
    }
}

hipError_t np8_launch_invariants(const int32_t *z, int64_t n, const int32_t *cnt, const int32_t *dense_of,
                                 const double *cand, int CS, int D, int kcap, int64_t n_global, int check_hist,
                                 int32_t *hist, unsigned long long *out, Ctl *ctl, hipStream_t s) {
    if (n > 0)
        hipLaunchKernelGGL(np8_inv_items, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, z, n, cnt, kcap, hist, out);
    hipLaunchKernelGGL(np8_inv_slots, dim3(1), dim3(1024), 0, s, cnt, dense_of, cand, CS, D, kcap, n_global, check_hist,
                       hist, out, ctl);
    return hipGetLastError();
}

// ---- membership change log (np8_changes) --------------------------------------------------------------
// One lane per item; a wave with moved items takes its output range with one atomic.
__global__ __launch_bounds__(256) void np8_changes_items(const int32_t *__restrict__ z, const int32_t *__restrict__ zb,
                                                         int64_t n, int64_t *__restrict__ oi, int32_t *__restrict__ os,
                                                         int64_t cap, unsigned long long *count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool moved = i < n && z[i] != zb[i];
    const uint64_t b = __ballot(moved);
    if (b == 0ull) return;
    const int lane = threadIdx.x & 63, lead = __ffsll((unsigned long long)b) - 1;
    unsigned long long base = 0ull;
    if (lane == lead) base = atomicAdd(count, (unsigned long long)__popcll(b));
    base = __shfl(base, lead);
    const int64_t q = (int64_t)base + __popcll(b & ((1ull << lane) - 1ull));
    if (moved && q < cap) {
        oi[q] = i;
        os[q] = z[i];
    }
}

__global__ __launch_bounds__(256) void np8_changes_slots(const int32_t *__restrict__ cnt, const int32_t *__restrict__ cb,
                                                         const double *__restrict__ mu, const double *__restrict__ mb,
                                                         const double *__restrict__ sg, const double *__restrict__ sb,
                                                         int D, int kcap, uint8_t *__restrict__ flags) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= kcap) return;
    const bool live = cnt[s] > 0, was = cb[s] > 0;
    uint8_t f = 0;
    if (live && !was) {
        f = 1;
    } else if (!live && was) {
        f = 2;
    } else if (live) {  // same slot live before and after: bitwise comparison of the parameters
        bool diff = false;
        for (int a = 0; a < D; ++a) diff |= __double_as_longlong(mu[(int64_t)s * D + a]) != __double_as_longlong(mb[(int64_t)s * D + a]);
        for (int a = 0; a < D * D; ++a)
            diff |= __double_as_longlong(sg[(int64_t)s * D * D + a]) != __double_as_longlong(sb[(int64_t)s * D * D + a]);
        f = diff ? 3 : 0;
    }
    flags[s] = f;
}

hipError_t np8_launch_changes(const int32_t *z, const int32_t *z_base, int64_t n, int64_t *out_item, int32_t *out_slot,
                              int64_t cap, unsigned long long *count, const int32_t *cnt, const int32_t *cnt_base,
                              const double *mu, const double *mu_base, const double *sg, const double *sg_base, int D,
                              int kcap, uint8_t *flags, hipStream_t s) {
    if (n > 0)
        hipLaunchKernelGGL(np8_changes_items, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, z, z_base, n, out_item,
                           out_slot, cap, count);
    hipLaunchKernelGGL(np8_changes_slots, dim3((unsigned)((kcap + 255) / 256)), dim3(256), 0, s, cnt, cnt_base, mu, mu_base,
                       sg, sg_base, D, kcap, flags);
    return hipGetLastError();
}

// The draw exactly as np8_assign runs it: state at candidate 0 (the item's own cluster), then pick_step over
// candidates 1..n-1 in order (skip rule included).
__global__ __launch_bounds__(256) void np8_pick_batch(const double *__restrict__ lw, int32_t n,
                                                      const double *__restrict__ u, int64_t n_draws,
                                                      int32_t *__restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_draws) return;
    PickState st;
    st.T = lw[0];
    st.S = 1.0;
    st.u = u[k];
    st.pick = 0;
    for (int32_t j = 1; j < n; ++j) pick_step(st, lw[j], j);
    out[k] = st.pick;
}

hipError_t np8_launch_pick_batch(const double *lw, int32_t n, const double *u, int64_t n_draws, int32_t *out,
                                 hipStream_t s) {
    if (n_draws <= 0) return hipSuccess;
    hipLaunchKernelGGL(np8_pick_batch, dim3((unsigned)((n_draws + 255) / 256)), dim3(256), 0, s, lw, n, u, n_draws,
                       out);
    return hipGetLastError();
}

hipError_t np8_launch_loglik_matrix(const AssignArgs &A, int D, int M, int prior, const int64_t *idx, int64_t n,
                                    double *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
#define X(d, m)                                                                                                 \
    if (D == d && M == m) {                                                                                     \
        if (prior == kPriorNiw)                                                                                 \
            hipLaunchKernelGGL((np8_loglik_matrix_kernel<d, m, kPriorNiw>), grid, block, 0, s, A, idx, n, out);   \
        else                                                                                                    \
            hipLaunchKernelGGL((np8_loglik_matrix_kernel<d, m, kPriorReference>), grid, block, 0, s, A, idx, n, \
                               out);                                                                            \
        return hipGetLastError();                                                                               \
    }
    NP8_FOR_EACH_DM(X)
#undef X
    if (np8_rt_supported(D, M, prior)) return np8_launch_loglik_matrix_rt(A, D, M, idx, n, out, s);
    return hipErrorInvalidValue;
}

hipError_t np8_launch_aux_bounds(const AssignArgs &A, int D, int M, const int64_t *idx, int64_t n, double *out,
                                 hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
#define X(d, m)                                                                                       \
    if (D == d && M == m) {                                                                           \
        hipLaunchKernelGGL((np8_aux_bounds_kernel<d, m>), grid, block, 0, s, A, idx, n, out);         \
        return hipGetLastError();                                                                     \
    }
    NP8_FOR_EACH_DM(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_resort(const SortArgs &S, hipStream_t s) {
    if (S.n <= 0) return hipSuccess;
    const int64_t per = (int64_t)kSortThreads * kSortItems;
    const unsigned nb = (unsigned)((S.n + per - 1) / per);
    const size_t bins = (size_t)S.kcap * S.nsub;
    hipLaunchKernelGGL(np8_sort_hist, dim3(nb), dim3(kSortThreads), sizeof(int) * bins, s, S);
    hipLaunchKernelGGL(np8_sort_scan, dim3(1), dim3(1024), 0, s, S);
    hipLaunchKernelGGL(np8_sort_scatter, dim3(nb), dim3(kSortThreads), 2 * sizeof(int) * bins, s, S);
    hipLaunchKernelGGL(np8_sort_copyback, dim3(1024), dim3(256), 0, s, S);
    return hipGetLastError();
}

size_t np8_finalize_lds_bytes(int kcap) {
    return sizeof(int64_t) * kReqMax + sizeof(int) * kReqMax * 2 + 2 * sizeof(int) * (size_t)kcap;
}

hipError_t np8_launch_finalize(const FinArgs &F, hipStream_t s) {
    hipLaunchKernelGGL(np8_finalize, dim3(1), dim3(kFinThreads), np8_finalize_lds_bytes(F.kcap), s, F);
    return hipGetLastError();
}

hipError_t np8_launch_step_tail(const AssignArgs &A, const FinArgs &F, const PruneArgs &P, const TailArgs &T0,
                                int64_t n_waves, int D, int M, hipStream_t s) {
    (void)n_waves;
    (void)M;
    // the fold reads one record per thread; otherwise one workgroup
    constexpr int64_t kTailBlocks = 256;
    int64_t nb = T0.fold ? (T0.fold_n + kFinThreads - 1) / kFinThreads : 1;
    nb = nb < 1 ? 1 : (nb > kTailBlocks ? kTailBlocks : nb);
    TailArgs T = T0;
    T.lds_bytes = (int64_t)np8_finalize_lds_bytes(F.kcap);
    const size_t lds = (size_t)T.lds_bytes;
    switch (D) {
#define Y(d)                                                                                              \
    case d:                                                                                               \
        hipLaunchKernelGGL((np8_step_tail<d>), dim3((unsigned)nb), dim3(kFinThreads), lds, s, A, F, P, T); \
        break;
        Y(1) Y(2) Y(3) Y(4) Y(5) Y(6) Y(7) Y(8) Y(9) Y(10) Y(11) Y(12) Y(13) Y(14) Y(15) Y(16)
#undef Y
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t np8_launch_fin_prune(const FinArgs &F, const PruneArgs &P, hipStream_t s) {
    int nP = (F.kcap + kFinThreads / 64 - 1) / (kFinThreads / 64);
    nP = nP < 1 ? 1 : (nP > kFpPruneBlocks ? kFpPruneBlocks : nP);
    const size_t lds = np8_finalize_lds_bytes(F.kcap);
    switch (F.D) {
#define Y(d)                                                                                                 \
    case d:                                                                                                  \
        hipLaunchKernelGGL((np8_fin_prune<d>), dim3((unsigned)(1 + nP)), dim3(kFinThreads), lds, s, F, P, nP); \
        break;
        Y(1) Y(2) Y(3) Y(4) Y(5) Y(6) Y(7) Y(8) Y(9) Y(10) Y(11) Y(12) Y(13) Y(14) Y(15) Y(16)
#undef Y
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t np8_launch_ll_header(const Ctl *ctl, const Fx *llpart, int64_t ll_n, unsigned char *rec, hipStream_t s) {
    hipLaunchKernelGGL(np8_ll_header, dim3(1), dim3(kFinThreads), 0, s, ctl, llpart, ll_n, rec);
    return hipGetLastError();
}

hipError_t np8_launch_req_select(const unsigned char *stage, int64_t stage_cap, unsigned char *rec, int64_t rec_cap,
                                 int kcap, int D, int req_max, const Fx *llpart, int64_t ll_n, hipStream_t s) {
    hipLaunchKernelGGL(np8_req_select, dim3(1), dim3(kFinThreads), sizeof(int) * 2048, s, stage, stage_cap, rec, rec_cap,
                       kcap, D, req_max, llpart, ll_n);
    return hipGetLastError();
}

hipError_t np8_launch_loglik(const LoglikArgs &A, int D, hipStream_t s) {
    const int64_t nb = (A.n_loc + 255) / 256;
    if (nb <= 0) return hipSuccess;
    switch (D) {
#define Y(d)                                                                       \
    case d:                                                                        \
        hipLaunchKernelGGL((np8_loglik<d>), dim3((unsigned)nb), dim3(256), 0, s, A); \
        break;
        Y(1) Y(2) Y(3) Y(4) Y(5) Y(6) Y(7) Y(8) Y(9) Y(10) Y(11) Y(12) Y(13) Y(14) Y(15) Y(16)
#undef Y
        default:
            return np8_launch_loglik_rt(A, D, s);
    }
    return hipGetLastError();
}

hipError_t np8_launch_loglik_reduce(const double *partial, int64_t nb, double *out, double *out2, hipStream_t s) {
    hipLaunchKernelGGL(np8_loglik_reduce, dim3(1), dim3(1024), 0, s, partial, nb, out, out2);
    return hipGetLastError();
}

hipError_t np8_launch_suffstats(const ParamArgs &A, hipStream_t s) {
    const int64_t per_block = 64 * kSuffRows;  // one wave per block
    const int64_t nb = (A.n_loc + per_block - 1) / per_block;
    if (nb <= 0) return hipSuccess;
    switch (A.D) {
#define Y(d)                                                                          \
    case d:                                                                           \
        hipLaunchKernelGGL((np8_suffstats<d>), dim3((unsigned)nb), dim3(64), 0, s, A); \
        break;
        Y(1) Y(2) Y(3) Y(4) Y(5) Y(6) Y(7) Y(8) Y(9) Y(10) Y(11) Y(12) Y(13) Y(14) Y(15) Y(16)
#undef Y
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t np8_launch_mh_g0(const ParamArgs &A, hipStream_t s) {
    switch (A.D) {
#define Y(d)                                                                       \
    case d:                                                                        \
        hipLaunchKernelGGL((np8_mh_g0<d>), dim3((unsigned)A.kcap), dim3(64), 0, s, A); \
        break;
        Y(1) Y(2) Y(3) Y(4) Y(5) Y(6) Y(7) Y(8) Y(9) Y(10) Y(11) Y(12) Y(13) Y(14) Y(15) Y(16)
#undef Y
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Standalone pass (after the mh_g0 update has moved means): four rows per block.
// A small grid strides over the live rows (one wave per row): K is only known on the device, and a
// grid sized for kcap would mostly launch blocks that exit at once.
// Lists from the radii in use; after the last step of a gathering sweep from the radii just gathered, which
// block 0 then makes the radii in use (no other block reads those in this pass).  Any radius is safe: a
// lane checks its own distance against the radius its list was built for (np8_assign).
template <int DT>
__global__ __launch_bounds__(256) void np8_prune(PruneArgs A) {
    if (A.ctl->halt) return;  // a halted compact sweep graph
    const int K = A.ctl->K;
    if (blockIdx.x == 0 && threadIdx.x == 0) A.ctl->lists_ok = 1;
    const double *src = A.r2 + (A.gathered ? A.kcap : 0);
    if (A.gathered && blockIdx.x == 0)
        for (int s = threadIdx.x; s < A.kcap; s += blockDim.x) A.r2[s] = A.r2[A.kcap + s];
    if (A.clear_next && blockIdx.x == 0)  // only the radii in use are read here (not gathered)
        for (int s = threadIdx.x; s < A.kcap; s += blockDim.x) A.r2[A.kcap + s] = 0.0;
    auto R2of = [&](int slot) { return src[slot]; };
    for (int k0 = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); k0 < K; k0 += gridDim.x * 4)  // wave-uniform
        prune_row<DT>(A.cand, R2of, A.plist, A.pdist, A.plen, A.plr2, A.plen_s, A.plr2_s, A.ls, A.D, K, k0, A.lb, A.kcap, A.lam);
}

__global__ void np8_advance_epoch(Ctl *ctl, uint32_t n) {
    if (!ctl->halt) ctl->t_base += n;
}

// a Ctl flag cleared in stream order, unless a compact sweep graph is halted (which = 0: best_sorted, 1: snap_pend)
__global__ void np8_ctl_clear(Ctl *ctl, int which) {
    if (ctl->halt) return;
    if (which == 0)
        ctl->best_sorted = 0;
    else
        ctl->snap_pend = 0;
}

hipError_t np8_launch_ctl_clear(Ctl *ctl, int which, hipStream_t s) {
    hipLaunchKernelGGL(np8_ctl_clear, dim3(1), dim3(1), 0, s, ctl, which);
    return hipGetLastError();
}

// p[0..n) = 0 in stream order, unless a compact sweep graph is halted: the memset a captured sweep would otherwise
// hold ignores ctl->halt and could clear the halted step's gathered radii before the host resumes that step
__global__ void np8_clear_unless_halted(double *p, int n, const Ctl *ctl) {
    if (ctl->halt) return;
    for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0.0;
}

hipError_t np8_launch_clear_unless_halted(double *p, int n, const Ctl *ctl, hipStream_t s) {
    hipLaunchKernelGGL(np8_clear_unless_halted, dim3(1), dim3(256), 0, s, p, n, ctl);
    return hipGetLastError();
}

hipError_t np8_launch_prune(const PruneArgs &A, int kcap, hipStream_t s) {
    const int nb = (kcap + 3) / 4;
    const dim3 g((unsigned)(nb < kPruneBlocks ? nb : kPruneBlocks));
    switch (A.D) {
#define Y(d)                                                              \
    case d:                                                               \
        hipLaunchKernelGGL((np8_prune<d>), g, dim3(256), 0, s, A);        \
        break;
        Y(1) Y(2) Y(3) Y(4) Y(5) Y(6) Y(7) Y(8) Y(9) Y(10) Y(11) Y(12) Y(13) Y(14) Y(15) Y(16)
#undef Y
        default:
            hipLaunchKernelGGL((np8_prune<0>), g, dim3(256), 0, s, A);
    }
    return hipGetLastError();
}

hipError_t np8_launch_advance_epoch(Ctl *ctl, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(np8_advance_epoch, dim3(1), dim3(1), 0, s, ctl, n);
    return hipGetLastError();
}

hipError_t np8_launch_snapshot_flush(const SnapArgs &A, Ctl *ctl, hipStream_t s) {
    int64_t n = A.n_loc > (int64_t)A.kcap * A.D * A.D ? A.n_loc : (int64_t)A.kcap * A.D * A.D;
    int64_t nb = (n + 255) / 256;
    if (nb > 2048) nb = 2048;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(np8_snapshot_flush, dim3((unsigned)nb), dim3(256), 0, s, A, ctl);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void np8_best_copy(const Ctl *__restrict__ ctl, const int32_t *__restrict__ src,
                                                     int32_t *__restrict__ dst, int64_t n) {
    if (!ctl->best_sorted || ctl->halt) return;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

__global__ __launch_bounds__(256) void np8_best_scatter(const Ctl *__restrict__ ctl, const int32_t *__restrict__ ids,
                                                        const int32_t *__restrict__ src, int32_t *__restrict__ dst,
                                                        int64_t n) {
    if (!ctl->best_sorted || ctl->halt) return;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
        dst[ids[p]] = src[p];
}

hipError_t np8_launch_best_unsort(Ctl *ctl, const int32_t *ids, int32_t *z_best, int32_t *scratch, int64_t n,
                                  hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t nb = (n + 255) / 256;
    if (nb > 2048) nb = 2048;
    hipLaunchKernelGGL(np8_best_copy, dim3((unsigned)nb), dim3(256), 0, s, ctl, z_best, scratch, n);
    hipLaunchKernelGGL(np8_best_scatter, dim3((unsigned)nb), dim3(256), 0, s, ctl, ids, scratch, z_best, n);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return np8_launch_ctl_clear(ctl, 0, s);
}

hipError_t np8_launch_snapshot(const SnapArgs &A, hipStream_t s) {
    int64_t n = A.n_loc > (int64_t)A.kcap * A.D * A.D ? A.n_loc : (int64_t)A.kcap * A.D * A.D;
    int64_t nb = (n + 255) / 256;
    if (nb > 2048) nb = 2048;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(np8_snapshot, dim3((unsigned)nb), dim3(256), 0, s, A);
    return hipGetLastError();
}
