// np8_device.h -- arithmetic shared by the gfx950 kernels and the library's host-side setup code
// (cluster initialisation, table entries).  Every formula here is the one DESIGN.md "Chain
// specification" fixes; fused multiply-adds are explicit (the library is built -ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define NP8_HD __host__ __device__ __forceinline__

namespace np8 {

constexpr double kLog2Pi = 1.8378770664093454835606594728112;
constexpr double kTwoPi = 6.283185307179586476925286766559;
constexpr int kReqMax = 4096;     // new-cluster requests one finalize can accept
constexpr int kMaxD = 128;  // (the fp64 path with D at run time, np8_rt.hip; the fp32 wide path stops at 80)
constexpr int kMaxM = 8;

enum Stream : uint32_t {
    kStreamAux = 1,
    kStreamPick = 2,
    kStreamInitTheta = 3,
    kStreamInitZ = 4,
    kStreamParam = 5,  // MH proposal normals (i = slot)
    kStreamParamU = 6,  // MH acceptance uniforms (i = slot)
    kStreamAuxDir = 7,  // direction of a picked auxiliary's xi orthogonal to the item (i = item);
                        // NIW: Bartlett off-diagonals and the z_perp direction of a picked auxiliary
    kStreamAuxNiw = 8,  // NIW prior: an auxiliary's Bartlett chi^2 draws, chi^2_{D-1} and z_1 (i = item)
    // (9 .. 11: split-merge, np8_sm.hip)
    kStreamAuxPre = 12  // reference prior: the auxiliaries' chi^2 prefixes (i = item, call 0; aux_pre_bits)
};

// Base measures (include/np8.h NP8_PRIOR_*).
enum Prior : int { kPriorReference = 0, kPriorNiw = 1 };

// Candidate-table entry layout (doubles):
//   [mu(D) | P'(D(D+1)/2) | c | logn | logn1 | slot | iso]
// P' = packed upper triangle of sym(Sigma^-1), off-diagonals doubled; iso = the common diagonal when
// P' is a multiple of I (every G0 draw under an isotropic Lambda), else 0.
NP8_HD int packed_size(int D) { return D * (D + 1) / 2; }
NP8_HD int cand_stride(int D) { return (D + packed_size(D) + 5 + 1) & ~1; }
enum CandField : int { kFieldC = 0, kFieldLogn = 1, kFieldLogn1 = 2, kFieldSlot = 3, kFieldIso = 4 };


// Philox4x32-10 (Salmon et al. SC'11).
NP8_HD void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                          uint32_t out[4]) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(NP8_EXP_PHILOX_HOISTED)
    // The key (the chain seed) is uniform at every call site.  An empty asm barrier makes the compiler rederive the
    // round-key schedule (18 scalar adds) at each call instead of hoisting 20 round keys into SGPRs for the whole
    // kernel: the C3 assign kernel's SGPR spills to VGPR lanes fall from 94 to 74 and its VGPR spills from 42 to 39,
    // 9% faster (profiles/r06/ab_keys).  No instruction is emitted; results are unchanged.
    asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        // one 32x32->64 product per multiplier: a single v_mad_u64_u32 instead of a
        // v_mul_hi_u32 + v_mul_lo_u32 pair
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        c1 = (uint32_t)p1;
        c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c3 = (uint32_t)p0;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

NP8_HD void philox_call(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call, uint32_t out[4]) {
    philox4x32_10((uint32_t)i, (uint32_t)(i >> 32), t, (stream << 24) | (call & 0xFFFFFFu), (uint32_t)seed,
                  (uint32_t)(seed >> 32), out);
}

// Odd 53-bit integer times 2^-53: uniform on (0,1), never 0 or 1 (the draws' uniforms).
NP8_HD double u01(uint32_t hi, uint32_t lo) {
    uint64_t v = ((((uint64_t)hi) << 32) | lo) >> 11;
    v |= 1u;
    return (double)v * 0x1.0p-53;
}

// (k + 1/2) 2^-32: a 32-bit uniform on (0,1), exact in fp64 (the Box-Muller inputs).
NP8_HD double u32_01(uint32_t k) { return fma((double)k, 0x1.0p-32, 0x1.0p-33); }

// 1/y for y in [2 - (1 - 1/sqrt2), 2 + (sqrt2 - 1)] (the log's s = f/(2+f)): minimax quadratic
// (relative error 1.3e-3) and three Newton steps, fma only -- no IEEE division sequence.
NP8_HD double recip_logden(double y) {
    double r = fma(fma(0.11686276, y, -0.72244362), y, 1.47775548);
#pragma unroll
    for (int k = 0; k < 3; ++k) r = fma(r, fma(-y, r, 1.0), r);
    return r;
}

// ---- elementary functions with identical bits on host and device (DESIGN.md "Math") ------------
// Weight for the draw: exp(x) for x <= 0 (x may be -inf).  Cody-Waite reduction by ln2, degree-13
// Taylor polynomial on |r| <= ln2/2, ldexp.  Below -800 the result is 0 (as IEEE exp would be).
NP8_HD double exp_le0(double x) {
    x = fmax(x, -800.0);
    const double k = rint(x * 1.4426950408889634);
    double r = fma(-k, 0.6931471803691238, x);
    r = fma(-k, 1.9082149292705877e-10, r);
    double p = 1.6059043836821613e-10;
    p = fma(p, r, 2.08767569878681e-09);
    p = fma(p, r, 2.505210838544172e-08);
    p = fma(p, r, 2.755731922398589e-07);
    p = fma(p, r, 2.7557319223985893e-06);
    p = fma(p, r, 2.48015873015873e-05);
    p = fma(p, r, 0.0001984126984126984);
    p = fma(p, r, 0.001388888888888889);
    p = fma(p, r, 0.008333333333333333);
    p = fma(p, r, 0.041666666666666664);
    p = fma(p, r, 0.16666666666666666);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return ldexp(p, (int)k);
}

// log(u) for a positive normal u: u = m 2^e with m in [1/sqrt2, sqrt2), log1p(m-1) = 2 atanh(s),
// s = (m-1)/(m+1), series to s^21.
NP8_HD double log_pos(double u) {
    int e;
    double m = frexp(u, &e);
    const bool lo = m < 0.70710678118654757;
    m = lo ? m + m : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0;
    const double s = f * recip_logden(2.0 + f);
    const double s2 = s * s;
    double p = 0.09523809523809523;
    p = fma(p, s2, 0.10526315789473684);
    p = fma(p, s2, 0.11764705882352941);
    p = fma(p, s2, 0.13333333333333333);
    p = fma(p, s2, 0.15384615384615385);
    p = fma(p, s2, 0.18181818181818182);
    p = fma(p, s2, 0.2222222222222222);
    p = fma(p, s2, 0.2857142857142857);
    p = fma(p, s2, 0.4);
    p = fma(p, s2, 0.6666666666666666);
    const double l1 = fma(s * s2, p, s + s);
    const double de = (double)e;
    return fma(de, 0.6931471803691238, fma(de, 1.9082149292705877e-10, l1));
}

// (sin 2 pi t, cos 2 pi t) for t in [0,1]: exact quadrant reduction f = t - q/4 in [-1/8, 1/8],
// Taylor polynomials of sin(2 pi f) (to f^17) and cos(2 pi f) (to f^18).
NP8_HD void sincos_2pi(double t, double &sn, double &cs) {
    const double q = rint(4.0 * t);
    const double f = t - 0.25 * q;
    const double f2 = f * f;
    double ps = 0.10422916220813984;
    ps = fma(ps, f2, -0.7181223017785006);
    ps = fma(ps, f2, 3.819952584848282);
    ps = fma(ps, f2, -15.09464257682299);
    ps = fma(ps, f2, 42.058693944897655);
    ps = fma(ps, f2, -76.70585975306139);
    ps = fma(ps, f2, 81.60524927607506);
    ps = fma(ps, f2, -41.34170224039976);
    ps = fma(ps, f2, 6.283185307179586);
    const double s0 = ps * f;
    double pc = -0.03638284114254567;
    pc = fma(pc, f2, 0.28200596845579123);
    pc = fma(pc, f2, -1.714390711088672);
    pc = fma(pc, f2, 7.903536371318469);
    pc = fma(pc, f2, -26.4262567833744);
    pc = fma(pc, f2, 60.24464137187666);
    pc = fma(pc, f2, -85.45681720669373);
    pc = fma(pc, f2, 64.9393940226683);
    pc = fma(pc, f2, -19.739208802178716);
    const double c0 = fma(pc, f2, 1.0);
    const int qi = ((int)q) & 3;
    const double a = (qi & 1) ? c0 : s0;
    const double b = (qi & 1) ? s0 : c0;
    sn = (qi & 2) ? -a : a;
    cs = ((qi + 1) & 2) ? -b : b;
}

// Four normals from one Philox call: two Box-Muller pairs over 32-bit uniforms,
// (r cos 2 pi u2, r sin 2 pi u2), r = sqrt(-2 log u1), (u1, u2) = words (0, 1) and (2, 3).
// A draw of n normals uses calls base .. base + ceil(n/4) - 1; normal k is g[k & 3] of call k >> 2.
NP8_HD void normal_quad(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call, double (&g)[4]) {
    uint32_t o[4];
    philox_call(seed, i, t, stream, call, o);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const double r = sqrt(-2.0 * log_pos(u32_01(o[2 * h])));
        double sn, cs;
        sincos_2pi(u32_01(o[2 * h + 1]), sn, cs);
        g[2 * h] = r * cs;
        g[2 * h + 1] = r * sn;
    }
}

// Philox calls per full G0 draw (D+1 normals: the scale normal, then xi) -- init and MH proposals.
NP8_HD int g0_calls(int D) { return (D + 4) / 4; }

// ---- auxiliary draws in the item's frame (DESIGN.md "G0") -------------------------------------------
// Auxiliary m of item i is theta = (v, mu0 + (|v|/sqrt kappa) L^T xi), xi ~ N(0, I_D).  With the item
// whitened, y0 = (L^T)^{-1}(x - mu0), the likelihood depends on xi only through xi_par = xi . y0/|y0|
// ~ N(0,1) and chi2 = |xi_perp|^2 ~ chi^2_{D-1}:  |y0 - s xi|^2 = (|y0| - s xi_par)^2 + s^2 chi2.  So
// the draw is (v, xi_par, chi2), from calls m*Qa .. m*Qa + Qa - 1 of stream AUX:
//   call 0: Box-Muller pair of words (0, 1) -> (v-normal, xi_par) = (r cos, r sin); words 2, 3 -> the
//           first two of the k = (D-1)/2 uniforms whose product gives chi^2_{2k} = -2 log(prod)
//   call 1 (when D-1 is odd or k > 2): words (0, 1) -> g_odd = r cos (chi^2 gets g_odd^2 for odd D-1);
//           words 2, 3 -> uniforms 2, 3
//   call 2 + c: uniforms 4 + 4c .. 7 + 4c
// (logs over products of at most 16 uniforms).  Everything an upper bound of the log-likelihood needs --
// v, xi_par and a lower bound of chi2 -- comes from call 0 (aux_screen_skips in np8_kernels.hip).
// Only a picked auxiliary needs xi itself: xi = xi_par yhat + sqrt(chi2) w_perp/|w_perp| with
// w ~ N(0, I_D) on stream AUX_DIR (exactly N(0, I) in distribution: independent radial, parallel and
// direction parts).
NP8_HD int aux_calls(int D) {
    const int k = (D - 1) / 2;
    return 1 + ((((D - 1) & 1) || k > 2) ? 1 : 0) + (k > 4 ? (k - 1) / 4 : 0);
}
NP8_HD int dir_calls(int D) { return (D + 3) / 4; }

// The screen prefixes (round 6, DESIGN.md "Auxiliary screen"), for D <= kPreMaxD (the fast kernel's level-0 screen; above
// it the draws are the round-5 ones and the kernels screen from each auxiliary's call 0, as before: their register
// budget has no room for the prefix words).  One Philox call per item and epoch -- stream AUX_PRE,
// call 0 -- holds the leading b bits of the first P = min(k, 3) chi^2 uniforms of all M auxiliaries, b = min(16,
// floor(128 / (M P))): field f = m P + j is bits [b f, b f + b) of the call's output (word 0 = bits 0 .. 31).  The
// 32-bit word that feeds chi^2 uniform j < P of auxiliary m is (field << (32 - b)) | (the word the calls above give it
// & (2^(32 - b) - 1)).  The chi^2 uniforms stay uniform and independent of everything else drawn; what the prefixes buy
// is a lower bound of every auxiliary's chi^2 -- so an upper bound of its log-likelihood, with the supremum over
// (v, xi_par) taken in closed form -- from one call per item instead of call 0 of every auxiliary.
constexpr int kPreMaxD = 8;
NP8_HD int aux_pre_n(int D) {
    const int k = (D - 1) / 2;
    return D > kPreMaxD ? 0 : (k < 3 ? k : 3);
}
NP8_HD int aux_pre_bits(int D, int M) {
    const int P = aux_pre_n(D);
    if (P <= 0 || M <= 0) return 0;
    const int b = 128 / (M * P);
    return b > 16 ? 16 : b;
}
// field f of width b (1..16) of the 128-bit prefix call (word selects instead of a run-time register index)
NP8_HD uint32_t aux_pre_field(const uint32_t (&W)[4], int f, int b) {
    const int lo = b * f, wi = lo >> 5, sh = lo & 31;
    const uint32_t a = wi == 0 ? W[0] : (wi == 1 ? W[1] : (wi == 2 ? W[2] : W[3]));
    const uint32_t n = wi == 0 ? W[1] : (wi == 1 ? W[2] : (wi == 2 ? W[3] : 0u));
    const uint64_t v = ((uint64_t)n << 32 | a) >> sh;
    return (uint32_t)v & ((1u << b) - 1u);
}
NP8_HD uint32_t aux_pre_word(uint32_t w, uint32_t field, int b) {
    return b > 0 ? ((field << (32 - b)) | (w & ((1u << (32 - b)) - 1u))) : w;
}
// chi^2 uniform j's word of auxiliary m (the word its own calls give, combined with its prefix when j < P)
NP8_HD uint32_t aux_chi_word(const uint32_t (&pre)[4], uint32_t w, int m, int j, int D, int M) {
    const int P = aux_pre_n(D), b = aux_pre_bits(D, M);
    return (j < P && b > 0) ? aux_pre_word(w, aux_pre_field(pre, m * P + j, b), b) : w;
}
NP8_HD void aux_pre_call(uint64_t seed, uint64_t i, uint32_t t, uint32_t out[4]) {
    philox_call(seed, i, t, kStreamAuxPre, 0u, out);
}

// w: the words of call m*Qa; w1g the words of call m*Qa + 1 when have_w1 (else drawn here).  Arrays by
// reference, never through a pointer: a pointer to a register array would move it to scratch memory.
// D is a template constant: the chi^2 loop unrolls and every word index is static (a run-time index
// into a register array would move the array to scratch memory).
// pre: the item's prefix call (aux_pre_call), M the auxiliaries per item (the prefixes' layout).
template <int D>
NP8_HD void aux_core_w(uint64_t seed, uint64_t i, uint32_t t, int m, double nu, double &v, double &xpar,
                       double &chi2, const uint32_t (&w)[4], bool have_w1, const uint32_t (&w1g)[4],
                       const uint32_t (&pre)[4], int M) {
    constexpr int k = (D - 1) / 2;
    constexpr bool odd = ((D - 1) & 1) != 0;
    const int Qa = aux_calls(D);
    const uint32_t base = (uint32_t)(m * Qa);
    uint32_t w1[4] = {0u, 0u, 0u, 0u}, wc[4] = {0u, 0u, 0u, 0u};
    {
        const double r = sqrt(-2.0 * log_pos(u32_01(w[0])));
        double sn, cs;
        sincos_2pi(u32_01(w[1]), sn, cs);
        v = fma(nu, r * cs, (double)D);
        xpar = r * sn;
    }
    double godd = 0.0;
    if (odd || k > 2) {
        if (have_w1) {
            for (int h = 0; h < 4; ++h) w1[h] = w1g[h];
        } else {
            philox_call(seed, i, t, kStreamAux, base + 1u, w1);
        }
        if (odd) {
            const double r = sqrt(-2.0 * log_pos(u32_01(w1[0])));
            double sn, cs;
            sincos_2pi(u32_01(w1[1]), sn, cs);
            godd = r * cs;
        }
    }
    double c2 = 0.0, prod = 1.0;
    int in_chunk = 0;
#pragma unroll
    for (int j = 0; j < k; ++j) {
        uint32_t word;
        if (j < 2) {
            word = aux_chi_word(pre, w[2 + j], m, j, D, M);
        } else if (j < 4) {
            word = aux_chi_word(pre, w1[j], m, j, D, M);
        } else {
            if (((j - 4) & 3) == 0) philox_call(seed, i, t, kStreamAux, base + 2u + (uint32_t)((j - 4) >> 2), wc);
            word = wc[(j - 4) & 3];
        }
        prod *= u32_01(word);
        if (++in_chunk == 16 || j == k - 1) {
            c2 = fma(-2.0, log_pos(prod), c2);
            prod = 1.0;
            in_chunk = 0;
        }
    }
    if (odd) c2 = fma(godd, godd, c2);
    chi2 = c2;
}

// aux_core_w's draws with D at run time (the wide path, D > kPreMaxD: no prefixes; D padded to a tile multiple): the
// same operations in the
// same order; the words of each further call are consumed four at a time with static indices.
NP8_HD void aux_core_rt(uint64_t seed, uint64_t i, uint32_t t, int m, int M, int D, double nu, double &v,
                        double &xpar, double &chi2) {
    const int k = (D - 1) / 2;
    const bool odd = ((D - 1) & 1) != 0;
    const uint32_t base = (uint32_t)(m * aux_calls(D));
    (void)M;  // (the wide path's D > kPreMaxD: no prefixes)
    uint32_t w[4], w1[4] = {0u, 0u, 0u, 0u};
    philox_call(seed, i, t, kStreamAux, base, w);
    {
        const double r = sqrt(-2.0 * log_pos(u32_01(w[0])));
        double sn, cs;
        sincos_2pi(u32_01(w[1]), sn, cs);
        v = fma(nu, r * cs, (double)D);
        xpar = r * sn;
    }
    double godd = 0.0;
    if (odd || k > 2) {
        philox_call(seed, i, t, kStreamAux, base + 1u, w1);
        if (odd) {
            const double r = sqrt(-2.0 * log_pos(u32_01(w1[0])));
            double sn, cs;
            sincos_2pi(u32_01(w1[1]), sn, cs);
            godd = r * cs;
        }
    }
    double c2 = 0.0, prod = 1.0;
    int in_chunk = 0;
    auto take = [&](uint32_t word, int j) {
        prod *= u32_01(word);
        if (++in_chunk == 16 || j == k - 1) {
            c2 = fma(-2.0, log_pos(prod), c2);
            prod = 1.0;
            in_chunk = 0;
        }
    };
    if (k > 0) take(w[2], 0);
    if (k > 1) take(w[3], 1);
    if (k > 2) take(w1[2], 2);
    if (k > 3) take(w1[3], 3);
    for (int c = 0; 4 + 4 * c < k; ++c) {
        uint32_t wc[4];
        philox_call(seed, i, t, kStreamAux, base + 2u + (uint32_t)c, wc);
#pragma unroll
        for (int h = 0; h < 4; ++h)
            if (4 + 4 * c + h < k) take(wc[h], 4 + 4 * c + h);
    }
    if (odd) c2 = fma(godd, godd, c2);
    chi2 = c2;
}

template <int D>
NP8_HD void aux_core(uint64_t seed, uint64_t i, uint32_t t, int m, int M, double nu, double &v, double &xpar,
                     double &chi2) {
    uint32_t w[4], pre[4] = {0u, 0u, 0u, 0u};
    const uint32_t none[4] = {0u, 0u, 0u, 0u};
    if (aux_pre_n(D) > 0) aux_pre_call(seed, i, t, pre);
    philox_call(seed, i, t, kStreamAux, (uint32_t)(m * aux_calls(D)), w);
    aux_core_w<D>(seed, i, t, m, nu, v, xpar, chi2, w, false, none, pre, M);
}

// Log-likelihood of the item under auxiliary (v, xi_par, chi2); ny = |y0|.
NP8_HD double aux_loglik(double ny, double v, double xpar, double chi2, int D, double rsk, double caux) {
    const double s = fabs(v) * rsk;
    const double d = fma(-s, xpar, ny);
    const double r2 = fma(d, d, (s * s) * chi2);
    const double q = r2 / (v * v);
    const double cm = fma(-(double)D, log_pos(fabs(v)), caux);
    return fma(-0.5, q, cm);
}

// xi of a picked auxiliary (see above); y0 and ny of the item.  DM bounds D at compile time (the
// kernels instantiate it with their D, host code and np8_finalize with kMaxD).
template <int DM>
NP8_HD void aux_xi(uint64_t seed, uint64_t i, uint32_t t, int m, int D, const double *y0, double ny, double xpar,
                   double chi2, double *xi /* D */) {
    double yh[DM], w[DM];
    for (int a = 0; a < D; ++a) yh[a] = (ny > 0.0) ? y0[a] / ny : (a == 0 ? 1.0 : 0.0);
    const int Qd = dir_calls(D);
    double g[4] = {0.0, 0.0, 0.0, 0.0};
    for (int a = 0; a < D; ++a) {
        if ((a & 3) == 0) normal_quad(seed, i, t, kStreamAuxDir, (uint32_t)(m * Qd + (a >> 2)), g);
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

// ---- NIW prior (DESIGN.md "Priors"; oracle/np8_oracle.c has the derivation) ----------------------
constexpr uint32_t kNiwAuxCalls = 8192u;   // Philox calls reserved per auxiliary m
constexpr uint32_t kNiwGammaCalls = 64u;   // calls reserved per chi^2 draw
constexpr uint32_t kNiwNormalCall0 = 8192u; // posterior draws: first call of the normals

// Marsaglia-Tsang Gamma(alpha, 1), alpha >= 1: two attempts per Philox call (Box-Muller pair from
// words 0, 1; 32-bit uniforms words 2, 3); at most 4096 calls, so every lane terminates.
NP8_HD double gamma_mt(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call0, double alpha) {
    const double d = alpha - 1.0 / 3.0;
    const double cc = 1.0 / sqrt(9.0 * d);
    for (uint32_t r = 0; r < 4096u; ++r) {
        uint32_t o[4];
        philox_call(seed, i, t, stream, call0 + r, o);
        const double rad = sqrt(-2.0 * log_pos(u32_01(o[0])));
        double sn, cs;
        sincos_2pi(u32_01(o[1]), sn, cs);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const double x = rad * (h ? sn : cs);
            const double v1 = fma(cc, x, 1.0);
            if (v1 <= 0.0) continue;
            const double v = v1 * v1 * v1;
            const double u = u32_01(o[2 + h]);
            const double x2 = x * x;
            if (u < fma(-0.0331, x2 * x2, 1.0)) return d * v;
            if (log_pos(u) < fma(0.5, x2, d * ((1.0 - v) + log_pos(v)))) return d * v;
        }
    }
    return d;
}

NP8_HD double chi2_mt(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call0, double dof) {
    return 2.0 * gamma_mt(seed, i, t, stream, call0, 0.5 * dof);
}

// Normal number n of stream (i, t) counted from call c0 (normal_quad layout).
NP8_HD double normal_at(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t c0, uint32_t n) {
    double g[4];
    normal_quad(seed, i, t, stream, c0 + (n >> 2), g);
    return g[n & 3];
}

// chi^2_{D-1} = |z_perp|^2 of auxiliary draw `base`: D-1 squared normals for D <= 4, else Marsaglia-Tsang.
NP8_HD double niw_chi_perp(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t base, int D) {
    const int k = D - 1;
    if (k <= 0) return 0.0;
    if (k <= 3) {
        double g[4];
        normal_quad(seed, i, t, stream, base + kNiwAuxCalls - 2u, g);
        double s = g[0] * g[0];
        for (int j = 1; j < k; ++j) s = fma(g[j], g[j], s);
        return s;
    }
    return chi2_mt(seed, i, t, stream, base + kNiwGammaCalls * (uint32_t)D, (double)k);
}

// Sum of logs of chi^2 draws, taken over products of at most 16.
struct LogAcc {
    double prod = 1.0, sumlog = 0.0;
    NP8_HD void add(double g, int idx, int last) {
        prod *= g;
        if ((idx & 15) == 15 || idx == last) {
            sumlog += log_pos(prod);
            prod = 1.0;
        }
    }
};

// Auxiliary m of item i under the NIW prior, in the item's frame: the D Bartlett chi^2 draws
// (sumlog = sum log, b00 = sqrt of the first), chi^2_{D-1} and z_1.
NP8_HD void niw_aux_core(uint64_t seed, uint64_t i, uint32_t t, int m, int D, double nu0, double &sumlog, double &b00,
                         double &chi, double &z1) {
    const uint32_t base = (uint32_t)m * kNiwAuxCalls;
    LogAcc la;
    b00 = 0.0;
    for (int a = 0; a < D; ++a) {
        const double g = chi2_mt(seed, i, t, kStreamAuxNiw, base + kNiwGammaCalls * (uint32_t)a, nu0 - a);
        if (a == 0) b00 = sqrt(g);
        la.add(g, a, D - 1);
    }
    sumlog = la.sumlog;
    chi = niw_chi_perp(seed, i, t, kStreamAuxNiw, base, D);
    z1 = normal_at(seed, i, t, kStreamAuxNiw, base + kNiwAuxCalls - 1u, 0);
}

// Screened NIW auxiliary (DESIGN.md "Auxiliary screen"): the exact log-likelihood, or kZeroLogWeight when an
// upper bound from the first Bartlett draw and z_1 alone (smax bounds the other D-1 log chi^2 draws, chi >=
// 0) is at or below thr -- an auxiliary the pick would skip; then the other D chi^2 draws are not made.
NP8_HD double niw_aux_ll_screened(uint64_t seed, uint64_t i, uint32_t t, int m, int D, double nu0, double nd,
                                  double rsk, double caux, double smax, double thr);

// Level 0 of the NIW auxiliary screen: true when niw_aux_ll_screened would return kZeroLogWeight for EVERY auxiliary
// of an item at distance nd, whatever its draws -- its level-1 bound ub = caux + (log g0 + smax)/2 - e^2/2,
// e = nd sqrt(g0) - z1 rsk, maximised over all draws the generators can return: |z1| <= zm = sqrt(-2 log 2^-33)
// (Box-Muller over 32-bit uniforms) and g0 = 2 d v, v = (1 + cc x)^3 with |x| <= zm (Marsaglia-Tsang, d = nu0/2 - 1/3,
// cc = 1/sqrt(9 d); the 4096-failure fallback 2 d lies inside).  With s = sqrt(g0), r = rsk zm:
// log s - (nd s - r)_+^2 / 2 increases up to s* = (r + sqrt(r^2 + 4)) / (2 nd) and decreases after, so its maximum over
// [sqrt(gmin), sqrt(gmax)] is at s* clamped.  The level-1 test's margins (1e-9 |magnitude| + 1e-6) are covered with
// room: the quadratic is taken at (1 - 1e-9) and 1e-9 of every bounded magnitude is added.  Saves the 3 x (two
// Philox calls, a Marsaglia-Tsang attempt, Box-Muller, a log) of items far from mu0 in the prior's metric.
NP8_HD bool niw_aux_all_below(double nd, double nu0, double rsk, double caux, double smax, double thr) {
    constexpr double zm = 6.7638;  // > sqrt(66 ln 2) = 6.76375...
    const double d = 0.5 * nu0 - 1.0 / 3.0, cc = 1.0 / sqrt(9.0 * d);
    const double vlo = fmax(fma(-cc, zm, 1.0), 0.0), vhi = fma(cc, zm, 1.0);
    const double gmin = 2.0 * d * (vlo * vlo * vlo) * (1.0 - 1e-9), gmax = 2.0 * d * (vhi * vhi * vhi) * (1.0 + 1e-9);
    const double s0 = sqrt(gmin), s1 = sqrt(gmax), r = rsk * zm * (1.0 + 1e-12);
    const double ss = (nd > 0.0) ? (r + sqrt(fma(r, r, 4.0))) / (2.0 * nd) : s1;
    const double sc = fmin(fmax(ss, s0), s1);
    if (!(sc > 0.0)) return false;
    const double e = fmax(fma(nd, sc, -r), 0.0);
    const double h = fma(-0.5 * (1.0 - 1e-9), e * e, log_pos(sc) + 1e-12);
    const double ub0 = fma(0.5, smax, caux) + h;
    const double lmag = fmax(fabs(log_pos(fmax(gmin, 1e-300))), fabs(log_pos(gmax)));
    const double margin = 1e-9 * (fabs(caux) + 0.5 * (lmag + fabs(smax)) + fabs(ub0) + fabs(thr)) + 2e-6;
    return ub0 + margin <= thr;
}

// ll = caux + sumlog/2 - q/2, q = (|dt| b00 - z1/sqrt(kappa0))^2 + chi/kappa0 (nd = |dt|).
NP8_HD double niw_aux_loglik(double nd, double sumlog, double b00, double chi, double z1, double rsk, double caux) {
    const double e = fma(-z1, rsk, nd * b00);
    const double q = fma(e, e, chi * (rsk * rsk));
    return fma(-0.5, q, fma(0.5, sumlog, caux));
}

// Log-weight standing for weight 0 (a singleton's own cluster): finite, so no -inf arithmetic.
constexpr double kZeroLogWeight = -1.0e300;

NP8_HD double niw_aux_ll_screened(uint64_t seed, uint64_t i, uint32_t t, int m, int D, double nu0, double nd,
                                  double rsk, double caux, double smax, double thr) {
    const uint32_t base = (uint32_t)m * kNiwAuxCalls;
    const double g0 = chi2_mt(seed, i, t, kStreamAuxNiw, base, nu0);  // Bartlett a = 0, as niw_aux_core draws it
    const double z1 = normal_at(seed, i, t, kStreamAuxNiw, base + kNiwAuxCalls - 1u, 0);
    const double e = fma(-z1, rsk, nd * sqrt(g0));
    const double l0 = log_pos(g0);
    const double ub = fma(-0.5, e * e, fma(0.5, l0 + smax, caux));
    const double mag = fabs(caux) + 0.5 * (fabs(l0) + fabs(smax)) + 0.5 * e * e;
    if (ub + 1e-9 * mag + 1e-6 <= thr) return kZeroLogWeight;
    double sumlog, b00, chi, zz;
    niw_aux_core(seed, i, t, m, D, nu0, sumlog, b00, chi, zz);
    return niw_aux_loglik(nd, sumlog, b00, chi, zz, rsk, caux);
}
// Candidates with log-weight <= running max - kSkip are skipped (DESIGN.md "Pick"): a relative weight
// below e^-80 (1.8e-35) that no 53-bit uniform can resolve -- the reference's random_weighted_pick
// (dim1algebra.hpp:2078-2104) draws one double u; skipping saves the exp and the division.
constexpr double kSkip = 80.0;

// log Gamma(n), integer n >= 1 (the std::lgamma of np_jain_neal_algorithm.cpp:48): a table of
// log((n-1)!) to 32, Stirling's series beyond (truncation error < 1e-17 relative).
NP8_HD double lgamma_int(int64_t n) {
    constexpr double tab[33] = {
        0.0, 0.0, 0.0, 0.693147180559945, 1.7917594692280554, 3.178053830347945, 4.787491742782047,
        6.579251212010102, 8.525161361065415, 10.604602902745249, 12.801827480081467, 15.104412573075514,
        17.502307845873887, 19.987214495661885, 22.55216385312342, 25.191221182738683, 27.89927138384089,
        30.671860106080672, 33.50507345013689, 36.39544520803305, 39.339884187199495, 42.335616460753485,
        45.38013889847691, 48.47118135183522, 51.60667556776438, 54.78472939811232, 58.00360522298052,
        61.26170176100201, 64.55753862700634, 67.88974313718153, 71.257038967168, 74.65823634883017,
        78.0922235533153};
    if (n <= 32) return tab[n < 1 ? 1 : n];
    const double x = (double)n;
    const double r = 1.0 / x, r2 = r * r;
    const double s = r * (0.083333333333333333 -
                          r2 * (0.0027777777777777778 - r2 * (0.00079365079365079365 - r2 * 0.00059523809523809524)));
    return ((x - 0.5) * log_pos(x) - x) + 0.91893853320467274178 + s;
}

NP8_HD double uniform(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t n) {
    uint32_t o[4];
    philox_call(seed, i, t, stream, n, o);
    return u01(o[0], o[1]);
}

NP8_HD uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

// Sub-step of item i (global index) in a data-parallel sweep of S synchronous sub-steps: a fixed hash
// partition of the items (identical in oracle/np8_oracle.c np8o_substep_of).
NP8_HD uint32_t substep_of(uint64_t seed, int64_t i, uint32_t S) {
    if (S <= 1) return 0;
    const uint32_t h = fmix32(fmix32((uint32_t)i ^ 0x5EB57E95u ^ (uint32_t)(seed >> 32)) ^ (uint32_t)seed);
    return (uint32_t)(((uint64_t)h * S) >> 32);
}

// Scan-order bijection of a chunked sweep (replaces the reference's std::shuffle,
// include/helper/dim1algebra.hpp:2066-2073).
struct Perm {
    uint32_t N, h, mask, k[4];
};

NP8_HD Perm make_perm(uint64_t seed, uint32_t t, uint32_t N) {
    Perm P;
    P.N = N;
    int b = 0;
    while ((1ull << b) < (uint64_t)N) ++b;
    if (b < 2) b = 2;
    if (b & 1) ++b;
    P.h = (uint32_t)(b / 2);
    P.mask = (P.h >= 32) ? 0xFFFFFFFFu : ((1u << P.h) - 1u);
    for (int r = 0; r < 4; ++r)
        P.k[r] = fmix32((uint32_t)seed ^ fmix32(t * 4u + (uint32_t)r + 0x9E3779B9u)) ^ (uint32_t)(seed >> 32);
    return P;
}

NP8_HD uint32_t perm_apply(const Perm &P, uint32_t p) {
    if (P.N <= 1) return 0;
    uint32_t x = p;
    do {
        uint32_t L = x >> P.h, R = x & P.mask;
        for (int r = 0; r < 4; ++r) {
            const uint32_t nl = R;
            R = L ^ (fmix32(R ^ P.k[r]) & P.mask);
            L = nl;
        }
        x = (L << P.h) | R;
    } while (x >= P.N);
    return x;
}

NP8_HD double clamp_u(double u) { return fmin(fmax(u, 0x1.0p-60), 0x1.fffffffffffffp-1); }

// State of the single-uniform weighted reservoir draw (DESIGN.md "Pick"): T running max log-weight,
// S = sum of exp(lw - T) over the candidates taken into account, u ~ U(0,1) independent of pick.
struct PickState {
    double T, S, u;
    int32_t pick;
};

// Candidate j with log-weight lw.  Equal in distribution to an inverse-CDF draw over exp(lw)
// (dim1algebra.hpp:2078-2104); one exp and one division, no stored weights.
NP8_HD void pick_step(PickState &st, double lw, int32_t j) {
    const double d = lw - st.T;
    if (d <= -kSkip) return;
    const bool gt = d > 0.0;
    const double e = exp_le0(-fabs(d));
    const double a = gt ? 1.0 : e;
    const double S = gt ? fma(st.S, e, 1.0) : st.S + e;
    const double uS = st.u * S;
    const bool take = uS < a;
    const double num = take ? uS : uS - a;
    const double den = take ? a : S - a;
    st.u = clamp_u(num / den);
    st.pick = take ? j : st.pick;
    st.T = gt ? lw : st.T;
    st.S = S;
}

// The wide path's contraction rows of one slot from its fp64 factor R (upper, R^T R = P; element (a, b) at
// R[a * LDR + b], any storage) and its fp64 mean: A = fp32(R) natural [D][D] (An) and in MFMA-fragment order
// (Af: chunks (mt, s4), s4 >= mt, compact; in chunk c lane l's float4 element e (k-step ks = 4 s4 + e) holds
// A[16 mt + (l & 15)][4 ks + (l >> 4)]; then muf transposed, [g][s] = muf[4 s + g]) and muf = fp32(mu) (wmu).
// All threads of the block (np8_wide_rows, np8_niw_post).
// D < DT (a dimension that is not a multiple of 16): every table is laid out for DT, rows and columns >= D zero, so
// the contraction's extra terms are exact zeros -- fmaf(0, 0 - 0, y) = y and fmaf(0, 0, s) = s -- and q is the one
// of the D x D factor (the padded items are zero in those dims too).
__device__ inline void wide_write_rows(int D, int DT, const double *R, int LDR, const double *mu, float *An, float *Af,
                                       float *wmu) {
    for (int k = threadIdx.x; k < DT * DT; k += blockDim.x) {
        const int a = k / DT, b = k - a * DT;
        An[k] = (b >= a && b < D) ? (float)R[a * LDR + b] : 0.0f;
    }
    const int S = DT / 4, S4 = DT / 16, MT = DT / 16, NCH = MT * (MT + 1) / 2;
    for (int k = threadIdx.x; k < NCH * 256; k += blockDim.x) {
        const int e = k & 3, l = (k >> 2) & 63, c = k >> 8;
        int mt = 0;
        while (c >= (mt + 1) * S4 - (mt * (mt + 1)) / 2) ++mt;  // chunk -> (mt, s4)
        const int s4 = mt + (c - (mt * S4 - (mt * (mt - 1)) / 2));
        const int ks = 4 * s4 + e;
        const int ra = 16 * mt + (l & 15), rb = 4 * ks + (l >> 4);
        Af[k] = (rb >= ra && rb < D) ? (float)R[ra * LDR + rb] : 0.0f;
    }
    for (int k = threadIdx.x; k < DT; k += blockDim.x) {
        const int g = k / S, st = k - g * S, a = 4 * st + g;
        Af[NCH * 256 + k] = (a < D) ? (float)mu[a] : 0.0f;
    }
    for (int a = threadIdx.x; a < DT; a += blockDim.x) wmu[a] = (a < D) ? (float)mu[a] : 0.0f;
}

// The wide path's tile dimension: D rounded up to a multiple of 16.
NP8_HD constexpr int wide_dt(int D) { return (D + 15) & ~15; }

}  // namespace np8
