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
constexpr int kPickBlock = 32;    // candidates per pick block (DESIGN.md "Pick")
constexpr int kReqMax = 4096;     // new-cluster requests one finalize can accept
constexpr int kMaxD = 64;
constexpr int kMaxM = 8;

enum Stream : uint32_t { kStreamAux = 1, kStreamPick = 2, kStreamInitTheta = 3, kStreamInitZ = 4 };

// Candidate-table entry layout (doubles): [mu(D) | P'(D(D+1)/2) | c | logn | logn1 | slot]
NP8_HD int packed_size(int D) { return D * (D + 1) / 2; }
NP8_HD int cand_stride(int D) { return (D + packed_size(D) + 4 + 1) & ~1; }

NP8_HD uint32_t mulhi32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }

// Philox4x32-10 (Salmon et al. SC'11).
NP8_HD void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                          uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
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

NP8_HD void philox_call(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call, uint32_t out[4]) {
    philox4x32_10((uint32_t)i, (uint32_t)(i >> 32), t, (stream << 24) | (call & 0xFFFFFFu), (uint32_t)seed,
                  (uint32_t)(seed >> 32), out);
}

// Odd 53-bit integer times 2^-53: uniform on (0,1), never 0 or 1.
NP8_HD double u01(uint32_t hi, uint32_t lo) {
    uint64_t v = ((((uint64_t)hi) << 32) | lo) >> 11;
    v |= 1u;
    return (double)v * 0x1.0p-53;
}

NP8_HD void normal_pair(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call, double &g0,
                        double &g1) {
    uint32_t o[4];
    philox_call(seed, i, t, stream, call, o);
    const double u1 = u01(o[0], o[1]);
    const double u2 = u01(o[2], o[3]);
    const double r = sqrt(-2.0 * log(u1));
    const double th = kTwoPi * u2;
    g0 = r * cos(th);
    g1 = r * sin(th);
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

NP8_HD double clamp_u(double u) {
    u = (u < 0x1.0p-60) ? 0x1.0p-60 : u;
    u = (u > 0x1.fffffffffffffp-1) ? 0x1.fffffffffffffp-1 : u;
    return u;
}

// Running state of the block-reservoir categorical draw (DESIGN.md "Pick").
struct PickState {
    double Tm, S, u;
    int32_t pick;
};

// One block of N candidate log-weights (entries beyond the live count are -inf).
template <int N>
NP8_HD void pick_block(PickState &st, const double (&lw)[N], int32_t base) {
    double mb = -INFINITY;
#pragma unroll
    for (int j = 0; j < N; ++j) mb = fmax(mb, lw[j]);
    if (mb == -INFINITY) return;
    double e[N];
    double Sb = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        e[j] = exp(lw[j] - mb);
        Sb = Sb + e[j];
    }
    double Sbs;
    if (mb > st.Tm) {
        st.S = st.S * exp(st.Tm - mb);
        st.Tm = mb;
        Sbs = Sb;
    } else {
        Sbs = Sb * exp(mb - st.Tm);
    }
    st.S = st.S + Sbs;
    const double r = Sbs / st.S;
    if (st.u < r) {
        const double ui = st.u / r;
        const double tgt = ui * Sb;
        double cum = 0.0, lo = 0.0, ej = 1.0;
        int pk = -1;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const double prev = cum;
            cum = cum + e[j];
            const bool hit = (pk < 0) && (cum >= tgt);
            pk = hit ? j : pk;
            lo = hit ? prev : lo;
            ej = hit ? e[j] : ej;
        }
        if (pk < 0) {  // rounding guard: last positive weight
            cum = 0.0;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const bool pos = e[j] > 0.0;
                pk = pos ? j : pk;
                lo = pos ? cum : lo;
                ej = pos ? e[j] : ej;
                cum = cum + e[j];
            }
        }
        st.pick = base + pk;
        st.u = clamp_u((tgt - lo) / ej);
    } else {
        st.u = clamp_u((st.u - r) / (1.0 - r));
    }
}

}  // namespace np8
