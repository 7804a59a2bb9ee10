// np8_sm.hip -- Jain-Neal split-merge on the device (DESIGN.md "Split-merge"; the reference's
// JainNealAlgorithm, src/np_jain_neal_algorithm.cpp, driven by src/np_mcmc.cpp:117-164 with two scan
// permutations).  The attempts of a sweep form one sequential Metropolis-Hastings chain; the host runs
// them in speculative batches: every attempt of a batch is evaluated against the batch-start state
// (np8_sm_eval), the lowest accepted one is applied (np8_sm_apply) and the batch restarts after it.
// Attempts before the first acceptance see exactly the state the sequential chain would show them, so
// the result equals oracle/np8_oracle.c np8o_sm_sweep attempt for attempt.
//
// Per state (rebuilt after every accepted attempt, np8_launch_sm_members):
//   mem/off   members of every slot in ascending item order (a stable counting sort of z),
//   own[i]    ll of item i under its own slot,
//   cross     cross[r][k] = canon_sum over the members of live slot r of ll under live slot k:
//             a merge attempt is then O(1); a split walks its cluster's members once.
// canon_sum: 256 lane-strided partials (ascending member rank), then a pairwise tree -- the block
// reduction both kernels use, restated by the oracle.
#include <algorithm>

#include "np8_kernels.h"

namespace np8 {
namespace {

constexpr int kSmThreads = 256;
constexpr int kMemItems = kSmMemItems;
constexpr int kCrossTile = 8;    // live slots per cross-matrix block
constexpr int kSplitBlocks = 8192;  // waves walking queued splits (32 per CU)
constexpr uint32_t kStreamSmTheta = 9, kStreamSmAlloc = 10, kStreamSmAccept = 11;

// ll of x under (mu, P' packed upper with doubled off-diagonals, c): the oracle's slot_ll order.
template <int D>
__device__ __forceinline__ double packed_ll(const double (&x)[D], const double *mu, const double *P, double c) {
    double d[D];
#pragma unroll
    for (int a = 0; a < D; ++a) d[a] = x[a] - mu[a];
    double q = 0.0;
    int k = 0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double t = P[k++] * d[a];
#pragma unroll
        for (int b = a + 1; b < D; ++b) t = fma(P[k++], d[b], t);
        q = fma(t, d[a], q);
    }
    return fma(-0.5, q, c);
}

// The sweep's candidate form: isotropic rows (P' = iso I) by the |d|^2 shortcut, else packed.
template <int D>
__device__ __forceinline__ double sm_ll(const double (&x)[D], const double *mu, const double *P, double c, double iso) {
    if (iso > 0.0) {
        double d0 = x[0] - mu[0];
        double acc = d0 * d0;
#pragma unroll
        for (int a = 1; a < D; ++a) {
            const double d = x[a] - mu[a];
            acc = fma(d, d, acc);
        }
        return fma(-0.5, acc * iso, c);
    }
    return packed_ll<D>(x, mu, P, c);
}

// the isotropic branch of sm_ll alone
template <int D>
__device__ __forceinline__ double iso_ll(const double (&x)[D], const double *mu, double c, double iso) {
    double d0 = x[0] - mu[0];
    double acc = d0 * d0;
#pragma unroll
    for (int a = 1; a < D; ++a) {
        const double d = x[a] - mu[a];
        acc = fma(d, d, acc);
    }
    return fma(-0.5, acc * iso, c);
}

template <int D>
__device__ __forceinline__ void load_x(const SmArgs &A, int32_t i, double (&x)[D]) {
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = A.X[(int64_t)a * A.N + i];
}

// Block tree over s[0..256): s[t] += s[t + h], h = 128 .. 1.  Every thread must call it.
__device__ __forceinline__ double tree256(double *s, double v) {
    const int t = threadIdx.x;
    s[t] = v;
    __syncthreads();
    for (int h = kSmThreads / 2; h >= 1; h >>= 1) {
        if (t < h) s[t] += s[t + h];
        __syncthreads();
    }
    const double r = s[0];
    __syncthreads();
    return r;
}

__device__ __forceinline__ bool sm_accept(double x, double u) { return (x >= 0.0) || !(exp_le0(x) < u); }

// ---- member lists: stable counting sort of the items by slot ------------------------------------------
__global__ __launch_bounds__(kSmThreads) void np8_sm_hist(SmArgs A) {
    extern __shared__ int lh[];
    for (int s = threadIdx.x; s < A.kcap; s += kSmThreads) lh[s] = 0;
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * kMemItems;
    for (int k = threadIdx.x; k < kMemItems; k += kSmThreads)
        if (i0 + k < A.N) atomicAdd(&lh[A.z[i0 + k]], 1);
    __syncthreads();
    for (int s = threadIdx.x; s < A.kcap; s += kSmThreads) A.hist[(int64_t)s * A.nbk + blockIdx.x] = lh[s];
}

// One block per slot: exclusive scan of its per-block counts (bases relative to the slot's start)
// and the slot total (into off[s], turned into the slot offset by np8_sm_scan_slots).
__global__ __launch_bounds__(kSmThreads) void np8_sm_scan_blocks(SmArgs A) {
    __shared__ int sc[kSmThreads];
    const int s = blockIdx.x, t = threadIdx.x;
    int carry = 0;
    for (int b0 = 0; b0 < A.nbk; b0 += kSmThreads) {
        const int64_t k = (int64_t)s * A.nbk + b0 + t;
        const int h = (b0 + t < A.nbk) ? A.hist[k] : 0;
        sc[t] = h;
        __syncthreads();
        for (int o = 1; o < kSmThreads; o <<= 1) {  // inclusive Hillis-Steele
            const int v = (t >= o) ? sc[t - o] : 0;
            __syncthreads();
            sc[t] += v;
            __syncthreads();
        }
        if (b0 + t < A.nbk) A.hist[k] = carry + sc[t] - h;
        carry += sc[kSmThreads - 1];
        __syncthreads();
    }
    if (t == 0) A.off[s] = carry;
}

// One block of 1024: exclusive scan of the slot totals into off[], the live list.
__global__ __launch_bounds__(1024) void np8_sm_scan_slots(SmArgs A) {
    __shared__ int part[1024];
    const int t = threadIdx.x;
    const int per = (A.kcap + 1023) / 1024;
    const int s0 = min(A.kcap, t * per), s1 = min(A.kcap, s0 + per);
    int sum = 0;
    for (int s = s0; s < s1; ++s) sum += A.off[s];
    part[t] = sum;
    __syncthreads();
    for (int h = 1; h < 1024; h <<= 1) {  // inclusive Hillis-Steele scan
        const int v = (t >= h) ? part[t - h] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - sum, iso = 1;
    for (int s = s0; s < s1; ++s) {
        const int tot = A.off[s];
        A.off[s] = run;
        run += tot;
        const int d = A.dense[s];
        if (d >= 0) {
            A.live[d] = s;
            iso &= (A.slot_iso[s] > 0.0) ? 1 : 0;
        }
    }
    iso = __syncthreads_and(iso);
    if (t == 1023) A.off[A.kcap] = part[1023];
    if (t == 0) A.sc->all_iso = iso;
}

// One wave per block of kMemItems items, 64 at a time in item order: rank among equal slots of the
// lower lanes, the last lane of each slot advances the base.
// ... and each item's row and own-slot likelihood into member order as it is placed (item-order reads
// coalesced; Xm[a][pos] = X[a][i], ownm[pos] = ll(x_i | z_i)).
template <int D>
__global__ __launch_bounds__(64) void np8_sm_scatter(SmArgs A) {
    constexpr int DP = D * (D + 1) / 2;
    extern __shared__ int base[];
    const int lane = threadIdx.x;
    for (int s = lane; s < A.kcap; s += 64) base[s] = A.off[s] + A.hist[(int64_t)s * A.nbk + blockIdx.x];
    __syncthreads();
    const int64_t i0 = (int64_t)blockIdx.x * kMemItems;
    for (int c = 0; c < kMemItems; c += 64) {
        const int64_t i = i0 + c + lane;
        const int key = (i < A.N) ? A.z[i] : -1;
        int below = 0, above = 0;
        for (int l = 0; l < 64; ++l) {
            const int kl = __shfl(key, l);
            below += (l < lane && kl == key);
            above += (l > lane && kl == key);
        }
        if (key >= 0) {
            const int pos = base[key] + below;
            A.mem[pos] = (int32_t)i;
            double x[D];
            load_x<D>(A, (int32_t)i, x);
#pragma unroll
            for (int a = 0; a < D; ++a) A.Xm[(int64_t)a * A.N + pos] = x[a];
            A.ownm[pos] = sm_ll<D>(x, A.slot_mu + (int64_t)key * D, A.slot_P + (int64_t)key * DP, A.slot_c[key],
                                   A.slot_iso[key]);
        }
        __syncthreads();
        if (key >= 0 && above == 0) base[key] += below + 1;
        __syncthreads();
    }
}

template <int D>
__device__ __forceinline__ void load_xm(const SmArgs &A, int64_t p, double (&x)[D]) {
#pragma unroll
    for (int a = 0; a < D; ++a) x[a] = A.Xm[(int64_t)a * A.N + p];
}

// Block (row r, tile of kCrossTile live slots): cross[r][k0 + kk].
template <int D>
__global__ __launch_bounds__(kSmThreads) void np8_sm_cross(SmArgs A) {
    constexpr int DP = D * (D + 1) / 2;
    __shared__ double th[kCrossTile][D + DP + 2];  // mu | P' | c | iso
    __shared__ double red[kSmThreads];
    const int r = blockIdx.x, k0 = blockIdx.y * kCrossTile;
    const int nk = min(kCrossTile, A.K - k0);
    for (int e = threadIdx.x; e < kCrossTile * (D + DP + 2); e += kSmThreads) {
        const int kk = e / (D + DP + 2), f = e - kk * (D + DP + 2);
        const int s = A.live[min(k0 + kk, A.K - 1)];  // padding rows repeat the last slot (unused)
        th[kk][f] = (f < D) ? A.slot_mu[(int64_t)s * D + f]
                            : (f < D + DP ? A.slot_P[(int64_t)s * DP + (f - D)]
                                          : (f == D + DP ? A.slot_c[s] : A.slot_iso[s]));
    }
    __syncthreads();
    const int sr = A.live[r];
    const int b = A.off[sr], n = A.off[sr + 1] - b;
    double acc[kCrossTile];
#pragma unroll
    for (int kk = 0; kk < kCrossTile; ++kk) acc[kk] = 0.0;
    for (int p = threadIdx.x; p < n; p += kSmThreads) {
        double x[D];
        load_xm<D>(A, b + p, x);
#pragma unroll
        for (int kk = 0; kk < kCrossTile; ++kk) {
            // re-read the parameters from LDS for every member (hoisting 8 x 45 doubles would spill)
            __asm__ __volatile__("" ::: "memory");
            acc[kk] += sm_ll<D>(x, &th[kk][0], &th[kk][D], th[kk][D + DP], th[kk][D + DP + 1]);
        }
    }
#pragma unroll
    for (int kk = 0; kk < kCrossTile; ++kk) {
        const double v = tree256(red, acc[kk]);
        if (kk < nk && threadIdx.x == 0) A.cross[(int64_t)r * A.K + k0 + kk] = v;
    }
}

// Triadic merge bound (DESIGN.md 2e "Merge bound"), per state: for live row r, over its members x,
//   mb[r][0] = sum max_k ll_k(x)          (every live slot k),   mb[r][1] = sum |max_k ll_k(x)|,
//   mb[r][2] = sum max_{k != own} ll_k(x) (every other slot),    mb[r][3] = sum |...|,
// with ll_k = sm_ll, the walk's own likelihood bit for bit.  A triadic merge moves every member of its
// three sources onto two of them, so its after-move sum is at most mb[r0][0] + mb[r1][0] + mb[r2][2].
// Block (row r, member chunk): the live slots staged in LDS 64 at a time; one atomic per block and sum
// (the order of these sums only enters the bound through its error margin).
constexpr int kBoundTile = 64, kBoundChunks = 16;
template <int D>
__global__ __launch_bounds__(kSmThreads) void np8_tri_bound(SmArgs A) {
    constexpr int DP = D * (D + 1) / 2, W = D + DP + 2;
    __shared__ double th[kBoundTile][W];
    __shared__ double red[kSmThreads];
    const int r = blockIdx.x;
    const int sr = A.live[r];
    const int b = A.off[sr], n = A.off[sr + 1] - b;
    const int per = (n + kBoundChunks - 1) / kBoundChunks;
    const int p0 = min(n, (int)blockIdx.y * per), p1 = min(n, p0 + per);
    double s_all = 0.0, a_all = 0.0, s_ex = 0.0, a_ex = 0.0;
    for (int pb = p0; pb < p1; pb += kSmThreads) {  // block-uniform
        const int p = pb + threadIdx.x;
        const bool valid = p < p1;
        double x[D];
#pragma unroll
        for (int a = 0; a < D; ++a) x[a] = 0.0;
        if (valid) load_xm<D>(A, b + p, x);
        double mall = -__builtin_huge_val(), mex = -__builtin_huge_val();
        for (int k0 = 0; k0 < A.K; k0 += kBoundTile) {
            const int nk = min(kBoundTile, A.K - k0);
            __syncthreads();
            for (int e = threadIdx.x; e < nk * W; e += kSmThreads) {
                const int kk = e / W, f = e - kk * W;
                const int s = A.live[k0 + kk];
                th[kk][f] = (f < D) ? A.slot_mu[(int64_t)s * D + f]
                                    : (f < D + DP ? A.slot_P[(int64_t)s * DP + (f - D)]
                                                  : (f == D + DP ? A.slot_c[s] : A.slot_iso[s]));
            }
            __syncthreads();
            if (valid) {
                for (int kk = 0; kk < nk; ++kk) {
                    __asm__ __volatile__("" ::: "memory");  // parameters stay in LDS
                    const double l = sm_ll<D>(x, &th[kk][0], &th[kk][D], th[kk][D + DP], th[kk][D + DP + 1]);
                    mall = fmax(mall, l);
                    mex = (k0 + kk == r) ? mex : fmax(mex, l);
                }
            }
        }
        if (valid) {
            s_all += mall;
            a_all += fabs(mall);
            s_ex += mex;
            a_ex += fabs(mex);
        }
    }
    const double v0 = tree256(red, s_all), v1 = tree256(red, a_all), v2 = tree256(red, s_ex), v3 = tree256(red, a_ex);
    if (threadIdx.x == 0 && p1 > p0) {
        atomicAdd(&A.mb[4 * r + 0], v0);
        atomicAdd(&A.mb[4 * r + 1], v1);
        atomicAdd(&A.mb[4 * r + 2], v2);
        atomicAdd(&A.mb[4 * r + 3], v3);
    }
}

// ---- attempts ----------------------------------------------------------------------------------------------
// Outcome codes as np8o_sm_sweep: 0 skipped, 1 split rejected, 2 merge rejected, 3 split accepted,
// 4 merge accepted, 5 split rejected for want of a free slot; kPending: a split not evaluated (its
// attempt lies after an accepted one).
constexpr uint8_t kPending = 255;

struct Pair {
    int32_t i, j, ci, cj;
};

__device__ __forceinline__ Pair sm_pair(const SmArgs &A, int64_t a) {
    Pair q;
    q.i = (int32_t)perm_apply(A.perm0, (uint32_t)a);
    q.j = (int32_t)perm_apply(A.perm1, (uint32_t)a);
    q.ci = A.z[q.i];
    q.cj = A.z[q.j];
    return q;
}

// merge ci into cj (np_jain_neal_algorithm.cpp:353-429): O(1) from the cross matrix
__device__ __forceinline__ bool sm_merge_accept(const SmArgs &A, const Pair &q, int64_t a) {
    const int r0 = A.dense[q.ci], r1 = A.dense[q.cj];
    const double lsrc = A.cross[(int64_t)r0 * A.K + r0], ldest = A.cross[(int64_t)r0 * A.K + r1];
    const int n0 = A.off[q.ci + 1] - A.off[q.ci], n1 = A.off[q.cj + 1] - A.off[q.cj];
    const double pr = A.log_alpha + lgamma_int(n0) + lgamma_int(n1) - lgamma_int((int64_t)n0 + n1);
    return sm_accept(-pr + (ldest - lsrc), uniform(A.seed, (uint64_t)a, A.t, kStreamSmAccept, 0));
}

// The new cluster of split attempt a: a G0 draw (v, mu) on stream SM_THETA (the oracle's sm_theta).
template <int D>
__device__ void sm_theta(const SmArgs &A, int64_t a, double *vmu) {
    double g[4 * ((D + 4) / 4)];
    for (int call = 0; call < g0_calls(D); ++call) {
        double q[4];
        normal_quad(A.seed, (uint64_t)a, A.t, kStreamSmTheta, (uint32_t)call, q);
        for (int e = 0; e < 4; ++e) g[4 * call + e] = q[e];
    }
    const double v = fma(A.nu, g[0], (double)D);
    const double sc = fabs(v) * A.rsk;
    for (int aa = 0; aa < D; ++aa) {
        double t0 = A.LT[aa * D + aa] * g[1 + aa];
        for (int bb = aa + 1; bb < D; ++bb) t0 = fma(A.LT[aa * D + bb], g[1 + bb], t0);
        vmu[1 + aa] = fma(sc, t0, A.mu0[aa]);
    }
    vmu[0] = v;
}

// One thread per attempt: pairs, skips and merges decided here, splits queued (with their new
// cluster's G0 draw) for np8_sm_split.
template <int D>
__global__ __launch_bounds__(kSmThreads) void np8_sm_classify(SmArgs A) {
    const int q = blockIdx.x * kSmThreads + threadIdx.x;
    if (q >= A.nb) return;
    const int64_t a = A.a0 + q;
    const Pair p = sm_pair(A, a);
    uint8_t out;
    if (p.i == p.j) {
        out = 0;
    } else if (p.ci != p.cj) {
        out = sm_merge_accept(A, p, a) ? 4 : 2;
        if (out == 4) atomicMin(reinterpret_cast<unsigned long long *>(&A.sc->first), (unsigned long long)a);
    } else {
        out = kPending;
        const int e = atomicAdd(&A.sc->nsplit, 1);
        A.slist[e] = a;
        sm_theta<D>(A, a, A.stheta + (int64_t)e * (D + 1));
    }
    A.typ[q] = out;
}

// Split of the common cluster c of (i, j) (np_jain_neal_algorithm.cpp:251-351), one wave.  The new
// cluster is a G0 draw.  Members are visited in ascending item order, 64 per step, one per lane: each
// lane computes its member's likelihood under the new cluster and its allocation uniform, then the
// wave resolves the sequential allocation (:146-171) of the 64 by fixpoint iteration: a lane's
// decision depends only on the decisions of the lanes before it (through the set sizes), so
// re-deciding every lane from the previous round's prefix counts fixes at least one more lane per
// round and stops at the unique fixpoint -- the sequential result, usually after 2 rounds.  Masked
// sums go to 256 canonical partials (member rank mod 256) reduced by canon_sum's tree.
// APPLY: write the moves.
template <int D, bool APPLY, bool ISO = false>  // ISO: the new cluster's P' is a multiple of I (gp_iso > 0)
__device__ int sm_split(const SmArgs &A, const FinArgs *F, const Pair &pq, int64_t a, const double *vmu) {
    constexpr int DP = D * (D + 1) / 2;
    __shared__ double s_red[2][256];
    __shared__ double s_th[D + DP + 3];  // mu' | P' | c' | v | iso'
    __shared__ int s_new_slot;
    const int lane = threadIdx.x;
    const int ci = pq.ci;
    if (lane == 0) {
        const double v = vmu[0];
        for (int aa = 0; aa < D; ++aa) s_th[aa] = vmu[1 + aa];
        const double v2 = v * v;
#pragma unroll 1
        for (int k = 0; k < DP; ++k) s_th[D + k] = A.Gp[k] / v2;
        s_th[D + DP] = fma(-(double)D, log_pos(fabs(v)), A.caux);
        s_th[D + DP + 1] = v;
        s_th[D + DP + 2] = (A.gp_iso > 0.0) ? A.gp_iso / v2 : 0.0;
        if (APPLY) {
            int s = -1;
            for (int k = 0; k < A.kcap; ++k)
                if (A.cnt[k] == 0) {
                    s = k;
                    break;
                }
            s_new_slot = s;
        }
    }
    __syncthreads();
    const int snew = APPLY ? s_new_slot : -1;
    const int b0 = A.off[ci], n0 = A.off[ci + 1] - b0;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));  // lanes < this one
    double dm = 1.0, dr = 1.0;  // sizes of the move (holds i) and remain (holds j) sets, wave-uniform
    double ps[4] = {0.0, 0.0, 0.0, 0.0}, pd[4] = {0.0, 0.0, 0.0, 0.0};  // partials lane + 64 k
    for (int cb = 0; cb < n0; cb += 64) {
        const int k = (cb >> 6) & 3;
        {
            const int p = cb + lane;
            const bool valid = p < n0;
            int32_t id = -1;
            double own = 0.0, nw = 0.0, u = 0.0;
            if (valid) {
                __asm__ __volatile__("" ::: "memory");  // the new cluster's P' stays in LDS (occupancy)
                double x[D];
                load_xm<D>(A, b0 + p, x);
                id = A.mem[b0 + p];
                own = A.ownm[b0 + p];
                nw = ISO ? iso_ll<D>(x, s_th, s_th[D + DP], s_th[D + DP + 2])
                         : sm_ll<D>(x, s_th, s_th + D, s_th[D + DP], s_th[D + DP + 2]);
                u = uniform(A.seed, (uint64_t)a, A.t, kStreamSmAlloc, (uint32_t)p);
            }
            const bool isI = id == pq.i, isJ = id == pq.j;
            const bool regular = valid && !isI && !isJ;
            const uint64_t reg = __ballot(regular);
            const int cnt = __popcll(reg & below);
            uint64_t mv = 0;  // regular lanes that move, as last decided
            for (int it = 0; it <= 64; ++it) {
                const int dl = __popcll(mv & below);
                const double a0 = own + (dr + (double)(cnt - dl)), a1 = nw + (dm + (double)dl);
                const double tot = a0 + a1;
                const double w = u * tot;
                const bool d = regular && ((tot < w) || (a0 < w));  // lower_bound over {a0, a0 + a1} > 0
                const uint64_t nmv = __ballot(d);
                if (nmv == mv) break;  // wave-uniform
                mv = nmv;
            }
            const bool moves = isI || ((mv >> lane) & 1ull);
            const int nm = __popcll(mv);
            dm += (double)nm;
            dr += (double)(__popcll(reg) - nm);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {  // static register indices
                ps[kk] = (moves && kk == k) ? ps[kk] + own : ps[kk];
                pd[kk] = (moves && kk == k) ? pd[kk] + nw : pd[kk];
            }
            if (APPLY && moves && snew >= 0) A.z[id] = snew;
        }
    }
    // canon_sum: partial t = lane + 64 k, then the pairwise tree
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        s_red[0][lane + 64 * k] = ps[k];
        s_red[1][lane + 64 * k] = pd[k];
    }
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {
        for (int t = lane; t < h; t += 64) {
            s_red[0][t] += s_red[0][t + h];
            s_red[1][t] += s_red[1][t + h];
        }
        __syncthreads();
    }
    const double lsrc = s_red[0][0], ldest = s_red[1][0];
    const int64_t m = (int64_t)dm, r = (int64_t)dr;
    int out = 1;
    if (lane == 0) {
        const double pr = A.log_alpha + lgamma_int(m) + lgamma_int(r) - lgamma_int(n0);
        const bool acc = sm_accept(pr + (ldest - lsrc), uniform(A.seed, (uint64_t)a, A.t, kStreamSmAccept, 0));
        out = !acc ? 1 : (A.K < A.kcap ? 3 : 5);
        if (APPLY && out == 3 && snew >= 0) {
            write_new_slot(*F, vmu, snew);
            if (F->wdirty) F->wdirty[snew] = 1;
            A.cnt[ci] -= (int32_t)m;
            A.cnt[snew] = (int32_t)m;
        }
    }
    __syncthreads();
    return out;  // lane 0's value
}

// The queued splits of the batch, one wave each (persistent over the queue); a split after an
// already accepted attempt is left pending -- the batch restarts before it.
template <int D, bool ISO>
__global__ __launch_bounds__(64) void np8_sm_split(SmArgs A) {
    const int ns = A.sc->nsplit;
    for (int e = blockIdx.x; e < ns; e += gridDim.x) {
        const int64_t a = A.slist[e];
        unsigned long long first = 0;
        if (threadIdx.x == 0) first = *reinterpret_cast<volatile unsigned long long *>(&A.sc->first);
        first = __shfl(first, 0);
        if ((unsigned long long)a > first) continue;  // wave-uniform
        const Pair p = sm_pair(A, a);
        const int out = sm_split<D, false, ISO>(A, nullptr, p, a, A.stheta + (int64_t)e * (D + 1));
        if (threadIdx.x == 0) {
            A.typ[a - A.a0] = (uint8_t)out;
            if (out == 3) atomicMin(reinterpret_cast<unsigned long long *>(&A.sc->first), (unsigned long long)a);
        }
    }
}

// Outcome counts of the attempts up to and including the first accepted one (grid-stride, one
// 64-bit atomic per block and outcome).
__global__ __launch_bounds__(kSmThreads) void np8_sm_tally(SmArgs A) {
    __shared__ int cnt[6];
    if (threadIdx.x < 6) cnt[threadIdx.x] = 0;
    __syncthreads();
    const int64_t first = A.sc->first;
    const int lim = (first == INT64_MAX) ? A.nb : (int)(first - A.a0 + 1);
    int c[6] = {0, 0, 0, 0, 0, 0};
    for (int q = blockIdx.x * kSmThreads + threadIdx.x; q < lim; q += gridDim.x * kSmThreads) {
        const uint8_t t = A.typ[q];
#pragma unroll
        for (int k = 0; k < 6; ++k) c[k] += (t == k);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (c[k]) atomicAdd(&cnt[k], c[k]);
    __syncthreads();
    if (threadIdx.x < 6 && cnt[threadIdx.x])
        atomicAdd(reinterpret_cast<unsigned long long *>(&A.sc->stats[threadIdx.x]), (unsigned long long)cnt[threadIdx.x]);
}

// The batch's first accepted attempt, re-evaluated by one wave and applied.
template <int D>
__global__ __launch_bounds__(64) void np8_sm_apply(SmArgs A, FinArgs F, int64_t a) {
    const Pair p = sm_pair(A, a);
    __syncthreads();  // the apply rewrites z: every lane has read z[i], z[j] first
    int out;
    if (p.i == p.j) {
        out = 0;
    } else if (p.ci != p.cj) {
        out = sm_merge_accept(A, p, a) ? 4 : 2;
        if (out == 4) {
            const int b0 = A.off[p.ci], n0 = A.off[p.ci + 1] - b0;
            for (int q = threadIdx.x; q < n0; q += 64) A.z[A.mem[b0 + q]] = p.cj;
            if (threadIdx.x == 0) {
                A.cnt[p.cj] += n0;
                A.cnt[p.ci] = 0;
            }
        }
    } else {
        __shared__ double vmu[D + 1];
        if (threadIdx.x == 0) sm_theta<D>(A, a, vmu);
        __syncthreads();
        out = sm_split<D, true>(A, &F, p, a, vmu);
    }
    if (threadIdx.x == 0) {
        if (out != 3 && out != 4) F.ctl->err |= kErrCapacity;  // cannot happen: re-evaluation
        F.ctl->cand_fresh = 0;  // counts and slots changed behind np8_finalize: recopy the rows
    }
}

// ---- triadic split-merge (src/np_triadic_algorithm.cpp; the oracle's tri_attempt) ------------------------
// Outcomes: 0 skipped, 1/2 dyadic merge rejected/accepted, 3/4 dyadic split, 5/6 triadic merge (3 -> 2),
// 7/8 triadic split (2 -> 3), 9 split without a free slot.
struct Tri {
    int kind;  // -1 skipped, 0 dyadic merge, 1 dyadic split, 2 triadic merge, 3 triadic split
    int ns, Q;  // source clusters, target clusters
    int32_t pk[3];
    int cl[3];
};

__device__ __forceinline__ int tri_dup(const int (&c)[3]) {
    if (c[1] == c[0]) return 1;
    return 2;  // c[2] repeats an earlier id, or all differ (duplicate_pick returns the last index)
}

__device__ Tri tri_case(const SmArgs &A, int64_t a) {
    Tri T;
#pragma unroll
    for (int r = 0; r < 3; ++r) T.pk[r] = (int32_t)perm_apply(A.tperm[r], (uint32_t)a);
    T.kind = -1;
    T.ns = T.Q = 0;
    if (T.pk[0] == T.pk[1] || T.pk[0] == T.pk[2] || T.pk[1] == T.pk[2]) return T;
#pragma unroll
    for (int r = 0; r < 3; ++r) T.cl[r] = A.z[T.pk[r]];
    const int uniq = 1 + (T.cl[1] != T.cl[0]) + (T.cl[2] != T.cl[0] && T.cl[2] != T.cl[1]);
    const double ub = uniform(A.seed, (uint64_t)a, A.t, kStreamSmAccept, 1);
    if (uniq == 1) {
        T.kind = 1;
        T.pk[1] = T.pk[2];
        T.cl[1] = T.cl[2];
    } else if (ub < 0.5) {
        T.kind = 0;
        if (tri_dup(T.cl) == 1) {
            T.pk[1] = T.pk[2];
            T.cl[1] = T.cl[2];
        }
    } else if (uniq == 2) {
        T.kind = 3;
        if (tri_dup(T.cl) == 1) {  // swap positions 1 and 2 (the duplicate goes last)
            const int32_t tp = T.pk[1];
            const int tc = T.cl[1];
            T.pk[1] = T.pk[2];
            T.cl[1] = T.cl[2];
            T.pk[2] = tp;
            T.cl[2] = tc;
        }
    } else {
        T.kind = 2;
    }
    T.ns = (T.kind == 1) ? 1 : (T.kind == 2 ? 3 : 2);
    T.Q = (T.kind == 0) ? 1 : (T.kind == 3 ? 3 : 2);
    return T;
}

__device__ __forceinline__ double tri_own(const SmArgs &A, int s) {
    const int r = A.dense[s];
    return A.cross[(int64_t)r * A.K + r];
}

// dyadic merge 2 -> 1 (:470-631 with C = 2): O(1) from the cross matrix
__device__ __forceinline__ bool tri_dyadic_merge_accept(const SmArgs &A, const Tri &T, int64_t a) {
    const int ra = A.dense[T.cl[0]], rb = A.dense[T.cl[1]];
    const double ld0 = A.cross[(int64_t)ra * A.K + ra], ld1 = A.cross[(int64_t)rb * A.K + rb];
    const double lp0 = (0.0 + ld0) + A.cross[(int64_t)rb * A.K + ra];
    const int na = A.off[T.cl[0] + 1] - A.off[T.cl[0]], nb = A.off[T.cl[1] + 1] - A.off[T.cl[1]];
    const double frac = ((0.0 + lgamma_int(na)) + lgamma_int(nb)) - lgamma_int((int64_t)na + nb);
    const double rP = -(A.log_alpha + frac);
    const double rLd = (0.0 + ld0) + ld1, rLdp = 0.0 + lp0;
    const double x = ((0.0 + rP) + A.lrr[0]) + (rLdp - rLd);
    return sm_accept(x, uniform(A.seed, (uint64_t)a, A.t, kStreamSmAccept, 0));
}

// Triadic merge 3 -> 2 rejected without its walk (DESIGN.md 2e "Merge bound"): the walk's acceptance
// exponent x = rP + rR + (after - before) is at most
//   rP  <= -(log alpha + sum_i lgamma(n_i) - lgamma(n - 1))   (sum_q lgamma(N_q) over N_0 + N_1 = n, N_q >= 1,
//                                                              is largest at (1, n - 1): lgamma is convex)
//   after <= mb[r0][0] + mb[r1][0] + mb[r2][2]                  (np8_tri_bound; targets are slots 0 and 1)
// plus a margin for the different summation orders (n u sum|terms| <= 1.2e-10 sum|terms| at n <= 2^20,
// lgamma_int's 2e-15).  When that bound is below log u by 1e-6, exp_le0(x) < u: the walk would reject.
__device__ __forceinline__ bool tri_merge_bound_rejects(const SmArgs &A, const Tri &T, int64_t a) {
    const int r0 = A.dense[T.cl[0]], r1 = A.dense[T.cl[1]], r2 = A.dense[T.cl[2]];
    const int n0 = A.off[T.cl[0] + 1] - A.off[T.cl[0]], n1 = A.off[T.cl[1] + 1] - A.off[T.cl[1]],
              n2 = A.off[T.cl[2] + 1] - A.off[T.cl[2]];
    const double g0 = lgamma_int(n0), g1 = lgamma_int(n1), g2 = lgamma_int(n2);
    const double gn = lgamma_int((int64_t)n0 + n1 + n2 - 1);
    const double rp = -(A.log_alpha + ((g0 + g1) + g2) - gn);
    const double before = (tri_own(A, T.cl[0]) + tri_own(A, T.cl[1])) + tri_own(A, T.cl[2]);
    const double after = (A.mb[4 * r0] + A.mb[4 * r1]) + A.mb[4 * r2 + 2];
    const double mag = A.mb[4 * r0 + 1] + A.mb[4 * r1 + 1] + A.mb[4 * r2 + 3] + fabs(before) + fabs(A.log_alpha) + g0 +
                       g1 + g2 + gn + fabs(A.lrr[2]);
    const double xub = ((rp + A.lrr[2]) + (after - before)) + (1e-9 * mag + 1e-6);
    if (!(xub < 0.0)) return false;
    const double u = uniform(A.seed, (uint64_t)a, A.t, kStreamSmAccept, 0);
    return xub < log_pos(u) - 1e-6;
}

template <int D>
__global__ __launch_bounds__(kSmThreads) void np8_tri_classify(SmArgs A) {
    const int q = blockIdx.x * kSmThreads + threadIdx.x;
    if (q >= A.nb) return;
    const int64_t a = A.a0 + q;
    const Tri T = tri_case(A, a);
    uint8_t out;
    if (T.kind < 0) {
        out = 0;
    } else if (T.kind == 0) {
        out = tri_dyadic_merge_accept(A, T, a) ? 2 : 1;
        if (out == 2) atomicMin(reinterpret_cast<unsigned long long *>(&A.sc->first), (unsigned long long)a);
    } else if (T.kind == 2 && A.mb && tri_merge_bound_rejects(A, T, a)) {
        out = 5;  // what the walk returns for a rejected triadic merge (1 + 2 kind)
    } else {
        out = kPending;
        const int e = atomicAdd(&A.sc->nsplit, 1);
        A.slist[e] = a;
        if (T.kind & 1) sm_theta<D>(A, a, A.stheta + (int64_t)e * (D + 1));
    }
    A.typ[q] = out;
}

// A walk move (dyadic split, triadic merge or split), one wave: every member of the sources is
// reallocated over the targets (picks fixed), 64 members per step resolved by fixpoint iteration
// over the target-size prefix counts; after-move likelihood sums per source in canon_sum order.
template <int D, bool APPLY, bool ISO = false>  // ISO: every target's P' is a multiple of I
__device__ int tri_walk(const SmArgs &A, const FinArgs *F, const Tri &T, int64_t a, const double *vmu) {
    constexpr int DP = D * (D + 1) / 2, W = D + DP + 2;  // mu | P' | c | iso
    __shared__ double s_tg[3][W];
    __shared__ double s_red[3][256];
    __shared__ int s_slot[3];
    __shared__ int s_new_slot;
    const int lane = threadIdx.x;
    const bool split = (T.kind & 1) != 0;
    const int Q = T.Q, ns = T.ns;
    // the case in scalars (indexing the struct with a loop variable would place it in scratch)
    const int32_t pk0 = T.pk[0], pk1 = T.pk[1], pk2 = T.pk[2];
    const int cl0 = T.cl[0], cl1 = T.cl[1], cl2 = T.cl[2];
    if (lane == 0) {
        for (int q = 0; q < Q; ++q) {
            const int s = (split && q == Q - 1) ? -1 : (q == 0 ? cl0 : (q == 1 ? cl1 : cl2));
            s_slot[q] = s;
            if (s >= 0) {
                for (int f = 0; f < D; ++f) s_tg[q][f] = A.slot_mu[(int64_t)s * D + f];
#pragma unroll 1
                for (int f = 0; f < DP; ++f) s_tg[q][D + f] = A.slot_P[(int64_t)s * DP + f];
                s_tg[q][D + DP] = A.slot_c[s];
                s_tg[q][D + DP + 1] = A.slot_iso[s];
            } else {
                const double v = vmu[0], v2 = v * v;
                for (int f = 0; f < D; ++f) s_tg[q][f] = vmu[1 + f];
#pragma unroll 1
                for (int f = 0; f < DP; ++f) s_tg[q][D + f] = A.Gp[f] / v2;
                s_tg[q][D + DP] = fma(-(double)D, log_pos(fabs(v)), A.caux);
                s_tg[q][D + DP + 1] = (A.gp_iso > 0.0) ? A.gp_iso / v2 : 0.0;
            }
        }
        if (APPLY) {
            int s = -1;
            if (split)
                for (int k = 0; k < A.kcap; ++k)
                    if (A.cnt[k] == 0) {
                        s = k;
                        break;
                    }
            s_new_slot = s;
        }
    }
    __syncthreads();
    const int snew = APPLY ? s_new_slot : -1;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    double Nq[3] = {1.0, 1.0, 1.0};  // target sizes, wave-uniform (each pick starts its target)
    double lp[3] = {0.0, 0.0, 0.0};  // lane 0
    int rank = 0;
    int nsrc[3] = {0, 0, 0};
    for (int si = 0; si < ns; ++si) {
        const int s = (si == 0) ? cl0 : (si == 1 ? cl1 : cl2);
        const int b0 = A.off[s], n = A.off[s + 1] - b0;
        double ps[3][4];
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int k = 0; k < 4; ++k) ps[q][k] = 0.0;
        for (int cb = 0; cb < n; cb += 64) {
            const int k = (cb >> 6) & 3;
            const int p = cb + lane;
            const bool valid = p < n;
            int32_t id = -1;
            double ll[3] = {0.0, 0.0, 0.0}, u = 0.0;
            if (valid) {
                double x[D];
                load_xm<D>(A, b0 + p, x);
                id = A.mem[b0 + p];
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    if (q >= Q) break;
                    __asm__ __volatile__("" ::: "memory");  // target parameters stay in LDS
                    ll[q] = ISO ? iso_ll<D>(x, &s_tg[q][0], s_tg[q][D + DP], s_tg[q][D + DP + 1])
                                : sm_ll<D>(x, &s_tg[q][0], &s_tg[q][D], s_tg[q][D + DP], s_tg[q][D + DP + 1]);
                }
                u = uniform(A.seed, (uint64_t)a, A.t, kStreamSmAlloc, (uint32_t)(rank + p));
            }
            int pq = -1;
#pragma unroll
            for (int q = 0; q < 3; ++q) pq = (q < Q && valid && id == (q == 0 ? pk0 : (q == 1 ? pk1 : pk2))) ? q : pq;
            const bool regular = valid && pq < 0;
            uint64_t m0 = 0, m1 = 0, m2 = 0;
            int d = 0;
            // log of every target size this step can see (base + 0..63), one per lane, fetched by shuffle
            const double tl0 = log_pos(Nq[0] + (double)lane), tl1 = log_pos(Nq[1] + (double)lane),
                         tl2 = (Q > 2) ? log_pos(Nq[2] + (double)lane) : 0.0;
            for (int it = 0; it <= 64; ++it) {
                const double lw0 = ll[0] + __shfl(tl0, __popcll(m0 & below)),
                             lw1 = ll[1] + __shfl(tl1, __popcll(m1 & below)),
                             lw2 = (Q > 2) ? ll[2] + __shfl(tl2, __popcll(m2 & below)) : 0.0;
                double mx = fmax(-__builtin_huge_val(), lw0);
                mx = fmax(mx, lw1);
                if (Q > 2) mx = fmax(mx, lw2);
                double tot = 0.0;
                tot += exp_le0(lw0 - mx);
                const double c0 = tot;
                tot += exp_le0(lw1 - mx);
                const double c1 = tot;
                if (Q > 2) tot += exp_le0(lw2 - mx);
                const double w = u * tot;
                d = (c0 >= w) ? 0 : ((c1 >= w || Q == 2) ? 1 : 2);
                const uint64_t n0m = __ballot(regular && d == 0), n1m = __ballot(regular && d == 1),
                               n2m = __ballot(regular && d == 2);
                if (n0m == m0 && n1m == m1 && n2m == m2) break;  // wave-uniform
                m0 = n0m;
                m1 = n1m;
                m2 = n2m;
            }
            Nq[0] += (double)__popcll(m0);
            Nq[1] += (double)__popcll(m1);
            Nq[2] += (double)__popcll(m2);
            const int dd = (pq >= 0) ? pq : d;
#pragma unroll
            for (int q = 0; q < 3; ++q)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) ps[q][kk] = (valid && dd == q && kk == k) ? ps[q][kk] + ll[q] : ps[q][kk];
            if (APPLY && valid) {
                const int ts = s_slot[dd];
                A.z[id] = (ts >= 0) ? ts : snew;
            }
        }
        // this source's canonical sums, per target
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) s_red[q][lane + 64 * kk] = ps[q][kk];
        __syncthreads();
        for (int h = 128; h >= 1; h >>= 1) {
            for (int t = lane; t < h; t += 64)
#pragma unroll
                for (int q = 0; q < 3; ++q) s_red[q][t] += s_red[q][t + h];
            __syncthreads();
        }
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (q < Q) lp[q] += s_red[q][0];
        }
        __syncthreads();
        nsrc[0] = (si == 0) ? n : nsrc[0];
        nsrc[1] = (si == 1) ? n : nsrc[1];
        nsrc[2] = (si == 2) ? n : nsrc[2];
        rank += n;
    }
    int out = 0;
    if (lane == 0) {
        double frac = 0.0;
        if (split) {
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (q < Q) frac += lgamma_int((int64_t)Nq[q]);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (i < ns) frac -= lgamma_int(nsrc[i]);
        } else {
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (i < ns) frac += lgamma_int(nsrc[i]);
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (q < Q) frac -= lgamma_int((int64_t)Nq[q]);
        }
        const double rP = split ? A.log_alpha + frac : -(A.log_alpha + frac);
        double rLd = 0.0, rLdp = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (i < ns) rLd += tri_own(A, i == 0 ? cl0 : (i == 1 ? cl1 : cl2));
#pragma unroll
        for (int q = 0; q < 3; ++q)
            if (q < Q) rLdp += lp[q];
        const double lrr = (T.kind == 0) ? A.lrr[0] : (T.kind == 1 ? A.lrr[1] : (T.kind == 2 ? A.lrr[2] : A.lrr[3]));
        const double x = ((0.0 + rP) + lrr) + (rLdp - rLd);
        const bool acc = sm_accept(x, uniform(A.seed, (uint64_t)a, A.t, kStreamSmAccept, 0));
        out = !acc ? 1 + 2 * T.kind : ((split && A.K >= A.kcap) ? 9 : 2 + 2 * T.kind);
        if (APPLY && out == 2 + 2 * T.kind) {
            if (split && snew >= 0) {
                write_new_slot(*F, vmu, snew);
                if (F->wdirty) F->wdirty[snew] = 1;
            }
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (i < ns) A.cnt[i == 0 ? cl0 : (i == 1 ? cl1 : cl2)] = 0;
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (q < Q) A.cnt[s_slot[q] >= 0 ? s_slot[q] : snew] = (int32_t)Nq[q];
        }
    }
    __syncthreads();
    return out;  // lane 0's value
}

template <int D, bool ISO>
__global__ __launch_bounds__(64) void np8_tri_walk(SmArgs A) {
    const int ns = A.sc->nsplit;
    for (int e = blockIdx.x; e < ns; e += gridDim.x) {
        const int64_t a = A.slist[e];
        unsigned long long first = 0;
        if (threadIdx.x == 0) first = *reinterpret_cast<volatile unsigned long long *>(&A.sc->first);
        first = __shfl(first, 0);
        if ((unsigned long long)a > first) continue;  // wave-uniform
        const Tri T = tri_case(A, a);
        const int out = tri_walk<D, false, ISO>(A, nullptr, T, a, A.stheta + (int64_t)e * (D + 1));
        if (threadIdx.x == 0) {
            A.typ[a - A.a0] = (uint8_t)out;
            if (out == 4 || out == 6 || out == 8)
                atomicMin(reinterpret_cast<unsigned long long *>(&A.sc->first), (unsigned long long)a);
        }
    }
}

__global__ __launch_bounds__(kSmThreads) void np8_tri_tally(SmArgs A) {
    __shared__ int cnt[10];
    if (threadIdx.x < 10) cnt[threadIdx.x] = 0;
    __syncthreads();
    const int64_t first = A.sc->first;
    const int lim = (first == INT64_MAX) ? A.nb : (int)(first - A.a0 + 1);
    int c[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int q = blockIdx.x * kSmThreads + threadIdx.x; q < lim; q += gridDim.x * kSmThreads) {
        const uint8_t t = A.typ[q];
#pragma unroll
        for (int k = 0; k < 10; ++k) c[k] += (t == k);
    }
#pragma unroll
    for (int k = 0; k < 10; ++k)
        if (c[k]) atomicAdd(&cnt[k], c[k]);
    __syncthreads();
    if (threadIdx.x < 10 && cnt[threadIdx.x])
        atomicAdd(reinterpret_cast<unsigned long long *>(&A.sc->tstats[threadIdx.x]), (unsigned long long)cnt[threadIdx.x]);
}

template <int D>
__global__ __launch_bounds__(64) void np8_tri_apply(SmArgs A, FinArgs F, int64_t a) {
    const Tri T = tri_case(A, a);
    __syncthreads();  // the apply rewrites z: every lane has read the picks' clusters first
    int out = 0;
    if (T.kind == 0) {
        out = tri_dyadic_merge_accept(A, T, a) ? 2 : 1;
        if (out == 2) {
            const int b0 = A.off[T.cl[1]], n1 = A.off[T.cl[1] + 1] - b0;
            for (int q = threadIdx.x; q < n1; q += 64) A.z[A.mem[b0 + q]] = T.cl[0];
            if (threadIdx.x == 0) {
                A.cnt[T.cl[0]] += n1;
                A.cnt[T.cl[1]] = 0;
            }
        }
    } else if (T.kind > 0) {
        __shared__ double vmu[D + 1];
        if (threadIdx.x == 0 && (T.kind & 1)) sm_theta<D>(A, a, vmu);
        __syncthreads();
        out = tri_walk<D, true>(A, &F, T, a, vmu);
    }
    if (threadIdx.x == 0) {
        if (out != 2 && out != 4 && out != 6 && out != 8) F.ctl->err |= kErrCapacity;  // cannot happen
        F.ctl->cand_fresh = 0;  // counts and slots changed behind np8_finalize: recopy the rows
    }
}

__global__ void np8_sm_reset(SmCtl *sc) {  // (both samplers)
    sc->first = INT64_MAX;
    sc->nsplit = 0;
}

}  // namespace
}  // namespace np8

using namespace np8;

#define NP8_SM_FOR_EACH_D(X) \
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

hipError_t np8_launch_sm_members(const SmArgs &A, hipStream_t s) {
    if (A.N <= 0) return hipSuccess;
    hipLaunchKernelGGL(np8_sm_hist, dim3(A.nbk), dim3(kSmThreads), sizeof(int) * A.kcap, s, A);
    hipLaunchKernelGGL(np8_sm_scan_blocks, dim3(A.kcap), dim3(kSmThreads), 0, s, A);
    hipLaunchKernelGGL(np8_sm_scan_slots, dim3(1), dim3(1024), 0, s, A);
    const dim3 gc((unsigned)A.K, (unsigned)((A.K + kCrossTile - 1) / kCrossTile));
#define X(d)                                                                                \
    if (A.D == d) {                                                                         \
        hipLaunchKernelGGL(np8_sm_scatter<d>, dim3(A.nbk), dim3(64), sizeof(int) * A.kcap, s, A); \
        if (A.K > 0) hipLaunchKernelGGL(np8_sm_cross<d>, gc, dim3(kSmThreads), 0, s, A);    \
        return hipGetLastError();                                                           \
    }
    NP8_SM_FOR_EACH_D(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_sm_eval(const SmArgs &A, hipStream_t s) {
    if (A.nb <= 0) return hipSuccess;
    hipLaunchKernelGGL(np8_sm_reset, dim3(1), dim3(1), 0, s, A.sc);
    const unsigned gs = (unsigned)std::min(A.nb, kSplitBlocks);
    const dim3 gq((unsigned)((A.nb + kSmThreads - 1) / kSmThreads));
#define X(d)                                                                   \
    if (A.D == d) {                                                            \
        hipLaunchKernelGGL(np8_sm_classify<d>, gq, dim3(kSmThreads), 0, s, A); \
        if (A.gp_iso > 0.0)                                                    \
            hipLaunchKernelGGL((np8_sm_split<d, true>), dim3(gs), dim3(64), 0, s, A); \
        else                                                                   \
            hipLaunchKernelGGL((np8_sm_split<d, false>), dim3(gs), dim3(64), 0, s, A); \
        hipLaunchKernelGGL(np8_sm_tally, dim3(256), dim3(kSmThreads), 0, s, A); \
        return hipGetLastError();                                              \
    }
    NP8_SM_FOR_EACH_D(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_sm_apply(const SmArgs &A, const FinArgs &F, int64_t a, hipStream_t s) {
#define X(d)                                                                    \
    if (A.D == d) {                                                             \
        hipLaunchKernelGGL(np8_sm_apply<d>, dim3(1), dim3(64), 0, s, A, F, a);  \
        return hipGetLastError();                                               \
    }
    NP8_SM_FOR_EACH_D(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_tri_bound(const SmArgs &A, hipStream_t s) {
    if (A.N <= 0 || A.K <= 0 || !A.mb) return hipSuccess;
    hipError_t e = hipMemsetAsync(A.mb, 0, sizeof(double) * 4 * (size_t)A.K, s);
    if (e != hipSuccess) return e;
#define X(d)                                                                                                  \
    if (A.D == d) {                                                                                           \
        hipLaunchKernelGGL(np8_tri_bound<d>, dim3((unsigned)A.K, kBoundChunks), dim3(kSmThreads), 0, s, A); \
        return hipGetLastError();                                                                             \
    }
    NP8_SM_FOR_EACH_D(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_tri_eval(const SmArgs &A, hipStream_t s) {
    if (A.nb <= 0) return hipSuccess;
    hipLaunchKernelGGL(np8_sm_reset, dim3(1), dim3(1), 0, s, A.sc);
    const unsigned gs = (unsigned)std::min(A.nb, kSplitBlocks);
    const dim3 gq((unsigned)((A.nb + kSmThreads - 1) / kSmThreads));
#define X(d)                                                                    \
    if (A.D == d) {                                                             \
        hipLaunchKernelGGL(np8_tri_classify<d>, gq, dim3(kSmThreads), 0, s, A); \
        if (A.iso_walk)                                                         \
            hipLaunchKernelGGL((np8_tri_walk<d, true>), dim3(gs), dim3(64), 0, s, A); \
        else                                                                    \
            hipLaunchKernelGGL((np8_tri_walk<d, false>), dim3(gs), dim3(64), 0, s, A); \
        hipLaunchKernelGGL(np8_tri_tally, dim3(256), dim3(kSmThreads), 0, s, A); \
        return hipGetLastError();                                               \
    }
    NP8_SM_FOR_EACH_D(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t np8_launch_tri_apply(const SmArgs &A, const FinArgs &F, int64_t a, hipStream_t s) {
#define X(d)                                                                     \
    if (A.D == d) {                                                              \
        hipLaunchKernelGGL(np8_tri_apply<d>, dim3(1), dim3(64), 0, s, A, F, a);  \
        return hipGetLastError();                                                \
    }
    NP8_SM_FOR_EACH_D(X)
#undef X
    return hipErrorInvalidValue;
}
