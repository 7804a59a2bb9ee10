// np8_kernels.h -- launch interface between the C-ABI host code (np8_capi.hip) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "np8_device.h"

namespace np8 {

// Device-resident control block (one per context).
struct Ctl {
    int32_t K;          // live clusters (rows of the dense candidate table)
    int32_t err;        // sticky error bits
    int32_t have_best;  // a max-likelihood snapshot exists
    int32_t pad;
    int64_t n_new;      // accepted new-cluster requests (cumulative)
    int64_t n_rejected; // rejected requests (cumulative)
    double L;           // last total log-likelihood (global after the exchange)
    double L_local;     // this rank's part
    double best[2];     // best L, double-buffered by check parity
    int64_t moved;      // items that changed cluster since the last re-sort (local)
    int32_t best_sorted; // z_best holds the snapshot in label-sorted position order (np8_assign_fast's lazy copy)
    int32_t do_sort;    // this re-sort pass runs (decided by np8_sort_scan)
    uint32_t done_blocks;
    uint32_t tail_done;   // np8_step_tail: workgroups finished (the last one runs the serial part, resets it)
    int64_t mh_accepted;  // accepted MH proposals (cumulative)
    uint32_t t_base;      // epoch = t_base + the launch's epoch offset (advanced on the device by
                          // replayed sweep graphs, np8_advance_epoch)
    int32_t lists_ok;     // the candidate lists describe the current table (set by the prune pass)
    int32_t n_pend;       // NIW prior: accepted requests waiting for np8_niw_aux_slots (set by np8_finalize)
    int32_t cand_fresh;   // the candidate rows' mu/P' match the slot tables (0 after a state upload:
                          // np8_finalize then copies them; parameter updates patch rows in place)
    unsigned long long n_screen_viol;  // count_eval runs: lanes with a screened auxiliary that pick_step would
                                       // not have skipped (the auxiliary screen's self-check; must stay 0)
    unsigned long long n_aux_exact[2]; // count_eval runs: (lane, auxiliary) pairs the screen did not skip,
                                       // and (wave, auxiliary) pairs in which at least one lane was not skipped
    uint32_t qwaves;                   // np8_assign_fast waves with deferred lanes this step (AssignArgs::qlist)
    uint32_t pad3;
    uint32_t fin_flag;    // np8_fin_prune: finalize done (set by workgroup 0, reset by the last list workgroup)
    uint32_t prune_exit;  // np8_fin_prune: list workgroups finished
    // folded max-likelihood check (DESIGN.md "Max likelihood"): the check sweep's finalize found an improvement;
    // the next np8_assign_fast copies the labelling into the snapshot buffers (or np8_snapshot_flush does)
    int32_t snap_pend;
    uint32_t list_builds;  // candidate-list builds by the conditional step tail (diagnostics)
    // compact exchange: a rank's requests of a step did not fit its compact record, which np8_finalize
    // finds in the gathered headers alike on every rank: it sets halt (and the step's epoch offset) and applies
    // nothing; every kernel of a sweep graph then does nothing until the host has run that step's exchange with the
    // full records and cleared it
    int32_t halt;
    uint32_t halt_t;
    int32_t req_peak;  // the largest request count of one rank in one step since the last replay's end (all ranks alike)
    int32_t pad4;
    // wide path, folded max-likelihood check (FinArgs::ll_defer): the assign's exact sum as finalize left it, completed
    // by np8_ll_fix_wide with the accepted requesters' log-likelihoods under their new slots
    uint64_t L_fx_lo;  // (an Fx, np8::fx_add's two's complement halves)
    int64_t L_fx_hi;
};

// Host-mapped mirror the last finalize of a replayed sweep graph writes (np8_sweep reads it once the replay is done):
// [0] halt, [1] the halted step's epoch offset, [2] req_peak over the replay's steps
constexpr int kMirrorInts = 4;

// Candidate lists are built with kListSlack nats of extra margin, so a list stays exact while no live slot's
// log n or log(n - 1) moves by more than kListSlack / 2 from its value at the build (np8_step_tail's
// conditional rebuild, DESIGN.md "Candidate pruning").
constexpr double kListSlack = 2.0;

// Exact sums of log-likelihoods (the folded max-likelihood check): x * 2^64 as a 128-bit two's-complement integer
// (lo, hi), exact for every double with 2^-11 <= |x| < 2^62 (below, truncated toward zero).  Integer addition is
// associative, so the sum is the same in any order -- whatever the label-sorted layout put into which wave, however
// many ranks the items are spread over.
struct Fx {
    uint64_t lo;
    int64_t hi;
};

NP8_HD Fx fx_add(Fx a, Fx b) {
    Fx r;
    r.lo = a.lo + b.lo;
    r.hi = (int64_t)((uint64_t)a.hi + (uint64_t)b.hi + (r.lo < a.lo ? 1ull : 0ull));
    return r;
}

NP8_HD Fx fx_neg(Fx a) {
    Fx r;
    r.lo = ~a.lo + 1ull;
    r.hi = (int64_t)(~(uint64_t)a.hi + (r.lo == 0ull ? 1ull : 0ull));
    return r;
}

NP8_HD Fx fx_of(double x) {
    union {
        double d;
        uint64_t u;
    } v;
    v.d = x;
    const int ex = (int)((v.u >> 52) & 0x7FF);
    Fx r;
    r.lo = 0ull;
    r.hi = 0;
    if (ex == 0 || ex == 0x7FF) return r;  // zero, subnormal (never an item's ll), inf / nan (never)
    const uint64_t m = (v.u & 0xFFFFFFFFFFFFFull) | 0x10000000000000ull;
    int sh = ex - 1075 + 64;  // x * 2^64 = m * 2^sh
    if (sh > 74) sh = 74;     // |x| >= 2^63: saturates (never an item's ll)
    if (sh >= 64) {
        r.hi = (int64_t)(m << (sh - 64));
    } else if (sh > 0) {
        r.lo = m << sh;
        r.hi = (int64_t)(m >> (64 - sh));
    } else if (sh == 0) {
        r.lo = m;
    } else if (sh > -64) {
        r.lo = m >> (-sh);
    }
    return (v.u >> 63) ? fx_neg(r) : r;
}

// The sum as a double: hi exactly (|hi| < 2^53), lo rounded, one fma -- a fixed function of the integer.
NP8_HD double fx_to_double(Fx a) { return fma((double)a.hi, 0x1.0p64, (double)a.lo) * 0x1.0p-64; }

// Executed work of np8_assign when AssignArgs::count_eval is set (timing mode): per wave, the cluster
// quadratic forms its items evaluated (own rows included) and how many took the isotropic form, added
// to counter pair (wave id mod kEvalSlots); regions 1-3 of evalc: exact auxiliaries (lanes, waves), full-table
// walks (lanes, waves), many-row waves and list entries walked -- spread over many addresses: one counter pair for every wave
// of the grid serialises the atomics in one L2 channel (4x the kernel time at C3).
constexpr int kEvalSlots = 1024;

enum : int32_t { kErrCapacity = 1, kErrSigma = 2, kErrInvariant = 4, kErrQueue = 8, kErrSpin = 16 };

// Exchange record of one rank for one synchronous step:
//   RecHeader | int32 delta[kcap] | Request req[rec_cap] | double vmu[rec_cap][D+1]
// vmu[q] = (v, mu) of the auxiliary request q asks to become a cluster (computed by the rank that
// owns the item: mu needs the item's data, DESIGN.md "G0").  One rank: rec_cap >= the items of a
// step, the assign kernel appends every request in arrival order.  Several ranks: the assign kernel
// appends to a staging record of the same layout and np8_req_select copies this rank's req_max
// requests of lowest scan position into the exchanged record (ascending), which is all np8_finalize
// can accept from it (DESIGN.md "Finalize").
struct RecHeader {
    int32_t nreq;
    int32_t nreq_all;  // the rank's requests before np8_req_select kept its req_max lowest (0: none were dropped, the
                       // one-rank record); the rejected-request count is the same on any number of ranks
    int32_t pad[2];
    Fx L_local;  // folded max-likelihood check: this rank's exact sum of log-likelihoods (np8_req_select)
};
constexpr int kRecHeaderBytes = 32;

struct Request {
    int64_t pos;   // global scan position (orders requests across ranks)
    int64_t i;     // item key: global item index | visit << 32 (the Philox key of the auxiliary draw)
    int32_t m;     // which auxiliary
    int32_t zold;  // slot the item leaves
    int32_t lpos;  // position in the owner's label-sorted layout (-1: none)
    int32_t pad;
    Fx dll;        // folded max-likelihood check: ll under the new slot - ll under zold, exact (added if accepted)
};

// Item keys (DESIGN.md "Randomness"): the Philox item counter of every per-item draw is
// global index | visit << 32, visit = how often the item was already updated in this epoch (0 in every
// sweep; repeated np8_update_points calls within one epoch carry it in the high word of the order entry).
NP8_HD int64_t key_item(int64_t key) { return (int64_t)((uint64_t)key & 0xFFFFFFFFull); }

NP8_HD int64_t record_vmu_offset(int kcap, int rec_cap) {
    return (kRecHeaderBytes + 4ll * kcap + (int64_t)sizeof(Request) * rec_cap + 15) & ~15ll;
}

NP8_HD int64_t record_bytes(int kcap, int rec_cap, int D) {
    int64_t b = record_vmu_offset(kcap, rec_cap) + 8ll * (D + 1) * rec_cap;
    return (b + 15) & ~15ll;
}

// Radius record of one assign wave (candidate pruning): the largest |x - mu|^2 over its 64 items and the
// slot they all sit in, or slot -1 when they do not share one (those items went to r2 by atomics).
// Plain stores instead of one device-scope atomic per wave on a handful of addresses: those serialise
// at the memory side and cost the sweep ~50 us at C3.  Written only on gathering sweeps.
struct WaveR2 {
    double d2;
    int32_t slot, pad;
};

struct AssignArgs {
    const double *X;   // [D][n_loc] (structure of arrays), item order
    int32_t *z;        // [n_loc] slot ids, item order
    int32_t sorted;    // run on the label-sorted layout (buffer 0 of Xs/zs/ids)
    const double *Xs[2];
    int32_t *zs[2];
    const int32_t *ids[2];  // position -> local item index
    const double *cand;
    const int32_t *dense_of;  // slot -> row of the candidate table
    Ctl *ctl;
    const double *hyp; // mu0 | UinvT packed | caux | rsk | logam | nu
    const int64_t *order;  // explicit scan order: local item | visit << 32
    unsigned char *rec;    // this rank's record (header, delta)
    // where new-cluster requests are appended: the record itself (one rank) or the staging record
    int32_t *nreq;
    Request *req;
    double *vmu;
    int64_t n_loc, offset;
    int64_t p0, p1;
    int32_t use_perm;
    Perm perm;
    uint64_t seed;
    uint32_t t;  // epoch offset: epoch = ctl->t_base + t
    int32_t kcap, req_cap;  // req_cap: entries of the request area (>= the items of the step)
    // candidate pruning (DESIGN.md "Pruning"): a wave whose items all sit in dense row k0 walks
    // plist[k0*ls .. +plen[k0]] instead of every row; r2 collects max |x - mu|^2 per slot for the
    // lists of the next sweep
    const int32_t *plist, *plen;
    const float *pdist;  // beside plist: |mu_j - mu_k0| of each listed row, rounded down (0: not measured)
    const double *plr2;  // per dense row: the squared radius its list assumes (+inf: a full list)
    int32_t ls, use_lists, collect_r2, count_eval;
    int32_t walk_screen;  // np8_assign_fast: screen each listed row for the wave before its quadratic forms
    int32_t max_groups;   // own rows per wave up to which the lanes walk their lists group by group (else the table)
    double *r2;      // [2][kcap]: radii in use | gathered this sweep (collect_r2: mixed waves atomicMax here)
    WaveR2 *wr2;     // [ceil(n_loc / 64)]: a wave whose 64 items sit in one slot stores its maximum here
    unsigned long long *evalc;  // [kEvalSlots][2]: quadratic forms, isotropic ones
    // wide path (np8_wide.hip): per slot, the used MFMA fragment chunks of the fp32 factor followed by
    // the fp32 mean in fragment order (Wide<D>::ROW floats)
    const float *wfrag;
    const float *wmu;          // natural fp32 means [kcap][D]
    const double *lam_lo;      // [kcap] precision eigenvalue lower bounds (np8_wide_rows)
    int32_t dim = 0;           // wide path: the data's D (the kernels are instantiated for DT = D rounded up to 16; the
                               // item rows, factors and means beyond D are zero)
    const double *uw = nullptr;  // wide path: mu0 [DT] | U^T packed [DT (DT + 1) / 2], zero beyond D (the item frame)
    int32_t screen16 = 0;        // wide path: the exact-distance screen's dot products in fp16 (every |x|^2 <= kScreen16X2)
    int32_t pad_s16 = 0;
    const double *wdist;       // [K][kcap] distances between row means (np8_wide_dist); null: no pruning
    // two-kernel step (np8_assign_fast + np8_assign): positions the fast kernel deferred; non-null makes
    // np8_assign run over them instead of [p0, p1)
    // (one wave per workgroup: fast-kernel wave w writes its deferred positions to queue[64 w ..] and their
    // number to qcount[w]; queue mode runs block w over them)
    int32_t *queue;
    int32_t *queue_out;        // np8_assign_fast: where deferred positions go
    int32_t *qcount;           // [waves of the step]
    int32_t *qlist;            // waves with deferred lanes (ctl->qwaves of them, cleared by np8_finalize)
    // np8_assign_fast: the own row by slot, in one round of loads (no slot -> dense row -> row chain)
    const double *slot_mu, *slot_c, *slot_iso, *slot_logn1;
    const int32_t *plen_s;     // plen of the slot's dense row (np8_prune)
    const double *plr2_s;      // plr2 of the slot's dense row
    // np8_assign_fast: the host launches no np8_assign_queue after it (every live row isotropic, so no lane is
    // deferred; a deferred lane would set kErrQueue)
    int32_t no_queue, pad_nq;
    // compact exchange (a sharded sweep graph's steps): the kernel does nothing once ctl->halt is set, and
    // each request it appends to the staging area (nreq, req, vmu) is also copied into the compact record's first
    // ccap entries (creq, cvmu) -- the record whose header holds the count (nreq) and whose deltas are at rec
    int32_t compact = 0, ccap = 0;
    Request *creq = nullptr;
    double *cvmu = nullptr;
    // np8_assign_fast, folded max-likelihood check (frozen parameters): ll_on = this sweep is a check sweep: each
    // wave stores the sum of its items' log-likelihoods under their new label in llpart[wave] (a requester counts
    // under its old slot; its Request carries the difference); snap_on = a snapshot may be pending
    // (ctl->snap_pend): copy the labelling as it stands before this sweep into the snapshot buffers
    Fx *llpart = nullptr;
    int32_t ll_on = 0, snap_on = 0;
    double gp0 = 0.0;  // Gp[0]: a new slot's isotropic precision is gp0 / v^2 (np8_finalize's write_new_slot)
    int32_t *z_best = nullptr, *cnt_best = nullptr;
    double *mu_best = nullptr, *sigma_best = nullptr;
    const int32_t *cnt = nullptr;
    const double *slot_sigma = nullptr;
    int32_t naux = 0, pad_rt = 0;  // np8_assign_rt (np8_rt.hip): M at run time (D in dim)
};

// Wide-path tables (np8_wide.hip), maintained for the slots flagged in dirty.
struct WideArgs {
    int32_t D, kcap;
    int32_t DT;  // D rounded up to a multiple of 16: the layout of wA [kcap][DT][DT], wfrag, wmu [kcap][DT] and the items
    int32_t *dirty;
    const int32_t *cnt;
    const double *slot_P, *slot_mu;
    float *wA, *wfrag, *wmu;  // wA natural [D][D]; wfrag as AssignArgs::wfrag; wmu natural [D]
    double *lam_lo;           // [kcap]: a lower bound of the smallest eigenvalue of the slot's precision
    Ctl *ctl;
    // candidate pruning (np8_wide_dist): squared distances between the fp32 means of dense rows [K][kcap]
    const double *cand;
    double *wdist;
};

// Builds the candidate lists of every live dense row from the radii r2 collected by the sweep
// (then clears r2 for the next one).  One block per row.
struct PruneArgs {
    const double *cand;
    Ctl *ctl;
    double *r2;         // [2][kcap]: radii in use | gathered this sweep
    int32_t *plist, *plen;
    float *pdist;       // beside plist: |mu_j - mu_k0| rounded down (AssignArgs::pdist)
    double *plr2;       // per dense row: the squared radius the list was built for
    int32_t *plen_s;    // plen and plr2 again, indexed by the row's slot (np8_assign_fast)
    double *plr2_s;
    int32_t ls, D, kcap;
    int32_t gathered;   // the sweep's last step of a gathering sweep: lists from the gathered radii, which
                        // then become the radii in use
    int32_t clear_next; // (not gathered) zero the gathered buffer for the next sweep, which gathers
    double *lb = nullptr;  // [2][kcap]: log n | log(n - 1) of each listed row's slot at the build (kListSlack test)
    // [2][kcap] bounds lo <= eig(P) <= hi of each slot's precision (FinArgs::slot_lam), or null: a row that is not
    // isotropic is then never left out of a list (and a non-isotropic own row lists every row)
    const double *lam = nullptr;
};

struct FinArgs {
    const unsigned char *recs;  // world records, rec_bytes apart
    unsigned char *local_rec;   // cleared after use
    int64_t rec_bytes;
    int32_t world, rec_cap, kcap, D, M;
    int32_t *cnt;
    int32_t *z;
    int32_t *zs[2];  // sorted-layout labels (buffer 0 is the layout), null when not in use
    int64_t n_loc, offset;
    double *slot_mu, *slot_P, *slot_c, *slot_sigma, *slot_iso;
    double *slot_logn1;  // log(n - 1) of each live slot (the own-row weight), as its dense row holds it
    double *cand;
    int32_t *dense_of;
    Ctl *ctl;
    const double *mu0, *LT, *Gp, *LTL;  // LT, LTL: D*D row-major; Gp packed
    double caux, rsk, nu;
    double gp_iso;  // common diagonal of Gp when (L^T L)^{-1} is a multiple of I, else 0
    uint64_t seed;
    uint32_t t;  // epoch offset: epoch = ctl->t_base + t
    double *r2;  // pruning radii [2][kcap]: +inf for every slot created here (unknown radius)
    // precision eigenvalue bounds [2][kcap] (lo | hi) of every slot, for the candidate lists of rows that are not
    // isotropic (PruneArgs::lam); a slot created here gets those of Gp / v^2.  Null: not kept.
    double *slot_lam = nullptr;
    double gp_lamlo = 0.0, gp_lamhi = 0.0;
    // NIW prior: accepted requests are listed in pend[4 q] = (byte offset of the request's record
    // payload in recs, item, m, slot) for np8_niw_aux_slots instead of being written here
    int32_t prior, req_max;  // req_max: new clusters one step may create
    int64_t *pend;
    // wide path: request payloads are the item frame (|y0|, y0); slots created here are flagged for
    // the table refresh
    int32_t frame_payload, pad3;
    const double *hyp;
    int32_t *wdirty;
    // folded max-likelihood check (AssignArgs::ll_on): L = sum of the per-wave partials (one rank, ll_rec = 0) or of
    // the records' L_local (rank order, ll_rec = 1), plus the accepted requests' dll; snapshot decision on best[par]
    const Fx *llpart = nullptr;
    int64_t ll_n = 0;
    int32_t ll_on = 0, ll_rec = 0;
    int32_t snap_clear = 0, par = 0;  // snap_clear: the step's assign consumed ctl->snap_pend
    double *best = nullptr;
    int32_t *have_best = nullptr;
    // conditional candidate lists (np8_step_tail, TailArgs::prune == 2): the lists of the last build stay exact while
    // every live slot's log n and log(n - 1) are within kListSlack / 2 of lb (PruneArgs::lb) and no slot changed
    const double *lb = nullptr;
    int32_t slack_test = 0;
    uint32_t advance = 0;               // ctl->t_base += advance at the end (a captured graph's last step)
    int64_t *moved_mirror = nullptr;    // host-mapped copy of ctl->moved (the host's re-sort decision), or null
    // compact exchange: the records are compact (rec_cap of them per rank): a rank with more requests halts the graph
    int32_t compact = 0;
    int32_t peak_out = 0;               // (a replay's last step) mirror req_peak and start it anew
    // wide path, folded check: the sum goes to ctl->L_fx and the decision to np8_ll_fix_wide (the new slots' rows exist
    // only after np8_frame_slots / np8_niw_aux_slots and np8_wide_rows); pend_ll[2 q] = the accepted requester's old
    // slot and position in the label-sorted layout
    int32_t ll_defer = 0, pad6 = 0;
    int64_t *pend_ll = nullptr;
    int32_t *mirror = nullptr;          // host-mapped [kMirrorInts]: halt as it happens, req_peak with peak_out
};

// A field of a kernel's argument struct (the kernel's only explicit argument: offset 0 of the kernarg segment) read
// where it is used: a scalar load behind an empty asm barrier on the segment pointer, so that the compiler neither loads
// it in the entry block nor holds it (spilled to VGPR lanes: a v_writelane / v_readlane pair each) across the kernel.
template <class T>
__device__ __forceinline__ T np8_late_arg(size_t off) {
    typedef const __attribute__((address_space(4))) char *KP;
    KP kp = (KP)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *(const __attribute__((address_space(4))) T *)(kp + off);
}

// Wave-aggregated atomics on a few hot addresses (count deltas, gathered radii): one atomic per distinct key
// among the wave's `on` lanes instead of one per lane.  Same-address device-scope atomics serialise at the
// memory side across the XCDs; in the regime the reference's start reaches (duplicate clusters, ~30% of the
// items moving per sweep) per-lane atomics on ~140 counters cost the assign kernel more than its arithmetic.
// Every active lane of the wave must call (ballots over the active lanes).
__device__ __forceinline__ void wave_add_by_key(int32_t *base, int32_t key, int32_t v, bool on) {
    const int lane = threadIdx.x & 63;
    uint64_t pend = __ballot(on);
    while (pend) {
        const int l = __ffsll((unsigned long long)pend) - 1;
        const int32_t k = __builtin_amdgcn_readlane(key, l);
        const uint64_t m = __ballot(on && key == k);
        if (lane == l) atomicAdd(base + k, v * (int32_t)__popcll(m));
        pend &= ~m;
    }
}

// A slot of a shared append area for each lane with `on` (one atomicAdd per wave); -1 for the others.
__device__ __forceinline__ int wave_append(int32_t *count, bool on) {
    const int lane = threadIdx.x & 63;
    const uint64_t m = __ballot(on);
    if (m == 0ull) return -1;
    const int l = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == l) base = atomicAdd(count, (int32_t)__popcll(m));
    base = __shfl(base, l);
    return on ? base + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// max of non-negative doubles (as their bit patterns) per distinct key, one atomicMax per key
__device__ __forceinline__ void wave_max_by_key(unsigned long long *base, int32_t key, double v, bool on) {
    const int lane = threadIdx.x & 63;
    uint64_t pend = __ballot(on);
    while (pend) {
        const int l = __ffsll((unsigned long long)pend) - 1;
        const int32_t k = __builtin_amdgcn_readlane(key, l);
        const bool in = on && key == k;
        const uint64_t m = __ballot(in);
        double r = in ? v : 0.0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r = fmax(r, __shfl_xor(r, o));
        if (lane == l) atomicMax(base + k, (unsigned long long)__double_as_longlong(r));
        pend &= ~m;
    }
}

// Auxiliary draw m of (item i, epoch t) -> a slot: the G0 draw of normalinvwishart.h:44-64 in the
// factored form (DESIGN.md "G0").
// Pruning radii (DESIGN.md "Candidate pruning") live in two buffers of kcap, by sweep parity: a slot whose
// parameters are new is unprunable (+inf) in both until a whole sweep has measured it.
__device__ __forceinline__ void r2_unknown(double *r2, int kcap, int s) {
    if (!r2) return;
    r2[s] = __longlong_as_double(0x7FF0000000000000ll);
    r2[kcap + s] = __longlong_as_double(0x7FF0000000000000ll);
}

// Slot s from an accepted request's (v, mu): element f of new_slot_elems(D) = D means, DP precision entries, D^2
// covariance entries and the scalars -- one thread per element (np8_finalize spreads a step's new slots over its
// workgroup: one thread writing all of a slot waited on ~100 dependent loads of Gp / LTL, 40k cycles a step), or all of
// them in order (write_new_slot).
__device__ __forceinline__ int new_slot_elems(int D) { return D + D * (D + 1) / 2 + D * D + 1; }

__device__ __forceinline__ void write_new_slot_elem(const FinArgs &F, const double *vmu, int s, int f) {
    const int D = F.D, DP = D * (D + 1) / 2;
    const double v = vmu[0], v2 = v * v;
    if (f < D) {
        F.slot_mu[(int64_t)s * D + f] = vmu[1 + f];
    } else if (f < D + DP) {
        const int k = f - D;
        F.slot_P[(int64_t)s * DP + k] = F.Gp[k] / v2;
    } else if (f < D + DP + D * D) {
        const int k = f - D - DP;
        F.slot_sigma[(int64_t)s * D * D + k] = v2 * F.LTL[k];
    } else {
        F.slot_c[s] = fma(-(double)D, log_pos(fabs(v)), F.caux);
        F.slot_iso[s] = (F.gp_iso > 0.0) ? F.Gp[0] / v2 : 0.0;
        r2_unknown(F.r2, F.kcap, s);  // radius unknown until a sweep measures it
        if (F.slot_lam) {  // P = Gp / v^2: its eigenvalues are Gp's over v^2 (the bounds carry a 1e-9 relative margin)
            F.slot_lam[s] = F.gp_lamlo / v2;
            F.slot_lam[F.kcap + s] = F.gp_lamhi / v2;
        }
    }
}

__device__ __forceinline__ void write_new_slot(const FinArgs &F, const double *vmu, int s) {
    const int ne = new_slot_elems(F.D);
    for (int f = 0; f < ne; ++f) write_new_slot_elem(F, vmu, s, f);
}

// Jain-Neal split-merge (np8_sm.hip, DESIGN.md "Split-merge").
// keys of the two scan permutations: make_perm(seed ^ kSmPermKey[r], epoch, N)
constexpr uint64_t kSmPermKey[2] = {0x4A4E53504C495430ull, 0x4A4E53504C495431ull};
// ... and the triadic sampler's three: make_perm(seed ^ kTriPermKey[r], epoch, N)
constexpr uint64_t kTriPermKey[3] = {0x5452494144494330ull, 0x5452494144494331ull, 0x5452494144494332ull};

constexpr int kSmMemItems = 512;  // items per block of the member-list counting sort (np8_sm_hist/scatter)

struct SmCtl {
    int64_t first;     // lowest accepted attempt of the batch (INT64_MAX: none)
    int64_t stats[6];  // outcomes: skipped, split rej, merge rej, split acc, merge acc, split at kcap
    int64_t tstats[10];  // triadic outcomes (np8_tri_stats order)
    int32_t nsplit;    // splits queued by np8_sm_classify
    int32_t all_iso;   // every live slot has an isotropic P' (set by the member-list build)
};

struct SmArgs {
    int32_t D, kcap;
    int32_t N, K;      // local items; live slots (host copy of ctl->K after the last table rebuild)
    const double *X;   // [D][N] (structure of arrays)
    int32_t *z, *cnt;
    const double *slot_mu, *slot_P, *slot_c, *slot_iso;
    const double *LT, *Gp, *mu0;  // LT: D*D row-major; Gp packed
    double gp_iso;                // diagonal of Gp when it is a multiple of I, else 0
    double caux, rsk, nu, log_alpha;
    uint64_t seed;
    uint32_t t, pad;
    Perm perm0, perm1;  // the two scan permutations of the sweep (np_mcmc.cpp:118-125)
    Perm tperm[3];      // triadic: three permutations
    double lrr[4];      // triadic rR for dyadic merge, dyadic split, triadic merge, triadic split
    int32_t *hist;      // [kcap][nbk] block histograms -> scatter bases
    int32_t nbk, pad2;
    int32_t *mem;       // [N] members of every slot, ascending item order
    int32_t *off;       // [kcap + 1]
    const int32_t *dense;  // slot -> live rank (np8_finalize's dense_of)
    int32_t *live;      // [kcap] live rank -> slot
    double *Xm;         // [D][N] items in member order
    double *ownm;       // [N] ll of member p under its own slot
    int64_t *slist;     // [batch] queued split attempts
    double *stheta;     // [batch][D + 1] their new clusters' (v, mu)
    double *cross;      // [K][K] canon_sum over row r's members of ll under live slot k
    SmCtl *sc;
    uint8_t *typ;       // [batch] attempt outcomes
    int64_t a0;
    int32_t nb;
    int32_t iso_walk;   // triadic: every target isotropic (all live slots and G0), the walk's fast form
    double *mb;         // triadic: [K][4] per live row, the merge bound's member sums (np8_tri_bound); null: off
};

// NIW prior kernels (np8_niw.hip): posterior / prior draws per slot and picked auxiliaries -> slots.
struct NiwArgs {
    int32_t D, kcap;
    double kappa0, nu0, rsk, caux;  // rsk = 1/sqrt(kappa0); caux = -D/2 log 2pi + sum log U_aa
    const double *mu0, *Psi0;       // Psi0: D x D row-major
    const double *U, *Uinv;         // U = chol(Psi0^{-1}) (lower) and its inverse, D x D row-major
    uint64_t seed;
    uint32_t t;  // epoch offset: epoch = ctl->t_base + t
    int32_t write_cand;  // also patch the candidate rows (dense_of valid)
    Ctl *ctl;
    const int32_t *cnt, *dense_of;
    double *acc;  // [kcap][D + DP] statistics (np8_suffstats), zeroed after use
    double *slot_mu, *slot_P, *slot_c, *slot_sigma, *slot_iso;
    double *cand;
    double *r2;
    int32_t init_k, pad;             // > 0: draw G0 sample b into slot init_map[b] (b < init_k)
    const int32_t *init_map;
    const unsigned char *recs;  // np8_niw_aux_slots: the records np8_finalize read
    const int64_t *pend;
    // np8_niw_post: the run records of np8_suffstats_wide (ParamArgs::part), n_rec headers; null: acc only
    const double *part = nullptr;
    const int32_t *part_slot = nullptr;
    int64_t n_rec = 0;
    // np8_niw_post on the wide path (else null): the drawn slot's contraction rows from the draw's own factor R
    // (WideArgs::wA / wfrag / wmu) and its precision eigenvalue bound (WideArgs::lam_lo)
    float *wA = nullptr, *wfrag = nullptr, *wmu = nullptr;
    double *lam_lo = nullptr;
    int32_t DT = 0;  // wide path: the tables' tile dimension (WideArgs::DT)
    int32_t valu = 0;  // np8_niw_post: the dense products on the vector ALU instead of the fp64 matrix cores (NP8_NIW_VALU=1)
};

// np8_step_tail (the end of a synchronous step in one launch): which parts run.
struct TailArgs {
    int32_t queue;   // (unused: np8_assign_fast's deferred lanes keep np8_assign_queue -- measured slower here)
    int32_t fold;    // the step's radius records (AssignArgs::wr2, fold_n of them) into the gathered radii
    int32_t select;  // np8_req_select: staging record -> exchanged record (sharded step; no finalize then)
    int32_t fin;     // np8_finalize (FinArgs)
    int32_t prune;   // np8_prune after it (PruneArgs; the frozen reference-prior sweep): 1 always, 2 only when
                     // finalize finds the last lists stale (FinArgs::slack_test)
    int32_t pad;
    int64_t fold_n;
    int64_t lds_bytes;  // dynamic LDS of the launch (np8_finalize_lds_bytes; prune_block stages rows in it)
    const unsigned char *stage;  // select: staging record, its request capacity, the exchanged record
    int64_t stage_cap;
    unsigned char *rec;
    int64_t rec_cap;
};

struct LoglikArgs {
    const double *X;
    const int32_t *z;
    const double *cand;
    const int32_t *dense_of;
    double *partial;
    int64_t n_loc;
};

// Cluster-parameter update (mh_g0): per-slot statistics of the current labelling about the slot's
// mean, then the MH chain of every live slot (DESIGN.md "Parameter update").
struct ParamArgs {
    const double *X;  // item-order layout [D][n_loc]
    const int32_t *z;
    const double *Xs[2];  // label-sorted layout (buffer 0) when sorted != 0
    const int32_t *zs[2];
    int32_t sorted;
    int64_t n_loc;
    int32_t kcap, D, steps;
    int32_t DT = 0;  // wide path: the items' row count (D rounded up to 16; rows >= D zero)
    double *acc;  // [kcap][D + DP]: sum d | packed sum d d^T, d = x - mu_slot
    const int32_t *cnt;
    const int32_t *dense_of;
    double *slot_mu, *slot_P, *slot_c, *slot_sigma, *slot_iso;
    double *cand;
    Ctl *ctl;
    const double *mu0, *LT, *Gp, *LTL;  // as FinArgs
    double caux, rsk, nu, gp_iso;
    uint64_t seed;
    uint32_t t;  // epoch offset: epoch = ctl->t_base + t
    double *r2;  // pruning radii: +inf for every slot whose parameters change
    // wide path, one rank (np8_suffstats_wide): each wave stores the sums of its first kSuffRuns slot runs as run
    // records (raw MFMA accumulator layout, no atomics; np8_niw_post reduces a slot's records in record order) and
    // only further runs (an unsorted layout) go to acc by atomics.  Null: every run to acc (ranks sum acc).
    double *part = nullptr;
    int32_t *part_slot = nullptr;  // [waves * kSuffRuns]: the run's slot, -1 unused
};

// Own rows per wave up to which np8_assign(_fast)'s lanes walk their rows' lists group by group (default of
// AssignArgs::max_groups; NP8_MAX_LIST_GROUPS overrides it).
constexpr int kMaxListGroups = 3;
// the wide path's fp16 exact-distance screen: for data with every |x|^2 at most this (its margin, 2e-3 (|x|^2 + |muf|^2),
// stays small against the distances between clusters; larger data keep the fp32 screen, margin 1e-5 (...))
constexpr double kScreen16X2 = 4096.0;
// the wide path's item rows carry, after the DT fp32 rows, the item's frame (|U^T (x - mu0)|, |x|^2) as two doubles in
// four 32-bit rows (low, high word each): computed once per data set (np8_wide_frame) and moved with the item by the
// layout's sort, so the assign reads it coalesced at the item's position
constexpr int kFrameRows = 4;
constexpr int kSuffRuns = 4;  // run records per wave of np8_suffstats_wide

struct SnapArgs {
    Ctl *ctl;  // best_sorted: cleared by the item-order copies
    const double *L;
    double *best;
    int32_t *have_best;
    int32_t par;
    const int32_t *z, *cnt;
    int32_t *z_best, *cnt_best;
    const double *slot_mu, *slot_sigma;
    double *mu_best, *sigma_best;
    int64_t n_loc;
    int32_t kcap, D;
};

}  // namespace np8

// Label-sorted layout (items grouped by cluster so that a wave shares its candidate set).
// force: rebuild from the item-order arrays (X, z); otherwise re-sort buffer 0 when more than n/32 items moved
// since the last sort.  The scatter writes buffer 1, np8_sort_copyback copies it back: the layout is always
// buffer 0.
struct SortArgs {
    const double *X;  // item-order layout [D][n]
    const int32_t *z;
    double *Xs[2];
    int32_t *zs[2], *ids[2];
    int32_t *hist, *cursor, *off;  // [kcap] scratch; hist is kept zero between passes
    np8::Ctl *ctl;
    int64_t n;
    int32_t kcap, D, force;
    int32_t esz;  // bytes per element of X: 8 (fp64) or 4 (wide path, fp32)
    // data-parallel sub-steps: the layout is sorted by (sub-step of the item, slot), nsub * kcap bins
    int32_t nsub, pad;
    int64_t offset;  // global index of local item 0
    uint64_t seed;
};

bool np8_supported(int D, int M);
bool np8_wide_supported(int D, int M);
hipError_t np8_launch_assign_wide(const np8::AssignArgs &A, int D, int M, int prior, hipStream_t s);
// the wide path's per-item frame over the fp32 items X [DT][n] and uw (AssignArgs::uw), into X's kFrameRows rows
hipError_t np8_launch_wide_frame(float *X, int64_t n, const double *uw, int DT, hipStream_t s);
// Wide-path pruning: the distance table of the current dense rows (after every table change).
hipError_t np8_launch_wide_dist(const np8::WideArgs &W, hipStream_t s);
hipError_t np8_launch_loglik_matrix_wide(const np8::AssignArgs &A, const np8::WideArgs &W, int D, int M, int prior,
                                         const int64_t *idx, int64_t n, double *out, hipStream_t s);
hipError_t np8_launch_loglik_wide(const np8::LoglikArgs &L, const np8::WideArgs &W, int D, hipStream_t s);
hipError_t np8_launch_loglik_wide_mfma(const np8::AssignArgs &A, int D, double *partial, hipStream_t s);
// Folded check on the wide path: L = ctl->L_fx + the accepted requesters' ll under the new slot - under the old one
// (the VALU form of the contraction, bit-identical to the MFMA), then the snapshot decision (best[par], snap_pend).
hipError_t np8_launch_ll_fix_wide(const np8::WideArgs &W, const float *Xs, int64_t n, const double *cand,
                                  const int32_t *dense_of, const double *slot_c, const int64_t *pend, const int64_t *pend_ll,
                                  double *best, int32_t *have_best, int par, np8::Ctl *ctl, hipStream_t s);
hipError_t np8_launch_wide_refresh(const np8::WideArgs &W, hipStream_t s);
size_t np8_niw_lds_bytes(int D);
hipError_t np8_niw_prepare(int D);
hipError_t np8_launch_niw_post(const np8::NiwArgs &A, int nblocks, hipStream_t s);
hipError_t np8_launch_niw_aux_slots(const np8::NiwArgs &A, hipStream_t s);
hipError_t np8_launch_resort(const SortArgs &S, hipStream_t s);
hipError_t np8_launch_assign(const np8::AssignArgs &A, int D, int M, int prior, hipStream_t s);
// np8_assign_fast (reference prior, isotropic Lambda, label-sorted layout): defers lanes into A.queue_out / ctl->qn
hipError_t np8_launch_assign_fast(const np8::AssignArgs &A, int D, int M, hipStream_t s);
// wide path, reference prior: the slots np8_finalize accepted (ctl->n_pend, F.pend)
hipError_t np8_launch_frame_slots(const np8::FinArgs &F, hipStream_t s);
// np8_assign_queue: the lanes np8_assign_fast deferred (A.queue, A.qcount, A.qlist, ctl->qwaves)
hipError_t np8_launch_assign_queue(const np8::AssignArgs &A, int D, int M, hipStream_t s);
// Pruning radii: the step's per-wave records (AssignArgs::wr2) into the gathered radii (r2 + kcap).
hipError_t np8_launch_fold_r2(const np8::WaveR2 *wr2, int64_t n, double *r2, int kcap, const np8::Ctl *ctl,
                              hipStream_t s);
// Debug invariants (np8_config / NP8_DEBUG_INVARIANTS): every label a live slot, the live slots' counts the
// label histogram (one rank) and summing to n_global, K the live slots, the dense table live slots only.
// Violations: bits in out[0] (1 label out of range or in an empty slot, 2 histogram != counts, 4 sum of
// counts != n_global, 8 K or the dense table wrong), counts in out[1..3]; ctl->err |= kErrInvariant.
hipError_t np8_launch_invariants(const int32_t *z, int64_t n, const int32_t *cnt, const int32_t *dense_of,
                                 const double *cand, int CS, int D, int kcap, int64_t n_global, int check_hist,
                                 int32_t *hist, unsigned long long *out, np8::Ctl *ctl, hipStream_t s);
// Membership change log (np8_changes): items whose slot differs from the baseline (wave-aggregated append,
// out[0..cap) kept, *count = all of them), and per slot 0 / 1 created / 2 removed / 3 parameters changed.
hipError_t np8_launch_changes(const int32_t *z, const int32_t *z_base, int64_t n, int64_t *out_item, int32_t *out_slot,
                              int64_t cap, unsigned long long *count, const int32_t *cnt, const int32_t *cnt_base,
                              const double *mu, const double *mu_base, const double *sg, const double *sg_base, int D,
                              int kcap, uint8_t *flags, hipStream_t s);
// Parity/debug: the sweep's categorical draw (pick_step) on given log-weights, one lane per draw.
hipError_t np8_launch_pick_batch(const double *lw, int32_t n, const double *u, int64_t n_draws, int32_t *out,
                                 hipStream_t s);
hipError_t np8_launch_aux_bounds(const np8::AssignArgs &A, int D, int M, const int64_t *idx, int64_t n, double *out,
                                 hipStream_t s);
hipError_t np8_launch_loglik_matrix(const np8::AssignArgs &A, int D, int M, int prior, const int64_t *idx, int64_t n,
                                    double *out, hipStream_t s);
size_t np8_finalize_lds_bytes(int kcap);
hipError_t np8_launch_finalize(const np8::FinArgs &F, hipStream_t s);
// np8_step_tail: grid sized for the deferred waves of a step of n_waves fast-kernel waves (T.queue) or the radius
// records (T.fold), else one workgroup
hipError_t np8_launch_step_tail(const np8::AssignArgs &A, const np8::FinArgs &F, const np8::PruneArgs &P,
                                const np8::TailArgs &T, int64_t n_waves, int D, int M, hipStream_t s);
hipError_t np8_launch_req_select(const unsigned char *stage, int64_t stage_cap, unsigned char *rec, int64_t rec_cap,
                                 int kcap, int D, int req_max, const np8::Fx *llpart, int64_t ll_n, hipStream_t s);
// compact exchange, check sweeps: this rank's exact sum of the step's per-wave log-likelihoods into the compact
// record's header (nothing once ctl->halt is set)
hipError_t np8_launch_ll_header(const np8::Ctl *ctl, const np8::Fx *llpart, int64_t ll_n, unsigned char *rec,
                                hipStream_t s);
// z_best back to item order if np8_assign_fast left it in label-sorted position order (ctl->best_sorted): through
// scratch (n ints) with the current layout's ids; a no-op otherwise.  Before every re-sort and every read of z_best.
hipError_t np8_launch_best_unsort(np8::Ctl *ctl, const int32_t *ids, int32_t *z_best, int32_t *scratch, int64_t n,
                                  hipStream_t s);
// A snapshot the folded max-likelihood check left pending (ctl->snap_pend): copy it now and clear the flag.
hipError_t np8_launch_snapshot_flush(const np8::SnapArgs &A, np8::Ctl *ctl, hipStream_t s);
hipError_t np8_launch_loglik(const np8::LoglikArgs &A, int D, hipStream_t s);
// np8_rt.hip: the fp64 kernels with D and M at run time, for the (D, M) np8_supported() has no instance of (the
// dispatchers above fall back to them): 8 < D <= kMaxD, reference prior
hipError_t np8_launch_assign_rt(const np8::AssignArgs &A, int D, int M, hipStream_t s);
hipError_t np8_launch_loglik_rt(const np8::LoglikArgs &A, int D, hipStream_t s);
hipError_t np8_launch_loglik_matrix_rt(const np8::AssignArgs &A, int D, int M, const int64_t *idx, int64_t n,
                                       double *out, hipStream_t s);
bool np8_rt_supported(int D, int M, int prior);
hipError_t np8_launch_loglik_reduce(const double *partial, int64_t nb, double *out, double *out2, hipStream_t s);
hipError_t np8_launch_snapshot(const np8::SnapArgs &A, hipStream_t s);
hipError_t np8_launch_suffstats(const np8::ParamArgs &A, hipStream_t s);
hipError_t np8_launch_suffstats_wide(const np8::ParamArgs &P, hipStream_t s);
int64_t np8_suffstats_wide_waves(int64_t n);   // waves of one np8_suffstats_wide launch
int64_t np8_suffstats_wide_record(int D);      // doubles of one run record
hipError_t np8_launch_mh_g0(const np8::ParamArgs &A, hipStream_t s);
hipError_t np8_launch_advance_epoch(np8::Ctl *ctl, uint32_t n, hipStream_t s);
// ctl->best_sorted (which = 0) or ctl->snap_pend (1) = 0 in stream order, unless a compact sweep graph is halted
hipError_t np8_launch_ctl_clear(np8::Ctl *ctl, int which, hipStream_t s);
// p[0..n) = 0 in stream order, unless a compact sweep graph is halted (the captured form of a memset)
hipError_t np8_launch_clear_unless_halted(double *p, int n, const np8::Ctl *ctl, hipStream_t s);
hipError_t np8_launch_prune(const np8::PruneArgs &A, int kcap, hipStream_t s);
hipError_t np8_launch_fin_prune(const np8::FinArgs &F, const np8::PruneArgs &P, hipStream_t s);
hipError_t np8_launch_sm_members(const np8::SmArgs &A, hipStream_t s);
hipError_t np8_launch_sm_eval(const np8::SmArgs &A, hipStream_t s);
hipError_t np8_launch_sm_apply(const np8::SmArgs &A, const np8::FinArgs &F, int64_t a, hipStream_t s);
hipError_t np8_launch_tri_bound(const np8::SmArgs &A, hipStream_t s);
hipError_t np8_launch_tri_eval(const np8::SmArgs &A, hipStream_t s);
hipError_t np8_launch_tri_apply(const np8::SmArgs &A, const np8::FinArgs &F, int64_t a, hipStream_t s);
