// np8_capi.hip -- the C ABI (include/np8.h): context, device memory, sweep orchestration, RCCL.
//
// Replaces, for the Neal-8 path, the reference's per-point call chain
//   MCMC::run (src/np_mcmc.cpp:109-175) -> NealAlgorithm8::update (src/np_neal_algorithm8.cpp:49-167)
//   -> membertrix retract/assign/addCluster (src/membertrix.cpp:87-244)
// with sweep-granular launches: per synchronous step one np8_assign grid and one np8_finalize
// workgroup (plus one ncclAllGather of the exchange record when sharded over ranks).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/np8.h"
#include "np8_device.h"
#include "np8_kernels.h"

using namespace np8;

namespace {

constexpr double kLog2PiC = 1.8378770664093454835606594728112;
constexpr int kPruneMaxKcap = 4096;  // kcap x kcap int32 candidate lists (64 MB at the limit)
#ifndef NP8_GATHER_EVERY
#define NP8_GATHER_EVERY 10  // divides kGraphSweeps (the gathering pattern is baked into the sweep graph)
#endif
#ifndef NP8_RESORT_EVERY
#define NP8_RESORT_EVERY 10
#endif
constexpr uint32_t kGatherEvery = NP8_GATHER_EVERY;  // data-parallel sweeps per gathering of fresh pruning radii
#ifndef NP8_GATHER_PHASE
#define NP8_GATHER_PHASE 1  // (0 put every gathering sweep on a max-likelihood sweep: 0.4% slower at C3)
#endif
constexpr uint32_t kGatherPhase = NP8_GATHER_PHASE;  // the epoch (mod kGatherEvery) of the gathering sweeps

// Host state of one step of a captured compact sweep graph, taken right after its assign was captured: what the rest
// of the step and end_sweep read.  A replay that halts at step i resumes from it (np8_sweep, recover_halt).
struct HostSnap {
    uint32_t di = 0;       // epoch offset from the graph's first sweep
    int32_t dchecks = 0;   // max-likelihood checks before it, in the graph
    int64_t dfolded = 0, dtail = 0;
    int64_t assign_waves = 0;
    bool step_ll = false, step_snap = false, sweep_ll = false, snap_lazy = false, collecting = false, gather = false,
         lists_valid = false, r2_zero = false, gath_clear = false, pruned_last = false, use_sorted = false,
         sorted_valid = false, churn = false;
};

struct Timer {
    hipEvent_t a = nullptr, b = nullptr;
    int phase = -1;  // -1: not timed
    hipGraphNode_t na = nullptr, nb = nullptr;  // event-record nodes when captured into a sweep graph
};

}  // namespace

struct np8_ctx {
    // configuration
    int D = 0, M = 0, DP = 0, CS = 0, kcap = 0;
    int DT = 0;  // the wide path's tile dimension: D rounded up to 16 (item rows and contraction tables, zero beyond D)
    int64_t uw_off = 0;  // wide path: offset of AssignArgs::uw in hyp
    int64_t rec_cap = 0;  // requests the exchanged record holds (one rank: every item of a step)
    int req_max = NP8_REQ_DEFAULT;
    double alpha = 1.0, kappa = 1.0, nu = 1.0;
    uint64_t seed = 0;
    int64_t chunk = 0;
    int device = 0;
    int param_update = NP8_PARAM_FROZEN, mh_steps = 20;
    int prior = NP8_PRIOR_REFERENCE;
    // NIW prior: U = chol(Psi0^{-1}) (lower), U^{-1}; device copies and the pending-request list
    std::vector<double> U, Uinv;
    double *d_U = nullptr, *d_Uinv = nullptr, *d_Psi0 = nullptr;
    int64_t *pend = nullptr;
    int64_t *pend_ll = nullptr;  // wide path, folded check: the accepted requesters' old slot and position (FinArgs)
    // wide path (NP8_CONTRACT_F32_MFMA, D in {32, 48, 64}): fp32 items in X/Xs, fp32 MFMA contraction
    int contraction = NP8_CONTRACT_F64;
    bool wide = false;
    bool rt = false;  // the fp64 kernels with D and M at run time (np8_rt.hip): a (D, M) without a templated instance
    float *wA = nullptr, *wfrag = nullptr, *wmu = nullptr;
    int32_t *wdirty = nullptr;
    double *lam_lo = nullptr, *wdist = nullptr;  // wide-path candidate pruning (np8_wide_dist)
    bool screen16 = false;  // wide path: every item's |x|^2 <= kScreen16X2 (the fp16 exact-distance screen, AssignArgs)
    double *acc = nullptr;  // [kcap][D + DP] parameter-update statistics
    // wide path, one rank, niw_conjugate: np8_suffstats_wide's run records (reduced by np8_niw_post, no atomics)
    double *part = nullptr;
    int32_t *part_slot = nullptr;
    int64_t part_waves = 0;
    // candidate pruning (np8_prune): per-slot radii and per-row candidate lists
    double *r2 = nullptr;
    WaveR2 *wr2 = nullptr;  // per-wave radius records of the sweep's assign (ceil(n_loc / 64))
    int32_t *plist = nullptr, *plen = nullptr;
    float *pdist = nullptr;  // beside plist: the listed rows' distances to the list's own row (the walk's screen)
    int32_t walk_screen = 1;  // NP8_WALK_SCREEN=0: np8_assign_fast evaluates every listed row
    int32_t max_groups = kMaxListGroups;  // NP8_MAX_LIST_GROUPS: own rows per wave walked list by list (more: the whole table)
    unsigned long long *evalc = nullptr;  // [kEvalSlots][2] executed-work counters (timing mode)
    bool prune_on = false;     // kcap small enough for kcap x kcap lists
    bool wide_prune_off = false;  // NP8_NO_PRUNE=1: the wide path evaluates every row (A/B runs)
    bool lists_valid = false;  // plist/plen describe the current table and membership
    bool r2_zero = false;      // the radii in use are initialised (cleared at (re)start: every lane walks all)
    bool collecting = false;   // the running sweep prunes (a data-parallel sweep): lists after every step
    bool gather = false;       // ... and gathers fresh radii (every kGatherEvery-th sweep, or after a restart)
    bool gath_clear = false;   // the last prune zeroed the gathered radius buffer for this sweep
    int64_t assign_waves = 0;  // waves of the last assign launch (its radius records)
    double *plr2 = nullptr;    // per dense row: the squared radius its candidate list assumes
    // two-kernel assign (np8_assign_fast, then np8_assign over the lanes it deferred): reference prior with a
    // diagonal base-measure whitening; NP8_NO_FAST=1 switches it off (A/B runs)
    double *slot_logn1 = nullptr;  // [kcap] log(n - 1) per live slot (np8_finalize)
    int32_t *plen_s = nullptr;     // [kcap] plen / plr2 by slot (np8_prune)
    double *plr2_s = nullptr;
    int32_t *queue = nullptr;  // [64 * waves] deferred positions, by fast-kernel wave
    int32_t *qcount = nullptr; // [waves] deferred lanes per wave
    int32_t *qlist = nullptr;  // [waves] the waves that deferred lanes (ctl->qwaves)
    bool diag_U = false, fast_off = false;
    // fewer launches per step (np8_step_tail): the radius fold, finalize and the candidate lists in one launch
    // (NP8_FUSE=1; off by default: 26.9 vs 23.1 us per sweep at N = 125k)
    bool fuse_off = false;
    bool queue_on = false;  // NP8_QUEUE=1: launch np8_assign_queue after the fast kernel even when no lane can defer
    bool pruned_last = false;    // the sweep's last step built the lists (end_sweep's prune already done)
    // conditional candidate lists (np8_step_tail, TailArgs::prune = 2): the lists of the last build are kept while
    // the counts stay within kListSlack of it; NP8_LISTS_ALWAYS=1 rebuilds them every step (A/B runs)
    double *lb = nullptr;        // [2][kcap] log n | log(n - 1) per slot at the last list build
    bool tailcond_off = false;
    // folded max-likelihood check (DESIGN.md "Max likelihood"): on check sweeps np8_assign_fast sums the items'
    // log-likelihoods per wave (llpart), finalize (or np8_req_select, per rank) reduces them and decides the
    // snapshot, which the next np8_assign_fast copies (snap_lazy: such a copy may be pending on the device, flushed
    // by np8_snapshot_flush before anything else touches the labels); NP8_NO_LLFOLD=1: the separate kernels
    Fx *llpart = nullptr;        // [waves]
    bool llfold_off = false;
    bool step_ll = false;        // the running step folds the check in
    bool wide_llfold = true;     // the wide path folds it too (NP8_WIDE_LLFOLD=0: the separate pass, see launch_assign)
    bool step_snap = false;      // the running step's assign consumes a pending snapshot
    bool sweep_ll = false;       // this sweep's check was folded into its step
    bool snap_lazy = false;
    int64_t n_folded = 0, n_tail_cond = 0;  // (np8_stats; replays of a captured graph add the graph's counts)
    int64_t cap_folded = 0, cap_tail = 0, graph_folded = 0, graph_tail = 0;
    bool host_exch_step = false; // np8_step_local's assign: the host exchange keeps the separate check kernels
    // re-sorts outside the sweep graphs: the graphs carry no periodic re-sort check; before a replay the host looks at
    // ctl->moved as the last finalize mirrored it (host-mapped, one replay behind) and re-sorts when more than n/32
    // items moved (the layout changes no result).  NP8_SORT_IN_GRAPH=1: the check every resort_every-th sweep inside
    int64_t *moved_host = nullptr, *moved_dev = nullptr;
    bool sort_in_graph = false;
    uint32_t fin_advance = 0;    // the next finalize advances ctl->t_base (a captured graph's last step)
    bool fin_advanced = false;
    bool capture_sort_outside = false;  // the graph being captured leaves the re-sort to np8_sweep (and mirrors moved)
    // churn: many items move per sweep (the mixed regime after a cold start; the moved mirror, with hysteresis):
    // sweeps keep the in-graph re-sort every resort_every-th sweep and the parallel np8_prune instead of the
    // conditional one-workgroup lists -- both are the better choice only while few items move (round-4 A/B: mixed
    // sweep 0.164 vs 0.176 ms with the conditional lists; warm sweep 39.8 vs 41.5 µs the other way round)
    bool churn = false, graph_churn = false;
    bool graph_sort_outside = false;    // ... the graph in hand does

    // data-parallel sweep in `substeps` synchronous sub-steps (np8_config.substeps): sub-step s is the
    // contiguous range [sub_start[s], sub_start[s+1]) of the label-sorted layout (sorted by sub-step, slot)
    int substeps = 1;
    bool substeps_auto = false;  // NP8_SUBSTEPS_AUTO: substeps chosen by np8_set_data
    std::vector<int64_t> sub_start;
    int sub_next = 0;  // host-exchange path: the sub-step np8_step_local runs next
    std::vector<double> mu0, Lambda;
    // base-measure precomputes (DESIGN.md "G0")
    std::vector<double> Lc, LT, UinvT, Gp, LTL;  // D*D row-major
    double caux = 0, rsk = 0, logam = 0;
    // data / state
    int64_t n_loc = 0, offset = 0, n_glob = 0;
    uint64_t data_hash = 0;  // of the items as np8_set_data received them (checkpoints name their data)
    bool have_data = false, have_state = false;
    uint32_t epoch = 0;
    int32_t checks = 0;
    // device buffers
    hipStream_t stream = nullptr;
    bool own_stream = false;
    double *X = nullptr;
    int32_t *z = nullptr, *z_best = nullptr;
    double *slot_mu = nullptr, *slot_P = nullptr, *slot_c = nullptr, *slot_sigma = nullptr, *slot_iso = nullptr;
    // [2][kcap] precision eigenvalue bounds lo | hi per slot (0: unknown -- the row is never left out of a list), for the
    // candidate lists of rows that are not isotropic; Gp's (G0 draws: P = Gp / v^2)
    double *slot_lam = nullptr;
    double gp_lamlo = 0.0, gp_lamhi = 0.0;
    double gp_iso = 0.0;
    // every row np8_assign_fast can meet is isotropic (the uploaded live slots, and every G0 draw: gp_iso > 0), so
    // it defers no lane and np8_assign_queue is left out of the step (a restored checkpoint: unknown, false)
    bool rows_iso = false;
    int32_t *cnt = nullptr, *cnt_best = nullptr;
    double *mu_best = nullptr, *sigma_best = nullptr;
    double *cand = nullptr;
    int32_t *dense_of = nullptr;
    Ctl *ctl = nullptr;
    double *hyp = nullptr, *d_mu0 = nullptr, *d_LT = nullptr, *d_Gp = nullptr, *d_LTL = nullptr;
    unsigned char *rec = nullptr, *gath = nullptr;
    int64_t rec_bytes = 0;
    // several ranks: the assign kernels append to the staging record (every item of a step), and
    // np8_req_select moves this rank's req_max lowest-position requests into rec
    unsigned char *stage = nullptr;
    int64_t stage_cap = 0;
    // np8_update_points: visits of each item within the current epoch (tag = epoch + 1)
    std::vector<uint32_t> vis_tag, vis_n;
    int64_t *order = nullptr;
    int64_t order_cap = 0;
    double *partial = nullptr;
    int64_t partial_cap = 0;
    // label-sorted layout (double-buffered) for the synchronous sweep
    double *Xs[2] = {nullptr, nullptr};
    int32_t *zs[2] = {nullptr, nullptr}, *ids[2] = {nullptr, nullptr};
    int32_t *s_hist = nullptr, *s_cursor = nullptr, *s_off = nullptr;
    bool use_sorted = false;
    bool sorted_valid = false;
    uint32_t resort_every = NP8_RESORT_EVERY;
    uint32_t churn_resort = NP8_RESORT_EVERY;  // ... while in churn mode (NP8_CHURN_RESORT; a divisor of kGraphSweeps)
    bool niw_valu = false;  // NP8_NIW_VALU=1: np8_niw_post's dense products on the vector ALU (A/B runs)
    // sweep graphs: kGraphSweeps synchronous sweeps captured once and replayed (launch gaps)
    uint32_t t_base = 0;  // host mirror of ctl->t_base
    hipGraphExec_t graph = nullptr;
    hipGraph_t graph_tmpl = nullptr;  // kept alive: its event-record nodes are re-pointed per replay
    int capture_timed_left = 0;
    int graph_par = -1;          // max-likelihood check parity the graph was captured at
    int graph_phase = -1;        // epoch mod kGraphSweeps the graph was captured at
    bool graph_mh = false;
    int graph_timing = 0;
    bool capturing = false, graphs_off = false;
    std::vector<Timer> graph_timers;
    bool graph_snap0 = false, graph_snap1 = false;  // snap_lazy when the graph's sweeps start and end
    // multi-GPU
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    // compact exchange: the steps of a sharded sweep graph all-gather compact records -- the count deltas
    // and at most c_cap requests per rank -- instead of the full ones (req_max requests); a step with more requests on
    // some rank halts the graph on every rank, and the host runs that step's exchange with the full records
    unsigned char *crec = nullptr, *cgath = nullptr;
    int64_t c_bytes = 0;
    int c_cap = 32;            // NP8_COMPACT_REQ (0: full records always)
    bool compact_on = false;   // the next captured sharded graph exchanges compact records (policy, alike on all ranks)
    bool compact_step = false; // the step being launched does
    bool host_compact = false; // np8_step_local_compact's assign (the host transport's compact step)
    bool host_cstep = false;   // ... its record awaits np8_step_merge_compact
    bool host_halted = false;  // ... which halted: np8_step_resume writes the step's full record
    bool graph_compact = false;
    int32_t *mirror_host = nullptr, *mirror_dev = nullptr;  // host-mapped [kMirrorInts] (np8::FinArgs::mirror)
    std::vector<HostSnap> graph_snaps, cap_snaps;
    uint32_t cap_sweep = 0;
    int32_t cap_checks0 = 0;
    // the last replay of a sharded graph, checked once the next one is queued (or by settle)
    bool pend_on = false, pend_compact = false;
    uint32_t pend_epoch = 0;
    int32_t pend_checks = 0;
    int64_t pend_folded = 0, pend_tail = 0;
    hipEvent_t rev[2] = {nullptr, nullptr};
    int rev_k = 0, pend_k = 0;
    int64_t n_halts = 0;
    // timing: event pairs around launches; count_eval: the assign kernels' executed-work counters
    bool timing = false, count_eval = false, time_all = false;
    std::vector<Timer> timers;
    std::vector<hipEvent_t> event_pool;
    double ms[6] = {0, 0, 0, 0, 0, 0};  // assign, finalize, loglik, params, sm members, sm eval
    int64_t n_timed[6] = {0, 0, 0, 0, 0, 0};
    // Jain-Neal split-merge (np8_sm_sweep): member lists, own/cross likelihoods, batch outcomes
    int32_t *sm_hist = nullptr, *sm_mem = nullptr, *sm_off = nullptr, *sm_live = nullptr;
    double *sm_Xm = nullptr, *sm_ownm = nullptr, *sm_cross = nullptr;
    int64_t *sm_slist = nullptr;
    double *sm_stheta = nullptr;
    SmCtl *sm_ctl = nullptr;
    uint8_t *sm_typ = nullptr;
    int64_t *sm_first_host = nullptr;  // pinned
    int64_t sm_n = -1, sm_cross_cap = 0;
    int32_t sm_batch = 1024;
    int32_t sm_K = 0;
    bool sm_all_iso = false;
    double *sm_mb = nullptr;  // triadic merge bound: [kcap][4] member sums per live row (np8_tri_bound)
    bool sm_mb_on = false, tri_bound_off = false;
    // NP8_FINPRUNE=1: finalize and the lists in one launch (np8_fin_prune), opt-in: measured slower (125k items:
    // 26.6 vs 21.1 us per sweep; 1e6: 51.7 vs 46.1) -- the agent-scope release/acquire between its workgroups
    // (L2 writeback and invalidate across the XCDs) costs more than the dependent dispatch it saves
    bool fp_off = true;
    // membership change log (np8_track_changes / np8_changes): the baseline state and the output staging
    int track = 0;
    int32_t *z_base = nullptr, *cnt_base = nullptr, *chg_slot = nullptr;
    double *mu_base = nullptr, *sigma_base = nullptr;
    int64_t *chg_item = nullptr;
    int64_t chg_cap = 0;
    unsigned long long *chg_count = nullptr;
    uint8_t *chg_flags = nullptr;
    // debug invariants (np8_check_invariants; every sweep with NP8_DEBUG_INVARIANTS=1)
    bool debug_inv = false;
    int32_t *inv_hist = nullptr;
    unsigned long long *inv_out = nullptr;
    std::string err;
};

namespace {

int fail(np8_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPC(ctx, expr)                                                                                   \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            return fail(ctx, NP8_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));           \
    } while (0)

#define NCCLC(ctx, expr)                                                                                  \
    do {                                                                                                 \
        ncclResult_t r_ = (expr);                                                                        \
        if (r_ != ncclSuccess) return fail(ctx, NP8_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

int packed_index(int D, int a, int b) { return a * D - (a * (a - 1)) / 2 + (b - a); }

// 64-bit FNV-1a over 8-byte words (checkpoint identity, not a security hash)
uint64_t hash_words(uint64_t h, const void *p, size_t bytes) {
    const unsigned char *b = static_cast<const unsigned char *>(p);
    for (size_t i = 0; i < bytes; i += 8) {
        uint64_t w = 0;
        std::memcpy(&w, b + i, (bytes - i) < 8 ? (bytes - i) : 8);
        h = (h ^ w) * 0x100000001b3ull;
        h ^= h >> 29;
    }
    return h;
}


// LU with partial pivoting (what Eigen's MatrixXd::inverse()/determinant() use,
// multivariatenormal.cpp:87,90).  Row-major.  Returns false when singular.
bool lu_inverse_det(const double *A, int D, double *inv, double *det) {
    std::vector<double> LU(A, A + (size_t)D * D);
    std::vector<int> perm(D);
    int sign = 1;
    for (int i = 0; i < D; ++i) perm[i] = i;
    for (int k = 0; k < D; ++k) {
        int p = k;
        double best = std::fabs(LU[k * D + k]);
        for (int i = k + 1; i < D; ++i)
            if (std::fabs(LU[i * D + k]) > best) {
                best = std::fabs(LU[i * D + k]);
                p = i;
            }
        if (best == 0.0) return false;
        if (p != k) {
            for (int j = 0; j < D; ++j) std::swap(LU[k * D + j], LU[p * D + j]);
            std::swap(perm[k], perm[p]);
            sign = -sign;
        }
        for (int i = k + 1; i < D; ++i) {
            const double f = LU[i * D + k] / LU[k * D + k];
            LU[i * D + k] = f;
            for (int j = k + 1; j < D; ++j) LU[i * D + j] = LU[i * D + j] - f * LU[k * D + j];
        }
    }
    double d = (double)sign;
    for (int k = 0; k < D; ++k) d *= LU[k * D + k];
    *det = d;
    std::vector<double> y(D);
    for (int col = 0; col < D; ++col) {
        for (int i = 0; i < D; ++i) {
            double s = (perm[i] == col) ? 1.0 : 0.0;
            for (int j = 0; j < i; ++j) s -= LU[i * D + j] * y[j];
            y[i] = s;
        }
        for (int i = D - 1; i >= 0; --i) {
            double s = y[i];
            for (int j = i + 1; j < D; ++j) s -= LU[i * D + j] * y[j];
            y[i] = s / LU[i * D + i];
        }
        for (int i = 0; i < D; ++i) inv[i * D + col] = y[i];
    }
    return true;
}

// Cholesky (lower) and lower-triangular inverse in the loop order of oracle/np8_oracle.c (chol_lower,
// inv_lower): the NIW precomputes must agree to the bit with the oracle's.
bool chol_lower(const double *A, int D, std::vector<double> &L) {
    L.assign((size_t)D * D, 0.0);
    for (int j = 0; j < D; ++j) {
        double s = A[j * D + j];
        for (int k = 0; k < j; ++k) s -= L[j * D + k] * L[j * D + k];
        if (!(s > 0.0)) return false;
        L[j * D + j] = std::sqrt(s);
        for (int i = j + 1; i < D; ++i) {
            double v = A[i * D + j];
            for (int k = 0; k < j; ++k) v -= L[i * D + k] * L[j * D + k];
            L[i * D + j] = v / L[j * D + j];
        }
    }
    return true;
}

void inv_lower(const std::vector<double> &L, int D, std::vector<double> &Li) {
    Li.assign((size_t)D * D, 0.0);
    for (int j = 0; j < D; ++j) {
        Li[j * D + j] = 1.0 / L[j * D + j];
        for (int r = j + 1; r < D; ++r) {
            double s = 0.0;
            for (int k = j; k < r; ++k) s -= L[r * D + k] * Li[k * D + j];
            Li[r * D + j] = s / L[r * D + r];
        }
    }
}

// NIW prior (DESIGN.md "Priors"): U = chol(Psi0^{-1}) with Psi0^{-1} = Lp^{-T} Lp^{-1}, Lp = chol(Psi0);
// UinvT holds U^T (the whitening of the item frame) and caux = -D/2 log 2pi + sum log U_aa.
bool prepare_niw(np8_ctx *c) {
    const int D = c->D;
    std::vector<double> Lp, Li, Pi((size_t)D * D);
    if (!chol_lower(c->Lambda.data(), D, Lp)) return false;
    inv_lower(Lp, D, Li);
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) {
            double s = 0.0;
            for (int k = (a > b ? a : b); k < D; ++k) s += Li[k * D + a] * Li[k * D + b];
            Pi[a * D + b] = s;
        }
    if (!chol_lower(Pi.data(), D, c->U)) return false;
    inv_lower(c->U, D, c->Uinv);
    double sl = 0.0;
    for (int a = 0; a < D; ++a) sl += std::log(c->U[a * D + a]);
    c->caux = -0.5 * (double)D * kLog2PiC + sl;
    c->UinvT.assign((size_t)D * D, 0.0);
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) c->UinvT[a * D + b] = c->U[b * D + a];
    c->LT.assign((size_t)D * D, 0.0);  // unused by the NIW prior
    c->Gp.assign((size_t)D * D, 0.0);
    c->LTL.assign((size_t)D * D, 0.0);
    c->gp_iso = 0.0;
    c->rsk = 1.0 / std::sqrt(c->kappa);
    c->logam = std::log(c->alpha / (double)c->M);
    return true;
}

// Bounds lo <= eig(S) <= hi of a symmetric n x n matrix S (row-major, overwritten): cyclic Jacobi rotations to an
// off-diagonal mass below 1e-30 of the total, then the diagonal's range widened by 1e-9 of the largest magnitude (the
// rotations' rounding is ~n eps of it).  For the candidate lists' bound (prune_row), which keeps 2 nats of margin.
void sym_eig_bounds(std::vector<double> &S, int n, double &lo, double &hi) {
    double tot = 0.0;
    for (double v : S) tot += v * v;
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) off += S[p * n + q] * S[p * n + q];
        if (off <= 1e-30 * tot) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = S[p * n + q];
                if (apq == 0.0) continue;
                const double th = (S[q * n + q] - S[p * n + p]) / (2.0 * apq);
                const double t = (th >= 0.0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
                const double cs = 1.0 / std::sqrt(t * t + 1.0), sn = t * cs;
                for (int k = 0; k < n; ++k) {  // columns p, q
                    const double skp = S[k * n + p], skq = S[k * n + q];
                    S[k * n + p] = cs * skp - sn * skq;
                    S[k * n + q] = sn * skp + cs * skq;
                }
                for (int k = 0; k < n; ++k) {  // rows p, q
                    const double spk = S[p * n + k], sqk = S[q * n + k];
                    S[p * n + k] = cs * spk - sn * sqk;
                    S[q * n + k] = sn * spk + cs * sqk;
                }
            }
    }
    lo = hi = S[0];
    double mag = 0.0;
    for (int a = 0; a < n; ++a) {
        lo = std::min(lo, S[a * n + a]);
        hi = std::max(hi, S[a * n + a]);
        mag = std::max(mag, std::fabs(S[a * n + a]));
    }
    lo -= 1e-9 * mag;
    hi += 1e-9 * mag;
    if (!(lo > 0.0)) lo = 0.0;  // (no bound: never left out)
}

// the bounds of a packed precision (upper triangle, off-diagonals doubled)
void packed_eig_bounds(const double *P, int D, double &lo, double &hi) {
    std::vector<double> S((size_t)D * D);
    for (int a = 0, q = 0; a < D; ++a)
        for (int b = a; b < D; ++b, ++q) {
            const double v = (a == b) ? P[q] : 0.5 * P[q];
            S[(size_t)a * D + b] = S[(size_t)b * D + a] = v;
        }
    sym_eig_bounds(S, D, lo, hi);
}

// Base-measure precomputes: L = chol(Lambda) (invwishart.h:40), (L^T)^{-1}, (L^T L)^{-1}, L^T L.
bool prepare_base(np8_ctx *c) {
    if (c->prior == NP8_PRIOR_NIW) return prepare_niw(c);
    const int D = c->D;
    c->Lc.assign((size_t)D * D, 0.0);
    std::vector<double> &L = c->Lc;
    for (int j = 0; j < D; ++j) {
        double s = c->Lambda[j * D + j];
        for (int k = 0; k < j; ++k) s -= L[j * D + k] * L[j * D + k];
        if (!(s > 0.0)) return false;
        L[j * D + j] = std::sqrt(s);
        for (int i = j + 1; i < D; ++i) {
            double v = c->Lambda[i * D + j];
            for (int k = 0; k < j; ++k) v -= L[i * D + k] * L[j * D + k];
            L[i * D + j] = v / L[j * D + j];
        }
    }
    c->LT.assign((size_t)D * D, 0.0);
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) c->LT[a * D + b] = L[b * D + a];
    c->UinvT.assign((size_t)D * D, 0.0);
    for (int col = 0; col < D; ++col)
        for (int i = col; i >= 0; --i) {
            double s = (i == col) ? 1.0 : 0.0;
            for (int j = i + 1; j <= col; ++j) s -= c->LT[i * D + j] * c->UinvT[j * D + col];
            c->UinvT[i * D + col] = s / c->LT[i * D + i];
        }
    c->Gp.assign((size_t)D * D, 0.0);
    c->LTL.assign((size_t)D * D, 0.0);
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
    for (int a = 0; a < D; ++a) sumlog += std::log(L[a * D + a]);
    c->caux = -0.5 * (double)D * kLog2PiC - sumlog;
    c->rsk = 1.0 / std::sqrt(c->kappa);
    c->logam = std::log(c->alpha / (double)c->M);
    bool iso = true;
    for (int a = 0; a < D; ++a)
        for (int b = 0; b < D; ++b) iso = iso && ((a == b) ? c->Gp[a * D + b] == c->Gp[0] : c->Gp[a * D + b] == 0.0);
    c->gp_iso = iso ? c->Gp[0] : 0.0;
    {  // Gp's eigenvalue bounds (a G0 draw's precision is Gp / v^2)
        std::vector<double> S((size_t)D * D);
        for (int a = 0; a < D; ++a)
            for (int b = a; b < D; ++b) {
                const double v = (a == b) ? c->Gp[a * D + b] : 0.5 * c->Gp[a * D + b];
                S[(size_t)a * D + b] = S[(size_t)b * D + a] = v;
            }
        sym_eig_bounds(S, D, c->gp_lamlo, c->gp_lamhi);
        if (c->gp_lamlo <= 0.0) c->gp_lamhi = 0.0;
    }
    return true;
}

// Host copy of a slot's parameters.
struct SlotHost {
    std::vector<double> mu, P, sigma;
    double c = 0.0;
};

// G0 draw from (scale normal g0, xi): v = D + nu g0, mu = mu0 + (|v|/sqrt(kappa)) L^T xi.
void slot_from_normals(const np8_ctx *c, double g0, const double *xi, SlotHost &o) {
    const int D = c->D;
    const double v = std::fma(c->nu, g0, (double)D);
    const double s = std::fabs(v) * c->rsk;
    o.mu.resize(D);
    for (int a = 0; a < D; ++a) {
        double t = c->LT[a * D + a] * xi[a];
        for (int b = a + 1; b < D; ++b) t = std::fma(c->LT[a * D + b], xi[b], t);
        o.mu[a] = std::fma(s, t, c->mu0[a]);
    }
    const double v2 = v * v;
    o.P.resize(c->DP);
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) o.P[packed_index(D, a, b)] = c->Gp[a * D + b] / v2;
    o.c = std::fma(-(double)D, log_pos(std::fabs(v)), c->caux);
    o.sigma.resize((size_t)D * D);
    for (int k = 0; k < D * D; ++k) o.sigma[k] = v2 * c->LTL[k];
}

bool slot_from_sigma(const np8_ctx *c, const double *mu, const double *Sigma, SlotHost &o) {
    const int D = c->D;
    std::vector<double> inv((size_t)D * D);
    double det = 0.0;
    if (!lu_inverse_det(Sigma, D, inv.data(), &det) || !(det > 0.0)) return false;
    o.mu.assign(mu, mu + D);
    o.sigma.assign(Sigma, Sigma + (size_t)D * D);
    o.P.resize(c->DP);
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b)
            o.P[packed_index(D, a, b)] = (a == b) ? inv[a * D + a] : inv[a * D + b] + inv[b * D + a];
    o.c = -0.5 * ((double)D * kLog2PiC + std::log(det));
    return true;
}

void free_device(np8_ctx *c) {
    void *niw_ptrs[] = {c->d_U, c->d_Uinv, c->d_Psi0, c->pend, c->wA, c->wfrag, c->wmu, c->wdirty, c->lam_lo, c->wdist,
                        c->pend_ll};
    for (void *p : niw_ptrs)
        if (p) (void)hipFree(p);
    c->d_U = c->d_Uinv = c->d_Psi0 = nullptr;
    c->pend = c->pend_ll = nullptr;
    c->wA = c->wfrag = c->wmu = nullptr;
    c->wdirty = nullptr;
    c->lam_lo = c->wdist = nullptr;
    void *ptrs[] = {c->X,      c->z,       c->z_best, c->slot_mu, c->slot_P,  c->slot_c,  c->slot_sigma,
                    c->cnt,    c->cnt_best, c->mu_best, c->sigma_best, c->cand, c->ctl,    c->hyp,
                    c->d_mu0,  c->d_LT,    c->d_Gp,   c->d_LTL,   c->rec,     c->gath,    c->order,
                    c->partial, c->dense_of, c->Xs[0], c->Xs[1], c->zs[0], c->zs[1], c->ids[0], c->ids[1],
                    c->s_hist, c->s_cursor, c->s_off, c->slot_iso, c->acc, c->r2, c->wr2, c->plist, c->pdist, c->plen, c->plr2,
                    c->sm_hist, c->sm_mem, c->sm_off, c->sm_live, c->sm_Xm, c->sm_ownm, c->sm_cross, c->sm_ctl,
                    c->sm_typ, c->sm_slist, c->sm_stheta, c->stage, c->evalc, c->z_base, c->cnt_base,
                    c->chg_slot, c->mu_base, c->sigma_base, c->chg_item, c->chg_count, c->chg_flags,
                    c->inv_hist, c->inv_out, c->queue, c->qcount, c->qlist, c->slot_logn1, c->plen_s,
                    c->plr2_s, c->sm_mb, c->lb, c->llpart, c->part, c->part_slot, c->crec, c->cgath, c->slot_lam};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    c->crec = c->cgath = nullptr;
    if (c->mirror_host) (void)hipHostFree(c->mirror_host);
    c->mirror_host = c->mirror_dev = nullptr;
    for (hipEvent_t &e : c->rev)
        if (e) {
            (void)hipEventDestroy(e);
            e = nullptr;
        }
    if (c->sm_first_host) (void)hipHostFree(c->sm_first_host);
    if (c->moved_host) (void)hipHostFree(c->moved_host);
    c->moved_host = c->moved_dev = nullptr;
    c->sm_hist = c->sm_mem = c->sm_off = c->sm_live = nullptr;
    c->sm_Xm = c->sm_ownm = c->sm_cross = nullptr;
    c->sm_slist = nullptr;
    c->sm_stheta = nullptr;
    c->sm_ctl = nullptr;
    c->sm_typ = nullptr;
    c->sm_first_host = nullptr;
    c->sm_n = -1;
    c->sm_cross_cap = 0;
    c->sm_mb = nullptr;
    for (int b = 0; b < 2; ++b) {
        c->Xs[b] = nullptr;
        c->zs[b] = c->ids[b] = nullptr;
    }
    c->s_hist = c->s_cursor = c->s_off = nullptr;
    c->slot_iso = nullptr;
    c->slot_lam = nullptr;
    c->lb = nullptr;
    c->llpart = nullptr;
    c->part = nullptr;
    c->part_slot = nullptr;
    c->acc = nullptr;
    c->r2 = nullptr;
    c->wr2 = nullptr;
    c->z_base = c->cnt_base = c->chg_slot = nullptr;
    c->mu_base = c->sigma_base = nullptr;
    c->chg_item = nullptr;
    c->chg_count = nullptr;
    c->chg_flags = nullptr;
    c->inv_hist = nullptr;
    c->inv_out = nullptr;
    c->chg_cap = 0;
    c->track = 0;
    c->plist = c->plen = nullptr;
    c->pdist = nullptr;
    c->plr2 = nullptr;
    c->X = nullptr;
    c->z = c->z_best = nullptr;
    c->slot_mu = c->slot_P = c->slot_c = c->slot_sigma = nullptr;
    c->cnt = c->cnt_best = nullptr;
    c->mu_best = c->sigma_best = c->cand = nullptr;
    c->ctl = nullptr;
    c->hyp = c->d_mu0 = c->d_LT = c->d_Gp = c->d_LTL = nullptr;
    c->rec = c->gath = c->stage = nullptr;
    c->evalc = nullptr;
    c->order = nullptr;
    c->partial = nullptr;
    c->dense_of = nullptr;
}

template <typename T>
int dalloc(np8_ctx *c, T **p, size_t n) {
    if (*p) {
        (void)hipFree(*p);
        *p = nullptr;
    }
    HIPC(c, hipMalloc((void **)p, sizeof(T) * (n ? n : 1)));
    HIPC(c, hipMemsetAsync(*p, 0, sizeof(T) * (n ? n : 1), c->stream));
    return NP8_OK;
}

// Exchange records (DESIGN.md "Finalize").  One rank: rec holds every item of a step (the assign kernel
// appends there).  Several ranks: rec holds the req_max requests np8_req_select picks and is what the
// ranks exchange; the staging record holds every item of a step.
int alloc_records(np8_ctx *c) {
    const int64_t items = c->n_loc > 0 ? c->n_loc : 1;
    if (items > 0x7FFFFFFFll) return fail(c, NP8_ERR_ARG, "more than 2^31 items on one rank");
    // exchanged records (several ranks, or an RCCL communicator of any size): a rank sends at most req_max
    // requests, its lowest scan positions (np8_req_select from the staging record)
    const bool exch = c->world > 1 || c->comm;
    c->rec_cap = exch ? c->req_max : (items > c->req_max ? items : c->req_max);
    c->stage_cap = exch ? items : 0;
    c->rec_bytes = record_bytes(c->kcap, (int)c->rec_cap, c->D);
    int r = dalloc(c, &c->rec, (size_t)c->rec_bytes);
    if (r) return r;
    if (exch) {
        if ((r = dalloc(c, &c->gath, (size_t)c->rec_bytes * c->world)) ||
            (r = dalloc(c, &c->stage, (size_t)record_bytes(c->kcap, (int)c->stage_cap, c->D))))
            return r;
    } else if (c->stage) {
        (void)hipFree(c->stage);
        c->stage = nullptr;
    }
    // compact records of the RCCL path's sweep graphs (the same layout with c_cap requests), and of the host
    // transport's compact steps (np8_step_local_compact)
    // (the wide path: the host transport's compact steps only -- its sweep graphs exchange the full records)
    if (exch && c->c_cap > 0) {
        c->c_bytes = record_bytes(c->kcap, c->c_cap, c->D);
        if ((r = dalloc(c, &c->crec, (size_t)c->c_bytes)) || (r = dalloc(c, &c->cgath, (size_t)c->c_bytes * c->world)))
            return r;
        c->compact_on = c->comm != nullptr && !c->wide;
    }
    return NP8_OK;
}

int upload_slots(np8_ctx *c, const std::vector<SlotHost> &slots, const std::vector<int32_t> &cnt) {
    const int D = c->D, DP = c->DP, K = (int)slots.size();
    std::vector<double> mu((size_t)c->kcap * D, 0.0), P((size_t)c->kcap * DP, 0.0), cc(c->kcap, 0.0),
        sg((size_t)c->kcap * D * D, 0.0), iso(c->kcap, 0.0);
    for (int s = 0; s < K; ++s) {
        std::memcpy(&mu[(size_t)s * D], slots[s].mu.data(), sizeof(double) * D);
        std::memcpy(&P[(size_t)s * DP], slots[s].P.data(), sizeof(double) * DP);
        std::memcpy(&sg[(size_t)s * D * D], slots[s].sigma.data(), sizeof(double) * D * D);
        cc[s] = slots[s].c;
        // isotropic precision: off-diagonals exactly 0 and one common diagonal (DESIGN.md "Pick")
        bool is = true;
        for (int a = 0, q = 0; a < D; ++a)
            for (int b = a; b < D; ++b, ++q)
                is = is && ((a == b) ? slots[s].P[q] == slots[s].P[0] : slots[s].P[q] == 0.0);
        iso[s] = is ? slots[s].P[0] : 0.0;
    }
    c->rows_iso = c->gp_iso > 0.0;
    for (int s = 0; s < K; ++s) c->rows_iso = c->rows_iso && (cnt[s] == 0 || iso[s] > 0.0);
    HIPC(c, hipMemcpyAsync(c->slot_iso, iso.data(), sizeof(double) * iso.size(), hipMemcpyHostToDevice, c->stream));
    if (c->slot_lam) {  // eigenvalue bounds of the live slots that are not isotropic (the candidate lists' bound)
        std::vector<double> lam(2 * (size_t)c->kcap, 0.0);
        for (int s = 0; s < K; ++s) {
            if (iso[s] > 0.0) {
                lam[s] = lam[c->kcap + s] = iso[s];
            } else if (cnt[s] > 0) {
                packed_eig_bounds(slots[s].P.data(), D, lam[s], lam[c->kcap + s]);
                if (lam[s] <= 0.0) lam[c->kcap + s] = 0.0;
            }
        }
        HIPC(c, hipMemcpyAsync(c->slot_lam, lam.data(), sizeof(double) * lam.size(), hipMemcpyHostToDevice, c->stream));
    }
    std::vector<int32_t> cn(c->kcap, 0);
    for (int s = 0; s < K; ++s) cn[s] = cnt[s];
    HIPC(c, hipMemcpyAsync(c->slot_mu, mu.data(), sizeof(double) * mu.size(), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->slot_P, P.data(), sizeof(double) * P.size(), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->slot_c, cc.data(), sizeof(double) * cc.size(), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->slot_sigma, sg.data(), sizeof(double) * sg.size(), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->cnt, cn.data(), sizeof(int32_t) * cn.size(), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

// Device timing: event pairs from a reusable pool (no event creation on the launch path).
void collect_timers(np8_ctx *c);

// Inside a stream capture hipEventRecord is not turned into a graph node; an event-record node is
// added to the capturing graph explicitly and becomes the stream's capture dependency.
void record_event(np8_ctx *c, hipEvent_t e, hipGraphNode_t *out = nullptr) {
    if (!c->capturing) {
        (void)hipEventRecord(e, c->stream);
        return;
    }
    hipStreamCaptureStatus st;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t *deps = nullptr;
    size_t nd = 0;
    hipGraphNode_t node;
    if (hipStreamGetCaptureInfo_v2(c->stream, &st, &id, &g, &deps, &nd) == hipSuccess &&
        hipGraphAddEventRecordNode(&node, g, deps, nd, e) == hipSuccess) {
        (void)hipStreamUpdateCaptureDependencies(c->stream, &node, 1, hipStreamSetCaptureDependencies);
        if (out) *out = node;
    }
}

// Event pair number k of the reusable pool.
void pool_pair(np8_ctx *c, size_t k, Timer &t) {
    while (c->event_pool.size() < 2 * (k + 1)) {
        hipEvent_t a;
        (void)hipEventCreate(&a);
        c->event_pool.push_back(a);
    }
    t.a = c->event_pool[2 * k];
    t.b = c->event_pool[2 * k + 1];
}

void timer_begin(np8_ctx *c, int phase, Timer &t) {
    if (!c->timing) return;
    if (c->capturing) {
        // a sweep graph times one assign launch per replay: event-record nodes whose events are
        // re-pointed to fresh pool events before every launch (run_graph)
        if (phase != 0 || c->capture_timed_left <= 0) return;
        c->capture_timed_left -= 1;
        pool_pair(c, 0, t);  // placeholder events, replaced per replay
        t.phase = phase;
        record_event(c, t.a, &t.na);
        return;
    }
    if (c->timers.size() + 1 >= 4096) collect_timers(c);  // bounded pool
    pool_pair(c, c->timers.size(), t);
    t.phase = phase;
    (void)hipEventRecord(t.a, c->stream);
}

void timer_end(np8_ctx *c, Timer &t) {
    if (!c->timing || t.phase < 0) return;
    record_event(c, t.b, &t.nb);
    (c->capturing ? c->graph_timers : c->timers).push_back(t);
}

void collect_timers(np8_ctx *c) {
    if (!c->timers.empty()) (void)hipEventSynchronize(c->timers.back().b);
    for (Timer &t : c->timers) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
            c->ms[t.phase] += ms;
            c->n_timed[t.phase] += 1;
        }
    }
    c->timers.clear();
}

FinArgs fin_args(np8_ctx *c, const unsigned char *recs, int world) {
    FinArgs F;
    std::memset(&F, 0, sizeof(F));
    F.recs = recs;
    F.local_rec = c->rec;
    F.rec_bytes = c->rec_bytes;
    F.world = world;
    F.rec_cap = (int32_t)c->rec_cap;
    F.kcap = c->kcap;
    F.D = c->D;
    F.M = c->M;
    F.cnt = c->cnt;
    F.z = c->z;
    F.zs[0] = c->use_sorted ? c->zs[0] : nullptr;
    F.zs[1] = c->use_sorted ? c->zs[1] : nullptr;
    F.n_loc = c->n_loc;
    F.offset = c->offset;
    F.slot_mu = c->slot_mu;
    F.slot_P = c->slot_P;
    F.slot_c = c->slot_c;
    F.slot_sigma = c->slot_sigma;
    F.slot_iso = c->slot_iso;
    F.slot_logn1 = c->slot_logn1;
    F.gp_iso = c->gp_iso;
    F.slot_lam = c->slot_lam;
    F.gp_lamlo = c->gp_lamlo;
    F.gp_lamhi = c->gp_lamhi;
    F.cand = c->cand;
    F.dense_of = c->dense_of;
    F.ctl = c->ctl;
    F.mu0 = c->d_mu0;
    F.LT = c->d_LT;
    F.Gp = c->d_Gp;
    F.LTL = c->d_LTL;
    F.caux = c->caux;
    F.rsk = c->rsk;
    F.nu = c->nu;
    F.seed = c->seed;
    F.t = c->epoch - c->t_base;
    F.r2 = c->r2;
    F.prior = c->prior;
    F.req_max = c->req_max;
    F.pend = c->pend;
    F.frame_payload = c->wide ? 1 : 0;
    F.pad3 = 0;
    F.hyp = c->hyp;
    F.wdirty = c->wdirty;
    F.ll_on = c->step_ll ? 1 : 0;
    F.ll_rec = c->comm ? 1 : 0;
    F.ll_defer = (c->step_ll && c->wide) ? 1 : 0;
    F.pend_ll = c->pend_ll;
    F.llpart = c->llpart;
    F.ll_n = c->assign_waves;
    F.snap_clear = c->step_snap ? 1 : 0;
    F.par = c->checks & 1;
    F.best = c->ctl->best;
    F.have_best = &c->ctl->have_best;
    F.lb = c->lb;
    // (np8_sweep's re-sort and churn decisions read it: a replay's last finalize, and eager steps)
    F.moved_mirror = (c->fin_advance || !c->capturing) ? c->moved_dev : nullptr;
    if (c->comm) {  // RCCL path: a halt as it happens; the requests' peak over a replay at its last step
        F.mirror = c->mirror_dev;
        F.peak_out = (c->capturing && c->fin_advance) ? 1 : 0;
    }
    if (c->compact_step) {  // the gathered compact records (np8_sweep)
        F.recs = c->cgath;
        F.rec_bytes = c->c_bytes;
        F.rec_cap = c->c_cap;
        F.local_rec = c->crec;
        F.compact = 1;
    }
    F.advance = c->fin_advance;
    if (c->fin_advance) c->fin_advanced = true;
    c->fin_advance = 0;
    return F;
}

WideArgs wide_args(np8_ctx *c) {
    WideArgs W;
    W.D = c->D;
    W.kcap = c->kcap;
    W.DT = c->DT;
    W.dirty = c->wdirty;
    W.cnt = c->cnt;
    W.slot_P = c->slot_P;
    W.slot_mu = c->slot_mu;
    W.wA = c->wA;
    W.wfrag = c->wfrag;
    W.wmu = c->wmu;
    W.lam_lo = c->lam_lo;
    W.ctl = c->ctl;
    W.cand = c->cand;
    W.wdist = c->wdist;
    return W;
}

// Wide path: factors, fp32 means and candidate offsets of the slots flagged in wdirty (all = 1).
int refresh_wide(np8_ctx *c, bool all) {
    if (!c->wide) return NP8_OK;
    if (all) HIPC(c, hipMemsetD32Async(reinterpret_cast<int *>(c->wdirty), 1, c->kcap, c->stream));
    HIPC(c, np8_launch_wide_refresh(wide_args(c), c->stream));
    return NP8_OK;
}

NiwArgs niw_args(np8_ctx *c) {
    NiwArgs A;
    std::memset(&A, 0, sizeof(A));
    A.D = c->D;
    A.kcap = c->kcap;
    A.DT = c->DT;
    A.valu = c->niw_valu ? 1 : 0;
    A.kappa0 = c->kappa;
    A.nu0 = c->nu;
    A.rsk = c->rsk;
    A.caux = c->caux;
    A.mu0 = c->d_mu0;
    A.Psi0 = c->d_Psi0;
    A.U = c->d_U;
    A.Uinv = c->d_Uinv;
    A.seed = c->seed;
    A.t = c->epoch - c->t_base;
    A.write_cand = 1;
    A.ctl = c->ctl;
    A.cnt = c->cnt;
    A.dense_of = c->dense_of;
    A.acc = c->acc;
    A.slot_mu = c->slot_mu;
    A.slot_P = c->slot_P;
    A.slot_c = c->slot_c;
    A.slot_sigma = c->slot_sigma;
    A.slot_iso = c->slot_iso;
    A.cand = c->cand;
    A.r2 = c->r2;
    if (c->wide) {  // the draw's own factor R becomes the slot's contraction rows (no np8_wide_rows factor)
        A.wA = c->wA;
        A.wfrag = c->wfrag;
        A.wmu = c->wmu;
        A.lam_lo = c->lam_lo;
    }
    return A;
}

AssignArgs assign_args(np8_ctx *c, int64_t p0, int64_t p1, const int64_t *order, bool use_perm) {
    AssignArgs A;
    A.X = c->X;
    A.z = c->z;
    A.sorted = c->use_sorted ? 1 : 0;
    for (int b = 0; b < 2; ++b) {
        A.Xs[b] = c->Xs[b];
        A.zs[b] = c->zs[b];
        A.ids[b] = c->ids[b];
    }
    A.cand = c->cand;
    A.dense_of = c->dense_of;
    A.ctl = c->ctl;
    A.hyp = c->hyp;
    A.order = order;
    A.rec = c->rec;
    {  // request area: the record itself (one rank) or the staging record
        unsigned char *area = c->stage ? c->stage : c->rec;
        const int64_t cap = c->stage ? c->stage_cap : c->rec_cap;
        A.nreq = &reinterpret_cast<RecHeader *>(area)->nreq;
        A.req = reinterpret_cast<Request *>(area + kRecHeaderBytes + 4ll * c->kcap);
        A.vmu = reinterpret_cast<double *>(area + record_vmu_offset(c->kcap, (int)cap));
        A.req_cap = (int32_t)cap;
    }
    A.n_loc = c->n_loc;
    A.offset = c->offset;
    A.p0 = p0;
    A.p1 = p1;
    A.use_perm = use_perm ? 1 : 0;
    A.perm = make_perm(c->seed, c->epoch, (uint32_t)c->n_glob);
    A.seed = c->seed;
    A.t = c->epoch - c->t_base;
    A.kcap = c->kcap;
    A.plist = c->plist;
    A.pdist = c->pdist;
    A.walk_screen = c->walk_screen;
    A.max_groups = c->max_groups;
    A.plen = c->plen;
    A.plr2 = c->plr2;
    A.ls = c->kcap;
    A.use_lists = 0;
    A.collect_r2 = 0;
    A.count_eval = c->count_eval ? 1 : 0;
    A.evalc = c->evalc;
    A.r2 = c->r2;
    A.wr2 = c->wr2;
    A.wfrag = c->wfrag;
    A.wmu = c->wmu;
    A.lam_lo = c->lam_lo;
    A.dim = c->D;
    A.uw = c->wide ? c->hyp + c->uw_off : nullptr;
    A.screen16 = c->screen16 ? 1 : 0;
    A.wdist = nullptr;  // set by launch_assign on the wide path (after np8_wide_dist)
    A.queue = A.queue_out = A.qcount = A.qlist = nullptr;
    A.slot_mu = c->slot_mu;
    A.slot_c = c->slot_c;
    A.slot_iso = c->slot_iso;
    A.slot_logn1 = c->slot_logn1;
    A.plen_s = c->plen_s;
    A.plr2_s = c->plr2_s;
    A.llpart = c->llpart;
    A.gp0 = c->Gp[0];
    A.z_best = c->z_best;
    A.cnt_best = c->cnt_best;
    A.mu_best = c->mu_best;
    A.sigma_best = c->sigma_best;
    A.cnt = c->cnt;
    A.slot_sigma = c->slot_sigma;
    return A;
}

PruneArgs prune_args(np8_ctx *c, bool last);
int launch_prune(np8_ctx *c, bool last);

SnapArgs snap_args(np8_ctx *c) {
    SnapArgs S;
    S.ctl = c->ctl;
    S.L = &c->ctl->L;
    S.best = c->ctl->best;
    S.have_best = &c->ctl->have_best;
    S.par = c->checks & 1;
    S.z = c->z;
    S.cnt = c->cnt;
    S.z_best = c->z_best;
    S.cnt_best = c->cnt_best;
    S.slot_mu = c->slot_mu;
    S.slot_sigma = c->slot_sigma;
    S.mu_best = c->mu_best;
    S.sigma_best = c->sigma_best;
    S.n_loc = c->n_loc;
    S.kcap = c->kcap;
    S.D = c->D;
    return S;
}

// A snapshot the folded check may have left for the next np8_assign_fast: copied now, before anything else reads
// or changes the labelling (every entry point but the data-parallel sweep's own continuation).
// z_best in item order (np8_assign_fast copies it in label-sorted position order; the layout's ids map it back)
int best_item_order(np8_ctx *c) {
    if (!c->z_best || !c->zs[1] || !c->ids[0] || c->n_loc <= 0) return NP8_OK;
    HIPC(c, np8_launch_best_unsort(c->ctl, c->ids[0], c->z_best, c->zs[1], c->n_loc, c->stream));
    return NP8_OK;
}

int flush_snapshot(np8_ctx *c) {
    if (c->snap_lazy) {
        c->snap_lazy = false;
        HIPC(c, np8_launch_snapshot_flush(snap_args(c), c->ctl, c->stream));
        HIPC(c, np8_launch_ctl_clear(c->ctl, 1, c->stream));  // snap_pend (not while a compact graph is halted)
    }
    return best_item_order(c);  // (every reader of z_best comes through here)
}

// prune: -1 none; 0 / 1 the candidate lists right after finalize, in the same launch (np8_step_tail), as
// launch_prune(c, false / true) would build them -- the frozen reference-prior sweep, where nothing changes the
// table between the two.
int launch_finalize(np8_ctx *c, const unsigned char *recs, int world, int prune = -1) {
    Timer t;
    timer_begin(c, 1, t);
    FinArgs F = fin_args(c, recs, world);
    // the one-workgroup tail (finalize + lists) on the sweeps that do not gather radii: a gathering sweep's fold
    // needs every assign record, i.e. a multi-workgroup launch whose last workgroup would run the serial part
    // behind agent-scope fences (their L2 writeback costs more than the dispatch it saves, §5)
    // the conditional form (the default): the lists of the last build stay when finalize finds every count within
    // kListSlack of it -- the frozen reference-prior sweep's step with valid lists; a rebuild then costs the one
    // workgroup what np8_prune does in parallel, so steps after which the lists are stale anyway keep np8_prune
    const bool cond = !c->tailcond_off && !c->churn && prune >= 0 && !c->gather && !c->wide && !c->rt &&
                      c->prior == NP8_PRIOR_REFERENCE && c->param_update == NP8_PARAM_FROZEN && c->lists_valid;
    const bool tail = cond || (!c->fuse_off && prune >= 0 && !c->gather && !c->wide && !c->rt && c->prior == NP8_PRIOR_REFERENCE);
    if (tail) {  // finalize (+ lists) in one launch
        TailArgs T;
        std::memset(&T, 0, sizeof(T));
        T.fold = 0;
        T.fold_n = c->assign_waves;
        T.fin = 1;
        PruneArgs P;
        std::memset(&P, 0, sizeof(P));
        if (prune >= 0) {
            P = prune_args(c, prune == 1);
            T.prune = cond ? 2 : 1;
            F.slack_test = cond ? 1 : 0;
            if (cond) (c->capturing ? c->cap_tail : c->n_tail_cond) += 1;
        }
        AssignArgs A = assign_args(c, 0, 0, nullptr, false);  // the radius records (wr2)
        HIPC(c, np8_launch_step_tail(A, F, P, T, c->assign_waves, c->D, c->M, c->stream));
        if (prune >= 0) c->lists_valid = true;
        timer_end(c, t);
        return NP8_OK;
    }
    if (c->gather)  // the step's radius records (any order with finalize: both only raise the gathered radii)
        HIPC(c, np8_launch_fold_r2(c->wr2, c->assign_waves, c->r2, c->kcap, c->ctl, c->stream));
    if (prune >= 0 && !c->fp_off && !c->wide && !c->rt && c->prior == NP8_PRIOR_REFERENCE) {
        // finalize and the lists in one launch, the lists still one per wave over several workgroups
        PruneArgs P = prune_args(c, prune == 1);
        HIPC(c, np8_launch_fin_prune(F, P, c->stream));
        c->lists_valid = true;
        timer_end(c, t);
        return NP8_OK;
    }
    HIPC(c, np8_launch_finalize(F, c->stream));
    if (F.frame_payload && c->prior != NP8_PRIOR_NIW) HIPC(c, np8_launch_frame_slots(F, c->stream));
    if (c->prior == NP8_PRIOR_NIW) {  // the accepted auxiliaries' full parameters
        NiwArgs A = niw_args(c);
        A.recs = recs;
        A.pend = c->pend;
        HIPC(c, np8_launch_niw_aux_slots(A, c->stream));
    }
    int r = refresh_wide(c, false);  // the slots created here
    if (r) return r;
    if (F.ll_defer)  // the folded check's accepted requesters under their new slots, then the decision
        HIPC(c, np8_launch_ll_fix_wide(wide_args(c), reinterpret_cast<const float *>(c->Xs[0]), c->n_loc, c->cand,
                                       c->dense_of, c->slot_c, c->pend, c->pend_ll, c->ctl->best, &c->ctl->have_best,
                                       c->checks & 1, c->ctl, c->stream));
    if (prune >= 0) {  // the lists the caller asked for (a gathering sweep, or the tail switched off)
        r = launch_prune(c, prune == 1);
        if (r) return r;
    }
    timer_end(c, t);
    return NP8_OK;
}

// Empty record: rebuild the candidate table from the slot arrays (after host uploads).  Only the header
// and the deltas are read (requests up to the header's count).
int rebuild(np8_ctx *c) {
    HIPC(c, hipMemsetAsync(c->rec, 0, kRecHeaderBytes + 4ull * c->kcap, c->stream));
    if (c->stage) HIPC(c, hipMemsetAsync(c->stage, 0, kRecHeaderBytes, c->stream));
    return launch_finalize(c, c->rec, 1);
}

int launch_assign(np8_ctx *c, int64_t p0, int64_t p1, const int64_t *order, bool use_perm) {
    Timer t;
    timer_begin(c, 0, t);
    AssignArgs A = assign_args(c, p0, p1, order, use_perm);
    A.collect_r2 = c->gather ? 1 : 0;
    A.use_lists = (c->collecting && c->lists_valid) ? 1 : 0;
    c->assign_waves = (p1 - p0 + 63) / 64;
    // the fast kernel over the whole sweep, every row isotropic: it can fold the max-likelihood check in (frozen
    // parameters: the labels after the step are what the check scores) and take a pending snapshot along
    const bool fast = !c->wide && !c->rt && c->diag_U && !c->fast_off && c->prior == NP8_PRIOR_REFERENCE && A.sorted && !order &&
                      !use_perm;
    const bool whole = fast && c->substeps == 1 && p0 == 0 && p1 == c->n_loc && c->rows_iso && !A.count_eval &&
                       !c->queue_on && (c->world == 1 || c->comm) && !c->host_exch_step;
    // the wide path folds it too (one rank, the whole step on the label-sorted layout, a diagonal base-measure frame):
    // np8_ll_fix_wide completes the sum once the accepted requests' slots exist
    // On by default since the per-item frame and the fp16 screen (late round 5): C5 frozen 4 312-4 323 sweeps/s folded
    // vs 4 091-4 122 with the separate np8_loglik_wide_mfma pass (0.09 ms every 5th sweep), A/B on one box; before them
    // the folded instance lost (3 543 vs 3 649).  NP8_WIDE_LLFOLD=0 keeps the separate pass (tests/test_gpu_fold.py
    // compares the two).
    const bool wide_fold = c->wide_llfold && c->wide && c->diag_U && c->substeps == 1 && p0 == 0 && p1 == c->n_loc &&
                           !order && !use_perm && A.sorted && c->world == 1 && !c->comm && !A.count_eval;
    c->step_ll = (whole || wide_fold) && !c->llfold_off && c->param_update == NP8_PARAM_FROZEN &&
                 (wide_fold || c->gp_iso > 0.0) && c->epoch % 5u == 0u && c->llpart;
    if (c->snap_lazy && (!whole || c->step_ll)) {  // (a check sweep never follows a check sweep)
        int r = flush_snapshot(c);
        if (r) return r;
    }
    c->step_snap = c->snap_lazy;  // consumed by this step's assign, cleared by its finalize
    c->snap_lazy = false;
    A.ll_on = c->step_ll ? 1 : 0;
    A.snap_on = c->step_snap ? 1 : 0;
    // compact exchange: a whole frozen step of a captured sharded graph with the folded check (every kernel such a
    // graph holds does nothing once a step halts it)
    c->compact_step = (whole && c->comm && c->capturing && c->compact_on && c->crec && c->fp_off &&
                       c->param_update == NP8_PARAM_FROZEN && !c->llfold_off && c->gp_iso > 0.0 && c->llpart) ||
                      c->host_compact;  // (np8_step_local_compact checked that the lean kernel takes every lane)
    if (c->compact_step) {
        A.compact = 1;
        A.rec = c->crec;  // the count deltas; requests to the staging area and the first c_cap also to crec
        A.nreq = &reinterpret_cast<RecHeader *>(c->crec)->nreq;
        A.creq = reinterpret_cast<Request *>(c->crec + kRecHeaderBytes + 4ll * c->kcap);
        A.cvmu = reinterpret_cast<double *>(c->crec + record_vmu_offset(c->kcap, c->c_cap));
        A.ccap = c->c_cap;
    }
    if (c->wide) {
        if (c->wdist && !c->wide_prune_off) {  // distances between the current rows' means (pruning)
            HIPC(c, np8_launch_wide_dist(wide_args(c), c->stream));
            A.wdist = c->wdist;
        }
        HIPC(c, np8_launch_assign_wide(A, c->D, c->M, c->prior, c->stream));
    }
    else if (!c->rt && c->diag_U && !c->fast_off && c->prior == NP8_PRIOR_REFERENCE && A.sorted && !order && !use_perm) {
        // the lean kernel for every lane, then the full one over the lanes it deferred (ctl->qn)
        A.queue_out = c->queue;
        A.qcount = c->qcount;
        A.qlist = c->qlist;
        A.no_queue = (c->rows_iso && !A.count_eval && !c->queue_on) ? 1 : 0;
        HIPC(c, np8_launch_assign_fast(A, c->D, c->M, c->stream));
        if (!A.no_queue) {
            A.queue = c->queue;
            A.queue_out = nullptr;
            HIPC(c, np8_launch_assign_queue(A, c->D, c->M, c->stream));  // a small grid walking ctl->qwaves
        }
    } else {
        HIPC(c, np8_launch_assign(A, c->D, c->M, c->prior, c->stream));
    }
    timer_end(c, t);
    return NP8_OK;
}

// Candidate lists for the next sweep from the radii this sweep collected (after every change of
// the table: finalize and the parameter update).
PruneArgs prune_args(np8_ctx *c, bool last) {
    PruneArgs P;
    P.cand = c->cand;
    P.ctl = c->ctl;
    P.r2 = c->r2;
    P.plist = c->plist;
    P.pdist = c->pdist;
    P.plen = c->plen;
    P.plr2 = c->plr2;
    P.plen_s = c->plen_s;
    P.plr2_s = c->plr2_s;
    P.ls = c->kcap;
    P.D = c->D;
    P.kcap = c->kcap;
    P.lb = c->lb;
    // eigenvalue bounds for rows that are not isotropic: kept exact only while every slot's parameters come from an
    // upload or a G0 draw (reference prior, frozen parameters)
    P.lam = (c->prior == NP8_PRIOR_REFERENCE && c->param_update == NP8_PARAM_FROZEN) ? c->slot_lam : nullptr;
    P.gathered = (last && c->gather) ? 1 : 0;
    // the next sweep gathers: clear its buffer here instead of with a memset node at its start (a stale
    // buffer would only raise radii: pruning stays exact)
    P.clear_next = (last && !P.gathered && c->r2_zero && (c->epoch + 1) % kGatherEvery == kGatherPhase) ? 1 : 0;
    c->gath_clear = P.clear_next != 0;
    return P;
}

int launch_prune(np8_ctx *c, bool last) {
    PruneArgs P = prune_args(c, last);
    HIPC(c, np8_launch_prune(P, c->kcap, c->stream));
    c->lists_valid = true;
    return NP8_OK;
}

// Label-sorted layout for the synchronous sweep: rebuilt from the item-order arrays when stale
// (after a state upload or a chunked / per-item step), refreshed from itself every resort_every
// sweeps so that items that moved cluster rejoin their group.
int launch_resort(np8_ctx *c, bool stale) {
    SortArgs S;
    S.X = c->X;
    S.z = c->z;
    for (int b = 0; b < 2; ++b) {
        S.Xs[b] = c->Xs[b];
        S.zs[b] = c->zs[b];
        S.ids[b] = c->ids[b];
    }
    S.hist = c->s_hist;
    S.cursor = c->s_cursor;
    S.off = c->s_off;
    S.ctl = c->ctl;
    S.n = c->n_loc;
    S.kcap = c->kcap;
    S.D = c->D;
    S.esz = c->wide ? 4 : 8;
    if (c->wide) S.D = c->DT + kFrameRows;  // (the wide path's item rows: DT, zero beyond D, then the item's frame)
    S.nsub = c->substeps;
    S.pad = 0;
    S.offset = c->offset;
    S.seed = c->seed;
    S.force = stale ? 1 : 0;  // otherwise the device re-sorts only if > n/32 items moved
    int r = best_item_order(c);  // (a snapshot in position order needs the ids it was taken under)
    if (r) return r;
    HIPC(c, np8_launch_resort(S, c->stream));
    c->sorted_valid = true;
    return NP8_OK;
}

int prepare_sorted(np8_ctx *c) {
    const bool stale = !c->sorted_valid;
    // sweeps launched one by one (the cold start's): re-sort as soon as a quarter of the items moved since the last sort
    // (the host-mapped count of the last finalize; the device re-checks) -- after init_random(20) the first sweeps move
    // half the items each, and a layout sorted for 20 clusters sends every wave through several groups' walks
    // (cold start 1 141 -> 1 358 sweeps/s measured with a re-sort every second sweep; graphs keep the cadence)
    if (!stale && !c->capturing && c->moved_host && (*(volatile int64_t *)c->moved_host) * 4 > c->n_loc)
        return launch_resort(c, false);
    if (!stale && c->epoch % (c->churn ? c->churn_resort : c->resort_every) != 0) return NP8_OK;
    if (!stale && c->capturing && c->capture_sort_outside) return NP8_OK;  // (np8_sweep re-sorts between replays)
    return launch_resort(c, stale);
}

// np8_sweep before a graph replay: the device's own check (> n/32 items moved since the last sort)
int prepare_sorted_now(np8_ctx *c) { return launch_resort(c, !c->sorted_valid); }

// One synchronous step over local positions [p0,p1): assign, exchange, finalize.  A whole-sweep
// step (no order, no permutation) runs on the label-sorted layout.
// One synchronous step.  sub >= 0: sub-step `sub` of a data-parallel sweep (positions of the label-sorted
// layout); otherwise local positions [p0,p1) of the chunked or explicit-order walk, and the whole
// data-parallel sweep when [p0,p1) = [0,n) with no order (substeps == 1).
int step_finish(np8_ctx *c, int sub);

int step(np8_ctx *c, int64_t p0, int64_t p1, const int64_t *order, bool use_perm, int sub = -1) {
    if (sub >= 0) {
        p0 = c->sub_start[(size_t)sub];
        p1 = c->sub_start[(size_t)sub + 1];
    }
    c->use_sorted = sub >= 0 || ((order == nullptr) && !use_perm && p0 == 0 && p1 == c->n_loc && c->n_loc > 0);
    if (c->use_sorted) {
        if (sub <= 0) {  // the layout is refreshed at the start of a sweep only
            int r = prepare_sorted(c);
            if (r) return r;
        }
    } else {
        c->sorted_valid = false;
    }
    // candidate pruning runs on data-parallel sweeps; any other step changes the membership behind the
    // lists' back
    c->collecting = c->prune_on && c->use_sorted;
    if (!c->use_sorted) c->lists_valid = c->r2_zero = false;
    if (c->collecting && sub <= 0) {  // the start of a data-parallel sweep: gather radii on this one?
        c->gather = !c->r2_zero || c->epoch % kGatherEvery == kGatherPhase;
        const bool cleared = c->gath_clear && c->r2_zero;  // by the previous sweep's prune
        c->gath_clear = false;
        if (!c->r2_zero) {  // no radii yet: every lane walks the table until the first gathered sweep ends
            HIPC(c, hipMemsetAsync(c->r2, 0, sizeof(double) * c->kcap, c->stream));
            c->r2_zero = true;
        }
        if (c->gather && !cleared) {
            if (c->capturing && c->comm)  // a sharded graph: a later sweep of a halted replay must not clear them
                HIPC(c, np8_launch_clear_unless_halted(c->r2 + c->kcap, c->kcap, c->ctl, c->stream));
            else
                HIPC(c, hipMemsetAsync(c->r2 + c->kcap, 0, sizeof(double) * c->kcap, c->stream));
        }
    }
    int r = launch_assign(c, p0, p1, order, use_perm);
    if (r) return r;
    if (c->world > 1 && !c->comm) return fail(c, NP8_ERR_STATE, "host-exchange mode: use np8_step_local/np8_step_merge");
    return step_finish(c, sub);
}

// The rest of a synchronous step after its assign: the exchange (RCCL: compact or full records) and finalize, the
// candidate lists.  Also the resumption of a halted compact step (recover_halt), with the full records.
int step_finish(np8_ctx *c, int sub) {
    int r = 0;
    // the lists right after finalize (np8_step_tail) when nothing changes the table in between: the next sub-step's
    // (radii in use), or the sweep's when its parameters are frozen (end_sweep's prune)
    const bool mid = sub >= 0 && sub + 1 < c->substeps;
    const int fprune = (c->collecting && (!c->fuse_off || !c->fp_off || !c->tailcond_off) && !c->wide &&
                        c->prior == NP8_PRIOR_REFERENCE &&
                        (mid || c->param_update == NP8_PARAM_FROZEN)) ? (mid ? 0 : 1) : -1;
    if (c->comm && c->compact_step) {  // a step of a compact sweep graph (np8_sweep)
        if (c->capturing) {  // where a replay halted at this step resumes
            HostSnap h;
            h.di = c->cap_sweep;
            h.dchecks = c->checks - c->cap_checks0;
            h.dfolded = c->cap_folded;
            h.dtail = c->cap_tail;
            h.assign_waves = c->assign_waves;
            h.step_ll = c->step_ll;
            h.step_snap = c->step_snap;
            h.sweep_ll = c->sweep_ll;
            h.snap_lazy = c->snap_lazy;
            h.collecting = c->collecting;
            h.gather = c->gather;
            h.lists_valid = c->lists_valid;
            h.r2_zero = c->r2_zero;
            h.gath_clear = c->gath_clear;
            h.pruned_last = c->pruned_last;
            h.use_sorted = c->use_sorted;
            h.sorted_valid = c->sorted_valid;
            h.churn = c->churn;
            c->cap_snaps.push_back(h);
        }
        if (c->step_ll) HIPC(c, np8_launch_ll_header(c->ctl, c->llpart, c->assign_waves, c->crec, c->stream));
        NCCLC(c, ncclAllGather(c->crec, c->cgath, (size_t)c->c_bytes, ncclUint8, c->comm, c->stream));
        r = launch_finalize(c, c->cgath, c->world, fprune);
        c->compact_step = false;
    } else if (c->comm) {  // the exchange over RCCL (also with a one-rank communicator)
        HIPC(c, np8_launch_req_select(c->stage, c->stage_cap, c->rec, c->rec_cap, c->kcap, c->D, c->req_max,
                                      c->step_ll ? c->llpart : nullptr, c->assign_waves, c->stream));
        NCCLC(c, ncclAllGather(c->rec, c->gath, (size_t)c->rec_bytes, ncclUint8, c->comm, c->stream));
        r = launch_finalize(c, c->gath, c->world, fprune);
    } else {
        r = launch_finalize(c, c->rec, 1, fprune);
    }
    c->sweep_ll = c->sweep_ll || c->step_ll;
    c->step_ll = c->step_snap = false;
    if (r) return r;
    if (fprune >= 0) {
        c->pruned_last = fprune == 1;
        return NP8_OK;
    }
    if (c->collecting && mid)
        return launch_prune(c, false);  // lists for the next sub-step (the radii in use)
    // the table changed: lists are valid again after the next prune (end of sweep or of a sub-step)
    c->lists_valid = false;
    return NP8_OK;
}

// The population update of one sweep (np_mcmc.cpp:146-164): chunks of `chunk` items in a keyed permutation,
// or the data-parallel sweep -- one synchronous step, or `substeps` of them.
int population(np8_ctx *c) {
    const int64_t N = c->n_loc;
    const int64_t chunk = (c->chunk <= 0 || c->chunk >= c->n_glob) ? N : c->chunk;
    const bool sync = chunk >= N;
    if (!sync && c->world > 1) return fail(c, NP8_ERR_ARG, "chunk < N is single-rank only");
    if (sync && c->substeps > 1) {
        for (int k = 0; k < c->substeps; ++k) {
            int r = step(c, 0, 0, nullptr, false, k);
            if (r) return r;
        }
        return NP8_OK;
    }
    if (N > 0) {
        for (int64_t p0 = 0; p0 < N; p0 += chunk) {
            const int64_t p1 = (p0 + chunk < N) ? p0 + chunk : N;
            int r = step(c, p0, p1, nullptr, !sync);
            if (r) return r;
        }
    } else if (c->comm) {
        return step(c, 0, 0, nullptr, false);  // still take part in the exchange
    }
    return NP8_OK;
}

int ensure_partial(np8_ctx *c) {
    const int64_t nb = (c->n_loc + 255) / 256;
    if (nb > c->partial_cap) {
        int r = dalloc(c, &c->partial, (size_t)nb);
        if (r) return r;
        c->partial_cap = nb;
    }
    return NP8_OK;
}

// sum_i log p(x_i | theta_{z_i}) into ctl->L (global when sharded over RCCL).
int launch_total_loglik(np8_ctx *c) {
    int r = ensure_partial(c);
    if (r) return r;
    Timer t;
    timer_begin(c, 2, t);
    LoglikArgs A;
    A.X = c->X;
    A.z = c->z;
    A.cand = c->cand;
    A.dense_of = c->dense_of;
    A.partial = c->partial;
    A.n_loc = c->n_loc;
    if (c->wide) {  // the own-cluster MFMA passes, on the label-sorted layout after a synchronous sweep
        AssignArgs W = assign_args(c, 0, c->n_loc, nullptr, false);
        W.sorted = (c->use_sorted && c->sorted_valid) ? 1 : 0;
        HIPC(c, np8_launch_loglik_wide_mfma(W, c->D, c->partial, c->stream));
    } else
        HIPC(c, np8_launch_loglik(A, c->D, c->stream));
    const bool sum_ranks = c->comm != nullptr;
    HIPC(c, np8_launch_loglik_reduce(c->partial, (c->n_loc + 255) / 256, &c->ctl->L_local,
                                     sum_ranks ? nullptr : &c->ctl->L, c->stream));
    if (sum_ranks) NCCLC(c, ncclAllReduce(&c->ctl->L_local, &c->ctl->L, 1, ncclFloat64, ncclSum, c->comm, c->stream));
    timer_end(c, t);
    return NP8_OK;
}

// UpdateClusters::update (np_mcmc.cpp:170) in mh_g0 mode: statistics of the current labelling
// (summed over ranks), then one MH chain per live slot; candidate rows are patched in place.
// stats_mode: 0 = compute the statistics (+ RCCL all-reduce when sharded) and update; 1 = compute the
// local statistics only (np8_param_stats_local); 2 = update from the statistics already placed in acc
// (np8_end_sweep_stats).
int param_update(np8_ctx *c, int stats_mode = 0) {
    if (c->param_update == NP8_PARAM_FROZEN) return NP8_OK;
    if (stats_mode == 0 && c->world > 1 && !c->comm)
        return fail(c, NP8_ERR_STATE,
                    "the parameter update needs the RCCL transport when sharded (or np8_param_stats_local / "
                    "np8_end_sweep_stats)");
    Timer t;
    timer_begin(c, 3, t);
    ParamArgs A;
    A.X = c->X;
    A.z = c->z;
    const bool sorted = c->use_sorted && c->sorted_valid;
    for (int b = 0; b < 2; ++b) {
        A.Xs[b] = c->Xs[b];
        A.zs[b] = c->zs[b];
    }
    A.sorted = sorted ? 1 : 0;
    A.n_loc = c->n_loc;
    A.kcap = c->kcap;
    A.D = c->D;
    A.DT = c->DT;
    A.steps = c->mh_steps;
    A.acc = c->acc;
    A.cnt = c->cnt;
    A.dense_of = c->dense_of;
    A.slot_mu = c->slot_mu;
    A.slot_P = c->slot_P;
    A.slot_c = c->slot_c;
    A.slot_sigma = c->slot_sigma;
    A.slot_iso = c->slot_iso;
    A.cand = c->cand;
    A.ctl = c->ctl;
    A.mu0 = c->d_mu0;
    A.LT = c->d_LT;
    A.Gp = c->d_Gp;
    A.LTL = c->d_LTL;
    A.caux = c->caux;
    A.rsk = c->rsk;
    A.nu = c->nu;
    A.gp_iso = c->gp_iso;
    A.seed = c->seed;
    A.t = c->epoch - c->t_base;
    A.r2 = c->r2;
    const size_t nacc = (size_t)c->kcap * (c->D + c->DP);
    // acc is all zero here: allocated zeroed, and np8_mh_g0 clears every row it reads (the only
    // rows np8_suffstats adds to are those of live slots)
    // one rank on the wide path: run records instead of atomics (the ranks' transports sum acc otherwise)
    const bool recs = c->wide && c->part && stats_mode == 0 && c->world == 1 && !c->comm &&
                      c->param_update == NP8_PARAM_NIW_CONJUGATE;
    if (recs) {
        A.part = c->part;
        A.part_slot = c->part_slot;
    }
    if (stats_mode != 2) {
        if (c->wide)
            HIPC(c, np8_launch_suffstats_wide(A, c->stream));
        else
            HIPC(c, np8_launch_suffstats(A, c->stream));
    }
    if (stats_mode == 1) {
        timer_end(c, t);
        return NP8_OK;
    }
    if (stats_mode == 0 && c->comm)
        NCCLC(c, ncclAllReduce(c->acc, c->acc, nacc, ncclFloat64, ncclSum, c->comm, c->stream));
    if (c->param_update == NP8_PARAM_NIW_CONJUGATE) {
        NiwArgs N = niw_args(c);
        if (recs) {
            N.part = c->part;
            N.part_slot = c->part_slot;
            N.n_rec = c->part_waves * kSuffRuns;
        }
        HIPC(c, np8_launch_niw_post(N, c->kcap, c->stream));
    }
    else
        HIPC(c, np8_launch_mh_g0(A, c->stream));
    // every live slot's parameters changed; np8_niw_post wrote the contraction rows of the slots it drew (a slot it
    // could not draw keeps its parameters and rows), np8_mh_g0 leaves them to np8_wide_rows
    int r = refresh_wide(c, c->param_update != NP8_PARAM_NIW_CONJUGATE);
    if (r) return r;
    timer_end(c, t);
    return NP8_OK;
}

int launch_invariants(np8_ctx *c) {
    int r = 0;
    if (!c->inv_hist && ((r = dalloc(c, &c->inv_hist, (size_t)c->kcap)) || (r = dalloc(c, &c->inv_out, 4)))) return r;
    HIPC(c, np8_launch_invariants(c->z, c->n_loc, c->cnt, c->dense_of, c->cand, c->CS, c->D, c->kcap, c->n_glob,
                                  c->world == 1 ? 1 : 0, c->inv_hist, c->inv_out, c->ctl, c->stream));
    return NP8_OK;
}

int end_sweep(np8_ctx *c, bool stats_given = false) {
    int r0 = param_update(c, stats_given ? 2 : 0);
    if (r0) return r0;
    if (c->collecting) {  // after finalize and the parameter update: the table is final
        if (!c->pruned_last) {  // (unless the step's np8_step_tail built the lists already)
            r0 = launch_prune(c, true);
            if (r0) return r0;
        }
        c->collecting = c->gather = false;
    }
    c->pruned_last = false;
    if (c->debug_inv && (r0 = launch_invariants(c))) return r0;
    if (c->epoch % 5u == 0u) {  // np_mcmc.cpp:172-174
        if (c->sweep_ll) {  // folded into the step: decided by its finalize, copied by the next np8_assign_fast
            c->snap_lazy = true;
            (c->capturing ? c->cap_folded : c->n_folded) += 1;
        } else {
            int r = flush_snapshot(c);
            if (r) return r;
            r = launch_total_loglik(c);
            if (r) return r;
            HIPC(c, np8_launch_snapshot(snap_args(c), c->stream));
        }
        c->checks += 1;
    }
    c->sweep_ll = false;
    c->epoch += 1;
    return NP8_OK;
}

int reset_ctl(np8_ctx *c) {
    Ctl h;
    std::memset(&h, 0, sizeof(h));
    h.best[0] = h.best[1] = -INFINITY;
    HIPC(c, hipMemcpyAsync(c->ctl, &h, sizeof(h), hipMemcpyHostToDevice, c->stream));
    c->epoch = 0;
    c->checks = 0;
    c->t_base = 0;
    return NP8_OK;
}

int read_ctl(np8_ctx *c, Ctl *h) {
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipMemcpy(h, c->ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
    return NP8_OK;
}

// ---- sweep graphs ---------------------------------------------------------------------------------
// A synchronous single-rank sweep is a fixed sequence of launches whose only per-sweep inputs are
// the epoch (read on the device as ctl->t_base + offset), the re-sort cadence (epoch % 4) and the
// max-likelihood cadence and parity (epoch % 5, check count).  kGraphSweeps = 20 sweeps therefore
// repeat exactly: they are captured once into a hipGraph and replayed, which removes the host
// launch gaps between kernels (≈6 µs each).  The graph ends with np8_advance_epoch (t_base += 20).
constexpr uint32_t kGraphSweeps = 20;

void drop_graph(np8_ctx *c) {
    if (c->graph) (void)hipGraphExecDestroy(c->graph);
    if (c->graph_tmpl) (void)hipGraphDestroy(c->graph_tmpl);
    c->graph = nullptr;
    c->graph_tmpl = nullptr;
    c->graph_timers.clear();
    c->graph_par = c->graph_phase = -1;
}

// The next sharded graph's records: compact (policy, alike on every rank) or full.
bool want_compact(const np8_ctx *c) { return c->comm && c->crec && c->compact_on; }

bool graph_eligible(np8_ctx *c, bool sync) {
    // sharded runs are captured with their RCCL collectives; the host-exchange path is not (host transport)
    return sync && !c->graphs_off && (c->world == 1 || c->comm) && c->n_loc > 0 && c->sorted_valid &&
           (!c->prune_on || (c->lists_valid && c->r2_zero));
}

// Captures kGraphSweeps sweeps starting at the current epoch.  Nothing runs during capture; on any
// failure the context falls back to launching sweeps one by one (graphs_off).
int capture_graph(np8_ctx *c) {
    drop_graph(c);
    int r = ensure_partial(c);  // no allocation inside the capture
    if (r) return r;
    const uint32_t e0 = c->epoch;
    const int32_t ch0 = c->checks;
    if (c->t_base != e0) {
        HIPC(c, hipMemsetD32Async(reinterpret_cast<int *>(&c->ctl->t_base), (int)e0, 1, c->stream));
        c->t_base = e0;
    }
    if (hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        c->graphs_off = true;
        return NP8_OK;
    }
    c->capturing = true;
    c->capture_timed_left = c->time_all ? (int)kGraphSweeps * c->substeps : 1;
    const bool snap0 = c->snap_lazy;
    c->cap_folded = c->cap_tail = 0;
    // the epoch advance in the last step's finalize when nothing after it reads t_base (frozen reference-prior sweep
    // of one step); otherwise np8_advance_epoch ends the graph
    const bool adv_fin = c->substeps == 1 && c->param_update == NP8_PARAM_FROZEN && !c->wide &&
                         c->prior == NP8_PRIOR_REFERENCE;
    c->fin_advanced = false;
    // the re-sort check leaves the graph when its last finalize mirrors ctl->moved for the host (np8_sweep)
    c->capture_sort_outside = adv_fin && !c->sort_in_graph && !c->churn && c->moved_dev != nullptr;
    c->graph_churn = c->churn;
    c->cap_snaps.clear();
    c->cap_checks0 = ch0;
    const bool cmode = want_compact(c);
    for (uint32_t i = 0; i < kGraphSweeps && !r; ++i) {
        if (adv_fin && i + 1 == kGraphSweeps) c->fin_advance = kGraphSweeps;
        c->cap_sweep = i;
        r = population(c);
        if (!r) r = end_sweep(c);
    }
    c->compact_step = false;
    c->fin_advance = 0;
    const bool snap1 = c->snap_lazy;
    c->snap_lazy = snap0;
    if (!r && !c->fin_advanced && np8_launch_advance_epoch(c->ctl, kGraphSweeps, c->stream) != hipSuccess)
        r = NP8_ERR_HIP;
    c->fin_advanced = false;
    hipGraph_t g = nullptr;
    const hipError_t ee = hipStreamEndCapture(c->stream, &g);
    c->capturing = false;
    c->epoch = e0;  // nothing has run yet
    c->checks = ch0;
    hipGraphExec_t exec = nullptr;
    if (!r && ee == hipSuccess && g && hipGraphInstantiate(&exec, g, nullptr, nullptr, 0) == hipSuccess) {
        c->graph = exec;
        c->graph_tmpl = g;
        g = nullptr;
        c->graph_par = ch0 & 1;
        c->graph_phase = (int)(e0 % kGraphSweeps);
        c->graph_snap0 = snap0;
        c->graph_snap1 = snap1;
        c->graph_sort_outside = c->capture_sort_outside;
        c->graph_folded = c->cap_folded;
        c->graph_tail = c->cap_tail;
        c->graph_compact = cmode;
        c->graph_snaps = c->cap_snaps;
        c->graph_timing = (c->timing ? 1 : 0) | (c->count_eval ? 2 : 0) | (c->time_all ? 4 : 0);
    } else {
        c->graph_timers.clear();
        c->graphs_off = true;
        (void)hipGetLastError();
    }
    if (g) (void)hipGraphDestroy(g);
    return NP8_OK;
}

// The graph for the sweeps starting at the current epoch (captured when missing or captured at another
// phase, check parity or timing setting).
bool graph_current(const np8_ctx *c) {
    return c->graph && c->graph_par == (c->checks & 1) && c->graph_phase == (int)(c->epoch % kGraphSweeps) &&
           c->graph_snap0 == c->snap_lazy && c->graph_churn == c->churn && c->graph_compact == want_compact(c) &&
           c->graph_timing == ((c->timing ? 1 : 0) | (c->count_eval ? 2 : 0) | (c->time_all ? 4 : 0));
}

int ensure_graph(np8_ctx *c) {
    if (!graph_current(c)) return capture_graph(c);
    return NP8_OK;
}

int run_graph(np8_ctx *c) {
    if (c->t_base != c->epoch) {  // the graph's epoch offsets are 0 .. kGraphSweeps-1
        HIPC(c, hipMemsetD32Async(reinterpret_cast<int *>(&c->ctl->t_base), (int)c->epoch, 1, c->stream));
        c->t_base = c->epoch;
    }
    std::vector<Timer> sampled;
    for (const Timer &g : c->graph_timers) {  // fresh events for this replay, collected lazily
        if (c->timers.size() + sampled.size() + 1 >= 4096) collect_timers(c);
        Timer t = g;
        pool_pair(c, c->timers.size() + sampled.size(), t);
        HIPC(c, hipGraphExecEventRecordNodeSetEvent(c->graph, g.na, t.a));
        HIPC(c, hipGraphExecEventRecordNodeSetEvent(c->graph, g.nb, t.b));
        sampled.push_back(t);
    }
    HIPC(c, hipGraphLaunch(c->graph, c->stream));
    for (const Timer &t : sampled) c->timers.push_back(t);
    c->snap_lazy = c->graph_snap1;
    c->n_folded += c->graph_folded;
    c->n_tail_cond += c->graph_tail;
    c->epoch += kGraphSweeps;
    c->checks += (int32_t)(kGraphSweeps / 5);
    c->t_base += kGraphSweeps;
    return NP8_OK;
}

// A compact replay halted at step i (every rank alike, np8_finalize): the host state of that step as its capture left
// it after the assign, then the step's exchange with the full records -- the deltas the assign wrote into the compact
// record and every request of the staging area -- and the rest of the sweep.  The halted replay's later kernels did
// nothing, as did a replay queued behind it; the chain continues from the resumed step as if nothing had halted.
// finish: then run the sweeps the host had already counted (up to the epoch it had reached) -- np8_sweep's own loop
// does that itself (it continues to its target), every other entry point needs them done before it reads the state.
int recover_halt(np8_ctx *c, bool finish) {
    const uint32_t reached = c->epoch;
    HIPC(c, hipStreamSynchronize(c->stream));
    const uint32_t i = (uint32_t)*(volatile int32_t *)&c->mirror_host[1];
    const HostSnap *hp = nullptr;
    for (const HostSnap &h : c->graph_snaps)
        if (h.di == i) hp = &h;
    if (!hp) return fail(c, NP8_ERR_STATE, "a compact sweep graph halted at a step without its host state");
    const HostSnap &h = *hp;
    c->epoch = c->pend_epoch + h.di;
    c->checks = c->pend_checks + h.dchecks;
    c->n_folded = c->pend_folded + h.dfolded;
    c->n_tail_cond = c->pend_tail + h.dtail;
    c->t_base = c->pend_epoch;  // (the halted replay's last finalize did not advance the device's)
    c->assign_waves = h.assign_waves;
    c->step_ll = h.step_ll;
    c->step_snap = h.step_snap;
    c->sweep_ll = h.sweep_ll;
    c->snap_lazy = h.snap_lazy;
    c->collecting = h.collecting;
    c->gather = h.gather;
    c->lists_valid = h.lists_valid;
    c->r2_zero = h.r2_zero;
    c->gath_clear = h.gath_clear;
    c->pruned_last = h.pruned_last;
    c->use_sorted = h.use_sorted;
    c->sorted_valid = h.sorted_valid;
    c->churn = h.churn;
    c->fin_advance = 0;
    c->fin_advanced = false;
    c->compact_step = false;
    c->compact_on = false;  // full records until a replay's requests fit the compact ones again (np8_sweep)
    c->n_halts += 1;
    HIPC(c, hipMemsetD32Async(reinterpret_cast<int *>(&c->ctl->halt), 0, 1, c->stream));
    HIPC(c, hipMemsetD32Async(reinterpret_cast<int *>(&c->ctl->t_base), (int)c->t_base, 1, c->stream));
    c->mirror_host[0] = 0;
    HIPC(c, hipMemcpyAsync(c->rec + kRecHeaderBytes, c->crec + kRecHeaderBytes, 4ull * c->kcap, hipMemcpyDeviceToDevice,
                           c->stream));
    HIPC(c, hipMemcpyAsync(&reinterpret_cast<RecHeader *>(c->stage)->nreq, &reinterpret_cast<RecHeader *>(c->crec)->nreq,
                           sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
    HIPC(c, hipMemsetAsync(c->crec, 0, kRecHeaderBytes + 4ull * c->kcap, c->stream));
    int r = step_finish(c, -1);
    if (r) return r;
    if ((r = end_sweep(c))) return r;
    while (finish && (int32_t)(reached - c->epoch) > 0) {  // (full records: the policy switched them off)
        if ((r = population(c)) || (r = end_sweep(c))) return r;
    }
    return NP8_OK;
}

// The last replay of a sharded graph, once it is done: resumed if it halted (recover_halt); otherwise its requests'
// peak may bring compact records back (decided alike on every rank: the peak is a function of the gathered headers).
// finish: see recover_halt (false only from np8_sweep's loop).
int settle(np8_ctx *c, bool *recovered = nullptr, bool finish = true) {
    if (recovered) *recovered = false;
    if (!c->pend_on) return NP8_OK;
    c->pend_on = false;
    HIPC(c, hipEventSynchronize(c->rev[c->pend_k]));
    if (*(volatile int32_t *)&c->mirror_host[0]) {
        if (recovered) *recovered = true;
        return recover_halt(c, finish);
    }
    if (!c->compact_on && c->crec && !c->pend_compact && *(volatile int32_t *)&c->mirror_host[2] * 2 <= c->c_cap)
        c->compact_on = true;
    return NP8_OK;
}

}  // namespace

// =====================================================================================================
extern "C" {

int np8_create(np8_ctx **out, const np8_config *cfg) { return np8_create_sized(out, cfg, sizeof(np8_config)); }

int np8_create_sized(np8_ctx **out, const np8_config *cfg_in, size_t cfg_bytes) {
    if (!out || !cfg_in || cfg_bytes < NP8_CONFIG_MIN_BYTES) return NP8_ERR_ARG;
    *out = nullptr;
    // the caller's prefix only: fields it does not have keep their zero ("default") values
    np8_config cfg_copy;
    std::memset(&cfg_copy, 0, sizeof(cfg_copy));
    std::memcpy(&cfg_copy, cfg_in, cfg_bytes < sizeof(cfg_copy) ? cfg_bytes : sizeof(cfg_copy));
    const np8_config *cfg = &cfg_copy;
    np8_ctx *c = new np8_ctx();
    c->D = cfg->D;
    c->M = cfg->M;
    if (c->D < 1 || c->D > kMaxD || c->M < 1 || c->M > kMaxM || !cfg->mu0 || !cfg->Lambda || !(cfg->kappa > 0.0) ||
        !(cfg->alpha > 0.0)) {
        delete c;
        return NP8_ERR_ARG;
    }
    // F64 at a (D, M) without a templated instance (16 < D <= kMaxD, or a rarer M): the run-time-D kernels, reference
    // prior, frozen parameters
    const bool rt = cfg->contraction == NP8_CONTRACT_F64 && !np8_supported(c->D, c->M) &&
                    np8_rt_supported(c->D, c->M, kPriorReference) && cfg->prior == NP8_PRIOR_REFERENCE &&
                    cfg->param_update == NP8_PARAM_FROZEN;
    if (!np8_supported(c->D, c->M) && !rt &&
        !(cfg->contraction == NP8_CONTRACT_F32_MFMA && np8_wide_supported(c->D, c->M))) {
        delete c;
        return NP8_ERR_ARG;
    }
    c->rt = rt;
    c->DP = packed_size(c->D);
    c->DT = (cfg->contraction == NP8_CONTRACT_F32_MFMA) ? wide_dt(c->D) : c->D;
    c->CS = cand_stride(c->D);
    c->kcap = cfg->kcap > 0 ? cfg->kcap : (cfg->contraction == NP8_CONTRACT_F32_MFMA ? 512 : 2048);

    // np8_finalize keeps two int[kcap] arrays in dynamic LDS beside 64 KB of request space, plus its
    // static shared memory: the whole must fit gfx950's 160 KB
    if (np8_finalize_lds_bytes(c->kcap) + 1024 > 160 * 1024 || cfg->req_max < 0 || cfg->req_max > NP8_REQ_MAX) {
        delete c;
        return NP8_ERR_ARG;
    }
    c->req_max = cfg->req_max > 0 ? cfg->req_max : NP8_REQ_DEFAULT;
    c->substeps_auto = cfg->substeps == NP8_SUBSTEPS_AUTO;
    c->substeps = cfg->substeps > 1 ? cfg->substeps : 1;
    c->debug_inv = std::getenv("NP8_DEBUG_INVARIANTS") != nullptr && std::getenv("NP8_DEBUG_INVARIANTS")[0] == '1';
    // the label-sorted layout is sorted by (sub-step, slot): substeps * kcap bins in the sort's LDS
    if ((cfg->substeps < 0 && !c->substeps_auto) || cfg->substeps > NP8_SUBSTEPS_MAX || (int64_t)c->substeps * c->kcap > 16384) {
        delete c;
        return NP8_ERR_ARG;
    }
    c->alpha = cfg->alpha;
    c->kappa = cfg->kappa;
    c->nu = cfg->nu;
    c->seed = cfg->seed;
    c->chunk = cfg->chunk;
    if (cfg->param_update < NP8_PARAM_FROZEN || cfg->param_update > NP8_PARAM_NIW_CONJUGATE || cfg->mh_steps < 0 ||
        cfg->mh_steps > 65536 || (cfg->prior != NP8_PRIOR_REFERENCE && cfg->prior != NP8_PRIOR_NIW)) {
        delete c;
        return NP8_ERR_ARG;
    }
    // mh_g0 proposes from the reference's G0; the conjugate update needs the NIW prior; the Bartlett
    // chi^2(nu0 - a), a < D, need nu0 >= D + 1 (Marsaglia-Tsang shape >= 1)
    const bool niw = cfg->prior == NP8_PRIOR_NIW;
    if ((niw && cfg->param_update == NP8_PARAM_MH_G0) || (!niw && cfg->param_update == NP8_PARAM_NIW_CONJUGATE) ||
        (niw && !(cfg->nu >= cfg->D + 1.0 && cfg->nu < 1e12)) ||
        // np8_niw_post holds four D x (D + 1) double matrices in LDS: at most D = 64
        (niw && cfg->contraction == NP8_CONTRACT_F32_MFMA && cfg->D > 64)) {
        delete c;
        return NP8_ERR_ARG;
    }
    c->prior = cfg->prior;
    c->contraction = cfg->contraction;
    c->wide = cfg->contraction == NP8_CONTRACT_F32_MFMA;
    if ((cfg->contraction != NP8_CONTRACT_F64 && !c->wide) ||
        (c->wide && (!np8_wide_supported(cfg->D, cfg->M) || cfg->param_update == NP8_PARAM_MH_G0))) {
        delete c;
        return NP8_ERR_ARG;
    }
    c->param_update = cfg->param_update;
    c->mh_steps = cfg->mh_steps > 0 ? cfg->mh_steps : 20;
    c->mu0.assign(cfg->mu0, cfg->mu0 + c->D);
    c->Lambda.assign(cfg->Lambda, cfg->Lambda + (size_t)c->D * c->D);
    if (!prepare_base(c)) {
        delete c;
        return NP8_ERR_ARG;
    }
    if (cfg->device >= 0) {
        c->device = cfg->device;
        if (hipSetDevice(c->device) != hipSuccess) {
            delete c;
            return NP8_ERR_HIP;
        }
    } else {
        (void)hipGetDevice(&c->device);
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return NP8_ERR_HIP;
    }
    c->own_stream = true;
    c->graphs_off = std::getenv("NP8_NO_GRAPH") != nullptr;  // A/B switch for launch-by-launch sweeps
    c->prune_on = !c->wide && c->kcap <= kPruneMaxKcap && std::getenv("NP8_NO_PRUNE") == nullptr;
    c->wide_prune_off = std::getenv("NP8_NO_PRUNE") != nullptr;
    c->fast_off = std::getenv("NP8_NO_FAST") != nullptr;
    {  // NP8_TRI_BOUND=0: every triadic merge walks (A/B of the merge bound)
        const char *tb = std::getenv("NP8_TRI_BOUND");
        c->tri_bound_off = tb != nullptr && tb[0] == '0';
    }
    {
        const char *fp = std::getenv("NP8_FINPRUNE");
        c->fp_off = !(fp != nullptr && fp[0] == '1');
    }
    c->fuse_off = std::getenv("NP8_FUSE") == nullptr;  // opt-in: measured slower than separate launches
    c->queue_on = std::getenv("NP8_QUEUE") != nullptr;
    c->tailcond_off = std::getenv("NP8_LISTS_ALWAYS") != nullptr;
    // the walk screen (np8_assign_fast): opt-in since the buffered pick of round 6 (mixed 137.6 vs 145.0 us per sweep
    // without it, profiles/r06/mixed_env_ab)
    c->walk_screen = std::getenv("NP8_WALK_SCREEN") && std::getenv("NP8_WALK_SCREEN")[0] == '1';
    if (const char *g = std::getenv("NP8_MAX_LIST_GROUPS")) c->max_groups = std::max(1, std::min(64, std::atoi(g)));
    c->sort_in_graph = std::getenv("NP8_SORT_IN_GRAPH") != nullptr;
    if (!c->sort_in_graph) {  // host-mapped mirror of ctl->moved (written by every finalize)
        if (hipHostMalloc((void **)&c->moved_host, sizeof(int64_t), hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void **)&c->moved_dev, c->moved_host, 0) != hipSuccess) {
            if (c->moved_host) (void)hipHostFree(c->moved_host);
            c->moved_host = c->moved_dev = nullptr;
            c->sort_in_graph = true;
        } else {
            *c->moved_host = 0;
        }
    }
    c->llfold_off = std::getenv("NP8_NO_LLFOLD") != nullptr;
    c->wide_llfold = !(std::getenv("NP8_WIDE_LLFOLD") != nullptr && std::getenv("NP8_WIDE_LLFOLD")[0] == '0');
    c->niw_valu = std::getenv("NP8_NIW_VALU") != nullptr;
    if (const char *cr = std::getenv("NP8_CHURN_RESORT")) {  // (A/B runs: 1, 2, 4, 5, 10 or 20)
        const int v = atoi(cr);
        if (v > 0 && 20 % v == 0) c->churn_resort = (uint32_t)v;
    }
    if (const char *cr = std::getenv("NP8_COMPACT_REQ")) c->c_cap = std::max(0, std::min(atoi(cr), c->req_max));
    if (hipHostMalloc((void **)&c->mirror_host, sizeof(int32_t) * kMirrorInts, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void **)&c->mirror_dev, c->mirror_host, 0) != hipSuccess) {
        if (c->mirror_host) (void)hipHostFree(c->mirror_host);
        c->mirror_host = c->mirror_dev = nullptr;
        c->c_cap = 0;  // (no mirror: no compact exchange)
    } else {
        for (int k = 0; k < kMirrorInts; ++k) c->mirror_host[k] = 0;
    }
    c->rec_cap = c->req_max;  // grown to the item count by np8_set_data (one rank)
    c->rec_bytes = record_bytes(c->kcap, (int)c->rec_cap, c->D);
    int r = 0;
    const int D = c->D, DP = c->DP, kc = c->kcap;
    if ((r = dalloc(c, &c->slot_mu, (size_t)kc * D)) || (r = dalloc(c, &c->slot_P, (size_t)kc * DP)) ||
        (r = dalloc(c, &c->slot_c, (size_t)kc)) || (r = dalloc(c, &c->slot_sigma, (size_t)kc * D * D)) ||
        (r = dalloc(c, &c->cnt, (size_t)kc)) || (r = dalloc(c, &c->cnt_best, (size_t)kc)) ||
        (r = dalloc(c, &c->mu_best, (size_t)kc * D)) || (r = dalloc(c, &c->sigma_best, (size_t)kc * D * D)) ||
        (r = dalloc(c, &c->cand, (size_t)kc * c->CS)) || (r = dalloc(c, &c->ctl, 1)) ||
        (r = dalloc(c, &c->dense_of, (size_t)kc)) || (r = dalloc(c, &c->slot_iso, (size_t)kc)) ||
        (r = dalloc(c, &c->slot_lam, 2 * (size_t)kc)) ||
        (r = dalloc(c, &c->slot_logn1, (size_t)kc)) || (r = dalloc(c, &c->plen_s, (size_t)kc)) ||
        (r = dalloc(c, &c->plr2_s, (size_t)kc)) ||
        (r = dalloc(c, &c->rec, (size_t)c->rec_bytes)) || (r = dalloc(c, &c->evalc, (size_t)10 * kEvalSlots)) ||
        (c->param_update != NP8_PARAM_FROZEN && (r = dalloc(c, &c->acc, (size_t)kc * (D + DP)))) ||
        (kc <= kPruneMaxKcap && ((r = dalloc(c, &c->r2, 2 * (size_t)kc)) || (r = dalloc(c, &c->plen, (size_t)kc)) ||
                                 (r = dalloc(c, &c->lb, 2 * (size_t)kc)) ||
                                (r = dalloc(c, &c->plr2, (size_t)kc)) ||
                                 (r = dalloc(c, &c->plist, (size_t)kc * kc)) || (r = dalloc(c, &c->pdist, (size_t)kc * kc))))) {
        free_device(c);
        delete c;
        return r;
    }
    // hyp: mu0 | UinvT packed | caux | rsk | logam | nu | LT packed | NIW sum-log bound
    std::vector<double> hyp;
    hyp.insert(hyp.end(), c->mu0.begin(), c->mu0.end());
    c->diag_U = true;
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) {
            hyp.push_back(c->UinvT[a * D + b]);
            if (b != a && c->UinvT[a * D + b] != 0.0) c->diag_U = false;
        }
    hyp.push_back(c->caux);
    hyp.push_back(c->rsk);
    hyp.push_back(c->logam);
    hyp.push_back(c->nu);
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) hyp.push_back(c->LT[a * D + b]);
    // NIW auxiliary screen (DESIGN.md "Auxiliary screen"): sum over a = 1..D-1 of log of the largest chi^2
    // value gamma_mt can return for nu0 - a degrees of freedom (its normals come from 32-bit uniforms:
    // |x| <= sqrt(-2 log 2^-33)), with a relative margin
    {
        double smax = 0.0;
        if (c->prior == NP8_PRIOR_NIW) {
            const double rmax = std::sqrt(-2.0 * std::log(std::ldexp(1.0, -33))) * (1.0 + 1e-9);
            for (int a = 1; a < D; ++a) {
                const double d = 0.5 * (c->nu - a) - 1.0 / 3.0, cc = 1.0 / std::sqrt(9.0 * d);
                const double v1 = 1.0 + cc * rmax;
                smax += std::log(2.0 * d * std::max(1.0, v1 * v1 * v1) * (1.0 + 1e-9));
            }
        }
        hyp.push_back(smax);
    }
    for (int a = 0; a < D; ++a) hyp.push_back(c->UinvT[a * D + a]);  // the whitening diagonal, contiguous (kUdiag)
    {  // level 0 of the auxiliary screen (kPre, aux_screen0_ub): 1/gamma, the |v| interval, c = rsk xmax; xmax = 6.77
       // bounds |r cos|, |r sin| of every Box-Muller pair of u32_01 uniforms (r <= sqrt(-2 log 2^-33) = 6.7638)
        const double xmax = 6.77, cc = c->rsk * xmax, an = std::fabs(c->nu);
        hyp.push_back(2.0 / (std::sqrt(cc * cc + 4.0 * D) + cc));
        hyp.push_back(std::max((double)D - an * xmax, 0.0));
        hyp.push_back((double)D + an * xmax);
        hyp.push_back(cc);
    }
    if (c->wide) {  // the wide kernels' item frame at DT: mu0 and U^T packed, zero beyond D (AssignArgs::uw)
        c->uw_off = (int64_t)hyp.size();
        for (int a = 0; a < c->DT; ++a) hyp.push_back(a < D ? c->mu0[a] : 0.0);
        for (int a = 0; a < c->DT; ++a)
            for (int b = a; b < c->DT; ++b) hyp.push_back((a < D && b < D) ? c->UinvT[a * D + b] : 0.0);
    }
    std::vector<double> gp;
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) gp.push_back(c->Gp[a * D + b]);
    if ((r = dalloc(c, &c->hyp, hyp.size())) || (r = dalloc(c, &c->d_mu0, (size_t)D)) ||
        (r = dalloc(c, &c->d_LT, (size_t)D * D)) || (r = dalloc(c, &c->d_Gp, gp.size())) ||
        (r = dalloc(c, &c->d_LTL, (size_t)D * D)) ||
        (c->prior == NP8_PRIOR_NIW &&
         ((r = dalloc(c, &c->d_U, (size_t)D * D)) || (r = dalloc(c, &c->d_Uinv, (size_t)D * D)) ||
          (r = dalloc(c, &c->d_Psi0, (size_t)D * D)) || (r = dalloc(c, &c->pend, (size_t)4 * kReqMax)))) ||
        (c->wide && c->prior != NP8_PRIOR_NIW && (r = dalloc(c, &c->pend, (size_t)4 * kReqMax))) ||
        (c->wide && (r = dalloc(c, &c->pend_ll, (size_t)2 * kReqMax))) ||
        (c->wide && ((r = dalloc(c, &c->wA, (size_t)kc * c->DT * c->DT)) ||
                     (r = dalloc(c, &c->wfrag, (size_t)kc * (c->DT * c->DT + c->DT))) ||  // >= the compact rows
                     (r = dalloc(c, &c->wmu, (size_t)kc * c->DT)) || (r = dalloc(c, &c->lam_lo, (size_t)kc)) ||
                     (r = dalloc(c, &c->wdist, (size_t)kc * kc)) ||
                     (r = dalloc(c, &c->wdirty, (size_t)kc))))) {
        free_device(c);
        delete c;
        return r;
    }
    // on the context's stream, behind the zero-fills dalloc queued there (a null-stream hipMemcpy does
    // not order against a non-blocking stream: the fill could land after the copy)
    const bool up_ok =
        hipMemcpyAsync(c->hyp, hyp.data(), sizeof(double) * hyp.size(), hipMemcpyHostToDevice, c->stream) == hipSuccess &&
        hipMemcpyAsync(c->d_mu0, c->mu0.data(), sizeof(double) * D, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
        hipMemcpyAsync(c->d_LT, c->LT.data(), sizeof(double) * D * D, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
        hipMemcpyAsync(c->d_Gp, gp.data(), sizeof(double) * gp.size(), hipMemcpyHostToDevice, c->stream) == hipSuccess &&
        hipMemcpyAsync(c->d_LTL, c->LTL.data(), sizeof(double) * D * D, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
        (c->prior != NP8_PRIOR_NIW ||
         (hipMemcpyAsync(c->d_U, c->U.data(), sizeof(double) * D * D, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
          hipMemcpyAsync(c->d_Uinv, c->Uinv.data(), sizeof(double) * D * D, hipMemcpyHostToDevice, c->stream) ==
              hipSuccess &&
          hipMemcpyAsync(c->d_Psi0, c->Lambda.data(), sizeof(double) * D * D, hipMemcpyHostToDevice, c->stream) ==
              hipSuccess));
    if (!up_ok || reset_ctl(c) || hipStreamSynchronize(c->stream) != hipSuccess ||
        (c->prior == NP8_PRIOR_NIW && np8_niw_prepare(D) != hipSuccess)) {
        free_device(c);
        delete c;
        return NP8_ERR_HIP;
    }
    *out = c;
    return NP8_OK;
}

int np8_destroy(np8_ctx *c) {
    if (!c) return NP8_OK;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    collect_timers(c);
    drop_graph(c);
    for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    free_device(c);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return NP8_OK;
}

const char *np8_last_error(const np8_ctx *c) { return c ? c->err.c_str() : "null context"; }

int np8_set_data(np8_ctx *c, const double *X, int64_t n, int32_t D, int64_t offset, int64_t n_global) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (D != c->D) return fail(c, NP8_ERR_ARG, "np8_set_data: D does not match the configuration");
    if (n < 0 || (n > 0 && !X)) return fail(c, NP8_ERR_ARG, "np8_set_data: bad buffer");
    if (n_global <= 0) n_global = n;
    if (offset < 0 || offset + n > n_global || n_global > 0x7FFFFFFFll)
        return fail(c, NP8_ERR_ARG, "np8_set_data: shard outside [0, n_global) or n_global >= 2^31");
    drop_graph(c);
    c->lists_valid = c->r2_zero = c->collecting = false;
    c->snap_lazy = false;  // (no state any more)
    c->n_loc = n;
    c->offset = offset;
    c->n_glob = n_global;
    c->part_waves = c->wide ? np8_suffstats_wide_waves(n) : 0;
    if (c->substeps_auto)  // (n_global only: the same choice on every rank)
        c->substeps = n_global <= NP8_SUBSTEPS_AUTO_N ? std::max(1, std::min(NP8_SUBSTEPS_AUTO_S, 16384 / c->kcap)) : 1;
    int r = 0;
    // wide path: fp32 items in DT rows (zero beyond D), then kFrameRows rows of the item's frame (np8_wide_frame)
    const size_t nx = c->wide ? ((size_t)n * (c->DT + kFrameRows) + 1) / 2 : (size_t)n * D;
    if ((r = dalloc(c, &c->X, nx)) || (r = dalloc(c, &c->z, (size_t)n)) ||
        (r = dalloc(c, &c->z_best, (size_t)n)) || (r = dalloc(c, &c->wr2, (size_t)((n + 63) / 64))) ||
        (r = dalloc(c, &c->llpart, (size_t)((n + 63) / 64))) ||
        (c->wide && c->param_update == NP8_PARAM_NIW_CONJUGATE &&
         ((r = dalloc(c, &c->part, (size_t)(np8_suffstats_wide_waves(n) * kSuffRuns * np8_suffstats_wide_record(D)))) ||
          (r = dalloc(c, &c->part_slot, (size_t)(np8_suffstats_wide_waves(n) * kSuffRuns))))) ||
        (r = dalloc(c, &c->queue, (size_t)(64 * ((n + 63) / 64) + 64))) ||
        (r = dalloc(c, &c->qcount, (size_t)((n + 63) / 64 + 1))) ||
        (r = dalloc(c, &c->qlist, (size_t)((n + 63) / 64 + 1))))
        return r;
    for (int b = 0; b < 2; ++b)
        if ((r = dalloc(c, &c->Xs[b], nx)) || (r = dalloc(c, &c->zs[b], (size_t)n)) ||
            (r = dalloc(c, &c->ids[b], (size_t)n)))
            return r;
    const size_t bins = (size_t)c->kcap * c->substeps;  // sort keys (sub-step, slot)
    if ((r = dalloc(c, &c->s_hist, bins)) || (r = dalloc(c, &c->s_cursor, bins)) || (r = dalloc(c, &c->s_off, bins)) ||
        (r = alloc_records(c)))
        return r;
    c->sub_start.assign((size_t)c->substeps + 1, 0);  // the sub-steps' ranges of the sorted layout
    for (int64_t p = 0; p < n; ++p) c->sub_start[substep_of(c->seed, offset + p, (uint32_t)c->substeps) + 1] += 1;
    for (int k = 0; k < c->substeps; ++k) c->sub_start[(size_t)k + 1] += c->sub_start[(size_t)k];
    c->sub_next = 0;
    c->data_hash = hash_words(0xcbf29ce484222325ull ^ (uint64_t)n, X, sizeof(double) * (size_t)n * D);
    c->track = 0;  // a change log needs a new baseline for the new items
    c->vis_tag.assign((size_t)n, 0u);
    c->vis_n.assign((size_t)n, 0u);
    c->sorted_valid = false;
    if (c->wide) {  // rounded to fp32 (round to nearest even), as oracle/np8_oracle.c set_data does
        std::vector<float> soa((size_t)n * c->DT, 0.0f);
        double x2max = 0.0;
        for (int64_t i = 0; i < n; ++i) {
            double x2 = 0.0;
            for (int a = 0; a < D; ++a) {
                const float v = (float)X[(size_t)i * D + a];
                soa[(size_t)a * n + i] = v;
                x2 += (double)v * v;
            }
            x2max = std::max(x2max, x2);
        }
        c->screen16 = x2max <= kScreen16X2 && std::getenv("NP8_SCREEN_F32") == nullptr;  // (NaN: false; env: A/B switch)
        HIPC(c, hipMemcpyAsync(c->X, soa.data(), sizeof(float) * soa.size(), hipMemcpyHostToDevice, c->stream));
        HIPC(c, np8_launch_wide_frame(reinterpret_cast<float *>(c->X), n, c->hyp + c->uw_off, c->DT,
                                      c->stream));
        HIPC(c, hipStreamSynchronize(c->stream));
    } else {
        std::vector<double> soa((size_t)n * D);
        for (int64_t i = 0; i < n; ++i)
            for (int a = 0; a < D; ++a) soa[(size_t)a * n + i] = X[(size_t)i * D + a];
        HIPC(c, hipMemcpyAsync(c->X, soa.data(), sizeof(double) * soa.size(), hipMemcpyHostToDevice, c->stream));
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    c->have_data = true;
    c->have_state = false;
    return NP8_OK;
}

// niw_init_map (NIW prior, np8_init_random): G0 draw k goes to slot (*niw_init_map)[k] (-1: dropped),
// drawn on the device by np8_niw_post before the candidate table is built.
static int set_state_common(np8_ctx *c, const std::vector<SlotHost> &slots, const std::vector<int32_t> &cnt,
                            const std::vector<int32_t> &zloc, const std::vector<int32_t> *niw_init_map = nullptr) {
    int r = upload_slots(c, slots, cnt);
    if (r) return r;
    if (niw_init_map) {
        int32_t *d_map = nullptr;
        const int kinit = (int)niw_init_map->size();
        HIPC(c, hipMalloc(&d_map, sizeof(int32_t) * kinit));
        HIPC(c, hipMemcpyAsync(d_map, niw_init_map->data(), sizeof(int32_t) * kinit, hipMemcpyHostToDevice, c->stream));
        NiwArgs A = niw_args(c);
        A.write_cand = 0;
        A.init_k = kinit;
        A.init_map = d_map;
        const hipError_t e = np8_launch_niw_post(A, kinit, c->stream);
        HIPC(c, hipStreamSynchronize(c->stream));
        (void)hipFree(d_map);
        HIPC(c, e);
    }
    HIPC(c, hipMemcpyAsync(c->z, zloc.data(), sizeof(int32_t) * zloc.size(), hipMemcpyHostToDevice, c->stream));
    c->snap_lazy = false;  // the snapshot restarts with the state (reset_ctl)
    c->sorted_valid = false;
    c->use_sorted = false;
    c->lists_valid = c->r2_zero = c->collecting = false;
    r = reset_ctl(c);
    if (r) return r;
    r = rebuild(c);
    if (r) return r;
    r = refresh_wide(c, niw_init_map == nullptr);  // (the NIW G0 draws wrote their own contraction rows)
    if (r) return r;
    HIPC(c, hipStreamSynchronize(c->stream));
    c->have_state = true;
    return NP8_OK;
}

int np8_set_state(np8_ctx *c, const int32_t *z, int32_t K, const double *mu, const double *Sigma) {
    return np8_set_state_counts(c, z, K, mu, Sigma, nullptr);
}

int np8_set_state_counts(np8_ctx *c, const int32_t *z, int32_t K, const double *mu, const double *Sigma,
                         const int64_t *counts) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_data) return fail(c, NP8_ERR_STATE, "np8_set_state: no data");
    if (K < 1 || K > c->kcap || !mu || !Sigma || (c->n_loc > 0 && !z))
        return fail(c, NP8_ERR_ARG, "np8_set_state: K outside [1,kcap] or null buffer");
    std::vector<SlotHost> slots(K);
    for (int k = 0; k < K; ++k)
        if (!slot_from_sigma(c, mu + (size_t)k * c->D, Sigma + (size_t)k * c->D * c->D, slots[k]))
            return fail(c, NP8_ERR_SIGMA, "np8_set_state: covariance " + std::to_string(k) + " has det <= 0");
    std::vector<int32_t> cnt(K, 0), zl(c->n_loc);
    for (int64_t i = 0; i < c->n_loc; ++i) {
        if (z[i] < 0 || z[i] >= K) return fail(c, NP8_ERR_RANGE, "np8_set_state: label out of range");
        zl[i] = z[i];
        cnt[z[i]]++;
    }
    if (counts) {  // caller-supplied global counts (host-exchange runs); local labels must fit in them
        std::vector<int32_t> g(K);
        for (int k = 0; k < K; ++k) {
            if (counts[k] < cnt[k] || counts[k] > 0x7FFFFFFFll)
                return fail(c, NP8_ERR_RANGE, "np8_set_state_counts: counts smaller than this rank's labels");
            g[k] = (int32_t)counts[k];
        }
        return set_state_common(c, slots, g, zl);
    }
    if (c->world > 1 && !c->comm)
        return fail(c, NP8_ERR_STATE, "np8_set_state: host-exchange mode needs np8_set_state_counts");
    if (c->comm) {  // counts are global
        int32_t *d = nullptr;
        HIPC(c, hipMalloc(&d, sizeof(int32_t) * K));
        HIPC(c, hipMemcpy(d, cnt.data(), sizeof(int32_t) * K, hipMemcpyHostToDevice));
        NCCLC(c, ncclAllReduce(d, d, K, ncclInt32, ncclSum, c->comm, c->stream));
        HIPC(c, hipStreamSynchronize(c->stream));
        HIPC(c, hipMemcpy(cnt.data(), d, sizeof(int32_t) * K, hipMemcpyDeviceToHost));
        (void)hipFree(d);
    }
    return set_state_common(c, slots, cnt, zl);
}

int np8_init_random(np8_ctx *c, int32_t K_init) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_data) return fail(c, NP8_ERR_STATE, "np8_init_random: no data");
    if (K_init < 1 || K_init > c->kcap) return fail(c, NP8_ERR_ARG, "np8_init_random: K_init outside [1,kcap]");
    const int D = c->D, Q = g0_calls(D);
    const bool niw = c->prior == NP8_PRIOR_NIW;  // NIW: the draws are made on the device (np8_niw_post)
    std::vector<SlotHost> draws(K_init);
    for (int k = 0; k < K_init; ++k) {  // InitClusters::init: K G0 draws (np_init_clusters.cpp:24-40)
        if (niw) {
            draws[k].mu.assign(D, 0.0);
            draws[k].P.assign(c->DP, 0.0);
            draws[k].sigma.assign((size_t)D * D, 0.0);
            continue;
        }
        std::vector<double> g(4 * Q);
        for (int q = 0; q < Q; ++q) {
            double gq[4];
            normal_quad(c->seed, (uint64_t)k, 0xFFFFFFFFu, kStreamInitTheta, (uint32_t)q, gq);
            for (int h = 0; h < 4; ++h) g[4 * q + h] = gq[h];
        }
        slot_from_normals(c, g[0], g.data() + 1, draws[k]);
    }
    // uniform assignment of every item (np_mcmc.cpp:69-85); counts over ALL items, so every rank
    // gets the same global counts without communication.
    std::vector<int32_t> cntk(K_init, 0), zl(c->n_loc);
    for (int64_t i = 0; i < c->n_glob; ++i) {
        const double u = uniform(c->seed, (uint64_t)i, 0xFFFFFFFFu, kStreamInitZ, 0);
        int k = (int)(u * (double)K_init);
        if (k >= K_init) k = K_init - 1;
        cntk[k]++;
        if (i >= c->offset && i < c->offset + c->n_loc) zl[i - c->offset] = k;
    }
    // cleanup: drop empty clusters, keep order (membertrix.cpp:343-364)
    std::vector<int32_t> remap(K_init, -1), cnt;
    std::vector<SlotHost> slots;
    for (int k = 0; k < K_init; ++k)
        if (cntk[k] > 0) {
            remap[k] = (int32_t)slots.size();
            slots.push_back(draws[k]);
            cnt.push_back(cntk[k]);
        }
    for (auto &v : zl) v = remap[v];
    return set_state_common(c, slots, cnt, zl, niw ? &remap : nullptr);
}

int np8_sweep(np8_ctx *c, int32_t n_sweeps) {
    if (!c) return NP8_ERR_ARG;
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_sweep: no state (np8_set_state/np8_init_random)");
    const int64_t N = c->n_loc;
    int64_t chunk = (c->chunk <= 0 || c->chunk >= c->n_glob) ? N : c->chunk;
    const bool sync = chunk >= N;
    if (!sync && c->world > 1) return fail(c, NP8_ERR_ARG, "np8_sweep: chunk < N is single-rank only");
    if (c->comm && c->world > 1 && N == 0)  // (its peers would replay graphs it cannot capture)
        return fail(c, NP8_ERR_ARG, "np8_sweep: every rank of a communicator needs at least one item");
    if (n_sweeps <= 0) return NP8_OK;
    int r = settle(c);
    if (r) return r;
    const uint32_t target = c->epoch + (uint32_t)n_sweeps;
    while ((int32_t)(target - c->epoch) > 0) {
        // churn (moved since the last re-sort, as of the last finalize): enter > n/8, leave < n/64.  Not under a
        // communicator: the mirror is this rank's own count, read while a replay runs, and churn selects the graph --
        // whether the pending replay is settled before or after the next one is queued must be alike on every rank
        // (the settle of a halted replay runs collectives), so a sharded context decides from rank-uniform state only
        if (c->moved_host && !c->comm) {
            const int64_t mv = *(volatile int64_t *)c->moved_host;
            c->churn = c->churn ? (mv * 64 >= c->n_loc) : (mv * 8 > c->n_loc);
        }
        const bool can_graph = graph_eligible(c, sync) && target - c->epoch >= kGraphSweeps;
        // a sharded replay still unchecked: anything but the next replay of the same graph waits for it
        if (c->pend_on && !(can_graph && graph_current(c))) {
            if ((r = settle(c, nullptr, false))) return r;
            continue;
        }
        if (can_graph) {
            if ((r = ensure_graph(c))) return r;
            if (!c->graph && c->comm)  // (a capture failed on this rank only: its peers replay graphs)
                return fail(c, NP8_ERR_HIP, "np8_sweep: a sharded sweep graph could not be captured");
            if (c->graph) {
                if (c->graph_sort_outside && (*(volatile int64_t *)c->moved_host) * 32 > c->n_loc) {
                    // the layout went stale (as of a replay ago): re-sort before this one (the device re-checks)
                    if ((r = prepare_sorted_now(c))) return r;
                    *(volatile int64_t *)c->moved_host = 0;  // (until a finalize reports again)
                }
                const uint32_t e0 = c->epoch;
                const int32_t ch0 = c->checks;
                const int64_t f0 = c->n_folded, t0 = c->n_tail_cond;
                if ((r = run_graph(c))) return r;
                if (c->comm) {  // checked once the next replay is queued (the device stays busy meanwhile)
                    const int k = c->rev_k;
                    c->rev_k ^= 1;
                    if (!c->rev[k]) HIPC(c, hipEventCreateWithFlags(&c->rev[k], hipEventDisableTiming));
                    HIPC(c, hipEventRecord(c->rev[k], c->stream));
                    bool rec = false;
                    if ((r = settle(c, &rec, false))) return r;
                    if (!rec) {  // (after a recovery this replay did nothing: the recovery rewound past it)
                        c->pend_on = true;
                        c->pend_k = k;
                        c->pend_epoch = e0;
                        c->pend_checks = ch0;
                        c->pend_folded = f0;
                        c->pend_tail = t0;
                        c->pend_compact = c->graph_compact;
                    }
                }
                continue;
            }
        }
        if ((r = population(c))) return r;
        if ((r = end_sweep(c))) return r;
    }
    // a sharded context returns with its last replay settled (a halted one resumed here, where every rank is), so
    // that no other entry point has collectives to run: a rank that alone asks for statistics or a checkpoint must
    // not block in an all-gather its peers never join
    if (c->comm && c->pend_on && (r = settle(c))) return r;
    return NP8_OK;
}

int np8_check_invariants(np8_ctx *c, int64_t out[4]) {
    if (!c || !out) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_check_invariants: no state");
    int r = launch_invariants(c);
    if (r) return r;
    unsigned long long h[4];
    HIPC(c, hipMemcpyAsync(h, c->inv_out, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemsetAsync(c->inv_out, 0, sizeof(h), c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < 4; ++k) out[k] = (int64_t)h[k];
    if (h[0]) {
        Ctl tmp;
        (void)read_ctl(c, &tmp);
        int32_t zero = 0;
        HIPC(c, hipMemcpy(&c->ctl->err, &zero, sizeof(zero), hipMemcpyHostToDevice));
        return fail(c, NP8_ERR_STATE, "np8_check_invariants: violated (bits " + std::to_string(h[0]) + ")");
    }
    return NP8_OK;
}

}  // extern "C"

namespace {
// Checkpoint layout: header, then z [n_loc] int32 (slots), cnt [kcap] int32, slot_mu, slot_P, slot_c,
// slot_sigma, slot_iso, z_best, cnt_best, mu_best, sigma_best -- raw device bits.
struct CkptHeader {
    char magic[8];
    int32_t D, M, kcap, substeps, prior, contraction, checks, have_best;
    int32_t param_update, mh_steps, req_max, pad0;
    int64_t chunk;
    int64_t n_loc, offset, n_glob, n_new, n_rejected, mh_accepted;
    uint64_t seed, hyper_hash, data_hash;
    uint32_t epoch, pad;
    double L, best[2];
};

// the chain's hyper-parameters: alpha, kappa, nu, mu0, Lambda (the base measure of either prior)
uint64_t hyper_hash(const np8_ctx *c) {
    uint64_t h = 0xcbf29ce484222325ull;
    const double s[3] = {c->alpha, c->kappa, c->nu};
    h = hash_words(h, s, sizeof(s));
    h = hash_words(h, c->mu0.data(), sizeof(double) * c->mu0.size());
    return hash_words(h, c->Lambda.data(), sizeof(double) * c->Lambda.size());
}

struct CkptPart {
    void *dev;
    size_t bytes;
};

std::vector<CkptPart> ckpt_parts(np8_ctx *c) {
    const size_t kc = (size_t)c->kcap, D = (size_t)c->D, DP = (size_t)c->DP, n = (size_t)c->n_loc;
    return {{c->z, 4 * n},
            {c->cnt, 4 * kc},
            {c->slot_mu, 8 * kc * D},
            {c->slot_P, 8 * kc * DP},
            {c->slot_c, 8 * kc},
            {c->slot_sigma, 8 * kc * D * D},
            {c->slot_iso, 8 * kc},
            {c->z_best, 4 * n},
            {c->cnt_best, 4 * kc},
            {c->mu_best, 8 * kc * D},
            {c->sigma_best, 8 * kc * D * D}};
}
}  // namespace

extern "C" {

int64_t np8_checkpoint_bytes(np8_ctx *c) {
    if (!c || !c->have_data) return 0;
    int64_t b = (int64_t)sizeof(CkptHeader);
    for (const CkptPart &p : ckpt_parts(c)) b += (int64_t)p.bytes;
    return b;
}

int np8_checkpoint(np8_ctx *c, void *out, int64_t bytes) {
    if (!c || !out) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_checkpoint: no state");
    if (bytes < np8_checkpoint_bytes(c)) return fail(c, NP8_ERR_ARG, "np8_checkpoint: buffer too small");
    int r = flush_snapshot(c);
    if (r) return r;
    Ctl h;
    r = read_ctl(c, &h);
    if (r) return r;
    CkptHeader H;
    std::memset(&H, 0, sizeof(H));
    std::memcpy(H.magic, "NP8CKPT2", 8);
    H.param_update = c->param_update;
    H.mh_steps = c->mh_steps;
    H.req_max = c->req_max;
    H.chunk = c->chunk;
    H.hyper_hash = hyper_hash(c);
    H.data_hash = c->data_hash;
    H.D = c->D;
    H.M = c->M;
    H.kcap = c->kcap;
    H.substeps = c->substeps;
    H.prior = c->prior;
    H.contraction = c->contraction;
    H.checks = c->checks;
    H.have_best = h.have_best;
    H.n_loc = c->n_loc;
    H.offset = c->offset;
    H.n_glob = c->n_glob;
    H.n_new = h.n_new;
    H.n_rejected = h.n_rejected;
    H.mh_accepted = h.mh_accepted;
    H.seed = c->seed;
    H.epoch = c->epoch;
    H.L = h.L;
    H.best[0] = h.best[0];
    H.best[1] = h.best[1];
    unsigned char *o = static_cast<unsigned char *>(out);
    std::memcpy(o, &H, sizeof(H));
    o += sizeof(H);
    for (const CkptPart &p : ckpt_parts(c)) {
        HIPC(c, hipMemcpy(o, p.dev, p.bytes, hipMemcpyDeviceToHost));
        o += p.bytes;
    }
    return NP8_OK;
}

int np8_restore(np8_ctx *c, const void *in, int64_t bytes) {
    if (!c || !in) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_data) return fail(c, NP8_ERR_STATE, "np8_restore: no data (np8_set_data with the same items first)");
    if (bytes < (int64_t)sizeof(CkptHeader) || bytes != np8_checkpoint_bytes(c))
        return fail(c, NP8_ERR_ARG, "np8_restore: size differs from this context's checkpoint");
    CkptHeader H;
    std::memcpy(&H, in, sizeof(H));
    if (std::memcmp(H.magic, "NP8CKPT2", 8) != 0 || H.D != c->D || H.M != c->M || H.kcap != c->kcap ||
        H.substeps != c->substeps || H.prior != c->prior || H.contraction != c->contraction ||
        H.param_update != c->param_update || H.mh_steps != c->mh_steps || H.req_max != c->req_max ||
        H.chunk != c->chunk || H.hyper_hash != hyper_hash(c) || H.seed != c->seed)
        return fail(c, NP8_ERR_ARG, "np8_restore: checkpoint of another configuration or seed");
    if (H.n_loc != c->n_loc || H.offset != c->offset || H.n_glob != c->n_glob || H.data_hash != c->data_hash)
        return fail(c, NP8_ERR_ARG, "np8_restore: checkpoint of other data or another data shard");
    drop_graph(c);
    HIPC(c, hipStreamSynchronize(c->stream));
    const unsigned char *p = static_cast<const unsigned char *>(in) + sizeof(H);
    for (const CkptPart &q : ckpt_parts(c)) {
        HIPC(c, hipMemcpy(q.dev, p, q.bytes, hipMemcpyHostToDevice));
        p += q.bytes;
    }
    c->rows_iso = false;  // raw slot tables: isotropy unknown (np8_assign_queue stays in)
    // eigenvalue bounds unknown for the restored slots (0: a row that is not isotropic stays in every list)
    if (c->slot_lam) HIPC(c, hipMemsetAsync(c->slot_lam, 0, sizeof(double) * 2 * c->kcap, c->stream));
    c->snap_lazy = false;  // the snapshot buffers are the checkpoint's
    c->sorted_valid = false;
    c->use_sorted = false;
    c->lists_valid = c->r2_zero = c->collecting = false;
    c->epoch = H.epoch;
    c->checks = H.checks;
    c->t_base = H.epoch;
    Ctl h;
    std::memset(&h, 0, sizeof(h));
    h.have_best = H.have_best;
    h.n_new = H.n_new;
    h.n_rejected = H.n_rejected;
    h.mh_accepted = H.mh_accepted;
    h.L = H.L;
    h.best[0] = H.best[0];
    h.best[1] = H.best[1];
    h.t_base = H.epoch;
    HIPC(c, hipMemcpyAsync(c->ctl, &h, sizeof(h), hipMemcpyHostToDevice, c->stream));  // (stream-ordered)
    HIPC(c, hipStreamSynchronize(c->stream));
    c->have_state = true;
    int r = rebuild(c);  // the dense table from the restored slots
    if (r) return r;
    if ((r = refresh_wide(c, true))) return r;
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

int np8_population_sweep(np8_ctx *c) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_population_sweep: no state (np8_set_state/np8_init_random)");
    return population(c);
}

int np8_track_changes(np8_ctx *c, int32_t mode) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (mode < 0 || mode > NP8_CHANGES_FROM_EMPTY) return fail(c, NP8_ERR_ARG, "np8_track_changes: bad mode");
    c->track = mode ? 1 : 0;
    if (!mode) return NP8_OK;
    if (!c->have_data) return fail(c, NP8_ERR_STATE, "np8_track_changes: no data");
    const int D = c->D, kc = c->kcap;
    int r = 0;
    if ((r = dalloc(c, &c->z_base, (size_t)c->n_loc)) || (r = dalloc(c, &c->cnt_base, (size_t)kc)) ||
        (r = dalloc(c, &c->mu_base, (size_t)kc * D)) || (r = dalloc(c, &c->sigma_base, (size_t)kc * D * D)) ||
        (r = dalloc(c, &c->chg_count, 1)) || (r = dalloc(c, &c->chg_flags, (size_t)kc)))
        return r;
    if (mode == NP8_CHANGES_FROM_EMPTY || !c->have_state) {  // every item unassigned, no live slot
        if (c->n_loc > 0) HIPC(c, hipMemsetD32Async(reinterpret_cast<int *>(c->z_base), -1, c->n_loc, c->stream));
    } else {
        HIPC(c, hipMemcpyAsync(c->z_base, c->z, sizeof(int32_t) * c->n_loc, hipMemcpyDeviceToDevice, c->stream));
        HIPC(c, hipMemcpyAsync(c->cnt_base, c->cnt, sizeof(int32_t) * kc, hipMemcpyDeviceToDevice, c->stream));
        HIPC(c, hipMemcpyAsync(c->mu_base, c->slot_mu, sizeof(double) * kc * D, hipMemcpyDeviceToDevice, c->stream));
        HIPC(c, hipMemcpyAsync(c->sigma_base, c->slot_sigma, sizeof(double) * kc * D * D, hipMemcpyDeviceToDevice,
                               c->stream));
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

int np8_changes(np8_ctx *c, int64_t item_cap, int64_t *item, int32_t *slot, int32_t *created, int32_t *removed,
                int32_t *updated, double *mu, double *Sigma, np8_changes_t *out) {
    if (!c || !out) return NP8_ERR_ARG;
    std::memset(out, 0, sizeof(*out));
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->track) return fail(c, NP8_ERR_STATE, "np8_changes: change tracking is off (np8_track_changes)");
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_changes: no state");
    if (int r = flush_snapshot(c)) return r;
    if (item_cap < 0 || (item_cap > 0 && (!item || !slot)) || !created || !removed || !updated)
        return fail(c, NP8_ERR_ARG, "np8_changes: bad arguments");
    const int D = c->D, kc = c->kcap;
    // staging for the moved items: grows to the largest request seen
    const int64_t need = item_cap < c->n_loc ? item_cap : c->n_loc;
    if (need > c->chg_cap) {
        int r = 0;
        if ((r = dalloc(c, &c->chg_item, (size_t)need)) || (r = dalloc(c, &c->chg_slot, (size_t)need))) return r;
        c->chg_cap = need;
    }
    HIPC(c, hipMemsetAsync(c->chg_count, 0, sizeof(unsigned long long), c->stream));
    HIPC(c, np8_launch_changes(c->z, c->z_base, c->n_loc, c->chg_item, c->chg_slot, need, c->chg_count, c->cnt, c->cnt_base,
                               c->slot_mu, c->mu_base, c->slot_sigma, c->sigma_base, D, kc, c->chg_flags, c->stream));
    unsigned long long nm = 0;
    std::vector<uint8_t> fl((size_t)kc);
    HIPC(c, hipMemcpyAsync(&nm, c->chg_count, sizeof(nm), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemcpyAsync(fl.data(), c->chg_flags, (size_t)kc, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    out->n_moved = (int64_t)nm;
    if ((int64_t)nm > item_cap) return fail(c, NP8_ERR_CAPACITY, "np8_changes: more moved items than item_cap");
    if (nm > 0) {
        std::vector<int64_t> it((size_t)nm);
        std::vector<int32_t> sl((size_t)nm);
        HIPC(c, hipMemcpy(it.data(), c->chg_item, sizeof(int64_t) * nm, hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(sl.data(), c->chg_slot, sizeof(int32_t) * nm, hipMemcpyDeviceToHost));
        std::vector<int64_t> ord((size_t)nm);
        for (size_t k = 0; k < nm; ++k) ord[k] = (int64_t)k;
        std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return it[a] < it[b]; });  // ascending items
        for (size_t k = 0; k < nm; ++k) {
            item[k] = it[ord[k]];
            slot[k] = sl[ord[k]];
        }
    }
    std::vector<int32_t> par;  // created then updated slots: their parameters go out
    for (int s = 0; s < kc; ++s) {
        if (fl[s] == 1) {
            created[out->n_created++] = s;
            par.push_back(s);
        } else if (fl[s] == 2) {
            removed[out->n_removed++] = s;
        }
    }
    for (int s = 0; s < kc; ++s)
        if (fl[s] == 3) {
            updated[out->n_updated++] = s;
            par.push_back(s);
        }
    if (!par.empty() && (mu || Sigma)) {
        std::vector<double> m((size_t)kc * D), sg((size_t)kc * D * D);
        HIPC(c, hipMemcpy(m.data(), c->slot_mu, sizeof(double) * m.size(), hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(sg.data(), c->slot_sigma, sizeof(double) * sg.size(), hipMemcpyDeviceToHost));
        for (size_t q = 0; q < par.size(); ++q) {
            if (mu) std::memcpy(mu + q * D, &m[(size_t)par[q] * D], sizeof(double) * D);
            if (Sigma) std::memcpy(Sigma + q * D * D, &sg[(size_t)par[q] * D * D], sizeof(double) * D * D);
        }
    }
    // the current state becomes the baseline
    HIPC(c, hipMemcpyAsync(c->z_base, c->z, sizeof(int32_t) * c->n_loc, hipMemcpyDeviceToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->cnt_base, c->cnt, sizeof(int32_t) * kc, hipMemcpyDeviceToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->mu_base, c->slot_mu, sizeof(double) * kc * D, hipMemcpyDeviceToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->sigma_base, c->slot_sigma, sizeof(double) * kc * D * D, hipMemcpyDeviceToDevice, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

int np8_prepare_sweeps(np8_ctx *c, int32_t n_sweeps) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_prepare_sweeps: no state");
    const int64_t chunk = (c->chunk <= 0 || c->chunk >= c->n_glob) ? c->n_loc : c->chunk;
    if (!graph_eligible(c, chunk >= c->n_loc) || (uint32_t)n_sweeps < kGraphSweeps) return NP8_OK;
    int r = ensure_graph(c);
    if (r) return r;
    if (c->graph) HIPC(c, hipGraphUpload(c->graph, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

int np8_update_points(np8_ctx *c, const int64_t *ids, int64_t n) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_update_points: no state");
    if (c->world > 1) return fail(c, NP8_ERR_ARG, "np8_update_points: single-rank only");
    if (n <= 0) return NP8_OK;
    if (int r = flush_snapshot(c)) return r;
    for (int64_t k = 0; k < n; ++k)
        if (ids[k] < 0 || ids[k] >= c->n_loc) return fail(c, NP8_ERR_RANGE, "np8_update_points: id out of range");
    if (n > c->order_cap) {
        int r = dalloc(c, &c->order, (size_t)n);
        if (r) return r;
        c->order_cap = n;
    }
    // the k-th visit of an item within this epoch draws with item key index | k << 32 (fresh auxiliaries
    // and pick uniform for every visit, also when the caller never ends the sweep)
    std::vector<int64_t> keys((size_t)n);
    const uint32_t tag = c->epoch + 1u;
    for (int64_t k = 0; k < n; ++k) {
        const int64_t i = ids[k];
        if (c->vis_tag[i] != tag) {
            c->vis_tag[i] = tag;
            c->vis_n[i] = 0;
        }
        keys[k] = i | ((int64_t)c->vis_n[i]++ << 32);
    }
    HIPC(c, hipMemcpyAsync(c->order, keys.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, c->stream));
    for (int64_t k = 0; k < n; ++k) {
        int r = step(c, k, k + 1, c->order, false);
        if (r) return r;
    }
    HIPC(c, hipStreamSynchronize(c->stream));  // ids buffer may be reused by the caller
    return NP8_OK;
}

int np8_end_sweep(np8_ctx *c) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_end_sweep: no state");
    if (c->sub_next != 0)
        return fail(c, NP8_ERR_STATE, "np8_end_sweep: the sweep's sub-steps are not all done (np8_step_local/np8_step_merge)");
    return end_sweep(c);
}

int np8_sync(np8_ctx *c) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    Ctl h;
    int r = read_ctl(c, &h);
    if (r) return r;
    if (h.err) {
        int32_t zero = 0;
        HIPC(c, hipMemcpy(&c->ctl->err, &zero, sizeof(zero), hipMemcpyHostToDevice));
        if (h.err & kErrSigma)
            return fail(c, NP8_ERR_SIGMA, "a cluster precision is not numerically positive definite (wide path factor)");
        if (h.err & kErrCapacity) return fail(c, NP8_ERR_CAPACITY, "a device table is full");
        if (h.err & kErrInvariant)
            return fail(c, NP8_ERR_STATE, "a debug invariant failed (np8_check_invariants: labels, counts, K, table)");
        if (h.err & kErrQueue)
            return fail(c, NP8_ERR_STATE, "internal: np8_assign_fast deferred a lane with no queue launched");
        if (h.err & kErrSpin)
            return fail(c, NP8_ERR_STATE, "internal: np8_fin_prune's list workgroups timed out waiting for finalize");
    }
    return NP8_OK;
}

int np8_get_state(np8_ctx *c, int32_t which, int32_t *z, int32_t *K, double *mu, double *Sigma, int64_t *counts) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_get_state: no state");
    int r = flush_snapshot(c);
    if (r) return r;
    Ctl h;
    r = read_ctl(c, &h);
    if (r) return r;
    if (which == 1 && !h.have_best) return fail(c, NP8_ERR_STATE, "np8_get_state: no max-likelihood snapshot yet");
    const int D = c->D, kc = c->kcap;
    std::vector<int32_t> cn(kc), zz(c->n_loc);
    HIPC(c, hipMemcpy(cn.data(), which ? c->cnt_best : c->cnt, sizeof(int32_t) * kc, hipMemcpyDeviceToHost));
    std::vector<int32_t> lab(kc, -1);
    int k = 0;
    for (int s = 0; s < kc; ++s)
        if (cn[s] > 0) lab[s] = k++;
    if (K) *K = k;
    if (z) {
        HIPC(c, hipMemcpy(zz.data(), which ? c->z_best : c->z, sizeof(int32_t) * c->n_loc, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < c->n_loc; ++i) z[i] = lab[zz[i]];
    }
    if (mu || Sigma || counts) {
        std::vector<double> m((size_t)kc * D), sg((size_t)kc * D * D);
        HIPC(c, hipMemcpy(m.data(), which ? c->mu_best : c->slot_mu, sizeof(double) * m.size(), hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(sg.data(), which ? c->sigma_best : c->slot_sigma, sizeof(double) * sg.size(),
                          hipMemcpyDeviceToHost));
        for (int s = 0; s < kc; ++s) {
            if (lab[s] < 0) continue;
            if (mu) std::memcpy(mu + (size_t)lab[s] * D, &m[(size_t)s * D], sizeof(double) * D);
            if (Sigma) std::memcpy(Sigma + (size_t)lab[s] * D * D, &sg[(size_t)s * D * D], sizeof(double) * D * D);
            if (counts) counts[lab[s]] = cn[s];
        }
    }
    return NP8_OK;
}

int np8_aux_bounds(np8_ctx *c, const int64_t *idx, int64_t n, double *out) {
    if (!c) return NP8_ERR_ARG;
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_aux_bounds: no state");
    if (c->wide || c->prior != NP8_PRIOR_REFERENCE)
        return fail(c, NP8_ERR_STATE, "np8_aux_bounds: the reference prior's fp64 path only");
    if (n <= 0) return NP8_OK;
    for (int64_t k = 0; k < n; ++k)
        if (idx[k] < 0 || idx[k] >= c->n_loc) return fail(c, NP8_ERR_RANGE, "np8_aux_bounds: index out of range");
    int64_t *d_idx = nullptr;
    double *d_out = nullptr;
    HIPC(c, hipMalloc(&d_idx, sizeof(int64_t) * n));
    HIPC(c, hipMalloc(&d_out, sizeof(double) * n * c->M));
    HIPC(c, hipMemcpy(d_idx, idx, sizeof(int64_t) * n, hipMemcpyHostToDevice));
    HIPC(c, np8_launch_aux_bounds(assign_args(c, 0, 0, nullptr, false), c->D, c->M, d_idx, n, d_out, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipMemcpy(out, d_out, sizeof(double) * n * c->M, hipMemcpyDeviceToHost));
    (void)hipFree(d_idx);
    (void)hipFree(d_out);
    return NP8_OK;
}

int np8_loglik_matrix(np8_ctx *c, const int64_t *idx, int64_t n, double *out) {
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_loglik_matrix: no state");
    if (n <= 0) return NP8_OK;
    for (int64_t k = 0; k < n; ++k)
        if (idx[k] < 0 || idx[k] >= c->n_loc) return fail(c, NP8_ERR_RANGE, "np8_loglik_matrix: index out of range");
    Ctl h;
    int r = read_ctl(c, &h);
    if (r) return r;
    const int64_t w = (int64_t)h.K + c->M;
    int64_t *d_idx = nullptr;
    double *d_out = nullptr;
    HIPC(c, hipMalloc(&d_idx, sizeof(int64_t) * n));
    HIPC(c, hipMalloc(&d_out, sizeof(double) * n * w));
    HIPC(c, hipMemcpy(d_idx, idx, sizeof(int64_t) * n, hipMemcpyHostToDevice));
    if (c->wide)
        HIPC(c, np8_launch_loglik_matrix_wide(assign_args(c, 0, 0, nullptr, false), wide_args(c), c->D, c->M, c->prior,
                                              d_idx, n, d_out, c->stream));
    else
        HIPC(c, np8_launch_loglik_matrix(assign_args(c, 0, 0, nullptr, false), c->D, c->M, c->prior, d_idx, n, d_out,
                                         c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipMemcpy(out, d_out, sizeof(double) * n * w, hipMemcpyDeviceToHost));
    (void)hipFree(d_idx);
    (void)hipFree(d_out);
    return NP8_OK;
}

int np8_pick_batch(np8_ctx *c, const double *lw, int32_t n, const double *u, int64_t n_draws, int32_t *out) {
    if (!c || !lw || !u || !out || n < 1 || n_draws < 0 || n_draws > (int64_t)1 << 31)
        return c ? fail(c, NP8_ERR_ARG, "np8_pick_batch: bad arguments") : NP8_ERR_ARG;
    if (n_draws == 0) return NP8_OK;
    double *d_lw = nullptr, *d_u = nullptr;
    int32_t *d_out = nullptr;
    HIPC(c, hipMalloc(&d_lw, sizeof(double) * n));
    HIPC(c, hipMalloc(&d_u, sizeof(double) * n_draws));
    HIPC(c, hipMalloc(&d_out, sizeof(int32_t) * n_draws));
    HIPC(c, hipMemcpy(d_lw, lw, sizeof(double) * n, hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(d_u, u, sizeof(double) * n_draws, hipMemcpyHostToDevice));
    HIPC(c, np8_launch_pick_batch(d_lw, n, d_u, n_draws, d_out, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipMemcpy(out, d_out, sizeof(int32_t) * n_draws, hipMemcpyDeviceToHost));
    (void)hipFree(d_lw);
    (void)hipFree(d_u);
    (void)hipFree(d_out);
    return NP8_OK;
}

int np8_total_loglik(np8_ctx *c, double *out) {
    if (!c || !out) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_total_loglik: no state");
    int r = launch_total_loglik(c);
    if (r) return r;
    Ctl h;
    r = read_ctl(c, &h);
    if (r) return r;
    *out = h.L;
    return NP8_OK;
}

namespace {
// The statistics as this build lays them out; np8_stats_sized copies the caller's prefix of it.
int fill_stats(np8_ctx *c, np8_stats_t *out) {
    Ctl h;
    int r = read_ctl(c, &h);
    if (r) return r;
    collect_timers(c);
    std::memset(out, 0, sizeof(*out));
    out->K = h.K;
    out->epoch = c->epoch;
    out->new_clusters = h.n_new;
    out->rejected_requests = h.n_rejected;
    out->existing_picks = -1;
    out->best_loglik = h.best[c->checks & 1];
    out->last_loglik = h.L;
    out->ms_assign = c->ms[0];
    out->ms_finalize = c->ms[1];
    out->ms_loglik = c->ms[2];
    out->ms_params = c->ms[3];
    out->n_timed_assign = c->n_timed[0];
    out->n_timed_finalize = c->n_timed[1];
    out->n_timed_loglik = c->n_timed[2];
    out->n_timed_params = c->n_timed[3];
    out->ms_sm_members = c->ms[4];
    out->ms_sm_eval = c->ms[5];
    out->n_timed_sm_members = c->n_timed[4];
    out->n_timed_sm_eval = c->n_timed[5];
    out->mh_accepted = h.mh_accepted;
    out->screen_violations = (int64_t)h.n_screen_viol;
    out->folded_checks = c->n_folded;
    out->tail_list_builds = (int64_t)h.list_builds;
    out->tail_steps = c->n_tail_cond;
    out->compact_halts = c->n_halts;
    out->substeps = c->substeps;
    {
        std::vector<unsigned long long> ev((size_t)10 * kEvalSlots);
        HIPC(c, hipMemcpy(ev.data(), c->evalc, sizeof(unsigned long long) * ev.size(), hipMemcpyDeviceToHost));
        for (int k = 0; k < kEvalSlots; ++k) {
            out->n_quad += (int64_t)ev[2 * k];
            out->n_quad_iso += (int64_t)ev[2 * k + 1];
            out->aux_exact_lanes += (int64_t)ev[2 * kEvalSlots + 2 * k];
            out->aux_exact_waves += (int64_t)ev[2 * kEvalSlots + 2 * k + 1];
            out->full_walk_lanes += (int64_t)ev[4 * kEvalSlots + 2 * k];
            out->full_walk_waves += (int64_t)ev[4 * kEvalSlots + 2 * k + 1];
            out->many_group_waves += (int64_t)ev[6 * kEvalSlots + 2 * k];
            out->list_entries += (int64_t)ev[6 * kEvalSlots + 2 * k + 1];
            out->pick_evals += (int64_t)ev[8 * kEvalSlots + 2 * k];
        }
    }
    return NP8_OK;
}
}  // namespace

int np8_stats_sized(np8_ctx *c, np8_stats_t *out, size_t out_bytes) {
    if (!c || !out || out_bytes < NP8_STATS_MIN_BYTES) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    np8_stats_t full;
    const int r = fill_stats(c, &full);
    if (r) return r;
    std::memcpy(out, &full, out_bytes < sizeof(full) ? out_bytes : sizeof(full));
    return NP8_OK;
}

int np8_stats(np8_ctx *c, np8_stats_t *out) { return np8_stats_sized(c, out, NP8_STATS_MIN_BYTES); }

int np8_set_timing(np8_ctx *c, int32_t enable) {
    if (!c) return NP8_ERR_ARG;
    c->timing = (enable & NP8_TIMING_EVENTS) != 0;
    c->count_eval = (enable & NP8_TIMING_COUNTERS) != 0;
    c->time_all = c->timing && (enable & NP8_TIMING_ALL_ASSIGNS) != 0;
    return NP8_OK;
}

int np8_set_stream(np8_ctx *c, void *stream) {
    if (!c) return NP8_ERR_ARG;
    (void)hipStreamSynchronize(c->stream);
    drop_graph(c);
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    c->stream = (hipStream_t)stream;
    c->own_stream = false;
    return NP8_OK;
}

int np8_comm_unique_id(uint8_t out[128]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return NP8_ERR_COMM;
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out, &id, sizeof(id));
    return NP8_OK;
}

static int resize_records(np8_ctx *c, int world) {
    drop_graph(c);  // a captured graph references the old records
    c->world = world;
    int r = alloc_records(c);
    if (r) return r;
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

int np8_comm_init(np8_ctx *c, const uint8_t id[128], int32_t rank, int32_t world) {
    // np8_finalize walks at most 64 records (base[65] in LDS)
    if (!c || world < 1 || world > 64 || rank < 0 || rank >= world) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!id) {  // host-exchange mode: the caller moves records (np8_step_local / np8_step_merge)
        c->rank = rank;
        return resize_records(c, world);
    }
    HIPC(c, hipSetDevice(c->device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    NCCLC(c, ncclCommInitRank(&c->comm, world, uid, rank));
    c->rank = rank;
    return resize_records(c, world);
}

int64_t np8_record_bytes(np8_ctx *c) { return c ? c->rec_bytes : 0; }

int np8_step_local(np8_ctx *c, void *record_out) {
    if (!c || !record_out) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_step_local: no state");
    const int sub = c->sub_next;  // sub-step sub of the data-parallel sweep (0 with one step)
    const int64_t p0 = c->sub_start[(size_t)sub], p1 = c->sub_start[(size_t)sub + 1];
    c->use_sorted = c->n_loc > 0;
    if (c->use_sorted && sub == 0) {
        int r0 = prepare_sorted(c);
        if (r0) return r0;
    }
    c->collecting = false;  // no pruning on the host-exchange path
    c->lists_valid = c->r2_zero = false;
    c->host_exch_step = true;
    int r = launch_assign(c, p0, p1, nullptr, false);
    c->host_exch_step = false;
    if (r) return r;
    if (c->stage)
        HIPC(c, np8_launch_req_select(c->stage, c->stage_cap, c->rec, c->rec_cap, c->kcap, c->D, c->req_max, nullptr, 0,
                                      c->stream));
    HIPC(c, hipMemcpyAsync(record_out, c->rec, (size_t)c->rec_bytes, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

int64_t np8_param_stats_bytes(np8_ctx *c) {
    return c ? (int64_t)sizeof(double) * c->kcap * (c->D + c->DP) : 0;
}

int np8_param_stats_local(np8_ctx *c, double *out) {
    if (!c || !out) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_param_stats_local: no state");
    if (c->param_update == NP8_PARAM_FROZEN) return fail(c, NP8_ERR_STATE, "np8_param_stats_local: frozen parameters");
    const size_t nacc = (size_t)c->kcap * (c->D + c->DP);
    int r = param_update(c, 1);
    if (r) return r;
    HIPC(c, hipMemcpyAsync(out, c->acc, sizeof(double) * nacc, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipMemsetAsync(c->acc, 0, sizeof(double) * nacc, c->stream));  // acc stays zero between sweeps
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

int np8_end_sweep_stats(np8_ctx *c, const double *summed) {
    if (!c || !summed) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_end_sweep_stats: no state");
    if (c->param_update == NP8_PARAM_FROZEN) return fail(c, NP8_ERR_STATE, "np8_end_sweep_stats: frozen parameters");
    if (c->sub_next != 0)
        return fail(c, NP8_ERR_STATE, "np8_end_sweep_stats: the sweep's sub-steps are not all done");
    const size_t nacc = (size_t)c->kcap * (c->D + c->DP);
    HIPC(c, hipMemcpyAsync(c->acc, summed, sizeof(double) * nacc, hipMemcpyHostToDevice, c->stream));
    int r = end_sweep(c, true);
    if (r) return r;
    HIPC(c, hipStreamSynchronize(c->stream));  // the caller's buffer may be reused
    return NP8_OK;
}

int np8_step_merge(np8_ctx *c, const void *records, int32_t world) {
    if (!c || !records || world < 1) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (world != c->world) return fail(c, NP8_ERR_ARG, "np8_step_merge: world differs from np8_comm_init");
    c->sub_next = (c->sub_next + 1) % c->substeps;
    if (world == 1) {
        HIPC(c, hipMemcpyAsync(c->rec, records, (size_t)c->rec_bytes, hipMemcpyHostToDevice, c->stream));
        return launch_finalize(c, c->rec, 1);
    }
    HIPC(c, hipMemcpyAsync(c->gath, records, (size_t)c->rec_bytes * world, hipMemcpyHostToDevice, c->stream));
    int r = launch_finalize(c, c->gath, world);
    if (r) return r;
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

// ---- compact records over the caller's transport ---------------------------------------
// The exchange an RCCL sweep graph runs, step by step over MPI / gloo: the compact record (count deltas and the
// first c_cap requests, its header counting all of them), the halt decision np8_finalize takes from the gathered
// headers (alike on every rank), and the resumption of a halted step with the full records.
namespace {
// the step's assign writes the compact record for every lane: the lean narrow kernel when it takes every lane (no
// deferred lane, no queue launch), or np8_assign_wide (any prior, any parameter update)
bool host_compact_ok(const np8_ctx *c) {
    if (!c->crec || c->comm || c->world <= 1 || c->count_eval || c->n_loc <= 0) return false;
    return c->wide || (c->diag_U && !c->fast_off && c->prior == NP8_PRIOR_REFERENCE && c->rows_iso && !c->queue_on);
}
}  // namespace

int64_t np8_compact_record_bytes(np8_ctx *c) { return (c && host_compact_ok(c)) ? c->c_bytes : 0; }

int np8_step_local_compact(np8_ctx *c, void *record_out) {
    if (!c || !record_out) return NP8_ERR_ARG;
    if (!c->have_state) return fail(c, NP8_ERR_STATE, "np8_step_local_compact: no state");
    if (!host_compact_ok(c))
        return fail(c, NP8_ERR_STATE, "np8_step_local_compact: no compact records here (np8_compact_record_bytes() == 0)");
    if (c->host_halted) return fail(c, NP8_ERR_STATE, "np8_step_local_compact: a halted step awaits np8_step_resume");
    const int sub = c->sub_next;
    const int64_t p0 = c->sub_start[(size_t)sub], p1 = c->sub_start[(size_t)sub + 1];
    c->use_sorted = true;
    if (sub == 0) {
        int r0 = prepare_sorted(c);
        if (r0) return r0;
    }
    c->collecting = false;  // no pruning on the host-exchange path
    c->lists_valid = c->r2_zero = false;
    c->host_exch_step = true;
    c->host_compact = true;
    int r = launch_assign(c, p0, p1, nullptr, false);
    c->host_exch_step = c->host_compact = false;
    c->compact_step = false;
    if (r) return r;
    HIPC(c, hipMemcpyAsync(record_out, c->crec, (size_t)c->c_bytes, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    c->host_cstep = true;
    return NP8_OK;
}

int np8_step_merge_compact(np8_ctx *c, const void *records, int32_t world, int32_t *halted) {
    if (!c || !records || !halted || world < 1) return NP8_ERR_ARG;
    if (world != c->world) return fail(c, NP8_ERR_ARG, "np8_step_merge_compact: world differs from np8_comm_init");
    if (!c->host_cstep) return fail(c, NP8_ERR_STATE, "np8_step_merge_compact: no np8_step_local_compact step pending");
    c->host_cstep = false;
    HIPC(c, hipMemcpyAsync(c->cgath, records, (size_t)c->c_bytes * world, hipMemcpyHostToDevice, c->stream));
    c->compact_step = true;  // (fin_args: the gathered compact records, their capacity, the local compact record)
    int r = launch_finalize(c, c->cgath, world);
    c->compact_step = false;
    if (r) return r;
    Ctl h;
    if ((r = read_ctl(c, &h))) return r;
    *halted = h.halt ? 1 : 0;
    if (!h.halt) {
        c->sub_next = (c->sub_next + 1) % c->substeps;
        return NP8_OK;
    }
    // some rank's requests did not fit its compact record: np8_finalize applied nothing; this step's full record
    // comes from the deltas the assign wrote into the compact record and every request of the staging area
    // (as recover_halt prepares it for the RCCL path)
    HIPC(c, hipMemsetD32Async(reinterpret_cast<int *>(&c->ctl->halt), 0, 1, c->stream));
    HIPC(c, hipMemcpyAsync(c->rec + kRecHeaderBytes, c->crec + kRecHeaderBytes, 4ull * c->kcap, hipMemcpyDeviceToDevice,
                           c->stream));
    HIPC(c, hipMemcpyAsync(&reinterpret_cast<RecHeader *>(c->stage)->nreq, &reinterpret_cast<RecHeader *>(c->crec)->nreq,
                           sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
    HIPC(c, hipMemsetAsync(c->crec, 0, kRecHeaderBytes + 4ull * c->kcap, c->stream));
    c->n_halts += 1;
    c->host_halted = true;
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;
}

int np8_step_resume(np8_ctx *c, void *record_out) {
    if (!c || !record_out) return NP8_ERR_ARG;
    if (!c->host_halted) return fail(c, NP8_ERR_STATE, "np8_step_resume: no halted compact step");
    c->host_halted = false;
    HIPC(c, np8_launch_req_select(c->stage, c->stage_cap, c->rec, c->rec_cap, c->kcap, c->D, c->req_max, nullptr, 0,
                                  c->stream));
    HIPC(c, hipMemcpyAsync(record_out, c->rec, (size_t)c->rec_bytes, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return NP8_OK;  // then the full records' all-gather and np8_step_merge, as after np8_step_local
}

// ---- Jain-Neal split-merge (np8_sm.hip; DESIGN.md "Split-merge") ------------------------------------
static SmArgs sm_args(np8_ctx *c) {
    SmArgs A;
    std::memset(&A, 0, sizeof(A));
    A.D = c->D;
    A.kcap = c->kcap;
    A.N = (int32_t)c->n_loc;
    A.K = c->sm_K;
    A.X = c->X;
    A.z = c->z;
    A.cnt = c->cnt;
    A.slot_mu = c->slot_mu;
    A.slot_P = c->slot_P;
    A.slot_c = c->slot_c;
    A.slot_iso = c->slot_iso;
    A.gp_iso = c->gp_iso;
    A.LT = c->d_LT;
    A.Gp = c->d_Gp;
    A.mu0 = c->d_mu0;
    A.caux = c->caux;
    A.rsk = c->rsk;
    A.nu = c->nu;
    A.log_alpha = std::log(c->alpha);
    A.seed = c->seed;
    A.t = c->epoch;
    A.perm0 = make_perm(c->seed ^ kSmPermKey[0], c->epoch, (uint32_t)c->n_loc);
    A.perm1 = make_perm(c->seed ^ kSmPermKey[1], c->epoch, (uint32_t)c->n_loc);
    for (int r = 0; r < 3; ++r) A.tperm[r] = make_perm(c->seed ^ kTriPermKey[r], c->epoch, (uint32_t)c->n_loc);
    // triadic rR (np_triadic_algorithm.cpp:116-131, beta = 0.5 at :63): 2 -> 1, 1 -> 2, 3 -> 2, 2 -> 3
    A.lrr[0] = -std::log(0.5);
    A.lrr[1] = std::log(0.5);
    A.lrr[2] = std::log(1.0 - 0.5);
    A.lrr[3] = -std::log(1.0 - 0.5);
    A.hist = c->sm_hist;
    A.nbk = (int32_t)((c->n_loc + kSmMemItems - 1) / kSmMemItems);
    A.mem = c->sm_mem;
    A.off = c->sm_off;
    A.dense = c->dense_of;
    A.live = c->sm_live;
    A.Xm = c->sm_Xm;
    A.ownm = c->sm_ownm;
    A.slist = c->sm_slist;
    A.stheta = c->sm_stheta;
    A.cross = c->sm_cross;
    A.sc = c->sm_ctl;
    A.typ = c->sm_typ;
    A.iso_walk = (c->sm_all_iso && c->gp_iso > 0.0) ? 1 : 0;
    A.mb = c->sm_mb_on ? c->sm_mb : nullptr;
    return A;
}

static constexpr int32_t kSmBatchMax = 1 << 20, kSmBatchMin = 1024;

static int sm_buffers(np8_ctx *c) {
    if (c->sm_n == c->n_loc) return NP8_OK;
    const int64_t nbk = (c->n_loc + kSmMemItems - 1) / kSmMemItems;
    int r;
    if ((r = dalloc(c, &c->sm_hist, (size_t)(c->kcap * (nbk > 0 ? nbk : 1)))) || (r = dalloc(c, &c->sm_mem, (size_t)c->n_loc)) ||
        (r = dalloc(c, &c->sm_off, (size_t)c->kcap + 1)) || (r = dalloc(c, &c->sm_live, (size_t)c->kcap)) ||
        (r = dalloc(c, &c->sm_ownm, (size_t)c->n_loc)) || (r = dalloc(c, &c->sm_Xm, (size_t)c->n_loc * c->D)) ||
        (r = dalloc(c, &c->sm_typ, (size_t)kSmBatchMax)) || (r = dalloc(c, &c->sm_slist, (size_t)kSmBatchMax)) ||
        (r = dalloc(c, &c->sm_stheta, (size_t)kSmBatchMax * (c->D + 1))) ||
        (!c->sm_mb && (r = dalloc(c, &c->sm_mb, (size_t)4 * c->kcap))))
        return r;
    if (!c->sm_ctl) {
        if ((r = dalloc(c, &c->sm_ctl, 1))) return r;
        HIPC(c, hipHostMalloc((void **)&c->sm_first_host, sizeof(int64_t)));
    }
    c->sm_n = c->n_loc;
    return NP8_OK;
}

// The state the attempts of a batch see: dense table, live count, member lists, own and cross.
static int sm_rebuild(np8_ctx *c, bool triadic) {
    int r = rebuild(c);
    if (r) return r;
    Ctl h;
    if ((r = read_ctl(c, &h))) return r;
    c->sm_K = h.K;
    if ((int64_t)h.K * h.K > c->sm_cross_cap) {
        const int64_t cap = std::max<int64_t>((int64_t)h.K * h.K, 64 * 64);
        if ((r = dalloc(c, &c->sm_cross, (size_t)cap))) return r;
        c->sm_cross_cap = cap;
    }
    Timer t;
    timer_begin(c, 4, t);
    HIPC(c, np8_launch_sm_members(sm_args(c), c->stream));
    c->sm_mb_on = triadic && !c->tri_bound_off;
    if (c->sm_mb_on) HIPC(c, np8_launch_tri_bound(sm_args(c), c->stream));  // the triadic merge bound's sums
    timer_end(c, t);
    int32_t all_iso = 0;  // every live slot isotropic: the triadic walk's fast form applies
    HIPC(c, hipMemcpyAsync(&all_iso, &c->sm_ctl->all_iso, sizeof(all_iso), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    c->sm_all_iso = all_iso != 0;
    return NP8_OK;
}

// n split-merge sweeps of one sampler: speculative attempt batches, the first accepted attempt
// applied, the state rebuilt, the batch restarted after it.
static int split_merge_sweeps(np8_ctx *c, int32_t n_sweeps, bool triadic) {
    const char *who = triadic ? "np8_tri_sweep" : "np8_sm_sweep";
    if (!c) return NP8_ERR_ARG;
    if (int r_ = settle(c)) return r_;  // a sharded replay still unchecked (np8_sweep)
    if (!c->have_state) return fail(c, NP8_ERR_STATE, std::string(who) + ": no state (np8_set_state/np8_init_random)");
    if (c->world > 1) return fail(c, NP8_ERR_ARG, std::string(who) + ": split-merge runs on one rank");
    if (c->wide || c->rt || c->prior != NP8_PRIOR_REFERENCE)
        return fail(c, NP8_ERR_ARG, std::string(who) + ": needs the reference prior and the fp64 contraction at D <= 16");
    if (c->n_loc > INT32_MAX) return fail(c, NP8_ERR_ARG, std::string(who) + ": at most 2^31-1 items");
    int r = flush_snapshot(c);
    if (r) return r;
    r = sm_buffers(c);
    if (r) return r;
    const int64_t N = c->n_loc;
    for (int s = 0; s < n_sweeps; ++s) {
        // the split-merge moves change z and the counts behind the label-sorted layout and the lists
        c->use_sorted = false;
        c->sorted_valid = false;
        c->lists_valid = c->r2_zero = c->collecting = false;
        if ((r = sm_rebuild(c, triadic))) return r;
        int64_t a = 0;
        while (a < N) {
            const int32_t nb = (int32_t)std::min<int64_t>(c->sm_batch, N - a);
            SmArgs A = sm_args(c);
            A.a0 = a;
            A.nb = nb;
            Timer t;
            timer_begin(c, 5, t);
            HIPC(c, triadic ? np8_launch_tri_eval(A, c->stream) : np8_launch_sm_eval(A, c->stream));
            timer_end(c, t);
            HIPC(c, hipMemcpyAsync(c->sm_first_host, &c->sm_ctl->first, sizeof(int64_t), hipMemcpyDeviceToHost,
                                   c->stream));
            HIPC(c, hipStreamSynchronize(c->stream));
            const int64_t first = *c->sm_first_host;
            if (first == INT64_MAX) {
                a += nb;
                c->sm_batch = (int32_t)std::min<int64_t>(2ll * c->sm_batch, kSmBatchMax);
                continue;
            }
            FinArgs F = fin_args(c, c->rec, 1);
            HIPC(c, triadic ? np8_launch_tri_apply(A, F, first, c->stream) : np8_launch_sm_apply(A, F, first, c->stream));
            if ((r = sm_rebuild(c, triadic))) return r;
            c->sm_batch = (int32_t)std::max<int64_t>(kSmBatchMin, std::min<int64_t>(kSmBatchMax, 2 * (first - a + 1)));
            a = first + 1;
        }
        if ((r = end_sweep(c))) return r;
    }
    return NP8_OK;
}

int np8_sm_sweep(np8_ctx *c, int32_t n_sweeps) { return split_merge_sweeps(c, n_sweeps, false); }

int np8_tri_sweep(np8_ctx *c, int32_t n_sweeps) { return split_merge_sweeps(c, n_sweeps, true); }

int np8_tri_stats(np8_ctx *c, int64_t out[10]) {
    if (!c || !out) return NP8_ERR_ARG;
    for (int k = 0; k < 10; ++k) out[k] = 0;
    if (!c->sm_ctl) return NP8_OK;
    SmCtl h;
    HIPC(c, hipMemcpyAsync(&h, c->sm_ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < 10; ++k) out[k] = h.tstats[k];
    return NP8_OK;
}

int np8_sm_stats(np8_ctx *c, int64_t out[6]) {
    if (!c || !out) return NP8_ERR_ARG;
    for (int k = 0; k < 6; ++k) out[k] = 0;
    if (!c->sm_ctl) return NP8_OK;
    SmCtl h;
    HIPC(c, hipMemcpyAsync(&h, c->sm_ctl, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < 6; ++k) out[k] = h.stats[k];
    return NP8_OK;
}

}  // extern "C"
