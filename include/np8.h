/*
 * np8.h -- C ABI of the MI355X (gfx950) Neal Algorithm 8 Gibbs sweep.
 *
 * This is the drop-in boundary for mrquincle/noparama's sampler plug-in
 *   class UpdateClusterPopulation { virtual void update(membertrix&, const data_ids_t&) = 0;
 *                                   virtual void printStatistics() = 0; }
 *   (reference include/np_update_cluster_population.h:13-44; Neal-8 implementation
 *    src/np_neal_algorithm8.cpp:17-176, constructed in src/np_main.cpp:433-438).
 * A C++ caller wraps it as `NealAlgorithm8Hip : UpdateClusterPopulation` (host/np_host.h);
 * a ctypes caller binds it directly (noparama_amd/np8.py).  Plain pointers and sizes only: the
 * library owns its device memory and copies host buffers in and out.
 *
 * Every entry point returns 0 on success or a negative np8_status; np8_last_error() has the text.
 * One host thread per context; contexts are independent (the reference is single-threaded and
 * non-reentrant: static RNGs in include/statistics/normal.h:61, multivariatenormal.cpp:41).
 */
#ifndef NP8_H
#define NP8_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct np8_ctx np8_ctx;

typedef enum {
    NP8_OK = 0,
    NP8_ERR_ARG = -1,      /* bad argument / unsupported configuration */
    NP8_ERR_SIGMA = -2,    /* a covariance with det <= 0 (reference would produce NaN weights) */
    NP8_ERR_RANGE = -3,    /* label or point index out of range */
    NP8_ERR_CAPACITY = -4, /* a fixed-size table is full (kcap / NP8_REQ_MAX limits of an entry point) */
    NP8_ERR_STATE = -5,    /* call order (no data / no state / no max-likelihood snapshot yet) */
    NP8_ERR_HIP = -6,      /* HIP runtime error (message has the HIP error string) */
    NP8_ERR_COMM = -7      /* RCCL error */
} np8_status;

#define NP8_REQ_MAX 4096     /* upper bound of np8_config.req_max */
#define NP8_REQ_DEFAULT 1024 /* req_max when the configuration gives 0 */

typedef struct {
    int32_t D;            /* dimension of the data items (data_t, include/np_data.h:9) */
    int32_t M;            /* auxiliary clusters per point; reference _M = 3 (np_neal_algorithm8.cpp:33) */
    double alpha;         /* DP concentration; reference alpha = 1 (np_main.cpp:164) */
    const double *mu0;    /* [D] G0 mean; reference (6,6) (np_main.cpp:368) */
    double kappa;         /* reference 1/500 (np_main.cpp:369) */
    double nu;            /* reference 4 (np_main.cpp:370); sd of the scale draw (invwishart.h:30-31) */
    const double *Lambda; /* [D*D] row-major, SPD; reference 0.01 I (np_main.cpp:371) */
    uint64_t seed;        /* Philox key: every draw is a pure function of (seed, point, epoch) */
    int32_t kcap;         /* cluster slot capacity (0 -> 2048) */
    int64_t chunk;        /* points per synchronous step: 0 = the whole sweep (data-parallel);
                             1 = the reference's exact sequential sweep (np_mcmc.cpp:146-164) */
    int32_t device;       /* HIP device ordinal, -1 = current */
    int32_t param_update; /* NP8_PARAM_*: cluster-parameter update after every sweep (np_mcmc.cpp:170) */
    int32_t mh_steps;     /* MH steps per cluster and sweep for NP8_PARAM_MH_G0; 0 -> 20 (np_mcmc.cpp:54) */
    int32_t prior;        /* NP8_PRIOR_*: the base measure G0 */
    int32_t contraction;  /* NP8_CONTRACT_*: arithmetic of the cluster likelihoods */
    int32_t req_max;      /* new clusters one synchronous step may create (0 -> NP8_REQ_DEFAULT, at most
                             NP8_REQ_MAX).  A step accepts the min(req_max, free slots, requests) requests of
                             lowest scan position; the other requesters keep their cluster until their next
                             update (DESIGN.md "Finalize").  Part of the chain's specification: the same
                             value gives the same chain on any number of ranks. */
    int32_t substeps;     /* the data-parallel sweep (chunk 0) as S synchronous sub-steps (0, 1 -> one step;
                             at most NP8_SUBSTEPS_MAX, and S * kcap <= 16384): sub-step s updates the items
                             with a fixed hash of the item index equal to s, against the state the earlier
                             sub-steps left (DESIGN.md "Sub-steps").  One step updates every item against
                             the same state; more sub-steps bring the chain's statistics to the sequential
                             sweep's (tests/test_gpu_chain_stats.py) at S launches of each step kernel.
                             NP8_SUBSTEPS_AUTO: chosen by np8_set_data from n_global (see below). */
} np8_config;

#define NP8_SUBSTEPS_MAX 64
/* np8_config.substeps = NP8_SUBSTEPS_AUTO: NP8_SUBSTEPS_AUTO_S sub-steps (or the most kcap allows) when the data set
 * has at most NP8_SUBSTEPS_AUTO_N items, one step above.  One synchronous step over-splits small data (twogaussians,
 * N = 200: K 15.6 vs the sequential sampler's 12.5) while 16 sub-steps hold SURVEY 8(d)'s tolerance; at N >= 1e5 one
 * step scores like 16 (tests/test_gpu_chain_stats.py).  The choice depends on n_global only, so every rank of a
 * sharded run makes the same one; np8_stats reports it (np8_stats_t.substeps). */
#define NP8_SUBSTEPS_AUTO (-1)
#define NP8_SUBSTEPS_AUTO_N 8192
#define NP8_SUBSTEPS_AUTO_S 16

/* ABI growth.  np8_config and np8_stats_t only ever grow at their end, and the entry points that take them have
 * sized forms that honour the caller's size: np8_create_sized reads the first cfg_bytes of the configuration (the
 * fields the caller does not have take their 0 = default values) and np8_stats_sized writes exactly
 * min(out_bytes, sizeof(np8_stats_t)) bytes, so a caller built against an older or newer header never has its
 * memory read or written past the struct it allocated.  Use NP8_CREATE / NP8_STATS, which pass sizeof of the
 * caller's own struct.  The unsized forms: np8_create reads sizeof(np8_config) of this header (callers built
 * against this header only); np8_stats writes the first NP8_STATS_MIN_BYTES (the first, smallest layout ever
 * shipped: K .. last_loglik) and nothing beyond, whatever header the caller was built with.
 * BEHAVIOUR CHANGE (round 5): a binary built against the round-4 header that calls the unsized np8_stats and reads
 * ms_assign .. pick_evals now finds those fields untouched (the library cannot tell a round-3 struct from a
 * round-4 one, and writing the round-4 layout overran round-3 callers).  Such callers must zero their struct
 * before the call or move to NP8_STATS; INTEGRATION.md "ABI growth" says the same. */
#define NP8_CONFIG_MIN_BYTES offsetof(np8_config, param_update) /* D .. device: the first released layout */

/* Cluster-likelihood arithmetic (DESIGN.md "Wide path", "Run-time D").
 * F64:      fp64 table form (packed sym(Sigma^{-1})), the reference's arithmetic: any D from 1 to 16 with M = 3 (the
 *           reference's), and M in {1, 2, 3, 4} for D in {1, 2, 3, 4, 8, 16} (templated kernels); any D from 9 to
 *           128 with any M <= 8 otherwise (np8_rt.hip: D and M at run time; reference prior, param_update FROZEN;
 *           bit-exact against oracle/'s F64 path, tests/test_gpu_rt.py).
 * F32_MFMA: 16 < D <= 80 (config C5: D = 64; tables padded with zero rows to D rounded up to 16; the NIW prior up to
 *           D = 64): items held in fp32, (x-mu)^T Sigma^{-1} (x-mu) = |A (x-mu)|^2 with
 *           A = fp32(chol(sym Sigma^{-1})) contracted on the matrix cores (v_mfma_f32_16x16x4_f32),
 *           |.|^2 in fp32, the draws and the pick in fp64; bit-exact against oracle/ (NP8O_CONTRACT_F32)
 *           and within 1e-5 relative of the fp64 formula.  param_update FROZEN or NIW_CONJUGATE. */
#define NP8_CONTRACT_F64 0
#define NP8_CONTRACT_F32_MFMA 1

/* Base measure G0 (dirichlet_process::sample_base, include/statistics/dirichlet.h:91-93).
 * REFERENCE: normal_inverse_wishart_distribution as the reference actually draws it
 *            (normalinvwishart.h:44-64, invwishart.h:30-46): v ~ N(D, nu), Sigma = v^2 chol(Lambda)^T
 *            chol(Lambda), mu ~ N(mu0, Sigma/kappa).
 * NIW:       a proper Normal-Inverse-Wishart(mu0, kappa0 = kappa, nu0 = nu, Psi0 = Lambda):
 *            Sigma ~ IW(Psi0, nu0), mu | Sigma ~ N(mu0, Sigma/kappa0); needs nu0 >= D + 1.  The
 *            extension config C5 of BASELINE.json runs on. */
#define NP8_PRIOR_REFERENCE 0
#define NP8_PRIOR_NIW 1

/* Cluster-parameter update (UpdateClusters::update, src/np_update_clusters.cpp:71-142).
 * FROZEN: parameters never change -- the reference's effective behaviour, because its accepted
 *         proposal is sliced away in cluster_t::setSuffies.
 * MH_G0:  what the reference intends: mh_steps independence-MH steps per live cluster with G0
 *         proposals, evaluated from per-cluster sufficient statistics on the device. */
/* NIW_CONJUGATE (NIW prior): every live cluster's (mu, Sigma) drawn from its exact Normal-Inverse-
 *         Wishart posterior given its items -- the Gibbs update the reference leaves as a stub
 *         (normal_inverse_wishart_distribution::update, include/statistics/normalinvwishart.h:66-75). */
#define NP8_PARAM_FROZEN 0
#define NP8_PARAM_MH_G0 1
#define NP8_PARAM_NIW_CONJUGATE 2

typedef struct {
    int32_t K;                  /* live clusters */
    uint32_t epoch;             /* sweeps completed */
    int64_t new_clusters;       /* cumulative "new cluster" events (np_statistics.h step[0].accept) */
    int64_t existing_picks;     /* cumulative "existing cluster" events (step[0].reject) */
    int64_t rejected_requests;  /* new-cluster requests not accepted in their step (req_max or no free slot):
                                   those items kept their cluster until their next update */
    double best_loglik;         /* max over checks of sum_i log p(x_i | theta_z_i) (np_mcmc.cpp:187-203) */
    double last_loglik;
    double ms_assign, ms_finalize, ms_loglik; /* accumulated device time (when timing is enabled) */
    int64_t mh_accepted;        /* cumulative accepted parameter proposals (NP8_PARAM_MH_G0) */
    double ms_params;           /* accumulated device time of the parameter update */
    /* launches behind ms_assign, ms_finalize, ms_loglik, ms_params: every launch when sweeps run one
     * by one; one np8_assign launch per replay when they run from a captured 20-sweep graph */
    int64_t n_timed_assign, n_timed_finalize, n_timed_loglik, n_timed_params;
    /* split-merge (np8_sm_sweep): device time of the state rebuilds (member lists, own and cross
     * likelihoods) and of the attempt batches, and the launches behind them */
    double ms_sm_members, ms_sm_eval;
    int64_t n_timed_sm_members, n_timed_sm_eval;
    /* executed work of the assign kernel while NP8_TIMING_COUNTERS is on (cumulative): cluster quadratic forms
     * evaluated per item (its own cluster included; rows left out by candidate pruning are not), and
     * how many of them took the isotropic form iso |x - mu|^2 */
    int64_t n_quad, n_quad_iso;
    /* NP8_TIMING_COUNTERS self-check of the auxiliary screen (DESIGN.md "Auxiliary screen"): lanes whose
     * screened-out auxiliary would not have been skipped by the pick.  0 unless the screen's margin is wrong. */
    int64_t screen_violations;
    /* NP8_TIMING_COUNTERS: (item, auxiliary) pairs the screen did not skip (the exact fp64 draw ran), and
     * (wave, auxiliary) pairs where at least one of the wave's 64 items needed it */
    int64_t aux_exact_lanes, aux_exact_waves;
    /* NP8_TIMING_COUNTERS, how the candidate walk went: lanes that walked the whole table (no usable list, or
     * outside the radius their list was built for) and waves with at least one such lane (the whole wave
     * pays the table loop); waves of more own rows than the list walk takes (a stale layout); list entries
     * walked by lanes */
    int64_t full_walk_lanes, full_walk_waves, many_group_waves, list_entries;
    /* how the per-sweep bookkeeping ran (DESIGN.md §5 "Fewer launches per sweep"): max-likelihood checks folded
     * into the data-parallel step (cumulative), candidate-list rebuilds by the conditional step tail (steps whose
     * counts moved beyond the lists' slack), and steps that kept the lists of the last build */
    int64_t folded_checks, tail_list_builds, tail_steps;
    /* NP8_TIMING_COUNTERS: walked candidate rows within kSkip (80 nats) of the running maximum, i.e. that pay the
     * pick's exp and division (cumulative) */
    int64_t pick_evals;
    /* RCCL path: steps of a compact sweep graph whose requests did not fit the compact records; each
     * halted its graph on every rank and was resumed by the host with the full records (cumulative) */
    int64_t compact_halts;
    /* the sub-steps of the data-parallel sweep in use (np8_config.substeps; NP8_SUBSTEPS_AUTO resolved by
     * np8_set_data) */
    int64_t substeps;
} np8_stats_t;

#define NP8_STATS_MIN_BYTES offsetof(np8_stats_t, ms_assign) /* K .. last_loglik: the first released layout */

/* Create / destroy.  Replaces NealAlgorithm8::NealAlgorithm8 (np_neal_algorithm8.cpp:17-34). */
int np8_create(np8_ctx **out, const np8_config *cfg);
/* np8_create reading only the first cfg_bytes of *cfg (>= NP8_CONFIG_MIN_BYTES); see "ABI growth" above */
int np8_create_sized(np8_ctx **out, const np8_config *cfg, size_t cfg_bytes);
#define NP8_CREATE(out, cfg) np8_create_sized((out), (cfg), sizeof *(cfg))
int np8_destroy(np8_ctx *ctx);
const char *np8_last_error(const np8_ctx *ctx);

/* Data items, row-major [n][D] (membertrix::addData, membertrix.cpp:120-138).  For a data-parallel
 * run over several ranks, pass this rank's contiguous shard [offset, offset+n) of n_global items. */
int np8_set_data(np8_ctx *ctx, const double *X, int64_t n, int32_t D, int64_t offset, int64_t n_global);

/* Explicit state: labels z[n] in [0,K) and per-cluster mu [K*D], Sigma [K*D*D] (row-major).
 * Sigma is used as the reference uses it: inverse and determinant of the matrix as given
 * (multivariatenormal.cpp:87,90), so a non-symmetric Sigma is accepted (test_mvn_likelihood.cpp:20). */
int np8_set_state(np8_ctx *ctx, const int32_t *z, int32_t K, const double *mu, const double *Sigma);
/* Same with the global cluster sizes given by the caller (counts[K]); for sharded runs whose
 * records move over the caller's transport (np8_step_local / np8_step_merge), where no device
 * reduction of the per-rank label counts is available. */
int np8_set_state_counts(np8_ctx *ctx, const int32_t *z, int32_t K, const double *mu, const double *Sigma,
                         const int64_t *counts);

/* Reference initialisation: K_init G0 draws, uniform random assignment, cleanup of empty clusters
 * (np_mcmc.cpp:49-92, np_init_clusters.cpp:24-40). */
int np8_init_random(np8_ctx *ctx, int32_t K_init);

/* n full sweeps (np_mcmc.cpp:109-175 with the population update of np_neal_algorithm8.cpp:49-167),
 * including the max-likelihood check every 5th sweep (np_mcmc.cpp:172-174).  Asynchronous on the
 * context's stream; errors raised on the device are reported by the next np8_sync().
 * With an RCCL communicator (np8_comm_init) np8_sweep is collective -- every rank calls it with the same n --
 * and returns once its last sweep graph is settled (a replay that halted on a compact record is resumed inside
 * the call), so the other entry points never run collectives: one rank may alone ask for statistics, the state
 * or a checkpoint.  Every rank of a communicator needs at least one item. */
int np8_sweep(np8_ctx *ctx, int32_t n_sweeps);
/* Prepares the next np8_sweep(ctx, n_sweeps) without running anything: captures and uploads the
 * 20-sweep graph it would replay (whole synchronous sweeps on one rank), so that capture and
 * instantiation are not paid inside the caller's timed region.  A no-op when no graph applies. */
int np8_prepare_sweeps(np8_ctx *ctx, int32_t n_sweeps);

/* Jain-Neal split-merge sweeps: the reference's `-a jain_neal_split` population update
 * (class JainNealAlgorithm, include/np_jain_neal_algorithm.h:52-98, update() at
 * src/np_jain_neal_algorithm.cpp:424-502), driven as src/np_mcmc.cpp:117-164 drives it (subset_count = 2,
 * np_main.cpp:440-445): each sweep makes N attempts on the item pairs of two scan permutations -- a
 * split of their common cluster (sams_prior allocation, new cluster from G0) or a merge of the first
 * item's cluster into the second's -- then the end-of-sweep step of np8_sweep (parameter update,
 * max-likelihood check).  Single rank, reference prior, fp64 contraction (any D <= 16).
 * Synchronous: returns when the sweeps are done. */
int np8_sm_sweep(np8_ctx *ctx, int32_t n_sweeps);
/* Cumulative attempt outcomes (the reference's _statistics.step[], np_jain_neal_algorithm.cpp:505-530):
 * [0] pairs skipped (equal items, np_mcmc.cpp:153-156), [1] splits rejected, [2] merges rejected,
 * [3] splits accepted, [4] merges accepted, [5] splits accepted by the ratio but dropped for want of a
 * free slot (kcap live clusters). */
int np8_sm_stats(np8_ctx *ctx, int64_t out[6]);

/* Triadic split-merge sweeps: the reference's `-a triadic` population update (class TriadicAlgorithm,
 * include/np_triadic_algorithm.h, update() at src/np_triadic_algorithm.cpp:633-795), driven with
 * subset_count = 3 (np_main.cpp:447-455): each sweep makes N attempts on the item triples of three scan
 * permutations -- a dyadic split 1 -> 2, a dyadic merge 2 -> 1 (probability beta = 0.5), a triadic
 * split 2 -> 3 or a triadic merge 3 -> 2, every member of the involved clusters reallocated by the
 * sams_prior proposal -- then the end-of-sweep step.  Same restrictions as np8_sm_sweep. */
int np8_tri_sweep(np8_ctx *ctx, int32_t n_sweeps);
/* Cumulative outcomes (the reference's _statistics.step[0..3], np_triadic_algorithm.cpp:797-832):
 * [0] triples skipped, [1]/[2] dyadic merges rejected/accepted, [3]/[4] dyadic splits, [5]/[6] triadic
 * merges (3 -> 2), [7]/[8] triadic splits (2 -> 3), [9] splits accepted by the ratio but dropped for want
 * of a free slot. */
int np8_tri_stats(np8_ctx *ctx, int64_t out[10]);

/* The population update of one sweep alone (np_mcmc.cpp:146-164: every item once, in chunks of `chunk`
 * against the state frozen at chunk start; chunk 0 = one data-parallel step), without the end-of-sweep
 * step: np8_sweep(ctx, 1) == np8_population_sweep + np8_end_sweep.  For callers that drive the reference's
 * MCMC::run loop themselves (UpdateClusters and considerMaxLikelihood on their own membertrix). */
int np8_population_sweep(np8_ctx *ctx);

/* Membership change log, for callers that keep their own membertrix coherent with the device (the
 * reference's MCMC::run reads it back every sweep: relabel np_mcmc.cpp:111-114, UpdateClusters :170,
 * considerMaxLikelihood :172-203; the plug-in mutates it in place, np_neal_algorithm8.cpp:62-64,139-157).
 * np8_track_changes(ctx, NP8_CHANGES_FROM_NOW) takes the current state as the baseline;
 * NP8_CHANGES_FROM_EMPTY starts from "no item assigned, no cluster", so the first np8_changes delivers the
 * whole state; 0 stops tracking.  np8_changes reports what differs from the baseline and makes the
 * current state the new baseline:
 *   item[0..n_moved) ascending, slot[..]: items (local indices) whose cluster changed and their new slot;
 *   created[0..n_created): slots that became live (membertrix::addCluster, membertrix.cpp:87-100);
 *   removed[0..n_removed): slots that became empty (retract's auto-remove, membertrix.cpp:200-203);
 *   updated[0..n_updated): slots live before and after whose parameters changed (the parameter update,
 *   or a slot emptied and re-used in between);
 *   mu [(n_created + n_updated) * D], Sigma [.. * D * D]: parameters of the created, then updated slots.
 * Slot ids are stable while a cluster lives: they are the cluster ids of a coherent membertrix.
 * created/removed/updated need room for kcap entries and mu/Sigma for kcap clusters (either may be NULL).
 * More moved items than item_cap: NP8_ERR_CAPACITY, out->n_moved set, the baseline unchanged.
 * Cost: one pass over the labels and the slot tables on the device; transfers O(changes). */
#define NP8_CHANGES_FROM_NOW 1
#define NP8_CHANGES_FROM_EMPTY 2
typedef struct {
    int64_t n_moved;
    int32_t n_created, n_removed, n_updated, pad;
} np8_changes_t;
int np8_track_changes(np8_ctx *ctx, int32_t mode);
int np8_changes(np8_ctx *ctx, int64_t item_cap, int64_t *item, int32_t *slot, int32_t *created, int32_t *removed,
                int32_t *updated, double *mu, double *Sigma, np8_changes_t *out);

/* The reference's per-call granularity: sequential single-point updates of the listed items, in
 * order, at the current epoch (NealAlgorithm8::update with data_ids.size()==1).  Call
 * np8_end_sweep() after the last point of a sweep. */
int np8_update_points(np8_ctx *ctx, const int64_t *ids, int64_t n);
int np8_end_sweep(np8_ctx *ctx);

/* Checkpoint / resume: the complete chain state -- labels as slots, every slot's parameters
 * and count, the epoch, the max-likelihood snapshot and its log-likelihood, the cumulative counters --
 * as raw bits in a flat buffer of np8_checkpoint_bytes() bytes.  np8_restore on a context of the same
 * configuration, seed and data (np8_set_data first) continues the chain bit for bit as if it had never
 * stopped (every draw is a function of (seed, item, epoch); the slot layout is kept). */
int64_t np8_checkpoint_bytes(np8_ctx *ctx);
int np8_checkpoint(np8_ctx *ctx, void *out, int64_t bytes);
int np8_restore(np8_ctx *ctx, const void *in, int64_t bytes);

/* Debug invariants: every label names a live slot, the live slots' counts equal the label
 * histogram (one rank) and sum to the global item count, K equals the live slots, the dense candidate
 * table holds exactly the live slots.  out[0]: violated bits (1 labels, 2 histogram, 4 sum, 8 K/table),
 * out[1] bad labels, out[2] slots whose count differs, out[3] the sum of counts.  NP8_ERR_STATE when
 * violated.  With the environment variable NP8_DEBUG_INVARIANTS=1 the check also runs at the end of every
 * sweep and a violation is reported by the next np8_sync. */
int np8_check_invariants(np8_ctx *ctx, int64_t out[4]);

/* Waits for queued work; returns the first device-side error since the last sync. */
int np8_sync(np8_ctx *ctx);

/* State out: which = 0 current, 1 max-likelihood snapshot (MCMC::getMaxLikelihoodMatrix,
 * np_mcmc.cpp:183-185).  Labels are dense 0..K-1 in ascending slot order.  Any pointer may be NULL;
 * mu/Sigma/counts need room for kcap clusters. */
int np8_get_state(np8_ctx *ctx, int32_t which, int32_t *z, int32_t *K, double *mu, double *Sigma, int64_t *counts);

/* Parity/debug: log-likelihood of the listed items (local indices) against every live cluster
 * (ascending slot order) and then against the M auxiliary draws of the current epoch;
 * out is n x (K+M) with K = current live count.  Same arithmetic as the sweep kernel. */
int np8_loglik_matrix(np8_ctx *ctx, const int64_t *idx, int64_t n, double *out);

/* Parity/debug: the sweep's categorical draw (DESIGN.md "Pick": the single-uniform reservoir over
 * log-weights with the -80 skip rule, np8_assign's pick_step) on caller-given log-weights: out[k] = the
 * candidate picked from lw[0..n) with uniform u[k] in (0,1), candidate 0 taking the place of the item's own
 * cluster.  Replaces algebra::random_weighted_pick (include/helper/dim1algebra.hpp:2078-2104) called at
 * np_neal_algorithm8.cpp:126; tests/test_gpu_pick.py checks it against the oracle and, in distribution,
 * against the reference function itself. */
int np8_pick_batch(np8_ctx *ctx, const double *lw, int32_t n, const double *u, int64_t n_draws, int32_t *out);

/* Debug: the level-0 auxiliary screen's upper bound (DESIGN.md "Auxiliary screen": from the item's prefix call alone,
 * the supremum over the auxiliary's other draws in closed form, without the threshold's own margin term) of each
 * listed item's M auxiliary log-likelihoods at the current epoch, out[n][M]; the reference prior's fp64 path only.
 * np8_assign_fast skips auxiliary m of an item when this bound lies below its running maximum by kSkip;
 * tests/test_gpu_screen.py holds it above the exact values np8_loglik_matrix returns. */
int np8_aux_bounds(np8_ctx *ctx, const int64_t *idx, int64_t n, double *out);

/* Sum over items of log p(x_i | theta_{z_i}) for the current state (MCMC::considerMaxLikelihood). */
int np8_total_loglik(np8_ctx *ctx, double *out);

/* Writes exactly min(out_bytes, sizeof(np8_stats_t)) bytes of the statistics (out_bytes >= NP8_STATS_MIN_BYTES);
 * np8_stats writes the first NP8_STATS_MIN_BYTES only (see "ABI growth"). */
int np8_stats_sized(np8_ctx *ctx, np8_stats_t *out, size_t out_bytes);
int np8_stats(np8_ctx *ctx, np8_stats_t *out);
#define NP8_STATS(ctx, out) np8_stats_sized((ctx), (out), sizeof *(out))
/* enable = NP8_TIMING_EVENTS: device-event timing of the kernels (event pairs around each launch, or
 * around one assign launch per replayed sweep graph); NP8_TIMING_COUNTERS: the assign kernel counts the
 * quadratic forms it executes (np8_stats_t.n_quad; a few scalar loads and two atomics per wave); 0 = off.
 * Any non-zero value without the counter bit is the events alone. */
#define NP8_TIMING_EVENTS 1
#define NP8_TIMING_COUNTERS 2
/* with NP8_TIMING_EVENTS: a replayed sweep graph times every assign launch (default: one per replay) */
#define NP8_TIMING_ALL_ASSIGNS 4
int np8_set_timing(np8_ctx *ctx, int32_t enable);
/* Launch on this stream instead of the context's own (hipStream_t as void*). */
int np8_set_stream(np8_ctx *ctx, void *stream);

/* Multi-GPU: one context per rank.  Rank 0 makes an id, the caller broadcasts the 128 bytes, every
 * rank calls np8_comm_init.  Each sweep then exchanges one fixed-size record per rank (count deltas
 * and new-cluster requests) with one ncclAllGather over xGMI; cluster tables stay replicated. */
int np8_comm_unique_id(uint8_t out[128]);
int np8_comm_init(np8_ctx *ctx, const uint8_t id[128], int32_t rank, int32_t world);

/* Host-exchange variant of the same protocol (for callers that move the record themselves, e.g.
 * over MPI or gloo): np8_comm_init(ctx, NULL, rank, world), then per sweep, once per sub-step
 * (np8_config.substeps times), np8_step_local (writes this rank's record), the caller all-gathers
 * np8_record_bytes() bytes from every rank in rank order, np8_step_merge(gathered, world); then
 * np8_end_sweep.  The max-likelihood check then uses this
 * rank's partial sum only. */
int64_t np8_record_bytes(np8_ctx *ctx);
int np8_step_local(np8_ctx *ctx, void *record_out);
int np8_step_merge(np8_ctx *ctx, const void *records, int32_t world);

/* Compact records over the caller's transport: the exchange an RCCL sweep graph runs, step by step.
 * np8_step_local_compact writes this rank's compact record (np8_compact_record_bytes() bytes: the count deltas and
 * the first NP8_COMPACT_REQ requests, its header counting all of them); the caller all-gathers them in rank order;
 * np8_step_merge_compact applies them, or -- when some rank's requests did not fit its compact record, which every
 * rank sees alike in the gathered headers -- applies nothing and sets *halted = 1.  After a halt every rank calls
 * np8_step_resume (this rank's full record of the same step, np8_record_bytes() bytes), the caller all-gathers those
 * and calls np8_step_merge as after np8_step_local.  The chain is the full records' chain bit for bit.
 * np8_compact_record_bytes() is 0 where the step cannot use them (on the fp64 path: the NIW prior, rows that are not
 * isotropic, D and M without a templated instance; NP8_COMPACT_REQ=0, or a context without the host transport): use
 * np8_step_local there.  The wide path (NP8_CONTRACT_F32_MFMA, any prior and parameter update) has them.
 * Replaces, for the sharded sweep, the per-point exchange-free loop of np_mcmc.cpp:146-164. */
int64_t np8_compact_record_bytes(np8_ctx *ctx);
int np8_step_local_compact(np8_ctx *ctx, void *record_out);
int np8_step_merge_compact(np8_ctx *ctx, const void *records, int32_t world, int32_t *halted);
int np8_step_resume(np8_ctx *ctx, void *record_out);

/* Host-exchange form of the cluster-parameter update (param_update != FROZEN): after the sweep's
 * np8_step_merge, np8_param_stats_local writes this rank's per-cluster statistics (np8_param_stats_bytes()
 * bytes: kcap rows of D + D(D+1)/2 doubles), the caller sums them over ranks (an all-reduce), and
 * np8_end_sweep_stats(summed) ends the sweep: the parameter update from the global statistics, then
 * the bookkeeping of np8_end_sweep. */
int64_t np8_param_stats_bytes(np8_ctx *ctx);
int np8_param_stats_local(np8_ctx *ctx, double *stats_out);
int np8_end_sweep_stats(np8_ctx *ctx, const double *summed_stats);

#ifdef __cplusplus
}
#endif
#endif
