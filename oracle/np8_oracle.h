/*
 * np8_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, single thread) of mrquincle/noparama's Neal Algorithm 8 Gibbs sweep
 * for a Dirichlet-process mixture of multivariate normals.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline -- never as the product path.  The product is noparama_amd/csrc (HIP, gfx950).
 *
 * Two layers:
 *   1. Faithful restatements of the reference functions, cited file:line, used to pin numbers:
 *        np8o_mvn_probability_ref / np8o_mvn_logprobability_ref  (src/statistics/multivariatenormal.cpp)
 *        np8o_weighted_pick_ref                                (include/helper/dim1algebra.hpp)
 *        np8o_similarity                                       (src/clustering_performance.cpp)
 *   2. The chain itself (np8o_ctx): the reference sampler's semantics (src/np_neal_algorithm8.cpp:49-167
 *      driven by src/np_mcmc.cpp:48-175) generalised to a `chunk` of points evaluated against a frozen
 *      state (chunk = 1 is exactly the reference's sequential sweep).  Randomness comes from keyed
 *      Philox4x32-10 streams instead of std::default_random_engine so that the HIP path can be
 *      checked against it assignment for assignment (see DESIGN.md "Chain specification").
 *
 * Parity pinning: the likelihood is pinned by the reference's only known-answer test
 * (test/test_mvn_likelihood.cpp:30-44); the weighted pick is pinned by compiling the reference's own
 * header (oracle/ref_pick_harness.cpp -> oracle/_ref/); Philox by Random123/rocRAND known answers;
 * the metrics by sklearn.  G0 and the chain have no reference fixture (the reference is unseeded,
 * src/np_main.cpp:180): they are pinned by moment tests and by the statistical comparison of
 * chunk=1 chains, see DESIGN.md.
 */
#ifndef NP8_ORACLE_H
#define NP8_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NP8O_DMAX 128
#define NP8O_MMAX 8
#define NP8O_KCAP_PICK 4096 /* kcap limit of NP8O_PICK_INVCDF (the weights of one update live on the stack) */
#define NP8O_REQMAX 4096 /* upper bound of req_max (must match NP8_REQ_MAX) */
#define NP8O_REQ_DEFAULT 1024 /* default req_max (must match NP8_REQ_DEFAULT) */
/* Item keys: the Philox item counter of a draw is key = item | (visit << 32), visit = how many times
 * the item was already updated in this epoch (0 in every sweep; repeated np8o_update_points calls on
 * the same item within one epoch get fresh draws). */
#define NP8O_ITEM(key) ((int64_t)((uint64_t)(key) & 0xFFFFFFFFull))

/* Philox stream ids (high byte of counter word 3). */
enum {
    NP8O_STREAM_AUX = 1,
    NP8O_STREAM_PICK = 2,
    NP8O_STREAM_INIT_THETA = 3,
    NP8O_STREAM_INIT_Z = 4,
    NP8O_STREAM_PARAM = 5,  /* MH proposal normals: i = slot, calls step*Q .. */
    NP8O_STREAM_PARAM_U = 6, /* MH acceptance uniform: i = slot, call = step */
    NP8O_STREAM_AUX_DIR = 7, /* direction of a picked auxiliary's xi orthogonal to the item; NIW:
                                the Bartlett off-diagonals and z_perp direction of a picked auxiliary */
    NP8O_STREAM_AUX_NIW = 8, /* NIW prior: the auxiliary's Bartlett chi^2 draws, chi^2_{D-1}, z_1 */
    NP8O_STREAM_SM_THETA = 9,  /* split-merge: G0 draw of a split's new cluster (i = attempt) */
    NP8O_STREAM_SM_ALLOC = 10, /* split-merge: SAMS allocation uniforms (i = attempt, call = member rank) */
    NP8O_STREAM_SM_ACCEPT = 11, /* split-merge: acceptance uniform (i = attempt) */
    NP8O_STREAM_AUX_PRE = 12   /* reference prior: the auxiliaries' chi^2 prefixes (i = item, call 0) */
};

/* Base measure G0 (DESIGN.md "Priors").
 *   REFERENCE: the reference's normal_inverse_wishart_distribution as it actually draws
 *              (v ~ N(D, nu), Sigma = v^2 L^T L, mu ~ N(mu0, Sigma/kappa)).
 *   NIW:       a proper Normal-Inverse-Wishart(mu0, kappa0, nu0, Psi0) (build extension for config C5:
 *              Sigma ~ IW(Psi0, nu0), mu | Sigma ~ N(mu0, Sigma/kappa0)); hyper-parameters come in the
 *              same fields (mu0, kappa, nu, Lambda = Psi0), nu0 >= D + 1. */
enum { NP8O_PRIOR_REFERENCE = 0, NP8O_PRIOR_NIW = 1 };

/* Cluster-parameter update after each sweep (np_mcmc.cpp:170). */
/* NIW_CONJUGATE (NIW prior only): every live cluster's (mu, Sigma) drawn from its exact NIW posterior
 * given the cluster's items (the Gibbs step the reference's stubbed NIW update would be,
 * include/statistics/normalinvwishart.h:66-75). */
enum { NP8O_PARAM_FROZEN = 0, NP8O_PARAM_MH_G0 = 1, NP8O_PARAM_NIW_CONJUGATE = 2 };

/* ---- primitives ---------------------------------------------------------------------------- */
void np8o_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double np8o_u01(uint32_t hi, uint32_t lo);
/* n-th standard normal of stream (i, t, stream) under key seed. */
double np8o_normal(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t n);
double np8o_uniform(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t n);
uint32_t np8o_perm(uint64_t seed, uint32_t t, uint32_t N, uint32_t p);
/* Elementary functions of the specification (identical polynomials in the HIP code). */
double np8o_exp_le0(double x);
double np8o_log_pos(double u);
void np8o_sincos_2pi(double t, double *sn, double *cs);

/* ---- faithful reference restatements ------------------------------------------------------- */
/* multivariatenormal.cpp:64-94 (clustering branch :82-93): exp(-0.5 d'Inv d)/sqrt((2pi)^D det). */
double np8o_mvn_probability_ref(const double *x, const double *mu, const double *Sigma, int D);
/* multivariatenormal.cpp:106-136: exponent - log(sqrt((2pi)^D det)). */
double np8o_mvn_logprobability_ref(const double *x, const double *mu, const double *Sigma, int D);
/* dim1algebra.hpp:2078-2104 with the uniform u supplied by the caller. */
int64_t np8o_weighted_pick_ref(const double *w, int64_t n, double u);
/* The specification's reservoir pick (DESIGN.md "Pick") over log-weights lw[0..n) with uniform u:
 * the state starts at candidate 0 (T = lw[0], S = 1), then candidates 1..n-1 in order, skip rule
 * included.  Exactly what a point update runs (candidate 0 = the item's own cluster). */
int64_t np8o_pick_reservoir(const double *lw, int64_t n, double u);
/* Batch form: out[k] = np8o_pick_reservoir(lw, n, u[k]) for k < n_draws. */
void np8o_pick_reservoir_batch(const double *lw, int64_t n, const double *u, int64_t n_draws, int32_t *out);
/* LU with partial pivoting (Eigen PartialPivLU): inverse (row-major) and determinant. 0 = ok. */
int np8o_lu_inverse_det(const double *A, int D, double *inv, double *det);
/* clustering_performance.cpp:14-82 in int64/double: out = {purity, rand_index, adjusted_rand_index}. */
void np8o_similarity(const int32_t *truth, const int32_t *result, int64_t n, double out[3]);

/* ---- the chain ------------------------------------------------------------------------------- */
typedef struct np8o_ctx np8o_ctx;

typedef struct {
    int32_t D, M;
    double alpha;
    double mu0[NP8O_DMAX];
    double kappa, nu;
    double Lambda[NP8O_DMAX * NP8O_DMAX];
    uint64_t seed;
    int32_t kcap;
    int64_t chunk; /* 0 => N (synchronous sweep) */
    int32_t param_update; /* NP8O_PARAM_*: frozen = the reference's effective behaviour */
    int32_t mh_steps;     /* MH steps per cluster and sweep (np_mcmc.cpp:54: 20); 0 -> 20 */
    int32_t prior;        /* NP8O_PRIOR_* */
    int32_t contraction;  /* NP8O_CONTRACT_*: arithmetic of the cluster likelihoods */
    int32_t req_max;      /* new clusters one step may create (0 -> NP8O_REQ_DEFAULT, <= NP8O_REQMAX) */
    int32_t pick;         /* NP8O_PICK_*: the categorical draw of a point update */
    int32_t substeps;     /* data-parallel sweep (chunk = 0) in S synchronous sub-steps (0, 1 -> one step):
                             sub-step s updates the items i with np8o_substep_of(seed, i, S) == s, in
                             ascending s, each against the state the previous sub-steps left */
} np8o_config;

/* Sub-step of item i in a data-parallel sweep of S sub-steps: a fixed hash partition of the items
 * (identical in noparama_amd/csrc/np8_device.h substep_of). */
uint32_t np8o_substep_of(uint64_t seed, int64_t i, uint32_t S);

/* Categorical draw of a point update.
 *   RESERVOIR: the specification (DESIGN.md "Pick"), what the HIP path runs.
 *   INVCDF:    the reference's own rule (dim1algebra.hpp:2078-2104: cumulative sum of linear weights,
 *              lower_bound of u * total) over w_j = exp(lw_j - max lw) in the candidate order, with the
 *              same uniform -- an independent sampler to compare chains with in distribution. */
enum { NP8O_PICK_RESERVOIR = 0, NP8O_PICK_INVCDF = 1 };

/* Cluster-likelihood arithmetic (DESIGN.md "Wide path").
 *   F64: fp64 table form, packed sym(Sigma^{-1}) (D <= 16 on the device).
 *   F32: 16 < D <= 80 (the device pads to D rounded up to 16): items rounded to fp32 at set_data; per cluster A = fp32(chol_upper(sym Sigma^{-1}))
 *        and muf = fp32(mu); for item x and candidate j:
 *          y_a = fmaf chain_b A_j[a][b] (x_b - muf_j[b]) from 0   (= the MFMA contraction, bit for bit),
 *          q = (s_0 + s_1) + (s_2 + s_3) in fp32, s_g = fp32 fmaf chain of y_a^2 over a = 16 mt + 4 g + r,
 *              mt outer, r = 0..3 inner (the 16x16 accumulator layout), ll = c_j - q/2 (fp64). */
enum { NP8O_CONTRACT_F64 = 0, NP8O_CONTRACT_F32 = 1 };

np8o_ctx *np8o_create(const np8o_config *cfg);
void np8o_destroy(np8o_ctx *c);
int np8o_set_data(np8o_ctx *c, const double *X, int64_t N);
/* z in [0,K), clusters given by mu [K*D] and Sigma [K*D*D] row-major. */
int np8o_set_state(np8o_ctx *c, const int32_t *z, int32_t K, const double *mu, const double *Sigma);
int np8o_init_random(np8o_ctx *c, int32_t K_init);
/* Runs n sweeps. Returns 0 or a negative error (capacity). */
int np8o_sweep(np8o_ctx *c, int32_t n);
/* Exact sequential updates of the listed points (chunk = 1, in the given order) at the current epoch. */
int np8o_update_points(np8o_ctx *c, const int64_t *ids, int64_t n);
/* Dense labels (ascending slot order), K, mu/Sigma per label (may be NULL), counts per label. */
int np8o_get_state(np8o_ctx *c, int32_t which, int32_t *z, int32_t *K, double *mu, double *Sigma, int64_t *counts);
int32_t np8o_num_clusters(np8o_ctx *c);
uint32_t np8o_epoch(np8o_ctx *c);
double np8o_best_loglik(np8o_ctx *c);
int64_t np8o_mh_accepted(np8o_ctx *c);
/* Threads of the synchronous step (OpenMP; results do not depend on it). */
void np8o_set_threads(int n);
double np8o_total_loglik(np8o_ctx *c);
/* ll of the given points vs. every live cluster (ascending slot) then the M auxiliaries of the
 * current epoch: out is n x (K+M). Table form (what the chain uses). */
int np8o_loglik_matrix(np8o_ctx *c, const int64_t *idx, int64_t n, double *out);
/* Same matrix computed with the faithful reference formula (general LU inverse, per call). */
int np8o_loglik_matrix_ref(np8o_ctx *c, const int64_t *idx, int64_t n, double *out);
/* The aux draws (mu [M*D], Sigma [M*D*D]) point i would see at the current epoch. */
int np8o_aux_params(np8o_ctx *c, int64_t i, double *mu, double *Sigma);

/* ---- sharded (multi-rank) protocol: the same exchange record the HIP path uses ------------- */
/* Evaluate positions [p0,p1) of the current chunk against the frozen state. Writes z for movers
 * to existing clusters, delta[kcap] (+/- counts of those moves) and new-cluster requests
 * (pos, i, m, old slot); *n_req counts every request, also those past req_cap. */
int np8o_assign_range(np8o_ctx *c, int64_t p0, int64_t p1, int32_t *delta, int64_t *req_pos,
                      int64_t *req_i, int32_t *req_m, int32_t *req_zold, int32_t req_cap, int32_t *n_req);
/* Apply summed deltas and the concatenated request list (any order); rebuild the candidate table.
 * Requests are accepted in ascending scan position, at most A = min(req_max, free slots, n_req) of
 * them, where the free slots are counted after the deltas and before any requester leaves its slot;
 * the other requesters keep their cluster (deferred to their next update).  req_i holds item keys
 * (NP8O_ITEM).  owner_lo/owner_hi: only points in [owner_lo, owner_hi) get z written (all if
 * owner_hi<0).  Returns the number of requests not accepted. */
int np8o_finalize(np8o_ctx *c, const int32_t *delta, const int64_t *req_pos, const int64_t *req_i,
                  const int32_t *req_m, const int32_t *req_zold, int32_t n_req, int64_t owner_lo, int64_t owner_hi);
/* Advance the epoch (end of sweep): cluster-parameter update (np_mcmc.cpp:170) when configured,
 * then max-likelihood bookkeeping (np_mcmc.cpp:172-174). */
int np8o_end_sweep(np8o_ctx *c);
/* Per-slot sufficient statistics of the current labelling about the slot's mean (anchor):
 * out[kcap][D + D(D+1)/2] = sum d | sum d_a d_b (packed upper), d = x - mu_slot, items in order. */
int np8o_suffstats(np8o_ctx *c, double *out);
/* mh_g0 update of every live slot from statistics laid out as np8o_suffstats writes them;
 * returns the number of accepted proposals. */
int64_t np8o_param_update(np8o_ctx *c, const double *stats);
int32_t *np8o_z_ptr(np8o_ctx *c);
/* Cumulative new-cluster requests: out[0] accepted, out[1] deferred (not accepted in their step). */
void np8o_request_stats(np8o_ctx *c, int64_t out[2]);

/* ---- NIW prior primitives (for distribution tests) ------------------------------------------- */
/* Marsaglia-Tsang Gamma(alpha, 1), alpha >= 1, from Philox calls call0, call0+1, .. of (i, t, stream). */
double np8o_gamma_mt(uint64_t seed, uint64_t i, uint32_t t, uint32_t stream, uint32_t call0, double alpha);
/* NIW posterior draw of slot s given the statistics np8o_suffstats writes (n = count); the prior
 * draw for n = 0.  Outputs mu [D], Sigma [D*D].  Does not change the chain.  0 = ok. */
int np8o_niw_draw(np8o_ctx *c, uint64_t i, uint32_t t, uint32_t stream, int64_t n, const double *stats,
                  const double *anchor, double *mu, double *Sigma);

/* ---- Jain-Neal split-merge (src/np_jain_neal_algorithm.cpp; DESIGN.md "Split-merge") ------- */
/* n sweeps of N split/merge attempts each, every sweep followed by np8o_end_sweep.  Reference prior,
 * fp64 contraction.  0 = ok, -1 = unsupported configuration. */
int np8o_sm_sweep(np8o_ctx *c, int32_t n);
/* Attempts [a0, a1) of the current sweep without the end-of-sweep step (timed CPU samples). */
int np8o_sm_attempts(np8o_ctx *c, int64_t a0, int64_t a1);
/* Cumulative attempt outcomes: [0] skipped (equal items), [1] split rejected, [2] merge rejected,
 * [3] split accepted, [4] merge accepted, [5] split rejected for want of a free slot. */
void np8o_sm_get_stats(np8o_ctx *c, int64_t out[6]);
/* Triadic split-merge (src/np_triadic_algorithm.cpp; DESIGN.md "Split-merge"): n sweeps of N attempts
 * on item triples, each sweep followed by np8o_end_sweep; np8o_tri_attempts runs attempts [a0, a1) of
 * the current sweep.  Outcomes: [0] skipped, [1]/[2] dyadic merge rejected/accepted, [3]/[4] dyadic
 * split, [5]/[6] triadic merge (3 -> 2), [7]/[8] triadic split (2 -> 3), [9] split without a free slot. */
int np8o_tri_sweep(np8o_ctx *c, int32_t n);
int np8o_tri_attempts(np8o_ctx *c, int64_t a0, int64_t a1);
void np8o_tri_get_stats(np8o_ctx *c, int64_t out[10]);
double np8o_lgamma_int(int64_t n);
double np8o_canon_sum(const double *v, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
