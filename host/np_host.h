// np_host.h -- C++ host mirror of noparama's sampler API over the MI355X C ABI (include/np8.h).
//
// Keeps the reference's names and call shapes so the HIP sampler drops into an np_mcmc.cpp-style
// driver:
//   data_t / dataset_t / data_ids_t            include/np_data.h:9-25
//   UpdateClusterPopulation                    include/np_update_cluster_population.h:13-44
//   membertrix (addData/addCluster/assign/retract/count/getClusterId/getClusters/cleanup/relabel)
//                                              include/membertrix.h:52-313
//   NealAlgorithm8Hip (ctor shape of NealAlgorithm8, include/np_neal_algorithm8.h:52-56)
//   MCMC (run/getMembershipMatrix/getMaxLikelihoodMatrix, include/np_mcmc.h:71-95)
//   clustering_performance (include/clustering_performance.h)
// The membership state is kept as labels + counts rather than the reference's dense N x C bool
// matrix (membertrix.h:30); cluster parameters are plain vectors (no Eigen in this image).
#pragma once

#include <cstdint>
#include <map>
#include <random>
#include <ostream>
#include <utility>
#include <string>
#include <unordered_map>
#include <vector>

#include "../include/np8.h"

typedef std::vector<double> data_t;
typedef std::vector<data_t *> dataset_t;
typedef int data_id_t;
typedef std::vector<data_id_t> data_ids_t;
typedef int cluster_id_t;

enum np_error_t { error_none, error_already_assigned, error_assignment_remaining, error_assignment_absent };

// Cluster parameters (Suffies_MultivariateNormal{mu, sigma}, include/np_suffies.h:187-200).
struct cluster_t {
    std::vector<double> mu, sigma;  // D, D*D row-major
};

typedef std::unordered_map<cluster_id_t, cluster_t *> clusters_t;

class membertrix {
   public:
    membertrix() = default;
    membertrix(const membertrix &other);  // relabels to 0..K-1 like the reference copy-ctor
    membertrix &operator=(const membertrix &other);
    ~membertrix();

    cluster_id_t addCluster(cluster_t *cluster);
    cluster_t *getCluster(cluster_id_t cluster_id);
    data_id_t addData(data_t &data);
    data_t *getDatum(data_id_t data_id) { return _data[data_id]; }
    np_error_t assign(cluster_id_t cluster_id, data_id_t data_id);
    np_error_t retract(data_id_t data_id, bool auto_remove = true);
    np_error_t remove(cluster_id_t cluster_id);
    bool assigned(data_id_t data_id) const { return _z[data_id] >= 0; }
    cluster_id_t getClusterId(data_id_t data_id) const { return _z[data_id]; }
    size_t count() const { return _z.size(); }
    size_t count(cluster_id_t cluster_id) const;
    size_t getClusterCount() const { return _clusters.size(); }
    const clusters_t &getClusters() const { return _clusters; }
    int cleanup();
    void relabel();
    const dataset_t &getData() const { return _data; }

    // Replace the whole state (labels 0..K-1, parameters per label) -- used to import the device state.
    void setState(const std::vector<int32_t> &z, const std::vector<cluster_t> &clusters);
    void setCluster(cluster_id_t cluster_id, const cluster_t &cluster) { *_clusters.at(cluster_id) = cluster; }
    // No cluster, no assignment (the data stay).
    void clearClusters();
    // relabel() renames the live clusters 0..K-1 in ascending id order; a sampler that patches this
    // membertrix follows the renamings made since the generation it last saw.
    int generation() const { return _generation; }
    std::vector<std::pair<int, std::map<cluster_id_t, cluster_id_t>>> relabelsSince(int generation) const;
    // Dense form of np8_get_state: labels 0..K-1 in ascending id order, counts, mu [K*D], Sigma [K*D*D].
    void dense(std::vector<int32_t> &z, std::vector<int64_t> &counts, std::vector<double> &mu,
               std::vector<double> &sigma) const;

   private:
    void clear_clusters();
    dataset_t _data;
    std::vector<cluster_id_t> _z;
    clusters_t _clusters;
    std::unordered_map<cluster_id_t, size_t> _counts;
    cluster_id_t _next_id = 0;
    int _generation = 0;
    std::vector<std::pair<int, std::map<cluster_id_t, cluster_id_t>>> _relabels;
};

class UpdateClusterPopulation {
   public:
    virtual ~UpdateClusterPopulation() {}
    virtual void update(membertrix &cluster_matrix, const data_ids_t &data_ids) = 0;
    virtual void printStatistics() = 0;
    // true: MCMC passes the whole permutation once per sweep instead of one id per call
    virtual bool sweepGranular() const { return false; }
};

// Base measure and DP parameters (src/np_main.cpp:164,365-372 defaults).
struct np8_prior {
    int D = 2;
    double alpha = 1.0;
    std::vector<double> mu0;       // default 6
    double kappa = 1.0 / 500;
    double nu = 4.0;
    std::vector<double> Lambda;    // default 0.01 I
    int M = 3;                     // np_neal_algorithm8.cpp:33
    int substeps = 1;              // the data-parallel sweep as S synchronous sub-steps (np8_config)
    int param_update = NP8_PARAM_FROZEN;  // UpdateClusters mode (np_mcmc.cpp:170), include/np8.h
    int mh_steps = 20;                    // np_mcmc.cpp:54
    int prior = NP8_PRIOR_REFERENCE;      // base measure (include/np8.h NP8_PRIOR_*)
    int contraction = NP8_CONTRACT_F64;   // NP8_CONTRACT_F32_MFMA: the wide path (D in {32, 64})
};

// The reference constructs its samplers from (generator, likelihood, dirichlet_process)
// (np_neal_algorithm8.h:52-56, np_main.cpp:433-438).  Host-side stand-ins with the same roles:
//   random_engine_t          the generator (np_main.cpp:180); the sampler's Philox key is drawn from it
//   multivariate_normal_distribution   the likelihood (multivariatenormal.h); only its arithmetic is chosen
//   normal_inverse_wishart_distribution  the base measure G0 (normalinvwishart.h:44-64, np_main.cpp:365-372)
//   dirichlet_process        concentration alpha (Suffies_Dirichlet, np_main.cpp:164) + base (dirichlet.h:20-41)
typedef std::mt19937_64 random_engine_t;
struct multivariate_normal_distribution {
    int contraction = NP8_CONTRACT_F64;  // NP8_CONTRACT_F32_MFMA: the wide path (D in {32, 64})
};
struct normal_inverse_wishart_distribution {
    std::vector<double> mu0;     // default 6
    double kappa = 1.0 / 500;
    double nu = 4.0;
    std::vector<double> Lambda;  // default 0.01 I
    int prior = NP8_PRIOR_REFERENCE;
};
struct dirichlet_process {
    double alpha = 1.0;
    normal_inverse_wishart_distribution &base;
};

class NealAlgorithm8Hip : public UpdateClusterPopulation {
   public:
    NealAlgorithm8Hip(uint64_t seed, const np8_prior &prior, int64_t chunk = 0, int device = -1, int kcap = 0);
    // The reference's constructor shape (np_neal_algorithm8.h:52-56); D from the base measure's mean.
    NealAlgorithm8Hip(random_engine_t &generator, const multivariate_normal_distribution &likelihood,
                      const dirichlet_process &nonparametrics, int64_t chunk = 0, int device = -1, int kcap = 0);
    ~NealAlgorithm8Hip() override;

    // NealAlgorithm8::update (np_neal_algorithm8.cpp:49-167): the population update of the listed items on
    // the device, then cluster_matrix patched in place from the change log (np8_changes: moved items,
    // created / emptied clusters), as the reference's update mutates it.  All items at once = one
    // population sweep (np8_population_sweep, data-parallel steps of `chunk` items).
    void update(membertrix &cluster_matrix, const data_ids_t &data_ids) override;
    void printStatistics() override;
    bool sweepGranular() const override { return true; }
    // The end of the sweep (np_mcmc.cpp:170): the cluster-parameter update on the device (np8_end_sweep),
    // its parameter changes patched into cluster_matrix.
    virtual void endSweep(membertrix &cluster_matrix);
    // Bring cluster_matrix up to the device state: the first call on a membertrix loads the whole state,
    // later calls apply only what changed (O(changes)).
    void patch(membertrix &cluster_matrix);

    void setData(const dataset_t &dataset);
    void initRandom(int K);                    // np_mcmc.cpp:49-92
    void setState(const membertrix &trix);     // upload an explicit state
    void sweep(int n);
    void exportState(membertrix &trix, int which);  // 0 current, 1 max-likelihood snapshot
    np8_stats_t stats();
    np8_ctx *ctx() { return _ctx; }
    int64_t numItems() const { return _N; }
    int kcap() const { return _kcap; }

   protected:
    void check(int r, const char *what);

   private:
    np8_ctx *_ctx = nullptr;
    np8_prior _prior;
    int64_t _N = 0;
    int _kcap = 2048;
    // change-log bookkeeping of the membertrix this sampler keeps coherent
    const membertrix *_tracked = nullptr;
    std::unordered_map<int32_t, cluster_id_t> _slot_id;
    int _gen = 0;
};

// UpdateClusters (include/np_update_clusters.h, src/np_update_clusters.cpp:71-142) for a HIP sampler: the
// parameter update runs on the device at the end of the sweep; update() ends the sweep and patches the
// membertrix.  mh_steps is fixed at construction of the sampler (np8_prior::mh_steps).
class UpdateClustersHip {
   public:
    explicit UpdateClustersHip(NealAlgorithm8Hip &sampler) : _sampler(sampler) {}
    void update(membertrix &cluster_matrix, int number_mh_steps) {
        (void)number_mh_steps;
        _sampler.endSweep(cluster_matrix);
    }

   private:
    NealAlgorithm8Hip &_sampler;
};

// The reference's split-merge population update (class JainNealAlgorithm,
// include/np_jain_neal_algorithm.h:52-98; `-a jain_neal_split`) on the same device context: each
// sweep-granular update() runs N split/merge attempts (np8_sm_sweep, include/np8.h).
class JainNealAlgorithmHip : public NealAlgorithm8Hip {
   public:
    using NealAlgorithm8Hip::NealAlgorithm8Hip;
    void update(membertrix &cluster_matrix, const data_ids_t &data_ids) override;
    void printStatistics() override;
    void endSweep(membertrix &cluster_matrix) override { patch(cluster_matrix); }  // np8_sm_sweep ended it
};

// The reference's triadic split-merge update (class TriadicAlgorithm, `-a triadic`): each sweep-granular
// update() runs N attempts on item triples (np8_tri_sweep, include/np8.h).
class TriadicAlgorithmHip : public NealAlgorithm8Hip {
   public:
    using NealAlgorithm8Hip::NealAlgorithm8Hip;
    void update(membertrix &cluster_matrix, const data_ids_t &data_ids) override;
    void printStatistics() override;
    void endSweep(membertrix &cluster_matrix) override { patch(cluster_matrix); }  // np8_tri_sweep ended it
};

// MCMC::run (np_mcmc.cpp:48-175) structured as the reference's: relabel every 10 sweeps, the population
// update of all items, UpdateClusters, considerMaxLikelihood every 5 sweeps on the membertrix (the
// log-likelihood of the state from the device's check, the snapshot a clone of the membertrix).
class MCMC {
   public:
    MCMC(NealAlgorithm8Hip &sampler, int k_init = 20);
    void run(dataset_t &dataset, int T);  // np_mcmc.cpp:48-175
    const membertrix &getMembershipMatrix();
    const membertrix &getMaxLikelihoodMatrix();
    // Check after every update that the membertrix equals the device state (np8_get_state); throws if not.
    void setVerify(bool on) { _verify = on; }
    // One JSON line per sweep (K, new clusters, deferred requests, items moved, log-likelihood
    // of the check, host-side ms) to this stream.
    void setSweepLog(std::ostream *os) { _log = os; }

   private:
    void considerMaxLikelihood(int t);
    void verify(int t, const char *where);
    NealAlgorithm8Hip &_sampler;
    UpdateClustersHip _update_clusters;
    int _k_init;
    bool _verify = false;
    std::ostream *_log = nullptr;
    double _max_likelihood;
    membertrix _membertrix, _max_likelihood_membertrix;
};

class clustering_performance {
   public:
    // rows = ground truth, cols = result (clustering_performance.cpp:14-36), int64 counts
    void calculate(const std::vector<int> &truth, const std::vector<int> &result);
    void write(const std::string &fname) const;  // results.score.txt (clustering_performance.cpp:84-93)
    double purity = 0, rand_index = 0, adjusted_rand_index = 0;
};
