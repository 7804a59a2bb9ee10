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

   private:
    void clear_clusters();
    dataset_t _data;
    std::vector<cluster_id_t> _z;
    clusters_t _clusters;
    std::unordered_map<cluster_id_t, size_t> _counts;
    cluster_id_t _next_id = 0;
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
    int param_update = NP8_PARAM_FROZEN;  // UpdateClusters mode (np_mcmc.cpp:170), include/np8.h
    int mh_steps = 20;                    // np_mcmc.cpp:54
    int prior = NP8_PRIOR_REFERENCE;      // base measure (include/np8.h NP8_PRIOR_*)
    int contraction = NP8_CONTRACT_F64;   // NP8_CONTRACT_F32_MFMA: the wide path (D in {32, 64})
};

class NealAlgorithm8Hip : public UpdateClusterPopulation {
   public:
    NealAlgorithm8Hip(uint64_t seed, const np8_prior &prior, int64_t chunk = 0, int device = -1, int kcap = 0);
    ~NealAlgorithm8Hip() override;

    // The device owns the state; membertrix is imported on demand (exportState).
    void update(membertrix &cluster_matrix, const data_ids_t &data_ids) override;
    void printStatistics() override;
    bool sweepGranular() const override { return true; }

    void setData(const dataset_t &dataset);
    void initRandom(int K);                    // np_mcmc.cpp:49-92
    void setState(const membertrix &trix);     // upload an explicit state
    void sweep(int n);
    void exportState(membertrix &trix, int which);  // 0 current, 1 max-likelihood snapshot
    np8_stats_t stats();
    np8_ctx *ctx() { return _ctx; }
    int64_t numItems() const { return _N; }

   private:
    void check(int r, const char *what);
    np8_ctx *_ctx = nullptr;
    np8_prior _prior;
    int64_t _N = 0;
    int _kcap = 2048;
};

// The reference's split-merge population update (class JainNealAlgorithm,
// include/np_jain_neal_algorithm.h:52-98; `-a jain_neal_split`) on the same device context: each
// sweep-granular update() runs N split/merge attempts (np8_sm_sweep, include/np8.h).
class JainNealAlgorithmHip : public NealAlgorithm8Hip {
   public:
    using NealAlgorithm8Hip::NealAlgorithm8Hip;
    void update(membertrix &cluster_matrix, const data_ids_t &data_ids) override;
    void printStatistics() override;
};

// The reference's triadic split-merge update (class TriadicAlgorithm, `-a triadic`): each sweep-granular
// update() runs N attempts on item triples (np8_tri_sweep, include/np8.h).
class TriadicAlgorithmHip : public NealAlgorithm8Hip {
   public:
    using NealAlgorithm8Hip::NealAlgorithm8Hip;
    void update(membertrix &cluster_matrix, const data_ids_t &data_ids) override;
    void printStatistics() override;
};

class MCMC {
   public:
    MCMC(NealAlgorithm8Hip &sampler, int k_init = 20);
    void run(dataset_t &dataset, int T);  // np_mcmc.cpp:48-175
    const membertrix &getMembershipMatrix();
    const membertrix &getMaxLikelihoodMatrix();

   private:
    NealAlgorithm8Hip &_sampler;
    int _k_init;
    membertrix _membertrix, _max_likelihood_membertrix;
};

class clustering_performance {
   public:
    // rows = ground truth, cols = result (clustering_performance.cpp:14-36), int64 counts
    void calculate(const std::vector<int> &truth, const std::vector<int> &result);
    void write(const std::string &fname) const;  // results.score.txt (clustering_performance.cpp:84-93)
    double purity = 0, rand_index = 0, adjusted_rand_index = 0;
};
