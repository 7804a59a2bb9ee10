// np_host.cpp -- implementation of the C++ host mirror (see np_host.h).
#include "np_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <limits>
#include <numeric>
#include <stdexcept>

// ---- membertrix ----------------------------------------------------------------------------------
membertrix::~membertrix() { clear_clusters(); }

void membertrix::clear_clusters() {
    for (auto &kv : _clusters) delete kv.second;
    _clusters.clear();
    _counts.clear();
}

membertrix::membertrix(const membertrix &other) { *this = other; }

// Like the reference copy constructor (membertrix.cpp:34-55): the copy has labels 0..K-1 assigned
// in ascending order of the source ids, empty clusters dropped.
membertrix &membertrix::operator=(const membertrix &other) {
    if (this == &other) return *this;
    clear_clusters();
    _data = other._data;
    std::map<cluster_id_t, cluster_id_t> remap;
    for (const auto &kv : other._clusters) remap[kv.first] = -1;
    cluster_id_t k = 0;
    for (auto &kv : remap) {
        if (other.count(kv.first) == 0) continue;
        kv.second = k;
        _clusters[k] = new cluster_t(*other._clusters.at(kv.first));
        _counts[k] = other.count(kv.first);
        ++k;
    }
    _next_id = k;
    _z.resize(other._z.size());
    for (size_t i = 0; i < _z.size(); ++i) _z[i] = other._z[i] < 0 ? -1 : remap[other._z[i]];
    return *this;
}

cluster_id_t membertrix::addCluster(cluster_t *cluster) {
    const cluster_id_t id = _next_id++;
    _clusters[id] = cluster;
    _counts[id] = 0;
    return id;
}

cluster_t *membertrix::getCluster(cluster_id_t cluster_id) { return _clusters.at(cluster_id); }

data_id_t membertrix::addData(data_t &data) {
    _data.push_back(&data);
    _z.push_back(-1);
    return (data_id_t)_data.size() - 1;
}

np_error_t membertrix::assign(cluster_id_t cluster_id, data_id_t data_id) {
    if (_z[data_id] >= 0) return error_already_assigned;
    _z[data_id] = cluster_id;
    _counts[cluster_id] += 1;
    return error_none;
}

np_error_t membertrix::retract(data_id_t data_id, bool auto_remove) {
    const cluster_id_t c = _z[data_id];
    if (c < 0) return error_assignment_absent;
    _z[data_id] = -1;
    if (--_counts[c] == 0 && auto_remove) remove(c);  // membertrix.cpp:200-203
    return error_none;
}

np_error_t membertrix::remove(cluster_id_t cluster_id) {
    if (count(cluster_id) != 0) return error_assignment_remaining;
    auto it = _clusters.find(cluster_id);
    if (it != _clusters.end()) {
        delete it->second;
        _clusters.erase(it);
    }
    _counts.erase(cluster_id);
    return error_none;
}

size_t membertrix::count(cluster_id_t cluster_id) const {
    auto it = _counts.find(cluster_id);
    return it == _counts.end() ? 0 : it->second;
}

int membertrix::cleanup() {
    std::vector<cluster_id_t> empty;
    for (const auto &kv : _clusters)
        if (count(kv.first) == 0) empty.push_back(kv.first);
    for (cluster_id_t c : empty) remove(c);
    return (int)empty.size();
}

void membertrix::relabel() {
    membertrix tmp(*this);
    *this = tmp;
}

void membertrix::setState(const std::vector<int32_t> &z, const std::vector<cluster_t> &clusters) {
    clear_clusters();
    for (size_t k = 0; k < clusters.size(); ++k) {
        _clusters[(cluster_id_t)k] = new cluster_t(clusters[k]);
        _counts[(cluster_id_t)k] = 0;
    }
    _next_id = (cluster_id_t)clusters.size();
    _z.assign(z.begin(), z.end());
    for (int32_t v : z) _counts[v] += 1;
}

// ---- NealAlgorithm8Hip ---------------------------------------------------------------------------
NealAlgorithm8Hip::NealAlgorithm8Hip(uint64_t seed, const np8_prior &prior, int64_t chunk, int device, int kcap)
    : _prior(prior) {
    const int D = prior.D;
    if (_prior.mu0.empty()) _prior.mu0.assign(D, 6.0);
    if (_prior.Lambda.empty()) {
        _prior.Lambda.assign((size_t)D * D, 0.0);
        for (int a = 0; a < D; ++a) _prior.Lambda[a * D + a] = 0.01;
    }
    np8_config cfg{};
    cfg.D = D;
    cfg.M = prior.M;
    cfg.alpha = prior.alpha;
    cfg.mu0 = _prior.mu0.data();
    cfg.kappa = prior.kappa;
    cfg.nu = prior.nu;
    cfg.Lambda = _prior.Lambda.data();
    cfg.seed = seed;
    cfg.kcap = kcap;
    if (kcap > 0) _kcap = kcap;
    cfg.chunk = chunk;
    cfg.device = device;
    cfg.param_update = prior.param_update;
    cfg.mh_steps = prior.mh_steps;
    cfg.prior = prior.prior;
    cfg.contraction = prior.contraction;
    check(np8_create(&_ctx, &cfg), "np8_create");
}

NealAlgorithm8Hip::~NealAlgorithm8Hip() { np8_destroy(_ctx); }

void NealAlgorithm8Hip::check(int r, const char *what) {
    if (r != NP8_OK)
        throw std::runtime_error(std::string(what) + " failed (" + std::to_string(r) + "): " + np8_last_error(_ctx));
}

void NealAlgorithm8Hip::setData(const dataset_t &dataset) {
    const int D = _prior.D;
    _N = (int64_t)dataset.size();
    std::vector<double> X((size_t)_N * D);
    for (int64_t i = 0; i < _N; ++i) {
        if ((int)dataset[i]->size() != D) throw std::runtime_error("data item with wrong dimension");
        for (int a = 0; a < D; ++a) X[(size_t)i * D + a] = (*dataset[i])[a];
    }
    check(np8_set_data(_ctx, X.data(), _N, D, 0, _N), "np8_set_data");
}

void NealAlgorithm8Hip::initRandom(int K) { check(np8_init_random(_ctx, K), "np8_init_random"); }

void NealAlgorithm8Hip::setState(const membertrix &trix) {
    membertrix c(trix);  // labels 0..K-1
    const int D = _prior.D, K = (int)c.getClusterCount();
    std::vector<int32_t> z((size_t)_N);
    for (int64_t i = 0; i < _N; ++i) z[i] = c.getClusterId((data_id_t)i);
    std::vector<double> mu((size_t)K * D), sg((size_t)K * D * D);
    for (const auto &kv : c.getClusters()) {
        std::copy(kv.second->mu.begin(), kv.second->mu.end(), mu.begin() + (size_t)kv.first * D);
        std::copy(kv.second->sigma.begin(), kv.second->sigma.end(), sg.begin() + (size_t)kv.first * D * D);
    }
    check(np8_set_state(_ctx, z.data(), K, mu.data(), sg.data()), "np8_set_state");
}

void NealAlgorithm8Hip::sweep(int n) { check(np8_sweep(_ctx, n), "np8_sweep"); }

// UpdateClusterPopulation::update: a whole permutation = one data-parallel sweep (the MCMC driver
// passes it once per sweep because sweepGranular() is true); otherwise the listed items are updated
// sequentially with the reference's per-point semantics.
void NealAlgorithm8Hip::update(membertrix &cluster_matrix, const data_ids_t &data_ids) {
    (void)cluster_matrix;  // the device owns the state; import with exportState()
    if ((int64_t)data_ids.size() == _N) {
        check(np8_sweep(_ctx, 1), "np8_sweep");
        return;
    }
    std::vector<int64_t> ids(data_ids.begin(), data_ids.end());
    check(np8_update_points(_ctx, ids.data(), (int64_t)ids.size()), "np8_update_points");
}

void NealAlgorithm8Hip::exportState(membertrix &trix, int which) {
    check(np8_sync(_ctx), "np8_sync");
    const int D = _prior.D;
    const int kc = _kcap;  // room for any snapshot's cluster count
    std::vector<int32_t> z((size_t)_N);
    int32_t K = 0;
    std::vector<double> mu((size_t)kc * D), sg((size_t)kc * D * D);
    check(np8_get_state(_ctx, which, z.data(), &K, mu.data(), sg.data(), nullptr), "np8_get_state");
    std::vector<cluster_t> cl((size_t)K);
    for (int k = 0; k < K; ++k) {
        cl[k].mu.assign(mu.begin() + (size_t)k * D, mu.begin() + (size_t)(k + 1) * D);
        cl[k].sigma.assign(sg.begin() + (size_t)k * D * D, sg.begin() + (size_t)(k + 1) * D * D);
    }
    trix.setState(z, cl);
}

np8_stats_t NealAlgorithm8Hip::stats() {
    np8_stats_t s{};
    check(np8_stats(_ctx, &s), "np8_stats");
    return s;
}

void NealAlgorithm8Hip::printStatistics() {
    np8_stats_t s = stats();
    std::cout << "Statistics:" << std::endl;
    std::cout << " # of new cluster events accepted: " << s.new_clusters << std::endl;
    std::cout << " # of rejected new-cluster requests: " << s.rejected_requests << std::endl;
    std::cout << " live clusters: " << s.K << ", sweeps: " << s.epoch << std::endl;
}

// A whole permutation = one split-merge sweep (N attempts on the library's two scan permutations,
// np_mcmc.cpp:117-164 with subset_count = 2).  The reference's per-pair call has no sweep-parallel form.
void JainNealAlgorithmHip::update(membertrix &cluster_matrix, const data_ids_t &data_ids) {
    (void)cluster_matrix;
    if ((int64_t)data_ids.size() != numItems())
        throw std::runtime_error("JainNealAlgorithmHip::update: pass all items (one split-merge sweep)");
    if (np8_sm_sweep(ctx(), 1) != NP8_OK) throw std::runtime_error(std::string("np8_sm_sweep: ") + np8_last_error(ctx()));
}

// The reference's statistics (np_jain_neal_algorithm.cpp:505-530).
void JainNealAlgorithmHip::printStatistics() {
    int64_t o[6];
    if (np8_sm_stats(ctx(), o) != NP8_OK) throw std::runtime_error(std::string("np8_sm_stats: ") + np8_last_error(ctx()));
    std::cout << "Statistics:" << std::endl;
    std::cout << " # of merge attempts: " << o[2] + o[4] << std::endl;
    std::cout << "   o of accepted merge cluster events: " << o[4] << std::endl;
    std::cout << " # of split attempts: " << o[1] + o[3] + o[5] << std::endl;
    std::cout << "   o of accepted split cluster events: " << o[3] << std::endl;
    std::cout << " live clusters: " << stats().K << ", sweeps: " << stats().epoch << std::endl;
}

// A whole permutation = one triadic split-merge sweep (N attempts on item triples, subset_count = 3).
void TriadicAlgorithmHip::update(membertrix &cluster_matrix, const data_ids_t &data_ids) {
    (void)cluster_matrix;
    if ((int64_t)data_ids.size() != numItems())
        throw std::runtime_error("TriadicAlgorithmHip::update: pass all items (one split-merge sweep)");
    if (np8_tri_sweep(ctx(), 1) != NP8_OK) throw std::runtime_error(std::string("np8_tri_sweep: ") + np8_last_error(ctx()));
}

// The reference's statistics (np_triadic_algorithm.cpp:797-832): merge 2 -> 1, split 1 -> 2,
// merge 3 -> 2, split 2 -> 3.
void TriadicAlgorithmHip::printStatistics() {
    int64_t o[10];
    if (np8_tri_stats(ctx(), o) != NP8_OK) throw std::runtime_error(std::string("np8_tri_stats: ") + np8_last_error(ctx()));
    const char *name[4] = {"merge (2 -> 1)", "split (1 -> 2)", "merge (3 -> 2)", "split (2 -> 3)"};
    std::cout << "Statistics:" << std::endl;
    for (int k = 0; k < 4; ++k) {
        std::cout << " # of " << name[k] << " attempts: " << o[1 + 2 * k] + o[2 + 2 * k] << std::endl;
        std::cout << "   o of accepted " << name[k] << " cluster events: " << o[2 + 2 * k] << std::endl;
    }
    std::cout << " live clusters: " << stats().K << ", sweeps: " << stats().epoch << std::endl;
}

// ---- MCMC ----------------------------------------------------------------------------------------
MCMC::MCMC(NealAlgorithm8Hip &sampler, int k_init) : _sampler(sampler), _k_init(k_init) {}

void MCMC::run(dataset_t &dataset, int T) {
    for (auto *d : dataset) {
        _membertrix.addData(*d);
        _max_likelihood_membertrix.addData(*d);
    }
    _sampler.setData(dataset);
    _sampler.initRandom(_k_init);
    data_ids_t all(dataset.size());
    std::iota(all.begin(), all.end(), 0);
    for (int t = 0; t < T; ++t) {
        // relabel every 10 sweeps (np_mcmc.cpp:111-114) has no effect on the device state (slots are
        // reused in ascending order); the permutation of np_mcmc.cpp:120-125 is the device's.
        if (_sampler.sweepGranular()) {
            _sampler.update(_membertrix, all);
        } else {
            for (data_id_t i : all) _sampler.update(_membertrix, {i});
        }
    }
    _sampler.exportState(_membertrix, 0);
}

const membertrix &MCMC::getMembershipMatrix() { return _membertrix; }

const membertrix &MCMC::getMaxLikelihoodMatrix() {
    _sampler.exportState(_max_likelihood_membertrix, 1);
    return _max_likelihood_membertrix;
}

// ---- clustering_performance -----------------------------------------------------------------------
void clustering_performance::calculate(const std::vector<int> &A, const std::vector<int> &B) {
    purity = rand_index = adjusted_rand_index = std::numeric_limits<double>::quiet_NaN();
    if (A.empty() || A.size() != B.size()) return;
    const int na = *std::max_element(A.begin(), A.end()) + 1, nb = *std::max_element(B.begin(), B.end()) + 1;
    std::vector<int64_t> F((size_t)na * nb, 0);
    for (size_t i = 0; i < A.size(); ++i) F[(size_t)A[i] * nb + B[i]] += 1;
    const int64_t N = (int64_t)A.size();
    int64_t ps = 0, a = 0, b = 0, c = 0;
    for (int j = 0; j < nb; ++j) {
        int64_t m = 0, cs = 0;
        for (int i = 0; i < na; ++i) {
            m = std::max(m, F[(size_t)i * nb + j]);
            cs += F[(size_t)i * nb + j];
        }
        ps += m;
        c += (cs * cs - cs) / 2;
    }
    for (int i = 0; i < na; ++i) {
        int64_t rs = 0;
        for (int j = 0; j < nb; ++j) {
            const int64_t f = F[(size_t)i * nb + j];
            a += (f * f - f) / 2;
            rs += f;
        }
        b += (rs * rs - rs) / 2;
    }
    purity = (double)ps / (double)N;
    const double S = ((double)N * (double)N - (double)N) / 2.0;
    if (S == 0.0) return;
    rand_index = (double)(2 * a - b - c) / S + 1.0;
    const double bc_S = (double)b * (double)c / S, bpc_2 = (double)(b + c) / 2.0;
    if (bc_S == bpc_2) return;
    adjusted_rand_index = ((double)a - bc_S) / (bpc_2 - bc_S);
}

void clustering_performance::write(const std::string &fname) const {
    std::ofstream f(fname);
    f << "Purity: " << purity << std::endl;
    f << "Rand Index: " << rand_index << std::endl;
    f << "Adjusted Rand Index: " << adjusted_rand_index << std::endl;
}
