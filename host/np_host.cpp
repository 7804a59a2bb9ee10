// np_host.cpp -- implementation of the C++ host mirror (see np_host.h).
#include "np_host.h"

#include <algorithm>
#include <chrono>
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
    _generation = other._generation;
    _relabels = other._relabels;
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
    std::map<cluster_id_t, cluster_id_t> remap;  // the copy's renumbering: live ids ascending -> 0..K-1
    cluster_id_t k = 0;
    for (const auto &kv : std::map<cluster_id_t, cluster_t *>(_clusters.begin(), _clusters.end()))
        if (count(kv.first) > 0) remap[kv.first] = k++;
    const int gen = _generation + 1;
    auto relabels = _relabels;
    membertrix tmp(*this);
    *this = tmp;
    _relabels = relabels;
    _generation = gen;
    _relabels.emplace_back(gen, remap);
}

std::vector<std::pair<int, std::map<cluster_id_t, cluster_id_t>>> membertrix::relabelsSince(int generation) const {
    std::vector<std::pair<int, std::map<cluster_id_t, cluster_id_t>>> out;
    for (const auto &r : _relabels)
        if (r.first > generation) out.push_back(r);
    return out;
}

void membertrix::clearClusters() {
    clear_clusters();
    std::fill(_z.begin(), _z.end(), -1);
}

void membertrix::dense(std::vector<int32_t> &z, std::vector<int64_t> &counts, std::vector<double> &mu,
                       std::vector<double> &sigma) const {
    std::map<cluster_id_t, int32_t> lab;
    for (const auto &kv : _clusters) lab[kv.first] = 0;
    int32_t k = 0;
    for (auto &kv : lab) kv.second = k++;
    z.resize(_z.size());
    for (size_t i = 0; i < _z.size(); ++i) z[i] = _z[i] < 0 ? -1 : lab.at(_z[i]);
    counts.assign((size_t)k, 0);
    mu.clear();
    sigma.clear();
    for (const auto &kv : lab) {
        counts[(size_t)kv.second] = (int64_t)count(kv.first);
        const cluster_t *c = _clusters.at(kv.first);
        mu.insert(mu.end(), c->mu.begin(), c->mu.end());
        sigma.insert(sigma.end(), c->sigma.begin(), c->sigma.end());
    }
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
    cfg.substeps = prior.substeps;
    check(NP8_CREATE(&_ctx, &cfg), "np8_create_sized");
}

namespace {
np8_prior prior_of(const multivariate_normal_distribution &likelihood, const dirichlet_process &dp) {
    np8_prior p;
    p.D = (int)dp.base.mu0.size();
    p.alpha = dp.alpha;
    p.mu0 = dp.base.mu0;
    p.kappa = dp.base.kappa;
    p.nu = dp.base.nu;
    p.Lambda = dp.base.Lambda;
    p.prior = dp.base.prior;
    p.contraction = likelihood.contraction;
    return p;
}
}  // namespace

NealAlgorithm8Hip::NealAlgorithm8Hip(random_engine_t &generator, const multivariate_normal_distribution &likelihood,
                                     const dirichlet_process &nonparametrics, int64_t chunk, int device, int kcap)
    : NealAlgorithm8Hip((uint64_t)generator(), prior_of(likelihood, nonparametrics), chunk, device, kcap) {}

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
    _tracked = nullptr;  // np8_set_data drops the device change log: the next patch reloads the whole state
    _slot_id.clear();
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

// UpdateClusterPopulation::update: all items = one population sweep (the MCMC driver passes them once
// per sweep because sweepGranular() is true); otherwise the listed items are updated sequentially with
// the reference's per-point semantics.  Then the membertrix is patched from the change log.
void NealAlgorithm8Hip::update(membertrix &cluster_matrix, const data_ids_t &data_ids) {
    if ((int64_t)data_ids.size() == _N) {
        check(np8_population_sweep(_ctx), "np8_population_sweep");
    } else {
        std::vector<int64_t> ids(data_ids.begin(), data_ids.end());
        check(np8_update_points(_ctx, ids.data(), (int64_t)ids.size()), "np8_update_points");
    }
    patch(cluster_matrix);
}

void NealAlgorithm8Hip::endSweep(membertrix &cluster_matrix) {
    check(np8_end_sweep(_ctx), "np8_end_sweep");
    patch(cluster_matrix);
}

// The change log applied to the membertrix: new clusters first (membertrix::addCluster), then the moved
// items (retract without auto-remove, assign), then the emptied clusters (remove) and new parameters.
void NealAlgorithm8Hip::patch(membertrix &trix) {
    const int D = _prior.D;
    if (_tracked != &trix) {  // first contact: the whole state, from an empty baseline
        check(np8_track_changes(_ctx, NP8_CHANGES_FROM_EMPTY), "np8_track_changes");
        trix.clearClusters();
        _tracked = &trix;
        _slot_id.clear();
        _gen = trix.generation();
    }
    for (const auto &r : trix.relabelsSince(_gen)) {  // relabel() renamed the clusters meanwhile
        for (auto &kv : _slot_id) kv.second = r.second.at(kv.second);
        _gen = r.first;
    }
    std::vector<int64_t> item((size_t)std::max<int64_t>(_N, 1));
    std::vector<int32_t> slot(item.size()), created((size_t)_kcap), removed((size_t)_kcap), updated((size_t)_kcap);
    std::vector<double> mu((size_t)_kcap * D), sg((size_t)_kcap * D * D);
    np8_changes_t ch{};
    check(np8_changes(_ctx, (int64_t)item.size(), item.data(), slot.data(), created.data(), removed.data(),
                      updated.data(), mu.data(), sg.data(), &ch),
          "np8_changes");
    auto params = [&](int q) {
        cluster_t c;
        c.mu.assign(mu.begin() + (size_t)q * D, mu.begin() + (size_t)(q + 1) * D);
        c.sigma.assign(sg.begin() + (size_t)q * D * D, sg.begin() + (size_t)(q + 1) * D * D);
        return c;
    };
    for (int q = 0; q < ch.n_created; ++q) _slot_id[created[q]] = trix.addCluster(new cluster_t(params(q)));
    for (int q = 0; q < ch.n_updated; ++q) trix.setCluster(_slot_id.at(updated[q]), params(ch.n_created + q));
    for (int64_t k = 0; k < ch.n_moved; ++k) {
        const data_id_t i = (data_id_t)item[k];
        if (trix.assigned(i)) trix.retract(i, false);
        trix.assign(_slot_id.at(slot[k]), i);
    }
    for (int q = 0; q < ch.n_removed; ++q) {
        const np_error_t e = trix.remove(_slot_id.at(removed[q]));
        if (e != error_none) throw std::runtime_error("patch: an emptied cluster still has items");
        _slot_id.erase(removed[q]);
    }
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
    check(NP8_STATS(_ctx, &s), "np8_stats_sized");
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
// np_mcmc.cpp:117-164 with subset_count = 2), the end-of-sweep step included.  The reference's per-pair
// call has no sweep-parallel form.
void JainNealAlgorithmHip::update(membertrix &cluster_matrix, const data_ids_t &data_ids) {
    if ((int64_t)data_ids.size() != numItems())
        throw std::runtime_error("JainNealAlgorithmHip::update: pass all items (one split-merge sweep)");
    check(np8_sm_sweep(ctx(), 1), "np8_sm_sweep");
    patch(cluster_matrix);
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
    if ((int64_t)data_ids.size() != numItems())
        throw std::runtime_error("TriadicAlgorithmHip::update: pass all items (one split-merge sweep)");
    check(np8_tri_sweep(ctx(), 1), "np8_tri_sweep");
    patch(cluster_matrix);
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
MCMC::MCMC(NealAlgorithm8Hip &sampler, int k_init)
    : _sampler(sampler), _update_clusters(sampler), _k_init(k_init),
      _max_likelihood(-std::numeric_limits<double>::infinity()) {}

void MCMC::run(dataset_t &dataset, int T) {
    const int N = (int)dataset.size();
    for (auto *d : dataset) _membertrix.addData(*d);  // np_mcmc.cpp:57-62
    _sampler.setData(dataset);
    // np_mcmc.cpp:64-92: K_init G0 clusters, uniform assignment, cleanup (on the device), loaded whole
    _sampler.initRandom(_k_init);
    _sampler.patch(_membertrix);
    const int number_mh_steps = 20;  // np_mcmc.cpp:54
    const int cycle_print = 10, cycle_max_likelihood = 5;
    data_ids_t all((size_t)N);
    std::iota(all.begin(), all.end(), 0);
    for (int t = 0; t < T; ++t) {
        const auto t0 = std::chrono::steady_clock::now();
        const np8_stats_t s0 = _sampler.stats();
        if (t % cycle_print == 0) _membertrix.relabel();  // np_mcmc.cpp:111-114
        // np_mcmc.cpp:117-164: every item once; the scan order (random_order) is the device's permutation
        if (_sampler.sweepGranular()) {
            _sampler.update(_membertrix, all);
        } else {
            for (data_id_t i : all) _sampler.update(_membertrix, {i});
        }
        if (_verify) verify(t, "population update");
        _update_clusters.update(_membertrix, number_mh_steps);  // np_mcmc.cpp:170
        if (_verify) verify(t, "cluster update");
        if (t % cycle_max_likelihood == 0) considerMaxLikelihood(t);  // np_mcmc.cpp:172-174
        if (_log) {
            const np8_stats_t s1 = _sampler.stats();
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            *_log << "{\"sweep\": " << t << ", \"K\": " << s1.K << ", \"new_clusters\": " << s1.new_clusters - s0.new_clusters
                  << ", \"deferred_requests\": " << s1.rejected_requests - s0.rejected_requests
                  << ", \"existing_picks\": " << s1.existing_picks - s0.existing_picks;
            if (t % cycle_max_likelihood == 0) *_log << ", \"loglik\": " << s1.last_loglik;
            *_log << ", \"ms\": " << ms << "}" << std::endl;
        }
    }
}

// np_mcmc.cpp:187-203: the log-likelihood of the membertrix's state is the device's check of this sweep
// (np8_end_sweep ran it on the same state); an improvement clones the membertrix.
void MCMC::considerMaxLikelihood(int t) {
    (void)t;
    const double L = _sampler.stats().last_loglik;
    if (L > _max_likelihood) {
        _max_likelihood = L;
        _max_likelihood_membertrix = _membertrix;
    }
}

namespace {
// Clusters renamed in order of their first item (ids are names: creation order and relabel() on the host,
// slots on the device); counts and parameters permuted alike.
void canonicalize(std::vector<int32_t> &z, std::vector<int64_t> &cnt, std::vector<double> &mu, std::vector<double> &sg,
                  int K, int D) {
    std::vector<int32_t> lut((size_t)K, -1), perm;
    for (int32_t &l : z) {
        if (lut[(size_t)l] < 0) {
            lut[(size_t)l] = (int32_t)perm.size();
            perm.push_back(l);
        }
        l = lut[(size_t)l];
    }
    std::vector<int64_t> c2(perm.size());
    std::vector<double> m2(perm.size() * D), s2(perm.size() * D * D);
    for (size_t k = 0; k < perm.size(); ++k) {
        c2[k] = cnt[(size_t)perm[k]];
        std::copy(mu.begin() + (size_t)perm[k] * D, mu.begin() + (size_t)(perm[k] + 1) * D, m2.begin() + k * D);
        std::copy(sg.begin() + (size_t)perm[k] * D * D, sg.begin() + (size_t)(perm[k] + 1) * D * D, s2.begin() + k * D * D);
    }
    cnt.swap(c2);
    mu.swap(m2);
    sg.swap(s2);
}
}  // namespace

void MCMC::verify(int t, const char *where) {
    np8_ctx *c = _sampler.ctx();
    const int64_t N = _sampler.numItems();
    std::vector<int32_t> z((size_t)N), zd;
    int32_t K = 0;
    const size_t kc = (size_t)_sampler.kcap();
    const int D = (int)(_membertrix.count() ? _membertrix.getDatum(0)->size() : 0);
    std::vector<double> mu(kc * D), sg(kc * D * D), mud, sgd;
    std::vector<int64_t> cnt(kc), cntd;
    if (np8_sync(c) != NP8_OK || np8_get_state(c, 0, z.data(), &K, mu.data(), sg.data(), cnt.data()) != NP8_OK)
        throw std::runtime_error(std::string("verify: np8_get_state: ") + np8_last_error(c));
    _membertrix.dense(zd, cntd, mud, sgd);
    bool ok = (int)cntd.size() == K;
    if (ok) {
        cnt.resize((size_t)K);
        mu.resize((size_t)K * D);
        sg.resize((size_t)K * D * D);
        canonicalize(z, cnt, mu, sg, K, D);
        canonicalize(zd, cntd, mud, sgd, K, D);
        ok = zd == z && cntd == cnt && mud == mu && sgd == sg;
    }
    if (!ok)
        throw std::runtime_error("verify: membertrix differs from the device state after the " + std::string(where) +
                                 " of sweep " + std::to_string(t));
}

const membertrix &MCMC::getMembershipMatrix() { return _membertrix; }

const membertrix &MCMC::getMaxLikelihoodMatrix() {
    if (_verify) {  // the host's clone equals the device's own snapshot (np8_get_state(which = 1))
        np8_ctx *c = _sampler.ctx();
        std::vector<int32_t> z((size_t)_sampler.numItems()), zd;
        int32_t K = 0;
        std::vector<int64_t> cntd;
        std::vector<double> mud, sgd;
        if (np8_get_state(c, 1, z.data(), &K, nullptr, nullptr, nullptr) != NP8_OK)
            throw std::runtime_error(std::string("verify: np8_get_state(1): ") + np8_last_error(c));
        _max_likelihood_membertrix.dense(zd, cntd, mud, sgd);
        if ((int)cntd.size() != K) throw std::runtime_error("verify: max-likelihood snapshot differs");
        std::vector<int64_t> cnt((size_t)K, 0);
        std::vector<double> mu, sg;
        for (int32_t l : z) cnt[(size_t)l] += 1;
        mud.clear();
        sgd.clear();
        canonicalize(z, cnt, mu, sg, K, 0);
        canonicalize(zd, cntd, mud, sgd, K, 0);
        if (zd != z || cntd != cnt) throw std::runtime_error("verify: max-likelihood snapshot differs");
    }
    return _max_likelihood_membertrix;
}

// ---- clustering_performance -----------------------------------------------------------------------
// (NaN where the reference returns early and leaves an index unset, clustering_performance.cpp:70-73: this
// mirror's convention for that early return, not a value the reference computes)
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
