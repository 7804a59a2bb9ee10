// np_main.cpp -- command-line driver mirroring the reference's `noparama` executable for the Neal-8
// clustering path (src/np_main.cpp:156-507):
//   np8_noparama -d <data> -a algorithm8 -T <sweeps> -c clustering [-s seed] [-C chunk] [-D dims]
// reads "x_1 .. x_D label" rows (np_main.cpp:57-148, generalised from 2 columns), runs MCMC on the
// GPU, and writes <workspace><YYYYmmdd_HH:MM>/{snapshot,results}{,<k>,.score}.txt and the LATEST
// symlink in the reference's formats (np_results.cpp:39-196, host/np_results.h) for the last state
// and the max-likelihood state.  Refuses to overwrite an existing workspace (exit 106,
// np_main.cpp:273-276).
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <memory>
#include <chrono>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <ctime>
#include <iomanip>
#include <numeric>
#include <random>
#include <sstream>
#include <string>

#include "np_host.h"
#include "np_results.h"

static void usage(const char *p) {
    std::cerr << "usage: " << p << " -d <datafile> -a algorithm8|jain_neal_split|triadic [-T sweeps=2000] [-c clustering] [-s seed]"
              << " [-C chunk (0 = data-parallel sweep, 1 = sequential)] [-D dims=2] [-w workspace]"
              << " [-u frozen|mh_g0|niw_conjugate (cluster-parameter update)] [-p reference|niw (base measure)]"
              << " [-x f64|f32 (cluster likelihoods; f32 = fp32 matrix cores, D in {32, 64})]"
              << " [-n subsample size=200, 0 = all items] [-S sub-steps of the data-parallel sweep, or auto (16 up to 8192 items, else 1)=auto] [-j per-sweep JSONL file] [-V (check the membertrix against the device after every update)]; data: 'x_1 .. x_D label' text or [N][D+1] .f64"
              << std::endl;
}

// Rows "x_1 .. x_D label" (np_main.cpp:57-148, generalised from 2 columns), or, for a file ending in
// ".f64", the same rows as raw little-endian float64 ([N][D+1], written by noparama_amd.datasets).
static bool read_data(const std::string &fn, int D, dataset_t &ds, std::vector<int> &gt) {
    if (fn.size() > 4 && fn.compare(fn.size() - 4, 4, ".f64") == 0) {
        std::ifstream f(fn, std::ios::binary);
        std::vector<double> row((size_t)D + 1);
        while (f.read(reinterpret_cast<char *>(row.data()), (std::streamsize)(sizeof(double) * row.size()))) {
            ds.push_back(new data_t(row.begin(), row.begin() + D));
            gt.push_back((int)row[D]);
        }
        return !ds.empty();
    }
    std::ifstream f(fn);
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        auto *d = new data_t(D);
        bool ok = true;
        for (int a = 0; a < D; ++a) ok = ok && static_cast<bool>(ss >> (*d)[a]);
        double c = 0;
        ok = ok && static_cast<bool>(ss >> c);
        if (!ok) {
            delete d;
            continue;
        }
        ds.push_back(d);
        gt.push_back((int)c);
    }
    return !ds.empty();
}

// np_main.cpp:283-295: a random permutation of the items, of which the first `n` are kept (the
// reference always subsamples, n = 200, :166-167); n <= 0 keeps all items in file order.
static void subsample(dataset_t &ds, std::vector<int> &gt, int n, uint64_t seed) {
    if (n <= 0) return;
    if ((size_t)n > ds.size()) n = (int)ds.size();  // the reference asserts here (:291)
    std::vector<size_t> idx(ds.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::mt19937_64 gen(seed ^ 0x5DEECE66DULL);
    std::shuffle(idx.begin(), idx.end(), gen);  // dim1algebra.hpp:2020-2025
    dataset_t out;
    std::vector<int> g;
    for (int i = 0; i < n; ++i) {
        out.push_back(ds[idx[i]]);
        g.push_back(gt[idx[i]]);
    }
    for (size_t i = n; i < idx.size(); ++i) delete ds[idx[i]];
    ds.swap(out);
    gt.swap(g);
}

int main(int argc, char *argv[]) {
    std::string data, algo, mode = "clustering", ws, upd = "frozen", base = "reference", contr = "f64";
    int T = 2000, D = 2, nsub = 200, substeps = NP8_SUBSTEPS_AUTO;
    long long chunk = 0;
    unsigned long long seed = 0;
    bool seeded = false, verify = false;
    std::string jsonl;
    int tok;
    while ((tok = getopt(argc, argv, "d:a:T:c:s:C:D:w:u:n:p:x:j:S:Vh?")) != EOF) {
        switch (tok) {
            case 'd': data = optarg; break;
            case 'a': algo = optarg; break;
            case 'T': T = std::stoi(optarg); break;
            case 'c': mode = optarg; break;
            case 's': seed = std::stoull(optarg); seeded = true; break;
            case 'C': chunk = std::stoll(optarg); break;
            case 'D': D = std::stoi(optarg); break;
            case 'w': ws = optarg; break;
            case 'u': upd = optarg; break;
            case 'n': nsub = std::stoi(optarg); break;
            case 'p': base = optarg; break;
            case 'x': contr = optarg; break;
            case 'j': jsonl = optarg; break;
            case 'V': verify = true; break;
            case 'S': substeps = std::string(optarg) == "auto" ? NP8_SUBSTEPS_AUTO : std::stoi(optarg); break;
            default: usage(argv[0]); return 1;
        }
    }
    if (data.empty() || algo.empty()) {
        usage(argv[0]);
        return 1;
    }
    if (algo != "algorithm8" && algo != "jain_neal_split" && algo != "triadic") {  // np_main.cpp:222-234
        std::cerr << "Unknown algorithm: " << algo << std::endl;
        return 1;
    }
    if (mode != "clustering") {
        std::cerr << "Unknown likelihood" << std::endl;
        return 107;
    }
    if (!seeded) seed = (unsigned long long)std::chrono::high_resolution_clock::now().time_since_epoch().count();
    if (ws.empty()) ws = "output/" + algo + "/" + data.substr(data.find_last_of('/') + 1) + "/";
    struct stat sb;
    if (stat(ws.c_str(), &sb) == 0) {
        std::cerr << "Directory already exists. Drop out. We don't want to overwrite it or do double work." << std::endl;
        return 106;
    }
    dataset_t dataset;
    std::vector<int> gt;
    if (!read_data(data, D, dataset, gt)) {
        std::cerr << "No data found... Check the file or the contents of the file." << std::endl;
        return 7;
    }
    subsample(dataset, gt, nsub, seed);
    np8_prior prior;
    prior.D = D;
    prior.substeps = substeps;
    if (upd == "mh_g0") {
        prior.param_update = NP8_PARAM_MH_G0;
    } else if (upd == "niw_conjugate") {
        prior.param_update = NP8_PARAM_NIW_CONJUGATE;
        base = "niw";
    } else if (upd != "frozen") {
        usage(argv[0]);
        return 1;
    }
    if (base == "niw") {  // a proper NIW(mu0 = 6, kappa0 = 0.01, nu0 = D + 2, Psi0 = I): E[Sigma] = I
        prior.prior = NP8_PRIOR_NIW;
        prior.kappa = 0.01;
        prior.nu = D + 2.0;
        prior.Lambda.assign((size_t)D * D, 0.0);
        for (int a = 0; a < D; ++a) prior.Lambda[(size_t)a * D + a] = 1.0;
    } else if (base != "reference") {
        usage(argv[0]);
        return 1;
    }
    if (contr == "f32") {
        prior.contraction = NP8_CONTRACT_F32_MFMA;
    } else if (contr != "f64") {
        usage(argv[0]);
        return 1;
    }
    try {
        std::unique_ptr<NealAlgorithm8Hip> smp;
        if (algo == "jain_neal_split")
            smp.reset(new JainNealAlgorithmHip(seed, prior, chunk));
        else if (algo == "triadic")
            smp.reset(new TriadicAlgorithmHip(seed, prior, chunk));
        else
            smp.reset(new NealAlgorithm8Hip(seed, prior, chunk));
        NealAlgorithm8Hip &sampler = *smp;
        MCMC mcmc(sampler);
        mcmc.setVerify(verify);
        std::ofstream jf;
        if (!jsonl.empty()) {
            jf.open(jsonl);
            mcmc.setSweepLog(&jf);
        }
        auto t0 = std::chrono::steady_clock::now();
        mcmc.run(dataset, T);
        double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        sampler.printStatistics();
        // np_main.cpp:476-497: <workspace><YYYYmmdd_HH:MM>/{snapshot,results}*, LATEST symlink
        const std::time_t now = std::time(nullptr);
        std::tm tm = *std::localtime(&now);
        std::stringstream tss;
        tss << std::put_time(&tm, "%Y%m%d_%H:%M");
        const std::string dirname = tss.str();
        for (int which = 0; which < 2; ++which) {
            const membertrix &m = which ? mcmc.getMaxLikelihoodMatrix() : mcmc.getMembershipMatrix();
            Results res(m, gt);
            res.write(ws, dirname, which ? "results" : "snapshot");
            const clustering_performance &cp = res.performance();
            std::cout << (which ? "results" : "snapshot") << ": K=" << m.getClusterCount() << " Purity: " << cp.purity
                      << " Rand Index: " << cp.rand_index << " Adjusted Rand Index: " << cp.adjusted_rand_index
                      << std::endl;
        }
        std::cout << "sweeps: " << T << " seconds: " << sec << " sweeps/s: " << T / sec << std::endl;
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return 2;
    }
    for (auto *d : dataset) delete d;
    return 0;
}
