// np_results.cpp -- see np_results.h (reference: src/np_results.cpp:39-196).
#include "np_results.h"

#include <algorithm>
#include <filesystem>
#include <fstream>
#include <iostream>

namespace fs = std::filesystem;

Results::Results(const membertrix &trix, const std::vector<int> &ground_truth) : _trix(trix), _gt(ground_truth) {
    std::vector<int> res(_trix.count());
    for (size_t i = 0; i < _trix.count(); ++i) res[i] = _trix.getClusterId((data_id_t)i);
    _perf.calculate(_gt, res);
}

void Results::write(const std::string &workspace, const std::string &path, const std::string &basename) {
    const std::string ws_path = workspace + path;
    std::error_code ec;
    fs::create_directories(ws_path, ec);  // the reference logs and continues on failure (:49-52)
    const std::string latest = workspace + "LATEST";
    if (fs::exists(fs::symlink_status(latest))) fs::remove(latest, ec);
    fs::create_symlink(path, latest, ec);

    std::vector<cluster_id_t> ids;
    for (const auto &kv : _trix.getClusters()) ids.push_back(kv.first);
    std::sort(ids.begin(), ids.end());
    const dataset_t &data = _trix.getData();
    int k = 0;
    for (cluster_id_t id : ids) {  // np_results.cpp:67-92
        std::ofstream f(ws_path + '/' + basename + std::to_string(k) + ".txt");
        for (size_t i = 0; i < _trix.count(); ++i) {
            if (_trix.getClusterId((data_id_t)i) != id) continue;
            for (double d : *data[i]) f << d << " ";
            f << std::endl;
        }
        ++k;
    }
    writeOctave(ws_path + '/' + basename + ".txt");
    _perf.write(ws_path + '/' + basename + ".score.txt");
}

// Octave text format with Eigen's IOFormats of np_results.cpp:109,148 at the stream's default
// precision: mu rows " m1 m2 ...", sigma matrices " a b \nc d".
void Results::writeOctave(const std::string &fname) const {
    std::ofstream f(fname);
    std::vector<cluster_id_t> ids;
    for (const auto &kv : _trix.getClusters()) ids.push_back(kv.first);
    std::sort(ids.begin(), ids.end());
    const size_t K = ids.size();
    if (K == 0) return;
    const auto &cl = _trix.getClusters();
    const size_t D = cl.at(ids[0])->mu.size();
    f << "# name: mu" << std::endl;
    f << "# type: matrix" << std::endl;
    f << "# rows: " << K << std::endl;
    f << "# columns: " << D << std::endl;
    for (cluster_id_t id : ids) {
        const cluster_t &c = *cl.at(id);
        f << " ";
        for (size_t a = 0; a < D; ++a) f << (a ? " " : "") << c.mu[a];
        f << std::endl;
    }
    f << std::endl << std::endl;
    f << "# name: sigma" << std::endl;
    f << "# type: matrix" << std::endl;
    f << "# ndims: 3" << std::endl;
    f << " " << D << " " << D << " " << K << std::endl;
    for (cluster_id_t id : ids) {
        const cluster_t &c = *cl.at(id);
        f << " ";
        for (size_t a = 0; a < D; ++a) {
            if (a) f << " \n";
            for (size_t b = 0; b < D; ++b) f << (b ? " " : "") << c.sigma[a * D + b];
        }
        f << std::endl;
    }
}
