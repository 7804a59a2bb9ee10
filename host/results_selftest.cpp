// results_selftest.cpp -- writes the output files of a small hand-built membertrix (no GPU needed);
// tests/test_host_driver.py checks their format against the reference's (src/np_results.cpp).
//
// results_selftest --metrics <file>: the product's clustering_performance::calculate (the one that
// writes results.score.txt, reference src/clustering_performance.cpp:38-82) over label pairs read
// from <file> -- two lines per case, the ground truth then the result, whitespace-separated ints --
// printing "purity rand_index adjusted_rand_index" per case at full precision.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>

#include "np_results.h"

static int metrics(const char *path) {
    std::ifstream in(path);
    if (!in) {
        std::cerr << "results_selftest: cannot read " << path << std::endl;
        return 2;
    }
    std::string lt, lr;
    while (std::getline(in, lt) && std::getline(in, lr)) {
        std::vector<int> a, b;
        std::istringstream st(lt), sr(lr);
        for (int v; st >> v;) a.push_back(v);
        for (int v; sr >> v;) b.push_back(v);
        clustering_performance cp;
        cp.calculate(a, b);
        std::printf("%.17g %.17g %.17g\n", cp.purity, cp.rand_index, cp.adjusted_rand_index);
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc == 3 && std::string(argv[1]) == "--metrics") return metrics(argv[2]);
    if (argc < 2) {
        std::cerr << "usage: results_selftest <workspace/> | --metrics <file>" << std::endl;
        return 1;
    }
    membertrix m;
    std::vector<data_t> pts = {{1.5, 2.25}, {1.0, 2.0}, {-3.0, 0.5}, {1.25, 2.5}, {-2.5, 0.75}};
    for (auto &p : pts) m.addData(p);
    cluster_t a{{1.25, 2.25}, {0.1, 0.0, 0.0, 0.2}}, b{{-2.75, 0.625}, {0.3, 0.01, 0.01, 0.4}};
    const cluster_id_t ia = m.addCluster(new cluster_t(a)), ib = m.addCluster(new cluster_t(b));
    for (data_id_t i : {0, 1, 3}) m.assign(ia, i);
    for (data_id_t i : {2, 4}) m.assign(ib, i);
    std::vector<int> gt = {0, 0, 1, 0, 1};
    Results r(m, gt);
    r.write(argv[1], "20261015_12:00", "results");
    std::cout << "purity " << r.performance().purity << std::endl;
    return 0;
}
