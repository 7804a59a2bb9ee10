// results_selftest.cpp -- writes the output files of a small hand-built membertrix (no GPU needed);
// tests/test_host_driver.py checks their format against the reference's (src/np_results.cpp).
#include <iostream>

#include "np_results.h"

int main(int argc, char **argv) {
    if (argc < 2) {
        std::cerr << "usage: results_selftest <workspace/>" << std::endl;
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
