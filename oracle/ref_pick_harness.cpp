// TEST INFRASTRUCTURE ONLY: exposes the reference's own random_weighted_pick
// (/root/reference/include/helper/dim1algebra.hpp:2078-2104) behind a C ABI so tests can feed it a
// chosen uniform and compare its index with the oracle restatement and the HIP pick.  The header is
// compiled where it lies (-I/root/reference/include/helper); nothing of it is copied here.
#include <cmath>
#include <cstdint>
#include <vector>

#include <dim1algebra.hpp>

namespace {
// A URBG with a 64-bit range that returns one preset word: std::generate_canonical<double,53> then
// draws exactly once and yields word / 2^64, so a 53-bit u in [0,1) is passed through unchanged.
struct FixedWord {
    using result_type = uint64_t;
    uint64_t w;
    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return ~uint64_t(0); }
    result_type operator()() { return w; }
};
}  // namespace

extern "C" int64_t np8ref_weighted_pick(const double *w, int64_t n, double u) {
    std::vector<double> v(w, w + n);
    FixedWord g{(uint64_t)std::ldexp(u, 64)};
    return (int64_t)algebra::random_weighted_pick(v.begin(), v.end(), g);
}
