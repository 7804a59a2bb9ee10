// Host-only check of the level-0 NIW auxiliary screen (np8_device.h niw_aux_all_below): wherever it declares every
// auxiliary of an item skippable, the level-1 screen (niw_aux_ll_screened) must skip each one, for any draw.  The
// draws are keyed (Philox), so many (item, auxiliary) keys sample the generators; also reports how often level 0
// fires, so the bound is not vacuous.  Built and run by tests/test_niw_screen.py (no GPU: no HIP API call).
#include <cmath>
#include <cstdio>
#include <vector>

#include "np8_device.h"

using namespace np8;

static double smax_of(int D, double nu) {  // as np8_capi.hip builds hyp's smax
    const double rmax = std::sqrt(-2.0 * std::log(std::ldexp(1.0, -33))) * (1.0 + 1e-9);
    double s = 0.0;
    for (int a = 1; a < D; ++a) {
        const double d = 0.5 * (nu - a) - 1.0 / 3.0, cc = 1.0 / std::sqrt(9.0 * d);
        const double v1 = 1.0 + cc * rmax;
        s += std::log(2.0 * d * std::max(1.0, v1 * v1 * v1) * (1.0 + 1e-9));
    }
    return s;
}

int main() {
    long fired = 0, cases = 0, checked = 0, bad = 0;
    const int Ds[] = {8, 32, 64};
    const double rsks[] = {10.0, 3.0, 0.5};
    for (int D : Ds)
        for (double rsk : rsks) {
            const double nu = D + 2.0, caux = -0.5 * D * kLog2Pi, smax = smax_of(D, nu);
            for (int ni = 0; ni <= 60; ++ni) {
                const double nd = 0.75 * ni;
                for (int ti = 0; ti < 40; ++ti) {
                    const double thr = -400.0 + 15.0 * ti;
                    ++cases;
                    if (!niw_aux_all_below(nd, nu, rsk, caux, smax, thr)) continue;
                    ++fired;
                    for (uint64_t i = 0; i < 400; ++i)
                        for (int m = 0; m < 3; ++m) {
                            ++checked;
                            const double v = niw_aux_ll_screened(7u + ni, i, 11u + ti, m, D, nu, nd, rsk, caux, smax, thr);
                            if (v != kZeroLogWeight) ++bad;
                        }
                }
            }
        }
    std::printf("cases %ld fired %ld checked %ld bad %ld\n", cases, fired, checked, bad);
    return (bad == 0 && fired > 0) ? 0 : 1;
}
