// Host check of monte_carlo_path_tracing_amd/csrc/acos_cr.h (driven by tools/acos_cr_check.py, which
// compares against mpmath): reads doubles x from argv[1], writes per x: acos_cr(x), glibc acos(x), and
// acos_cr with the libm start value moved by -2, -1, +1, +2 ulp (ocml's acos is within 1 ulp, so the
// Newton step must land on the same result from any nearby start).
#include <cmath>
#include <cstdio>
#include <vector>

#include "acos_cr.h"

using namespace mcpt;

static double from_start(double x, double y0s, int ulps) {
    double y0 = y0s;
    for (int k = 0; k < (ulps < 0 ? -ulps : ulps); k++) y0 = std::nextafter(y0, ulps < 0 ? -INFINITY : INFINITY);
    if (x >= 0.0) return y0 + acos_newton_corr(x, y0);
    const double c = acos_newton_corr(-x, y0);
    const DD d = dd_two_sum(0x1.921fb54442d18p+1, -y0);
    return d.h + ((d.l + 0x1.1a62633145c07p-53) - c);
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<double> xs;
    double v;
    while (std::fread(&v, sizeof v, 1, f) == 1) xs.push_back(v);
    std::fclose(f);
    FILE* o = std::fopen(argv[2], "wb");
    if (!o) return 2;
    for (double x : xs) {
        const double ax = x < 0 ? -x : x;
        const double y0 = std::acos(ax);
        double r[6] = {acos_cr(x), std::acos(x), 0, 0, 0, 0};
        const int d[4] = {-2, -1, 1, 2};
        for (int k = 0; k < 4; k++) r[2 + k] = (ax < 1.0) ? from_start(x, y0, d[k]) : r[0];
        std::fwrite(r, sizeof r, 1, o);
    }
    std::fclose(o);
    return 0;
}
