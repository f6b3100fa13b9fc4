// Uniform grid of the reference (Myobj::cal_scene_boundingbox + Myobj::meshing, Myobj.cpp:78-162),
// built on the host for the GPU's reference-faithful traversal mode (MCPT_ACCEL_GRID).
//
//  * bounding box: every facet vertex and the camera eye (Myobj.cpp:84-88; no ray/box clipping);
//  * cell edge d = (largest box extent) / n0^(1/3); cells per axis lim = floor(len / d) + 2
//    (Myobj.cpp:405) -- the grid spans [0, lim] per axis, so (lim + 1)^3 cells are stored;
//  * a facet is listed in every cell its own axis-aligned box overlaps, cells scanned in facet order
//    (so a cell's list is in ascending facet id, which makes the traversal's first-wins tie rule the
//    same as the BVH's lower-facet rule).
// The device side (grid_trace in render.hip) runs the 3D-DDA with the reference's in-cell acceptance.
#include <cfloat>
#include <cmath>

#include "mcpt_internal.h"

namespace mcpt {

Grid build_grid(const HostScene& s, const double eye[3], int n0) {
    Grid g;
    for (int i = 0; i < 3; i++) {
        g.mn[i] = eye[i];
        g.mx[i] = eye[i];
        g.eye[i] = eye[i];
    }
    g.n0 = n0;
    for (int f = 0; f < s.F; f++)
        for (int k = 0; k < 3; k++)
            for (int i = 0; i < 3; i++) {
                const double v = s.pos[9 * f + 3 * k + i];
                g.mn[i] = std::fmin(g.mn[i], v);
                g.mx[i] = std::fmax(g.mx[i], v);
            }
    double len[3];
    for (int i = 0; i < 3; i++) len[i] = g.mx[i] - g.mn[i];
    g.d = std::fmax(std::fmax(len[0], len[1]), len[2]) / std::pow((double)n0, 1.0 / 3);
    // a box of zero or non-finite extent (no facets, a single point, inf coordinates) has no cell
    // size; the reference would divide by it (Myobj.cpp:119).  Refused (g.ok stays false) -- found
    // by the sanitizer build (`make sanitize`), as was the cell-count cap below
    if (!(g.d > 0) || !std::isfinite(g.d) || !std::isfinite(len[0] + len[1] + len[2])) return g;
    g.inv_d = 1.0 / g.d;
    for (int i = 0; i < 3; i++) {
        g.lim[i] = (int)std::floor(len[i] / g.d) + 2;
        g.gd[i] = g.lim[i] + 1;
    }
    const size_t ncell = (size_t)g.gd[0] * g.gd[1] * g.gd[2];
    if (ncell > (size_t)1 << 31) return g;  // n0 beyond any sane grid
    // per facet: its cell range per axis (the facet's own box)
    std::vector<int> rng(6 * (size_t)s.F);
    for (int f = 0; f < s.F; f++) {
        for (int i = 0; i < 3; i++) {
            double lo = DBL_MAX, hi = -DBL_MAX;
            for (int k = 0; k < 3; k++) {
                const double v = s.pos[9 * f + 3 * k + i];
                lo = std::fmin(lo, v);
                hi = std::fmax(hi, v);
            }
            // a facet with a non-finite coordinate is listed nowhere (fmin / fmax skip its NaNs)
            const bool fin = std::isfinite(lo) && std::isfinite(hi);
            rng[6 * f + 2 * i] = fin ? (int)std::floor((lo - g.mn[i]) / g.d) : 1;
            rng[6 * f + 2 * i + 1] = fin ? (int)std::floor((hi - g.mn[i]) / g.d) : 0;
        }
    }
    // counting pass, prefix sum, fill pass (CSR: cell -> facets in facet order)
    g.cell_start.assign(ncell + 1, 0);
    auto each_cell = [&](int f, auto&& fn) {
        const int* r = &rng[6 * (size_t)f];
        for (int i = r[0]; i <= r[1]; i++)
            for (int j = r[2]; j <= r[3]; j++)
                for (int k = r[4]; k <= r[5]; k++) fn(((size_t)i * g.gd[1] + j) * g.gd[2] + k);
    };
    for (int f = 0; f < s.F; f++) each_cell(f, [&](size_t c) { g.cell_start[c + 1]++; });
    for (size_t c = 0; c < ncell; c++) g.cell_start[c + 1] += g.cell_start[c];
    g.cell_tri.resize(std::max<size_t>((size_t)g.cell_start[ncell], 1));
    std::vector<int32_t> fill(g.cell_start.begin(), g.cell_start.end() - 1);
    for (int f = 0; f < s.F; f++) each_cell(f, [&](size_t c) { g.cell_tri[fill[c]++] = f; });
    g.ok = true;
    return g;
}

}  // namespace mcpt
