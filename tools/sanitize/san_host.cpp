// Sanitizer driver (host code only, no GPU): built with -fsanitize=address,undefined by
// `make -C monte_carlo_path_tracing_amd/csrc sanitize` together with the library's host sources
// (scene_io.cpp, bvh.cpp, grid.cpp, image.cpp) and the oracle (oracle/mcpt_oracle.c).
//
// For every (obj, xml) pair on the command line it runs what mcpt_scene_load does on the host --
// Myobj::read / Mylight::read / gather_light_triangles (scene_io.cpp, the reference's Myobj.cpp:10-28,
// Mylight.cpp:11-100) -- then the BVH build, 4-wide collapse and quantisation (bvh.cpp), the
// reference's uniform grid (grid.cpp, Myobj.cpp:78-162), the tone map and BMP writer (image.cpp),
// and the same file through the oracle's loader plus a few oracle queries and a tiny render.  A
// malformed file must come back as an error, never as a sanitizer report.
//
//   san_host OUT_DIR obj1 xml1 [obj2 xml2 ...]
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mcpt_internal.h"

extern "C" {
#include "mcpt_oracle.h"
}

using namespace mcpt;

static int run_library(const char* obj, const char* xml, const std::string& out_dir, int idx) {
    HostScene hs;
    std::vector<LightDef> lights;
    std::string err;
    if (!load_obj_mtl(obj, hs, err) || !load_light_xml(xml, hs, lights, err)) return 1;
    if (!finalize_scene(hs, lights, err)) return 2;
    std::vector<int32_t> all(hs.F), lt(hs.light_facet);
    for (int f = 0; f < hs.F; f++) all[f] = f;
    for (int leaf : {1, 2, 8}) {
        const Bvh b = build_bvh(hs, all, leaf), lb = build_bvh(hs, lt, leaf);
        const std::vector<BvhNode4> b4 = collapse_bvh4(b), lb4 = collapse_bvh4(lb);
        const std::vector<BvhNode4Q> q = quantize_bvh4(b4), lq = quantize_bvh4(lb4);
        if (q.size() != b4.size() || lq.size() != lb4.size()) return 3;
        // the 8-wide trees (leaf 8: binary leaves of up to 8 triangles, split by build_bvh8): every reference of
        // the binary tree once (a facet split spatially -- this build makes spatial splits in every tree -- has
        // several references)
        for (const Bvh* bb : {&b, &lb}) {
            const Bvh8 b8 = build_bvh8(hs, *bb);
            std::vector<int> seen(hs.F, 0), want(hs.F, 0);
            for (int32_t f : bb->leaf_facets)
                if (f >= 0 && f < hs.F) want[f]++;
            size_t used = 0;
            for (int32_t f : b8.tri_facets)
                if (f >= 0) {
                    if (f >= hs.F || ++seen[f] > want[f]) return 6;
                    used++;
                }
            if (used != bb->leaf_facets.size() || b8.nodes.empty()) return 6;
        }
    }
    const double eye[3] = {hs.has_cam ? hs.cam.eye[0] : 0.0, hs.has_cam ? hs.cam.eye[1] : 0.0,
                           hs.has_cam ? hs.cam.eye[2] : 0.0};
    if (std::isfinite(eye[0]) && std::isfinite(eye[1]) && std::isfinite(eye[2])) {
        const Grid g = build_grid(hs, eye, 1000);
        (void)g;
    }
    const int W = 7, H = 5;
    std::vector<double> hdr(3 * W * H);
    for (size_t k = 0; k < hdr.size(); k++) hdr[k] = (k % 5 == 0) ? NAN : (k % 7 == 0 ? -1.0 : 0.37 * k);
    std::vector<uint8_t> rgb8(3 * W * H);
    if (mcpt_tone_map(hdr.data(), W, H, 380.0, 0.25, rgb8.data())) return 4;
    const std::string bmp = out_dir + "/san_" + std::to_string(idx) + ".bmp";
    if (mcpt_write_bmp(bmp.c_str(), rgb8.data(), W, H)) return 5;
    std::remove(bmp.c_str());
    return 0;
}

static int run_oracle(const char* obj, const char* xml) {
    orc_scene* s = orc_scene_load(obj, xml);
    if (!s) return 1;
    int F = 0, M = 0, NL = 0;
    orc_scene_counts(s, &F, &M, &NL);
    const double eye[3] = {28.2792, 5.2, 1.23612e-06};
    orc_grid_build(s, eye, 1000);
    double tbg[3];
    for (int k = 0; k < 16; k++) {
        const double ro[3] = {0.1 * k, 1.0, -0.5 * k}, rd[3] = {0.6, -0.48, 0.64};
        (void)orc_closest_hit(s, ro, rd, -1, tbg);
        (void)orc_closest_light_hit(s, ro, rd, -1, tbg);
        const double x1[3] = {0.3 * k, 0.01, 0.2 * k}, n[3] = {0, 1, 0};
        int cnt = 0;
        std::vector<int> idx(NL + 1);
        std::vector<double> w(NL + 1);
        (void)orc_light_prep(s, x1, n, &cnt, idx.data(), w.data());
        double o6[6];
        orc_light_sample_u(s, x1, n, 0.37, 0.5, 0.5, o6);
    }
    if (F > 0 && F < 200000) {  // a tiny counter-RNG render of every integrator
        orc_camera cam;
        std::memset(&cam, 0, sizeof cam);
        if (orc_scene_camera(s, &cam) != 0) {
            const double e[3] = {28.2792, 5.2, 1.23612e-06}, l[3] = {0, 2.8, 0}, u[3] = {0, 1, 0};
            std::memcpy(cam.eye, e, sizeof e);
            std::memcpy(cam.lookat, l, sizeof l);
            std::memcpy(cam.up, u, sizeof u);
            cam.fovy = 20.1143;
            cam.dist_scale = 2.0;
        }
        cam.width = 8;
        cam.height = 6;
        std::vector<double> img(3 * 8 * 6);
        uint64_t stats[4];
        for (int mode = 0; mode < 4; mode++)
            (void)orc_render(s, &cam, mode, 20240430ull, 2, 0, 2, 1, 0, 1, img.data(), stats);
    }
    orc_scene_free(s);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 4 || (argc - 2) % 2) {
        std::fprintf(stderr, "usage: %s OUT_DIR obj xml [obj xml ...]\n", argv[0]);
        return 2;
    }
    const std::string out_dir = argv[1];
    int loaded = 0, rejected = 0, oloaded = 0, orejected = 0;
    for (int a = 2; a + 1 < argc; a += 2) {
        const int r = run_library(argv[a], argv[a + 1], out_dir, a);
        (r == 0 ? loaded : rejected)++;
        const int ro = run_oracle(argv[a], argv[a + 1]);
        (ro == 0 ? oloaded : orejected)++;
    }
    std::printf("san_host: %d scene pairs; library loaded %d rejected %d; oracle loaded %d rejected %d; no sanitizer report\n",
                (argc - 2) / 2, loaded, rejected, oloaded, orejected);
    return 0;
}
