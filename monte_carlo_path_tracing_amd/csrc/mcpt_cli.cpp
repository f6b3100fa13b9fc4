// mcpt_render -- the reference's render driver (main.cpp:497-600) as a host C++ program over the
// C ABI: load the scene (Myobj::read / Mylight::read, main.cpp:500-504), set the camera
// (main.cpp:507-510, eye pulled back 2x by default), render(scene, camera, spp, mode), tone-map
// (380, 0.25; main.cpp:583) and save the BMP (main.cpp:596).  Unlike the reference, size, spp,
// integrator and output path are flags instead of edits to main.cpp.
//
//   mcpt_render --scene scenes/veach-mis/veach-mis [--width 1280 --height 720] [--spp 10]
//               [--mode mis|brdf|shade|shade-area] [--seed 20240430] [--out test.bmp] [--hdr out.pfm] [--progress]
//               [--grid] [--devices 0,1,2,3,4,5,6,7] [--precision fp64|fp32]
//   --devices renders on several GPUs of this node: the sample range is split into one contiguous shard
//   per listed device, rendered concurrently, and summed by ONE RCCL reduce into the first device
//   (mcpt_render_opts.devices; the reference itself is single-threaded, README.md:418).
//   --grid traverses the reference's uniform grid (Myobj.cpp:78-162, n0 = 100000) instead of the BVH.
//   --precision fp32 selects the opt-in FP32_STABLE light prep (MCPT_RENDER_PRECISION_FP32); fp64 (the
//   reference's, default) otherwise.
//   --progress prints the share of camera samples dispatched (the reference prints per-row progress
//   and updates its EasyX window, main.cpp:539-592) through mcpt_render_opts.progress.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mcpt.h"

namespace {

int print_progress(void* user, uint64_t done, uint64_t total) {
    int* last = static_cast<int*>(user);
    const int pct = total ? (int)(100 * done / total) : 100;
    if (pct / 10 != *last / 10) {
        std::fprintf(stderr, "\rrendering: %3d%% of %llu camera samples dispatched", pct, (unsigned long long)total);
        if (pct == 100) std::fprintf(stderr, "\n");
        *last = pct;
    }
    return 0;
}

// render(scene, camera, spp, mode): main.cpp:547-588 lifted into a function.
int render(mcpt_scene* scene, const mcpt_camera& cam, int spp, int mode, uint64_t seed, bool progress, bool grid, int flags,
           const std::vector<int32_t>& devices, std::vector<double>& hdr, mcpt_stats* st) {
    hdr.assign(3ull * cam.width * cam.height, 0.0);
    mcpt_render_opts o;
    mcpt_render_opts_init(&o);
    o.spp = spp;
    o.mode = mode;
    o.seed = seed;
    o.accel = grid ? MCPT_ACCEL_GRID : MCPT_ACCEL_BVH;
    o.flags = flags;
    if (!devices.empty()) {  // one process, several GPUs: shards + one RCCL reduce
        o.num_devices = (int32_t)devices.size();
        o.devices = devices.data();
    }
    int last = -10;
    if (progress) {
        o.progress = print_progress;
        o.progress_user = &last;
    }
    return mcpt_render(scene, &cam, &o, hdr.data(), st);
}

bool write_pfm(const char* path, const std::vector<double>& hdr, int W, int H) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    std::fprintf(f, "PF\n%d %d\n-1.0\n", W, H);
    std::vector<float> row(3ull * W);
    for (int i = H - 1; i >= 0; i--) {  // PFM is bottom-up
        for (int k = 0; k < 3 * W; k++) row[k] = static_cast<float>(hdr[3ull * i * W + k]);
        std::fwrite(row.data(), sizeof(float), row.size(), f);
    }
    std::fclose(f);
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    std::string scene_base = "scenes/veach-mis/veach-mis", out = "test.bmp", hdr_out;
    int W = 1280, H = 720, spp = 10, mode = MCPT_MODE_MIS;
    double dist_scale = 2.0;
    uint64_t seed = 20240430;
    bool xml_cam = false, progress = false, grid = false;
    int flags = 0;
    std::vector<int32_t> devices;
    for (int a = 1; a < argc; a++) {
        auto next = [&]() -> const char* {
            if (a + 1 >= argc) {
                std::fprintf(stderr, "missing value for %s\n", argv[a]);
                std::exit(2);
            }
            return argv[++a];
        };
        if (!std::strcmp(argv[a], "--scene")) scene_base = next();
        else if (!std::strcmp(argv[a], "--width")) W = std::atoi(next());
        else if (!std::strcmp(argv[a], "--height")) H = std::atoi(next());
        else if (!std::strcmp(argv[a], "--spp")) spp = std::atoi(next());
        else if (!std::strcmp(argv[a], "--mode")) {
            const char* m = next();
            if (!std::strcmp(m, "mis")) mode = MCPT_MODE_MIS;
            else if (!std::strcmp(m, "brdf")) mode = MCPT_MODE_BRDF;
            else if (!std::strcmp(m, "shade")) mode = MCPT_MODE_SHADE;
            else if (!std::strcmp(m, "shade-area")) mode = MCPT_MODE_SHADE_AREA;
            else {
                std::fprintf(stderr, "unknown --mode %s (mis, brdf, shade, shade-area)\n", m);
                return 2;
            }
        }
        else if (!std::strcmp(argv[a], "--seed")) seed = std::strtoull(next(), nullptr, 10);
        else if (!std::strcmp(argv[a], "--out")) out = next();
        else if (!std::strcmp(argv[a], "--hdr")) hdr_out = next();
        else if (!std::strcmp(argv[a], "--dist-scale")) dist_scale = std::atof(next());
        else if (!std::strcmp(argv[a], "--xml-camera")) xml_cam = true;
        else if (!std::strcmp(argv[a], "--progress")) progress = true;
        else if (!std::strcmp(argv[a], "--grid")) grid = true;
        else if (!std::strcmp(argv[a], "--precision")) {
            const char* v = next();
            if (!std::strcmp(v, "fp32")) flags |= MCPT_RENDER_PRECISION_FP32;
            else if (std::strcmp(v, "fp64")) {
                std::fprintf(stderr, "--precision: fp64 or fp32, not %s\n", v);
                return 2;
            }
        }
        else if (!std::strcmp(argv[a], "--devices")) {
            for (const char* p = next(); *p;) {
                char* e = nullptr;
                devices.push_back((int32_t)std::strtol(p, &e, 10));
                if (e == p) {
                    std::fprintf(stderr, "bad --devices list\n");
                    return 2;
                }
                p = *e == ',' ? e + 1 : e;
            }
        }
        else {
            std::fprintf(stderr, "unknown option %s\n", argv[a]);
            return 2;
        }
    }
    mcpt_scene* scene = nullptr;
    if (mcpt_scene_load((scene_base + ".obj").c_str(), (scene_base + ".xml").c_str(), &scene) != MCPT_OK) {
        std::fprintf(stderr, "scene load failed: %s\n", mcpt_last_error());
        return 1;
    }
    int32_t nf, nm, nl;
    mcpt_scene_counts(scene, &nf, &nm, &nl);
    std::printf("facets %d, materials %d, light triangles %d\n", nf, nm, nl);
    mcpt_camera cam{};
    if (!xml_cam || mcpt_scene_camera(scene, &cam) != MCPT_OK) {  // main.cpp:507-510
        const double eye[3] = {28.2792, 5.2, 1.23612e-06}, look[3] = {0.0, 2.8, 0.0}, up[3] = {0, 1, 0};
        std::memcpy(cam.eye, eye, sizeof eye);
        std::memcpy(cam.lookat, look, sizeof look);
        std::memcpy(cam.up, up, sizeof up);
        cam.fovy = 20.1143;
    }
    cam.dist_scale = dist_scale;
    cam.width = W;
    cam.height = H;
    std::vector<double> hdr;
    mcpt_stats st{};
    const auto t0 = std::chrono::steady_clock::now();
    if (render(scene, cam, spp, mode, seed, progress, grid, flags, devices, hdr, &st) != MCPT_OK) {
        std::fprintf(stderr, "render failed: %s\n", mcpt_last_error());
        return 1;
    }
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("%dx%d @ %d spp (%s): %.3f s wall, %.3f s device, %.2f Msamples/s on %d device(s)\n", W, H, spp,
                mode == MCPT_MODE_MIS ? "MIS" : mode == MCPT_MODE_BRDF ? "BRDF" : mode == MCPT_MODE_SHADE ? "shade" : "shade-area",
                sec, st.seconds,
                st.camera_samples / st.seconds * 1e-6, st.devices_used);
    if (st.devices_used > 1) {  // where a multi-device call's time went
        std::printf("  comm init %.3f s, device setup %.3f s (max), reduce %.4f s; per device:", st.comm_init_seconds,
                    st.device_setup_seconds, st.reduce_seconds);
        for (int u = 0; u < st.devices_used && u < MCPT_STATS_MAX_DEVICES; u++) std::printf(" %.3f", st.device_seconds[u]);
        std::printf(" s\n");
    }
    std::vector<uint8_t> rgb8(hdr.size());
    mcpt_tone_map(hdr.data(), W, H, 380.0, 0.25, rgb8.data());  // main.cpp:583
    if (mcpt_write_bmp(out.c_str(), rgb8.data(), W, H) != MCPT_OK) {
        std::fprintf(stderr, "%s\n", mcpt_last_error());
        return 1;
    }
    if (!hdr_out.empty() && !write_pfm(hdr_out.c_str(), hdr, W, H)) {
        std::fprintf(stderr, "cannot write %s\n", hdr_out.c_str());
        return 1;
    }
    mcpt_scene_destroy(scene);
    return 0;
}
