// TEST INFRASTRUCTURE ONLY -- golden-vector generator built against the compiled reference.
//
// Built by `make -C oracle ref` (oracle/Makefile) from the reference's own library translation
// units where they lie under /root/reference (vec, matrix3d, BRDF, RadianceRGB, Myobj, Mylight,
// pugixml), with oracle/fakeclock.h force-included so the clock-seeded RNG is replayable.
// main.cpp is NOT compiled: it includes the Windows-only EasyX <graphics.h> (main.cpp:13), which
// this image lacks, so it is unbuildable here.  The three integrators of main.cpp (shade
// main.cpp:269-344, shade_with_brdf :348-399, shade_with_mis :402-494) and the camera of main.cpp:547-564 are
// therefore restated below in a few lines each, calling the REAL reference components for
// everything else (grid traversal, light prep/sampling, BRDF, RNG sites).  Outputs go to
// tests/golden/*.npy and pin oracle/mcpt_oracle.c (tests/test_oracle_golden.py).
//
// usage: ref_harness <scene.obj> <lights.xml> <outdir> [stat <mode> <W> <H> <spp> <row0> <row1> <clock0>]
#define TINYOBJLOADER_IMPLEMENTATION
#include "Myobj.h"
#include "Mylight.h"
#include "BRDF.h"
#include "matrix3d.h"
#include "RadianceRGB.h"

#include <cstdint>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

using u64 = unsigned long long;

// ------------------------------------------------------------------------------------------
// minimal .npy writer
static void write_npy(const std::string& path, const char* descr, const std::vector<size_t>& shape,
                      const void* data, size_t elem) {
    std::string shp = "(";
    size_t n = 1;
    for (size_t i = 0; i < shape.size(); i++) {
        shp += std::to_string(shape[i]);
        shp += (shape.size() == 1 || i + 1 < shape.size()) ? "," : "";
        n *= shape[i];
    }
    shp += ")";
    std::string hdr = std::string("{'descr': '") + descr + "', 'fortran_order': False, 'shape': " + shp + ", }";
    while ((10 + hdr.size() + 1) % 64) hdr += ' ';
    hdr += '\n';
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { perror(path.c_str()); exit(2); }
    const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    fwrite(magic, 1, 8, f);
    unsigned short hl = (unsigned short)hdr.size();
    fwrite(&hl, 2, 1, f);
    fwrite(hdr.data(), 1, hdr.size(), f);
    fwrite(data, elem, n, f);
    fclose(f);
}
static void npy_f64(const std::string& p, const std::vector<double>& v, size_t cols) {
    write_npy(p, "<f8", {v.size() / cols, cols}, v.data(), 8);
}
static void npy_f32(const std::string& p, const std::vector<float>& v, size_t cols) {
    write_npy(p, "<f4", {v.size() / cols, cols}, v.data(), 4);
}
static void npy_i64(const std::string& p, const std::vector<long long>& v, size_t cols) {
    write_npy(p, "<i8", {v.size() / cols, cols}, v.data(), 8);
}

// ------------------------------------------------------------------------------------------
static Myobj* veach;
static Mylight* lights;
static std::vector<size_t> shape_off;  // global facet index = shape_off[s] + f

static long long gid(size_t s, size_t f) { return (long long)(shape_off[s] + f); }
static u64& clk() { return std::chrono::mcpt_fake_clock::ctr; }

static tinyobj::material_t mat_of(size_t s, size_t f) {
    return veach->reader.GetMaterials().at(veach->reader.GetShapes().at(s).mesh.material_ids[f]);
}
static vec kd_of(const tinyobj::material_t& m) { return vec(m.diffuse[0], m.diffuse[1], m.diffuse[2]); }
static vec ks_of(const tinyobj::material_t& m) { return vec(m.specular[0], m.specular[1], m.specular[2]); }

static vec interp(const std::array<vec, 3>& t, double b, double g) {
    return t[0] * (1.0 - b - g) + t[1] * b + t[2] * g;
}
static double rr_uniform() {  // the RR draw of main.cpp:377-380 / :431-434
    unsigned seed1 = std::chrono::system_clock::now().time_since_epoch().count();
    std::default_random_engine generator(seed1);
    std::uniform_real_distribution<double> distribution(0.0, 1.0);
    return distribution(generator);
}

// Restatement of main.cpp:348-399 (shade_with_brdf), reference components underneath.
static RadianceRGB ref_shade_brdf(intersec_result point, vec wo) {
    vec p = interp(veach->get_vertexes_of_facet(point.s, point.f), point.beta, point.gamma);
    vec N = interp(veach->get_normals_of_facet(point.s, point.f), point.beta, point.gamma).normalized();
    if (N.dot_product(wo) < 0) return RadianceRGB(0, 0, 0);
    auto li = lights->islight.find(triangle(point.s, point.f));
    if (li != lights->islight.end()) return li->second;
    tinyobj::material_t mtl = mat_of(point.s, point.f);
    RadianceRGB L;
    if (rr_uniform() > 0.6) return L;
    sampledRay wi = BRDF::sample_from_phong(N, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
    if (wi.dir.dot_product(N) < 0) return L;
    intersec_result rsq = veach->closet_ray_intersect(p, wi.dir, triangle(point.s, point.f));
    if (rsq.isIntersec) {
        BRDF brdf = BRDF::get_brdf_phong(N, wi.dir, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
        L = ref_shade_brdf(rsq, wi.dir * -1) * brdf * (wi.dir.dot_product(N) / wi.pdf / 0.6);
    }
    return L;
}

// Restatement of main.cpp:402-494 (shade_with_mis), reference components underneath; the
// stale light-sampler state after recursion A (main.cpp:443 vs :487) happens naturally here.
static RadianceRGB ref_shade_mis(intersec_result point, vec wo) {
    vec p = interp(veach->get_vertexes_of_facet(point.s, point.f), point.beta, point.gamma);
    vec N = interp(veach->get_normals_of_facet(point.s, point.f), point.beta, point.gamma).normalized();
    if (N.dot_product(wo) < 0) return RadianceRGB(0, 0, 0);
    auto li = lights->islight.find(triangle(point.s, point.f));
    if (li != lights->islight.end()) return li->second;
    tinyobj::material_t mtl = mat_of(point.s, point.f);
    if (rr_uniform() > 0.6) return RadianceRGB();
    RadianceRGB L_light;
    lights->prepared_for_lights_spherical_triangle_sampling(p, N, *veach);
    sampledLightPoint lp = lights->lights_spherical_triangle_sampling(p, N, *veach);
    vec wl = (lp.coord - p).normalized();
    if (wl.dot_product(N) > 0) {
        intersec_result r1 = veach->closet_ray_intersect(p, wl, triangle(point.s, point.f));
        if (r1.isIntersec) {
            BRDF brdf = BRDF::get_brdf_phong(N, wl, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
            double phongPdf = BRDF::eval_sample_from_phong_pdf(N, wl, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
            L_light = ref_shade_mis(r1, wl * -1) * brdf * (wl.dot_product(N) / (lp.prob + phongPdf) / 0.6);
        }
    }
    RadianceRGB L_brdf;
    sampledRay wi = BRDF::sample_from_phong(N, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
    if (wi.dir.dot_product(N) < 0) return L_light + L_brdf;
    intersec_result r2 = veach->closet_ray_intersect(p, wi.dir, triangle(point.s, point.f));
    if (r2.isIntersec) {
        BRDF brdf = BRDF::get_brdf_phong(N, wi.dir, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
        double light_pdf = 0;
        intersec_result rl = veach->closet_ray_intersect_light_triangle(p, wi.dir, triangle(point.s, point.f), lights->islight);
        if (rl.isIntersec) light_pdf = lights->eval_spherical_triangle_sampling_pdf(triangle(rl.s, rl.f), *veach);
        L_brdf = ref_shade_mis(r2, wi.dir * -1) * brdf * (wi.dir.dot_product(N) / (wi.pdf + light_pdf) / 0.6);
    }
    return L_light + L_brdf;
}

// Restatement of main.cpp:269-344 (shade, the integrator main() ships with, main.cpp:575); direct
// light through the reference's select_a_point_from_lights_spherical_triangle (Mylight.cpp:163),
// or -- area = true -- through its uniform-area sampler select_a_point_from_lights
// (Mylight.cpp:102-160), the alternative left commented out at main.cpp:296.
static RadianceRGB ref_shade(intersec_result point, vec wo, bool area = false) {
    vec p = interp(veach->get_vertexes_of_facet(point.s, point.f), point.beta, point.gamma);
    vec N = interp(veach->get_normals_of_facet(point.s, point.f), point.beta, point.gamma).normalized();
    if (N.dot_product(wo) < 0) return RadianceRGB(0, 0, 0);
    auto li = lights->islight.find(triangle(point.s, point.f));
    if (li != lights->islight.end()) return li->second;
    tinyobj::material_t mtl = mat_of(point.s, point.f);
    RadianceRGB L_dir;
    sampledLightPoint lp = area ? lights->select_a_point_from_lights(*veach)
                                : lights->select_a_point_from_lights_spherical_triangle(p, N, *veach);
    vec x1 = lp.coord;
    vec n1 = veach->get_unique_normal_of_facet(lp.s, lp.f);
    vec wl = (x1 - p).normalized();
    if (wl.dot_product(N) > 0 && (wl * -1).dot_product(n1) > 0) {
        intersec_result r1 = veach->closet_ray_intersect(p, wl, triangle(point.s, point.f));
        if (r1.isIntersec && r1.s == lp.s && r1.f == lp.f) {
            BRDF brdf = BRDF::get_brdf_phong(N, wl, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
            L_dir = lp.I * brdf * (wl.dot_product(N) * (wl * -1).dot_product(n1) / (x1 - p).dot_product(x1 - p) / lp.prob);
        }
    }
    RadianceRGB L_indir;
    if (rr_uniform() > 0.6) return L_dir + L_indir;
    sampledRay wi = BRDF::sample_from_phong(N, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
    if (wi.dir.dot_product(N) < 0) return L_dir + L_indir;
    intersec_result r2 = veach->closet_ray_intersect(p, wi.dir, triangle(point.s, point.f));
    if (r2.isIntersec && lights->islight.find(triangle(r2.s, r2.f)) == lights->islight.end()) {
        BRDF brdf = BRDF::get_brdf_phong(N, wi.dir, wo, kd_of(mtl), ks_of(mtl), mtl.shininess);
        L_indir = ref_shade(r2, wi.dir * -1, area) * brdf * (wi.dir.dot_product(N) / wi.pdf / 0.6);
    }
    return L_dir + L_indir;
}

// Camera of main.cpp:507-510,547-564 generalised to W x H.
struct Cam {
    vec eye;
    matrix3d T;
    double wlen, pixellen;
    int W, H;
};
static Cam make_cam(int W, int H) {
    vec start = vec(28.2792, 5.2, 1.23612e-06);
    vec w = (vec(0.0, 2.8, 0.0) - start);
    start = start - w;
    w = w * 2;
    Cam c;
    c.eye = start;
    c.wlen = w.norm2();
    c.pixellen = tan(20.1143 / 360) * w.norm2() / (H / 2.0);
    vec N = w.normalized();
    vec V = N.cross_product(vec(0, 1, 0)).normalized();
    vec U = V.cross_product(N).normalized();
    c.T = matrix3d(U, V, N);
    c.W = W;
    c.H = H;
    return c;
}
static vec cam_dir(const Cam& c, int i, int j) {
    vec delta(-c.pixellen * (i - (c.H - 1) / 2.0), c.pixellen * (j - (c.W - 1) / 2.0), 0);
    return (c.T * (delta + vec(0, 0, c.wlen))).normalized();
}

static void put_hit(std::vector<double>& o, const intersec_result& r) {
    o.push_back(r.isIntersec ? (double)gid(r.s, r.f) : -1.0);
    o.push_back(r.isIntersec ? r.t : 0.0);
    o.push_back(r.isIntersec ? r.beta : 0.0);
    o.push_back(r.isIntersec ? r.gamma : 0.0);
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s scene.obj lights.xml outdir\n", argv[0]);
        return 2;
    }
    const std::string out = argv[3];
    veach = new Myobj(argv[1]);
    lights = new Mylight(argv[2]);
    veach->read();
    lights->read();
    lights->gather_light_triangles(veach->reader);
    const auto& shapes = veach->reader.GetShapes();
    size_t F = 0;
    for (size_t s = 0; s < shapes.size(); s++) {
        shape_off.push_back(F);
        F += shapes[s].mesh.num_face_vertices.size();
    }
    Cam cam0 = make_cam(400, 300);
    veach->cal_scene_boundingbox(cam0.eye);
    veach->meshing(100000);

    // ---- G8 statistical reference: `... <outdir> stat <mode> <W> <H> <spp> <row0>
    // <row1> <clock0>` renders rows [row0, row1) of a W x H frame with spp fake-clock samples per
    // pixel and writes per-pixel sum L and sum L^2 (rows x W x 6) to <outdir>/stat_<mode>_<row0>.npy.
    // Run as several processes over disjoint rows (the reference's global state is not thread-safe).
    if (argc >= 12 && std::string(argv[4]) == "stat") {
        const int mode = atoi(argv[5]), W = atoi(argv[6]), H = atoi(argv[7]), spp = atoi(argv[8]);
        const int r0 = atoi(argv[9]), r1 = atoi(argv[10]);
        clk() = strtoull(argv[11], nullptr, 10);
        Cam c = make_cam(W, H);
        std::vector<double> o;
        for (int i = r0; i < r1; i++)
            for (int j = 0; j < W; j++) {
                vec dir = cam_dir(c, i, j);
                intersec_result rs = veach->closet_ray_intersect(c.eye, dir, triangle(-1, -1));
                double s1[3] = {0, 0, 0}, s2[3] = {0, 0, 0};
                for (int k = 0; k < spp && rs.isIntersec; k++) {
                    RadianceRGB L = mode == 0 ? ref_shade_mis(rs, dir * -1)
                                    : mode == 1 ? ref_shade_brdf(rs, dir * -1) : ref_shade(rs, dir * -1, mode == 3);
                    for (int q = 0; q < 3; q++) {
                        s1[q] += L.RGB[q];
                        s2[q] += L.RGB[q] * L.RGB[q];
                    }
                }
                for (int q = 0; q < 3; q++) o.push_back(s1[q]);
                for (int q = 0; q < 3; q++) o.push_back(s2[q]);
            }
        npy_f64(out + "/stat_" + std::to_string(mode) + "_" + std::to_string(r0) + ".npy", o, 6);
        return 0;
    }

    // ---- G0/G6 loader, unique normals, light table ------------------------------------
    {
        std::vector<float> fac;
        std::vector<long long> mat;
        std::vector<double> un;
        for (size_t s = 0; s < shapes.size(); s++)
            for (size_t f = 0; f < shapes[s].mesh.num_face_vertices.size(); f++) {
                auto v = veach->get_vertexes_of_facet(s, f);
                auto n = veach->get_normals_of_facet(s, f);
                for (int k = 0; k < 3; k++)
                    for (int c = 0; c < 3; c++) fac.push_back((float)v[k].xyz[c]);
                for (int k = 0; k < 3; k++)
                    for (int c = 0; c < 3; c++) fac.push_back((float)n[k].xyz[c]);
                mat.push_back(shapes[s].mesh.material_ids[f]);
                vec u = veach->get_unique_normal_of_facet(s, f);
                for (int c = 0; c < 3; c++) un.push_back(u.xyz[c]);
            }
        npy_f32(out + "/loader_facets.npy", fac, 18);
        npy_i64(out + "/loader_mat.npy", mat, 1);
        npy_f64(out + "/unique_normal.npy", un, 3);
        std::vector<float> mt;
        for (auto& m : veach->reader.GetMaterials()) {
            for (int c = 0; c < 3; c++) mt.push_back(m.diffuse[c]);
            for (int c = 0; c < 3; c++) mt.push_back(m.specular[c]);
            mt.push_back(m.shininess);
        }
        npy_f32(out + "/materials.npy", mt, 7);
        std::vector<long long> lid;
        std::vector<double> lar;
        for (auto& kv : lights->lightsTriangles)
            for (auto& t : kv.second) {
                lid.push_back(gid(t.s, t.f));
                RadianceRGB L = lights->lightsRadiance.at(kv.first);
                lar.push_back(t.area);
                lar.push_back(L.RGB[0]);
                lar.push_back(L.RGB[1]);
                lar.push_back(L.RGB[2]);
            }
        npy_i64(out + "/light_order.npy", lid, 1);
        npy_f64(out + "/light_area_radiance.npy", lar, 4);
        std::vector<double> bb;
        for (int i = 0; i < 3; i++) {
            bb.push_back(veach->xyzmm[i][0]);
            bb.push_back(veach->xyzmm[i][1]);
        }
        bb.push_back(veach->gridCellWidth);
        bb.push_back(0);
        npy_f64(out + "/grid_bbox.npy", bb, 8);
    }

    std::mt19937_64 rng(20240430);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    auto rand_dir = [&](void) {
        double z = 1 - 2 * U(rng), ph = 2 * 3.14159265358979323846 * U(rng), s = sqrt(fmax(0.0, 1 - z * z));
        return vec(s * cos(ph), s * sin(ph), z);
    };
    std::vector<std::pair<size_t, size_t>> nonlight;
    for (size_t s = 0; s < shapes.size(); s++)
        for (size_t f = 0; f < shapes[s].mesh.num_face_vertices.size(); f++)
            if (!lights->islight.count(triangle(s, f))) nonlight.push_back({s, f});
    std::vector<std::pair<size_t, size_t>> lighttris;
    for (auto& kv : lights->lightsTriangles)
        for (auto& t : kv.second) lighttris.push_back({t.s, t.f});
    auto rand_surface = [&](std::pair<size_t, size_t>& tri, double& b, double& g) {
        tri = nonlight[rng() % nonlight.size()];
        b = U(rng);
        g = U(rng);
        if (b + g > 1) { b = 1 - b; g = 1 - g; }
    };

    // ---- G1 primary-hit map, 400x300 ------------------------------------------------------
    {
        std::vector<double> o;
        for (int i = 0; i < cam0.H; i++)
            for (int j = 0; j < cam0.W; j++)
                put_hit(o, veach->closet_ray_intersect(cam0.eye, cam_dir(cam0, i, j), triangle(-1, -1)));
        npy_f64(out + "/primary_400x300.npy", o, 4);
    }

    // ---- G2 random rays: closest hit and light-only hit -------------------------------------
    {
        std::vector<double> in, hit, lhit;
        const int NR = 12000;
        for (int r = 0; r < NR; r++) {
            vec ro, rd;
            long long ex = -1;
            size_t es = (size_t)-1, ef = (size_t)-1;
            int kind = r % 3;
            if (kind == 0) {  // from the eye, jittered around the view
                ro = cam0.eye;
                rd = cam_dir(cam0, (int)(U(rng) * 300), (int)(U(rng) * 400));
                rd = (rd + rand_dir() * 0.01).normalized();
            } else {
                std::pair<size_t, size_t> tri;
                double b, g;
                rand_surface(tri, b, g);
                ro = interp(veach->get_vertexes_of_facet(tri.first, tri.second), b, g);
                es = tri.first; ef = tri.second; ex = gid(es, ef);
                if (kind == 1) {
                    rd = rand_dir();
                } else {  // toward a random point of a random light triangle
                    auto lt = lighttris[rng() % lighttris.size()];
                    double lb = U(rng), lg = U(rng);
                    if (lb + lg > 1) { lb = 1 - lb; lg = 1 - lg; }
                    rd = (interp(veach->get_vertexes_of_facet(lt.first, lt.second), lb, lg) - ro).normalized();
                }
            }
            for (int c = 0; c < 3; c++) in.push_back(ro.xyz[c]);
            for (int c = 0; c < 3; c++) in.push_back(rd.xyz[c]);
            in.push_back((double)ex);
            put_hit(hit, veach->closet_ray_intersect(ro, rd, triangle(es, ef)));
            put_hit(lhit, veach->closet_ray_intersect_light_triangle(ro, rd, triangle(es, ef), lights->islight));
        }
        npy_f64(out + "/rays_in.npy", in, 7);
        npy_f64(out + "/rays_hit.npy", hit, 4);
        npy_f64(out + "/rays_lighthit.npy", lhit, 4);
    }

    // ---- G3 light prep + spherical-triangle sampling at random shading points --------------
    {
        std::vector<double> in, o;
        const int NP = 2000;
        for (int r = 0; r < NP; r++) {
            std::pair<size_t, size_t> tri;
            double b, g;
            rand_surface(tri, b, g);
            vec p = interp(veach->get_vertexes_of_facet(tri.first, tri.second), b, g);
            vec N = interp(veach->get_normals_of_facet(tri.first, tri.second), b, g).normalized();
            u64 c0 = 1000003ull * (r + 1);
            clk() = c0;
            lights->prepared_for_lights_spherical_triangle_sampling(p, N, *veach);
            sampledLightPoint lp = lights->lights_spherical_triangle_sampling(p, N, *veach);
            u64 c1 = clk();
            for (int c = 0; c < 3; c++) in.push_back(p.xyz[c]);
            for (int c = 0; c < 3; c++) in.push_back(N.xyz[c]);
            in.push_back((double)c0);
            // survivors: count, sum of light-order positions, first 2 weights
            double possum = 0;
            size_t pos = 0;
            std::vector<double> firstw;
            for (auto& kv : lights->lightsTriangles)
                for (auto& t : kv.second) {
                    auto it = lights->indiceMap.find(triangle(t.s, t.f));
                    if (it != lights->indiceMap.end()) {
                        possum += (double)pos;
                        if (firstw.size() < 2) firstw.push_back(lights->weights[it->second]);
                    }
                    pos++;
                }
            while (firstw.size() < 2) firstw.push_back(-1);
            o.push_back(lights->weights_sum);
            o.push_back((double)lights->weights.size());
            o.push_back(possum);
            o.push_back(firstw[0]);
            o.push_back(firstw[1]);
            // sampled point (RefRng-dependent)
            bool empty = lights->weights.empty() || fabs(lights->weights_sum) < 1e-8;
            o.push_back(empty ? -1.0 : (double)gid(lp.s, lp.f));
            for (int c = 0; c < 3; c++) o.push_back(lp.coord.xyz[c]);
            o.push_back(lp.prob);
            o.push_back((double)(c1 - c0));
            // pdf of 2 fixed light triangles
            for (int q = 0; q < 2; q++) {
                auto lt = lighttris[(q * 1531 + r * 7) % lighttris.size()];
                o.push_back(lights->eval_spherical_triangle_sampling_pdf(triangle(lt.first, lt.second), *veach));
                o.push_back((double)gid(lt.first, lt.second));
            }
        }
        npy_f64(out + "/prep_in.npy", in, 7);
        npy_f64(out + "/prep_out.npy", o, 15);
    }

    // ---- G4 BRDF eval / pdf / sampling ----------------------------------------------------
    {
        std::vector<double> in, o;
        const auto& mats = veach->reader.GetMaterials();
        const int NB = 10000;
        for (int r = 0; r < NB; r++) {
            vec n = rand_dir(), wi = rand_dir(), wr = rand_dir();
            if (r % 4 != 0) {  // mostly upper-hemisphere configurations
                if (wi.dot_product(n) < 0) wi = wi * -1;
                if (wr.dot_product(n) < 0) wr = wr * -1;
            }
            if (r % 97 == 0) n = vec(1, 0, 0) * (r % 2 ? 1.0 : -1.0);
            size_t m = rng() % mats.size();
            vec kd(mats[m].diffuse[0], mats[m].diffuse[1], mats[m].diffuse[2]);
            vec ks(mats[m].specular[0], mats[m].specular[1], mats[m].specular[2]);
            if (kd.dot_product(vec(1, 1, 1)) + ks.dot_product(vec(1, 1, 1)) <= 0) continue;  // lights
            BRDF f = BRDF::get_brdf_phong(n, wi, wr, kd, ks, mats[m].shininess);
            double pdf = BRDF::eval_sample_from_phong_pdf(n, wi, wr, kd, ks, mats[m].shininess);
            u64 c0 = 7777777ull * (r + 1);
            clk() = c0;
            sampledRay sr = BRDF::sample_from_phong(n, wr, kd, ks, mats[m].shininess);
            for (int c = 0; c < 3; c++) in.push_back(n.xyz[c]);
            for (int c = 0; c < 3; c++) in.push_back(wi.xyz[c]);
            for (int c = 0; c < 3; c++) in.push_back(wr.xyz[c]);
            in.push_back((double)m);
            in.push_back((double)c0);
            for (int c = 0; c < 3; c++) o.push_back(f.RGB[c]);
            o.push_back(pdf);
            for (int c = 0; c < 3; c++) o.push_back(sr.dir.xyz[c]);
            o.push_back(sr.pdf);
        }
        npy_f64(out + "/brdf_in.npy", in, 11);
        npy_f64(out + "/brdf_out.npy", o, 8);
    }

    // ---- G5 tone mapping ------------------------------------------------------------------
    {
        std::vector<double> in;
        std::vector<long long> o;
        for (int r = 0; r < 4000; r++) {
            double L[3];
            for (int c = 0; c < 3; c++) L[c] = (r < 3000) ? pow(10.0, -6 + 9 * U(rng)) : 380.0 * U(rng);
            if (r == 0) { L[0] = 0; L[1] = 380; L[2] = 1e9; }
            RadianceRGB R(L[0], L[1], L[2]);
            auto t = R.tone_mapping(380, 0.25);
            for (int c = 0; c < 3; c++) { in.push_back(L[c]); o.push_back(t[c]); }
        }
        npy_f64(out + "/tonemap_in.npy", in, 3);
        npy_i64(out + "/tonemap_out.npy", o, 3);
    }

    // ---- G7 per-sample radiance, both integrators, RefRng replay keys -----------------------
    for (int mode = 0; mode < 4; mode++) {  // 0 shade_with_mis, 1 shade_with_brdf, 2 shade, 3 shade (area lights)
        std::vector<double> o;
        const int NS = mode == 1 ? 6000 : 3000;  // MIS / shade run a light prep per node
        for (int r = 0; r < NS; r++) {
            int i = (int)(U(rng) * cam0.H), j = (int)(U(rng) * cam0.W);
            vec dir = cam_dir(cam0, i, j);
            intersec_result rs = veach->closet_ray_intersect(cam0.eye, dir, triangle(-1, -1));
            u64 c0 = 1ull + 100000007ull * (u64)r;
            clk() = c0;
            RadianceRGB L(0, 0, 0);
            if (rs.isIntersec)
                L = mode == 0 ? ref_shade_mis(rs, dir * -1) : mode == 1 ? ref_shade_brdf(rs, dir * -1)
                                                                  : ref_shade(rs, dir * -1, mode == 3);
            o.push_back(i);
            o.push_back(j);
            o.push_back((double)c0);
            o.push_back((double)(clk() - c0));
            for (int c = 0; c < 3; c++) o.push_back(L.RGB[c]);
        }
        npy_f64(out + (mode == 0 ? "/sample_mis.npy" : mode == 1 ? "/sample_brdf.npy"
                                           : mode == 2 ? "/sample_shade.npy" : "/sample_shade_area.npy"), o, 7);
    }
    printf("golden vectors written to %s (F=%zu)\n", out.c_str(), F);
    return 0;
}
