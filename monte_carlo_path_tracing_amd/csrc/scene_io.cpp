// Scene loaders -- the Myobj / Mylight equivalents of the drop-in boundary.
//
//  * OBJ/MTL: the subset of the vendored tinyobjloader the reference relies on
//    (Myobj.cpp:10-28; ObjReader with triangulation on, real_t = float): `v`, `vn`, `f`,
//    `usemtl`, `mtllib`, and in the MTL `newmtl`, `Kd`, `Ks`, `Ns`.  Numbers go through the same
//    decimal-to-double algorithm as tinyobjloader's tryParseDouble (tiny_obj_loader.h:897-1028)
//    so the float vertices are bit-identical to what the reference loads.  Quads are split on the
//    shorter diagonal as tinyobj does (tiny_obj_loader.h:1509-1605); larger polygons are
//    fan-triangulated (tinyobj would ear-clip -- documented deviation).
//  * XML: top-level `<light mtlname="..." radiance="r,g,b"/>` elements (Mylight.cpp:21-28,
//    radiance parsed like RadianceRGB(std::string): getline(',') + stod, RadianceRGB.cpp:17-27)
//    and the `<camera>` block (README.md:339-343).
#include <cctype>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

#include "mcpt_internal.h"

namespace mcpt {

namespace {

bool read_text(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// tinyobjloader's decimal parser: integer digits accumulated in a double, fraction digits
// added as digit * 10^-k (table for k < 8), exponent applied as ldexp(m * 5^e, e).
// A restructured restatement of tinyobjloader's tryParseDouble (tiny_obj_loader.h:897-1028, as
// vendored by the reference), kept so that vertices parse to the reference's exact floats.
// tinyobjloader: The MIT License (MIT), Copyright (c) 2012-Present, Syoyo Fujita and many
// contributors.  Permission is hereby granted, free of charge, to any person obtaining a copy of
// that software and associated documentation files, to deal in the Software without restriction,
// subject to including the copyright notice and permission notice in all copies or substantial
// portions of the Software; it is provided "AS IS", without warranty of any kind.
bool parse_decimal(const char* s, const char* e, double* result) {
    static const double kFrac[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
    if (s >= e) return false;
    double m = 0.0;
    int ex = 0, nread = 0;
    bool neg = false, neg_exp = false, lead_dot = false;
    const char* c = s;
    if (*c == '+' || *c == '-') {
        neg = (*c == '-');
        ++c;
        lead_dot = (c != e && *c == '.');
    } else if (*c == '.') {
        lead_dot = true;
    } else if (!std::isdigit(static_cast<unsigned char>(*c))) {
        return false;
    }
    if (!lead_dot) {
        for (; c != e && std::isdigit(static_cast<unsigned char>(*c)); ++c, ++nread) {
            m *= 10;
            m += static_cast<int>(*c - '0');
        }
        if (nread == 0) return false;
    }
    if (c != e && *c == '.') {
        ++c;
        for (int k = 1; c != e && std::isdigit(static_cast<unsigned char>(*c)); ++c, ++k)
            m += static_cast<int>(*c - '0') * (k < 8 ? kFrac[k] : std::pow(10.0, -k));
    } else if (c != e && *c != 'e' && *c != 'E') {
        c = e;  // anything else ends the number
    }
    if (c != e && (*c == 'e' || *c == 'E')) {
        ++c;
        if (c != e && (*c == '+' || *c == '-')) {
            neg_exp = (*c == '-');
            ++c;
        } else if (c == e || !std::isdigit(static_cast<unsigned char>(*c))) {
            return false;
        }
        int nexp = 0;
        for (; c != e && std::isdigit(static_cast<unsigned char>(*c)); ++c, ++nexp) {
            if (ex > 2147483647 / 10) return false;
            ex = ex * 10 + static_cast<int>(*c - '0');
        }
        if (nexp == 0) return false;
        if (neg_exp) ex = -ex;
    }
    *result = (neg ? -1 : 1) * (ex ? std::ldexp(m * std::pow(5.0, ex), ex) : m);
    return true;
}

// parseReal: skip blanks, token up to blank/CR, default on failure, narrowed to float.
float next_real(const char*& p, double dflt = 0.0) {
    p += std::strspn(p, " \t");
    const char* end = p + std::strcspn(p, " \t\r\n");
    double v = dflt;
    parse_decimal(p, end, &v);
    p = end;
    return static_cast<float>(v);
}

bool starts_kw(const char* t, const char* kw) {
    size_t n = std::strlen(kw);
    return std::strncmp(t, kw, n) == 0 && (t[n] == ' ' || t[n] == '\t');
}

std::string word(const char* p) {
    p += std::strspn(p, " \t");
    return std::string(p, std::strcspn(p, " \t\r\n"));
}

void load_mtl_file(const std::string& path, HostScene& s, std::map<std::string, int>& index) {
    std::string text;
    if (!read_text(path, text)) return;
    std::istringstream in(text);
    std::string line;
    bool open = false;
    std::string name;
    float kd[3] = {0, 0, 0}, ks[3] = {0, 0, 0}, ns = 1.0f;  // InitMaterial defaults
    auto flush = [&]() {
        if (!open || name.empty()) return;
        index[name] = s.M++;
        s.mtl_names.push_back(name);
        s.mtl.insert(s.mtl.end(), {kd[0], kd[1], kd[2], ks[0], ks[1], ks[2], ns});
    };
    while (std::getline(in, line)) {
        const char* t = line.c_str() + std::strspn(line.c_str(), " \t");
        if (starts_kw(t, "newmtl")) {
            flush();
            std::string rest(t + 7);
            size_t a = rest.find_first_not_of(" \t");
            size_t b = rest.find_last_not_of(" \t\r\n");
            name = (a == std::string::npos) ? "" : rest.substr(a, b - a + 1);
            kd[0] = kd[1] = kd[2] = ks[0] = ks[1] = ks[2] = 0.0f;
            ns = 1.0f;
            open = true;
        } else if (starts_kw(t, "Kd")) {
            const char* p = t + 2;
            for (float& c : kd) c = next_real(p);
        } else if (starts_kw(t, "Ks")) {
            const char* p = t + 2;
            for (float& c : ks) c = next_real(p);
        } else if (starts_kw(t, "Ns")) {
            const char* p = t + 2;
            ns = next_real(p);
        }
    }
    flush();
}

long resolve_index(long idx, size_t n) { return idx > 0 ? idx - 1 : (idx < 0 ? static_cast<long>(n) + idx : -1); }

}  // namespace

bool load_obj_mtl(const std::string& obj_path, HostScene& s, std::string& err) {
    std::string text;
    if (!read_text(obj_path, text)) {
        err = "cannot open " + obj_path;
        return false;
    }
    std::string dir;
    size_t slash = obj_path.find_last_of('/');
    if (slash != std::string::npos) dir = obj_path.substr(0, slash + 1);
    std::vector<float> V, N;
    std::map<std::string, int> mindex;
    int cur_mat = -1;
    size_t pos = 0;
    while (pos < text.size()) {
        size_t eol = text.find('\n', pos);
        if (eol == std::string::npos) eol = text.size();
        std::string line = text.substr(pos, eol - pos);
        pos = eol + 1;
        const char* t = line.c_str() + std::strspn(line.c_str(), " \t");
        if (t[0] == 'v' && (t[1] == ' ' || t[1] == '\t')) {
            const char* p = t + 2;
            for (int c = 0; c < 3; c++) V.push_back(next_real(p));
        } else if (t[0] == 'v' && t[1] == 'n' && (t[2] == ' ' || t[2] == '\t')) {
            const char* p = t + 3;
            for (int c = 0; c < 3; c++) N.push_back(next_real(p));
        } else if (t[0] == 'f' && (t[1] == ' ' || t[1] == '\t')) {
            std::vector<long> vi, ni;
            const char* p = t + 2;
            while (true) {
                p += std::strspn(p, " \t");
                if (!*p || *p == '\r') break;
                char* endp;
                long a = std::strtol(p, &endp, 10), c = 0;
                p = endp;
                if (*p == '/') {
                    ++p;
                    if (*p != '/') {
                        std::strtol(p, &endp, 10);
                        p = endp;
                    }
                    if (*p == '/') {
                        ++p;
                        c = std::strtol(p, &endp, 10);
                        p = endp;
                    }
                }
                p += std::strcspn(p, " \t\r");
                long va = resolve_index(a, V.size() / 3), na = c ? resolve_index(c, N.size() / 3) : -1;
                if (va < 0 || na < 0) {
                    err = obj_path + ": face without a vertex normal (the reference reads normal_index >= 0)";
                    return false;
                }
                // an index past the vertices / normals read so far (found by the sanitizer build:
                // it was read out of bounds)
                if ((size_t)va >= V.size() / 3 || (size_t)na >= N.size() / 3) {
                    err = obj_path + ": face index out of range";
                    return false;
                }
                vi.push_back(va);
                ni.push_back(na);
            }
            const size_t nv = vi.size();
            if (nv < 3) continue;  // tinyobj skips degenerate faces
            std::vector<int> tri;
            if (nv == 3) {
                tri = {0, 1, 2};
            } else if (nv == 4) {  // shorter diagonal, float arithmetic as tinyobj
                auto P = [&](long v, int c) { return V[3 * v + c]; };
                float e02[3], e13[3];
                for (int c = 0; c < 3; c++) {
                    e02[c] = P(vi[2], c) - P(vi[0], c);
                    e13[c] = P(vi[3], c) - P(vi[1], c);
                }
                float s02 = e02[0] * e02[0] + e02[1] * e02[1] + e02[2] * e02[2];
                float s13 = e13[0] * e13[0] + e13[1] * e13[1] + e13[2] * e13[2];
                tri = s02 < s13 ? std::vector<int>{0, 1, 2, 0, 2, 3} : std::vector<int>{0, 1, 3, 1, 2, 3};
            } else {
                for (size_t k = 1; k + 1 < nv; k++) tri.insert(tri.end(), {0, static_cast<int>(k), static_cast<int>(k + 1)});
            }
            for (size_t q = 0; q < tri.size(); q += 3) {
                for (int k = 0; k < 3; k++)
                    for (int c = 0; c < 3; c++) s.pos.push_back(V[3 * vi[tri[q + k]] + c]);
                for (int k = 0; k < 3; k++)
                    for (int c = 0; c < 3; c++) s.nrm.push_back(N[3 * ni[tri[q + k]] + c]);
                s.mat.push_back(cur_mat);
            }
        } else if (starts_kw(t, "usemtl")) {
            auto it = mindex.find(word(t + 7));
            cur_mat = it == mindex.end() ? -1 : it->second;
        } else if (starts_kw(t, "mtllib")) {
            load_mtl_file(dir + word(t + 7), s, mindex);
        }
    }
    s.F = static_cast<int>(s.mat.size());
    return true;
}

namespace {
bool xml_attr(const std::string& tag, const char* name, std::string& out) {
    const size_t n = std::strlen(name);
    for (size_t p = tag.find(name); p != std::string::npos; p = tag.find(name, p + 1)) {
        if (p > 0 && !std::isspace(static_cast<unsigned char>(tag[p - 1]))) continue;
        size_t q = tag.find_first_not_of(" \t\r\n", p + n);
        if (q == std::string::npos || tag[q] != '=') continue;
        q = tag.find_first_not_of(" \t\r\n", q + 1);
        if (q == std::string::npos || (tag[q] != '"' && tag[q] != '\'')) continue;
        size_t e = tag.find(tag[q], q + 1);
        if (e == std::string::npos) return false;
        out = tag.substr(q + 1, e - q - 1);
        return true;
    }
    return false;
}
}  // namespace

bool load_light_xml(const std::string& xml_path, HostScene& s, std::vector<LightDef>& lights, std::string& err) {
    std::string text;
    if (!read_text(xml_path, text)) {
        err = "cannot open " + xml_path;
        return false;
    }
    std::map<std::string, LightDef> by_name;  // Mylight::lightsRadiance (later entries win)
    int depth = 0;
    bool in_cam = false;
    for (size_t p = text.find('<'); p != std::string::npos; p = text.find('<', p)) {
        if (text.compare(p, 4, "<!--") == 0) {
            size_t e = text.find("-->", p);
            if (e == std::string::npos) break;
            p = e + 3;
            continue;
        }
        size_t e = text.find('>', p);
        if (e == std::string::npos) break;
        if (text[p + 1] == '?' || text[p + 1] == '!') {
            p = e + 1;
            continue;
        }
        if (text[p + 1] == '/') {
            if (--depth == 0) in_cam = false;
            p = e + 1;
            continue;
        }
        const std::string tag = text.substr(p + 1, e - p - 1);
        const bool self_close = !tag.empty() && tag.back() == '/';
        const std::string name = tag.substr(0, tag.find_first_of(" \t\r\n/"));
        if (depth == 0 && name == "light") {
            std::string mtl, rad;
            xml_attr(tag, "mtlname", mtl);
            if (!xml_attr(tag, "radiance", rad)) {
                err = "light without radiance in " + xml_path;
                return false;
            }
            LightDef d;
            d.name = mtl;
            std::stringstream ss(rad);
            std::string item;
            for (double& c : d.rgb) {
                std::getline(ss, item, ',');
                char* endp = nullptr;
                c = std::strtod(item.c_str(), &endp);
                if (endp == item.c_str()) {
                    err = "bad radiance '" + rad + "'";
                    return false;
                }
            }
            by_name[mtl] = d;
        } else if (depth == 0 && name == "camera") {
            std::string a;
            s.has_cam = true;
            s.cam = mcpt_camera{};
            s.cam.dist_scale = 1.0;
            s.cam.up[1] = 1.0;
            if (xml_attr(tag, "width", a)) s.cam.width = std::atoi(a.c_str());
            if (xml_attr(tag, "height", a)) s.cam.height = std::atoi(a.c_str());
            if (xml_attr(tag, "fovy", a)) s.cam.fovy = std::strtod(a.c_str(), nullptr);
            in_cam = !self_close;
        } else if (depth == 1 && in_cam && (name == "eye" || name == "lookat" || name == "up")) {
            double* dst = name == "eye" ? s.cam.eye : (name == "lookat" ? s.cam.lookat : s.cam.up);
            std::string a;
            if (xml_attr(tag, "x", a)) dst[0] = std::strtod(a.c_str(), nullptr);
            if (xml_attr(tag, "y", a)) dst[1] = std::strtod(a.c_str(), nullptr);
            if (xml_attr(tag, "z", a)) dst[2] = std::strtod(a.c_str(), nullptr);
        }
        if (!self_close) ++depth;
        p = e + 1;
    }
    lights.clear();
    for (auto& kv : by_name) lights.push_back(kv.second);  // std::map: name order
    return true;
}

// lightTriangle::area (Mylight.cpp:66-69): n = (b-a) x (c-a), n = n * (1 / |n|), area = 0.5 *
// det(b-a, c-a, n) with det(a, b, c) = (a x b) . c (vec.cpp:84-87), in the reference's fp64 order
double light_triangle_area(const HostScene& s, int f) {
    double v[3][3], ba[3], ca[3], n[3], t[3];
    for (int k = 0; k < 3; k++)
        for (int c = 0; c < 3; c++) v[k][c] = s.pos[9 * f + 3 * k + c];
    for (int c = 0; c < 3; c++) {
        ba[c] = v[1][c] - v[0][c];
        ca[c] = v[2][c] - v[0][c];
    }
    auto cross = [](const double* a, const double* b, double* o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    cross(ba, ca, n);
    const double inv = 1.0 / std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (int c = 0; c < 3; c++) n[c] = n[c] * inv;
    cross(ba, ca, t);
    double d = 0;
    d += t[0] * n[0];
    d += t[1] * n[1];
    d += t[2] * n[2];
    return 0.5 * d;
}

bool finalize_scene(HostScene& s, std::vector<LightDef> lights, std::string& err) {
    for (int f = 0; f < s.F; f++)
        if (s.mat[f] < 0 || s.mat[f] >= s.M) {
            err = "facet " + std::to_string(f) + " has no material (the reference throws, main.cpp:425)";
            return false;
        }
    auto sub = [](const double* a, const double* b, double* o) {
        for (int c = 0; c < 3; c++) o[c] = a[c] - b[c];
    };
    auto cross = [](const double* a, const double* b, double* o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    auto dot = [](const double* a, const double* b) {
        double r = 0;
        r += a[0] * b[0];
        r += a[1] * b[1];
        r += a[2] * b[2];
        return r;
    };
    auto norm = [](const double* a) { return std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); };
    auto vert = [&](int f, int k, double* o) {
        for (int c = 0; c < 3; c++) o[c] = s.pos[9 * f + 3 * k + c];
    };
    // gather_light_triangles (Mylight.cpp:32-100): table in light-name order, facets in order
    std::vector<int> lmat(s.F, -1);
    for (int f = 0; f < s.F; f++)
        for (size_t k = 0; k < lights.size(); k++)
            if (s.mtl_names[s.mat[f]] == lights[k].name) {
                lmat[f] = static_cast<int>(k);
                break;
            }
    s.light_of.assign(s.F, -1);
    s.light_facet.clear();
    s.light_rad.clear();
    s.light_sum.clear();
    s.light_area.clear();
    s.group_rsum.clear();
    s.group_start.clear();
    s.group_count.clear();
    for (size_t k = 0; k < lights.size(); k++) {
        s.group_rsum.push_back(lights[k].rgb[0] + lights[k].rgb[1] + lights[k].rgb[2]);  // RadianceRGB::sum
        s.group_start.push_back(static_cast<int32_t>(s.light_facet.size()));
        for (int f = 0; f < s.F; f++) {
            if (lmat[f] != static_cast<int>(k)) continue;
            s.light_of[f] = static_cast<int>(s.light_facet.size());
            s.light_facet.push_back(f);
            s.light_rad.insert(s.light_rad.end(), lights[k].rgb, lights[k].rgb + 3);
            s.light_sum.push_back(lights[k].rgb[0] + lights[k].rgb[1] + lights[k].rgb[2]);
            s.light_area.push_back(light_triangle_area(s, f));
        }
        s.group_count.push_back(static_cast<int32_t>(s.light_facet.size()) - s.group_start.back());
    }
    s.NL = static_cast<int>(s.light_facet.size());
    // unique normals (Myobj.cpp:680-709): geometric normal flipped toward the vertex normals
    s.unique_n.resize(3 * static_cast<size_t>(s.F));
    for (int f = 0; f < s.F; f++) {
        double a[3], b[3], c[3], ba[3], ca[3], n[3], nv[3][3];
        vert(f, 0, a);
        vert(f, 1, b);
        vert(f, 2, c);
        for (int k = 0; k < 3; k++) {
            double t[3] = {s.nrm[9 * f + 3 * k], s.nrm[9 * f + 3 * k + 1], s.nrm[9 * f + 3 * k + 2]};
            double l = norm(t);
            for (int q = 0; q < 3; q++) nv[k][q] = t[q] / l;
        }
        sub(b, a, ba);
        sub(c, a, ca);
        cross(ba, ca, n);
        double l = norm(n);
        for (double& q : n) q = q / l;
        double nr[3] = {n[0] * -1, n[1] * -1, n[2] * -1};
        double w = dot(n, nv[0]) + dot(n, nv[1]) + dot(n, nv[2]);
        double wr = dot(nr, nv[0]) + dot(nr, nv[1]) + dot(nr, nv[2]);
        const double* u = w > wr ? n : nr;
        for (int q = 0; q < 3; q++) s.unique_n[3 * f + q] = u[q];
    }
    (void)err;
    return true;
}

static thread_local char g_error[512];
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_error, sizeof g_error, fmt, ap);
    va_end(ap);
}

}  // namespace mcpt

extern "C" const char* mcpt_last_error(void) { return mcpt::g_error; }
