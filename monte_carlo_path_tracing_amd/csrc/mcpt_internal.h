// Host-side scene representation shared by the loaders, the BVH builder and the HIP renderer.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "mcpt.h"

namespace mcpt {

// Flattened scene: facets in the reference's (shape, face) order, the light table in
// Mylight::lightsTriangles order (Mylight.cpp:88: material name, then facet).
struct HostScene {
    int F = 0, M = 0, NL = 0;
    std::vector<float> pos;         // F*9  v0 v1 v2
    std::vector<float> nrm;         // F*9  vertex normals
    std::vector<int32_t> mat;       // F
    std::vector<float> mtl;         // M*7  Kd Ks Ns
    std::vector<std::string> mtl_names;
    std::vector<int32_t> light_facet;   // NL
    std::vector<double> light_rad;      // NL*3
    std::vector<double> light_sum;      // NL  RadianceRGB::sum()
    std::vector<int32_t> light_of;      // F -> light index or -1
    std::vector<double> unique_n;       // F*3  Myobj::get_unique_normal_of_facet
    std::vector<double> light_area;     // NL   lightTriangle::area (Mylight.cpp:66-69)
    // Mylight::lightsRadiance in map order (every XML light, also one without triangles):
    // RadianceRGB::sum() and the run [start, start + count) of its triangles in the light table
    std::vector<double> group_rsum;
    std::vector<int32_t> group_start, group_count;
    bool has_cam = false;
    mcpt_camera cam{};
};

// scene_io.cpp
bool load_obj_mtl(const std::string& obj_path, HostScene& s, std::string& err);
struct LightDef {
    std::string name;
    double rgb[3];
};
bool load_light_xml(const std::string& xml_path, HostScene& s, std::vector<LightDef>& lights, std::string& err);
// gather_light_triangles + unique normals (Mylight.cpp:32-100, Myobj.cpp:680-709)
bool finalize_scene(HostScene& s, std::vector<LightDef> lights, std::string& err);
double light_triangle_area(const HostScene& s, int f);  // Mylight.cpp:66-69

// bvh.cpp -- binary BVH over a facet subset, flattened for the GPU.
struct BvhNode {       // 64 B: both children's boxes in one node (one fetch per visit)
    float lo[2][3];    // child 0/1 AABB min
    float hi[2][3];    // child 0/1 AABB max
    int32_t child[2];  // >= 0: inner node index; < 0: leaf, ~child = first leaf slot
    int32_t count[2];  // leaf triangle count (0 for inner children)
};
struct Bvh {
    std::vector<BvhNode> nodes;
    std::vector<int32_t> leaf_facets;  // facet ids in leaf order
};
Bvh build_bvh(const HostScene& s, const std::vector<int32_t>& facets, int max_leaf);

// 4-wide node (128 B, two cache lines): the four children's boxes as per-axis float4s, so a
// node visit is 8 dwordx4 loads and four independent slab tests.  Children as in BvhNode;
// unused slots hold kBvh4Empty.
constexpr int32_t kBvh4Empty = 0x7fffffff;
struct BvhNode4 {
    float lo[3][4];    // lo[axis][child]
    float hi[3][4];
    int32_t child[4];  // >= 0: inner node; < 0: leaf ~first slot; kBvh4Empty: no child
    int32_t count[4];
};
// compressed 4-wide node (64 B, half a cache line): per axis the children's union minimum `org` and
// a power-of-two scale 2^(ex_a - 127); each child plane is a byte q with plane = fma(q, scale, org)
// in fp32, rounded outward at build time against that exact fp32 expression, so every decoded box
// contains its BvhNode4 box (conservative: the traversal only prunes with it).  Loaded as four
// dwordx4: (org, ex), (q lo.x, hi.x, lo.y, hi.y), (q lo.z, hi.z, -, -), children.
struct BvhNode4Q {
    float org[3];
    uint32_t ex;       // byte a: biased fp32 exponent of axis a's scale
    uint32_t q[6];     // q[2a] lo planes, q[2a + 1] hi planes of axis a; byte k = child k
    uint32_t pad[2];
    int32_t child[4];  // as BvhNode4 (leaf codes already packed)
};
static_assert(sizeof(BvhNode4Q) == 64, "BvhNode4Q must be 64 B");
std::vector<BvhNode4Q> quantize_bvh4(const std::vector<BvhNode4>& in);

// collapses a binary BVH into a 4-wide one (greedy: expand the largest-area inner child until
// four children); leaves and leaf slots are shared with the binary tree
std::vector<BvhNode4> collapse_bvh4(const Bvh& b);

// 8-wide compressed node (128 B, one cache line) for the wide traversal (k_rays_cw8), after Ylitie, Karras &
// Laine's compressed wide BVH (HPG 2017), adapted: the same conservative byte planes as BvhNode4Q for eight
// children, children ordered by OCTANT -- slot s holds the child whose centre lies on the negative side of
// the node centre along axis a iff bit a of s is set (greedy assignment) -- so that a ray visits hit
// children in (slot XOR its octant code) order, near to far, with no sort; inner child s at node base + s
// (eight node slots reserved per node with inner children: a stack entry is (base << 8 | hit bits), no
// child code needs loading) and each leaf child's <= 2 triangles at fixed triangle slots (a triangle
// group is a base and a 16-bit mask).  Binary leaves with more than two triangles are split (by index
// halves) before the collapse.
struct BvhNode8Q {
    float org[3];
    uint32_t ex;           // bytes 0-2: biased fp32 exponent of axis a's scale; byte 3: imask (slots of inner children)
    uint32_t qlo[3][2];    // qlo[a][h]: byte k = lo plane of child 4 h + k on axis a (plane = fma(q, 2^(e - 127), org))
    uint32_t qhi[3][2];
    int32_t base_inner;    // inner child of slot s: node base_inner + s
    int32_t base_tri;      // triangle j (0, 1) of leaf child s: triangle slot base_tri + 2 s + j
    uint32_t tvalid;       // bit 2 s + j: that triangle slot holds a triangle
    uint32_t pad[13];
};
static_assert(sizeof(BvhNode8Q) == 128, "BvhNode8Q must be 128 B");
struct Bvh8 {
    std::vector<BvhNode8Q> nodes;      // node 0 = root
    std::vector<int32_t> tri_facets;   // facet of each triangle slot (-1: unused)
    int depth = 0;                     // levels of nodes (the 8-wide traversal stack holds at most one entry per level)
};
// the 8-wide tree of a binary BVH built by build_bvh over the same facets (boxes conservative: every decoded
// child box contains the fp32 box the binary tree holds for it, or its triangles' for a split leaf)
Bvh8 build_bvh8(const HostScene& s, const Bvh& b);

// grid.cpp -- the reference's uniform grid (Myobj.cpp:78-162) for the MCPT_ACCEL_GRID mode
struct Grid {
    bool ok = false;
    double eye[3] = {0, 0, 0};  // camera point the bounding box was built with
    int n0 = 0;
    double mn[3], mx[3];        // bounding box of every vertex and the eye
    double d = 0, inv_d = 0;    // cell edge and its reciprocal
    int lim[3], gd[3];          // last cell index per axis; cells per axis (lim + 1)
    std::vector<int32_t> cell_start;  // CSR over cells (x-major, then y, then z)
    std::vector<int32_t> cell_tri;    // facets per cell, ascending facet id
};
Grid build_grid(const HostScene& s, const double eye[3], int n0);

void set_error(const char* fmt, ...);

}  // namespace mcpt
