"""CPU-side checks of the native library (no GPU needed): it loads, exports every symbol that
include/mcpt.h declares, and its host code (OBJ/MTL/XML loaders, unique normals, tone map, BMP
writer) matches the compiled reference's golden vectors bit for bit."""
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, SCENE_OBJ, SCENE_XML
import monte_carlo_path_tracing_amd as mcpt
from oracle import pyoracle as po


def test_library_exports_every_declared_symbol():
    hdr = (ROOT / "include" / "mcpt.h").read_text()
    declared = set(re.findall(r"\b(mcpt_[a-z_0-9]+)\s*\(", hdr))
    assert declared == set(mcpt.EXPORTS), declared ^ set(mcpt.EXPORTS)
    L = mcpt.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert L.mcpt_version() == mcpt.MCPT_VERSION
    assert int(re.search(r"#define MCPT_VERSION (\d+)", hdr).group(1)) == mcpt.MCPT_VERSION
    dbg = (ROOT / "include" / "mcpt_debug.h").read_text()
    assert set(re.findall(r"\b(mcpt_[a-z_0-9]+)\s*\(", dbg)) == set(mcpt.DEBUG_EXPORTS)
    for name in mcpt.DEBUG_EXPORTS:
        assert hasattr(L, name), name


def test_abi_struct_layouts_match_header(tmp_path):
    """sizeof/offsetof of mcpt_render_opts, mcpt_stats and mcpt_camera from a C program compiled
    against include/mcpt.h equal the ctypes mirror's; mcpt_render_opts_init sets struct_size."""
    import ctypes as C
    import subprocess
    structs = {"mcpt_render_opts": mcpt.RenderOpts, "mcpt_stats": mcpt.Stats, "mcpt_camera": mcpt.Camera}
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "mcpt.h"', "int main(void) {"]
    for cname, py in structs.items():
        src.append('printf("%s sizeof %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            src.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    src.append("return 0; }")
    (tmp_path / "layout.c").write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", str(ROOT / "include"), str(tmp_path / "layout.c"), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        c, f, v = line.split()
        got[(c, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)
    o = mcpt.RenderOpts()
    mcpt.lib().mcpt_render_opts_init(C.byref(o))
    assert o.struct_size == C.sizeof(mcpt.RenderOpts) and o.device == -1 and o.spp == 10
    assert o.stats_size == C.sizeof(mcpt.Stats)


def test_render_rejects_a_foreign_struct_size():
    """ABI guard (include/mcpt.h struct_size): a caller built against another header is refused
    before any other field is read -- no GPU involved."""
    import ctypes as C
    s = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    cam = mcpt.Camera.reference(8, 6)
    o = mcpt.RenderOpts()
    mcpt.lib().mcpt_render_opts_init(C.byref(o))
    o.struct_size -= 8
    out = np.zeros((6, 8, 3))
    rc = mcpt.lib().mcpt_render(s.h, C.byref(cam), C.byref(o), out.reshape(-1), None)
    assert rc == -1 and b"struct_size" in mcpt.lib().mcpt_last_error()


@pytest.fixture(scope="module")
def scene():
    return mcpt.Scene.load(SCENE_OBJ, SCENE_XML)


def test_loader_matches_reference_bitexact(scene):
    a = scene.arrays()
    gf = np.load(GOLDEN / "loader_facets.npy")
    assert np.array_equal(a["positions"].view(np.uint32), gf[:, :9].view(np.uint32))
    assert np.array_equal(a["normals"].view(np.uint32), gf[:, 9:].view(np.uint32))
    assert np.array_equal(a["material_id"], np.load(GOLDEN / "loader_mat.npy")[:, 0])
    assert np.array_equal(a["materials"], np.load(GOLDEN / "materials.npy"))
    assert np.array_equal(a["light_facet"], np.load(GOLDEN / "light_order.npy")[:, 0])
    assert np.array_equal(a["light_radiance"], np.load(GOLDEN / "light_area_radiance.npy")[:, 1:])
    assert np.array_equal(a["unique_normal"], np.load(GOLDEN / "unique_normal.npy"))


def test_scene_xml_camera(scene):
    c = scene.camera()
    assert tuple(c.eye) == (28.2792, 5.2, 1.23612e-06) and tuple(c.lookat) == (0.0, 2.8, 0.0)
    assert c.fovy == 20.1143 and (c.width, c.height) == (1280, 720)


def test_load_errors_are_reported(tmp_path):
    with pytest.raises(mcpt.MCPTError, match="cannot open"):
        mcpt.Scene.load(str(tmp_path / "nope.obj"), SCENE_XML)
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    with pytest.raises(mcpt.MCPTError, match="normal"):
        mcpt.Scene.load(str(bad), SCENE_XML)
    nomat = tmp_path / "nomat.obj"
    nomat.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf 1//1 2//1 3//1\n")
    with pytest.raises(mcpt.MCPTError, match="material"):
        mcpt.Scene.load(str(nomat), SCENE_XML)


def test_quad_split_and_negative_indices(tmp_path):
    """tinyobj splits quads on the shorter diagonal (tiny_obj_loader.h:1561-1605)."""
    (tmp_path / "q.mtl").write_text("newmtl m\nKd 0.5 0.5 0.5\n")
    (tmp_path / "q.obj").write_text("mtllib q.mtl\nv 0 0 0\nv 2 0 0\nv 2 1 0\nv 0 1 0\nvn 0 0 1\n"
                                    "usemtl m\nf -4//1 -3//1 -2//1 -1//1\n")
    (tmp_path / "q.xml").write_text('<light mtlname="x" radiance="1,1,1"/>\n')
    s = mcpt.Scene.load(str(tmp_path / "q.obj"), str(tmp_path / "q.xml"))
    assert s.nfacets == 2 and s.nlights == 0
    p = s.arrays()["positions"].reshape(2, 3, 3)
    # |e02| = |e13| -> not "<" -> [0,1,3],[1,2,3]
    assert np.array_equal(p[0], [[0, 0, 0], [2, 0, 0], [0, 1, 0]])
    assert np.array_equal(p[1], [[2, 0, 0], [2, 1, 0], [0, 1, 0]])


def test_tone_map_matches_reference():
    tin = np.load(GOLDEN / "tonemap_in.npy")
    tout = np.load(GOLDEN / "tonemap_out.npy")
    got = mcpt.tone_map(tin.reshape(1, -1, 3))
    assert np.array_equal(got.reshape(-1, 3), tout.astype(np.uint8))


# first 54 bytes of the reference's test.bmp (EasyX saveimage, 1280x720): fixture value
REF_BMP_HEADER = bytes.fromhex("424d3640380000000000360000002800000000050000d0020000010020000000"
                               "000000000000c40e0000c40e00000000000000000000")


def test_bmp_layout_matches_reference_header(tmp_path):
    img = np.zeros((720, 1280, 3), np.uint8)
    img[0, 0] = (1, 2, 3)       # top-left pixel
    img[719, 0] = (4, 5, 6)     # bottom-left pixel
    p = tmp_path / "t.bmp"
    mcpt.write_bmp(str(p), img)
    d = p.read_bytes()
    assert d[:54] == REF_BMP_HEADER and len(d) == 3686454
    assert d[54:58] == bytes([6, 5, 4, 0])  # bottom-up rows, B G R 0
    top = 54 + 4 * 1280 * 719
    assert d[top:top + 4] == bytes([3, 2, 1, 0])


def test_counter_rng_matches_oracle():
    from oracle import pyoracle as po
    from monte_carlo_path_tracing_amd import rng
    for args in [(20240430, 0, 0, 1, 0), (20240430, 479999, 1023, 2 ** 40 + 3, 6), (1, 2, 3, 4, 5)]:
        assert rng.counter_uniform(*args) == po.counter_uniform(*args)


QUANT_HARNESS = r"""
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include "mcpt_internal.h"
using namespace mcpt;
static float dec(uint32_t q, uint32_t ex, int a, int k, float org) {
    uint32_t bits = ((ex >> (8 * a)) & 0xffu) << 23;
    float sc;
    std::memcpy(&sc, &bits, 4);
    return std::fmaf((float)((q >> (8 * k)) & 0xffu), sc, org);
}
int main() {
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> U(0, 1);
    std::vector<BvhNode4> in;
    for (int i = 0; i < 20000; i++) {
        BvhNode4 n{};
        const double scale = std::pow(10.0, -4 + 8 * U(rng)), off = (U(rng) - 0.5) * 1e3 * (i % 3);
        for (int k = 0; k < 4; k++) {
            n.child[k] = (i % 7 == 0 && k == 3) ? kBvh4Empty : k;
            for (int a = 0; a < 3; a++) {
                double lo = off + scale * U(rng), hi = lo + ((i % 5 == 0 && a == 1) ? 0.0 : scale * U(rng));
                n.lo[a][k] = n.child[k] == kBvh4Empty ? FLT_MAX : (float)lo;
                n.hi[a][k] = n.child[k] == kBvh4Empty ? -FLT_MAX : std::nextafter((float)hi, FLT_MAX);
            }
        }
        in.push_back(n);
    }
    std::vector<BvhNode4Q> q = quantize_bvh4(in);
    long bad = 0, loose = 0;
    for (size_t i = 0; i < in.size(); i++)
        for (int a = 0; a < 3; a++) {
            float lo = FLT_MAX, hi = -FLT_MAX;
            for (int k = 0; k < 4; k++)
                if (in[i].child[k] != kBvh4Empty) lo = std::fmin(lo, in[i].lo[a][k]), hi = std::fmax(hi, in[i].hi[a][k]);
            for (int k = 0; k < 4; k++) {
                if (q[i].child[k] != in[i].child[k]) bad++;
                if (in[i].child[k] == kBvh4Empty) continue;
                const float dl = dec(q[i].q[2 * a], q[i].ex, a, k, q[i].org[a]), dh = dec(q[i].q[2 * a + 1], q[i].ex, a, k, q[i].org[a]);
                if (!(dl <= in[i].lo[a][k]) || !(dh >= in[i].hi[a][k])) bad++;
                const double tol = 2.0 * (hi - lo) / 255.0 + 4 * std::fabs(std::nextafter(std::fabs(hi) + std::fabs(lo), FLT_MAX) - (std::fabs(hi) + std::fabs(lo)));
                if (in[i].lo[a][k] - dl > tol || dh - in[i].hi[a][k] > tol) loose++;
            }
        }
    std::printf("%ld %ld\n", bad, loose);
    return 0;
}
"""


def test_bvh4_quantization_is_conservative(tmp_path):
    """quantize_bvh4 (csrc/bvh.cpp, the 64-B nodes of k_rays_persistent): every decoded plane
    fma(byte, 2^(ex-127), org) -- evaluated with the same correctly rounded fp32 fma as the GPU --
    lies outside its fp32 box (the traversal only prunes with it), within two quantisation steps of
    it, over random boxes of 1e-4..1e4 extents, offsets, flat axes and empty slots"""
    src = tmp_path / "quant.cpp"
    src.write_text(QUANT_HARNESS)
    exe = tmp_path / "quant"
    csrc = ROOT / "monte_carlo_path_tracing_amd" / "csrc"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", str(ROOT / "include"), "-I", str(csrc), str(src), str(csrc / "bvh.cpp"),
                    "-o", str(exe)], check=True)
    bad, loose = map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    assert bad == 0
    assert loose == 0


def test_malformed_scene_corpus_fails_cleanly(tmp_path):
    """tools/sanitize/make_corpus.py's malformed OBJ/MTL/XML cases and seeded mutations of the stand-in
    (the corpus `make sanitize` runs under ASan/UBSan) through mcpt_scene_load and the oracle's loader:
    each loads or returns an error -- no crash (out-of-range face indices, directories, NUL bytes and
    zero-extent grids were found this way)."""
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "sanitize" / "make_corpus.py"), str(tmp_path), "30"],
                         check=True, capture_output=True, text=True).stdout.split()
    pairs = list(zip(out[0::2], out[1::2]))
    loaded = 0
    for obj, xml in pairs:
        try:
            sc = mcpt.Scene.load(obj, xml)
            loaded += 1
            try:
                sc.meshing((0.0, 0.0, 0.0))
            except mcpt.MCPTError:  # zero-extent box: refused, not divided by
                pass
            sc.close()
        except mcpt.MCPTError:
            pass
        try:
            po.Scene(obj, xml)
        except RuntimeError:
            pass
    assert 0 < loaded < len(pairs)


_SHIM_LOAD = r"""
import os, sys
sys.path.insert(0, os.environ["MCPT_ROOT"])
import monte_carlo_path_tracing_amd as mcpt
mcpt.set_collective_lib(os.environ["SHIM"])
uid = mcpt.Comm.unique_id()  # the shim's ncclGetUniqueId (no GPU involved)
assert len(uid) == mcpt.COMM_ID_BYTES and uid[:8] == b"MCPTSHIM", uid[:16]
try:
    mcpt.set_collective_lib(os.environ["SHIM"])
    raise SystemExit("second set_collective_lib accepted after the library was resolved")
except mcpt.MCPTError as e:
    assert "already resolved" in str(e), e
# a collective library without the NCCL entry points is refused with a message, not a crash
print("ok")
"""


def test_collective_lib_override_loads_the_shim(tmp_path):
    """mcpt_debug_set_collective_lib (include/mcpt_debug.h): the library resolves its NCCL entry points
    from tests/collshim/libmcpt_collshim.so instead of RCCL (the multi-rank GPU tests' stand-in), and
    refuses a change once resolved.  The shim's unique id needs no GPU."""
    shim = ROOT / "tests" / "collshim" / "libmcpt_collshim.so"
    if not shim.exists():
        subprocess.run(["make", "-s", "-C", str(shim.parent)], check=True)
    script = tmp_path / "shim.py"
    script.write_text(_SHIM_LOAD)
    import os
    r = subprocess.run([sys.executable, str(script)], env=dict(os.environ, MCPT_ROOT=str(ROOT), SHIM=str(shim)),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
    nm = subprocess.run(["nm", "-D", "--defined-only", str(shim)], capture_output=True, text=True, check=True).stdout
    for sym in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommInitAll", "ncclReduce", "ncclGroupStart", "ncclGroupEnd",
                "ncclCommDestroy", "ncclCommAbort", "ncclGetErrorString"):
        assert sym in nm, sym
