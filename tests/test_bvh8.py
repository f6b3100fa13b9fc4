"""The 8-wide compressed BVH (BvhNode8Q, mcpt_internal.h) and its persistent traversal k_rays_cw8
(render.hip), which replaces the reference's grid DDA (Myobj.cpp:334-474 closest hit, :476-622 light-only
hit) for scenes beyond an XCD's L2 (config C5).

CPU: the tree against its binary tree (mcpt_debug_bvh8_check, host only): every facet reached, each reference's
triangle covered by the decoded boxes of the slots on its path (the conservative pruning that keeps hits exact;
a facet split spatially sits in several leaves, test_bvh4.py).
GPU: hits bit-identical to the 4-wide traversal -- the reference's golden rays (which the 4-wide traversal
matches, test_gpu_parity.py) and rays aimed at vertices / edges -- and renders through k_rays_cw8 equal to
the default kernels' up to fp64 accumulation order (<= 1e-12 relative L2).
"""
import numpy as np
import pytest

from conftest import GOLDEN, SCENE_OBJ, SCENE_XML, cornell_scene
import monte_carlo_path_tracing_amd as mcpt

def max_dup(r):
    """repeated references a tree may hold: none, except where the builder makes spatial splits (trees of at
    least 65 536 triangles, bvh.cpp MCPT_BVH_SPATIAL_MIN; at most 0.3 per triangle)"""
    return 0 if r["facets"] < 65536 else 0.3 * r["facets"]

import scenegen

SEED = 20240430


def rel_l2(g, c):
    return float(np.linalg.norm(g - c) / max(np.linalg.norm(c), 1e-300))


@pytest.fixture(scope="module")
def scene():
    return mcpt.Scene.load(SCENE_OBJ, SCENE_XML)


@pytest.mark.parametrize("light_only", [False, True])
def test_bvh8_structure_veach(scene, light_only):
    r = mcpt.debug_bvh8_check(scene, light_only)
    print("veach bvh8 (light_only=%s): %s" % (light_only, r))
    assert r["tris"] == r["facets"] == (scene.nlights if light_only else scene.nfacets)
    assert r["duplicates"] <= max_dup(r) and r["errors"] == 0 and r["nodes"] > 0


@pytest.mark.parametrize("name", ["occluded_room", "sphere_mix", "slivers", "tiny_far", "dense_sphere", "light_panel"])
def test_bvh8_structure_generated(tmp_path, name):
    gen = getattr(scenegen, name, None)
    if gen is None:
        pytest.skip("no scene %s" % name)
    sc = mcpt.Scene.load(*gen(str(tmp_path)))
    for lo in (False, True):
        r = mcpt.debug_bvh8_check(sc, lo)
        assert r["tris"] == r["facets"] and r["duplicates"] <= max_dup(r) and r["errors"] == 0, (name, lo, r)


def test_bvh8_structure_cornell_1m():
    sc = mcpt.Scene.load(*cornell_scene(1000000))
    r = mcpt.debug_bvh8_check(sc)
    print("cornell-1M bvh8: %s" % r)
    assert r["tris"] == r["facets"] == sc.nfacets and r["duplicates"] <= max_dup(r) and r["errors"] == 0
    assert r["depth"] <= 12  # 8-wide: ~log8(1M) levels (the stack holds 48 groups)


@pytest.mark.gpu
@pytest.mark.parametrize("light_only", [False, True])
def test_golden_rays_through_bvh8(scene, light_only):
    """the reference's 12 000 golden rays: the 8-wide batch query equals the 4-wide one bit for bit (facet,
    t, beta, gamma), which test_gpu_parity.py checks against the reference's grid"""
    rin = np.load(GOLDEN / "rays_in.npy")
    ex = rin[:, 6].astype(np.int32)
    f4, t4 = mcpt.closest_hit(scene, rin[:, :3], rin[:, 3:6], ex, light_only)
    f8, t8 = mcpt.closest_hit(scene, rin[:, :3], rin[:, 3:6], ex, light_only, wide=True)
    assert np.array_equal(f8, f4)
    assert np.array_equal(t8[f8 >= 0], t4[f4 >= 0])
    print("bvh8 golden rays (light_only=%s): %d/%d hit, identical" % (light_only, (f8 >= 0).sum(), len(f8)))


@pytest.mark.gpu
@pytest.mark.parametrize("light_only", [False, True])
def test_edge_and_vertex_rays_through_bvh8(scene, light_only):
    """rays at vertices, edge points and a few ulps off them (test_gpu_parity.py's construction): identical
    to the 4-wide traversal"""
    arr = scene.arrays()
    P = arr["positions"].astype(np.float64).reshape(-1, 3, 3)
    rng = np.random.default_rng(11)
    n = 20000
    tri = rng.integers(0, len(P), n) if not light_only else np.asarray(arr["light_facet"])[rng.integers(0, scene.nlights, n)]
    kind = rng.integers(0, 3, n)
    w = rng.random((n, 3))
    w[kind == 0] = np.eye(3)[rng.integers(0, 3, (kind == 0).sum())]
    e = rng.integers(0, 3, n)
    w[(kind == 1), e[kind == 1]] = 0.0
    w /= w.sum(axis=1, keepdims=True)
    target = np.einsum("nk,nkc->nc", w, P[tri]) * (1.0 + rng.choice([0.0, 1e-15, -1e-15, 1e-12], (n, 1)))
    lo, hi = P.reshape(-1, 3).min(axis=0), P.reshape(-1, 3).max(axis=0)
    ro = lo + rng.random((n, 3)) * (hi - lo)
    near = rng.random(n) < 0.3
    ro[near] = target[near] + rng.normal(0, 0.05, (near.sum(), 3))
    rd = target - ro
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    ex = np.where(rng.random(n) < 0.2, tri, -1).astype(np.int32)
    f4, t4 = mcpt.closest_hit(scene, ro, rd, ex, light_only)
    f8, t8 = mcpt.closest_hit(scene, ro, rd, ex, light_only, wide=True)
    assert np.array_equal(f8, f4) and np.array_equal(t8, t4)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,spp", [("mis", 8), ("shade", 8), ("shade_area", 16)])
def test_render_through_k_rays_cw8_equals_default(scene, mode, spp):
    """MCPT_DEBUG_RAYS_PERSIST | MCPT_DEBUG_RAYS_CW8: the MIS / shade ray sets of the small stand-in through
    the persistent 8-wide traversal (and the persistent 4-wide one) -- the same hits, so the same frame up to
    fp64 accumulation order"""
    cam = mcpt.Camera.reference(160, 120)
    a, _ = mcpt.render(scene, cam, spp, mode=mode, seed=SEED)
    cw8 = mcpt.DEBUG_RAYS_PERSIST | mcpt.DEBUG_RAYS_CW8
    b, _ = mcpt.render(scene, cam, spp, mode=mode, seed=SEED, flags=cw8)
    c, sc = mcpt.render(scene, cam, spp, mode=mode, seed=SEED, flags=cw8 | mcpt.DEBUG_COUNT_TRAVERSAL)
    d, _ = mcpt.render(scene, cam, spp, mode=mode, seed=SEED, flags=mcpt.DEBUG_RAYS_PERSIST)
    assert rel_l2(d, a) <= 1e-12
    print("%s 160x120x%d through k_rays_cw8: rel L2 vs default %.2e; %d visits, %d tests" % (
        mode, spp, rel_l2(b, a), sc.node_visits, sc.tri_tests))
    assert rel_l2(b, a) <= 1e-12 and rel_l2(c, a) <= 1e-12
    assert sc.node_visits > 0 and sc.tri_tests > 0


@pytest.mark.gpu
def test_cornell_1m_cw8_equals_bvh4_persistent():
    """C5's scene (1M random triangles, trees beyond L2: the persistent traversal) through the 8-wide trees
    (MCPT_DEBUG_RAYS_CW8) against the 4-wide ones, and random rays through both batch queries"""
    sc = mcpt.Scene.load(*cornell_scene(1000000))
    cam = sc.camera()
    cam.width, cam.height = 128, 96
    a, sa = mcpt.render(sc, cam, 8, mode="mis", seed=SEED, flags=mcpt.DEBUG_RAYS_CW8 | mcpt.DEBUG_COUNT_TRAVERSAL)
    b, sb = mcpt.render(sc, cam, 8, mode="mis", seed=SEED, flags=mcpt.DEBUG_COUNT_TRAVERSAL)
    print("cornell-1M 128x96x8 MIS: cw8 vs 4-wide rel L2 %.2e; visits per ray %.2f (cw8) vs %.2f (4-wide)" % (
        rel_l2(a, b), sa.node_visits / max(sa.rays + sa.light_rays, 1), sb.node_visits / max(sb.rays + sb.light_rays, 1)))
    assert rel_l2(a, b) <= 1e-12
    rng = np.random.default_rng(5)
    n = 50000
    ro = rng.random((n, 3)) * 556.0
    rd = rng.normal(size=(n, 3))
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    ex = np.full(n, -1, np.int32)
    f4, t4 = mcpt.closest_hit(sc, ro, rd, ex)
    f8, t8 = mcpt.closest_hit(sc, ro, rd, ex, wide=True)
    assert np.array_equal(f8, f4) and np.array_equal(t8, t4)
    print("cornell-1M: %d random rays, %d hits, identical" % (n, (f8 >= 0).sum()))
