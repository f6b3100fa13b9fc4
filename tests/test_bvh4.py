"""The 4-wide tree every traversal kernel reads (collapse_bvh4 of the binary SAH tree, bvh.cpp) and its
quantized form (quantize_bvh4, the persistent traversal's 64-B nodes), checked on the host through
mcpt_debug_bvh4_check: every facet of the binary tree reached -- once, with every vertex inside the fp32 box
of every slot on its path, or (spatial splits) in several leaves whose path regions together cover the
triangle -- and every quantized slot box containing its fp32 box -- the conservative
pruning that keeps the closest hits equal to the reference's (Myobj.cpp:334-474 / :476-622 replaced by the
BVH).  The GPU side (the same trees' hits against the reference's golden rays and the
brute force) is test_gpu_parity.py."""
import pytest

from conftest import SCENE_OBJ, SCENE_XML, cornell_scene
import monte_carlo_path_tracing_amd as mcpt

def max_dup(r):
    """repeated references a tree may hold: none, except where the builder makes spatial splits (trees of at
    least 65 536 triangles, bvh.cpp MCPT_BVH_SPATIAL_MIN; at most 0.3 per triangle)"""
    return 0 if r["facets"] < 65536 else 0.3 * r["facets"]

import scenegen


def ok(r, nf):
    return r["tris"] == r["facets"] == nf and r["duplicates"] <= max_dup(r) and r["errors"] == 0 and r["nodes"] > 0


@pytest.mark.parametrize("light_only", [False, True])
def test_bvh4_structure_veach(light_only):
    sc = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    r = mcpt.debug_bvh4_check(sc, light_only)
    print("veach bvh4 (light_only=%s): %s" % (light_only, r))
    assert ok(r, sc.nlights if light_only else sc.nfacets), r


@pytest.mark.parametrize("name", ["occluded_room", "sphere_mix", "slivers", "tiny_far", "dense_sphere", "light_panel"])
def test_bvh4_structure_generated(tmp_path, name):
    gen = getattr(scenegen, name, None)
    if gen is None:
        pytest.skip("no scene %s" % name)
    sc = mcpt.Scene.load(*gen(str(tmp_path)))
    for lo in (False, True):
        r = mcpt.debug_bvh4_check(sc, lo)
        assert ok(r, sc.nlights if lo else sc.nfacets), (name, lo, r)


def test_bvh4_structure_cornell_1m():
    sc = mcpt.Scene.load(*cornell_scene(1000000))
    r = mcpt.debug_bvh4_check(sc)
    print("cornell-1M bvh4: %s" % r)
    assert ok(r, sc.nfacets), r
    assert r["depth"] <= 40  # the traversal stacks hold 48 entries


def test_builder_is_deterministic():
    """the parallel plan phase (split searches of disjoint ranges on their own threads) and the spatial splits
    of a >= 65 536-triangle tree give the same tree on every load"""
    paths = cornell_scene(200000)
    a, b = mcpt.Scene.load(*paths), mcpt.Scene.load(*paths)
    assert a.accel_bytes() == b.accel_bytes()
    for lo in (False, True):
        assert mcpt.debug_bvh4_check(a, lo) == mcpt.debug_bvh4_check(b, lo)
        assert mcpt.debug_bvh8_check(a, lo) == mcpt.debug_bvh8_check(b, lo)
    assert mcpt.debug_bvh4_check(a)["duplicates"] > 0  # spatial splits did happen


def test_builder_is_deterministic_when_the_spatial_budget_runs_out(tmp_path):
    """a scene whose spatial splits want more duplicates than the budget (0.3 per triangle) allows: the budget is
    handed down the tree by value (bvh.cpp splan), so the exhausted budget still gives the same tree on every load
    -- parallel builder threads never race for it -- and the cap holds for the whole tree"""
    paths = scenegen.needles(str(tmp_path))
    a, b = mcpt.Scene.load(*paths), mcpt.Scene.load(*paths)
    assert a.accel_bytes() == b.accel_bytes()
    ra, rb = mcpt.debug_bvh4_check(a), mcpt.debug_bvh4_check(b)
    print("needles bvh4: %s" % ra)
    assert ra == rb and ok(ra, a.nfacets), ra
    assert ra["duplicates"] > 0.2 * ra["facets"]  # the budget was (nearly) used up
    assert mcpt.debug_bvh8_check(a) == mcpt.debug_bvh8_check(b)
