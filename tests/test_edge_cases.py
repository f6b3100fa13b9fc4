"""Edge cases of the render path against the CPU oracle (GPU) and of the host logic (CPU):
scenes without lights, > 4096 light candidates per point (the sequential batch search of the
full prep and of the root-cache pick), N_L beyond the LDS candidate list (the LDS-queue prep
variant without root cache), 1 spp (no root cache), 1x1 / odd frames, cameras that miss
everything, and render-option validation."""
import numpy as np
import pytest

import monte_carlo_path_tracing_amd as mcpt
from conftest import SCENE_OBJ, SCENE_XML
from oracle import pyoracle as po
import scenegen

SEED = 20240430
L2_TOL = 1e-3
OMODE = {"mis": po.MODE_MIS, "brdf": po.MODE_BRDF, "shade": po.MODE_SHADE}


def rel_l2(g, c):
    return float(np.linalg.norm(g - c) / max(np.linalg.norm(c), 1e-300))


def max_px_rel(g, c):
    """max over pixels of ||g_px - c_px|| / ||c_px|| (pixels black in both count 0)"""
    d = np.linalg.norm((g - c).reshape(-1, 3), axis=1)
    n = np.linalg.norm(c.reshape(-1, 3), axis=1)
    return float(np.max(np.where(n > 0, d / np.maximum(n, 1e-300), np.where(d > 0, np.inf, 0.0))))


def pair(obj, xml, W, H, spp, mode):
    s = mcpt.Scene.load(obj, xml)
    g = s.camera()
    g.width, g.height = W, H
    img, st = mcpt.render(s, g, spp, mode=mode, seed=SEED)
    o = po.Scene(obj, xml)
    c = o.camera()
    c.width, c.height = W, H
    e, _ = po.camera_ray(c, 0, 0)
    o.build_grid(e)
    ref, _ = o.render(c, OMODE[mode], SEED, spp, nthreads=8)
    return img, ref, st


def test_synthetic_scenes_load(tmp_path):
    for make, nl in ((scenegen.no_lights, 0), (scenegen.light_panel, 7200), (scenegen.dense_sphere, 14160)):
        obj, xml = make(str(tmp_path))
        s = mcpt.Scene.load(obj, xml)
        assert s.nlights == nl
        o = po.Scene(obj, xml)
        v18, mat, lo, un = o.facets()
        assert np.array_equal(s.arrays()["positions"], v18[:, :9])


def test_render_option_validation():
    s = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    cam = mcpt.Camera.reference(8, 6)
    for bad in (dict(spp=0), dict(spp=4, sample_range=(3, 2)), dict(spp=4, sample_range=(0, 5)),
                dict(spp=4, mode="nope")):
        spp = bad.pop("spp")
        with pytest.raises((mcpt.MCPTError, ValueError)):
            mcpt.render(s, cam, spp, **bad)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["mis", "shade", "brdf"])
def test_no_lights_renders_black(tmp_path, mode):
    img, ref, _ = pair(*scenegen.no_lights(str(tmp_path)), 16, 12, 4, mode)
    assert np.isfinite(img).all() and not img.any() and not ref.any()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,spp", [("mis", 4), ("shade", 4), ("mis", 1)])
def test_more_than_4096_candidates(tmp_path, mode, spp):
    """floor points under a 7200-triangle panel: every panel triangle is a candidate (113 batches)"""
    img, ref, st = pair(*scenegen.light_panel(str(tmp_path)), 16, 12, spp, mode)
    assert ref.sum() > 0 and rel_l2(img, ref) <= L2_TOL and max_px_rel(img, ref) <= L2_TOL, (rel_l2(img, ref), max_px_rel(img, ref))
    assert st.light_evals_candidates > 4096 * st.prep_full_nodes // 2


@pytest.mark.gpu
@pytest.mark.parametrize("nx", [20, 32, 40, 60])
def test_root_cache_pick_paths(tmp_path, nx):
    """Light panels of 2 nx^2 triangles that every floor point sees: <= 16 (nx 20), <= 32 (32),
    <= 64 (40) and > 64 (60) candidate batches per root, i.e. every batch-search path of k_prep_pick
    (four roots per wave scan, two, one, sequential).  The root-point cache must give the frame the
    full prep gives (MCPT_DEBUG_NO_ROOT_CACHE) up to fp64 accumulation order, and the oracle's."""
    obj, xml = scenegen.light_panel(str(tmp_path), nx, nx)
    s = mcpt.Scene.load(obj, xml)
    g = s.camera()
    g.width, g.height = 24, 18
    a, sa = mcpt.render(s, g, 4, mode="mis", seed=SEED)
    b, sb = mcpt.render(s, g, 4, mode="mis", seed=SEED, flags=mcpt.DEBUG_NO_ROOT_CACHE)
    assert sa.prep_cached_nodes > 0 and sb.prep_cached_nodes == 0
    assert a.sum() > 0 and rel_l2(a, b) <= 1e-12, rel_l2(a, b)
    img, ref, _ = pair(obj, xml, 24, 18, 4, "mis")
    assert rel_l2(img, ref) <= L2_TOL and max_px_rel(img, ref) <= L2_TOL, (rel_l2(img, ref), max_px_rel(img, ref))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["mis", "shade"])
def test_light_table_beyond_the_lds_list(tmp_path, mode):
    """N_L = 14160 > 7680: the LDS-queue prep variant, no root-point cache"""
    img, ref, st = pair(*scenegen.dense_sphere(str(tmp_path)), 16, 12, 4, mode)
    assert st.prep_cached_nodes == 0
    assert ref.sum() > 0 and rel_l2(img, ref) <= L2_TOL and max_px_rel(img, ref) <= L2_TOL, (rel_l2(img, ref), max_px_rel(img, ref))


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,spp,mode", [(1, 1, 16, "mis"), (7, 3, 1, "mis"), (5, 9, 3, "shade"), (13, 1, 2, "brdf")])
def test_tiny_and_odd_frames(W, H, spp, mode):
    s = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    img, st = mcpt.render(s, mcpt.Camera.reference(W, H), spp, mode=mode, seed=SEED)
    o = po.Scene(SCENE_OBJ, SCENE_XML)
    e, _ = po.camera_ray(po.reference_camera(400, 300), 0, 0)
    o.build_grid(e)
    ref, _ = o.render(po.reference_camera(W, H), OMODE[mode], SEED, spp, nthreads=4)
    assert img.shape == (H, W, 3) and rel_l2(img, ref) <= L2_TOL and max_px_rel(img, ref) <= L2_TOL
    if spp == 1:
        assert st.prep_cached_nodes == 0


@pytest.mark.gpu
def test_camera_missing_everything():
    s = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    cam = mcpt.Camera.reference(32, 24)
    cam.eye[:], cam.lookat[:] = (100.0, 0.0, 0.0), (200.0, 0.0, 0.0)  # outside the scene, looking away
    cam.dist_scale = 1.0
    for mode in ("mis", "shade", "brdf"):
        img, st = mcpt.render(s, cam, 4, mode=mode, seed=SEED)
        assert not img.any() and st.shading_nodes == 0


def test_occluded_room_is_supercritical(tmp_path):
    """the oracle's own node count shows the room grows trees of ~1.2 children per node (CPU)"""
    obj, xml = scenegen.occluded_room(str(tmp_path))
    o = po.Scene(obj, xml)
    c = o.camera()
    c.width, c.height = 4, 3
    e, _ = po.camera_ray(c, 0, 0)
    o.build_grid(e)
    _, ost = o.render(c, po.MODE_MIS, SEED, 1, nthreads=8)
    assert ost[1] > 100 * 12  # prep nodes per camera sample, far above a subcritical tree's ~2


def test_depth_cap_truncates_nothing_measurable(tmp_path):
    """The counter-RNG trees stop below depth 48 (device_math.h MCPT_MAX_DEPTH, the oracle's COUNTER_MAX_DEPTH);
    the reference has no cap (main.cpp:429-437).  On the supercritical room (m ~ 1.13 children per node, the
    node count per level GROWS) the frame cut at 48 equals the frame cut at 62 to rounding, and already at 24
    the deeper levels carry < 1e-12 of the frame: a level's contribution decays with the surfaces' albedo
    (~0.15 per level here), not with the tree's size (tools/depth_cap_study.py, profiles/round6_depth_cap.json)."""
    obj, xml = scenegen.occluded_room(str(tmp_path))
    o = po.Scene(obj, xml)
    c = o.camera()
    c.width, c.height = 4, 3
    e, _ = po.camera_ray(c, 0, 0)
    o.build_grid(e)
    f24, _ = o.depth_study(c, SEED, 2, 24, nthreads=8)
    f48, h48 = o.depth_study(c, SEED, 2, 48, nthreads=8)
    f62, h62 = o.depth_study(c, SEED, 2, 62, nthreads=8)
    n = h62[:63].astype(float)
    assert n[40] > n[20] > n[5] > 0  # supercritical: more nodes at every deeper level
    assert h48[63] > 0  # the cap does cut nodes here
    assert rel_l2(f48, f62) <= 1e-15 and rel_l2(f24, f62) <= 1e-12, (rel_l2(f48, f62), rel_l2(f24, f62))


@pytest.mark.gpu
def test_supercritical_tree_spills_and_matches_oracle(tmp_path):
    """Binary recursion main.cpp:455-491 with occluded lights: each generation outgrows the queue
    (queue_factor 1, one camera sample per pixel per refill), so the excess is parked on the spill
    stack and drained later; the frame must equal the default-queue render and the oracle, with
    exactly the oracle's number of shading nodes (no node lost or duplicated)."""
    obj, xml = scenegen.occluded_room(str(tmp_path))
    s = mcpt.Scene.load(obj, xml)
    g = s.camera()
    g.width, g.height = 8, 6
    img, st = mcpt.render(s, g, 2, mode="mis", seed=SEED, samples_per_launch=1, queue_factor=1)
    big, st2 = mcpt.render(s, g, 2, mode="mis", seed=SEED)
    o = po.Scene(obj, xml)
    c = o.camera()
    c.width, c.height = 8, 6
    e, _ = po.camera_ray(c, 0, 0)
    o.build_grid(e)
    ref, ost = o.render(c, po.MODE_MIS, SEED, 2, nthreads=8)
    assert st.spilled_nodes > 0
    assert st.shading_nodes == st2.shading_nodes == int(ost[1])
    assert ref.sum() > 0 and rel_l2(img, big) <= 1e-12 and rel_l2(img, ref) <= L2_TOL and max_px_rel(img, ref) <= L2_TOL, (
        rel_l2(img, big), rel_l2(img, ref), max_px_rel(img, ref))
