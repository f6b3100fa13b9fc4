"""MCPT_ACCEL_GRID: the reference's own uniform grid (Myobj::cal_scene_boundingbox + meshing,
Myobj.cpp:78-162) and its 3D-DDA with the in-cell acceptance rule (Myobj.cpp:334-474, light-only
476-622) on the GPU -- SURVEY.md §8(f) row 3.  Unlike the BVH it reproduces the reference hit for
hit, including the bbox "crack" (rays whose origin rounds to cell -1 miss), so the 12 000 golden
random rays of the compiled reference must match with NO exceptions."""
import numpy as np
import pytest

from conftest import GOLDEN, SCENE_OBJ, SCENE_XML, TIGHT_L2
import monte_carlo_path_tracing_amd as mcpt
from oracle import pyoracle as po

SEED = 20240430


@pytest.fixture(scope="module")
def scene():
    s = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    eye, _ = po.camera_ray(po.reference_camera(400, 300), 0, 0)  # the eye the goldens were made with
    s.meshing(eye, 100000)
    return s


def test_grid_box_and_cell_match_reference(scene):
    """host-side build (no GPU): bbox with the camera and cell edge bit-exact vs the reference"""
    box, cells = scene.grid_info()
    gb = np.load(GOLDEN / "grid_bbox.npy")[0]
    assert np.array_equal(box, gb[:7])
    assert (cells >= 2).all()


def test_grid_invalid_arguments(scene):
    with pytest.raises(mcpt.MCPTError):
        scene.meshing([0.0, 0.0, 0.0], 0)
    s2 = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    with pytest.raises(mcpt.MCPTError):
        s2.grid_info()  # no grid yet


@pytest.mark.gpu
@pytest.mark.parametrize("light_only,name", [(False, "rays_hit.npy"), (True, "rays_lighthit.npy")])
def test_grid_rays_bitexact_vs_reference_including_crack(scene, light_only, name):
    rin, gold = np.load(GOLDEN / "rays_in.npy"), np.load(GOLDEN / name)
    f, tbg = mcpt.closest_hit(scene, rin[:, :3], rin[:, 3:6], rin[:, 6].astype(np.int32), light_only, grid=True)
    assert np.array_equal(f, gold[:, 0].astype(np.int32))
    hit = f >= 0
    assert np.array_equal(tbg[hit], gold[hit, 1:])
    bb = np.load(GOLDEN / "grid_bbox.npy")[0]
    crack = (np.floor((rin[:, :3] - bb[[0, 2, 4]]) * (1.0 / bb[6])) < 0).any(axis=1)
    fb, _ = mcpt.closest_hit(scene, rin[:, :3], rin[:, 3:6], rin[:, 6].astype(np.int32), light_only)
    print("grid: %d/%d rays bit-exact; %d crack rays where the BVH (true closest hit) differs from the "
          "reference grid: %d" % (len(rin), len(rin), crack.sum(), (fb != f).sum()))
    assert crack.any() and ((fb != f) <= crack).all()


@pytest.mark.gpu
def test_grid_query_needs_meshing():
    s2 = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    with pytest.raises(mcpt.MCPTError):
        mcpt.closest_hit(s2, np.zeros((1, 3)), np.array([[1.0, 0, 0]]), grid=True)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,spp", [("mis", 8), ("brdf", 32), ("shade", 8)])
def test_grid_render_vs_oracle_and_bvh(mode, spp):
    """grid renders against the oracle (which traverses the same grid) and against the BVH render"""
    sc = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    cam = mcpt.Camera.reference(80, 60)
    g, st = mcpt.render(sc, cam, spp, mode=mode, seed=SEED, accel="grid")
    b, _ = mcpt.render(sc, cam, spp, mode=mode, seed=SEED)
    o = po.Scene(SCENE_OBJ, SCENE_XML)
    ocam = po.reference_camera(80, 60)
    e, _ = po.camera_ray(ocam, 0, 0)
    o.build_grid(e)
    c, _ = o.render(ocam, {"mis": po.MODE_MIS, "brdf": po.MODE_BRDF, "shade": po.MODE_SHADE}[mode], SEED, spp, nthreads=8)
    err = float(np.linalg.norm(g - c) / np.linalg.norm(c))
    dgb = float(np.linalg.norm(g - b) / np.linalg.norm(b))
    print("grid %s 80x60x%d: rel L2 vs oracle %.2e, vs BVH render %.2e, %.4f s device" % (mode, spp, err, dgb, st.seconds))
    assert np.isfinite(g).all() and err <= 1e-3 and dgb <= 1e-3
    assert err <= TIGHT_L2 and dgb <= 1e-12, (err, dgb)  # what the build achieves (tests/conftest.py)
