"""Pin the CPU oracle (oracle/mcpt_oracle.c) against golden vectors of the compiled reference.

The goldens in tests/golden/ were produced by oracle/ref_harness.cpp linked against the
reference's own translation units (`make -C oracle golden`, see tests/golden/README.md).  Every
comparison here is BIT-EXACT (fp64 ==), except where a test says otherwise.
"""
import numpy as np
import pytest

from conftest import GOLDEN, SCENE_OBJ, SCENE_XML
from oracle import pyoracle as po

pytestmark = pytest.mark.oracle


@pytest.fixture(scope="module")
def scene():
    s = po.Scene(SCENE_OBJ, SCENE_XML)
    cam = po.reference_camera(400, 300)
    eye, _ = po.camera_ray(cam, 0, 0)
    s.build_grid(eye)
    return s


def g(name):
    return np.load(GOLDEN / name)


def test_loader_facets_bitexact(scene):
    v, mat, light_of, un = scene.facets()
    gv = g("loader_facets.npy")
    assert v.shape == gv.shape
    assert np.array_equal(v.view(np.uint32), gv.view(np.uint32))
    assert np.array_equal(mat, g("loader_mat.npy")[:, 0])
    assert np.array_equal(un, g("unique_normal.npy"))  # Myobj.cpp:680-709


def test_loader_materials_and_lights(scene):
    assert np.array_equal(scene.materials(), g("materials.npy"))
    f, a = scene.lights()
    assert np.array_equal(f, g("light_order.npy")[:, 0])  # Mylight.cpp:88 map order
    assert np.array_equal(a, g("light_area_radiance.npy"))


def test_grid_bbox(scene):
    gb = g("grid_bbox.npy")[0]
    assert np.array_equal(scene.grid_info(), gb[:7])


def test_primary_hit_map(scene):
    cam = po.reference_camera(400, 300)
    gp = g("primary_400x300.npy")
    out = []
    for i in range(cam.height):
        for j in range(cam.width):
            e, d = po.camera_ray(cam, i, j)
            f, tbg = scene.closest_hit(e, d, -1)
            out.append((f, tbg[0], tbg[1], tbg[2]) if f >= 0 else (-1, 0, 0, 0))
    assert np.array_equal(np.array(out, np.float64), gp)


def test_random_rays_closest_and_light_only(scene):
    rin, gh, gl = g("rays_in.npy"), g("rays_hit.npy"), g("rays_lighthit.npy")
    for r in range(rin.shape[0]):
        ro, rd, ex = rin[r, :3], rin[r, 3:6], int(rin[r, 6])
        for light_only, gold in ((False, gh), (True, gl)):
            f, tbg = scene.closest_hit(ro, rd, ex, light_only)
            got = (f, tbg[0], tbg[1], tbg[2]) if f >= 0 else (-1, 0, 0, 0)
            assert np.array_equal(np.array(got, np.float64), gold[r]), (r, light_only, got, gold[r])


def test_light_prep_sampling_and_pdf(scene):
    pin, gout = g("prep_in.npy"), g("prep_out.npy")
    lf, _ = scene.lights()
    pos = {int(f): k for k, f in enumerate(lf)}
    for r in range(pin.shape[0]):
        x1, n, ctr = pin[r, :3], pin[r, 3:6], int(pin[r, 6])
        ws, idx, w = scene.light_prep(x1, n)
        o = gout[r]
        assert ws == o[0] and len(idx) == o[1] and float(idx.sum()) == o[2], r
        fw = list(w[:2]) + [-1.0] * (2 - min(2, len(w)))
        assert fw[0] == o[3] and fw[1] == o[4]
        s = scene.light_sample_ref(ctr, x1, n)
        assert s[0] == o[5], r
        assert np.array_equal(s[1:4], o[6:9]) and s[4] == o[9] and s[5] == o[10], (r, s, o[5:11])
        for q in range(2):
            assert scene.light_pdf(x1, n, int(o[12 + 2 * q])) == o[11 + 2 * q]
        assert all(int(f) in pos for f in [o[12], o[14]])


def test_brdf_eval_pdf_sample(scene):
    bin_, bout = g("brdf_in.npy"), g("brdf_out.npy")
    mats = scene.materials().astype(np.float64)
    for r in range(bin_.shape[0]):
        n, wi, wr, m, ctr = bin_[r, :3], bin_[r, 3:6], bin_[r, 6:9], int(bin_[r, 9]), int(bin_[r, 10])
        kd, ks, ns = mats[m, :3], mats[m, 3:6], mats[m, 6]
        o = bout[r]
        assert np.array_equal(po.brdf_phong(n, wi, wr, kd, ks, ns), o[:3]), r
        assert po.phong_pdf(n, wi, wr, kd, ks, ns) == o[3] or (np.isnan(o[3]) and np.isnan(po.phong_pdf(n, wi, wr, kd, ks, ns)))
        s = po.sample_phong_ref(ctr, n, wr, kd, ks, ns)
        assert np.array_equal(s, o[4:], equal_nan=True), (r, s, o[4:])


def test_tone_mapping():
    tin, tout = g("tonemap_in.npy"), g("tonemap_out.npy")
    for r in range(tin.shape[0]):
        assert np.array_equal(po.tone_map(tin[r]), tout[r].astype(np.int32)), r


@pytest.mark.parametrize("mode,name", [(po.MODE_MIS, "sample_mis.npy"), (po.MODE_BRDF, "sample_brdf.npy"),
                                       (po.MODE_SHADE, "sample_shade.npy"),
                                       (po.MODE_SHADE_AREA, "sample_shade_area.npy")])
def test_integrator_refrng_replay_bitexact(scene, mode, name):
    """RefRng replay of main.cpp:269-494 (DFS order, stale-pdf quirk) vs the reference components."""
    cam = po.reference_camera(400, 300)
    gs = g(name)
    for r in range(gs.shape[0]):
        i, j, ctr, draws = int(gs[r, 0]), int(gs[r, 1]), int(gs[r, 2]), int(gs[r, 3])
        rgb, d = scene.shade_sample(cam, mode, po.RNG_REF, ctr, i, j)
        assert d == draws and np.array_equal(rgb, gs[r, 4:7]), (r, rgb, gs[r, 4:7], d, draws)
