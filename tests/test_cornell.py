"""Config C5: the Cornell + random-triangles stand-in (scenes/gen_cornell_random.py)
-- the BVH / memory stress case: 1,000,062 facets, 2 light triangles, the XML camera of
main.cpp:512-513 (no pull-back).  CPU tests check the generator and both loaders; GPU tests check
primary hits and rendered frames against the CPU oracle (uniform grid of Myobj.cpp:78-162) at the
full 1M-triangle size, with the tolerances of test_gpu_parity.py."""
import hashlib

import numpy as np
import pytest

from conftest import TIGHT_L2, TIGHT_PX, cornell_scene
import monte_carlo_path_tracing_amd as mcpt
from oracle import pyoracle as po

SEED = 20240430
L2_TOL = 1e-3
N_BIG = 1_000_000


def max_px_rel(g, c):
    """max over pixels of ||g_px - c_px|| / ||c_px|| (pixels black in both count 0)"""
    d = np.linalg.norm((g - c).reshape(-1, 3), axis=1)
    n = np.linalg.norm(c.reshape(-1, 3), axis=1)
    return float(np.max(np.where(n > 0, d / np.maximum(n, 1e-300), np.where(d > 0, np.inf, 0.0))))


def rel_l2(g, c):
    return float(np.linalg.norm(g - c) / max(np.linalg.norm(c), 1e-300))


def test_generator_is_deterministic_and_loads(tmp_path):
    import subprocess
    import sys
    from conftest import ROOT

    obj, xml = cornell_scene(300)
    d2 = tmp_path / "again"
    subprocess.run([sys.executable, str(ROOT / "scenes" / "gen_cornell_random.py"), "--triangles", "300", str(d2)],
                   check=True, capture_output=True)
    for name in ("cornell-random.obj", "cornell-random.mtl", "cornell-random.xml"):
        a = open(obj.replace("cornell-random.obj", name), "rb").read()
        b = open(d2 / name, "rb").read()
        assert hashlib.sha256(a).digest() == hashlib.sha256(b).digest(), name
    s = mcpt.Scene.load(obj, xml)
    assert (s.nfacets, s.nlights) == (5 * 12 + 2 + 300, 2)
    cam = s.camera()
    assert list(cam.eye) == [278.0, 273.0, -800.0] and list(cam.lookat) == [278.0, 273.0, -799.0]
    assert cam.dist_scale == 1.0 and (cam.width, cam.height) == (800, 600)
    # native loader == oracle loader, bit for bit
    o = po.Scene(obj, xml)
    v18, mat, lof, un = o.facets()
    a = s.arrays()
    assert np.array_equal(a["positions"], v18[:, :9]) and np.array_equal(a["normals"], v18[:, 9:])
    assert np.array_equal(a["material_id"], mat) and np.array_equal(a["unique_normal"], un)
    # the light faces down into the box and every facet is strictly inside the bbox
    assert (a["unique_normal"][a["light_facet"], 1] < 0).all()
    P = a["positions"].reshape(-1, 3)
    assert P.min() >= -1.0 and P.max() <= 557.0


@pytest.fixture(scope="module")
def big():
    obj, xml = cornell_scene(N_BIG)
    s = mcpt.Scene.load(obj, xml)
    o = po.Scene(obj, xml)
    cam = o.camera()
    e, _ = po.camera_ray(cam, 0, 0)
    o.build_grid(e)
    return s, o


def cams(W, H):
    g = mcpt.Camera()
    g.eye[:], g.lookat[:], g.up[:] = (278.0, 273.0, -800.0), (278.0, 273.0, -799.0), (0.0, 1.0, 0.0)
    g.fovy, g.dist_scale, g.width, g.height = 20.1143, 1.0, W, H
    c = po.Camera()
    c.eye[:], c.lookat[:], c.up[:] = (278.0, 273.0, -800.0), (278.0, 273.0, -799.0), (0.0, 1.0, 0.0)
    c.fovy, c.dist_scale, c.width, c.height = 20.1143, 1.0, W, H
    return g, c


@pytest.mark.gpu
def test_cornell_1m_primary_hits_vs_grid(big):
    s, o = big
    g, c = cams(160, 120)
    f, tbg = mcpt.primary_hits(s, g)
    bad = 0
    for i in range(0, 120, 3):
        for j in range(0, 160, 3):
            e, d = po.camera_ray(c, i, j)
            of, otbg = o.closest_hit(e, d)
            k = i * 160 + j
            if of != f[k] or (of >= 0 and not np.array_equal(otbg, tbg[k])):
                bad += 1
    assert bad == 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode,omode,spp", [("mis", po.MODE_MIS, 8), ("shade", po.MODE_SHADE, 8),
                                            ("brdf", po.MODE_BRDF, 32)])
def test_cornell_1m_render_parity(big, mode, omode, spp):
    s, o = big
    g, c = cams(64, 48)
    img, st = mcpt.render(s, g, spp, mode=mode, seed=SEED)
    ref, _ = o.render(c, omode, SEED, spp, nthreads=8)
    err, mx = rel_l2(img, ref), max_px_rel(img, ref)
    print("cornell-1M %s 64x48x%d rel L2 %.3e, max per-pixel %.3e, %.2f Msamples/s" % (
        mode, spp, err, mx, st.camera_samples / st.seconds / 1e6))
    assert np.isfinite(img).all() and (img >= 0).all() and ref.sum() > 0
    assert err <= L2_TOL and mx <= L2_TOL
    assert err <= TIGHT_L2 and mx <= TIGHT_PX, (err, mx)


@pytest.mark.gpu
def test_cornell_1m_full_size_pixel_subset(big):
    s, o = big
    g, c = cams(800, 600)
    img, st = mcpt.render(s, g, 8, mode="mis", seed=SEED)
    ref, _ = o.render(c, po.MODE_MIS, SEED, 8, stride=20, offset=7, nthreads=8)
    sub = (slice(7, None, 20), slice(7, None, 20))
    err, mx = rel_l2(img[sub], ref[sub]), max_px_rel(img[sub], ref[sub])
    print("cornell-1M mis 800x600x8 subset rel L2 %.3e, max per-pixel %.3e; %.2f Msamples/s" % (
        err, mx, st.camera_samples / st.seconds / 1e6))
    assert err <= L2_TOL and mx <= L2_TOL
    assert err <= TIGHT_L2 and mx <= TIGHT_PX, (err, mx)
