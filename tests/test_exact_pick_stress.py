"""The exact light pick beyond the Veach stand-in (reference Mylight.cpp:322-482).

The renderer's prep weighs light triangles with its fp64 Van Oosterom-Strackee form and redoes a pick
with the reference's literal chain (k_prep_exact) whenever its slack lies inside the ambiguity band
(DESIGN.md §4.3.3), whose constants were calibrated on the stand-in.  These scenes stress it
(tests/scenegen.py STRESS):
  * sphmix  -- spheres of 8x4 .. 64x32 segments, N_L = 5200 > 4096 (roots take the wave-per-root
               k_prep_pick, 82 chunks);
  * slivers -- light blinds seen edge-on from the floor next to them and a panel 2 degrees off the
               vertical (spherical slivers, where the reference's sA is decided by its last bits);
  * tinyfar -- tiny lights (radius 1e-2 .. 1e-6) 20-90 units away: the reference's sA is mostly its
               own rounding, edge culls fire;
  * dense   -- one sphere of 14 160 triangles > 7680: the LDS-queue prep (k_prep) without candidate
               words and without root cache (k_prep_band must not read stale words).
On each: 2 000 surface points through mcpt_light_prep vs the oracle -- survivor counts and picks EXACT,
weights_sum within 1e-3 relative (the reference's own rounding noise; the literal fallback's nodes are
bit-exact up to glibc's misrounded acos) -- and a 64x48 MIS frame vs the oracle at the same seed:
relative L2 <= 1e-3 and every pixel <= 1e-3 (north star).  tools/band_margin_study.py --stress reports
each scene's band margin (round 6, 8 seeds: veach x10, sphmix x17, slivers x2.7 (x2.1 over 32 seeds), dense x24,
soup x111; tinyfar: the band always covers the pick, every node takes the literal fallback);
tests/test_band_margin.py checks the margin on CPU.
"""
import numpy as np
import pytest

import monte_carlo_path_tracing_amd as mcpt
from monte_carlo_path_tracing_amd import rng
from oracle import pyoracle as po
import scenegen
from conftest import TIGHT_L2, TIGHT_PX

pytestmark = pytest.mark.gpu
SEED = 20240430
TOL = 1e-3


def rel_l2(g, c):
    return float(np.linalg.norm(g - c) / max(np.linalg.norm(c), 1e-300))


def max_px_rel(g, c):
    d = np.linalg.norm((g - c).reshape(-1, 3), axis=1)
    n = np.linalg.norm(c.reshape(-1, 3), axis=1)
    return float(np.max(np.where(n > 0, d / np.maximum(n, 1e-300), np.where(d > 0, np.inf, 0.0))))


def surface_points(osc, m, seed=3):
    """m shading points area-sampled over the non-light facets (interpolated normals), and their u"""
    v, _, light_of, _ = osc.facets()
    P = v[:, :9].astype(np.float64).reshape(-1, 3, 3)
    N = v[:, 9:].astype(np.float64).reshape(-1, 3, 3)
    r = np.random.default_rng(seed)
    nonlight = np.nonzero(light_of < 0)[0]
    area = 0.5 * np.linalg.norm(np.cross(P[nonlight, 1] - P[nonlight, 0], P[nonlight, 2] - P[nonlight, 0]), axis=1)
    fs = nonlight[r.choice(len(nonlight), m, p=area / area.sum())]
    b = r.random((m, 2))
    sw = b.sum(1) > 1
    b[sw] = 1 - b[sw]
    X = (1 - b.sum(1))[:, None] * P[fs, 0] + b[:, :1] * P[fs, 1] + b[:, 1:] * P[fs, 2]
    Nn = (1 - b.sum(1))[:, None] * N[fs, 0] + b[:, :1] * N[fs, 1] + b[:, 1:] * N[fs, 2]
    Nn /= np.linalg.norm(Nn, axis=1)[:, None]
    u = np.array([rng.counter_uniform(SEED, k, 0, 1, 1) for k in range(m)])
    return X, Nn, u


@pytest.fixture(scope="module")
def scenes(tmp_path_factory):
    d = tmp_path_factory.mktemp("stress")
    out = {}
    for name, (make, nl) in scenegen.STRESS.items():
        obj, xml = make(str(d / name))
        out[name] = (obj, xml, nl)
    return out


@pytest.mark.parametrize("name", sorted(scenegen.STRESS))
def test_light_prep_picks_exact(scenes, name):
    obj, xml, nl = scenes[name]
    s = mcpt.Scene.load(obj, xml)
    assert s.nlights == nl
    osc = po.Scene(obj, xml)
    X, N, u = surface_points(osc, 2000)
    ws, cnt, pick = mcpt.light_prep(s, X, N, u)
    ows = np.zeros(len(X))
    ocnt = np.zeros(len(X), np.int32)
    opick = np.zeros(len(X), np.int32)
    for k in range(len(X)):
        w, idx, _ = osc.light_prep(X[k], N[k])
        ows[k], ocnt[k] = w, len(idx)
        opick[k] = int(osc.light_sample_u(X[k], N[k], u[k], 0.5, 0.5)[0])
    lit = ocnt > 0
    rel = np.abs(ws - ows) / np.maximum(np.abs(ows), 1e-300)
    print("%s: N_L %d, %d of %d points see lights; counts equal %d, picks equal %d; weights_sum max rel diff %.2e" % (
        name, nl, lit.sum(), len(X), (cnt == ocnt).sum(), (pick == opick).sum(), rel[lit].max() if lit.any() else 0))
    assert lit.sum() >= 200
    assert np.array_equal(cnt, ocnt), np.nonzero(cnt != ocnt)[0][:10]
    assert np.array_equal(pick, opick), np.nonzero(pick != opick)[0][:10]
    assert rel[lit].max() <= TOL


@pytest.mark.parametrize("name", sorted(scenegen.STRESS))
def test_mis_frame_vs_oracle(scenes, name):
    obj, xml, _ = scenes[name]
    s = mcpt.Scene.load(obj, xml)
    cam = s.camera()
    cam.width, cam.height = 64, 48
    img, st = mcpt.render(s, cam, 8, mode="mis", seed=SEED)
    osc = po.Scene(obj, xml)
    oc = osc.camera()
    oc.width, oc.height = 64, 48
    e, _ = po.camera_ray(oc, 0, 0)
    osc.build_grid(e)
    ref, _ = osc.render(oc, po.MODE_MIS, SEED, 8, nthreads=16)
    l2, mx = rel_l2(img, ref), max_px_rel(img, ref)
    print("%s 64x48x8 MIS: rel L2 %.3e, max per-pixel %.3e; %d shading nodes, %d band tests, %d exact preps" % (
        name, l2, mx, st.shading_nodes, st.prep_band_nodes, st.prep_exact_nodes))
    assert np.isfinite(img).all() and ref.sum() > 0
    assert l2 <= TOL and mx <= TOL
    assert l2 <= TIGHT_L2 and mx <= TIGHT_PX, (l2, mx)  # what the build achieves (tests/conftest.py)


@pytest.mark.parametrize("name", ["veach"] + sorted(scenegen.STRESS))
def test_cull_chunk_classes_change_no_candidate(scenes, name):
    """The cull's chunk classes (a 64-light chunk wholly above / below a node's tangent
    plane skips the plane test / the whole chunk) and the node order that makes them wave-uniform change
    work only: 20 000 points area-sampled on both sides of every non-light facet (above, below and
    straddling chunks all occur), prep variant 17 (ordered, classes on) vs 18 (the plain cull) --
    weights_sum and picks bit-identical.  Also prep variant 8 (the cheap stages inside k_prep_pk2, one wave per
    node, chunks below the tangent plane skipped: MCPT_DEBUG_FUSED_CULL's form) -- the same candidates in the
    same order, so the same bits."""
    if name == "veach":
        from conftest import SCENE_OBJ as obj, SCENE_XML as xml
    else:
        obj, xml, _ = scenes[name]
    s = mcpt.Scene.load(obj, xml)
    if s.nlights <= 64 or s.nlights > 7680:  # k_prep_lane / k_prep: no candidate words, no classes
        pytest.skip("prep without the split cull")
    X, N, u = surface_points(po.Scene(obj, xml), 20000, seed=11)
    _, ws17, p17 = mcpt.debug_prep_bench(s, X, N, u, variant=17, iters=1)
    _, ws18, p18 = mcpt.debug_prep_bench(s, X, N, u, variant=18, iters=1)
    _, ws8, p8 = mcpt.debug_prep_bench(s, X, N, u, variant=8, iters=1)
    assert (ws17 > 0).sum() >= 2000
    assert np.array_equal(ws17.view(np.int64), ws18.view(np.int64))
    assert np.array_equal(p17, p18)
    assert np.array_equal(ws17.view(np.int64), ws8.view(np.int64))
    assert np.array_equal(p17, p8)


def test_cull_order_at_scale_changes_no_candidate():
    """The cull's node order at the size of a real generation's share (10^6 nodes: ~500 blocks of the
    order kernels, bucket counters under contention): prep variant 17 vs 18 bit-identical on the
    stand-in (both sides of every facet, so every chunk class occurs)."""
    from conftest import SCENE_OBJ, SCENE_XML
    s = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    X, N, u = surface_points(po.Scene(SCENE_OBJ, SCENE_XML), 1 << 20, seed=17)
    _, ws17, p17 = mcpt.debug_prep_bench(s, X, N, u, variant=17, iters=1)
    _, ws18, p18 = mcpt.debug_prep_bench(s, X, N, u, variant=18, iters=1)
    assert (ws17 > 0).sum() >= 100000
    assert np.array_equal(ws17.view(np.int64), ws18.view(np.int64))
    assert np.array_equal(p17, p18)


def test_deferred_duplicate_roots_change_nothing(scenes):
    """k_prep_exact defers a root whose pixel another wave of the same launch is computing to a follow-up launch
    that only searches the stored literal sums (MCPT_EXACT_DEFER, round 6).  On tinyfar every pick is inside the
    band, so every root takes the literal fallback and most of a pixel's roots share a launch: the render with the
    deferral and the one that recomputes every root (MCPT_DEBUG_NO_EXACT_DEFER) list the same nodes, shade the same
    nodes and give the same frame up to fp64 atomic order."""
    obj, xml, _ = scenes["tinyfar"]
    s = mcpt.Scene.load(obj, xml)
    cam = s.camera()
    cam.width, cam.height = 32, 24
    a, sa = mcpt.render(s, cam, 64, mode="mis", seed=SEED)
    b, sb = mcpt.render(s, cam, 64, mode="mis", seed=SEED, flags=mcpt.DEBUG_NO_EXACT_DEFER)
    print("tinyfar 32x24x64: %d exact preps, %d cached roots" % (sa.prep_exact_nodes, sa.prep_cached_nodes))
    assert sa.prep_exact_nodes == sb.prep_exact_nodes and sa.prep_exact_nodes > 10000
    assert sa.shading_nodes == sb.shading_nodes and sa.prep_cached_nodes > 0
    assert rel_l2(a, b) < 1e-12 and max_px_rel(a, b) < 1e-10
