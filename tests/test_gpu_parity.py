"""GPU parity: the HIP path (through the C ABI of libmcpt_hip.so) against the CPU oracle and the
compiled reference's golden vectors.  Run on the MI355X box: `pytest -m gpu`.

Tolerances (BASELINE.json north star: <= 1e-3 relative per-pixel L2 vs the CPU path at a fixed
seed):
  * traversal / primary hits / random rays: facet EXACT, (t, beta, gamma) EXACT (the fp64 Cramer
    rule of Myobj.cpp:165-192 is evaluated in the same order with FMA contraction off);
  * light prep: the cheap culls are exact; the full stage is an fp64 reformulation (rsqrt
    normalisation, Van Oosterom-Strackee excess) equal up to rounding (weights_sum to ~1e-7
    relative, the reference's own cancellation); picks whose u*weights_sum lies inside that rounding
    band of a CDF boundary, and nodes whose survivor count could differ, are redone with the
    reference's literal formulas and order (k_prep_exact), so survivor counts and picks are EXACT;
  * rendered frames: relative L2 ||G - C|| / ||C|| <= 1e-3 over the whole W x H x 3 HDR frame
    (measured far below: the GPU and CPU differ only by fp64 rounding).
"""
import numpy as np
import pytest

from conftest import GOLDEN, SCENE_OBJ, SCENE_XML
import monte_carlo_path_tracing_amd as mcpt
from monte_carlo_path_tracing_amd import rng
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
SEED = 20240430
from conftest import NORTH_STAR_TOL as L2_TOL, TIGHT_L2, TIGHT_PX, TIGHT_PX_FRAME  # noqa: E402


@pytest.fixture(scope="module")
def scene():
    return mcpt.Scene.load(SCENE_OBJ, SCENE_XML)


@pytest.fixture(scope="module")
def oscene():
    s = po.Scene(SCENE_OBJ, SCENE_XML)
    e, _ = po.camera_ray(po.reference_camera(400, 300), 0, 0)
    s.build_grid(e)
    return s


def rel_l2(g, c):
    return float(np.linalg.norm(g - c) / max(np.linalg.norm(c), 1e-300))


def max_px_rel(g, c):
    """max over pixels of ||g_px - c_px|| / ||c_px|| (pixels black in both count 0)"""
    d = np.linalg.norm((g - c).reshape(-1, 3), axis=1)
    n = np.linalg.norm(c.reshape(-1, 3), axis=1)
    return float(np.max(np.where(n > 0, d / np.maximum(n, 1e-300), np.where(d > 0, np.inf, 0.0))))


def test_primary_hit_map_vs_reference(scene):
    f, tbg = mcpt.primary_hits(scene, mcpt.Camera.reference(400, 300))
    gp = np.load(GOLDEN / "primary_400x300.npy")
    assert np.array_equal(f, gp[:, 0].astype(np.int32))
    hit = f >= 0
    assert np.array_equal(tbg[hit], gp[hit, 1:])


def brute_force_hits(scene_arrays, rin, light_only):
    """Closest hit over ALL facets with the reference's fp64 Cramer rule (Myobj.cpp:165-192)."""
    P = scene_arrays["positions"].astype(np.float64).reshape(-1, 3, 3)
    a, b, c = P[:, 0], P[:, 1], P[:, 2]
    is_light = np.zeros(len(P), bool)
    is_light[scene_arrays["light_facet"]] = True

    def det(x, y, z):
        cr = np.stack([x[..., 1] * y[..., 2] - x[..., 2] * y[..., 1], x[..., 2] * y[..., 0] - x[..., 0] * y[..., 2],
                       x[..., 0] * y[..., 1] - x[..., 1] * y[..., 0]], -1)
        return ((0 + cr[..., 0] * z[..., 0]) + cr[..., 1] * z[..., 1]) + cr[..., 2] * z[..., 2]

    out = np.full(len(rin), -1)
    ab, ac = a - b, a - c
    for r in range(len(rin)):
        ro, rd, ex = rin[r, :3], np.broadcast_to(rin[r, 3:6], a.shape), int(rin[r, 6])
        ar = a - ro
        dA = det(ab, ac, rd)
        with np.errstate(all="ignore"):
            be, ga, t = det(ar, ac, rd) / dA, det(ab, ar, rd) / dA, det(ab, ac, ar) / dA
        ok = (np.abs(dA) >= 1e-8) & ~((be < 0) | (ga < 0) | (be + ga > 1) | (t < 0) | (np.abs(t) < 1e-8))
        if ex >= 0:
            ok[ex] = False
        if light_only:
            ok &= is_light
        if ok.any():
            out[r] = int(np.argmin(np.where(ok, t, np.inf)))
    return out


@pytest.mark.parametrize("light_only,name", [(False, "rays_hit.npy"), (True, "rays_lighthit.npy")])
def test_random_rays_vs_reference(scene, light_only, name):
    """Exact match with the reference grid, except rays whose origin rounds to just outside the
    scene bbox (on a bbox-minimum face): the reference's DDA starts in cell -1 and returns no hit
    (the grid "crack" of SURVEY.md §0 item 10 / Myobj.cpp:336-342,405).  Those rays (37/12000, all
    from back faces of the floor/backdrop boxes, unreachable from the camera) must match the
    brute-force closest hit instead."""
    rin, gold = np.load(GOLDEN / "rays_in.npy"), np.load(GOLDEN / name)
    bb = np.load(GOLDEN / "grid_bbox.npy")[0]
    crack = (np.floor((rin[:, :3] - bb[[0, 2, 4]]) * (1.0 / bb[6])) < 0).any(axis=1)
    f, tbg = mcpt.closest_hit(scene, rin[:, :3], rin[:, 3:6], rin[:, 6].astype(np.int32), light_only)
    ok = ~crack
    assert np.array_equal(f[ok], gold[ok, 0].astype(np.int32))
    hit = ok & (f >= 0)
    assert np.array_equal(tbg[hit], gold[hit, 1:])
    bf = brute_force_hits(scene.arrays(), rin[crack], light_only)
    assert np.array_equal(f[crack], bf)
    print("%d/%d rays hit the reference grid's bbox crack; GPU == brute force there" % (crack.sum(), len(rin)))


@pytest.mark.parametrize("light_only", [False, True])
def test_edge_and_vertex_rays_vs_brute_force(scene, light_only):
    """Rays aimed exactly at triangle vertices, edge points and points a few ulps off the edges
    (from near and far origins, including grazing ones): the traversal's fp32 triangle pre-test
    (tri_filter, render.hip) only skips triangles the reference's fp64 test (Myobj.cpp:165-192)
    surely rejects, so the closest hit equals the fp64 brute force over every facet, bit for bit."""
    arr = scene.arrays()
    P = arr["positions"].astype(np.float64).reshape(-1, 3, 3)
    rng = np.random.default_rng(7)
    n = 3000
    tri = rng.integers(0, len(P), n)
    if light_only:
        tri = np.asarray(arr["light_facet"])[rng.integers(0, len(arr["light_facet"]), n)]
    kind = rng.integers(0, 3, n)
    w = rng.random((n, 3))
    w[kind == 0] = np.eye(3)[rng.integers(0, 3, (kind == 0).sum())]  # a vertex
    e = rng.integers(0, 3, n)
    w[(kind == 1), e[kind == 1]] = 0.0  # a point on an edge
    w /= w.sum(axis=1, keepdims=True)
    target = np.einsum("nk,nkc->nc", w, P[tri])
    target *= 1.0 + rng.choice([0.0, 1e-15, -1e-15, 1e-12, -1e-12], (n, 1))
    lo, hi = P.reshape(-1, 3).min(axis=0), P.reshape(-1, 3).max(axis=0)
    ro = lo + rng.random((n, 3)) * (hi - lo)
    near = rng.random(n) < 0.3
    ro[near] = target[near] + rng.normal(0, 0.05, (near.sum(), 3))
    rd = target - ro
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    ex = np.where(rng.random(n) < 0.2, tri, -1).astype(np.int32)
    f, _ = mcpt.closest_hit(scene, ro, rd, ex, light_only)
    bf = brute_force_hits(arr, np.concatenate([ro, rd, ex[:, None]], axis=1), light_only)
    assert np.array_equal(f, bf)
    print("%d/%d edge/vertex rays hit" % ((f >= 0).sum(), n))


def test_light_prep_vs_reference_and_oracle(scene, oscene):
    pin, pout = np.load(GOLDEN / "prep_in.npy"), np.load(GOLDEN / "prep_out.npy")
    u = np.array([rng.counter_uniform(SEED, k, 0, 1, 1) for k in range(len(pin))])
    ws, cnt, pick = mcpt.light_prep(scene, pin[:, :3], pin[:, 3:6], u)
    gcnt = pout[:, 1].astype(np.int32)
    # survivor counts EXACT (nodes with a full-stage cull or a near-degenerate sliver go through the
    # literal chain of k_prep_exact)
    assert np.array_equal(cnt, gcnt), np.nonzero(cnt != gcnt)
    rel = np.abs(ws - pout[:, 0]) / np.maximum(np.abs(pout[:, 0]), 1e-300)
    print("light prep: weights_sum max rel err %.2e" % rel[pout[:, 0] > 0].max())
    # the reference sums alpha+beta+gamma-pi (cancellation for tiny triangles); 1e-6 covers that
    assert np.allclose(ws, pout[:, 0], rtol=1e-6, atol=1e-300)
    opick = np.array([int(oscene.light_sample_u(pin[k, :3], pin[k, 3:6], u[k], 0.5, 0.5)[0]) for k in range(len(pin))])
    assert np.array_equal(pick, opick), np.nonzero(pick != opick)  # picks EXACT


def test_light_prep_exact_fallback_is_the_reference(scene, oscene):
    """k_prep_exact alone (the fallback of picks inside the band) on the 2 000 golden points: the
    reference's literal chain and index-order sum (Mylight.cpp:335-418) with a correctly rounded acos
    (csrc/acos_cr.h), its survivor counts and the oracle's counter-RNG picks EXACT, also at u next to a
    cumulative boundary.  weights_sum is bit-identical wherever glibc's acos (the oracle's) is correctly
    rounded on all of the point's survivors: glibc rounds ~5e-4 of arguments the other way
    (tools/acos_cr_check.py), so ~0.1% of the light weights differ in their last bits and ~20% of the
    points' sums (~900 survivors each) slightly: sA = alpha + beta + gamma - pi cancels, so one angle's
    ulp (4.4e-16) moves a small triangle's weight by 4.4e-16 / sA relative (measured <= 4e-12 on the sums;
    asserted <= 1e-10)."""
    pin, pout = np.load(GOLDEN / "prep_in.npy"), np.load(GOLDEN / "prep_out.npy")
    u = np.array([rng.counter_uniform(SEED, k, 0, 1, 1) for k in range(len(pin))])
    ws, cnt, pick = mcpt.debug_light_prep_exact(scene, pin[:, :3], pin[:, 3:6], u)
    same = ws == pout[:, 0]
    rel = np.abs(ws - pout[:, 0]) / np.maximum(np.abs(pout[:, 0]), 1e-300)
    print("exact fallback: weights_sum bit-identical on %d/%d points, max rel diff of the rest %.2e" % (
        same.sum(), len(pin), rel.max()))
    assert same.mean() >= 0.7 and rel.max() <= 1e-10, (np.nonzero(~same)[0][:10], rel[~same][:5])
    assert np.array_equal(cnt, pout[:, 1].astype(np.int32))
    opick = np.array([int(oscene.light_sample_u(pin[k, :3], pin[k, 3:6], u[k], 0.5, 0.5)[0]) for k in range(len(pin))])
    assert np.array_equal(pick, opick)
    # targets a hair below / above a cumulative boundary of the oracle's own sums: the pick flips
    # exactly where the reference's does
    sel = np.nonzero((pout[:, 1] >= 4) & same)[0][:200]  # sums bit-identical: boundaries coincide
    ub, expect = [], []
    for k in sel:
        wsum, idx, w = oscene.light_prep(pin[k, :3], pin[k, 3:6])
        c = np.cumsum(w)  # sequential, the oracle's order
        j = len(c) // 2
        for uu in (np.nextafter(c[j] / wsum, 0), c[j] / wsum, np.nextafter(c[j] / wsum, 1)):
            ub.append(uu)
            expect.append(int(oscene.light_sample_u(pin[k, :3], pin[k, 3:6], uu, 0.5, 0.5)[0]))
    xs = np.repeat(pin[sel, :3], 3, axis=0)
    ns = np.repeat(pin[sel, 3:6], 3, axis=0)
    _, _, pe = mcpt.debug_light_prep_exact(scene, xs, ns, np.array(ub))
    _, _, pr = mcpt.light_prep(scene, xs, ns, np.array(ub))
    print("boundary targets: exact %d/%d, renderer's prep %d/%d equal to the oracle" % (
        (pe == expect).sum(), len(ub), (pr == expect).sum(), len(ub)))
    assert np.array_equal(pe, expect) and np.array_equal(pr, expect)


def test_exact_pick_statistics(scene):
    """the exact-pick bookkeeping of a cached-root MIS render (mcpt_stats, ABI 2.1): some preps reach the
    per-chunk band test and some of those (plus ambiguous cached roots) the literal fallback, a small
    fraction of all shading nodes; the fp32 opt-in precision makes no exactness claim and runs none"""
    cam = mcpt.Camera.reference(200, 150)
    _, st = mcpt.render(scene, cam, 64, mode="mis", seed=SEED, device=0)
    print("200x150x64 MIS: %d shading nodes, %d band tests, %d exact preps, root cache build %.2f ms" % (
        st.shading_nodes, st.prep_band_nodes, st.prep_exact_nodes, 1e3 * st.cache_build_seconds))
    assert st.prep_band_nodes > 0 and st.prep_exact_nodes > 0
    assert st.prep_exact_nodes < 1e-2 * st.shading_nodes and st.cache_build_seconds > 0
    _, s32 = mcpt.render(scene, cam, 64, mode="mis", seed=SEED, device=0, flags=mcpt.RENDER_PRECISION_FP32)
    assert s32.prep_exact_nodes == 0 and s32.prep_band_nodes == 0


OMODE = {"mis": po.MODE_MIS, "brdf": po.MODE_BRDF, "shade": po.MODE_SHADE, "shade_area": po.MODE_SHADE_AREA}


def _render_pair(scene, oscene, W, H, spp, mode, stride=1, nthreads=8):
    cam = mcpt.Camera.reference(W, H)
    g, st = mcpt.render(scene, cam, spp, mode=mode, seed=SEED)
    ocam = po.reference_camera(W, H)
    c, _ = oscene.render(ocam, OMODE[mode], SEED, spp, stride=stride,
                         nthreads=nthreads)
    return g, c, st


@pytest.mark.parametrize("mode,spp", [("mis", 8), ("brdf", 32), ("shade", 8), ("shade_area", 16)])
def test_render_parity_small(scene, oscene, mode, spp):
    g, c, st = _render_pair(scene, oscene, 80, 60, spp, mode)
    err, mx = rel_l2(g, c), max_px_rel(g, c)
    print("%s 80x60x%d rel L2 %.3e, max per-pixel %.3e, device %.4fs" % (mode, spp, err, mx, st.seconds))
    assert np.isfinite(g).all() and (g >= 0).all()
    assert err <= L2_TOL and mx <= L2_TOL
    assert err <= TIGHT_L2 and mx <= TIGHT_PX, (err, mx)


@pytest.mark.parametrize("mode,spp", [("mis", 16), ("brdf", 64), ("shade", 16), ("shade_area", 32)])
def test_render_parity_full_size_pixel_subset(scene, oscene, mode, spp):
    """BASELINE size 800x600: the counter RNG is keyed per pixel, so the oracle renders every 20th
    pixel in x and y (SURVEY.md §8(d) stratified subset) and those pixels must match."""
    cam = mcpt.Camera.reference(800, 600)
    g, st = mcpt.render(scene, cam, spp, mode=mode, seed=SEED)
    c, _ = oscene.render(po.reference_camera(800, 600), OMODE[mode], SEED, spp,
                         stride=20, offset=7, nthreads=8)
    sub = (slice(7, None, 20), slice(7, None, 20))
    err, mx = rel_l2(g[sub], c[sub]), max_px_rel(g[sub], c[sub])
    print("%s 800x600x%d subset rel L2 %.3e, max per-pixel %.3e; %.2f Msamples/s" % (
        mode, spp, err, mx, st.camera_samples / st.seconds / 1e6))
    assert np.isfinite(g).all() and (g >= 0).all()
    assert err <= L2_TOL and mx <= L2_TOL
    assert err <= TIGHT_L2 and mx <= TIGHT_PX, (err, mx)
    assert g.mean() > 0


def test_c3_full_frame_vs_oracle(scene, oscene):
    """C3's frame (800x600, MIS with the reference's stale light pdf) in full, every pixel against the
    oracle at the same seed: 2 spp (960 000 camera samples, the same counter-RNG samples on both sides;
    the oracle on 16 host threads) -- relative L2 and every pixel <= 1e-3 (north star)."""
    cam = mcpt.Camera.reference(800, 600)
    g, st = mcpt.render(scene, cam, 2, mode="mis", seed=SEED)
    c, _ = oscene.render(po.reference_camera(800, 600), po.MODE_MIS, SEED, 2, nthreads=16)
    err, mx = rel_l2(g, c), max_px_rel(g, c)
    print("mis 800x600x2 full frame: rel L2 %.3e, max per-pixel %.3e; %d shading nodes, %d exact preps" % (
        err, mx, st.shading_nodes, st.prep_exact_nodes))
    assert np.isfinite(g).all() and (g >= 0).all() and c.sum() > 0
    assert err <= L2_TOL and mx <= L2_TOL
    assert err <= TIGHT_L2 and mx <= TIGHT_PX_FRAME, (err, mx)


@pytest.mark.parametrize("mode,spp", [("brdf", 4), ("shade_area", 2)])
def test_full_frame_other_modes_vs_oracle(scene, oscene, mode, spp):
    """C2's frame (800x600 BRDF-only) and shade() with uniform-area light sampling at 800x600 in full, every
    pixel against the oracle at the same seed (the counter-RNG samples on both sides; the oracle on 16 host
    threads, ~10 s): relative L2 and every pixel <= 1e-3 (north star), and what the build achieves
    (tests/conftest.py).  shade()'s spherical sampler stays on the stride-20 subset above (its oracle frame
    would take ~1 min)."""
    cam = mcpt.Camera.reference(800, 600)
    g, st = mcpt.render(scene, cam, spp, mode=mode, seed=SEED)
    c, _ = oscene.render(po.reference_camera(800, 600), OMODE[mode], SEED, spp, nthreads=16)
    err, mx = rel_l2(g, c), max_px_rel(g, c)
    print("%s 800x600x%d full frame: rel L2 %.3e, max per-pixel %.3e; %d shading nodes" % (
        mode, spp, err, mx, st.shading_nodes))
    assert np.isfinite(g).all() and (g >= 0).all() and c.sum() > 0
    assert err <= L2_TOL and mx <= L2_TOL
    assert err <= TIGHT_L2 and mx <= TIGHT_PX_FRAME, (err, mx)


@pytest.mark.parametrize("W,H,spp", [(80, 60, 8), (800, 600, 16)])
def test_mis_fresh_pdf_flag_vs_oracle(scene, oscene, W, H, spp):
    """MCPT_RENDER_FRESH_PDF (the node's own light pdf, not the reference's stale sampler state,
    main.cpp:443 vs :487) against the oracle's ORC_FLAG_FRESH_PDF; the default (stale) render must
    differ from it where light branches recurse"""
    cam = mcpt.Camera.reference(W, H)
    g, _ = mcpt.render(scene, cam, spp, mode="mis", seed=SEED, flags=mcpt.RENDER_FRESH_PDF)
    stride = 1 if W < 200 else 20
    off = 0 if stride == 1 else 7
    c, _ = oscene.render(po.reference_camera(W, H), po.MODE_MIS | po.FLAG_FRESH_PDF, SEED, spp, stride=stride,
                         offset=off, nthreads=8)
    sub = (slice(off, None, stride), slice(off, None, stride))
    err, mx = rel_l2(g[sub], c[sub]), max_px_rel(g[sub], c[sub])
    print("fresh-pdf MIS %dx%dx%d rel L2 %.3e, max per-pixel %.3e" % (W, H, spp, err, mx))
    assert err <= L2_TOL and mx <= L2_TOL
    assert err <= TIGHT_L2 and mx <= TIGHT_PX, (err, mx)
    d, _ = mcpt.render(scene, cam, spp, mode="mis", seed=SEED)
    assert rel_l2(d[sub], g[sub]) > 1e-9


@pytest.mark.parametrize("mode,W,H,spp", [("mis", 80, 60, 8), ("mis", 800, 600, 16), ("shade", 800, 600, 16)])
def test_precision_fp32_vs_oracle(scene, oscene, mode, W, H, spp):
    """MCPT_RENDER_PRECISION_FP32 (opt-in): packed-fp32 light weights,
    summed in fp64.  Tolerance: frame relative L2 <= 1e-3 against the fp64 oracle (the north star's);
    per pixel, a pick whose u * weights_sum lies within ~1e-6 of a CDF boundary may take the adjacent
    light triangle (measured ~1e-4 of prep nodes), so <= 1% of pixels may exceed 1e-3 and none 0.5."""
    cam = mcpt.Camera.reference(W, H)
    g, _ = mcpt.render(scene, cam, spp, mode=mode, seed=SEED, flags=mcpt.RENDER_PRECISION_FP32)
    d, _ = mcpt.render(scene, cam, spp, mode=mode, seed=SEED)
    stride = 1 if W < 200 else 20
    off = 0 if stride == 1 else 7
    c, _ = oscene.render(po.reference_camera(W, H), OMODE[mode], SEED, spp, stride=stride, offset=off, nthreads=8)
    sub = (slice(off, None, stride), slice(off, None, stride))
    err, mx = rel_l2(g[sub], c[sub]), max_px_rel(g[sub], c[sub])
    dn = np.linalg.norm((g[sub] - c[sub]).reshape(-1, 3), axis=1)
    cn = np.linalg.norm(c[sub].reshape(-1, 3), axis=1)
    frac = float(np.mean(dn > 1e-3 * np.maximum(cn, 1e-300)))
    print("fp32 light prep %s %dx%dx%d: rel L2 vs oracle %.3e (fp64 GPU %.3e), max per-pixel %.3e, "
          "pixels > 1e-3: %.4f; fp32 vs fp64 GPU frame %.3e" % (
              mode, W, H, spp, err, rel_l2(d[sub], c[sub]), mx, frac, rel_l2(g, d)))
    assert np.isfinite(g).all() and (g >= 0).all()
    assert err <= L2_TOL
    assert frac <= 0.01 and mx <= 0.5
    assert rel_l2(g, d) > 0  # the flag changes the arithmetic


def test_sample_range_split_is_invariant(scene):
    """Sharding by sample range (multi-GPU, sequential calls) gives the same frame up to fp64 order."""
    cam = mcpt.Camera.reference(64, 48)
    full, _ = mcpt.render(scene, cam, 6, seed=SEED)
    part = np.zeros_like(full)
    for a, b in [(0, 1), (1, 4), (4, 6)]:
        mcpt.render(scene, cam, 6, seed=SEED, sample_range=(a, b), out=part)
    assert rel_l2(part, full) < 1e-12


def test_batching_is_invariant(scene):
    cam = mcpt.Camera.reference(64, 48)
    a, _ = mcpt.render(scene, cam, 4, seed=SEED, samples_per_launch=1)
    b, _ = mcpt.render(scene, cam, 4, seed=SEED, samples_per_launch=4)
    assert rel_l2(a, b) < 1e-12


def test_fused_cull_switch_changes_no_pick(scene):
    """MCPT_DEBUG_FUSED_CULL (the round-6 A/B of the fused cull, prep variant 8: cheap stages inside k_prep_pk2, one
    wave per node) gives the renderer the same candidates, weights and picks as the default split cull, so the same
    shading nodes and the same frame up to fp64 atomic order; a debug switch must not change the image"""
    cam = mcpt.Camera.reference(96, 72)
    a, sa = mcpt.render(scene, cam, 4, seed=SEED)
    b, sb = mcpt.render(scene, cam, 4, seed=SEED, flags=mcpt.DEBUG_FUSED_CULL)
    assert sa.shading_nodes == sb.shading_nodes and sa.prep_full_nodes == sb.prep_full_nodes
    assert sa.light_evals_candidates == sb.light_evals_candidates
    assert rel_l2(a, b) < 1e-12


def test_seed_changes_image(scene):
    cam = mcpt.Camera.reference(64, 48)
    a, _ = mcpt.render(scene, cam, 2, seed=1)
    b, _ = mcpt.render(scene, cam, 2, seed=2)
    assert rel_l2(a, b) > 1e-3


def test_invalid_options_fail_loudly(scene):
    cam = mcpt.Camera.reference(8, 8)
    with pytest.raises(mcpt.MCPTError):
        mcpt.render(scene, cam, 0)
    with pytest.raises(mcpt.MCPTError):
        mcpt.render(scene, cam, 4, sample_range=(2, 9))


def test_render_device_buffer_with_torch(scene):
    torch = pytest.importorskip("torch")
    cam = mcpt.Camera.reference(64, 48)
    fb = torch.zeros((48, 64, 3), dtype=torch.float64, device="cuda")
    st = mcpt.render_device(scene, cam, 4, fb.data_ptr(), seed=SEED, device=torch.cuda.current_device())
    torch.cuda.synchronize()
    host, _ = mcpt.render(scene, cam, 4, seed=SEED)
    assert rel_l2(fb.cpu().numpy(), host) < 1e-12
    assert st.camera_samples == 64 * 48 * 4


@pytest.mark.parametrize("small_lights", [False, True])
def test_no_backface_stats_flag(scene, small_lights, tmp_path):
    """mcpt_render_opts.flags = MCPT_RENDER_NO_BACKFACE_STATS (bench.py's timed steps): the same
    image and work; only the light-side cull statistic is folded into the plane-cull count -- for
    the split light cull (Veach) and the lane-per-node prep of small light sets (N_L <= 64) alike."""
    torch = pytest.importorskip("torch")
    cam = mcpt.Camera.reference(64, 48)
    if small_lights:
        import scenegen
        scene = mcpt.Scene.load(*scenegen.occluded_room(str(tmp_path)))
        cam = scene.camera()
        cam.width, cam.height = 64, 48
    dev = torch.cuda.current_device()
    fa = torch.zeros((48, 64, 3), dtype=torch.float64, device="cuda")
    fb = torch.zeros_like(fa)
    a = mcpt.render_device(scene, cam, 8, fa.data_ptr(), seed=SEED, device=dev).as_dict()
    b = mcpt.render_device(scene, cam, 8, fb.data_ptr(), seed=SEED, device=dev,
                           flags=mcpt.RENDER_NO_BACKFACE_STATS).as_dict()
    torch.cuda.synchronize()
    assert rel_l2(fb.cpu().numpy(), fa.cpu().numpy()) < 1e-12  # fp64 atomic accumulation order only
    assert a["light_evals_culled_backface"] > 0 and b["light_evals_culled_backface"] == 0
    assert b["light_evals_culled_plane"] == a["light_evals_culled_plane"] + a["light_evals_culled_backface"]
    for k in ("light_evals_total", "light_evals_candidates", "light_evals_survived", "prep_full_nodes", "rays"):
        assert a[k] == b[k], k
    with pytest.raises(mcpt.MCPTError, match="flags"):
        mcpt.render_device(scene, cam, 8, fb.data_ptr(), seed=SEED, device=dev, flags=1 << 12)


def test_progress_callback_and_cancel(scene):
    """mcpt_render_opts.progress (the reference's per-row progress, main.cpp:539-592): monotone
    reports ending at the call's total; a truthy return cancels with an error."""
    cam = mcpt.Camera.reference(64, 48)
    seen = []
    img, st = mcpt.render(scene, cam, 16, seed=SEED, samples_per_launch=2,
                          progress=lambda done, total: seen.append((done, total)) and False)
    total = 64 * 48 * 16
    assert seen and all(t == total for _, t in seen)
    assert [d for d, _ in seen] == sorted(d for d, _ in seen) and seen[-1][0] == total
    ref, _ = mcpt.render(scene, cam, 16, seed=SEED, samples_per_launch=2)
    assert rel_l2(img, ref) < 1e-12  # fp64 atomic accumulation order only
    calls = []
    with pytest.raises(mcpt.MCPTError, match="cancelled"):
        mcpt.render(scene, cam, 16, seed=SEED, samples_per_launch=2, progress=lambda d, t: calls.append(d) or True)
    assert len(calls) == 1
