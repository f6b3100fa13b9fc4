"""Soundness of the traversal's fp32 triangle pre-test (tri_filter, render.hip) against the
reference's fp64 ray/triangle test (Myobj.cpp:165-192), on the host (no GPU): a triangle the
pre-test drops must be one the fp64 test rejects (or whose hit lies beyond the traversal's current
limit), and a "sure hit" must be one the fp64 test accepts, at a t no larger than the reported bound.
Cases aim rays at vertices, edges and points a few ulps off them, from near and grazing origins."""
import numpy as np
import pytest

import monte_carlo_path_tracing_amd as mcpt

FLT_MAX = np.finfo(np.float32).max


def fp64_test(tri, ro, rd):
    """tri_hit (device_math.h) / Myobj::intersect_with_triangle in numpy fp64, same operation order."""
    P = tri.astype(np.float64).reshape(-1, 3, 3)
    a, b, c = P[:, 0], P[:, 1], P[:, 2]

    def det(x, y, z):
        cr = np.stack([x[:, 1] * y[:, 2] - x[:, 2] * y[:, 1], x[:, 2] * y[:, 0] - x[:, 0] * y[:, 2],
                       x[:, 0] * y[:, 1] - x[:, 1] * y[:, 0]], -1)
        return ((0 + cr[:, 0] * z[:, 0]) + cr[:, 1] * z[:, 1]) + cr[:, 2] * z[:, 2]

    ab, ac, ar = a - b, a - c, a - ro
    dA = det(ab, ac, rd)
    with np.errstate(all="ignore"):
        be, ga, t = det(ar, ac, rd) / dA, det(ab, ar, rd) / dA, det(ab, ac, ar) / dA
    ok = (np.abs(dA) >= 1e-8) & ~((be < 0) | (ga < 0) | (be + ga > 1) | (t < 0) | (np.abs(t) < 1e-8))
    margin = np.minimum(np.minimum(be, ga), 1 - be - ga)  # barycentric distance to the nearest edge
    return ok, t, margin


def make_cases(rng, n):
    scale = 10.0 ** rng.uniform(-3, 1, (n, 1, 1))
    centre = rng.uniform(-20, 20, (n, 1, 3))
    tri = (centre + scale * rng.normal(size=(n, 3, 3))).astype(np.float32)
    kind = rng.integers(0, 4, n)
    w = rng.random((n, 3))
    w[kind == 0] = np.eye(3)[rng.integers(0, 3, (kind == 0).sum())]  # a vertex
    e = rng.integers(0, 3, n)
    w[kind == 1, e[kind == 1]] = 0.0  # an edge
    w[kind == 3] = rng.normal(size=((kind == 3).sum(), 3))  # anywhere in the plane (mostly outside)
    w /= w.sum(axis=1, keepdims=True)
    target = np.einsum("nk,nkc->nc", w, tri.astype(np.float64))
    target *= 1.0 + rng.choice([0.0, 1e-15, -1e-15, 1e-9, -1e-9, 1e-6, -1e-6], (n, 1))
    ro = target + rng.normal(size=(n, 3)) * 10.0 ** rng.uniform(-2, 1.5, (n, 1))
    graze = rng.random(n) < 0.2  # origins close to the triangle's plane
    nrm = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]).astype(np.float64)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True) + 1e-300
    off = ro - target
    ro[graze] = (target + off - nrm * np.einsum("nc,nc->n", off, nrm)[:, None] * (1 - 1e-4))[graze]
    rd = target - ro
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    return tri.reshape(n, 9), ro, rd


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tri_filter_is_sound(seed):
    rng = np.random.default_rng(seed)
    n = 200_000
    tri, ro, rd = make_cases(rng, n)
    ok, t, margin = fp64_test(tri, ro, rd)
    # the traversal's limit: none, or (for a third) just above / at / below this triangle's own t
    tlim = np.full(n, FLT_MAX, np.float32)
    sel = (rng.random(n) < 0.35) & ok
    tlim[sel] = (t[sel] * (1.0 + rng.choice([-1e-3, -1e-6, 0.0, 1e-6, 1e-3], sel.sum()))).astype(np.float32)
    verdict, tup = mcpt.debug_tri_filter(tri, ro, rd, tlim)
    dropped = verdict == 0
    # dropped: rejected by the fp64 test, or a hit strictly beyond the limit (not the closest)
    bad = dropped & ok & ~(t > tlim.astype(np.float64))
    assert not bad.any(), "pre-test dropped %d fp64-accepted triangles, e.g. %s" % (bad.sum(), np.flatnonzero(bad)[:5])
    sure = verdict == 2
    assert not (sure & ~ok).any(), "a sure hit the fp64 test rejects"
    assert (t[sure] <= tup[sure].astype(np.float64)).all(), "a sure hit's t above its bound"
    # and it is a filter: clear misses and clear hits (1e-2 of the triangle away from an edge, the
    # ray at least ~6 degrees off the plane, no limit) are decided in fp32; rays aimed at edges and
    # vertices, and grazing rays (|det| within its bound), stay undecided by design
    P = tri.astype(np.float64).reshape(-1, 3, 3)
    nrm = np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0])
    steep = np.abs(np.einsum("nc,nc->n", nrm, rd)) > 0.1 * np.linalg.norm(nrm, axis=1)
    clear_miss, clear_hit = steep & ~ok & (margin < -1e-2), steep & ok & (margin > 1e-2) & (tlim == FLT_MAX)
    assert dropped[clear_miss].mean() > 0.9 and sure[clear_hit].mean() > 0.9  # tiny far triangles: fp32 origin rounding
    print("clear misses dropped: %.4f; clear hits sure: %.4f; all fp64 rejections dropped: %.4f; undecided: %.4f"
          % (dropped[clear_miss].mean(), sure[clear_hit].mean(), dropped[~ok].mean(), (verdict == 1).mean()))
