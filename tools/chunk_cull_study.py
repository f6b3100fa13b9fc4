"""Chunk-level light cull: how often could a wave of the
lane-per-node cull (k_prep_cull_lanes) skip a half-chunk of 32 light triangles because EVERY node of
the wave culls all 32 by the two cheap stages (Mylight.cpp:340-357)?  CPU study on 12 800 surface
points area-sampled over the Veach stand-in's non-light facets (the shading points of secondary
bounces), in fp64 with the reference's tests.  Test infrastructure only (it loads the oracle).

    python tools/chunk_cull_study.py
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import pyoracle as po  # noqa: E402


def main():
    s = po.Scene("scenes/veach-mis/veach-mis.obj", "scenes/veach-mis/veach-mis.xml")
    v, _, light_of, un = s.facets()
    lf, _ = s.lights()
    P = v[:, :9].astype(np.float64).reshape(-1, 3, 3)[lf]
    UN, NL = un[lf], len(lf)
    rng = np.random.default_rng(3)
    nonlight = np.nonzero(light_of < 0)[0]
    Pf = v[:, :9].astype(np.float64).reshape(-1, 3, 3)
    Nf = v[:, 9:].astype(np.float64).reshape(-1, 3, 3)
    area = 0.5 * np.linalg.norm(np.cross(Pf[nonlight, 1] - Pf[nonlight, 0], Pf[nonlight, 2] - Pf[nonlight, 0]), axis=1)
    M = 64 * 200
    fs = nonlight[rng.choice(len(nonlight), M, p=area / area.sum())]
    b = rng.random((M, 2))
    sw = b.sum(1) > 1
    b[sw] = 1 - b[sw]
    X = (1 - b.sum(1))[:, None] * Pf[fs, 0] + b[:, :1] * Pf[fs, 1] + b[:, 1:] * Pf[fs, 2]
    N = (1 - b.sum(1))[:, None] * Nf[fs, 0] + b[:, :1] * Nf[fs, 1] + b[:, 1:] * Nf[fs, 2]
    N /= np.linalg.norm(N, axis=1)[:, None]
    c1 = np.einsum("lk,nlk->nl", UN, X[:, None, :] - P[None, :, 0]) < 1e-8  # light-side test
    t = np.stack([np.einsum("nk,nlk->nl", N, P[None, :, j] - X[:, None, :]) for j in range(3)], 0)
    cull = c1 | (t < 1e-8).all(0)  # or below the tangent plane
    nh = (NL + 31) // 32
    pad = np.ones((M, nh * 32), bool)
    pad[:, :NL] = cull
    hc = pad.reshape(M, nh, 32).all(2)
    print("(node, light) pairs culled by the cheap stages: %.3f" % cull.mean())
    print("half-chunks wholly culled for one node:          %.3f" % hc.mean())
    print("... for all 64 nodes of a wave (queue order):    %.5f" % hc.reshape(-1, 64, nh).all(1).mean())
    order = np.lexsort((X[:, 2], X[:, 1], X[:, 0]))
    print("... for all 64 nodes of a spatially sorted wave: %.3f" % hc[order].reshape(-1, 64, nh).all(1).mean())


if __name__ == "__main__":
    main()


def bound_study():
    """Wave-per-node alternative: per (node, 64-light chunk) conservative bounds -- the chunk's vertex
    sphere wholly below the node's tangent plane, or the node wholly behind every light's plane (normal
    cone: axis a, spread e = max |n_l - a|) -- against the exact per-light outcome."""
    s = po.Scene("scenes/veach-mis/veach-mis.obj", "scenes/veach-mis/veach-mis.xml")
    v, _, light_of, un = s.facets()
    lf, _ = s.lights()
    P = v[:, :9].astype(np.float64).reshape(-1, 3, 3)[lf]
    UN, NL = un[lf], len(lf)
    nch = (NL + 63) // 64
    rng = np.random.default_rng(3)
    nonlight = np.nonzero(light_of < 0)[0]
    Pf = v[:, :9].astype(np.float64).reshape(-1, 3, 3)
    Nf = v[:, 9:].astype(np.float64).reshape(-1, 3, 3)
    area = 0.5 * np.linalg.norm(np.cross(Pf[nonlight, 1] - Pf[nonlight, 0], Pf[nonlight, 2] - Pf[nonlight, 0]), axis=1)
    M = 4000
    fs = nonlight[rng.choice(len(nonlight), M, p=area / area.sum())]
    b = rng.random((M, 2))
    sw = b.sum(1) > 1
    b[sw] = 1 - b[sw]
    X = (1 - b.sum(1))[:, None] * Pf[fs, 0] + b[:, :1] * Pf[fs, 1] + b[:, 1:] * Pf[fs, 2]
    N = (1 - b.sum(1))[:, None] * Nf[fs, 0] + b[:, :1] * Nf[fs, 1] + b[:, 1:] * Nf[fs, 2]
    N /= np.linalg.norm(N, axis=1)[:, None]
    c1 = np.einsum("lk,nlk->nl", UN, X[:, None, :] - P[None, :, 0]) < 1e-8
    t = np.stack([np.einsum("nk,nlk->nl", N, P[None, :, j] - X[:, None, :]) for j in range(3)], 0)
    cull = c1 | (t < 1e-8).all(0)
    exact = np.ones((M, nch), bool)
    plane = np.zeros((M, nch), bool)
    side = np.zeros((M, nch), bool)
    for c in range(nch):
        sl = slice(64 * c, min(NL, 64 * c + 64))
        exact[:, c] = cull[:, sl].all(1)
        pts = P[sl].reshape(-1, 3)
        ctr = (pts.min(0) + pts.max(0)) / 2
        R = np.linalg.norm(pts - ctr, axis=1).max()
        a = UN[sl].mean(0)
        a /= np.linalg.norm(a)
        e = np.linalg.norm(UN[sl] - a, axis=1).max()
        vv = X - ctr
        plane[:, c] = N @ ctr - np.einsum("nk,nk->n", N, X) + R < 1e-8
        side[:, c] = vv @ a + e * np.linalg.norm(vv, axis=1) + R < 1e-8
    print("(node, chunk) wholly culled, exact: %.3f; by the plane bound: %.3f; by the cone bound: %.3f; either: %.3f" % (
        exact.mean(), plane.mean(), side.mean(), (plane | side).mean()))


if __name__ == "__main__":
    bound_study()
