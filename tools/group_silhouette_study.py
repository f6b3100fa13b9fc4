"""Gated study: how much of the light prep's full-stage work could a per-light-group
solid angle replace?

The reference's prep (Mylight.cpp:329-418) weighs every light triangle that passes the two cheap culls
by sA * sum L.  The stand-in's lights are tessellated spheres (one material = one convex closed mesh,
contiguous in the light order).  When a group lies wholly above a shading point's tangent plane (no
triangle plane-culled, Mylight.cpp:347-357) and the point is outside it, its candidates are exactly its
front-facing triangles (Mylight.cpp:340-345), whose spherical triangles tile the group's silhouette, so
sum_j sA_j = the silhouette's solid angle -- computable in O(silhouette edges), not O(triangles).  The
pick then needs the per-triangle weights only inside the picked group.

Measured here (CPU, fp64 numpy, the reference's cheap culls and the VOS sA): over secondary shading
points -- BRDF bounces of primary hits through the 800x600 reference camera, as the MIS tree's BRDF
children are -- the share of full-stage candidates in eligible groups, and the expected full-stage
evaluations per node if eligible groups cost only when picked (plus their silhouette rim).  Test
infrastructure only (loads the oracle).

    python tools/group_silhouette_study.py [points]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import pyoracle as po  # noqa: E402


def secondary_points(s, cam, m, rng):
    v, mat, light_of, un = s.facets()
    mats = s.materials()
    P = v[:, :9].astype(np.float64).reshape(-1, 3, 3)
    Nv = v[:, 9:].astype(np.float64).reshape(-1, 3, 3)
    pts, nrm = [], []
    W, H = cam.width, cam.height
    tries = 0
    while len(pts) < m and tries < 50 * m:
        tries += 1
        i, j = int(rng.integers(0, H)), int(rng.integers(0, W))
        e, d = po.camera_ray(cam, i, j)
        f, tbg = s.closest_hit(e, d)
        if f < 0 or light_of[f] >= 0:
            continue
        b, g = tbg[1], tbg[2]
        x = (1 - b - g) * P[f, 0] + b * P[f, 1] + g * P[f, 2]
        n = (1 - b - g) * Nv[f, 0] + b * Nv[f, 1] + g * Nv[f, 2]
        n /= np.linalg.norm(n)
        if np.dot(n, -np.asarray(d)) < 0:
            continue
        # one Phong-ish bounce: cosine hemisphere about n (diffuse) or near the mirror direction (glossy)
        kd, ks = mats[mat[f], :3].mean(), mats[mat[f], 3:6].mean()
        if rng.random() < ks / max(kd + ks, 1e-12):
            r = np.asarray(d) - 2 * np.dot(np.asarray(d), n) * n
            w = r + 0.05 * rng.normal(size=3)
        else:
            u1, u2 = rng.random(), rng.random()
            t = np.cross(n, [1.0, 0, 0] if abs(n[0]) < 0.9 else [0, 1.0, 0])
            t /= np.linalg.norm(t)
            bb = np.cross(n, t)
            ph = 2 * np.pi * u1
            w = np.sqrt(u2) * (np.cos(ph) * t + np.sin(ph) * bb) + np.sqrt(1 - u2) * n
        w /= np.linalg.norm(w)
        if np.dot(w, n) <= 0:
            continue
        f2, tbg2 = s.closest_hit(x, w, exclude=f)
        if f2 < 0 or light_of[f2] >= 0:
            continue
        b, g = tbg2[1], tbg2[2]
        x2 = (1 - b - g) * P[f2, 0] + b * P[f2, 1] + g * P[f2, 2]
        n2 = (1 - b - g) * Nv[f2, 0] + b * Nv[f2, 1] + g * Nv[f2, 2]
        n2 /= np.linalg.norm(n2)
        if np.dot(n2, -w) < 0:
            continue
        pts.append(x2)
        nrm.append(n2)
    return np.array(pts), np.array(nrm)


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    s = po.Scene("scenes/veach-mis/veach-mis.obj", "scenes/veach-mis/veach-mis.xml")
    v, mat, light_of, un = s.facets()
    lf, la = s.lights()
    P = v[:, :9].astype(np.float64).reshape(-1, 3, 3)[lf]
    UN = un[lf]
    SL = la[:, 1:].sum(1)
    gid = mat[lf]
    groups = []
    for g in np.unique(gid):
        idx = np.nonzero(gid == g)[0]
        assert (np.diff(idx) == 1).all(), "a light group is not contiguous in the light order"
        pts = P[idx].reshape(-1, 3)
        c = pts.mean(0)
        R = np.linalg.norm(pts - c, axis=1).max()
        groups.append((idx, c, R))
    cam = po.reference_camera(800, 600)
    e, _ = po.camera_ray(cam, 0, 0)
    s.build_grid(e)
    rng = np.random.default_rng(5)
    X, N = secondary_points(s, cam, m, rng)
    M = len(X)
    c1 = np.einsum("lk,nlk->nl", UN, X[:, None, :] - P[None, :, 0]) <= 1e-8
    t = np.stack([np.einsum("nk,nlk->nl", N, P[None, :, j] - X[:, None, :]) for j in range(3)], 0)
    cand = ~(c1 | (t <= 1e-8).all(0))
    # VOS sA per (node, light)
    A = P[None, :, 0] - X[:, None, :]
    B = P[None, :, 1] - X[:, None, :]
    Cc = P[None, :, 2] - X[:, None, :]
    A /= np.linalg.norm(A, axis=2)[..., None]
    B /= np.linalg.norm(B, axis=2)[..., None]
    Cc /= np.linalg.norm(Cc, axis=2)[..., None]
    num = np.abs(np.einsum("nlk,nlk->nl", A, np.cross(B, Cc)))
    den = 1 + np.einsum("nlk,nlk->nl", A, B) + np.einsum("nlk,nlk->nl", B, Cc) + np.einsum("nlk,nlk->nl", Cc, A)
    sA = 2 * np.arctan2(num, den)
    w = np.where(cand, sA * SL[None, :], 0.0)
    tot = cand.sum()
    elig_c = 0
    work_now = tot
    work_new = 0.0
    sliver_rim = 0
    for idx, c, R in groups:
        d = X - c
        dist = np.linalg.norm(d, axis=1)
        above = np.einsum("nk,nk->n", N, c - X) - R > 1e-6
        elig = above & (dist > R)
        nc = cand[:, idx].sum(1)
        wg = w[:, idx].sum(1)
        pg = wg / np.maximum(w.sum(1), 1e-300)
        elig_c += nc[elig].sum()
        # sliver candidates (band's 4 - den > 1000 num): these need their own full-stage term
        sl = ((4 - den[:, idx] > 1000 * num[:, idx]) & cand[:, idx]).sum(1)
        sliver_rim += sl[elig].sum()
        work_new += np.where(elig, pg * nc + sl, nc).sum()
    print("secondary shading points: %d; full-stage candidates per point: %.1f" % (M, tot / M))
    print("share of candidates in groups wholly above the tangent plane: %.3f" % (elig_c / tot))
    print("sliver candidates (4 - den > 1000 num) in eligible groups per point: %.2f" % (sliver_rim / M))
    print("expected full-stage evaluations per point: now %.1f, group scheme %.1f (x%.2f fewer)" % (
        work_now / M, work_new / M, work_now / max(work_new, 1)))
    for k, (idx, c, R) in enumerate(groups):
        above = np.einsum("nk,nk->n", N, c - X) - R > 1e-6
        print("  group %d (%d tris, R %.3f): eligible at %.3f of points, mean candidates %.1f, mean pick prob %.3f" % (
            k, len(idx), R, above.mean(), cand[:, idx].sum(1).mean(), (w[:, idx].sum(1) / np.maximum(w.sum(1), 1e-300)).mean()))


if __name__ == "__main__":
    main()


def fan_study(m=400):
    """The boundary-edge (fan) form of a group's weight: sum over the candidate triangles of a light group
    of their spherical excess = sum over the candidate set's boundary edges (a -> b, in the triangle's
    winding about its outward unique normal) of the signed solid angle of (r, a, b), r = the direction
    to the group's centre.  Checks the identity against the per-triangle VOS sum and counts the
    boundary edges per (point, group)."""
    s = po.Scene("scenes/veach-mis/veach-mis.obj", "scenes/veach-mis/veach-mis.xml")
    v, mat, light_of, un = s.facets()
    lf, la = s.lights()
    P = v[:, :9].astype(np.float64).reshape(-1, 3, 3)[lf]
    UN = un[lf]
    NL = len(lf)
    # orient every triangle CCW about its unique normal
    cr = np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0])
    flip = (cr * UN).sum(1) < 0
    P[flip] = P[flip][:, [0, 2, 1]]
    gid = mat[lf]
    # adjacency by exact vertex positions within a group: edge k of t = (P[t,k] -> P[t,k+1])
    key = {}
    for t in range(NL):
        for k in range(3):
            a, b = P[t, k].tobytes(), P[t, (k + 1) % 3].tobytes()
            key[(gid[t], a, b)] = (t, k)
    nb = -np.ones((NL, 3), np.int64)
    bad = 0
    for t in range(NL):
        for k in range(3):
            a, b = P[t, k].tobytes(), P[t, (k + 1) % 3].tobytes()
            o = key.get((gid[t], b, a))
            if o is None:
                bad += (gid[t], a, b) in key and False
            else:
                nb[t, k] = o[0]
    print("edges without an opposite twin: %d of %d" % ((nb < 0).sum(), 3 * NL))
    cam = po.reference_camera(800, 600)
    e, _ = po.camera_ray(cam, 0, 0)
    s.build_grid(e)
    X, N = secondary_points(s, cam, m, np.random.default_rng(5))
    groups = [np.nonzero(gid == g)[0] for g in np.unique(gid)]
    ctrs = [P[idx].reshape(-1, 3).mean(0) for idx in groups]
    worst, nedges, ncand = 0.0, [], []
    for x1, n in zip(X, N):
        c1 = (UN * (x1 - P[:, 0])).sum(1) <= 1e-8
        t = np.stack([((P[:, j] - x1) * n).sum(1) for j in range(3)], 0)
        cand = ~(c1 | (t <= 1e-8).all(0))
        for gi, idx in enumerate(groups):
            ci = idx[cand[idx]]
            if len(ci) == 0:
                continue
            A = P[ci] - x1
            A /= np.linalg.norm(A, axis=2)[..., None]
            num = (A[:, 0] * np.cross(A[:, 1], A[:, 2])).sum(1)
            den = 1 + (A[:, 0] * A[:, 1]).sum(1) + (A[:, 1] * A[:, 2]).sum(1) + (A[:, 2] * A[:, 0]).sum(1)
            tri = 2 * np.arctan2(np.abs(num), den)
            r = ctrs[gi] - x1
            r /= np.linalg.norm(r)
            tot, ne = 0.0, 0
            for t_ in ci:
                for k in range(3):
                    o = nb[t_, k]
                    if o >= 0 and cand[o]:
                        continue
                    a = P[t_, k] - x1
                    b = P[t_, (k + 1) % 3] - x1
                    a /= np.linalg.norm(a)
                    b /= np.linalg.norm(b)
                    tot += 2 * np.arctan2(r @ np.cross(a, b), 1 + r @ a + a @ b + b @ r)
                    ne += 1
            worst = max(worst, abs(abs(tot) - tri.sum()) / tri.sum())
            nedges.append(ne)
            ncand.append(len(ci))
    print("fan vs per-triangle sum: max rel diff %.2e; boundary edges per (point, group) mean %.1f, candidates %.1f" % (
        worst, np.mean(nedges), np.mean(ncand)))
