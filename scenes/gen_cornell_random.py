#!/usr/bin/env python3
"""Deterministic generator for the Cornell + random-triangles stand-in.

The reference's `cornell-box` scene (main.cpp:20, camera main.cpp:512-513) ships in
`example-scenes-cg23.zip`, which is missing from the reference checkout.  This script authors a
stand-in of the shape SURVEY.md §8(d) prescribes:

* an open-front box with interior [0, 556]^3 (floor, ceiling, back wall, red left wall, green right
  wall); every wall is a slab 1 unit thick, so the visible faces lie strictly inside the scene
  bounding box and the reference grid's bbox-face crack cannot fire;
* a 2-triangle area light just below the ceiling (x 213..343, z 227..332, facing down);
* N random triangles (default 1,000,000): centroids uniform in [6, 550]^3, equilateral with edge
  length ~ U(0.5, 5), uniformly random orientation, diffuse kd 0.5 (one-sided like every facet of
  the reference: the vertex normal is the geometric normal);
* the XML camera of main.cpp:512-513 (eye (278, 273, -800), lookat (278, 273, -799), up +y, fovy
  20.1143 with the reference's `/360` quirk); an XML camera has no pull-back (dist_scale 1).

    python scenes/gen_cornell_random.py [--triangles N] [--seed S] [outdir]

writes <outdir>/cornell-random.{obj,mtl,xml}; byte-identical for the same (N, seed).
"""
import argparse
import os

import numpy as np

BOX = 556.0
T = 1.0  # wall thickness
LIGHT = (213.0, 343.0, 227.0, 332.0, BOX - 0.1)  # x0, x1, z0, z1, y
LIGHT_RADIANCE = (17.0, 12.0, 4.0)

MATERIALS = [  # name, kd
    ("white", (0.73, 0.73, 0.73)),
    ("red", (0.63, 0.065, 0.05)),
    ("green", (0.14, 0.45, 0.091)),
    ("clutter", (0.5, 0.5, 0.5)),
    ("light", (0.0, 0.0, 0.0)),
]


def slab(lo, hi):
    """12 outward-facing triangles of the axis-aligned box [lo, hi] (each face's normal points away
    from the slab's centre)."""
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    tris, nrm = [], []
    for ax in range(3):
        for side, n in ((lo, -1.0), (hi, 1.0)):
            u, v = (ax + 1) % 3, (ax + 2) % 3
            c = []
            for a, b in ((0, 0), (1, 0), (1, 1), (0, 1)):
                p = np.empty(3)
                p[ax] = side[ax]
                p[u] = (lo, hi)[a][u]
                p[v] = (lo, hi)[b][v]
                c.append(p)
            nv = np.zeros(3)
            nv[ax] = n
            q = [c[0], c[1], c[2], c[3]]
            if np.dot(np.cross(q[1] - q[0], q[2] - q[0]), nv) < 0:
                q = q[::-1]
            tris += [(q[0], q[1], q[2]), (q[0], q[2], q[3])]
            nrm += [nv, nv]
    return np.array(tris), np.array(nrm)


def random_triangles(n, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(6.0, BOX - 6.0, size=(n, 3))
    edge = rng.uniform(0.5, 5.0, size=n)
    # uniformly random orientation: a random unit normal and a random in-plane angle
    z = rng.normal(size=(n, 3))
    z /= np.linalg.norm(z, axis=1)[:, None]
    a = np.where(np.abs(z[:, :1]) < 0.9, np.array([[1.0, 0, 0]]), np.array([[0, 1.0, 0]]))
    x = np.cross(z, a)
    x /= np.linalg.norm(x, axis=1)[:, None]
    y = np.cross(z, x)
    th0 = rng.uniform(0, 2 * np.pi, size=n)
    r = edge / np.sqrt(3.0)
    v = np.empty((n, 3, 3))
    for k in range(3):
        th = th0 + 2 * np.pi * k / 3
        v[:, k] = c + r[:, None] * (np.cos(th)[:, None] * x + np.sin(th)[:, None] * y)
    gn = np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])
    gn /= np.linalg.norm(gn, axis=1)[:, None]
    return v, gn


def write_obj(path, groups):
    """groups: list of (name, material, tris (n,3,3), normals (n,3))"""
    with open(path, "w", newline="\n") as f:
        f.write("# Cornell + random triangles stand-in (scenes/gen_cornell_random.py)\n")
        f.write("mtllib cornell-random.mtl\n")
        vbase = nbase = 1
        for name, mtl, tris, nrm in groups:
            n = len(tris)
            f.write("o %s\nusemtl %s\n" % (name, mtl))
            vv = tris.reshape(-1, 3).astype(np.float32).astype(np.float64)
            f.write(("v %.7g %.7g %.7g\n" * len(vv)) % tuple(vv.ravel()))
            nn = nrm.astype(np.float32).astype(np.float64)
            f.write(("vn %.7g %.7g %.7g\n" * n) % tuple(nn.ravel()))
            vi = np.arange(vbase, vbase + 3 * n).reshape(n, 3)
            ni = np.arange(nbase, nbase + n)
            idx = np.stack([vi[:, 0], ni, vi[:, 1], ni, vi[:, 2], ni], axis=1)
            f.write(("f %d//%d %d//%d %d//%d\n" * n) % tuple(idx.ravel()))
            vbase += 3 * n
            nbase += n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--triangles", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=20240430)
    ap.add_argument("outdir", nargs="?", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "cornell-random"))
    a = ap.parse_args()
    os.makedirs(a.outdir, exist_ok=True)
    groups = []
    walls = [  # name, material, slab lo, slab hi
        ("floor", "white", (-T, -T, -T), (BOX + T, 0.0, BOX + T)),
        ("ceiling", "white", (-T, BOX, -T), (BOX + T, BOX + T, BOX + T)),
        ("back", "white", (-T, -T, BOX), (BOX + T, BOX + T, BOX + T)),
        ("left", "red", (BOX, -T, -T), (BOX + T, BOX + T, BOX + T)),
        ("right", "green", (-T, -T, -T), (0.0, BOX + T, BOX + T)),
    ]
    for name, mtl, lo, hi in walls:
        t, n = slab(lo, hi)
        groups.append((name, mtl, t, n))
    x0, x1, z0, z1, y = LIGHT
    q = np.array([[x0, y, z0], [x1, y, z0], [x1, y, z1], [x0, y, z1]])
    lt = np.array([(q[0], q[1], q[2]), (q[0], q[2], q[3])])
    ln = np.cross(lt[:, 1] - lt[:, 0], lt[:, 2] - lt[:, 0])
    ln /= np.linalg.norm(ln, axis=1)[:, None]
    assert (ln[:, 1] < 0).all()  # facing down into the box
    groups.append(("light", "light", lt, ln))
    if a.triangles > 0:
        v, gn = random_triangles(a.triangles, a.seed)
        groups.append(("clutter", "clutter", v, gn))
    write_obj(os.path.join(a.outdir, "cornell-random.obj"), groups)
    with open(os.path.join(a.outdir, "cornell-random.mtl"), "w", newline="\n") as f:
        for name, kd in MATERIALS:
            f.write("newmtl %s\nKd %.6f %.6f %.6f\nKs 0.000000 0.000000 0.000000\nNs 1.000000\n\n" % ((name,) + kd))
    with open(os.path.join(a.outdir, "cornell-random.xml"), "w", newline="\n") as f:
        f.write('<camera type="perspective" width="800" height="600" fovy="20.1143">\n'
                '\t<eye x="278.0" y="273.0" z="-800.0"/>\n\t<lookat x="278.0" y="273.0" z="-799.0"/>\n'
                '\t<up x="0.0" y="1.0" z="0.0"/>\n</camera>\n')
        f.write('<light mtlname="light" radiance="%.6f,%.6f,%.6f"/>\n' % LIGHT_RADIANCE)
    print("wrote %s (%d triangles)" % (a.outdir, sum(len(g[2]) for g in groups)))


if __name__ == "__main__":
    main()
