#!/usr/bin/env python3
"""Deterministic generator for the Veach-MIS stand-in scene.

The reference loads `.\\Debug\\veach-mis\\veach-mis.{obj,mtl,xml}` (main.cpp:19,23-24) from
`example-scenes-cg23.zip`, which is listed in `/root/reference/.MISSING_LARGE_BLOBS` and is not
available.  This script authors a stand-in with the same structure:

* camera of the reference XML (README.md:339-343): eye (28.2792, 5.2, 1.23612e-06),
  lookat (0, 2.8, 0), up (0, 1, 0), fovy 20.1143 -- main.cpp:507-510 pulls the eye back 2x;
* four glossy Phong plates (thin boxes) with ascending roughness, tilted so that each one
  mirrors the light row toward the 2x camera;
* four tessellated sphere lights of radius 0.0333/0.1/0.3/0.9 (24x12 UV spheres, 528 triangles
  each) with equal power, plus one large light of radius 0.8 (30x16, 900 triangles) that is
  directly visible in the top-right corner like the reference renders (radiance 10, the value
  recovered from the tone-mapped reference BMPs);
* single-channel radiances sum to 380, the tone-map maximum of main.cpp:583
  (`exp_report/Veach场景的Monte Carlo Path Tracing.md:300`);
* 3012 light triangles as in the survey's probe stand-in;
* every surface strictly inside the scene bounding box (the floor and backdrop are boxes with
  thickness), so the reference grid's bbox-face crack cannot fire.

Run `python scenes/gen_veach_mis.py [outdir]`; output is byte-identical on every run.
"""
import math
import os
import sys

EYE = (28.2792, 5.2, 1.23612e-06)
LOOKAT = (0.0, 2.8, 0.0)
EYE2 = tuple(2 * e - l for e, l in zip(EYE, LOOKAT))  # main.cpp:509 start -= w

LIGHT_Y = 7.0
LIGHT_X = -4.0
SMALL_LIGHTS = [  # (name, z, radius); left of the image is +z
    ("light_xs", 3.3, 0.0333),
    ("light_s", 1.1, 0.1),
    ("light_m", -1.1, 0.3),
    ("light_l", -3.3, 0.9),
]
BIG_LIGHT = ("light_big", (-8.0, 6.2, -4.0), 0.8, 10.0)
TOTAL_RADIANCE = 380.0

# plates: (name, centre x, centre y, half length, Ns)
PLATES = [
    ("plate1", -2.5, 4.45, 1.25, 5000.0),
    ("plate2", -0.5, 2.85, 1.20, 800.0),
    ("plate3", 1.5, 1.30, 1.15, 120.0),
    ("plate4", 3.5, -0.05, 1.10, 20.0),
]
PLATE_HALF_Z = 5.6
PLATE_HALF_T = 0.025


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def mul(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def norm(a):
    n = math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])
    return (a[0] / n, a[1] / n, a[2] / n)


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


class Obj:
    def __init__(self):
        self.v = []
        self.vn = []
        self.groups = []  # (name, mtl, [(v0,n0),(v1,n1),(v2,n2)] list)

    def vert(self, p):
        self.v.append(p)
        return len(self.v)  # OBJ indices are 1-based

    def normal(self, n):
        self.vn.append(n)
        return len(self.vn)

    def box(self, name, mtl, centre, axes):
        """axes: three (unit direction, half extent) pairs."""
        faces = []
        for ax in range(3):
            d, h = axes[ax]
            o1, o2 = [axes[k] for k in range(3) if k != ax]
            for sgn in (1.0, -1.0):
                n = mul(d, sgn)
                c = add(centre, mul(d, sgn * h))
                corners = []
                for s1, s2 in ((-1, -1), (1, -1), (1, 1), (-1, 1)):
                    corners.append(add(add(c, mul(o1[0], s1 * o1[1])), mul(o2[0], s2 * o2[1])))
                vi = [self.vert(p) for p in corners]
                ni = self.normal(n)
                faces.append(((vi[0], ni), (vi[1], ni), (vi[2], ni)))
                faces.append(((vi[0], ni), (vi[2], ni), (vi[3], ni)))
        self.groups.append((name, mtl, faces))

    def sphere(self, name, mtl, centre, r, nseg, nring):
        top = self.vert(add(centre, (0.0, r, 0.0)))
        ntop = self.normal((0.0, 1.0, 0.0))
        rings = []
        for k in range(1, nring):
            th = math.pi * k / nring
            ring = []
            for s in range(nseg):
                ph = 2.0 * math.pi * s / nseg
                d = (math.sin(th) * math.cos(ph), math.cos(th), math.sin(th) * math.sin(ph))
                ring.append((self.vert(add(centre, mul(d, r))), self.normal(d)))
            rings.append(ring)
        bot = self.vert(add(centre, (0.0, -r, 0.0)))
        nbot = self.normal((0.0, -1.0, 0.0))
        faces = []
        for s in range(nseg):
            a, b = rings[0][s], rings[0][(s + 1) % nseg]
            faces.append(((top, ntop), b, a))
        for k in range(nring - 2):
            for s in range(nseg):
                a, b = rings[k][s], rings[k][(s + 1) % nseg]
                c, d = rings[k + 1][s], rings[k + 1][(s + 1) % nseg]
                faces.append((a, b, d))
                faces.append((a, d, c))
        for s in range(nseg):
            a, b = rings[-1][s], rings[-1][(s + 1) % nseg]
            faces.append(((bot, nbot), a, b))
        self.groups.append((name, mtl, faces))

    def write(self, path, mtllib):
        with open(path, "w", newline="\n") as f:
            f.write("# Veach-MIS stand-in scene, generated by scenes/gen_veach_mis.py\n")
            f.write("mtllib %s\n" % mtllib)
            for p in self.v:
                f.write("v %.6f %.6f %.6f\n" % p)
            for n in self.vn:
                f.write("vn %.6f %.6f %.6f\n" % n)
            for name, mtl, faces in self.groups:
                f.write("o %s\nusemtl %s\n" % (name, mtl))
                for tri in faces:
                    f.write("f %s\n" % " ".join("%d//%d" % vn for vn in tri))


def plate_frame(cx, cy):
    """Normal = half vector between the directions to the 2x eye and to the light row."""
    c = (cx, cy, 0.0)
    to_eye = norm(sub(EYE2, c))
    to_light = norm(sub((LIGHT_X, LIGHT_Y, 0.0), c))
    n = norm(add(to_eye, to_light))
    t = (n[1], -n[0], 0.0)
    return c, n, t


def build():
    obj = Obj()
    mtls = []
    # floor and backdrop: thick diffuse boxes, strictly inside the bbox
    obj.box("floor", "floor", (0.925, -1.6, 0.0),
            [((1.0, 0.0, 0.0), 13.075), ((0.0, 1.0, 0.0), 0.1), ((0.0, 0.0, 1.0), 13.0)])
    obj.box("backdrop", "backdrop", (-12.1, 5.65, 0.0),
            [((1.0, 0.0, 0.0), 0.1), ((0.0, 1.0, 0.0), 7.25), ((0.0, 0.0, 1.0), 13.0)])
    mtls.append(("floor", (0.4, 0.4, 0.4), (0.0, 0.0, 0.0), 1.0))
    mtls.append(("backdrop", (0.3, 0.3, 0.3), (0.0, 0.0, 0.0), 1.0))
    for name, cx, cy, hl, ns in PLATES:
        c, n, t = plate_frame(cx, cy)
        obj.box(name, name, c, [(t, hl), ((0.0, 0.0, 1.0), PLATE_HALF_Z), (n, PLATE_HALF_T)])
        mtls.append((name, (0.07, 0.09, 0.13), (0.1, 0.2, 0.3), ns))
    # equal-power small lights; single-channel radiances of all five lights sum to 380
    inv_area = [1.0 / (r * r) for _, _, r in SMALL_LIGHTS]
    power = (TOTAL_RADIANCE - BIG_LIGHT[3]) / sum(inv_area)
    radiance = {}
    for (name, z, r), ia in zip(SMALL_LIGHTS, inv_area):
        obj.sphere(name, name, (LIGHT_X, LIGHT_Y, z), r, 24, 12)
        radiance[name] = power * ia
        mtls.append((name, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0))
    bname, bc, br, brad = BIG_LIGHT
    obj.sphere(bname, bname, bc, br, 30, 16)
    radiance[bname] = brad
    mtls.append((bname, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0))
    return obj, mtls, radiance


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    obj, mtls, radiance = build()
    obj.write(os.path.join(outdir, "veach-mis.obj"), "veach-mis.mtl")
    with open(os.path.join(outdir, "veach-mis.mtl"), "w", newline="\n") as f:
        for name, kd, ks, ns in mtls:
            f.write("newmtl %s\n" % name)
            f.write("Kd %.6f %.6f %.6f\n" % kd)
            f.write("Ks %.6f %.6f %.6f\n" % ks)
            f.write("Ns %.6f\n\n" % ns)
    with open(os.path.join(outdir, "veach-mis.xml"), "w", newline="\n") as f:
        f.write('<camera type="perspective" width="1280" height="720" fovy="20.1143">\n')
        f.write('\t<eye x="28.2792" y="5.2" z="1.23612e-06"/>\n')
        f.write('\t<lookat x="0.0" y="2.8" z="0.0"/>\n')
        f.write('\t<up x="0.0" y="1.0" z="0.0"/>\n')
        f.write('</camera>\n')
        for name in sorted(radiance):
            r = radiance[name]
            f.write('<light mtlname="%s" radiance="%.6f,%.6f,%.6f"/>\n' % (name, r, r, r))
    ntri = sum(len(g[2]) for g in obj.groups)
    nlight = sum(len(g[2]) for g in obj.groups if g[1] in radiance)
    print("wrote %s: %d triangles, %d light triangles" % (outdir, ntri, nlight))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "veach-mis"))
