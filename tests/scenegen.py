"""Small synthetic scenes for the edge-case tests, written with the Veach generator's OBJ writer
(scenes/gen_veach_mis.py): a scene without lights, a dense light panel (more than 4096 candidates
per shading point: the sequential batch-search path) and a very finely tessellated sphere light
(N_L > 7680: the LDS-queue prep variant, no root cache)."""
import math
import os
import sys

from conftest import ROOT

sys.path.insert(0, str(ROOT / "scenes"))
import gen_veach_mis as gv  # noqa: E402


def _write(outdir, name, obj, mtls, lights, cam):
    os.makedirs(outdir, exist_ok=True)
    obj.write(os.path.join(outdir, name + ".obj"), name + ".mtl")
    with open(os.path.join(outdir, name + ".mtl"), "w", newline="\n") as f:
        for m, kd, ks, ns in mtls:
            f.write("newmtl %s\nKd %.6f %.6f %.6f\nKs %.6f %.6f %.6f\nNs %.6f\n\n" % ((m,) + kd + ks + (ns,)))
    with open(os.path.join(outdir, name + ".xml"), "w", newline="\n") as f:
        eye, look = cam
        f.write('<camera type="perspective" width="16" height="12" fovy="20.1143">\n'
                '\t<eye x="%r" y="%r" z="%r"/>\n\t<lookat x="%r" y="%r" z="%r"/>\n'
                '\t<up x="0.0" y="1.0" z="0.0"/>\n</camera>\n' % (eye + look))
        for m, rad in lights:
            f.write('<light mtlname="%s" radiance="%.6f,%.6f,%.6f"/>\n' % ((m,) + rad))
    return os.path.join(outdir, name + ".obj"), os.path.join(outdir, name + ".xml")


def _floor(obj, mtls):
    obj.box("floor", "floor", (0.0, -0.1, 0.0), [((1.0, 0.0, 0.0), 4.0), ((0.0, 1.0, 0.0), 0.1), ((0.0, 0.0, 1.0), 4.0)])
    obj.box("block", "glossy", (0.5, 0.4, 0.3), [((1.0, 0.0, 0.0), 0.4), ((0.0, 1.0, 0.0), 0.4), ((0.0, 0.0, 1.0), 0.4)])
    mtls += [("floor", (0.5, 0.5, 0.5), (0.0, 0.0, 0.0), 1.0), ("glossy", (0.1, 0.1, 0.1), (0.4, 0.4, 0.4), 50.0)]


CAM = ((0.0, 3.0, 9.0), (0.0, 0.5, 0.0))


def no_lights(outdir):
    obj, mtls = gv.Obj(), []
    _floor(obj, mtls)
    return _write(outdir, "nolight", obj, mtls, [], CAM)


def light_panel(outdir, nx=60, nz=60):
    """a downward-facing light panel of nx x nz quads (2 nx nz triangles) above the floor"""
    obj, mtls = gv.Obj(), []
    _floor(obj, mtls)
    faces = []
    n = obj.normal((0.0, -1.0, 0.0))
    y, x0, x1, z0, z1 = 2.5, -1.5, 1.5, -1.5, 1.5
    for i in range(nx):
        for k in range(nz):
            xa, xb = x0 + (x1 - x0) * i / nx, x0 + (x1 - x0) * (i + 1) / nx
            za, zb = z0 + (z1 - z0) * k / nz, z0 + (z1 - z0) * (k + 1) / nz
            a, b = obj.vert((xa, y, za)), obj.vert((xb, y, za))
            c, d = obj.vert((xb, y, zb)), obj.vert((xa, y, zb))
            faces.append(((a, n), (b, n), (c, n)))  # (b-a) x (c-a) = -y: faces the floor
            faces.append(((a, n), (c, n), (d, n)))
    obj.groups.append(("panel", "panel", faces))
    mtls.append(("panel", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0))
    return _write(outdir, "panel", obj, mtls, [("panel", (2.0, 2.0, 2.0))], CAM)


def dense_sphere(outdir, nseg=120, nring=60):
    obj, mtls = gv.Obj(), []
    _floor(obj, mtls)
    obj.sphere("bulb", "bulb", (-0.8, 1.6, 0.0), 0.5, nseg, nring)
    mtls.append(("bulb", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0))
    return _write(outdir, "bulb", obj, mtls, [("bulb", (20.0, 18.0, 15.0))], CAM)


def occluded_room(outdir):
    """A closed room (inward faces of six wall slabs) with a down-facing ceiling lamp and an up-facing
    floor lamp, each hidden behind a close, wider cap: a light sample from almost any point hits a
    cap, and the cap's outer side faces the OTHER lamp, so an MIS node has two non-emitter children
    with probability ~0.6 each -- a supercritical tree (~1.2 children per node, main.cpp:455-491)
    whose generations outgrow any fixed wavefront queue."""
    obj, mtls = gv.Obj(), []
    X, Y, Z, T = 2.0, 3.0, 2.0, 0.1  # room half extents (y from 0 to Y), wall thickness
    ex, ey, ez = (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0)
    walls = [((0.0, -T, 0.0), [(ex, X + T), (ey, T), (ez, Z + T)]),
             ((0.0, Y + T, 0.0), [(ex, X + T), (ey, T), (ez, Z + T)]),
             ((-X - T, Y / 2, 0.0), [(ex, T), (ey, Y / 2), (ez, Z + T)]),
             ((X + T, Y / 2, 0.0), [(ex, T), (ey, Y / 2), (ez, Z + T)]),
             ((0.0, Y / 2, -Z - T), [(ex, X), (ey, Y / 2), (ez, T)]),
             ((0.0, Y / 2, Z + T), [(ex, X), (ey, Y / 2), (ez, T)])]
    for k, (c, axes) in enumerate(walls):
        obj.box("wall%d" % k, "wall", c, axes)
    faces = []
    for x0, y, ny in ((-0.8, Y - 0.05, -1.0), (0.8, 0.05, 1.0)):  # lamp quads: 0.4 x 0.4
        n = obj.normal((0.0, ny, 0.0))
        q = [obj.vert((x0 + sx * 0.2, y, sz * 0.2)) for sx, sz in ((-1, -1), (1, -1), (1, 1), (-1, 1))]
        tri = [(q[0], q[2], q[1]), (q[0], q[3], q[2])] if ny < 0 else [(q[0], q[1], q[2]), (q[0], q[2], q[3])]
        tri = [t if ny > 0 else t for t in tri]
        faces += [tuple((v, n) for v in t) for t in tri]
        obj.box("cap%d" % len(faces), "wall", (x0, y + 0.1 * ny, 0.0), [(ex, 0.35), (ey, 0.01), (ez, 0.35)])
    obj.groups.append(("lamp", "lamp", faces))
    mtls += [("wall", (0.7, 0.7, 0.7), (0.0, 0.0, 0.0), 1.0), ("lamp", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0)]
    return _write(outdir, "room", obj, mtls, [("lamp", (5.0, 5.0, 5.0))], ((0.0, 1.5, 1.8), (0.0, 0.4, 0.0)))


# ---- exact-pick stress scenes (the band + literal fallback beyond the stand-in) ----

def sphere_mix(outdir):
    """Four sphere lights of 8x4, 16x8, 32x16 and 64x32 segments (48 + 224 + 960 + 3968 = 5200 light
    triangles: more than 4096, so roots take the wave-per-root k_prep_pick), different radii, distances
    and radiances over the floor and a glossy block."""
    obj, mtls = gv.Obj(), []
    _floor(obj, mtls)
    lights = []
    for k, (seg, ring, c, r, rad) in enumerate([(8, 4, (-1.6, 1.9, -1.0), 0.35, (3.0, 2.0, 1.0)),
                                                (16, 8, (1.6, 2.1, -1.2), 0.2, (9.0, 9.0, 12.0)),
                                                (32, 16, (0.0, 2.6, -1.6), 0.5, (2.0, 2.5, 2.0)),
                                                (64, 32, (-0.3, 1.5, 1.4), 0.3, (4.0, 3.0, 3.0))]):
        name = "sph%d" % k
        obj.sphere(name, name, c, r, seg, ring)
        mtls.append((name, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0))
        lights.append((name, rad))
    return _write(outdir, "sphmix", obj, mtls, lights, CAM)


def slivers(outdir, strips=24):
    """Lights seen nearly edge-on from the floor: vertical light blinds (planes x = const, split into
    long thin triangles) standing on the floor region, whose planes pass through the floor points next
    to them -- their spherical triangles are slivers (one vertex angle near pi), where the reference's
    alpha + beta + gamma - pi is decided by the last bits of its acos; plus a panel tilted 2 degrees
    off the vertical (near-grazing for the points below it)."""
    obj, mtls = gv.Obj(), []
    _floor(obj, mtls)
    faces = []
    for xk in (-1.2, -0.4, 0.4, 1.2):
        for side in (1.0, -1.0):  # two thin layers facing +x and -x
            x = xk + 0.002 * side
            n = obj.normal((side, 0.0, 0.0))
            for s in range(strips):
                y0, y1 = 0.3 + 1.5 * s / strips, 0.3 + 1.5 * (s + 1) / strips
                a, b = obj.vert((x, y0, -1.5)), obj.vert((x, y0, 1.5))
                c, d = obj.vert((x, y1, 1.5)), obj.vert((x, y1, -1.5))
                tri = [(a, b, c), (a, c, d)]
                if side < 0:
                    tri = [(a, c, b), (a, d, c)]
                faces += [tuple((v, n) for v in t) for t in tri]
    obj.groups.append(("blinds", "blinds", faces))
    faces = []
    t = math.radians(2.0)
    n = obj.normal((math.cos(t), math.sin(t), 0.0))
    for s in range(40):  # tilted panel of 80 thin triangles near x = 2.2
        z0, z1 = -1.5 + 3.0 * s / 40, -1.5 + 3.0 * (s + 1) / 40
        p = [(2.2 - 1.6 * math.sin(t) * h, 0.2 + 1.6 * math.cos(t) * h, z) for h, z in ((0, z0), (0, z1), (1, z1), (1, z0))]
        q = [obj.vert(v) for v in p]
        faces += [((q[0], n), (q[2], n), (q[1], n)), ((q[0], n), (q[3], n), (q[2], n))]
    obj.groups.append(("tilt", "tilt", faces))
    mtls += [("blinds", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0), ("tilt", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0)]
    return _write(outdir, "slivers", obj, mtls, [("blinds", (4.0, 4.0, 4.0)), ("tilt", (6.0, 5.0, 4.0))], CAM)


def tiny_far(outdir):
    """Distant tiny lights: 8x4 spheres of radius 1e-2, 1e-3, 1e-4 and 1e-6 at distances 20-90 above the
    floor, plus one ordinary light.  Their spherical triangles span ~1e-2 .. 1e-8 rad: the reference's
    alpha + beta + gamma - pi is mostly its own rounding there (the unit vectors' rounding amplified by
    distance / edge), and the edge-length culls (< 1e-8 rad, Mylight.cpp:379-382) fire on the smallest."""
    obj, mtls = gv.Obj(), []
    _floor(obj, mtls)
    lights = []
    k = 0
    for r in (1e-2, 1e-3, 1e-4, 1e-6):
        for dist, az in ((20.0, 0.3), (45.0, 1.9), (90.0, 4.0)):
            name = "tiny%02d" % k
            c = (dist * 0.3 * math.cos(az), dist, dist * 0.3 * math.sin(az))
            obj.sphere(name, name, c, r, 8, 4)
            mtls.append((name, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0))
            lights.append((name, (4000.0, 3000.0, 2000.0)))
            k += 1
    obj.sphere("lamp", "lamp", (1.2, 2.2, -0.8), 0.25, 16, 8)
    mtls.append(("lamp", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0))
    lights.append(("lamp", (5.0, 5.0, 5.0)))
    return _write(outdir, "tinyfar", obj, mtls, lights, CAM)


def light_soup(outdir, n=1500, seed=3):
    """n unrelated light triangles (round 6): random positions 0.3-40 units above / around the floor, random
    orientations, sizes spanning 1e-4 .. 1 (log-uniform) and shapes from equilateral to slivers (one vertex pulled
    to within 1e-3 of the opposite edge), one of five radiances each -- no tessellated sphere, no shared edges, so
    the spherical triangles of a shading point cover every size, aspect and viewing angle the band must bound"""
    import random
    rng = random.Random(seed)
    obj, mtls = gv.Obj(), []
    _floor(obj, mtls)
    groups = {k: [] for k in range(5)}
    for _ in range(n):
        c = (rng.uniform(-8.0, 8.0), 0.3 + 40.0 * rng.random() ** 2, rng.uniform(-8.0, 8.0))
        size = 10.0 ** rng.uniform(-4.0, 0.0)
        u = gv.norm((rng.gauss(0, 1), rng.gauss(0, 1), rng.gauss(0, 1)))
        w = gv.norm(gv.cross(u, gv.norm((rng.gauss(0, 1), rng.gauss(0, 1), rng.gauss(0, 1)))))
        a = gv.add(c, gv.mul(u, -size))
        b = gv.add(c, gv.mul(u, size))
        h = size * (1e-3 if rng.random() < 0.2 else rng.uniform(0.2, 1.7))
        d = gv.add(gv.add(c, gv.mul(u, size * rng.uniform(-0.9, 0.9))), gv.mul(w, h))
        nrm = gv.norm(gv.cross(gv.sub(b, a), gv.sub(d, a)))
        ni = obj.normal(nrm)
        groups[rng.randrange(5)].append(((obj.vert(a), ni), (obj.vert(b), ni), (obj.vert(d), ni)))
    lights = []
    for k, faces in groups.items():
        name = "soup%d" % k
        obj.groups.append((name, name, faces))
        mtls.append((name, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0))
        lights.append((name, (3.0 * (k + 1), 2.0 * (k + 1), 1.0 * (k + 1))))
    return _write(outdir, "soup", obj, mtls, lights, CAM)


STRESS = {"sphmix": (sphere_mix, 5200), "slivers": (slivers, 8 * 24 * 2 + 80), "tinyfar": (tiny_far, 12 * 48 + 224),
          "dense": (dense_sphere, 14160), "soup": (light_soup, 1500)}


def needles(outdir, n=70000, seed=7, length=1.0):
    """n thin random triangles ("needles", up to `length` long) in a 10-unit box in every direction, plus the floor:
    nearly every object split of such a tree overlaps, so a >= 65 536-triangle build wants far more spatial-split
    duplicates than its budget (bvh.cpp MCPT_BVH_SPATIAL_BUDGET) allows -- the budget-exhausting case of the
    builder's determinism test"""
    import random
    rng = random.Random(seed)
    obj, mtls = gv.Obj(), []
    _floor(obj, mtls)
    ni = obj.normal((0.0, 1.0, 0.0))
    faces = []
    for _ in range(n):
        a = tuple(rng.uniform(-5.0, 5.0) for _ in range(3))
        b = tuple(min(5.0, max(-5.0, x + rng.uniform(-length, length))) for x in a)
        c = tuple(x + rng.uniform(-0.02, 0.02) for x in a)
        faces.append(((obj.vert(a), ni), (obj.vert(b), ni), (obj.vert(c), ni)))
    obj.groups.append(("needles", "floor", faces))
    return _write(outdir, "needles", obj, mtls, [], CAM)
