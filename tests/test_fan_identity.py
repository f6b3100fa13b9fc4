"""The boundary-edge ("fan") form of the light prep on the CPU (reference Mylight.cpp:329-418).

k_prep_fan weighs a light group (one <light> material, a contiguous run of the light table) by the
boundary edges of its candidate set instead of triangle by triangle.  These tests check the host tables
it relies on (mcpt_debug_fan_tables: neighbours from bit-identical vertices, orientation flips, sliver-
suspect factors) and the two facts the kernel's exactness rests on, in numpy fp64 over surface points of
the Veach stand-in and the stress scenes (tests/scenegen.py):
  * the identity: sum over a group's candidates of sA * sum L (Van Oosterom-Strackee, as k_prep_pk2
    weighs them) = sum over the candidate set's boundary edges of the signed fan term (r, A, B) * 2 sum L
    (flip applied), whenever x1 lies outside the group's bounding sphere and the group's shortest edge
    exceeds 1e-4 of its distance (k_prep_fan's node conditions) -- to 1e-10 relative;
  * every sliver of the band (4 - den > 1000 num, device_math.h) among the candidates satisfies the suspect
    test s = nl.(x1 - p0) <= eps_l D^3 / D'^2 (D, D' from the chunk's bounding sphere, as
    k_prep_cull_lanes<.., kSusp> evaluates it), so none escapes the band's sliver term.
"""
import numpy as np
import pytest

import monte_carlo_path_tracing_amd as mcpt
from conftest import SCENE_OBJ, SCENE_XML
from oracle import pyoracle as po
import scenegen

TAU = 1000.0


def unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def surface_points(osc, m, seed):
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
    return X, unit(Nn)


def check_scene(obj, xml, m=120, seed=5):
    s = mcpt.Scene.load(obj, xml)
    t = mcpt.debug_fan_tables(s)
    osc = po.Scene(obj, xml)
    v, _, _, un = osc.facets()
    lf, la = osc.lights()
    P = v[:, :9].astype(np.float64).reshape(-1, 3, 3)[lf]
    UN = un[lf]
    lsum2 = 2 * la[:, 1:].sum(1)
    nbr, eps, groups, ok = t["nbr"], t["eps"].astype(np.float64), t["groups"], t["ok"]
    gid = nbr[:, 3] & 0x3fffffff
    flip = (nbr[:, 3] >> 30) & 1
    NL = len(lf)
    # chunk spheres as get_device_state builds them (float centre, radius rounded up)
    chunks = []
    for c in range((NL + 63) // 64):
        pts = P[64 * c:64 * c + 64].reshape(-1, 3)
        ctr = np.float32(0.5 * (pts.min(0) + pts.max(0))).astype(np.float64)
        chunks.append((ctr, np.linalg.norm(pts - ctr, axis=1).max() * (1 + 1e-6) + 1e-6))
    X, N = surface_points(osc, m, seed)
    worst, fan_checked, slivers = 0.0, 0, 0
    for x1, n in zip(X, N):
        s_l = (UN * (x1 - P[:, 0])).sum(1)
        tpl = np.stack([((P[:, j] - x1) * n).sum(1) for j in range(3)], 0)
        cand = (s_l > 1e-8) & ~(tpl <= 1e-8).all(0)
        A = unit(P - x1[None, None, :])
        num = np.einsum("lk,lk->l", A[:, 0], np.cross(A[:, 1], A[:, 2]))
        den = 1 + (A[:, 0] * A[:, 1]).sum(1) + (A[:, 1] * A[:, 2]).sum(1) + (A[:, 2] * A[:, 0]).sum(1)
        half = np.arctan2(np.abs(num), den)
        # every band sliver among the candidates is a suspect
        sl = cand & (4 - den > TAU * np.abs(num))
        for li in np.nonzero(sl)[0]:
            ctr, R = chunks[li // 64]
            d = np.linalg.norm(x1 - ctr)
            thr = np.inf if d - R <= 0 else eps[li] * (d + R) ** 3 / (d - R) ** 2
            assert s_l[li] <= thr, (li, s_l[li], thr)
            slivers += 1
        for g in range(len(groups)):
            if not ok[g]:
                continue
            first, count = int(groups[g, 6]), int(groups[g, 7])
            c, R = groups[g, :3], groups[g, 3]
            dist = np.linalg.norm(x1 - c)
            if dist <= R or groups[g, 4] <= 1e-4 * (dist + R):  # k_prep_fan's node conditions
                continue
            idx = np.arange(first, first + count)
            ci = idx[cand[idx]]
            if len(ci) < 4:
                continue
            direct = (half[ci] * lsum2[ci]).sum()
            r = unit(c - x1)
            fan = 0.0
            for li in ci:
                for k in range(3):
                    o = nbr[li, k]
                    if o >= 0 and cand[o]:
                        continue  # an interior edge: cancels against its twin
                    a, b = A[li, k], A[li, (k + 1) % 3]
                    nm = r @ np.cross(a, b)
                    h = np.arctan2(abs(nm), 1 + r @ a + a @ b + b @ r) * np.sign(nm)
                    fan += (-h if flip[li] else h) * lsum2[li]
            worst = max(worst, abs(fan - direct) / direct)
            fan_checked += 1
            assert gid[ci].tolist() == [g] * len(ci)
    return worst, fan_checked, slivers, ok


def test_fan_tables_veach():
    s = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    t = mcpt.debug_fan_tables(s)
    assert len(t["ok"]) == 5 and t["ok"].all()  # five closed UV-sphere lights
    assert (t["nbr"][:, :3] >= 0).all()  # closed meshes: every edge has its twin
    worst, n, nsl, _ = check_scene(SCENE_OBJ, SCENE_XML)
    print("veach: %d (point, group) fan sums, max rel diff %.2e; %d slivers, all suspects" % (n, worst, nsl))
    assert n > 100 and worst < 1e-10


@pytest.mark.parametrize("name", ["sphmix", "slivers", "tinyfar"])
def test_fan_identity_stress_scenes(tmp_path, name):
    make, _ = scenegen.STRESS[name]
    obj, xml = make(str(tmp_path))
    worst, n, nsl, ok = check_scene(obj, xml, m=80)
    print("%s: groups eligible %s; %d (point, group) fan sums, max rel diff %.2e; %d slivers, all suspects" % (
        name, ok.tolist(), n, worst, nsl))
    assert worst < 1e-10
