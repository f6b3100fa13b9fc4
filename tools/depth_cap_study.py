#!/usr/bin/env python3
"""Depth-cap study: what the counter-RNG trees lose by cutting the MIS
recursion (main.cpp:429-437, 464, 491 -- unbounded in the reference, only Russian roulette ends it) below depth
MCPT_MAX_DEPTH = 48 (device_math.h; the oracle's COUNTER_MAX_DEPTH).

Method (oracle/mcpt_oracle.c orc_depth_study, the GPU's counter-RNG semantics): the same camera samples rendered
with the tree cut at several depths D.  Nodes are keyed by (seed, pixel, sample, heap id), so every node at depth
<= D is the same in every run and two caps' frames differ exactly by what the levels between them contribute.
Reported per scene:
  * n_d, the nodes past entry + RR at depth d (cap 62, the deepest the 64-bit heap ids admit), and the branching
    factor m = n_{d+1} / n_d -- a Galton-Watson tree's expected node count at depth d is n_0 m^d;
  * for every cap D: the frame's relative L2 and mean change against cap 62, i.e. the mass of depths (D, 62].
    The contribution of depth d decays like rho^d with rho the transport operator's norm (albedo), not like
    P_RR^d: RR is compensated by its 1/0.6 weight, so it thins the tree without shrinking its expectation.

Scenes: the Veach stand-in (every 20th pixel of 800x600, the bench's subset) and tests/scenegen.occluded_room
(lights behind occluders: m > 1, supercritical -- the reference's recursion there terminates only with
probability < 1, so a cap is what makes it finite at all).

  python3 tools/depth_cap_study.py [--spp 64] [--out profiles/round6_depth_cap.json]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import pyoracle as po  # noqa: E402

SEED = 20240430
CAPS = [4, 8, 12, 16, 20, 24, 32, 40, 48, 56, 62]


def study(name, osc, cam, spp, stride, offset, nthreads):
    e, _ = po.camera_ray(cam, 0, 0)
    osc.build_grid(e)
    frames, hists, secs = {}, {}, {}
    for cap in CAPS:
        t = time.perf_counter()
        frames[cap], hists[cap] = osc.depth_study(cam, SEED, spp, cap, stride=stride, offset=offset, nthreads=nthreads)
        secs[cap] = time.perf_counter() - t
        print("%s cap %2d: %.1f s, %d nodes, %d cut" % (name, cap, secs[cap], int(hists[cap][:63].sum()), int(hists[cap][63])),
              flush=True)
    ref = frames[62]
    sub = ref[offset::stride, offset::stride]
    n = hists[62][:63].astype(float)
    last = int(np.nonzero(n)[0].max()) if n.any() else 0
    ratios = [float(n[d + 1] / n[d]) for d in range(last) if n[d] > 0 and n[d + 1] > 0]
    # the steady branching factor: median ratio over the levels with enough nodes for a stable estimate
    steady = [float(n[d + 1] / n[d]) for d in range(last) if n[d] >= 1000 and n[d + 1] > 0]
    out = {"scene": name, "spp": spp, "pixels": int(sub.shape[0] * sub.shape[1]), "seed": SEED,
           "nodes_per_depth_cap62": [int(v) for v in n[:last + 1]],
           "branching_ratio_per_depth": [round(r, 4) for r in ratios],
           "branching_factor_m": float(np.median(steady)) if steady else None,
           "caps": {}}
    for cap in CAPS:
        f = frames[cap][offset::stride, offset::stride]
        d = f - sub
        out["caps"][str(cap)] = {
            "rel_l2_vs_cap62": float(np.linalg.norm(d) / max(np.linalg.norm(sub), 1e-300)),
            "mean_rel_vs_cap62": float(d.sum() / max(sub.sum(), 1e-300)),
            "nodes": int(hists[cap][:63].sum()), "nodes_cut": int(hists[cap][63]), "seconds": round(secs[cap], 2)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--room-spp", type=int, default=4)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "round6_depth_cap.json"))
    args = ap.parse_args()
    res = []
    scene = os.path.join(ROOT, "scenes", "veach-mis")
    osc = po.Scene(scene + "/veach-mis.obj", scene + "/veach-mis.xml")
    res.append(study("veach 800x600 stride-20 subset", osc, po.reference_camera(800, 600), args.spp, 20, 7, args.threads))
    import scenegen
    d = tempfile.mkdtemp()
    obj, xml = scenegen.occluded_room(d)
    osc = po.Scene(obj, xml)
    cam = osc.camera()
    cam.width, cam.height = 8, 6
    res.append(study("occluded room 8x6 (supercritical)", osc, cam, args.room_spp, 1, 0, args.threads))
    with open(args.out, "w") as f:
        json.dump({"tool": "tools/depth_cap_study.py", "depth_cap": 48, "studies": res}, f, indent=1)
    for r in res:
        print(r["scene"], "m =", r["branching_factor_m"])
        for cap in ("16", "24", "32", "48"):
            print("  cap %s: rel L2 %.3e, mean %.3e vs cap 62" % (cap, r["caps"][cap]["rel_l2_vs_cap62"],
                                                               r["caps"][cap]["mean_rel_vs_cap62"]))


if __name__ == "__main__":
    main()
