#!/usr/bin/env python3
"""Size of the reference's stale-pdf quirk on the Veach-MIS stand-in (SURVEY.md §0
item 5).  shade_with_mis evaluates the BRDF branch's light pdf after the light branch's recursion
has overwritten the light sampler's members (main.cpp:443 vs :487, Mylight.cpp:484-493); the GPU
path uses the node's own prep (fresh).  The oracle renders the same pixels and samples with the same
counter RNG both ways (default = the reference's stale state; ORC_FLAG_FRESH_PDF), so the
difference is the quirk alone.

    python tools/stale_pdf_delta.py [--spp 1024 --threads 8]   -> profiles/stale_pdf_delta.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=600)
    ap.add_argument("--stride", type=int, default=20)
    ap.add_argument("--seed", type=int, default=20240430)
    a = ap.parse_args()
    from oracle import pyoracle as po
    d = os.path.join(ROOT, "scenes", "veach-mis")
    s = po.Scene(os.path.join(d, "veach-mis.obj"), os.path.join(d, "veach-mis.xml"))
    cam = po.reference_camera(a.width, a.height)
    e, _ = po.camera_ray(cam, 0, 0)
    s.build_grid(e)
    off = 7
    t = time.perf_counter()
    fresh, _ = s.render(cam, po.MODE_MIS | po.FLAG_FRESH_PDF, a.seed, a.spp, stride=a.stride, offset=off,
                        nthreads=a.threads)
    stale, _ = s.render(cam, po.MODE_MIS, a.seed, a.spp, stride=a.stride, offset=off, nthreads=a.threads)
    dt = time.perf_counter() - t
    sub = (slice(off, None, a.stride), slice(off, None, a.stride))
    f, g = fresh[sub], stale[sub]
    dpx = np.linalg.norm((g - f).reshape(-1, 3), axis=1)
    npx = np.linalg.norm(f.reshape(-1, 3), axis=1)
    out = {
        "what": "shade_with_mis, counter RNG, stale (the reference's, and the GPU default since round 2) vs fresh (MCPT_RENDER_FRESH_PDF) light pdf of the BRDF branch, "
                "same pixels and samples",
        "frame": "%dx%d, every %dth pixel in x and y from %d (%d px) x %d spp, seed %d" % (
            a.width, a.height, a.stride, off, f.shape[0] * f.shape[1], a.spp, a.seed),
        "rel_l2_stale_vs_fresh": float(np.linalg.norm(g - f) / np.linalg.norm(f)),
        "image_mean_fresh": float(f.mean()), "image_mean_stale": float(g.mean()),
        "image_mean_shift_rel": float((g.mean() - f.mean()) / f.mean()),
        "pixels_differing": int((dpx > 0).sum()), "pixels": int(dpx.size),
        "max_pixel_rel": float(np.max(np.where(npx > 0, dpx / np.maximum(npx, 1e-300), 0.0))),
        "north_star_tolerance": 1e-3,
        "seconds": round(dt, 1),
        "method": "tools/stale_pdf_delta.py (oracle/liboracle.so, default vs ORC_FLAG_FRESH_PDF)",
    }
    out["within_tolerance"] = out["rel_l2_stale_vs_fresh"] <= 1e-3
    print(json.dumps(out, indent=1))
    with open(os.path.join(ROOT, "profiles", "stale_pdf_delta.json"), "w") as fo:
        json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
