#!/usr/bin/env python3
"""Splits the full light-prep time into its cheap-stage + per-node part and its fp64 batch part:
the same 800x600 primary shading points once with their own normals and once with the normal
flipped away from every light (every light triangle culled by the cheap stages).  GPU only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import monte_carlo_path_tracing_amd as mcpt  # noqa: E402
from prep_variants import shading_points  # noqa: E402


def main():
    scene = mcpt.Scene.load(os.path.join(ROOT, "scenes/veach-mis/veach-mis.obj"),
                            os.path.join(ROOT, "scenes/veach-mis/veach-mis.xml"))
    x1, n = shading_points(scene)
    u = np.random.default_rng(1).random(len(x1))
    down = np.zeros_like(n)
    down[:, 1] = -1.0  # every light is above y = 5; a downward normal culls all by the tangent-plane test
    _, _, _ = mcpt.debug_prep_bench(scene, x1, n, u, variant=-1, iters=2)
    ms_full, ws, _ = mcpt.debug_prep_bench(scene, x1, n, u, variant=-1, iters=10)
    ms_cheap, ws0, _ = mcpt.debug_prep_bench(scene, x1, down, u, variant=-1, iters=10)
    _, cnt, _ = mcpt.light_prep(scene, x1, n, u)
    N = len(x1)
    print("points %d: full %.3f ms (%.2f ns/node), cheap-only %.3f ms (%.2f ns/node, weights_sum all zero: %s)"
          % (N, ms_full, ms_full * 1e6 / N, ms_cheap, ms_cheap * 1e6 / N, bool((ws0 == 0).all())))
    ms_pin, _, _ = mcpt.debug_prep_bench(scene, x1, down, u, variant=13, iters=10)
    print("cheap-only with the table loads pinned to one chunk (L1-resident; diagnostic): %.2f ns/node"
          % (ms_pin * 1e6 / N))
    print("fp64 batch part: %.2f ns/node (%.0f%%); survivors per node %.0f -> %.2f ns per 64 survivors"
          % ((ms_full - ms_cheap) * 1e6 / N, 100 * (ms_full - ms_cheap) / ms_full, cnt.mean(),
             (ms_full - ms_cheap) * 1e6 / N / (cnt.mean() / 64)))


if __name__ == "__main__":
    main()
