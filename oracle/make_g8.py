#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY -- G8, the statistical reference of SURVEY.md §8(c): the compiled
reference (oracle/_ref/ref_harness, fake clock) renders a 32x24 frame of the Veach-MIS stand-in at
1024 spp per integrator (65536 for the heavy-tailed BRDF-only one); the per-pixel mean and
variance of one sample go to tests/golden/stat_<mode>_32x24x<spp>.npy (H x W x 6: mean rgb, var rgb).  8 processes over disjoint
row bands, each with its own fake-clock start.  Run in this container only (needs /root/reference):

    python oracle/make_g8.py --modes 0,2 --spp 1024 && python oracle/make_g8.py --modes 1 --spp 65536
"""
import argparse
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
NAMES = {0: "mis", 1: "brdf", 2: "shade", 3: "shade_area"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--width", type=int, default=32)
    ap.add_argument("--height", type=int, default=24)
    a = ap.parse_args()
    W, H = a.width, a.height
    exe = os.path.join(HERE, "_ref", "ref_harness")
    scene = os.path.join(ROOT, "scenes", "veach-mis")
    with tempfile.TemporaryDirectory() as tmp:
        for mode in (int(m) for m in a.modes.split(",")):
            bands = np.linspace(0, H, a.jobs + 1).astype(int)
            procs = []
            for k in range(a.jobs):
                r0, r1 = int(bands[k]), int(bands[k + 1])
                clock0 = 1 + (mode * 64 + k) * (1 << 40)  # disjoint fake-clock ranges per process
                procs.append(subprocess.Popen([exe, "veach-mis.obj", "veach-mis.xml", tmp, "stat", str(mode), str(W),
                                               str(H), str(a.spp), str(r0), str(r1), str(clock0)], cwd=scene,
                                              stdout=subprocess.DEVNULL))
            for p in procs:
                if p.wait() != 0:
                    raise SystemExit("ref_harness failed")
            rows = [np.load(os.path.join(tmp, "stat_%d_%d.npy" % (mode, int(bands[k])))) for k in range(a.jobs)]
            s = np.concatenate(rows).reshape(H, W, 6)
            mean = s[..., :3] / a.spp
            var = np.maximum(s[..., 3:] / a.spp - mean * mean, 0.0) * a.spp / (a.spp - 1)
            out = os.path.join(ROOT, "tests", "golden", "stat_%s_%dx%dx%d.npy" % (NAMES[mode], W, H, a.spp))
            np.save(out, np.concatenate([mean, var], axis=2))
            print("wrote", out, "image mean", mean.mean())


if __name__ == "__main__":
    main()
