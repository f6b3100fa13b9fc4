#!/usr/bin/env python3
"""Times the reference's own single-threaded CPU path against the oracle restatement on identical
frames, in THIS container (the compiled reference needs /root/reference; it never travels to the
GPU box).  Writes profiles/cpu_reference_vs_oracle.json, which bench.py reads to state a
reference-equivalent CPU baseline next to the oracle ("port") it times on the GPU box's host.

  reference: oracle/_ref/ref_harness `stat` mode -- the reference's Myobj/Mylight/BRDF/RadianceRGB
             translation units compiled from /root/reference (oracle/Makefile), its uniform grid
             (meshing(100000)), its shade_with_mis / shade_with_brdf / shade restated in
             ref_harness.cpp exactly as main.cpp:269-494, fake-clock RNG; 1 process = 1 core.
             Scene load + meshing are timed separately (a run with zero rows) and subtracted.
  oracle:    oracle/liboracle.so (fp64 C restatement, counter RNG), nthreads=1, the same W x H
             frame, camera and spp.

Both trace the primary ray once per pixel (the reference's main.cpp:572 re-traces it every sample;
that redundant work is not counted on either side).

    python tools/time_reference_cpu.py [--width 40 --height 30 --spp 8]
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = {0: "mis", 1: "brdf", 2: "shade"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def time_reference(exe, scene_dir, mode, W, H, spp, rows):
    with tempfile.TemporaryDirectory() as tmp:
        def run(r1):
            t = time.perf_counter()
            subprocess.run([exe, "veach-mis.obj", "veach-mis.xml", tmp, "stat", str(mode), str(W), str(H), str(spp), "0",
                            str(r1), "1"], cwd=scene_dir, check=True, stdout=subprocess.DEVNULL)
            return time.perf_counter() - t
        t0 = min(run(0) for _ in range(2))  # load + gather + meshing only
        return run(rows) - t0, t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=40)
    ap.add_argument("--height", type=int, default=30)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--brdf-spp", type=int, default=64)
    ap.add_argument("--modes", default="0,1,2")
    a = ap.parse_args()
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        raise SystemExit("build the compiled reference first: make -C oracle ref")
    from oracle import pyoracle as po
    scene_dir = os.path.join(ROOT, "scenes", "veach-mis")
    obj, xml = os.path.join(scene_dir, "veach-mis.obj"), os.path.join(scene_dir, "veach-mis.xml")
    W, H = a.width, a.height
    res = {}
    for mode in (int(m) for m in a.modes.split(",")):
        spp = a.brdf_spp if mode == 1 else a.spp
        samples = W * H * spp
        t_ref, t_load = time_reference(exe, scene_dir, mode, W, H, spp, H)
        osc = po.Scene(obj, xml)
        cam = po.reference_camera(W, H)
        e, _ = po.camera_ray(po.reference_camera(400, 300), 0, 0)  # the harness's grid: eye of make_cam(400, 300)
        osc.build_grid(e)
        om = {0: po.MODE_MIS, 1: po.MODE_BRDF, 2: po.MODE_SHADE}[mode]
        t = time.perf_counter()
        osc.render(cam, om, 20240430, spp, nthreads=1)
        t_orc = time.perf_counter() - t
        res[NAMES[mode]] = {
            "frame": "%dx%d x %d spp (%d camera samples)" % (W, H, spp, samples),
            "reference_s": round(t_ref, 3), "reference_load_s": round(t_load, 3),
            "reference_samples_per_s": round(samples / t_ref, 1),
            "oracle_s": round(t_orc, 3), "oracle_samples_per_s": round(samples / t_orc, 1),
            "oracle_over_reference": round(t_ref / t_orc, 3),
        }
        print(NAMES[mode], res[NAMES[mode]], flush=True)
    out = {
        "what": "single-thread CPU throughput of the compiled reference (oracle/_ref/ref_harness, the reference's "
                "own translation units) vs the oracle restatement (oracle/liboracle.so) on identical frames of the "
                "Veach-MIS stand-in; oracle_over_reference = reference time / oracle time",
        "host": cpu_model(), "cores_used": 1, "modes": res,
        "method": "tools/time_reference_cpu.py; reference load+meshing subtracted; primary ray traced once per pixel "
                  "on both sides",
    }
    path = os.path.join(ROOT, "profiles", "cpu_reference_vs_oracle.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
