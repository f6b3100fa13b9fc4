#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X path tracer on the Veach-MIS stand-in (BASELINE.json).

Workload (BASELINE.json configs[2]): MIS (light + BRDF sampling), 800x600 at 1024 spp.  A "step"
is one pass of the hot path over one batch: spp_per_step samples of every pixel of the 800x600
frame (default 1024: each step renders the whole 1024-spp frame of BASELINE.json), by one
mcpt_render_device call (wavefront kernels, fp64 framebuffer resident in HBM); the run accumulates
steps x gpus x spp_per_step samples per pixel.
Each call computes everything it uses, including its root-point light-prep cache;
nothing is carried from one step to the next except the framebuffer.

Multi-GPU: sample-range sharding -- weak scaling for --config c3 (each rank S samples per step), strong
scaling for --config c4 (1600x1200, one 4096-spp frame per step split over the ranks, BASELINE.json
configs[3]).  Step k is the job [k*G*S, (k+1)*G*S) of global sample indices, which the library splits
into one S-sample shard per GPU and ends with ONE ncclReduce(sum) of the fp64 framebuffers into GPU 0.
Two launch forms:
  * `python3 bench.py --gpus N` (no WORLD_SIZE in the environment): one process drives all N GPUs
    through the library's device list (mcpt_render_opts.devices = 0..N-1: a host thread and stream
    per GPU, ncclCommInitAll, one grouped reduce per step);
  * `torchrun --nproc-per-node N bench.py --gpus N`: one process per GPU, each joining the library's own
    RCCL communicator (mcpt_comm: rank 0's ncclUniqueId is broadcast over torch.distributed, then
    mcpt_comm_init_rank); torch.distributed only provides the barrier and the max-over-ranks timing.
    WORLD_SIZE must equal --gpus.

Also reported: the roofline of the dominant kernel (k_prep: fp64 VALU-bound light prep), the
CPU baseline (the C oracle on a bounded stratified pixel subset, rank 0, N=1 only) and the
relative L2 of the GPU frame against that CPU render on the same pixels and samples.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec (whole node) + per-pixel L2 vs CPU, Veach-MIS 800×600@1024spp"
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X fp64 vector (spec); see DESIGN.md §roofline
HBM_PEAK_GBS = 8000.0
SMALL_NL = 64  # render.hip kSmallNL: light tables this small take the lane-per-node prep (k_prep_lane)
# algorithmic fp64 operations of one light-triangle evaluation of Mylight.cpp:335-413 by the
# stage at which it ends (+,-,*,/,sqrt,acos,fmin/fmax each 1)
FLOPS_CULL_BACKFACE = 8
FLOPS_CULL_PLANE = 32
FLOPS_FULL = 269
# algorithmic HBM bytes of one prep node: reads p, N (48 B) + pixel, sample, node id (16 B) for the
# RNG key; writes weights_sum + pick (12 B).  The light table (240 KB) is L2/MALL resident.
PREP_BYTES_PER_NODE = 76
# traversal: a BVH node visit tests its children's slabs in fp32 -- 12 flops per
# child box, 4 children per 4-wide node -- and every ray/triangle test is the reference's fp64 Cramer
# rule (Myobj.cpp:165-192, 74 flops).  VALU model in fp32-equivalent flops (an fp64 op issues at
# half the fp32 rate on MI355X: 78.6 vs 157.3 TFLOP/s).  Memory model: every node visit fetches its
# 128-B node and every test its 48-B triangle, from the cache level that holds the structure --
# the peak is MI355X_MICROARCH.md's measured chip-wide random-row gather rate of that level: L2
# (an XCD's 4 MiB, 16.8-18.8 TB/s), Infinity Cache (256 MB, 8.6 TB/s), else HBM.
FP32_VECTOR_PEAK_TFLOPS = 157.3
GATHER_PEAKS = [(4 << 20, "l2", 17800.0), (256 << 20, "infinity_cache", 8600.0), (1 << 62, "hbm", HBM_PEAK_GBS)]
FLOPS_NODE_VISIT = 48
FLOPS_TRI_TEST_FP64 = 74
# bytes one node visit fetches: the 128-B BvhNode4 (k_mis_rays, k_extend_brdf) or the 64-B compressed
# BvhNode4Q that k_rays_persistent reads ("Compressed nodes")
BYTES_NODE_VISIT = {"k_mis_rays": 128, "k_extend_brdf": 128, "k_rays_persistent": 64}
BYTES_TRI_TEST = 48
# --config: BASELINE.json configs as bench workloads.  c3 (default) is the metric's configuration;
# c4 is the 1600x1200 frame whose 4096-spp job is split over the ranks (strong scaling)
CONFIGS = {"c3": dict(width=800, height=600, job_spp=None, scaling="weak"),
           "c4": dict(width=1600, height=1200, job_spp=4096, scaling="strong")}
SCENE = os.path.join(ROOT, "scenes", "veach-mis")
SCENES = {  # --scene: (metric, data note)
    "veach": (METRIC, "synthetic: Veach-MIS stand-in scene (scenes/gen_veach_mis.py; the reference's scene files are missing)"),
    "cornell1m": ("Msamples/sec (whole node) + per-pixel L2 vs CPU, Cornell + 1M random triangles 800×600@1024spp",
                  "synthetic: Cornell + 1,000,000 random triangles stand-in (scenes/gen_cornell_random.py, "
                  "SURVEY.md §8(d) C5; generated at start-up)"),
}


def scene_files(name):
    """(obj, xml, camera-from-XML?) of a --scene"""
    if name == "veach":
        return SCENE + "/veach-mis.obj", SCENE + "/veach-mis.xml", False
    import subprocess
    import tempfile
    d = os.path.join(tempfile.gettempdir(), "mcpt_cornell_1000000_20240430")
    obj, xml = d + "/cornell-random.obj", d + "/cornell-random.xml"
    if not (os.path.exists(obj) and os.path.exists(xml)):
        subprocess.run([sys.executable, os.path.join(ROOT, "scenes", "gen_cornell_random.py"), "--triangles",
                        "1000000", "--seed", "20240430", d], check=True, capture_output=True)
    return obj, xml, True


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_json(path):
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def rel_l2(g, c):
    return float(np.linalg.norm(g - c) / max(np.linalg.norm(c), 1e-300))


def max_px_rel(g, c):
    """max over pixels of ||g_px - c_px|| / ||c_px|| (pixels black in both count 0)"""
    d = np.linalg.norm((g - c).reshape(-1, 3), axis=1)
    n = np.linalg.norm(c.reshape(-1, 3), axis=1)
    return float(np.max(np.where(n > 0, d / np.maximum(n, 1e-300), np.where(d > 0, np.inf, 0.0))))


def host_cpu_model():
    """lscpu's "Model name" of this host (from /proc/cpuinfo), or None"""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_threads():
    """the CPU share to use: OMP_NUM_THREADS (16 on the GPU box), at most the visible CPUs"""
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    return max(1, min(n, 16, os.cpu_count() or 1))


def cpu_baseline(scene_name, W, H, mode, seed, full_spp, max_s, single_s):
    """The C oracle (oracle/liboracle.so: the reference's algorithm incl. its uniform grid and O(N_L) light
    prep per node, fp64) on the stratified pixel subset of BASELINE.md §3 -- every 20th pixel in x and y.

    Two legs, both measured on this host:
      * single thread (the baseline BASELINE.md §3 / north_star name: the reference's loop main.cpp:557-588
        is single-threaded, README.md:418): the subset at as many spp as fit in single_s seconds (the oracle's
        time per camera sample does not depend on spp: it caches nothing across samples), so `value` is a
        measured 1-core rate, `cores` 1;
      * all of the host's CPU share (cpu_threads(): the oracle parallelises over pixels) at the workload's
        FULL spp if that fits in max_s (else fewer spp, extrapolated; stated), whose image is the L2
        reference of the bench line.
    Returns (dict, subset image of the multi-thread leg, its spp)."""
    from oracle import pyoracle as po

    obj, xml, xml_cam = scene_files(scene_name)
    osc = po.Scene(obj, xml)
    if xml_cam:
        ocam = osc.camera()
        ocam.width, ocam.height = W, H
    else:
        ocam = po.reference_camera(W, H)
    e, _ = po.camera_ray(ocam, 0, 0)
    osc.build_grid(e)
    m = {"mis": po.MODE_MIS, "brdf": po.MODE_BRDF, "shade": po.MODE_SHADE, "shade_area": po.MODE_SHADE_AREA}[mode]
    npx = len(range(7, H, 20)) * len(range(7, W, 20))
    nt = cpu_threads()
    # ---- multi-thread leg: full spp (the L2 reference image) ----
    t = time.perf_counter()
    osc.render(ocam, m, seed, 4, s1=4, stride=20, offset=7, nthreads=nt)  # calibration: 4 spp
    t4 = time.perf_counter() - t
    est = t4 / 4 * full_spp
    spp = full_spp if est <= max_s else int(max(1, min(full_spp, max_s / max(t4 / 4, 1e-6))))
    t = time.perf_counter()
    img, _ = osc.render(ocam, m, seed, spp, stride=20, offset=7, nthreads=nt)
    dt = time.perf_counter() - t
    mt_value = npx * spp / dt / 1e6
    # ---- single-thread leg: the same subset, samples [0, spp1) at the same seed ----
    per_sample_1t = dt * nt / (npx * spp)  # first guess from the multi-thread leg
    spp1 = int(max(1, min(full_spp, single_s / max(per_sample_1t * npx, 1e-9))))
    t = time.perf_counter()
    osc.render(ocam, m, seed, spp1, stride=20, offset=7, nthreads=1)
    dt1 = time.perf_counter() - t
    value = npx * spp1 / dt1 / 1e6
    out = {"value": value, "unit": "Msamples/s", "cores": 1, "kind": "port",
           "host_cpu": host_cpu_model(), "host_cpus_visible": os.cpu_count(),
           "single_thread_value": value, "single_thread_spp": spp1, "single_thread_seconds": round(dt1, 2),
           "multi_thread_value": mt_value, "multi_thread_cores": nt, "multi_thread_spp": spp,
           "multi_thread_full_spp": spp == full_spp, "multi_thread_seconds": round(dt, 2),
           "subset_pixels": npx,
           "sample": "oracle/mcpt_oracle.c (fp64 C restatement incl. the reference's uniform grid) on 1 core: every 20th "
                     "pixel in x and y of %dx%d (%d px = 1/400 of the frame) x %d spp %s = %d camera samples in %.1f s "
                     "(time per sample is independent of spp; full %d spp extrapolated: %.0f s); also %d threads at %d spp "
                     "in %.1f s (%.4f Msamples/s), whose image is the L2 reference" % (
                         W, H, npx, spp1, mode.upper(), npx * spp1, dt1, full_spp, dt1 * full_spp / spp1, nt, spp, dt,
                         mt_value)}
    out["full_frame_seconds_extrapolated_1core"] = dt1 * (full_spp / spp1) * (W * H / npx)
    # The reference itself cannot travel to the GPU box.  Its single-thread speed relative to this
    # restatement was measured on identical frames in the build container (tools/time_reference_cpu.py) --
    # a cross-host factor (another CPU), applied to the single-thread value measured here.
    ref = load_json(os.path.join(ROOT, "profiles", "cpu_reference_vs_oracle.json"))
    r = (ref or {}).get("modes", {}).get(mode) if scene_name == "veach" else None
    if r:
        out["oracle_over_reference_cross_host"] = r["oracle_over_reference"]
        out["reference_equivalent_value"] = value / r["oracle_over_reference"]
        out["reference_equivalent_source"] = ("single_thread_value (measured on this host) / oracle_over_reference_cross_host "
                                              "(profiles/cpu_reference_vs_oracle.json: compiled reference %.0f vs oracle "
                                              "%.0f samples/s, 1 core of '%s', not this host; %s)" % (
                                                  r["reference_samples_per_s"], r["oracle_samples_per_s"],
                                                  ref.get("host", "?"), r["frame"]))
    return out, img, spp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    # samples per render call: every call rebuilds its root-point cache and drains its wavefront
    # queue, so larger calls amortise more (round 1: 64 -> 360, 128 -> 379, 256 -> 391, 1024 -> 399
    # Msamples/s; round 2e: 256 -> 467-468, 1024 -> 480-481); the default step is the whole
    # 1024-spp frame of BASELINE.json in one call, as the reference renders it
    ap.add_argument("--spp-per-step", type=int, default=1024)
    ap.add_argument("--width", type=int, default=None, help="default: the --config's (800)")
    ap.add_argument("--height", type=int, default=None, help="default: the --config's (600)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS),
                    help="c3: BASELINE.json's metric config (800x600, spp_per_step samples per rank, weak scaling); "
                         "c4: 1600x1200, each step one 4096-spp frame split over the ranks (strong scaling)")
    ap.add_argument("--mode", default="mis", choices=["mis", "brdf", "shade", "shade_area"])
    ap.add_argument("--scene", default="veach", choices=sorted(SCENES),
                    help="veach: the north-star workload (C3); cornell1m: config C5")
    ap.add_argument("--seed", type=int, default=20240430)
    ap.add_argument("--cpu-seconds", type=float, default=90.0,
                    help="CPU baseline budget: the full-spp subset runs if it fits, else fewer spp, extrapolated")
    ap.add_argument("--cpu-single-seconds", type=float, default=20.0,
                    help="budget of the single-thread CPU baseline leg (spp reduced to fit; rate per sample)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline and L2 check")
    ap.add_argument("--no-replay", action="store_true",
                    help="skip the untimed statistics replay (PMC passes: the profile then holds only the warmup and "
                         "timed steps' kernel instances; the line has no traversal roofline, whose events it counts)")
    ap.add_argument("--fresh-pdf", action="store_true",
                    help="MIS with the node's own light pdf (MCPT_RENDER_FRESH_PDF) instead of the reference's stale one")
    ap.add_argument("--precision", default="fp64", choices=["fp64", "fp32"],
                    help="light-prep precision: fp64 (the reference's, the headline) or the opt-in FP32_STABLE mode "
                         "(MCPT_RENDER_PRECISION_FP32: packed-fp32 weights summed in fp64)")
    ap.add_argument("--no-root-cache", action="store_true",
                    help="disable the per-pixel root-point light-prep cache (MCPT_DEBUG_NO_ROOT_CACHE): every root runs "
                         "the full O(N_L) prep, the regime of frames whose cache exceeds the HBM budget")
    ap.add_argument("--debug-flags", type=lambda v: int(v, 0), default=0,
                    help="extra mcpt_render_opts.flags bits of include/mcpt_debug.h (A/B experiments)")
    ap.add_argument("--out", default="", help="optional .bmp of the rendered frame (rank 0)")
    ap.add_argument("--collective-lib", default="",
                    help="rehearsal on fewer GPUs than ranks (test infrastructure): the library's reduce goes through this "
                         "NCCL-API library (tests/collshim/libmcpt_collshim.so, host shared memory) instead of RCCL, ranks "
                         "share GPUs round-robin and torch.distributed uses gloo")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    # Two launch forms, one per-GPU shard each:
    #  * torchrun (WORLD_SIZE set): one process per GPU, the library's per-process communicator
    #    (mcpt_comm, ncclCommInitRank); WORLD_SIZE must equal --gpus;
    #  * plain `python3 bench.py --gpus N` (no WORLD_SIZE): ONE process drives N GPUs through the
    #    library's device list (mcpt_render_opts.devices = 0..N-1: one host thread + stream per GPU,
    #    ncclCommInitAll, ONE grouped ncclReduce per step into device 0).
    launched = "WORLD_SIZE" in os.environ
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if launched and world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d ranks (WORLD_SIZE)" % (args.gpus, world))
    import torch
    import torch.distributed as dist

    import monte_carlo_path_tracing_amd as mcpt

    import hashlib
    with open(mcpt.LIB_PATH, "rb") as f:  # the binary this run times (the PMC profiles name theirs the same way)
        lib_sha = hashlib.sha256(f.read()).hexdigest()
    rehearsal = bool(args.collective_lib)
    if rehearsal:
        mcpt.set_collective_lib(args.collective_lib)
    ndev = torch.cuda.device_count()  # counts without initialising the GPU (no HIP call yet)
    devices = None  # the in-process device list (plain launch with --gpus > 1)
    if not launched and args.gpus > 1:
        if ndev < args.gpus and not rehearsal:
            raise SystemExit("bench.py --gpus %d: only %d GPUs visible" % (args.gpus, ndev))
        # rehearsal on fewer GPUs (test infrastructure): the list repeats devices and every entry is its own
        # rank of the (shim) communicator, MCPT_DEBUG_SHARD_RANKS
        devices = [k % max(ndev, 1) for k in range(args.gpus)]
        world = args.gpus
    if rehearsal:
        local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    if launched and world > 1:
        if rehearsal:  # RCCL refuses two ranks on one GPU: barrier and timing over gloo
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    comm = None
    comm_init_s = 0.0  # communicator creation: mcpt_comm_init_rank here, ncclCommInitAll in the first device-list call
    if devices is None:
        # the library's RCCL communicator (one rank per process); a 1-rank communicator at N=1
        uid = [mcpt.Comm.unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        tc = time.perf_counter()
        comm = mcpt.Comm(world, rank, uid[0], device=local)
        comm_init_s = time.perf_counter() - tc
    multi = dict(comm=comm) if devices is None else dict(devices=devices)
    list_flags = mcpt.DEBUG_SHARD_RANKS if devices is not None and rehearsal else 0

    def barrier():
        if launched and world > 1:
            dist.barrier()

    cfg = CONFIGS[args.config]
    W = args.width or cfg["width"]
    H = args.height or cfg["height"]
    if cfg["job_spp"]:  # strong scaling: the step's job is fixed, split over the ranks by the library
        if cfg["job_spp"] % world:
            raise SystemExit("--config %s: %d spp do not split over %d ranks" % (args.config, cfg["job_spp"], world))
        S = cfg["job_spp"] // world
    else:
        S = args.spp_per_step
    frame_spp = args.steps * world * S
    obj, xml, xml_cam = scene_files(args.scene)
    scene = mcpt.Scene.load(obj, xml)
    if xml_cam:  # the XML camera (main.cpp:512-513 for the Cornell scene): no pull-back
        cam = scene.camera()
        cam.width, cam.height = W, H
    else:
        cam = mcpt.Camera.reference(W, H)
    fb = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda")
    scratch = torch.zeros_like(fb)

    mode_flags = (mcpt.RENDER_FRESH_PDF if args.fresh_pdf else 0) | (
        mcpt.RENDER_PRECISION_FP32 if args.precision == "fp32" else 0) | (
        mcpt.DEBUG_NO_ROOT_CACHE if args.no_root_cache else 0) | args.debug_flags | list_flags
    flags = mcpt.RENDER_NO_BACKFACE_STATS | mode_flags
    setup_s = None  # the first call's device setup (scene upload, BVH, buffers): outside the timed region
    for k in range(args.warmup):  # warmup renders (same kernels and flags as the timed steps) go to scratch
        wst = mcpt.render_device(scene, cam, world * S, scratch.data_ptr(), mode=args.mode, seed=args.seed + 1,
                                 sample_range=(0, world * S), flags=flags, **multi)
        comm_init_s += wst.comm_init_seconds
        if setup_s is None:
            setup_s = wst.device_setup_seconds
    totals = {}
    per_dev = None  # per rank: sum over the timed steps of its shard wall time (mcpt_stats.device_seconds)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tlog = t0
    for k in range(args.steps):  # the job of step k: [k*G*S, (k+1)*G*S), S samples per rank, 1 reduce
        st = mcpt.render_device(scene, cam, frame_spp, fb.data_ptr(), mode=args.mode, seed=args.seed,
                                sample_range=(k * world * S, (k + 1) * world * S), flags=flags, **multi)
        for key, v in st.as_dict().items():
            totals[key] = totals.get(key, 0) + v
        pd = st.per_device_seconds()
        per_dev = pd if per_dev is None else [a + b for a, b in zip(per_dev, pd)]
        comm_init_s += st.comm_init_seconds  # 0 unless the timed steps created a communicator (they must not)
        # device time of the step: a device list runs its distinct devices concurrently, so its wall time on
        # each of them (the shards' kernel times are summed in the other fields)
        totals["device_seconds"] = totals.get("device_seconds", 0.0) + st.seconds * max(st.devices_used, 1)
        if rank == 0 and time.perf_counter() - tlog > 30:
            tlog = time.perf_counter()
            log("step %d/%d, %.1f s" % (k + 1, args.steps, tlog - t0))
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if launched and world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearsal else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # one process per GPU: every rank's shard time and communicator creation, gathered to all
        g = [None] * world
        dist.all_gather_object(g, (per_dev[0] if per_dev else 0.0, comm_init_s))
        per_dev = [x[0] for x in g]
        comm_init_s = max(x[1] for x in g)
    samples = float(W * H) * frame_spp
    value = samples / elapsed / 1e6
    # Untimed statistics replay: the same steps (same seed and sample ranges, so the same nodes and
    # rays) into the scratch buffer, with the light-side cull statistic on (the timed steps skip it,
    # mcpt_render_opts.flags) and the traversal kernel's node-visit / triangle-test counters
    # (MCPT_DEBUG_COUNT_TRAVERSAL); the work both runs counted must be identical.
    rep = {}
    for k in range(0 if args.no_replay else args.steps):
        st = mcpt.render_device(scene, cam, frame_spp, scratch.data_ptr(), mode=args.mode, seed=args.seed,
                                sample_range=(k * world * S, (k + 1) * world * S),
                                flags=mcpt.DEBUG_COUNT_TRAVERSAL | mode_flags, **multi)
        for key, v in st.as_dict().items():
            rep[key] = rep.get(key, 0) + v
    if not args.no_replay:
        for key in ("light_evals_total", "light_evals_candidates", "light_evals_survived", "prep_full_nodes", "rays",
                    "light_rays", "shading_nodes"):
            assert rep.get(key) == totals.get(key), (key, rep.get(key), totals.get(key))
        for key in ("light_evals_culled_backface", "light_evals_culled_plane", "node_visits", "tri_tests"):
            totals[key] = rep[key]

    log("rank %d totals: %s" % (rank, json.dumps({k: v for k, v in totals.items()})))
    if rank != 0:
        comm.close()
        dist.destroy_process_group()
        return
    pmc = load_json(os.path.join(ROOT, "profiles", "pmc_latest.json")) or {"kernels": {}}
    # the PMC figures of this workload when they were profiled (tools/summarize_profiles.py), else the
    # headline's
    wl = "brdf" if args.mode == "brdf" else ("cornell" if args.scene != "veach" else "c3")
    pk = pmc.get("configs", {}).get(wl, {}).get("kernels") or pmc["kernels"]
    # bounded VALU figure from the SQ pass (tools/summarize_profiles.py): 4 x SQ_INSTS_VALU / (SIMDs x
    # cycles) -- the issue slots the kernel's VALU instructions hold (>= 4 cycles each for wave64)
    def busy(*names):  # a name ending in "*>" matches any launch bound: "k_prep_pk2<*, false, true, false>"
        out = {}
        for n in names:
            head, _, tail = n.partition("*")
            for k, v in pk.items():
                if (k == n or (tail and k.startswith(head) and k.endswith(tail))) and v.get("valu_issue_frac") is not None:
                    out[k] = v["valu_issue_frac"]
        return out
    def pmc_src(*names):  # the summaries the matched kernels' PMC figures came from, and whether their binary is this one
        ks = [k for n in names for k in busy(n)]
        srcs = sorted({pk[k].get("source") or pmc.get("source") for k in ks})
        if not srcs:
            return None
        shas = {pk[k].get("lib_sha256") for k in ks}
        same = shas == {lib_sha}
        return "; ".join(s for s in srcs if s) + (" -- profiled binary sha256 %s %s this run's" % (
            "/".join(sorted(str(x)[:12] for x in shas)), "==" if same else "!="))
    def pmc_same_binary(*names):
        ks = [k for n in names for k in busy(n)]
        return bool(ks) and {pk[k].get("lib_sha256") for k in ks} == {lib_sha}
    dev_s = max(totals.get("device_seconds", 0.0), 1e-12)
    # ---- roofline of the light prep (rank 0's launches; HIP events on its stream) ----
    roof_prep = None
    prep_s = totals.get("prep_seconds", 0.0)
    if args.mode != "brdf" and prep_s > 0:
        ev_tot, c1, cand = (totals.get(k, 0) for k in ("light_evals_total", "light_evals_culled_backface",
                                                       "light_evals_candidates"))
        launches = max(totals.get("prep_launches", 0), 1)
        c2 = ev_tot - c1 - cand
        # the children's prep kernels: lane per node for small light tables (render.hip kSmallNL), else
        # the cull + wave-per-node pk2
        small = scene.nlights <= SMALL_NL
        prep_k = (("k_prep_lane<*, false>",) if small else
                  ("k_prep_cull_lanes<false>", "k_prep_pk2<*, false, true, %s>" % ("true" if args.precision == "fp32" else "false")))
        flops = c1 * FLOPS_CULL_BACKFACE + c2 * FLOPS_CULL_PLANE + cand * FLOPS_FULL
        t_launch = prep_s / launches
        achieved = flops / launches / t_launch / 1e12
        nodes = totals.get("prep_full_nodes", 0)
        traffic, tsrc = None, None
        hb = None if small else load_json(os.path.join(ROOT, "profiles", "k_prep_hbm_bytes_per_node.json"))
        lane_k = [k for k in busy(*prep_k) if pk[k].get("hbm_bytes_per_dispatch")] if small else []
        if lane_k:
            traffic = pk[lane_k[0]]["hbm_bytes_per_dispatch"]
            tsrc = "PMC profile, not this run: %s HBM bytes per dispatch (%s)" % (lane_k[0], pmc_src(*prep_k))
        elif hb and hb.get("hbm_bytes_per_node") is not None:
            traffic = hb["hbm_bytes_per_node"] * nodes / launches
            tsrc = ("PMC profile, not this run: %.1f HBM B/node (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                    "profiles/k_prep_hbm_bytes_per_node.json%s) x this run's %.0f full-prep nodes per launch"
                    % (hb["hbm_bytes_per_node"], ", profiled binary sha256 %s %s this run's" % (
                        str(hb.get("lib_sha256"))[:12], "==" if hb.get("lib_sha256") == lib_sha else "!="),
                       nodes / launches))
        alg_gbs = nodes * PREP_BYTES_PER_NODE / prep_s / 1e9
        # the opt-in fp32 precision runs the full stage in packed fp32: its roof is the fp32 vector peak
        fp32 = args.precision == "fp32"
        peak = FP32_VECTOR_PEAK_TFLOPS if fp32 else FP64_VECTOR_PEAK_TFLOPS
        roof_prep = {
            "bound": "valu_fp32" if fp32 else "valu_fp64", "kernel": "k_prep_lane" if small else "k_prep_cull_lanes+k_prep_pk2",
            "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": traffic, "traffic_source": tsrc,
            "valu_issue_frac": busy(*prep_k),
            "valu_issue_frac_source": pmc_src(*prep_k),
            "pmc_same_binary": pmc_same_binary(*prep_k) and bool(hb is None or hb.get("lib_sha256") == lib_sha),
            "hbm_frac_algorithmic": round(alg_gbs / HBM_PEAK_GBS, 5),
            "hbm_frac_measured": round(traffic / t_launch / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
            "avg_launch_ms": round(t_launch * 1e3, 3), "launches": launches, "flop_per_launch": flops / launches,
            "share_of_device_time": round(prep_s / dev_s, 3), "hbm_algorithmic_GBs": round(alg_gbs, 3),
            "full_prep_nodes": nodes, "cached_root_nodes": totals.get("prep_cached_nodes", 0),
            "hbm_peak_GBs": HBM_PEAK_GBS}
    # ---- roofline of the traversal kernel (k_mis_rays; BRDF-only: k_extend_brdf) ----
    roof_trace = None
    tr_s, tr_n = totals.get("trace_seconds", 0.0), max(totals.get("trace_launches", 0), 1)
    visits, tests = totals.get("node_visits", 0), totals.get("tri_tests", 0)
    if tr_s > 0 and visits > 0:
        accel = scene.accel_bytes()
        # the library traces MIS / shade rays with persistent refilling waves when the BVHs exceed an
        # XCD's 4 MiB L2 (render.hip MCPT_RAYS_PERSISTENT) and always for shade-area's rays
        # (MCPT_PERSIST_SHADE_AREA, round 5), one ray per thread otherwise
        pers = accel > (4 << 20) or args.mode == "shade_area"
        kname = "k_extend_brdf" if args.mode == "brdf" else ("k_rays_persistent" if pers else "k_mis_rays")
        t_launch = tr_s / tr_n
        fl = (visits * FLOPS_NODE_VISIT + tests * FLOPS_TRI_TEST_FP64 * 2) / tr_n
        by = (visits * BYTES_NODE_VISIT[kname] + tests * BYTES_TRI_TEST) / tr_n
        _, level, mem_peak = next(g for g in GATHER_PEAKS if accel <= g[0])
        v_frac, h_frac = fl / t_launch / 1e12 / FP32_VECTOR_PEAK_TFLOPS, by / t_launch / 1e9 / mem_peak
        valu_bound = v_frac >= h_frac
        pk_name = ("k_extend_brdf<false>" if args.mode == "brdf" else
                   "k_rays_persistent<false>" if pers else "k_mis_rays<false, false>")
        hbm_meas = pk.get(pk_name, {}).get("hbm_bytes_per_dispatch")
        # the fetch model against the HBM peak is meaningful only when the structure lives in HBM; a
        # cache-resident tree (Veach: 0.5 MB in L2; Cornell-1M: 150 MB in the Infinity Cache) is
        # priced at its cache level above, and the HBM ratio of that model is not reported
        hbm_model = round(by / t_launch / 1e9 / HBM_PEAK_GBS, 4) if level == "hbm" else None
        roof_trace = {
            "bound": "valu" if valu_bound else level, "kernel": kname,
            "achieved": round(fl / t_launch / 1e12, 3) if valu_bound else round(by / t_launch / 1e9, 1),
            "peak": FP32_VECTOR_PEAK_TFLOPS if valu_bound else mem_peak,
            "unit": "TFLOP/s (fp32-equivalent: fp64 op = 2)" if valu_bound else "GB/s (node + triangle fetch model)",
            "frac": round(max(v_frac, h_frac), 4), "valu_frac": round(v_frac, 4), "mem_model_frac": round(h_frac, 4),
            "accel_bytes": accel, "bytes_per_node_visit": BYTES_NODE_VISIT[kname], "structure_level": level,
            "hbm_model_frac": hbm_model,
            "traffic": hbm_meas, "traffic_source": ("PMC profile, not this run: %s" % pmc_src(pk_name)) if hbm_meas else None,
            "valu_issue_frac": busy(pk_name), "valu_issue_frac_source": pmc_src(pk_name),
            "pmc_same_binary": pmc_same_binary(pk_name),
            "avg_launch_ms": round(t_launch * 1e3, 3), "launches": tr_n,
            "node_visits_per_ray": round(visits / max(totals.get("rays", 0) + totals.get("light_rays", 0), 1), 2),
            "tri_tests_per_ray": round(tests / max(totals.get("rays", 0) + totals.get("light_rays", 0), 1), 2),
            "share_of_device_time": round(tr_s / dev_s, 3)}
    # the line's roofline is the kernel with the larger share of device time
    cands = [r for r in (roof_prep, roof_trace) if r]
    roofline = max(cands, key=lambda r: r["share_of_device_time"]) if cands else None

    cpu = None
    l2 = l2max = None
    if world == 1 and not args.no_cpu:
        log("cpu baseline (<= ~%.0f + %.0f s) ..." % (args.cpu_seconds, args.cpu_single_seconds))
        cpu, cimg, cspp = cpu_baseline(args.scene, W, H, args.mode, args.seed, S, args.cpu_seconds,
                                       args.cpu_single_seconds)
        g, _ = mcpt.render(scene, cam, cspp, mode=args.mode, seed=args.seed, device=local, flags=mode_flags)
        sub = (slice(7, None, 20), slice(7, None, 20))
        l2 = rel_l2(g[sub], cimg[sub])
        l2max = max_px_rel(g[sub], cimg[sub])
        cpu["gpu_over_single_thread"] = round(value / cpu["value"], 1)
        cpu["gpu_over_host_threads"] = round(value / cpu["multi_thread_value"], 1)
    if args.out:
        mcpt.write_bmp(args.out, mcpt.tone_map(fb.cpu().numpy()))
    line = {
        "metric": SCENES[args.scene][0], "value": round(value, 4), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": cfg["scaling"],
        # BASELINE.md publishes no number for this metric (only render times of another frame on unstated
        # hardware), so there is nothing to divide by; the GPU/CPU ratios live in cpu_baseline
        "vs_baseline": None,
        "dtype": "f64" if args.precision == "fp64" else "f64 (light-prep weights f32, MCPT_RENDER_PRECISION_FP32)",
        "data": SCENES[args.scene][1],
        "config": {"workload": "%s %s %dx%d" % ("veach-mis" if args.scene == "veach" else "cornell-1M", args.mode.upper(), W, H),
                   "config": args.config, "width": W, "height": H,
                   "mode": args.mode, "spp_per_step": S, "frame_spp": frame_spp, "seed": args.seed,
                   "precision": args.precision, "root_cache": not args.no_root_cache,
                   "parallelism": ("sample-shard x%d + 1 RCCL reduce per step (library mcpt_comm, one process per GPU)" % world
                                   if devices is None else
                                   "sample-shard x%d + 1 grouped RCCL reduce per step (library device list %s, one process)"
                                   % (world, devices)) + (
                       " [rehearsal: collective %s, ranks sharing GPUs]" % os.path.basename(args.collective_lib)
                       if rehearsal else ""),
                   "launch": "torchrun" if launched else "single process",
                   "job_spp_per_step": world * S},
        "roofline": roofline,
        "roofline_prep": roof_prep,
        "roofline_trace": roof_trace,
        "cpu_baseline": cpu,
        "l2_vs_cpu": l2,
        "l2_vs_cpu_max_pixel": l2max,
        "device_seconds": round(totals.get("seconds", 0.0), 4),
        "samples": samples,
        "lib_sha256": lib_sha,
        # where a multi-GPU step's time went (mcpt_stats ABI 2.2): each rank's shard wall time summed over the
        # timed steps (setup and reduce excluded; max/min = load imbalance), the reduces' time, and -- outside the
        # timed region -- the communicator's creation and the first call's device setup
        "per_device_seconds": [round(v, 4) for v in (per_dev or [])],
        "device_imbalance": round(max(per_dev) / max(min(per_dev), 1e-12), 4) if per_dev else None,
        "reduce_seconds": round(totals.get("reduce_seconds", 0.0), 4),
        "comm_init_seconds": round(comm_init_s, 4),
        "device_setup_seconds": round(setup_s, 4) if setup_s is not None else None,
    }
    print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if launched and world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
