"""Multi-rank collective protocol of the library on ONE GPU (the reference's loop that
shards is main.cpp:557-588, single-threaded there, README.md:418).

RCCL refuses two ranks on one device, so these tests point the library at the test-only host-memory
collective tests/collshim/libmcpt_collshim.so (mcpt_debug_set_collective_lib, include/mcpt_debug.h),
which implements the NCCL entry points comm.cpp binds.  Everything above that line is the production
code the driver's 8-GPU run executes: render_rank's shard split, the in-place ncclReduce from a non-root
rank's library buffer (render.hip render_rank), the status slot that makes rank 0 report a failed peer,
comm_all_reduce_sum's ncclGroupStart / ncclReduce x N / ncclGroupEnd over an ncclCommInitAll
communicator (render_multi with MCPT_DEBUG_SHARD_RANKS), and bench.py --gpus N under torchrun.

Processes: world 2 and 4 on cuda:0 (gloo only broadcasts the communicator id).  Tolerances: frames vs
the single-call frame <= 1e-12 relative L2 (fp64 summation order is the only difference, the RNG is
keyed by the global sample index); the C4 split vs the CPU oracle <= 1e-3 frame and per pixel (north
star).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, SCENE_OBJ, SCENE_XML, TIGHT_L2, TIGHT_PX_FRAME
import monte_carlo_path_tracing_amd as mcpt

pytestmark = pytest.mark.gpu
SEED = 20240430
SHIM = str(ROOT / "tests" / "collshim" / "libmcpt_collshim.so")


def rel_l2(g, c):
    return float(np.linalg.norm(g - c) / max(np.linalg.norm(c), 1e-300))


def max_px_rel(g, c):
    d = np.linalg.norm((g - c).reshape(-1, 3), axis=1)
    n = np.linalg.norm(c.reshape(-1, 3), axis=1)
    return float(np.max(np.where(n > 0, d / np.maximum(n, 1e-300), np.where(d > 0, np.inf, 0.0))))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_WORKER = r"""
import json, os, sys
sys.path.insert(0, os.environ["MCPT_ROOT"])
import numpy as np
import torch
import torch.distributed as dist
import monte_carlo_path_tracing_amd as mcpt

mcpt.set_collective_lib(os.environ["SHIM"])
world, rank = int(os.environ["WORLD"]), int(os.environ["RANK"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%s" % os.environ["PORT"], rank=rank, world_size=world)
uid = [mcpt.Comm.unique_id() if rank == 0 else None]
dist.broadcast_object_list(uid, src=0)  # the only use of torch.distributed: the communicator id
comm = mcpt.Comm(world, rank, uid[0], device=0)
scene = mcpt.Scene.load(os.environ["OBJ"], os.environ["XML"])
out_dir = os.environ["OUT"]
res = {}
case = os.environ["CASE"]
if case == "protocol":
    cam = mcpt.Camera.reference(80, 60)
    # 1. the job split over the ranks, reduced into rank 0's buffer; other ranks' buffers unchanged
    sentinel = 7.25
    out = np.zeros((60, 80, 3)) if rank == 0 else np.full((60, 80, 3), sentinel)
    img, st = mcpt.render(scene, cam, 8, mode="mis", seed=20240430, out=out, comm=comm)
    res["camera_samples"] = int(st.camera_samples)
    res["reduce_seconds"] = st.reduce_seconds
    if rank == 0:
        np.save(os.path.join(out_dir, "mis.npy"), img)
    else:
        res["nonroot_unchanged"] = bool((img == sentinel).all())
    # 2. a device buffer (mcpt_render_device) and a sub-range of the job
    fb = torch.full((60, 80, 3), 0.0 if rank == 0 else sentinel, dtype=torch.float64, device="cuda:0")
    mcpt.render_device(scene, cam, 8, fb.data_ptr(), mode="brdf", seed=20240430, sample_range=(3, 7), comm=comm)
    torch.cuda.synchronize()
    if rank == 0:
        np.save(os.path.join(out_dir, "brdf_range.npy"), fb.cpu().numpy())
    else:
        res["nonroot_device_unchanged"] = bool((fb == sentinel).all().item())
    # 3. one rank's shard fails (its own progress callback cancels): it still joins the reduce, rank 0
    #    reports the failure and adds nothing, no rank hangs
    bad = world - 1
    out = np.zeros((60, 80, 3))
    try:
        mcpt.render(scene, cam, 8, mode="mis", seed=20240430, out=out, comm=comm, samples_per_launch=1,
                    progress=(lambda d, t: True) if rank == bad else None)
        res["fail_rc"] = "ok"
    except mcpt.MCPTError as e:
        res["fail_rc"] = str(e)
    res["fail_out_untouched"] = bool((out == 0).all())
    # 4. the communicator still works: the same frame as in 1
    img2, _ = mcpt.render(scene, cam, 8, mode="mis", seed=20240430, comm=comm)
    if rank == 0:
        np.save(os.path.join(out_dir, "mis_again.npy"), img2)
    # 5. an invalid option fails on every rank before the reduce
    try:
        mcpt.render(scene, cam, 8, mode="mis", seed=20240430, comm=comm, flags=1 << 12)
        res["invalid_rc"] = "ok"
    except mcpt.MCPTError as e:
        res["invalid_rc"] = str(e)
elif case == "c4":
    W, H, spp = 1600, 1200, 4
    cam = mcpt.Camera.reference(W, H)
    img, st = mcpt.render(scene, cam, spp, mode="mis", seed=20240430, comm=comm)
    res["camera_samples"] = int(st.camera_samples)
    res["cache_points"] = int(st.prep_cache_points)
    if rank == 0:
        np.save(os.path.join(out_dir, "c4_sub.npy"), img[7::20, 7::20])
with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
    json.dump(res, f)
comm.close()
scene.close()
dist.destroy_process_group()
"""


def run_world(tmp_path, world, case, timeout=240):
    script = tmp_path / "worker.py"
    script.write_text(_WORKER)
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MCPT_ROOT=str(ROOT), SHIM=SHIM, WORLD=str(world), RANK=str(r), PORT=str(port),
                   OBJ=SCENE_OBJ, XML=SCENE_XML, OUT=str(tmp_path), CASE=case, MCPT_COLLSHIM_TIMEOUT="90")
        procs.append(subprocess.Popen([sys.executable, "-u", str(script)], env=env))
    rcs = []
    try:
        for p in procs:
            rcs.append(p.wait(timeout=timeout))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world, rcs
    return [json.loads((tmp_path / ("rank%d.json" % r)).read_text()) for r in range(world)]


@pytest.fixture(scope="module")
def scene():
    return mcpt.Scene.load(SCENE_OBJ, SCENE_XML)


@pytest.fixture(scope="module")
def singles(scene):
    cam = mcpt.Camera.reference(80, 60)
    mis, _ = mcpt.render(scene, cam, 8, mode="mis", seed=SEED, device=0)
    brdf, _ = mcpt.render(scene, cam, 8, mode="brdf", seed=SEED, sample_range=(3, 7), device=0)
    return mis, brdf


@pytest.mark.parametrize("world", [2, 4])
def test_render_rank_multi_rank_protocol(tmp_path, singles, world):
    """render_rank with nranks > 1: each rank renders its shard of the job's sample range, the non-root
    ranks reduce in place from their library buffers into rank 0 (ncclReduce through the collective
    shim), and rank 0's frame equals the single call; non-root buffers are never written; a rank whose
    shard fails still joins the reduce, so rank 0 reports it (MCPT_E_DEVICE) and nobody hangs; the
    communicator is usable afterwards; an invalid option fails on every rank before the reduce."""
    res = run_world(tmp_path, world, "protocol")
    mis, brdf = singles
    got = np.load(tmp_path / "mis.npy")
    l2 = rel_l2(got, mis)
    print("world %d: MIS frame vs single call rel L2 %.3e" % (world, l2))
    assert l2 <= 1e-12
    assert rel_l2(np.load(tmp_path / "brdf_range.npy"), brdf) <= 1e-12
    assert rel_l2(np.load(tmp_path / "mis_again.npy"), mis) <= 1e-12
    assert sum(r["camera_samples"] for r in res) == 80 * 60 * 8  # every sample rendered once
    for r in res[1:]:
        assert r["nonroot_unchanged"] and r["nonroot_device_unchanged"]
    assert "%d of %d ranks failed" % (1, world) in res[0]["fail_rc"]
    assert "cancelled" in res[world - 1]["fail_rc"]
    for r in res[1:world - 1]:
        assert r["fail_rc"] == "ok"  # healthy non-root ranks: their part succeeded
    assert all(r["fail_out_untouched"] for r in res)
    assert all("flags" in r["invalid_rc"] for r in res)


_LIST_WORKER = r"""
import json, os, sys
sys.path.insert(0, os.environ["MCPT_ROOT"])
import numpy as np
import monte_carlo_path_tracing_amd as mcpt
mcpt.set_collective_lib(os.environ["SHIM"])
scene = mcpt.Scene.load(os.environ["OBJ"], os.environ["XML"])
cam = mcpt.Camera.reference(80, 60)
res = {}
for n in (2, 4):
    img, st = mcpt.render(scene, cam, 8, mode="mis", seed=20240430, devices=[0] * n, flags=mcpt.DEBUG_SHARD_RANKS)
    np.save(os.path.join(os.environ["OUT"], "list%d.npy" % n), img)
    res[str(n)] = dict(devices_used=st.devices_used, camera_samples=int(st.camera_samples), reduce=st.reduce_seconds)
import torch
fb = torch.zeros((60, 80, 3), dtype=torch.float64, device="cuda:0")
st = mcpt.render_device(scene, cam, 8, fb.data_ptr(), mode="mis", seed=20240430, devices=[0, 0, 0],
                        flags=mcpt.DEBUG_SHARD_RANKS)
torch.cuda.synchronize()
np.save(os.path.join(os.environ["OUT"], "list3_dev.npy"), fb.cpu().numpy())
res["3"] = dict(devices_used=st.devices_used, camera_samples=int(st.camera_samples), reduce=st.reduce_seconds)
with open(os.path.join(os.environ["OUT"], "list.json"), "w") as f:
    json.dump(res, f)
"""


def test_device_list_group_reduce_over_several_ranks(tmp_path, singles):
    """render_multi + comm_all_reduce_sum with 2, 3 and 4 communicator ranks (ncclCommInitAll, then
    ncclGroupStart / one ncclReduce per rank / ncclGroupEnd): every list entry its own rank
    (MCPT_DEBUG_SHARD_RANKS), ranks on the one device render one after another into their own buffers,
    and the grouped reduce sums them into the root's (host or device) buffer."""
    script = tmp_path / "list_worker.py"
    script.write_text(_LIST_WORKER)
    env = dict(os.environ, MCPT_ROOT=str(ROOT), SHIM=SHIM, OBJ=SCENE_OBJ, XML=SCENE_XML, OUT=str(tmp_path),
               MCPT_COLLSHIM_TIMEOUT="60")
    assert subprocess.run([sys.executable, "-u", str(script)], env=env, timeout=240).returncode == 0
    res = json.loads((tmp_path / "list.json").read_text())
    mis = singles[0]
    for n in (2, 3, 4):
        r = res[str(n)]
        img = np.load(tmp_path / ("list3_dev.npy" if n == 3 else "list%d.npy" % n))
        assert rel_l2(img, mis) <= 1e-12, n
        assert r["devices_used"] == n and r["camera_samples"] == 80 * 60 * 8 and r["reduce"] > 0


def test_c4_split_over_two_ranks_vs_oracle(tmp_path):
    """BASELINE C4's frame (1600x1200 MIS) with its job split over two ranks of one communicator (each
    rank its half of the samples and its own root-point cache), reduced into rank 0, against the CPU
    oracle on every 20th pixel in x and y at the same seed and samples."""
    from oracle import pyoracle as po
    res = run_world(tmp_path, 2, "c4", timeout=400)
    W, H, spp = 1600, 1200, 4
    assert sum(r["camera_samples"] for r in res) == W * H * spp
    assert all(r["cache_points"] > 0 for r in res)
    g = np.load(tmp_path / "c4_sub.npy")
    osc = po.Scene(SCENE_OBJ, SCENE_XML)
    ocam = po.reference_camera(W, H)
    e, _ = po.camera_ray(ocam, 0, 0)
    osc.build_grid(e)
    ref, _ = osc.render(ocam, po.MODE_MIS, SEED, spp, stride=20, offset=7, nthreads=16)
    c = ref[7::20, 7::20]
    l2, mx = rel_l2(g, c), max_px_rel(g, c)
    print("C4 1600x1200x%d MIS split over 2 ranks, subset vs oracle: rel L2 %.3e, max per-pixel %.3e" % (spp, l2, mx))
    assert l2 <= 1e-3 and mx <= 1e-3
    assert l2 <= TIGHT_L2 and mx <= TIGHT_PX_FRAME, (l2, mx)  # what the build achieves (tests/conftest.py)


def test_bench_two_ranks_under_torchrun(tmp_path):
    """bench.py --gpus 2 as the driver launches it (torch.distributed.run, one process per rank) on the
    one GPU, with the collective shim standing in for RCCL (--collective-lib): the rank split, the ONE
    reduce per step, the barrier + max-over-ranks timing and rank 0's JSON line."""
    port = free_port()
    out = tmp_path / "bench.log"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "1", "--spp-per-step", "8", "--no-cpu", "--collective-lib", SHIM]
    with open(out, "w") as f:
        rc = subprocess.run(cmd, stdout=f, stderr=subprocess.STDOUT, timeout=300,
                            env=dict(os.environ, MCPT_COLLSHIM_TIMEOUT="90")).returncode
    text = out.read_text()
    assert rc == 0, text[-3000:]
    line = json.loads([ln for ln in text.splitlines() if ln.startswith("{\"metric\"")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["samples"] == 800 * 600 * 2 * 8
    assert line["config"]["job_spp_per_step"] == 16
    # every rank's shard time, gathered over torch.distributed; mcpt_comm_init_rank timed by the caller
    assert len(line["per_device_seconds"]) == 2 and min(line["per_device_seconds"]) > 0
    assert line["comm_init_seconds"] > 0 and line["reduce_seconds"] > 0


def test_bench_plain_launch_uses_n_gpus(tmp_path):
    """`python3 bench.py --gpus 2` exactly as the driver invokes it -- no torchrun, no WORLD_SIZE: ONE
    process renders the job over the library's device list (one shard per GPU, ncclCommInitAll, one
    grouped reduce per step).  On this one-GPU box the two list entries share cuda:0 as two ranks of the
    collective shim (--collective-lib); the line must say n_gpus 2 and count both shards' samples."""
    out = tmp_path / "bench_plain.log"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--spp-per-step", "8", "--no-cpu", "--collective-lib", SHIM]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MCPT_COLLSHIM_TIMEOUT"] = "90"
    with open(out, "w") as f:
        rc = subprocess.run(cmd, stdout=f, stderr=subprocess.STDOUT, timeout=300, env=env).returncode
    text = out.read_text()
    assert rc == 0, text[-3000:]
    line = json.loads([ln for ln in text.splitlines() if ln.startswith("{\"metric\"")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["samples"] == 800 * 600 * 2 * 8
    assert line["config"]["job_spp_per_step"] == 16 and line["config"]["launch"] == "single process"
    assert "device list [0, 0]" in line["config"]["parallelism"]



@pytest.mark.parametrize("config", ["c3", "c4"])
def test_bench_plain_launch_eight_ranks(tmp_path, config):
    """The driver's whole-node command, `python3 bench.py --gpus 8` (no torchrun), rehearsed on the one GPU:
    one process, a device list of 8 entries, each its own rank of an 8-rank ncclCommInitAll clique of the
    collective shim (RCCL refuses ranks sharing a device), one grouped reduce per step.  c3: 8 x 800x600 x S
    samples per step (weak scaling); c4: BASELINE's C4 job, 1600x1200 x 4096 spp per step split into 8
    shards of 512 spp (strong scaling).  The line must carry per-rank shard times, the reduce time and the
    communicator's creation time (created before any device work, outside the timed region)."""
    out = tmp_path / ("bench_plain8_%s.log" % config)
    extra = ["--spp-per-step", "2"] if config == "c3" else ["--config", "c4"]
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1", "--no-cpu",
           "--no-replay", "--collective-lib", SHIM] + extra
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MCPT_COLLSHIM_TIMEOUT"] = "120"
    with open(out, "w") as f:
        rc = subprocess.run(cmd, stdout=f, stderr=subprocess.STDOUT, timeout=420, env=env).returncode
    text = out.read_text()
    assert rc == 0, text[-3000:]
    line = json.loads([ln for ln in text.splitlines() if ln.startswith("{\"metric\"")][-1])
    print("bench --gpus 8 --config %s (rehearsal): %.1f Msamples/s, per rank %s s, reduce %.4f s, comm init %.4f s, "
          "setup %.3f s" % (config, line["value"], line["per_device_seconds"], line["reduce_seconds"],
                            line["comm_init_seconds"], line["device_setup_seconds"]))
    samples = 8 * 800 * 600 * 2 if config == "c3" else 1600 * 1200 * 4096
    assert line["n_gpus"] == 8 and line["value"] > 0 and line["samples"] == samples
    assert line["config"]["launch"] == "single process" and line["config"]["config"] == config
    assert "device list [0, 0, 0, 0, 0, 0, 0, 0]" in line["config"]["parallelism"]
    assert line["config"]["job_spp_per_step"] == (16 if config == "c3" else 4096)
    assert line["config"]["spp_per_step"] == (2 if config == "c3" else 512)
    pd = line["per_device_seconds"]
    assert len(pd) == 8 and min(pd) > 0 and line["device_imbalance"] >= 1.0
    assert line["comm_init_seconds"] > 0 and line["reduce_seconds"] > 0 and line["device_setup_seconds"] is not None
