"""Multi-GPU paths of the C ABI on the HIP kernels (the reference loop that shards
is main.cpp:557-588, single-threaded in the reference, README.md:418).

The box these run on has ONE MI355X, so the device-list path is exercised with the device repeated:
devices=[0, 0] runs two sample-range shards (each a full wavefront render) into device 0's buffer
and then the library's RCCL ncclReduce over its ncclCommInitAll communicator (one distinct device
-> a 1-rank communicator); the multi-process path runs a 1-rank mcpt_comm, and two processes on
cuda:0 render their shards through the HIP path and sum host copies over gloo.  Every form must
equal the single-call frame to 1e-12 (fp64 summation order is the only difference, as the RNG is
keyed by the global sample index), and the C4-shaped frame (1600x1200) must match the CPU oracle on
its stride-20 pixel subset.

Tolerances: frame relative L2 <= 1e-12 between HIP renders; <= 1e-3 (north star) vs the oracle,
with the max per-pixel relative error reported and bounded the same way.

Not covered here (unpinned until the driver's 8-GPU run): a communicator with more than one rank.
RCCL refuses two ranks on the same GPU, so the non-root rank's in-place reduce (rank_fb) and
comm_all_reduce_sum's group over several devices never run on this one-GPU box; the 2-process test
sums host copies over gloo instead, and tests/test_distributed.py covers the rank split on CPU.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, SCENE_OBJ, SCENE_XML, TIGHT_L2, TIGHT_PX_FRAME
import monte_carlo_path_tracing_amd as mcpt
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
SEED = 20240430


def rel_l2(g, c):
    return float(np.linalg.norm(g - c) / max(np.linalg.norm(c), 1e-300))


def max_px_rel(g, c):
    """max over pixels of ||g_px - c_px|| / ||c_px|| (pixels black in both count 0)"""
    d = np.linalg.norm((g - c).reshape(-1, 3), axis=1)
    n = np.linalg.norm(c.reshape(-1, 3), axis=1)
    return float(np.max(np.where(n > 0, d / np.maximum(n, 1e-300), np.where(d > 0, np.inf, 0.0))))


@pytest.fixture(scope="module")
def scene():
    return mcpt.Scene.load(SCENE_OBJ, SCENE_XML)


@pytest.fixture(scope="module")
def single(scene):
    cam = mcpt.Camera.reference(80, 60)
    img, st = mcpt.render(scene, cam, 8, mode="mis", seed=SEED, device=0)
    return img, st


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_device_list_equals_single_call(scene, single, devices):
    cam = mcpt.Camera.reference(80, 60)
    img, st = mcpt.render(scene, cam, 8, mode="mis", seed=SEED, devices=devices)
    ref, st1 = single
    assert rel_l2(img, ref) <= 1e-12
    assert st.camera_samples == st1.camera_samples == 80 * 60 * 8
    assert st.devices_used == 1 and st.reduce_seconds > 0
    # the same shading nodes: each shard builds its own root-point cache (prep_cache_points per call)
    nodes = lambda t: t.prep_full_nodes - t.prep_cache_points + t.prep_cached_nodes  # noqa: E731
    assert nodes(st) == nodes(st1) and st.shading_nodes == st1.shading_nodes


def test_device_list_reports_where_the_time_went():
    """mcpt_stats ABI 2.2: the first device-list call over a device set creates the communicator
    (ncclCommInitAll, on the calling thread before any device work) and reports its wall time; the next
    call reuses it (0).  Per-rank shard times are recorded and lie within the call's wall time."""
    sc = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)  # its own handle: the communicator is cached per scene
    cam = mcpt.Camera.reference(80, 60)
    _, st1 = mcpt.render(sc, cam, 8, mode="mis", seed=SEED, devices=[0, 0])
    _, st2 = mcpt.render(sc, cam, 8, mode="mis", seed=SEED, devices=[0, 0])
    print("comm init %.4f s then %.4f s; setup %.4f / %.4f s; per device %s / %s; call %.4f / %.4f s" % (
        st1.comm_init_seconds, st2.comm_init_seconds, st1.device_setup_seconds, st2.device_setup_seconds,
        st1.per_device_seconds(), st2.per_device_seconds(), st1.seconds, st2.seconds))
    assert st1.comm_init_seconds > 0 and st2.comm_init_seconds == 0
    for st in (st1, st2):
        pd = st.per_device_seconds()
        assert len(pd) == 1 and 0 < pd[0] <= st.seconds and st.device_setup_seconds <= st.seconds
    assert st1.device_setup_seconds > st2.device_setup_seconds  # the first call uploads the scene
    sc.close()


def test_stats_written_only_up_to_the_callers_size(scene):
    """mcpt_render_opts.stats_size (ABI 2.2): a caller whose mcpt.h has a smaller mcpt_stats (2.1: up to
    prep_band_nodes) gets that prefix filled and nothing written past it"""
    import ctypes as C
    cam = mcpt.Camera.reference(16, 12)
    o = mcpt._opts(2, "mis", SEED, None, 0, 0, 0)
    o.stats_size = mcpt.Stats.comm_init_seconds.offset  # the 2.1 struct
    buf = (C.c_uint8 * (C.sizeof(mcpt.Stats) + 64))(*([0xAB] * (C.sizeof(mcpt.Stats) + 64)))
    out = np.zeros((12, 16, 3))
    rc = mcpt.lib().mcpt_render(scene.h, C.byref(cam), C.byref(o), out.reshape(-1), C.cast(buf, C.POINTER(mcpt.Stats)))
    assert rc == 0, mcpt.lib().mcpt_last_error()
    st = mcpt.Stats.from_buffer_copy(bytes(buf[:C.sizeof(mcpt.Stats)]))
    assert st.camera_samples == 16 * 12 * 2 and st.seconds > 0
    assert all(b == 0xAB for b in buf[o.stats_size:])


def test_device_list_into_device_buffer(scene, single):
    import torch
    cam = mcpt.Camera.reference(80, 60)
    fb = torch.zeros((60, 80, 3), dtype=torch.float64, device="cuda:0")
    st = mcpt.render_device(scene, cam, 8, fb.data_ptr(), mode="mis", seed=SEED, devices=[0, 0])
    torch.cuda.synchronize()
    assert rel_l2(fb.cpu().numpy(), single[0]) <= 1e-12 and st.devices_used == 1


def test_device_list_job_range_and_empty_shards(scene):
    """the device list splits the JOB's [sample_begin, sample_end); more shards than samples leaves
    some empty"""
    cam = mcpt.Camera.reference(40, 30)
    a, _ = mcpt.render(scene, cam, 8, seed=SEED, sample_range=(3, 5), device=0)
    b, st = mcpt.render(scene, cam, 8, seed=SEED, sample_range=(3, 5), devices=[0, 0, 0, 0])
    assert rel_l2(b, a) <= 1e-12 and st.camera_samples == 40 * 30 * 2


def test_comm_single_rank_equals_single_call(scene, single):
    uid = mcpt.Comm.unique_id()
    comm = mcpt.Comm(1, 0, uid, device=0)
    try:
        cam = mcpt.Camera.reference(80, 60)
        img, st = mcpt.render(scene, cam, 8, mode="mis", seed=SEED, comm=comm)
        assert rel_l2(img, single[0]) <= 1e-12
        assert st.reduce_seconds > 0 and st.camera_samples == 80 * 60 * 8
    finally:
        comm.close()


def test_device_list_rejects_bad_devices(scene):
    cam = mcpt.Camera.reference(8, 6)
    with pytest.raises(mcpt.MCPTError, match="no such device"):
        mcpt.render(scene, cam, 2, devices=[0, 4096])


def test_device_buffer_must_be_device_memory(scene):
    import ctypes as C
    cam = mcpt.Camera.reference(8, 6)
    host = np.zeros((6, 8, 3))
    with pytest.raises(mcpt.MCPTError, match="coarse-grained device memory"):
        mcpt.render_device(scene, cam, 2, host.ctypes.data_as(C.c_void_p).value, device=0)


_WORKER = r"""
import os, sys
sys.path.insert(0, os.environ["MCPT_ROOT"])
sys.path.insert(0, os.path.join(os.environ["MCPT_ROOT"], "tests"))
import numpy as np
import torch
import torch.distributed as dist
import monte_carlo_path_tracing_amd as mcpt
from shard import sample_range
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%s" % os.environ["PORT"],
                        rank=int(os.environ["RANK"]), world_size=2)
rank = dist.get_rank()
scene = mcpt.Scene.load(os.environ["OBJ"], os.environ["XML"])
cam = mcpt.Camera.reference(80, 60)
img, st = mcpt.render(scene, cam, 8, seed=20240430, sample_range=sample_range(rank, 2, 8), device=0)
t = torch.from_numpy(img)
dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
if rank == 0:
    np.save(os.environ["OUT"], t.numpy())
dist.destroy_process_group()
"""


def test_two_processes_render_hip_shards(tmp_path, single):
    """world size 2 on the one GPU: two processes each run the HIP path on their sample shard of the
    frame (main.cpp:557-588 split by sample), gloo sums the host copies"""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = tmp_path / "worker.py"
    script.write_text(_WORKER)
    out = tmp_path / "sum.npy"
    procs = []
    for r in range(2):
        env = dict(os.environ, MCPT_ROOT=str(ROOT), PORT=str(port), RANK=str(r), OBJ=SCENE_OBJ, XML=SCENE_XML,
                   OUT=str(out))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env))
    for p in procs:
        assert p.wait(timeout=110) == 0
    assert rel_l2(np.load(out), single[0]) <= 1e-12


def test_c4_frame_1600x1200_vs_oracle_subset(scene):
    """config C4's frame size (1600x1200, the root-point cache at 60 GB) on the device-list path,
    against the CPU oracle on every 20th pixel in x and y at the same seed and samples"""
    W, H, spp = 1600, 1200, 4
    cam = mcpt.Camera.reference(W, H)
    img, st = mcpt.render(scene, cam, spp, mode="mis", seed=SEED, devices=[0, 0])
    assert st.prep_cache_points > 0  # the root-point cache fits and was built
    osc = po.Scene(SCENE_OBJ, SCENE_XML)
    ocam = po.reference_camera(W, H)
    e, _ = po.camera_ray(ocam, 0, 0)
    osc.build_grid(e)
    ref, _ = osc.render(ocam, po.MODE_MIS, SEED, spp, stride=20, offset=7, nthreads=16)
    g, c = img[7::20, 7::20], ref[7::20, 7::20]
    l2, mx = rel_l2(g, c), max_px_rel(g, c)
    print("C4 1600x1200x%d MIS subset: rel L2 %.3e, max per-pixel %.3e" % (spp, l2, mx))
    assert l2 <= 1e-3 and mx <= 1e-3
    assert l2 <= TIGHT_L2 and mx <= TIGHT_PX_FRAME, (l2, mx)  # what the build achieves (tests/conftest.py)


def test_comm_failures_join_the_reduce_and_leave_the_comm_usable(scene, single):
    """A rank's failure never skips the collective (render_rank): options are validated on every rank
    before the reduce (an unknown flag fails alike everywhere), and a shard that fails later (here: its own
    progress callback cancels) still joins the reduce with a zero frame and the failure flag, so rank 0
    reports the failure instead of the peers hanging.  Multi-rank RCCL on distinct GPUs is the driver's
    8-GPU run; RCCL refuses two ranks on one device, so these run on a 1-rank communicator."""
    uid = mcpt.Comm.unique_id()
    comm = mcpt.Comm(1, 0, uid, device=0)
    try:
        cam = mcpt.Camera.reference(80, 60)
        with pytest.raises(mcpt.MCPTError, match="flags"):
            mcpt.render(scene, cam, 8, mode="mis", seed=SEED, comm=comm, flags=1 << 12)
        out = np.zeros((60, 80, 3))
        with pytest.raises(mcpt.MCPTError, match="cancelled"):
            mcpt.render(scene, cam, 8, mode="mis", seed=SEED, comm=comm, out=out, samples_per_launch=1,
                        progress=lambda d, t: True)
        assert not out.any()  # a failed job adds nothing to rank 0's buffer
        img, _ = mcpt.render(scene, cam, 8, mode="mis", seed=SEED, comm=comm)
        assert rel_l2(img, single[0]) <= 1e-12  # the communicator still works
    finally:
        comm.close()


def test_device_list_with_reference_grid(scene):
    """accel="grid" over a device list: the grid is built once on the calling thread before the device
    workers start (they only read it), and the frame equals the single-device grid render"""
    cam = mcpt.Camera.reference(40, 30)
    a, _ = mcpt.render(scene, cam, 4, mode="mis", seed=SEED, accel="grid", device=0)
    b, st = mcpt.render(scene, cam, 4, mode="mis", seed=SEED, accel="grid", devices=[0, 0])
    assert rel_l2(b, a) <= 1e-12 and st.camera_samples == 40 * 30 * 4


def test_c4_split_512spp_per_shard_reports_cache_build(scene):
    """BASELINE C4's split on the device-list path: a 1600x1200 job split into 512-spp shards (two on
    this one-GPU box; 8 x 512 = 4096 spp on the driver's node).  Each shard builds its own root-point
    cache over the 1.92 M pixels; the time it takes is reported (mcpt_stats.cache_build_seconds)."""
    W, H = 1600, 1200
    cam = mcpt.Camera.reference(W, H)
    img, st = mcpt.render(scene, cam, 1024, mode="mis", seed=SEED, devices=[0, 0])
    assert st.camera_samples == W * H * 1024 and np.isfinite(img).all() and img.mean() > 0
    assert st.prep_cache_points >= 2 * 0.9 * W * H  # both shards built the cache
    print("C4 split 2 x 512 spp at 1600x1200: %.2f Msamples/s (wall, incl. reduce); root-point cache build "
          "%.1f ms per shard of %.0f ms device time per shard" % (
              st.camera_samples / st.seconds / 1e6, 1e3 * st.cache_build_seconds / 2, 1e3 * st.seconds / 2))
