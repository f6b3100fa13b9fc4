"""Multi-rank sharding logic on CPU (gloo, world size 2): each rank renders its sample range of the
frame with the CPU oracle (this container has no GPU) and gloo sums them on rank 0.  The reduced
frame must equal the single-process frame (the RNG is keyed by the global sample index), which is
the property the library's RCCL paths rely on.  The same split on the HIP kernels -- two processes
on one GPU, the device-list path and the library communicator -- is tests/test_multi_gpu.py (-m gpu)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, SCENE_OBJ, SCENE_XML

W, H, SPP, SEED = 24, 18, 6, 20240430


def _worker(rank, world, port, out_path):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from shard import reduce_framebuffers, sample_range
    from oracle import pyoracle as po

    s = po.Scene(SCENE_OBJ, SCENE_XML)
    cam = po.reference_camera(W, H)
    e, _ = po.camera_ray(cam, 0, 0)
    s.build_grid(e)
    a, b = sample_range(rank, world, SPP)
    img, _ = s.render(cam, po.MODE_MIS, SEED, SPP, s0=a, s1=b, nthreads=1)
    fb = torch.from_numpy(img.copy())
    reduce_framebuffers(fb, dist, dst=0)
    if rank == 0:
        np.save(out_path, fb.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_sample_range_partition():
    from shard import sample_range
    for world in (1, 2, 3, 8):
        for spp in (0, 1, 7, 1024):
            for begin in (0, 5):
                r = [sample_range(k, world, spp, begin) for k in range(world)]
                assert r[0][0] == begin and r[-1][1] == begin + spp
                assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
                assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1
    with pytest.raises(ValueError):
        sample_range(2, 2, 8)


def test_two_rank_gloo_reduce_equals_single_process(tmp_path):
    out = str(tmp_path / "fb.npy")
    port = 29500 + os.getpid() % 1000
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    sys.path.insert(0, str(ROOT))
    from oracle import pyoracle as po

    s = po.Scene(SCENE_OBJ, SCENE_XML)
    cam = po.reference_camera(W, H)
    e, _ = po.camera_ray(cam, 0, 0)
    s.build_grid(e)
    full, _ = s.render(cam, po.MODE_MIS, SEED, SPP, nthreads=1)
    red = np.load(out)
    assert np.linalg.norm(red - full) / np.linalg.norm(full) < 1e-12

