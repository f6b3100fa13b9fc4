#!/usr/bin/env python3
"""High-spp GPU renders of the 32x24 G8 frame (tests/golden/stat_*_32x24x1024.npy), to tell noise
from bias when the 1024-spp reference statistics and the counter-RNG oracle disagree."""
import sys, os, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import monte_carlo_path_tracing_amd as m
s = m.Scene.load(ROOT + '/scenes/veach-mis/veach-mis.obj', ROOT + '/scenes/veach-mis/veach-mis.xml')
cam = m.Camera.reference(32, 24)
out = {}
for mode, spp in (("mis", 1 << 16), ("shade", 1 << 16), ("brdf", 1 << 20)):
    t = time.time()
    img, st = m.render(s, cam, spp, mode=mode, seed=99)
    g = np.load(ROOT + '/tests/golden/stat_%s_32x24x1024.npy' % mode)
    out[mode] = img
    print("%s %d spp: gpu mean %.6f  reference(1024 spp) %.6f  ratio %.4f  (%.1fs)" %
          (mode, spp, img.mean(), g[..., :3].mean(), g[..., :3].mean() / img.mean(), time.time() - t), flush=True)
np.save(ROOT + '/gpurun_out/g8_gpu.npy', np.stack([out["mis"], out["brdf"], out["shade"]]))
