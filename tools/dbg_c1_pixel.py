"""Debug: the C1 MIS pixel with the largest GPU-vs-oracle relative error, sample by sample."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import monte_carlo_path_tracing_amd as mcpt
from oracle import pyoracle as po
W, H, SPP, SEED = 400, 300, 4, 20240430
d = "scenes/veach-mis"
obj, xml = d + "/veach-mis.obj", d + "/veach-mis.xml"
s = po.Scene(obj, xml)
cam = po.reference_camera(W, H)
e, _ = po.camera_ray(cam, 0, 0)
s.build_grid(e)
ref, _ = s.render(cam, po.MODE_MIS, SEED, SPP, nthreads=16)
g = mcpt.Scene.load(obj, xml)
img, _ = mcpt.render(g, mcpt.Camera.reference(W, H), SPP, mode="mis", seed=SEED)
dd = np.linalg.norm((img - ref).reshape(-1, 3), axis=1)
nn = np.linalg.norm(ref.reshape(-1, 3), axis=1)
rel = np.where(nn > 0, dd / np.maximum(nn, 1e-300), 0)
order = np.argsort(-rel)[:5]
for q in order:
    i, j = divmod(int(q), W)
    print("pixel (%d,%d) rel %.3e gpu %s ref %s" % (i, j, rel[q], img[i, j], ref[i, j]))
q = int(order[0])
i, j = divmod(q, W)
for k in range(SPP):
    gk, _ = mcpt.render(g, mcpt.Camera.reference(W, H), SPP, mode="mis", seed=SEED, sample_range=(k, k + 1))
    ok_, _ = s.render(cam, po.MODE_MIS, SEED, SPP, s0=k, s1=k + 1, nthreads=16)
    print("sample %d: gpu %s oracle %s" % (k, gk[i, j] * SPP, ok_[i, j] * SPP))
    rgb, _ = s.shade_sample(cam, po.MODE_MIS, po.RNG_COUNTER, SEED, i, j, sample=k)
    print("   oracle shade_sample %s" % rgb)
