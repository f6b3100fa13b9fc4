"""GPU diagnostics: the light prep at the nodes of C1's former outlier sample (pixel (297, 390), sample 3,
MIS; nodes from the oracle's orc_debug_mis_sample) through the renderer's prep (band + exact fallback),
the exact fallback alone and the oracle, and that sample's radiance GPU vs oracle.  Test infrastructure.
"""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, ".")
import monte_carlo_path_tracing_amd as mcpt  # noqa: E402
from monte_carlo_path_tracing_amd import rng  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

OBJ, XML = "scenes/veach-mis/veach-mis.obj", "scenes/veach-mis/veach-mis.xml"
W, H, SEED, I, J, K = 400, 300, 20240430, 297, 390, 3

s = po.Scene(OBJ, XML)
cam = po.reference_camera(W, H)
e, _ = po.camera_ray(cam, 0, 0)
s.build_grid(e)
L = po.lib()
L.orc_debug_mis_sample.argtypes = [C.c_void_p, C.POINTER(po.Camera), C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_int,
                                   np.ctypeslib.ndpointer(np.float64, flags="C"), C.c_int]
rec = np.zeros(20 * 64)
nn = L.orc_debug_mis_sample(s.h, C.byref(cam), 0, SEED, I, J, K, rec, 64)
rec = rec.reshape(64, 20)[:nn]
g = mcpt.Scene.load(OBJ, XML)
x1, n = rec[:, 2:5].copy(), rec[:, 5:8].copy()
pix = I * W + J
u = np.array([rng.counter_u(rng.counter_key(SEED, pix, K, int(r[0])), 1) for r in rec])
ws, cnt, pick = mcpt.light_prep(g, x1, n, u)
we, ce, pe = mcpt.debug_light_prep_exact(g, x1, n, u)
for k in range(nn):
    o = s.light_sample_u(x1[k], n[k], u[k], 0.5, 0.5)
    print("node %d: u %.17g | renderer pick %d wsum %.17g | exact pick %d wsum %.17g | oracle pick %d wsum %.17g" % (
        rec[k, 0], u[k], pick[k], ws[k], pe[k], we[k], int(o[0]), o[5]))
gk, _ = mcpt.render(g, mcpt.Camera.reference(W, H), 4, mode="mis", seed=SEED, sample_range=(K, K + 1))
rgb, _ = s.shade_sample(cam, po.MODE_MIS, po.RNG_COUNTER, SEED, I, J, sample=K)
print("sample radiance gpu", gk[I, J] * 4, "oracle", rgb)
