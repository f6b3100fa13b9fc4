"""Debug: GPU vs oracle light prep at the nodes of the C1 worst sample (tools/_dbg_nodes.npy)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import monte_carlo_path_tracing_amd as mcpt
from oracle import pyoracle as po
d = "scenes/veach-mis"
obj, xml = d + "/veach-mis.obj", d + "/veach-mis.xml"
r = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_dbg_nodes.npy"))
g = mcpt.Scene.load(obj, xml)
s = po.Scene(obj, xml)
x1, n = r[:, 2:5].copy(), r[:, 5:8].copy()
u = np.full(len(r), 0.5)
ws, cnt, pick = mcpt.light_prep(g, x1, n, u)
for k in range(len(r)):
    o = s.light_prep(x1[k], n[k])
    print("node %d: gpu wsum %.12e count %d | oracle wsum %.12e count %d | rel %.3e" % (
        r[k, 0], ws[k], cnt[k], o[0], len(o[1]), abs(ws[k] - o[0]) / max(o[0], 1e-300)))
    if k == 2:
        oi, ow = np.array(o[1]), np.array(o[2])
        print("  oracle survivors", len(oi), "sum", ow.sum())
from monte_carlo_path_tracing_amd import rng
pix = 297 * 400 + 390
uu = np.array([rng.counter_u(rng.counter_key(20240430, pix, 3, int(r[k, 0])), 1) for k in range(len(r))])
ws2, cnt2, pick2 = mcpt.light_prep(g, x1, n, uu)
lf = s.lights()[0]
for k in range(len(r)):
    print("node %d: u %.17g gpu pick facet %d | oracle pick light %d = facet %d" % (
        r[k, 0], uu[k], pick2[k], r[k, 9], lf[int(r[k, 9])] if r[k, 9] >= 0 else -1))
