"""debug: dump light-prep results and small renders of one library build (MCPT_LIB_PATH) to an
npz, or compare two such dumps:  dbg_cmp.py dump OUT.npz | dbg_cmp.py cmp A.npz B.npz"""
import sys, os, tempfile, numpy as np
root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, root); sys.path.insert(0, os.path.join(root, "tests"))
if sys.argv[1] == "cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        x, y = a[k], b[k]
        if x.dtype.kind == "f":
            print(k, "max abs diff %.3g" % np.max(np.abs(x - y)), "rel l2 %.3g" % (np.linalg.norm(x - y) / max(np.linalg.norm(x), 1e-300)))
        else:
            print(k, "mismatches", int((x != y).sum()), "of", x.size)
    sys.exit(0)
import monte_carlo_path_tracing_amd as mcpt
import scenegen
from conftest import SCENE_OBJ, SCENE_XML
d = tempfile.mkdtemp()
out = {}
for name, (obj, xml) in (("veach", (SCENE_OBJ, SCENE_XML)), ("panel", scenegen.light_panel(d))):
    s = mcpt.Scene.load(obj, xml)
    rng = np.random.default_rng(1)
    n = 2048
    x1 = np.stack([rng.uniform(-1.4, 1.4, n), np.zeros(n), rng.uniform(-1.4, 1.4, n)], 1)
    nn = np.tile([0.0, 1.0, 0.0], (n, 1))
    u = rng.uniform(0, 1, n)
    ws, cnt, pick = mcpt.light_prep(s, x1, nn, u)
    out[name + "_ws"], out[name + "_cnt"], out[name + "_pick"] = ws, cnt, pick
    g = s.camera()
    g.width, g.height = 16, 12
    for mode, spp in (("mis", 1), ("mis", 4), ("shade", 4)):
        img, st = mcpt.render(s, g, spp, mode=mode, seed=20240430)
        out["%s_%s%d" % (name, mode, spp)] = img
np.savez(sys.argv[2], **out)
