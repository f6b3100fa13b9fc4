import sys, time, numpy as np
sys.path.insert(0, '.')
import monte_carlo_path_tracing_amd as m
s = m.Scene.load('scenes/veach-mis/veach-mis.obj', 'scenes/veach-mis/veach-mis.xml')
cam = m.Camera.reference(200, 150)
res = {}
for mode, spp in (("mis", 4096), ("brdf", 65536), ("shade", 4096)):
    t = time.time()
    img, st = m.render(s, cam, spp, mode=mode, seed=7)
    res[mode] = img
    print(mode, spp, "mean %.6f" % img.mean(), "time %.1fs" % (time.time() - t), flush=True)
np.save('gpurun_out/means_200x150.npy', np.stack([res["mis"], res["brdf"], res["shade"]]))
a, b = res["mis"], res["brdf"]
for name, sl in (("all", np.s_[:, :]), ("top", np.s_[:50, :]), ("mid", np.s_[50:100, :]), ("bot", np.s_[100:, :])):
    print(name, "mis %.6f brdf %.6f ratio %.4f" % (a[sl].mean(), b[sl].mean(), b[sl].mean() / a[sl].mean()))
