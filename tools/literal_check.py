"""GPU diagnostics (run on the box): the reference's literal light-prep chain on the GPU
(mcpt_debug_light_literal: fp64 sqrt, division, ocml acos) against the same formulas on the host
(numpy float64 in the reference's operation order, glibc acos through math.acos -- numpy's own
arccos is a vector implementation that is not glibc's) and the oracle's weights, at the golden
prep points -- locates the first intermediate that differs.  Test infrastructure (loads the oracle).

    python tools/literal_check.py [npoints]
"""
import math
import sys

import numpy as np

sys.path.insert(0, ".")
import monte_carlo_path_tracing_amd as mcpt  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

OBJ, XML = "scenes/veach-mis/veach-mis.obj", "scenes/veach-mis/veach-mis.xml"


def dot(a, b):
    return ((0.0 + a[..., 0] * b[..., 0]) + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def norm(a):
    l = np.sqrt(a[..., 0] * a[..., 0] + a[..., 1] * a[..., 1] + a[..., 2] * a[..., 2])
    return a / l[..., None]


def cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1], a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], -1)


_acos = np.vectorize(math.acos, otypes=[np.float64])


def main():
    npts = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    sc = mcpt.Scene.load(OBJ, XML)
    os_ = po.Scene(OBJ, XML)
    arr = sc.arrays()
    P = arr["positions"].astype(np.float64).reshape(-1, 3, 3)[arr["light_facet"]]
    pin = np.load("tests/golden/prep_in.npy")
    names = ["A", "B", "C", "a", "b", "c", "alpha", "beta", "gamma", "sA", "w", "alpha_arg", "BC"]
    diff = {k: 0 for k in names}
    wdiff = 0
    tot = 0
    for k in range(npts):
        x1, n = pin[k, :3], pin[k, 3:6]
        g = mcpt.debug_light_literal(sc, x1, n)
        ok = g[:, 0] == 0
        A, B, C = norm(P[:, 0] - x1), norm(P[:, 1] - x1), norm(P[:, 2] - x1)
        sw = dot(cross(norm(C - A), norm(B - A)), n) < 0
        B2, C2 = np.where(sw[:, None], C, B), np.where(sw[:, None], B, C)
        B, C = B2, C2
        h = {}
        h["A"], h["B"], h["C"] = A, B, C
        h["a"] = _acos(np.clip(dot(B, C), -1, 1))
        h["b"] = _acos(np.clip(dot(A, C), -1, 1))
        h["c"] = _acos(np.clip(dot(A, B), -1, 1))
        h["alpha_arg"] = -dot(norm(cross(B, A)), norm(cross(A, C)))
        h["BC"] = dot(B, C)
        h["alpha"] = _acos(np.clip(h["alpha_arg"], -1, 1))
        h["beta"] = _acos(np.clip(-dot(norm(cross(C, B)), norm(cross(B, A))), -1, 1))
        h["gamma"] = _acos(np.clip(-dot(norm(cross(A, C)), norm(cross(C, B))), -1, 1))
        h["sA"] = h["alpha"] + h["beta"] + h["gamma"] - 3.141592653589793
        gv = {"A": g[:, 1:4], "B": g[:, 4:7], "C": g[:, 7:10], "a": g[:, 10], "b": g[:, 11], "c": g[:, 12],
              "alpha": g[:, 13], "beta": g[:, 14], "gamma": g[:, 15], "sA": g[:, 16], "w": g[:, 17],
              "alpha_arg": g[:, 18], "BC": g[:, 19]}
        for key in names:
            if key == "w":
                continue
            a_, b_ = gv[key][ok], h[key][ok]
            bad = (a_ != b_) if a_.ndim == 1 else (a_ != b_).any(axis=1)
            diff[key] += int(bad.sum())
            if key in ("alpha", "alpha_arg") and bad.any() and k < 3:
                j = np.nonzero(bad)[0][:3]
                print(key, "gpu", a_[j], "host", b_[j])
        ws, idx, w = os_.light_prep(x1, n)
        gw = g[idx, 17]
        wdiff += int((gw != w).sum())
        tot += int(ok.sum())
    print("survivors compared: %d" % tot)
    for key in names:
        if key != "w":
            print("  %-9s differs on %d" % (key, diff[key]))
    print("  GPU literal w vs oracle w differ on %d" % wdiff)


if __name__ == "__main__":
    main()
