"""Calibration study for the light prep's exact-pick fallback.

The GPU's light weights (Van Oosterom-Strackee excess, device_math.h light_weight_bf) differ from
the reference's literal chain (Mylight.cpp:360-413: six acos, alpha+beta+gamma-pi) by rounding.  A
pick whose target u*W lies closer to a cumulative-weight boundary than the prefix sums' difference
can take the neighbouring triangle.  This script measures, on the CPU (oracle = literal chain,
numpy long double = the GPU formula without its rounding), how large that difference is against a
per-candidate error model

    m_i = u * lsum_i * (1 + d_i / l_i)        (u = 2^-53, d_i = |p0 - x1|, l_i = shortest edge)

and prints the constants the GPU's ambiguity band uses.  Test infrastructure only (it loads the
oracle); not part of the product.

    python tools/prep_error_study.py [npoints]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import pyoracle as po  # noqa: E402

U = 2.0 ** -53


def main():
    npts = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    s = po.Scene("scenes/veach-mis/veach-mis.obj", "scenes/veach-mis/veach-mis.xml")
    v, mat, light_of, un = s.facets()
    lf, la = s.lights()
    P = v[:, :9].astype(np.float64).reshape(-1, 3, 3)
    N = v[:, 9:].astype(np.float64).reshape(-1, 3, 3)
    LP = P[lf].astype(np.longdouble)
    lsum = la[:, 1] + la[:, 2] + la[:, 3]
    edges = np.stack([np.linalg.norm(P[lf, 1] - P[lf, 0], axis=1), np.linalg.norm(P[lf, 2] - P[lf, 1], axis=1),
                      np.linalg.norm(P[lf, 0] - P[lf, 2], axis=1)], 1)
    lmin = edges.min(1)
    rng = np.random.default_rng(11)
    nonlight = np.nonzero(light_of < 0)[0]
    area = 0.5 * np.linalg.norm(np.cross(P[nonlight, 1] - P[nonlight, 0], P[nonlight, 2] - P[nonlight, 0]), axis=1)
    pts = []
    gin = np.load("tests/golden/prep_in.npy")
    for k in range(min(len(gin), npts // 2)):
        pts.append((gin[k, :3], gin[k, 3:6]))
    while len(pts) < npts:
        f = nonlight[rng.choice(len(nonlight), p=area / area.sum())]
        b = rng.random(2)
        if b.sum() > 1:
            b = 1 - b
        x = (1 - b.sum()) * P[f, 0] + b[0] * P[f, 1] + b[1] * P[f, 2]
        n = (1 - b.sum()) * N[f, 0] + b[0] * N[f, 1] + b[1] * N[f, 2]
        n /= np.linalg.norm(n)
        pts.append((x, n))
    ratio_max, kappa_max, lin_max, rel_max = 0.0, 0.0, 0.0, 0.0
    worst = None
    for x1, n in pts:
        ws, idx, w = s.light_prep(x1, n)
        if len(idx) == 0:
            continue
        X = np.asarray(x1, np.longdouble)
        a, b, c = LP[idx, 0] - X, LP[idx, 1] - X, LP[idx, 2] - X
        A = a / np.sqrt((a * a).sum(1))[:, None]
        B = b / np.sqrt((b * b).sum(1))[:, None]
        Cc = c / np.sqrt((c * c).sum(1))[:, None]
        num = np.abs((A * np.cross(B, Cc)).sum(1))
        den = 1 + (A * B).sum(1) + (B * Cc).sum(1) + (Cc * A).sum(1)
        wv = 2 * np.arctan2(num, den) * lsum[idx].astype(np.longdouble)
        dw = (wv - w.astype(np.longdouble)).astype(np.float64)
        d = np.linalg.norm(P[lf[idx], 0] - x1, axis=1)
        m = U * lsum[idx] * (1 + d / lmin[idx])
        ratio_max = max(ratio_max, float(np.max(np.abs(dw) / m)))
        cref = np.cumsum(w)  # numpy cumsum of float64 is sequential: the oracle's order
        cv = np.cumsum(wv)
        err = np.abs((cv - cref.astype(np.longdouble)).astype(np.float64))
        sig = np.sqrt(np.sum(m * m))
        lin = np.sum(m)
        kap = float(err.max() / sig)
        if kap > kappa_max:
            kappa_max = kap
            worst = (x1, len(idx), err.max() / ws, sig / ws, lin / ws)
        lin_max = max(lin_max, float(err.max() / lin))
        rel_max = max(rel_max, float(err.max() / ws))
    print("points %d" % len(pts))
    print("max |dw_i| / m_i                       %.3f" % ratio_max)
    print("max prefix error / sqrt(sum m_i^2)      %.3f   (kappa)" % kappa_max)
    print("max prefix error / sum m_i              %.3e" % lin_max)
    print("max prefix error / W                    %.3e" % rel_max)
    print("worst kappa node: ncand %d, err/W %.2e, sigma/W %.2e, linear/W %.2e" % worst[1:])


if __name__ == "__main__":
    main()
