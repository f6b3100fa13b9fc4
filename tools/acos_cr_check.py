"""Host check of csrc/acos_cr.h against mpmath (correctly rounded acos) and glibc's acos.

Builds tools/acos_cr_check.cpp with g++, feeds it random arguments over [-1, 1] (uniform, clustered
near -1, 0, 1, and the literal chain's vertex-angle arguments' typical range), and reports how often
acos_cr, its variants started 1-2 ulp off, and glibc differ from the correctly rounded value.

    python tools/acos_cr_check.py [n]
"""
import os
import subprocess
import sys
import tempfile

import mpmath as mp
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    rng = np.random.default_rng(7)
    xs = np.concatenate([
        rng.uniform(-1, 1, n),
        1 - 10.0 ** rng.uniform(-16, -1, n // 4),
        -1 + 10.0 ** rng.uniform(-16, -1, n // 4),
        (2 * rng.integers(0, 2, n // 4) - 1) * 10.0 ** rng.uniform(-300, 0, n // 4),
        rng.uniform(-0.05, 0.05, n // 4),  # |x| near 0: z = y0^2 largest, the series' truncation largest
        np.array([0.0, -0.0, 0.5, -0.5, 1.0, -1.0, np.nextafter(1, 0), np.nextafter(-1, 0), 1e-300, -1e-300]),
    ])
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "chk")
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I",
                               os.path.join(ROOT, "monte_carlo_path_tracing_amd", "csrc"), "-o", exe,
                               os.path.join(ROOT, "tools", "acos_cr_check.cpp")])
        xs.astype(np.float64).tofile(os.path.join(d, "x.bin"))
        subprocess.check_call([exe, os.path.join(d, "x.bin"), os.path.join(d, "y.bin")])
        out = np.fromfile(os.path.join(d, "y.bin")).reshape(-1, 6)
    mp.mp.prec = 200
    cr = np.array([float(mp.acos(mp.mpf(float(x)))) for x in xs])
    names = ["acos_cr", "glibc", "start-2ulp", "start-1ulp", "start+1ulp", "start+2ulp"]
    for k, name in enumerate(names):
        bad = out[:, k] != cr
        print("%-11s differs from correctly rounded on %d of %d" % (name, int(bad.sum()), len(xs)))
        if bad.any() and k != 1:
            j = np.nonzero(bad)[0][:5]
            for i in j:
                print("   x %r: got %r want %r" % (xs[i], out[i, k], cr[i]))
    return 0 if not (out[:, [0, 2, 3, 4, 5]] != cr[:, None]).any() else 1


if __name__ == "__main__":
    sys.exit(main())
