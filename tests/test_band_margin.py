"""The exact pick's ambiguity band bounds the fast-vs-reference prefix-sum difference.

tools/band_margin_study.py compares, at random shading points, every prefix sum of the renderer's light
weights (Van Oosterom-Strackee excess, device_math.h sph_excess, in long double) with the reference's
(the oracle's literal acos chain, Mylight.cpp:375-398) and divides by the band the kernels compute with
the constants they are built with (read from csrc).  A margin below 1 means a pick could be taken from
the fast weights where the reference picks another light.  CPU only: loads the oracle, no GPU.
"""
import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import band_margin_study as bms  # noqa: E402
import scenegen  # noqa: E402


def test_study_uses_the_kernels_constants():
    assert (bms.KAPPA, bms.SLIVER, bms.TAU) == bms.kernel_constants()
    assert bms.SLIVER >= 0.5 and bms.TAU <= 300.0


@pytest.mark.parametrize("seed", [11, 26, 37])
def test_band_covers_the_sliver_scene(seed):
    # seed 26 is the point set whose worst point exceeded the round-3 band (sliver 0.25, tau 1000) 1.48x
    d = tempfile.mkdtemp()
    obj, xml = scenegen.STRESS["slivers"][0](os.path.join(d, "slivers"))
    r = bms.study(obj, xml, 300, seed=seed)
    assert r["points"] > 100
    assert r["margin"] >= 1.5, r


def test_band_covers_the_stand_in():
    r = bms.study(os.path.join(ROOT, "scenes/veach-mis/veach-mis.obj"),
                  os.path.join(ROOT, "scenes/veach-mis/veach-mis.xml"), 250, seed=11)
    assert r["points"] > 100 and r["margin"] >= 2.0, r
