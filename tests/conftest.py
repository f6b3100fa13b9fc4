import os
import pathlib
import subprocess
import sys
import tempfile

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

GOLDEN = ROOT / "tests" / "golden"
SCENE_DIR = ROOT / "scenes" / "veach-mis"
SCENE_OBJ = str(SCENE_DIR / "veach-mis.obj")
SCENE_XML = str(SCENE_DIR / "veach-mis.xml")

# Parity gates.  The north star's statement is <= 1e-3 relative (frame L2 and per pixel); every frame test
# asserts it.  The build reproduces the oracle far more closely than that (fp64 throughout, picks exact), so
# the frame tests also assert what it achieves, with 10-100x margin over the round-4 measurements
# (profiles/round4m_gputests.log): frame relative L2 <= 1e-8 (measured <= 3.1e-10), max per-pixel <= 1e-6 on
# the stride-20 subsets and small frames (measured <= 3.2e-8), <= 2e-5 on whole 400x300 / 800x600 frames,
# whose worst pixels carry glibc-vs-correctly-rounded acos differences (measured 8.2e-7 / 2.4e-6).  A pick or
# ordering regression that moves any pixel by ~1e-5 fails these.
NORTH_STAR_TOL = 1e-3
TIGHT_L2 = 1e-8
TIGHT_PX = 1e-6
TIGHT_PX_FRAME = 2e-5


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "oracle: checks the CPU oracle against the reference goldens")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle and the native library once per session if they are missing."""
    if not (ROOT / "oracle" / "liboracle.so").exists():
        os.system("make -s -C %s" % (ROOT / "oracle"))
    yield


def cornell_scene(triangles, seed=20240430):
    """(obj, xml) of the Cornell + random-triangles stand-in (scenes/gen_cornell_random.py, config C5),
    generated once per (triangles, seed) into the temp directory."""
    d = pathlib.Path(tempfile.gettempdir()) / ("mcpt_cornell_%d_%d" % (triangles, seed))
    obj, xml = d / "cornell-random.obj", d / "cornell-random.xml"
    if not (obj.exists() and xml.exists()):
        subprocess.run([sys.executable, str(ROOT / "scenes" / "gen_cornell_random.py"), "--triangles",
                        str(triangles), "--seed", str(seed), str(d)], check=True, capture_output=True)
    return str(obj), str(xml)
