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
