import os
import pathlib
import sys

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
