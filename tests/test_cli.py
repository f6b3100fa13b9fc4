"""The host C++ driver `mcpt_render` (csrc/mcpt_cli.cpp: the reference's main(), main.cpp:497-600,
as a program over the C ABI) end to end on the GPU: its HDR output equals the Python mirror's
render of the same (scene, camera, spp, mode, seed), its BMP equals the tone-mapped frame, and its
flags (--mode, --grid, --progress, errors) behave."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, SCENE_OBJ, SCENE_XML
import monte_carlo_path_tracing_amd as mcpt

pytestmark = pytest.mark.gpu
CLI = os.path.join(ROOT, "monte_carlo_path_tracing_amd", "mcpt_render")
SCENE_BASE = os.path.splitext(str(SCENE_OBJ))[0]


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), dtype="<f4" if scale < 0 else ">f4").reshape(h, w, 3)
    return data[::-1].astype(np.float64)  # PFM rows are bottom-up


def run_cli(tmp_path, *args):
    bmp, pfm = str(tmp_path / "out.bmp"), str(tmp_path / "out.pfm")
    r = subprocess.run([CLI, "--scene", SCENE_BASE, "--out", bmp, "--hdr", pfm, *args], capture_output=True,
                       text=True, timeout=120)
    return r, bmp, pfm


@pytest.mark.parametrize("mode", ["mis", "shade", "brdf"])
def test_cli_matches_python_render(tmp_path, mode):
    r, bmp, pfm = run_cli(tmp_path, "--width", "64", "--height", "48", "--spp", "4", "--mode", mode, "--seed", "7")
    assert r.returncode == 0, r.stderr
    hdr = read_pfm(pfm)
    scene = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    ref, _ = mcpt.render(scene, mcpt.Camera.reference(64, 48), 4, mode=mode, seed=7)
    assert np.allclose(hdr, ref.astype(np.float32), rtol=1e-6, atol=1e-30)  # PFM stores fp32
    with open(bmp, "rb") as f:
        data = f.read()
    tm = mcpt.tone_map(ref)
    mcpt.write_bmp(str(tmp_path / "py.bmp"), tm)
    with open(tmp_path / "py.bmp", "rb") as f:
        assert f.read() == data  # identical file: header, BGRA layout, pixels


def test_cli_grid_and_progress(tmp_path):
    r, _, pfm = run_cli(tmp_path, "--width", "32", "--height", "24", "--spp", "4", "--grid", "--progress")
    assert r.returncode == 0, r.stderr
    assert "100%" in r.stderr
    hdr = read_pfm(pfm)
    scene = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    ref, _ = mcpt.render(scene, mcpt.Camera.reference(32, 24), 4, accel="grid")
    assert np.allclose(hdr, ref.astype(np.float32), rtol=1e-6, atol=1e-30)


def test_cli_precision_fp32(tmp_path):
    """--precision fp32 = MCPT_RENDER_PRECISION_FP32 (the opt-in FP32_STABLE light prep)"""
    r, _, pfm = run_cli(tmp_path, "--width", "48", "--height", "36", "--spp", "4", "--mode", "mis", "--precision", "fp32")
    assert r.returncode == 0, r.stderr
    hdr = read_pfm(pfm)
    scene = mcpt.Scene.load(SCENE_OBJ, SCENE_XML)
    ref, _ = mcpt.render(scene, mcpt.Camera.reference(48, 36), 4, flags=mcpt.RENDER_PRECISION_FP32)
    assert np.allclose(hdr, ref.astype(np.float32), rtol=1e-6, atol=1e-30)
    r = subprocess.run([CLI, "--precision", "fp16"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2


def test_cli_errors(tmp_path):
    r = subprocess.run([CLI, "--scene", str(tmp_path / "missing")], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "scene load failed" in r.stderr
    r = subprocess.run([CLI, "--mode", "nope"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
