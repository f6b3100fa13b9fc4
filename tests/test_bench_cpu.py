"""bench.py's CPU-side contract (no GPU): the CPU baseline's two legs (the oracle on ONE
core, the reference's loop main.cpp:557-588 being single-threaded per README.md:418, beside the host's
thread share at full spp) and the launcher check of --gpus."""
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_cpu_baseline_single_thread_leg():
    out, img, spp = bench.cpu_baseline("veach", 80, 60, "mis", 20240430, 8, 5.0, 0.5)
    assert out["cores"] == 1 and out["kind"] == "port" and out["value"] == out["single_thread_value"] > 0
    assert out["multi_thread_value"] > 0 and out["multi_thread_cores"] >= 1 and spp == out["multi_thread_spp"]
    assert 1 <= out["single_thread_spp"] <= 8 and out["subset_pixels"] == len(range(7, 60, 20)) * len(range(7, 80, 20))
    assert out["reference_equivalent_value"] == out["value"] / out["oracle_over_reference_cross_host"]
    assert img.shape == (60, 80, 3) and img[7::20, 7::20].sum() > 0


def test_bench_gpus_must_match_launcher():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--no-cpu"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode != 0 and "--gpus 4" in r.stderr
