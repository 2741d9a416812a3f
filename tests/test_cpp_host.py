"""The C++ host (include/eray/, eray_amd/host/): its unit tests (tests/cpp/test_host.cpp, which
mirror the reference's graph / shader / image tests) on CPU, and on the GPU the shaderlib graph,
a render through the Engine API and main.rs's CLI against the golden digests."""
import hashlib
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "eray_amd", "bin")


@pytest.fixture(scope="module")
def host_bins():
    from eray_amd import build as B
    B.build_host()
    return {n: os.path.join(BIN, n) for n in ("test_host", "eray_main")}


def _digests():
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        return json.load(f)


def _sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def test_host_unit_tests_cpu(host_bins, tmp_path):
    r = subprocess.run([host_bins["test_host"], "--root", ROOT], capture_output=True, text=True, timeout=120,
                       cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed checks" in r.stdout


@pytest.mark.gpu
def test_host_unit_tests_gpu(host_bins, tmp_path):
    ppm = str(tmp_path / "c1.ppm")
    r = subprocess.run([host_bins["test_host"], "--gpu", "--root", ROOT, "--ppm", ppm], capture_output=True,
                       text=True, timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert _sha(ppm) == _digests()["c1"]["ppm_file_sha256"]


@pytest.mark.gpu
def test_main_rs_cli_output_ppm(host_bins, tmp_path):
    """eray_main = src/main.rs: cube.obj, the example material graph, 1024x1024 -> output.ppm, and
    the reference's debug side-effect files color.ppm (material.rs:41-50) and rgb.ppm (rgb.rs:96)
    in the working directory."""
    out = str(tmp_path / "output.ppm")
    r = subprocess.run([host_bins["eray_main"], "--mesh", os.path.join(ROOT, "objects", "cube.obj"), "--output", out],
                       capture_output=True, text=True, timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    g = _digests()["main_rs"]
    assert _sha(out) == g["ppm_file_sha256"]
    assert _sha(str(tmp_path / "color.ppm")) == g["color_ppm_sha256"]
    assert _sha(str(tmp_path / "rgb.ppm")) == g["rgb_ppm_sha256"]
