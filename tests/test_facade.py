"""The C++ facade (include/tbdk.hpp) compiles against libtbdk.so and maps the
C status codes to exceptions; on a GPU box it runs a warp -> GFTT -> PyrLK
round trip through the cv::cuda-shaped classes."""
import os
import subprocess

import pytest

from opencv_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(tmp_path):
    exe = str(tmp_path / "facade_check")
    libdir = os.path.dirname(_lib.LIB_PATH)
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "facade_check.cpp"), "-L", libdir, "-ltbdk",
           f"-Wl,-rpath,{libdir}", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return exe


def test_facade_compiles_and_fails_loudly_without_gpu(tmp_path):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu variant")
    exe = build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "TBDK_ENODEV" in r.stdout


@pytest.mark.gpu
def test_facade_round_trip_on_gpu(tmp_path, gpu):
    exe = build(tmp_path)
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
