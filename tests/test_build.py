"""Build-system checks (reference CMakeLists.txt / GNUmakefile): the CMake
project configures for gfx950 with the reference's option names."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not installed")
def test_cmake_configures():
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["cmake", "-S", ROOT, "-B", d, "-DCMAKE_HIP_COMPILER=/opt/rocm/llvm/bin/clang++",
                            "-Dbuild_tests=ON", "-Dc_api=ON"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        cache = open(os.path.join(d, "CMakeCache.txt")).read()
        assert "CMAKE_HIP_ARCHITECTURES:STRING=gfx950" in cache


def test_cmake_rejects_other_archs():
    if shutil.which("cmake") is None:
        pytest.skip("cmake not installed")
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["cmake", "-S", ROOT, "-B", d, "-DCMAKE_HIP_COMPILER=/opt/rocm/llvm/bin/clang++",
                            "-DCMAKE_HIP_ARCHITECTURES=gfx942"], capture_output=True, text=True, timeout=300)
        assert r.returncode != 0
