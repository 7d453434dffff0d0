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


def test_tsan_threaded_runtime():
    """`make tsan`: every host source built with -fsanitize=thread, then the
    in-process ranks (run_in_process / ThreadComm), the scheduler lanes (p x q
    LU, Cholesky and QR with lookahead 1 and 2) and tile send / recv / bcast
    run on the host target on 1x2, 2x2 and 2x1 in-process grids.  Any data
    race TSan sees is fatal (halt_on_error); the residual checks must pass."""
    r = subprocess.run(["make", "-j8", "tsan"], cwd=ROOT, capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 history_size=4", OMP_NUM_THREADS="1")
    r = subprocess.run([os.path.join(ROOT, "bin", "tsan_check")], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "TSAN_CHECK OK" in out and "ThreadSanitizer" not in out, out[-6000:]
