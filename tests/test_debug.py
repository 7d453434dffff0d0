"""Debug utilities (reference src/auxiliary/Debug.hh): tile maps with MOSI
states, liveness / layout checks, LAPACK tile diffs, allocator report."""
import numpy as np
import pytest

import slate_d35_amd as s
from slate_d35_amd.utils import debug


def _mat(target):
    A = s.Matrix(100, 70, 32, np.float64)
    A.insertLocalTiles(s.target_of(target))
    s._slate.generate_matrix_d("rands", A, 3, -1.0, s.opts(target))
    return A


def test_print_tiles_and_checks_host():
    A = _mat("h")
    txt = debug.print_tiles(A)
    lines = txt.strip().splitlines()
    assert len(lines) == 1 + 4                      # header + 4 tile rows
    assert all(len(l.split()) == 3 for l in lines[1:])
    assert "0:M-" in txt                            # host instance Modified, no device instance
    assert debug.check_tiles_lives(A) == 0
    assert debug.check_tiles_layout(A)


def test_diff_lapack_matrices():
    a = np.random.default_rng(0).standard_normal((70, 50))
    b = a.copy()
    b[40, 33] += 1.0                                # tile (1, 1) with 32 x 32 tiles
    nd, tmap = debug.diff_lapack_matrices(a, b, 32, 32)
    assert nd == 1
    assert tmap.splitlines() == ["..", ".#", ".."]
    nd, _ = debug.diff_lapack_matrices(a, b, 32, 32, tol=10.0)
    assert nd == 0


def test_on_off_and_mem_report(capfd):
    debug.on()
    try:
        assert debug.enabled()
        debug.print_tiles(_mat("h"))
        assert "tiles" in capfd.readouterr().out    # echoed when enabled
    finally:
        debug.off()
    assert not debug.enabled()
    assert "allocator" in debug.mem_report()
    assert debug.device_memory_leaks() >= 0 and debug.host_memory_leaks() >= 0


@pytest.mark.gpu
def test_debug_device():
    A = _mat("d")
    txt = debug.print_tiles(A)
    assert ":-M" in txt or ":IM" in txt or ":SM" in txt   # device instance Modified
    rep = debug.mem_report()
    assert "blocks" in rep and debug.device_memory_leaks() > 0   # A's device array is live
    del A
