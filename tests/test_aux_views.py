"""Aux drivers on sliced trapezoid / general views whose diagonal does not run
through tile corners (row0 != col0): tzadd, set, scale must act on exactly the
view's triangle (reference src/add.cc, set.cc, scale.cc semantics)."""
import numpy as np
import pytest

import slate_d35_amd as s

G = None


def grid():
    return s._slate.Grid.self()


@pytest.mark.parametrize("uplo", ["L", "U"])
@pytest.mark.parametrize("off", [(0, 1), (3, 0), (2, 7), (5, 5)])
def test_tz_ops_on_offset_views(uplo, off):
    n, nb = 23, 4
    r0, c0 = off
    m2, n2 = n - r0 - 2, n - c0 - 1
    a0 = np.zeros((n, n)); b0 = np.arange(n * n, dtype=float).reshape(n, n) + 1
    U = s.Uplo.Lower if uplo == "L" else s.Uplo.Upper
    tri = np.tril if uplo == "L" else np.triu

    A = s.from_numpy(a0, nb=nb, grid=grid()); B = s.from_numpy(b0, nb=nb, grid=grid())
    TA = s.TrapezoidMatrix(U, s.Diag.NonUnit, A.slice(r0, r0 + m2 - 1, c0, c0 + n2 - 1))
    TB = s.TrapezoidMatrix(U, s.Diag.NonUnit, B.slice(r0, r0 + m2 - 1, c0, c0 + n2 - 1))
    s._slate.tzadd_d(2.0, TB, 1.0, TA, s.opts("h"))
    exp = a0.copy()
    exp[r0:r0 + m2, c0:c0 + n2] += 2 * tri(b0[r0:r0 + m2, c0:c0 + n2])
    np.testing.assert_array_equal(s.to_numpy(A), exp)

    s._slate.set_d(7.0, 9.0, TA, s.opts("h"))
    blk = exp[r0:r0 + m2, c0:c0 + n2]
    mask = tri(np.ones_like(blk)) > 0
    blk[mask] = 7.0
    np.fill_diagonal(blk, 9.0)
    np.testing.assert_array_equal(s.to_numpy(A), exp)

    s._slate.scale_d(3.0, 1.0, TA, s.opts("h"))
    blk[mask] *= 3
    np.testing.assert_array_equal(s.to_numpy(A), exp)


@pytest.mark.parametrize("off", [(0, 3), (6, 1)])
def test_general_set_diag_on_offset_view(off):
    n, nb = 19, 4
    r0, c0 = off
    A = s.from_numpy(np.zeros((n, n)), nb=nb, grid=grid())
    V = A.slice(r0, n - 1, c0, n - 1)
    s._slate.set_d(1.0, 5.0, V, s.opts("h"))
    exp = np.zeros((n, n))
    blk = exp[r0:, c0:]
    blk[:] = 1.0
    np.fill_diagonal(blk, 5.0)
    np.testing.assert_array_equal(s.to_numpy(A), exp)


@pytest.mark.parametrize("tg", ["h", pytest.param("d", marks=pytest.mark.gpu)])
def test_masked_norms_whole_block(tg):
    # Hermitian / unit-triangular norms on a 1 x 1 grid take the whole-block
    # path (one launch with the trapezoid mask); checked against numpy
    import subprocess, sys, os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "masked_norm_check.py"), tg],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "masked norms ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("n", [1, 2, 5])
def test_hermitian_max_norm_real_diagonal(n):
    """lanhe semantics: the Hermitian Max norm reads only Re of the diagonal,
    also for n == 1 (empty strict triangle)."""
    a = np.zeros((n, n), np.complex128)
    a[np.tril_indices(n, -1)] = 0.5 + 0.25j
    np.fill_diagonal(a, 0.75 + 3.0j)      # imaginary part must be ignored
    H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a, nb=2, grid=grid()))
    v = s.norm(s.Norm.Max, H, target="h")
    assert abs(v - 0.75) < 1e-15


def test_set_rectangular_tiles_equal_values():
    """set(offdiag == diag) on tiles that are not square (mb != nb): every
    tile is overwritten, including the columns left of the tile's diagonal
    run (regression: only the diagonal-run sub-block used to be written)."""
    A = s.Matrix(100, 100, 100, np.float64, mb=32)
    A.insertLocalTiles(s.Target.Host)
    A.set_local(np.asfortranarray(np.random.default_rng(0).random((100, 100))))
    s._slate.set_d(0.0, 0.0, A, s.opts("t"))
    assert np.abs(s.to_numpy(A)).max() == 0.0
    s._slate.set_d(2.0, 5.0, A, s.opts("t"))
    ref = np.full((100, 100), 2.0)
    np.fill_diagonal(ref, 5.0)
    assert np.array_equal(s.to_numpy(A), ref)
