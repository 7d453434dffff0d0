"""Matrix class unit tests (reference unit_test/test_Matrix.cc semantics)."""
import numpy as np
import pytest

import slate_d35_amd as s
from helpers import rnd


def test_dims_and_tiles():
    A = s.Matrix(100, 70, nb=32)
    assert (A.m, A.n, A.mt, A.nt, A.mb, A.nb) == (100, 70, 4, 3, 32, 32)
    assert [A.tileMb(i) for i in range(4)] == [32, 32, 32, 4]
    assert [A.tileNb(j) for j in range(3)] == [32, 32, 6]
    assert A.tileIsLocal(0, 0) and A.tileRank(3, 2) == 0


def test_sub_slice_transpose():
    a = rnd(100, 70, np.float64, 1)
    A = s.from_numpy(a, nb=32)
    B = A.sub(1, 2, 0, 1)
    assert (B.m, B.n, B.mt, B.nt) == (64, 64, 2, 2)
    np.testing.assert_array_equal(s.to_numpy(B), a[32:96, 0:64])
    C = A.slice(5, 40, 3, 9)
    np.testing.assert_array_equal(s.to_numpy(C), a[5:41, 3:10])
    T = A.transpose()
    assert (T.m, T.n, T.mt, T.nt) == (70, 100, 3, 4)
    np.testing.assert_array_equal(s.to_numpy(T), a.T)


def test_conj_transpose_complex():
    a = rnd(20, 30, np.complex128, 2)
    A = s.from_numpy(a, nb=8)
    np.testing.assert_array_equal(s.to_numpy(A.conj_transpose()), a.conj().T)


def test_roundtrip_and_local_indices():
    a = rnd(50, 40, np.float32, 3)
    A = s.from_numpy(a, nb=16)
    assert A.local_row_indices() == list(range(50))
    np.testing.assert_array_equal(s.to_numpy(A), a)
    loc = A.get_local()
    np.testing.assert_array_equal(loc, a)


def test_empty_like_and_kinds():
    A = s.Matrix(64, 64, nb=16)
    A.insertLocalTiles()
    B = A.emptyLike()
    assert (B.m, B.n, B.nb) == (64, 64, 16)
    H = s.HermitianMatrix(s.Uplo.Lower, A)
    assert H.uplo == s.Uplo.Lower
    Tt = s.TriangularMatrix(s.Uplo.Upper, s.Diag.Unit, A)
    assert Tt.diag == s.Diag.Unit and Tt.uplo == s.Uplo.Upper
    with pytest.raises(Exception):
        s.HermitianMatrix(s.Uplo.General, A)


def test_set_and_norms():
    A = s.Matrix(30, 20, nb=8)
    A.insertLocalTiles()
    s.set(2.0, 5.0, A, target="h")
    a = s.to_numpy(A)
    ref = np.full((30, 20), 2.0); np.fill_diagonal(ref, 5.0)
    np.testing.assert_array_equal(a, ref)
    for kind, npk in [(s.Norm.Max, None), (s.Norm.One, 1), (s.Norm.Inf, np.inf), (s.Norm.Fro, "fro")]:
        v = s.norm(kind, A, target="h")
        r = np.abs(ref).max() if npk is None else np.linalg.norm(ref, npk)
        assert abs(v - r) < 1e-10 * max(1, r)


def test_set_lambda():
    A = s.Matrix(10, 12, nb=4)
    A.insertLocalTiles()
    s.set_lambda(lambda i, j: float(i * 100 + j), A)
    a = s.to_numpy(A)
    i, j = np.meshgrid(np.arange(10), np.arange(12), indexing="ij")
    np.testing.assert_array_equal(a, i * 100 + j)


def test_func_and_version():
    assert s.version()
    assert s.choose_grid(8) == (2, 4) and s.choose_grid(4) == (2, 2) and s.choose_grid(2) == (1, 2)


def test_inproc_allreduce_host():
    """The in-process transport's host mode (no GPU): all-reduce across rank threads."""
    import slate_d35_amd as s
    if s.device_available():
        pytest.skip("host-mode check")
    assert s._slate.inproc_allreduce_check(3, 5000) < 1e-12
    assert s._slate.inproc_allreduce_check(4, 1 << 18, 6) < 1e-12
