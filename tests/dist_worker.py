"""Multi-process driver checks, run under torch.distributed.run by test_dist.py
(reference test strategy: the tester with --grid p x q under mpirun, SURVEY.md
§4.1; here ranks talk over gloo host comms, or RCCL on a multi-GPU node).

usage: dist_worker.py P Q TARGET CASE[,CASE...]
Every rank computes the same global result from replicated inputs and checks
it against numpy; a failure raises (non-zero exit of that rank).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)

import torch  # noqa: F401,E402  (HIP runtime first)
import slate_d35_amd as s  # noqa: E402
from slate_d35_amd import parallel  # noqa: E402
from helpers import rnd, relerr, butterfly_dense  # noqa: E402


def tol(dt):
    return 5e-4 if dt in (np.float32, np.complex64) else 1e-11


def case_gemm(tg, dt, nb):
    a, b, c = rnd(150, 90, dt, 1), rnd(90, 120, dt, 2), rnd(150, 120, dt, 3)
    A, B, C = (s.from_numpy(x, nb=nb, target=tg) for x in (a, b, c))
    s.gemm(1.5, A, B, -0.5, C, target=tg)
    assert relerr(s.to_numpy(C), 1.5 * a @ b - 0.5 * c) < tol(dt)


def case_gemm_wide(tg, dt, nb):
    """SUMMA steps of w tiles (SLATE_SUMMA_K): one tile per step, 2 tiles
    (a short last step), all tiles in one step; tiles of the step come from
    different process columns / rows."""
    a, b, c = rnd(150, 7 * nb + 5, dt, 51), rnd(7 * nb + 5, 110, dt, 52), rnd(150, 110, dt, 53)
    old = os.environ.get("SLATE_SUMMA_K")
    try:
        for kk in (1, 2 * nb, 3 * nb, 100 * nb):
            os.environ["SLATE_SUMMA_K"] = str(kk)
            A, B, C = (s.from_numpy(x, nb=nb, target=tg) for x in (a, b, c))
            s.gemm(1.5, A, B, -0.5, C, target=tg, method_gemm="C")
            assert relerr(s.to_numpy(C), 1.5 * a @ b - 0.5 * c) < tol(dt), kk
    finally:
        if old is None:
            os.environ.pop("SLATE_SUMMA_K", None)
        else:
            os.environ["SLATE_SUMMA_K"] = old


def case_herk(tg, dt, nb):
    a = rnd(130, 70, dt, 4)
    A = s.from_numpy(a, nb=nb, target=tg)
    C = s.from_numpy(np.zeros((130, 130), dt), nb=nb, target=tg)
    H = s.HermitianMatrix(s.Uplo.Lower, C)
    s.herk(1.0, A, 0.0, H, target=tg)
    ref = a @ a.conj().T
    assert relerr(np.tril(s.to_numpy(C)), np.tril(ref)) < tol(dt)


def case_rank2k(tg, dt, nb):
    """syrk / her2k / syr2k on p x q grids (triangle-only SUMMA), both uplos, beta != 0."""
    n, k = 140, 60
    a, b = rnd(n, k, dt, 41), rnd(n, k, dt, 42)
    c0 = rnd(n, n, dt, 43)
    c0 = c0 + c0.conj().T
    for uplo, tri in ((s.Uplo.Lower, np.tril), (s.Uplo.Upper, np.triu)):
        C = s.from_numpy(c0, nb=nb, target=tg)
        s.syrk(1.5, s.from_numpy(a, nb=nb, target=tg), 0.5, s.SymmetricMatrix(uplo, C), target=tg)
        assert relerr(tri(s.to_numpy(C)), tri(1.5 * a @ a.T + 0.5 * c0)) < tol(dt), ("syrk", uplo)
        C = s.from_numpy(c0, nb=nb, target=tg)
        s.her2k(2.0, s.from_numpy(a, nb=nb, target=tg), s.from_numpy(b, nb=nb, target=tg), 0.5,
                s.HermitianMatrix(uplo, C), target=tg)
        ref = 2.0 * a @ b.conj().T + 2.0 * b @ a.conj().T + 0.5 * c0
        assert relerr(tri(s.to_numpy(C)), tri(ref)) < tol(dt), ("her2k", uplo)
        C = s.from_numpy(c0, nb=nb, target=tg)
        s.syr2k(1.0, s.from_numpy(a, nb=nb, target=tg), s.from_numpy(b, nb=nb, target=tg), -1.0,
                s.SymmetricMatrix(uplo, C), target=tg)
        ref = a @ b.T + b @ a.T - c0
        assert relerr(tri(s.to_numpy(C)), tri(ref)) < tol(dt), ("syr2k", uplo)


def case_trsm(tg, dt, nb):
    n = 140
    t = (np.tril(rnd(n, n, dt, 5)) / n + 2 * np.eye(n)).astype(dt)
    b = rnd(n, 60, dt, 6)
    T = s.TriangularMatrix(s.Uplo.Lower, s.Diag.NonUnit, s.from_numpy(t, nb=nb, target=tg))
    B = s.from_numpy(b, nb=nb, target=tg)
    s.trsm(s.Side.Left, 1.0, T, B, target=tg)
    assert relerr(t @ s.to_numpy(B), b) < tol(dt)
    # Right side (native column sweep, B in place): every uplo / op / diag
    m = 90
    a0 = rnd(n, n, dt, 7) / n + 2 * np.eye(n, dtype=dt)
    for uplo, tri in ((s.Uplo.Lower, np.tril), (s.Uplo.Upper, np.triu)):
        for diag in (s.Diag.NonUnit, s.Diag.Unit):
            teff = tri(a0).copy()
            if diag == s.Diag.Unit:
                np.fill_diagonal(teff, 1)
            for op in ("n", "t", "c"):
                b = rnd(m, n, dt, 8)
                T = s.TriangularMatrix(uplo, diag, s.from_numpy(a0, nb=nb, target=tg))
                opt = teff
                if op == "t":
                    T, opt = s.transpose(T), teff.T
                elif op == "c":
                    T, opt = s.conj_transpose(T), teff.conj().T
                B = s.from_numpy(b, nb=nb, target=tg)
                s.trsm(s.Side.Right, dt(2), T, B, target=tg, method_trsm="trsmB")
                assert relerr(s.to_numpy(B) @ opt, 2 * b) < 10 * tol(dt), (uplo, diag, op)


def case_trmm(tg, dt, nb):
    """Distributed trmm (triangle-skipping SUMMA) on every side / uplo / op / diag."""
    m, n = 130, 70
    for side in (s.Side.Left, s.Side.Right):
        na = m if side == s.Side.Left else n
        for uplo, tri in ((s.Uplo.Lower, np.tril), (s.Uplo.Upper, np.triu)):
            t = rnd(na, na, dt, 51)
            for diag in (s.Diag.NonUnit, s.Diag.Unit):
                teff = tri(t).copy()
                if diag == s.Diag.Unit:
                    np.fill_diagonal(teff, 1)
                for op in ("n", "t", "c"):
                    b = rnd(m, n, dt, 52)
                    T = s.TriangularMatrix(uplo, diag, s.from_numpy(t, nb=nb, target=tg))
                    opt = teff
                    if op == "c":
                        T = s.conj_transpose(T)
                        opt = teff.conj().T
                    elif op == "t":
                        T = s.transpose(T)
                        opt = teff.T
                    B = s.from_numpy(b, nb=nb, target=tg)
                    s.trmm(side, dt(1.5), T, B, target=tg)
                    ref = 1.5 * (opt @ b if side == s.Side.Left else b @ opt)
                    assert relerr(s.to_numpy(B), ref) < tol(dt), (side, uplo, diag, op)


def case_hemm(tg, dt, nb):
    """Distributed hemm / symm: hemmC (stored-triangle SUMMA) and hemmA
    (stationary A), Left / Right, Lower / Upper, narrow and wide B."""
    n = 130
    a = rnd(n, n, dt, 71)
    h = a + a.conj().T
    sy = a + a.T
    for ncol in (20, 90):
        for side in (s.Side.Left, s.Side.Right):
            shp = (n, ncol) if side == s.Side.Left else (ncol, n)
            b, c0 = rnd(*shp, dt, 72), rnd(*shp, dt, 73)
            for uplo, tri in ((s.Uplo.Lower, np.tril), (s.Uplo.Upper, np.triu)):
                for meth in ("hemmA", "hemmC"):
                    for herm, full, fn, cls in ((True, h, s.hemm, s.HermitianMatrix),
                                                (False, sy, s.symm, s.SymmetricMatrix)):
                        # only the stored triangle is valid: garbage in the other one
                        st = tri(full) + (np.triu(rnd(n, n, dt, 74), 1) if uplo == s.Uplo.Lower
                                          else np.tril(rnd(n, n, dt, 74), -1))
                        A = cls(uplo, s.from_numpy(st, nb=nb, target=tg))
                        B = s.from_numpy(b, nb=nb, target=tg)
                        C = s.from_numpy(c0, nb=nb, target=tg)
                        fn(side, 1.5, A, B, 0.5, C, target=tg, method_hemm=meth)
                        ref = 1.5 * (full @ b if side == s.Side.Left else b @ full) + 0.5 * c0
                        assert relerr(s.to_numpy(C), ref) < tol(dt), (ncol, side, uplo, meth, herm)


def case_stationary(tg, dt, nb):
    """gemmA and trsmA (stationary A, narrow operand replicated on the device)
    against gemmC / trsmB on every side / uplo / op."""
    m, k = 140, 110
    a, b, c0 = rnd(m, k, dt, 81), rnd(k, 30, dt, 82), rnd(m, 30, dt, 83)
    for meth in ("gemmA", "gemmC"):
        C = s.from_numpy(c0, nb=nb, target=tg)
        s.gemm(2.0, s.from_numpy(a, nb=nb, target=tg), s.from_numpy(b, nb=nb, target=tg), -1.0, C,
               target=tg, method_gemm=meth)
        assert relerr(s.to_numpy(C), 2.0 * a @ b - c0) < tol(dt), meth
    n = 130
    t = (rnd(n, n, dt, 84) / n + 2 * np.eye(n)).astype(dt)
    for side in (s.Side.Left, s.Side.Right):
        for uplo, tri in ((s.Uplo.Lower, np.tril), (s.Uplo.Upper, np.triu)):
            for op in ("n", "c"):
                for meth in ("trsmA", "trsmB"):
                    shp = (n, 25) if side == s.Side.Left else (25, n)
                    b = rnd(*shp, dt, 85)
                    T = s.TriangularMatrix(uplo, s.Diag.NonUnit, s.from_numpy(t, nb=nb, target=tg))
                    opt = tri(t)
                    if op == "c":
                        T = s.conj_transpose(T)
                        opt = opt.conj().T
                    B = s.from_numpy(b, nb=nb, target=tg)
                    s.trsm(side, 2.0, T, B, target=tg, method_trsm=meth)
                    x = s.to_numpy(B)
                    lhs = opt @ x if side == s.Side.Left else x @ opt
                    assert relerr(lhs, 2.0 * b) < 10 * tol(dt), (side, uplo, op, meth)


def case_rbt(tg, dt, nb):
    """Butterfly levels with partner rows / columns on other processes
    (grouped exchange) against the dense U^T A V, and gesv_rbt."""
    m, n = 150, 130
    a = rnd(m, n, dt, 91)
    A = s.from_numpy(a, nb=nb, target=tg)
    s.gerbt(A, 2, 1, 2, target=tg)
    ref = butterfly_dense(m, 2, 1).T @ a @ butterfly_dense(n, 2, 2)
    assert relerr(s.to_numpy(A), ref) < tol(dt)
    a = rnd(n, n, dt, 92) + 2 * np.eye(n, dtype=dt)
    b = rnd(n, 3, dt, 93)
    A, B = s.from_numpy(a, nb=nb, target=tg), s.from_numpy(b, nb=nb, target=tg)
    X = s.from_numpy(np.zeros_like(b), nb=nb, target=tg)
    info, it = s.gesv_rbt(A, B, X, target=tg)
    assert info == 0
    assert relerr(a @ s.to_numpy(X), b) < 100 * tol(dt)


def case_heev(tg, dt, nb):
    """Two-stage heev on the grid (he2hb two-sided update, band-only gather,
    distributed back-transforms): eigenvalues vs numpy and ||H Z - Z L||."""
    n = 150
    a = rnd(n, n, dt, 97)
    h = (a + a.conj().T).astype(dt)
    H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target=tg))
    Z = s.from_numpy(np.zeros((n, n), dt), nb=nb, target=tg)
    lam = s.heev(H, Z, target=tg)
    ref = np.linalg.eigvalsh(h)
    assert np.abs(np.sort(lam) - ref).max() <= 100 * tol(dt) * np.abs(ref).max(), "eigenvalues"
    z = s.to_numpy(Z)
    assert np.linalg.norm(h @ z - z * lam) <= 100 * tol(dt) * np.linalg.norm(h) * np.sqrt(n), "vectors"
    # stage 2 distributed: QL with the rotations on each rank's rows of Z
    # (method_eig="qr"), and divide and conquer with many merges and heavy
    # deflation (repeated eigenvalues) -- Q stays on the 2-D grid
    H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target=tg))
    Z = s.from_numpy(np.zeros((n, n), dt), nb=nb, target=tg)
    lam = s.heev(H, Z, target=tg, method_eig="qr")
    assert np.abs(np.sort(lam) - ref).max() <= 100 * tol(dt) * np.abs(ref).max(), "qr eigenvalues"
    z = s.to_numpy(Z)
    assert np.linalg.norm(h @ z - z * lam) <= 100 * tol(dt) * np.linalg.norm(h) * np.sqrt(n), "qr vectors"
    n3 = 260
    q3, _ = np.linalg.qr(rnd(n3, n3, dt, 96))
    ev3 = np.repeat(np.arange(1.0, 14.0), 20)
    h3 = ((q3 * ev3) @ q3.conj().T).astype(dt)
    h3 = ((h3 + h3.conj().T) / 2).astype(dt)
    H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h3, nb=nb, target=tg))
    Z = s.from_numpy(np.zeros((n3, n3), dt), nb=nb, target=tg)
    lam = s.heev(H, Z, target=tg)
    assert np.abs(np.sort(lam) - np.sort(ev3)).max() <= 200 * tol(dt) * 13, "dc deflated eigenvalues"
    z = s.to_numpy(Z)
    assert np.linalg.norm(h3 @ z - z * lam) <= 200 * tol(dt) * np.linalg.norm(h3) * np.sqrt(n3), "dc deflated vectors"
    assert np.abs(z.conj().T @ z - np.eye(n3)).max() < 200 * tol(dt) * n3, "dc orthogonality"
    sv = s.svd_vals(s.from_numpy(a, nb=nb, target=tg), target=tg)
    assert np.abs(np.sort(sv)[::-1] - np.linalg.svd(a, compute_uv=False)).max() <= 100 * tol(dt) * sv.max()
    for (m2, n2) in ((170, 120), (110, 160)):
        b2 = rnd(m2, n2, dt, 98)
        k2 = min(m2, n2)
        U = s.from_numpy(np.zeros((m2, k2), dt), nb=nb, target=tg)
        VT = s.from_numpy(np.zeros((k2, n2), dt), nb=nb, target=tg)
        sv = s.svd(s.from_numpy(b2, nb=nb, target=tg), U, VT, target=tg)
        u, vt = s.to_numpy(U), s.to_numpy(VT)
        assert relerr((u * sv) @ vt, b2) < 100 * tol(dt), ("svd", m2, n2)
        assert np.abs(u.conj().T @ u - np.eye(k2)).max() < 100 * tol(dt) * k2
        assert np.abs(vt @ vt.conj().T - np.eye(k2)).max() < 100 * tol(dt) * k2


def case_stages(tg, dt, nb):
    """Stage API on the grid: he2hb -> hb2st (band-only storage input) ->
    stedc / steqr2 with the vectors distributed -> unmtr_hb2st ->
    unmtr_he2hb; ge2tb -> tb2bd -> bdsqr on distributed U / VT -> unmbr."""
    n = 120
    t = tol(dt)
    a = rnd(n, n, dt, 71)
    a = ((a + a.conj().T) / 2).astype(dt)
    F = s.from_numpy(a, nb=nb, target=tg)
    Ts = s.he2hb(F, target=tg)
    f = s.to_numpy(F)
    band = np.where((np.subtract.outer(np.arange(n), np.arange(n)) >= 0)
                    & (np.subtract.outer(np.arange(n), np.arange(n)) <= nb), f, 0).astype(dt)
    Hd = s.HermitianBandMatrix(s.Uplo.Lower, nb, s.from_numpy(band, nb=nb, target=tg))
    ref = np.linalg.eigvalsh(a)
    # the same band in band-only storage: hb2st reads the stored band only
    Hs = s.hermitian_band_matrix(s.Uplo.Lower, n, nb, nb, dtype=dt, target=tg)
    assert Hs.is_band_storage
    s.copy(Hd, Hs, target=tg)
    ds, es, _ = s.hb2st_band(Hs, target=tg)
    for solver in ("stedc", "steqr2"):
        d, e, V = s.hb2st_band(Hd, target=tg)
        assert np.abs(np.asarray(d) - np.asarray(ds)).max() < 100 * t * np.abs(ref).max(), "band-storage hb2st"
        Zr = s.from_numpy(np.eye(n), nb=nb, target=tg)
        if solver == "stedc":
            lam = s.stedc_matrix(d, e, Zr, target=tg)
        else:
            lam = s.steqr2(s.Job.Vec, d, e, Zr, target=tg)
        assert np.abs(np.sort(lam) - ref).max() < 100 * t * np.abs(ref).max(), solver
        Z = s.from_numpy(s.to_numpy(Zr).astype(dt), nb=nb, target=tg)
        s.unmtr_hb2st(s.Side.Left, s.Op.NoTrans, V, Z, target=tg)
        s.unmtr_he2hb(s.Side.Left, s.Op.NoTrans, F, Ts, Z, target=tg)
        z = s.to_numpy(Z)
        assert relerr(a @ z, z * lam[None, :]) < 100 * t, solver
    m2, n2 = 100, 72
    b = rnd(m2, n2, dt, 72)
    W = s.from_numpy(b, nb=nb, target=tg)
    TU, TV = s.ge2tb(W, target=tg)
    w = s.to_numpy(W)
    ii, jj = np.meshgrid(np.arange(m2), np.arange(n2), indexing="ij")
    ub = np.where((jj >= ii) & (jj - ii <= nb), w, 0)[:n2, :].astype(dt)
    B = s.TriangularBandMatrix(s.Uplo.Upper, s.Diag.NonUnit, nb, s.from_numpy(ub, nb=nb, target=tg))
    d, e, U2, V2 = s.tb2bd_band(B, target=tg)
    Ub = s.from_numpy(np.eye(n2, dtype=dt), nb=nb, target=tg)
    VTb = s.from_numpy(np.eye(n2, dtype=dt), nb=nb, target=tg)
    sig = s.bdsqr_matrix(s.Job.Vec, s.Job.Vec, d, e, Ub, VTb, target=tg)
    assert np.abs(np.sort(sig)[::-1] - np.linalg.svd(b, compute_uv=False)).max() < 100 * t * sig.max()
    s.unmbr_tb2bd(s.Side.Left, s.Op.NoTrans, U2, Ub, target=tg)
    s.unmbr_tb2bd(s.Side.Right, s.Op.ConjTrans, V2, VTb, target=tg)
    U = s.from_numpy(np.vstack([s.to_numpy(Ub), np.zeros((m2 - n2, n2), dt)]), nb=nb, target=tg)
    s.unmbr_ge2tb(s.Side.Left, s.Op.NoTrans, W, TU, U, target=tg)
    s.unmbr_ge2tb(s.Side.Right, s.Op.NoTrans, W, TV, VTb, target=tg)
    u, vt = s.to_numpy(U), s.to_numpy(VTb)
    assert relerr((u * sig[None, :]) @ vt, b) < 100 * t


def band_of(a, kl, ku):
    i, j = np.indices(a.shape)
    return np.where((i - j <= kl) & (j - i <= ku), a, 0).astype(a.dtype)


def case_band(tg, dt, nb):
    """Distributed blocked gbtrf / pbtrf (block-column slabs, one broadcast per
    panel) through gbsv / pbsv; bandwidths below and above the tile size."""
    n = 170
    for kl, ku in ((3, 2), (20, 35), (60, 10)):
        a = band_of(rnd(n, n, dt, 101 + kl), kl, ku)
        b = rnd(n, 2, dt, 102)
        A = s.BandMatrix(kl, ku, s.from_numpy(a, nb=nb, target=tg))
        B = s.from_numpy(b, nb=nb, target=tg)
        info, piv = s.gbsv(A, B, target=tg)
        assert info == 0
        x = s.to_numpy(B)
        assert np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x)) < 100 * tol(dt), (kl, ku)
    for kd in (4, 50):
        for uplo in (s.Uplo.Lower, s.Uplo.Upper):
            c0 = band_of(rnd(n, n, dt, 103 + kd), kd, kd)
            h = (c0 + c0.conj().T + 4 * kd * np.eye(n)).astype(dt)
            st = np.tril(h) if uplo == s.Uplo.Lower else np.triu(h)
            b = rnd(n, 3, dt, 104)
            A = s.HermitianBandMatrix(uplo, kd, s.from_numpy(st, nb=nb, target=tg))
            B = s.from_numpy(b, nb=nb, target=tg)
            assert s.pbsv(A, B, target=tg) == 0
            x = s.to_numpy(B)
            assert relerr(h @ x, b) < 100 * tol(dt), (kd, uplo)


def case_band_storage(tg, dt, nb):
    """Band-only storage (reference BaseBandMatrix.hh:219-258): the sized band
    constructors allocate only the tiles intersecting the band (+ gbtrf
    fill); gbsv / pbsv / gbmm / hbmm / norms on it, and O(n * bandwidth)
    local memory."""
    n = 230
    for kl, ku in ((3, 2), (20, 35), (60, 10)):
        a = band_of(rnd(n, n, dt, 201 + kl), kl, ku) + 3 * np.eye(n, dtype=dt)
        A = s.band_matrix(n, n, kl, ku, nb, dtype=dt, target=tg)
        assert A.is_band_storage
        s.copy(s.from_numpy(a, nb=nb, target=tg), A, target=tg)
        assert relerr(s.to_numpy(A), a) == 0
        for nm, o in ((s.Norm.One, 1), (s.Norm.Inf, np.inf), (s.Norm.Fro, "fro")):
            assert abs(s.norm(nm, A, target=tg) - np.linalg.norm(a, o)) <= 1e-5 * np.linalg.norm(a, o)
        b, c = rnd(n, 4, dt, 202), rnd(n, 4, dt, 203)
        C = s.from_numpy(c, nb=nb, target=tg)
        s.gbmm(2.0, A, s.from_numpy(b, nb=nb, target=tg), 0.5, C, target=tg)
        assert relerr(s.to_numpy(C), 2.0 * a @ b + 0.5 * c) < tol(dt), (kl, ku)
        B = s.from_numpy(b, nb=nb, target=tg)
        info, piv = s.gbsv(A, B, target=tg)
        assert info == 0
        x = s.to_numpy(B)
        assert np.linalg.norm(a @ x - b) / (np.linalg.norm(a) * np.linalg.norm(x)) < 100 * tol(dt), (kl, ku)
    # memory: a narrow band in a large matrix
    nbig, kb = 40 * nb, 3
    A = s.band_matrix(nbig, nbig, kb, kb, nb, dtype=dt, target=tg)
    g = parallel.current_grid()
    dense_local = -(-nbig // g.p) * -(-nbig // g.q) * np.dtype(dt).itemsize
    assert A.storage_bytes < dense_local / 4, (A.storage_bytes, dense_local)
    for kd in (4, 50):
        for uplo in (s.Uplo.Lower, s.Uplo.Upper):
            c0 = band_of(rnd(n, n, dt, 205 + kd), kd, kd)
            h = (c0 + c0.conj().T + 4 * kd * np.eye(n)).astype(dt)
            st = np.tril(h) if uplo == s.Uplo.Lower else np.triu(h)
            H = s.hermitian_band_matrix(uplo, n, kd, nb, dtype=dt, target=tg)
            s.copy(s.from_numpy(st, nb=nb, target=tg), H, target=tg)
            bt = rnd(3, n, dt, 206)
            Ct = s.from_numpy(np.zeros((3, n), dt), nb=nb, target=tg)
            s.hbmm(s.Side.Right, 1.0, H, s.from_numpy(bt, nb=nb, target=tg), 0.0, Ct, target=tg)
            assert relerr(s.to_numpy(Ct), bt @ h) < tol(dt), (kd, uplo)
            b = rnd(n, 3, dt, 207)
            B = s.from_numpy(b, nb=nb, target=tg)
            assert s.pbsv(H, B, target=tg) == 0
            assert relerr(h @ s.to_numpy(B), b) < 100 * tol(dt), (kd, uplo)


def case_band_blas(tg, dt, nb):
    """gbmm / hbmm / tbsm / pbtrs over band chunks (distributed GEMM / TRSM on
    the sub-views the band touches), bandwidths below and above the tile."""
    n, nr = 150, 7
    for kl, ku in ((3, 5), (40, 9)):
        a = rnd(n, n, dt, 111 + kl)
        b, c = rnd(n, nr, dt, 112), rnd(n, nr, dt, 113)
        A = s.BandMatrix(kl, ku, s.from_numpy(a, nb=nb, target=tg))
        B, C = s.from_numpy(b, nb=nb, target=tg), s.from_numpy(c, nb=nb, target=tg)
        s.gbmm(2.0, A, B, 0.5, C, target=tg)
        assert relerr(s.to_numpy(C), 2.0 * band_of(a, kl, ku) @ b + 0.5 * c) < tol(dt), (kl, ku)
        h = (a + a.conj().T) / 2
        for uplo in (s.Uplo.Lower, s.Uplo.Upper):
            st = np.tril(h) if uplo == s.Uplo.Lower else np.triu(h)
            H = s.HermitianBandMatrix(uplo, kl, s.from_numpy(st, nb=nb, target=tg))
            bt = rnd(nr, n, dt, 114)
            Bt, Ct = s.from_numpy(bt, nb=nb, target=tg), s.from_numpy(np.zeros((nr, n), dt), nb=nb, target=tg)
            s.hbmm(s.Side.Right, 1.0, H, Bt, 0.0, Ct, target=tg)
            assert relerr(s.to_numpy(Ct), bt @ band_of(h, kl, kl)) < tol(dt), (kl, uplo)
            t = band_of(st, kl, kl) + 4 * np.eye(n, dtype=dt) * (1 + kl)
            Tb = s.TriangularBandMatrix(uplo, s.Diag.NonUnit, kl, s.from_numpy(t, nb=nb, target=tg))
            X = s.from_numpy(b, nb=nb, target=tg)
            s.tbsm(s.Side.Left, 1.0, s.conj_transpose(Tb), X, target=tg)
            assert relerr(t.conj().T @ s.to_numpy(X), b) < 100 * tol(dt), (kl, uplo)
            Y = s.from_numpy(bt, nb=nb, target=tg)
            s.tbsm(s.Side.Right, 2.0, Tb, Y, target=tg)
            assert relerr(s.to_numpy(Y) @ t, 2.0 * bt) < 100 * tol(dt), (kl, uplo)


def case_layout(tg, dt, nb):
    """Arbitrary distribution + non-uniform tiles (reference lambda
    constructor): drivers on lambda-layout operands (block-cyclic working
    copies), results read back through the tile-by-tile redistribution."""
    P = int(os.environ.get("WORLD_SIZE", "1"))
    n = 150
    rs = [17, 40, 23, 31, 39]
    cs = [33, 12, 50, 28, 27]
    own = lambda i, j: (3 * i + j) % P
    a = rnd(n, n, dt, 111)
    bm = rnd(n, 40, dt, 112)

    def lay(x, rows, cols):
        L = s.matrix_layout(x.shape[0], x.shape[1], rows, cols, own, dtype=dt, target=tg)
        s.copy(s.from_numpy(x, nb=nb, target=tg), L, target=tg)
        return L

    def back(L):
        B = s.from_numpy(np.zeros((L.m, L.n), dt), nb=nb, target=tg)
        s.copy(L, B, target=tg)
        return s.to_numpy(B)
    A = lay(a, rs, cs)
    assert A.arbitrary_layout()
    assert relerr(back(A), a) == 0
    C = lay(np.zeros((n, 40), dt), rs, [40])
    s.gemm(1.0, A, lay(bm, cs, [15, 25]), 0.0, C, target=tg)
    assert relerr(back(C), a @ bm) < tol(dt)
    assert abs(s.norm(s.Norm.One, A, target=tg) - np.linalg.norm(a, 1)) <= 1e-4 * np.linalg.norm(a, 1)
    h = (a @ a.conj().T + n * np.eye(n)).astype(dt)
    H = s.HermitianMatrix(s.Uplo.Lower, lay(h, rs, rs))
    B = lay(bm, rs, [40])
    assert s.posv(H, B, target=tg) == 0
    assert relerr(h @ back(B), bm) < 10 * tol(dt)
    G = lay(a + n * np.eye(n, dtype=dt), cs, rs)
    B = lay(bm, cs, [20, 20])
    info, _ = s.gesv(G, B, target=tg)
    assert info == 0 and relerr((a + n * np.eye(n)) @ back(B), bm) < 10 * tol(dt)
    # getrf then getrs / getri as separate calls, max tileNb (50) > max
    # tileMb (40), arbitrary-layout right-hand side with its own row tiling
    ad = a + 0.1 * np.eye(n, dtype=dt)
    G = lay(ad, rs, cs)
    info, piv = s.getrf(G, target=tg)
    assert info == 0
    B = lay(bm, [60, 45, 45], [40])
    s.getrs(G, piv, B, target=tg)
    assert relerr(ad @ back(B), bm) < 1e3 * tol(dt)
    B = lay(bm, cs, [40])
    s.getrs(G, piv, B, target=tg, trans=s.Op.Trans)
    assert relerr(ad.T @ back(B), bm) < 1e3 * tol(dt)
    s.getri(G, piv, target=tg)
    assert relerr(back(G) @ ad, np.eye(n)) < 1e3 * tol(dt)
    # geqrf then unmqr on an arbitrary-layout A and C
    Q = lay(a, rs, cs)
    T = s.geqrf(Q, target=tg)
    C = lay(bm, cs, [40])
    s.unmqr(s.Side.Left, s.Op.ConjTrans, Q, T, C, target=tg)
    r = np.triu(back(Q))
    qhb = back(C)
    # Q^H b has the norm of b column by column, and R^{-1} (Q^H b) solves a x = b
    x = np.linalg.solve(r, qhb)
    assert relerr(a @ x, bm) < 1e4 * tol(dt)


def case_aasen(tg, dt, nb):
    """Distributed blocked Aasen (hetrf / hetrs / hesv with the reference's
    signatures): indefinite Hermitian solves, and P A P^T = L T L^H rebuilt
    from the factors."""
    for n in (150, 97):
        a = rnd(n, n, dt, 121 + n)
        h = (a + a.conj().T).astype(dt)
        b = rnd(n, 3, dt, 122)
        A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target=tg))
        T = s.BandMatrix(nb, nb, s.from_numpy(np.zeros((n, n), dt), nb=nb, target=tg))
        B = s.from_numpy(b, nb=nb, target=tg)
        info, p1, p2 = s.hesv_aasen(A, T, B, target=tg)
        assert info == 0
        x = s.to_numpy(B)
        assert np.linalg.norm(h @ x - b) / (np.linalg.norm(h) * np.linalg.norm(x)) < 100 * tol(dt), n
        # the same factors through hetrs on new right-hand sides
        b2 = rnd(n, 2, dt, 123)
        B2 = s.from_numpy(b2, nb=nb, target=tg)
        s.hetrs_aasen(A, p1, T, p2, B2, target=tg)
        x2 = s.to_numpy(B2)
        assert np.linalg.norm(h @ x2 - b2) / (np.linalg.norm(h) * np.linalg.norm(x2)) < 100 * tol(dt), n


def case_potrf(tg, dt, nb):
    n = 200
    a = rnd(n, n, dt, 7)
    a = (a @ a.conj().T + n * np.eye(n)).astype(dt)
    b = rnd(n, 3, dt, 8)
    A = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(a, nb=nb, target=tg))
    B = s.from_numpy(b, nb=nb, target=tg)
    info = s.posv(A, B, target=tg)
    assert info == 0
    assert relerr(a @ s.to_numpy(B), b) < 10 * tol(dt)
    # Upper storage (in place, potrf_upper): U^H U = A, lookahead 1 and 2
    for la in (1, 2):
        A = s.HermitianMatrix(s.Uplo.Upper, s.from_numpy(a, nb=nb, target=tg))
        assert s.potrf(A, target=tg, lookahead=la) == 0
        U = np.triu(s.to_numpy(A))
        assert relerr(U.conj().T @ U, a) < 10 * tol(dt), la
        B = s.from_numpy(b, nb=nb, target=tg)
        s.potrs(A, B, target=tg)
        assert relerr(a @ s.to_numpy(B), b) < 10 * tol(dt), la


def case_getrf(tg, dt, nb):
    n = 190
    a = rnd(n, n, dt, 9)
    b = rnd(n, 4, dt, 10)
    for method in ("ppiv", "tntpiv"):
        A = s.from_numpy(a, nb=nb, target=tg)
        B = s.from_numpy(b, nb=nb, target=tg)
        kw = {"method_lu": 2} if method == "tntpiv" else {}
        info, _ = s.gesv(A, B, target=tg, **kw)
        assert info == 0
        assert relerr(a @ s.to_numpy(B), b) < 100 * tol(dt), method


def case_getrf_thresh(tg, dt, nb):
    """PivotThreshold in the distributed per-column pivot search: P A = L U
    and |L| <= 1 / threshold."""
    n = 170
    a = rnd(n, n, dt, 95) + 1.5 * np.eye(n, dtype=dt)
    for thresh in (0.5, 0.1):
        A = s.from_numpy(a, nb=nb, target=tg)
        info, piv = s.getrf(A, target=tg, pivot_threshold=thresh)
        assert info == 0
        f = s.to_numpy(A)
        Lf = np.tril(f, -1) + np.eye(n, dtype=dt)
        pa = a.copy()
        for i, r in enumerate(ipiv_of(piv, nb)):
            if r != i:
                pa[[i, r]] = pa[[r, i]]
        assert relerr(Lf @ np.triu(f), pa) < 100 * tol(dt), thresh
        bound = (np.sqrt(2) if np.iscomplexobj(a) else 1) / thresh   # pivots chosen by |re| + |im|
        assert np.abs(Lf).max() <= bound * (1 + 1e-5), (thresh, np.abs(Lf).max())


def case_pplu_exact(tg, dt, nb):
    """Partial pivoting on p > 1 is EXACT partial pivoting (one all-gather
    per panel, the assembled panel factored redundantly): the same pivots as
    LAPACK getrf (scipy.linalg.lu_factor, |re| + |im| pivot choice)."""
    import scipy.linalg as sla
    for (m, n) in ((190, 190), (230, 140)):
        a = rnd(m, n, dt, 97)
        A = s.from_numpy(a, nb=nb, target=tg)
        info, piv = s.getrf(A, target=tg)
        assert info == 0
        _, ref = sla.lu_factor(a.astype(np.complex128 if np.iscomplexobj(a) else np.float64))
        got = ipiv_of(piv, nb)
        assert list(got) == list(ref[:len(got)]), (m, n)


def case_lanes(tg, dt, nb):
    """Communication lanes (Grid.row_fast / col_fast): critical-path tasks --
    tournament / panel gather, pivot + LU11 + L broadcasts, lookahead row
    exchanges, TSQR, (V, T) broadcasts -- are enqueued on the panel queue (1);
    the trailing chunks' row exchanges / W all-reduces and the left swaps on
    the comm queue (3), with their slot pack / unpack kernels on a compute
    queue.  Also: PPLU issues one collective task per panel."""
    n = 6 * nb + 7
    a = rnd(n, n, dt, 131)
    crit_getrf = {"getrf_tnt_send", "getrf_tnt_recv", "getrf_bcast_winners", "getrf_panel_perm", "getrf_bcast_row",
                  "getrf_bcast_L", "getrf_pp_panel"}
    for fn, kw in ((s.getrf_tntpiv, {}), (s.getrf, {})):
        A = s.from_numpy(a, nb=nb, target=tg)
        s._slate.lane_log_enable(True)
        fn(A, target=tg, **kw)
        log = s._slate.lane_log_take()
        s._slate.lane_log_enable(False)
        for label, qu in log:
            if label in crit_getrf:
                assert qu == 1, (label, qu)
            if label == "getrf_left_swap":
                assert qu == 3, (label, qu)
            # slot pack / unpack are compute: never on the comm queue
            if label in ("getrf_rows_pack", "getrf_rows_unpack", "getrf_left_pack", "getrf_left_unpack"):
                assert qu != 3, (label, qu)
        if parallel.current_grid().p > 1:
            labels = {label for label, _ in log}
            assert {"getrf_left_pack", "getrf_left_unpack"} <= labels, labels
        qs = {qu for label, qu in log if label == "getrf_rows_exchange"}
        assert qs <= {1, 3} and (1 in qs or parallel.current_grid().p == 1), qs
        if fn is s.getrf and parallel.current_grid().p > 1:
            # the process column of each panel runs exactly one panel task (one collective)
            g = parallel.current_grid()
            mine = sum(1 for k in range((n + nb - 1) // nb) if k % g.q == g.mycol)
            assert sum(1 for label, _ in log if label == "getrf_pp_panel") == mine
            assert not any(label == "getrf_pp_column" for label, _ in log)
    A = s.from_numpy(a, nb=nb, target=tg)
    s._slate.lane_log_enable(True)
    s.geqrf(A, target=tg)
    log = s._slate.lane_log_take()
    s._slate.lane_log_enable(False)
    for label, qu in log:
        if label.startswith("geqrf_tsqr") or label == "geqrf_bcast":
            assert qu == 1, (label, qu)
    qs = {qu for label, qu in log if label == "geqrf_update_allreduce"}
    assert qs <= {1, 3}, qs
    # potrf: every panel message is critical-path -> panel queue (fast lane)
    h = (a @ a.conj().T + n * np.eye(n)).astype(dt)
    H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target=tg))
    s._slate.lane_log_enable(True)
    assert s.potrf(H, target=tg) == 0
    log = s._slate.lane_log_take()
    s._slate.lane_log_enable(False)
    labels = {label for label, _ in log}
    g = parallel.current_grid()
    assert g.p * g.q == 1 or "bcast_panel" in labels, labels
    for label, qu in log:
        if label in ("bcast_diag", "bcast_panel"):
            assert qu == 1, (label, qu)


def case_solve_notemp(tg, dt, nb):
    """Transposed / few-RHS distributed solves make no n x n temporary:
    potrs (L then L^H), getrs with Trans / ConjTrans and posv_mixed (whose
    only n x n temporary is the fp32 factor) -- the transposed sweeps read
    op(A) from A's own local array on the transposed process grid and only
    B is redistributed.  Checked with the matrix-storage allocation peak
    (host target: on the device target the host-origin inputs' device
    instances are staged in and released by every driver, which the peak
    would count too)."""
    chk = (tg == "h")
    n, nrhs = 5 * nb + 3, 3
    a = rnd(n, n, dt, 141)
    h = (a @ a.conj().T + n * np.eye(n)).astype(dt)
    b = rnd(n, nrhs, dt, 142)
    g = parallel.current_grid()
    p, q = g.p, g.q
    s._slate.storage_alloc_reset()
    s.from_numpy(np.zeros((n, n), dt), nb=nb, target=tg)
    full = s._slate.storage_alloc_max()          # this rank's local n x n array (padded ld)
    H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target=tg))
    assert s.potrf(H, target=tg) == 0
    B = s.from_numpy(b, nb=nb, target=tg)
    s._slate.storage_alloc_reset()
    s.potrs(H, B, target=tg)
    assert not chk or s._slate.storage_alloc_max() < full / 4, (s._slate.storage_alloc_max(), full)
    assert relerr(h @ s.to_numpy(B), b) < 100 * tol(dt)
    A = s.from_numpy(a + 0.2 * np.eye(n, dtype=dt), nb=nb, target=tg)
    info, piv = s.getrf(A, target=tg)
    assert info == 0
    ad = a + 0.2 * np.eye(n, dtype=dt)
    for op, ref in ((s.Op.Trans, ad.T), (s.Op.ConjTrans, ad.conj().T)):
        B = s.from_numpy(b, nb=nb, target=tg)
        s._slate.storage_alloc_reset()
        s.getrs(A, piv, B, target=tg, trans=op)
        assert not chk or s._slate.storage_alloc_max() < full / 4, (op, s._slate.storage_alloc_max(), full)
        assert relerr(ref @ s.to_numpy(B), b) < 1e3 * tol(dt), op
    for meth in ("trsmA", "trsmB"):
        # op(A) = L^T with B already on the transposed grid (no redistribution)
        L = s.TriangularMatrix(s.Uplo.Lower, s.Diag.NonUnit, s.from_numpy(np.tril(h), nb=nb, target=tg))
        Bt = s.from_numpy(b, nb=nb, target=tg, grid=g.transposed())
        s._slate.storage_alloc_reset()
        s.trsm(s.Side.Left, 1.0, s.transpose(L), Bt, target=tg, method_trsm=meth)
        assert not chk or s._slate.storage_alloc_max() < full / 4, meth
        assert relerr(np.tril(h).T @ s.to_numpy(Bt), b) < 100 * tol(dt), meth
    # Right-side solve on an n x n B: the column sweep works on B in place
    # (no transposed copy of B), op(A) = A^H with A on B's grid included
    L = s.TriangularMatrix(s.Uplo.Lower, s.Diag.NonUnit, s.from_numpy(np.tril(h), nb=nb, target=tg))
    for opname in ("n", "c"):
        bb = rnd(n, n, dt, 143)
        Bn = s.from_numpy(bb, nb=nb, target=tg)
        Lop = L if opname == "n" else s.conj_transpose(L)
        ref = np.tril(h) if opname == "n" else np.tril(h).conj().T
        s._slate.storage_alloc_reset()
        s.trsm(s.Side.Right, 1.0, Lop, Bn, target=tg)
        assert not chk or s._slate.storage_alloc_max() < full / 4, ("trsm right", opname, s._slate.storage_alloc_max(), full)
        assert relerr(s.to_numpy(Bn) @ ref, bb) < 100 * tol(dt), ("trsm right", opname)
    # unmqr Right (C Q, C Q^H) in place on C (C's columns = Q's rows)
    A = s.from_numpy(a, nb=nb, target=tg)
    T = s.geqrf(A, target=tg)
    Qe = s.from_numpy(np.eye(n, dtype=dt), nb=nb, target=tg)
    s.unmqr(s.Side.Left, s.Op.NoTrans, A, T, Qe, target=tg)
    Qm = s.to_numpy(Qe)
    for opq, ref in ((s.Op.NoTrans, Qm), (s.Op.ConjTrans, Qm.conj().T)):
        cc = rnd(n, n, dt, 147)
        Cn = s.from_numpy(cc, nb=nb, target=tg)
        s._slate.storage_alloc_reset()
        s.unmqr(s.Side.Right, opq, A, T, Cn, target=tg)
        assert not chk or s._slate.storage_alloc_max() < full / 4, ("unmqr right", opq, s._slate.storage_alloc_max(), full)
        assert relerr(s.to_numpy(Cn), cc @ ref) < 100 * tol(dt), ("unmqr right", opq)
    # potrf on Upper storage: in place (no conj-transposed n x n copies)
    Hu = s.HermitianMatrix(s.Uplo.Upper, s.from_numpy(h, nb=nb, target=tg))
    s._slate.storage_alloc_reset()
    assert s.potrf(Hu, target=tg) == 0
    assert not chk or s._slate.storage_alloc_max() < full / 4, ("potrf upper", s._slate.storage_alloc_max(), full)
    Uu = np.triu(s.to_numpy(Hu))
    assert relerr(Uu.conj().T @ Uu, h) < 100 * tol(dt), "potrf upper"
    # hemm Right on n x n B, C: in place, no (conj-)transposed copies
    H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target=tg))
    bb, cc = rnd(n, n, dt, 145), rnd(n, n, dt, 146)
    Bn, Cn = s.from_numpy(bb, nb=nb, target=tg), s.from_numpy(cc, nb=nb, target=tg)
    s._slate.storage_alloc_reset()
    s.hemm(s.Side.Right, dt(1.5), H, Bn, dt(0.5), Cn, target=tg)
    assert not chk or s._slate.storage_alloc_max() < full / 4, ("hemm right", s._slate.storage_alloc_max(), full)
    assert relerr(s.to_numpy(Cn), 1.5 * bb @ h + 0.5 * cc) < 100 * tol(dt), "hemm right"
    for opname in ("n", "t"):
        bb = rnd(n, n, dt, 144)
        Bn = s.from_numpy(bb, nb=nb, target=tg)
        Lop = L if opname == "n" else s.transpose(L)
        ref = np.tril(h) if opname == "n" else np.tril(h).T
        s._slate.storage_alloc_reset()
        s.trmm(s.Side.Right, dt(0.5), Lop, Bn, target=tg)
        assert not chk or s._slate.storage_alloc_max() < full / 4, ("trmm right", opname, s._slate.storage_alloc_max(), full)
        assert relerr(s.to_numpy(Bn), 0.5 * bb @ ref) < 100 * tol(dt), ("trmm right", opname)
    if dt in (np.float64, np.complex128):
        H = s.HermitianMatrix(s.Uplo.Lower, s.from_numpy(h, nb=nb, target=tg))
        B = s.from_numpy(b, nb=nb, target=tg)
        X = s.from_numpy(np.zeros_like(b), nb=nb, target=tg)
        s._slate.storage_alloc_reset()
        s.from_numpy(np.zeros((n, n), np.float32 if dt == np.float64 else np.complex64), nb=nb, target=tg)
        lo = s._slate.storage_alloc_max()          # the fp32 factor's local array
        s._slate.storage_alloc_reset()
        info, it = s.posv_mixed(H, B, X, target=tg)
        assert info == 0 and it >= 0
        assert not chk or s._slate.storage_alloc_max() <= lo < full, (s._slate.storage_alloc_max(), lo, full)
        assert relerr(h @ s.to_numpy(X), b) < 100 * tol(dt)


def case_gelqf(tg, dt, nb):
    """Native LQ on row panels (TSQR over the process row when q > 1): L Q = A
    rebuilt through unmlq (Right), Q^H Q = I through unmlq (Left, both ops),
    and the minimum-norm gels (m < n).  No transposed copy of A."""
    for (m, n) in ((120, 230), (150, 150), (170, 100)):
        a = rnd(m, n, dt, 151 + m)
        A = s.from_numpy(a, nb=nb, target=tg)
        T = s.gelqf(A, target=tg)
        f = s.to_numpy(A)
        k = min(m, n)
        Lf = np.zeros((m, n), dt)
        Lf[:, :k] = np.tril(f[:, :k])
        C = s.from_numpy(Lf, nb=nb, target=tg)
        s.unmlq(s.Side.Right, s.Op.NoTrans, A, T, C, target=tg)
        assert relerr(s.to_numpy(C), a) < 100 * tol(dt), (m, n)
        c = rnd(n, 4, dt, 152)
        C = s.from_numpy(c, nb=nb, target=tg)
        s.unmlq(s.Side.Left, s.Op.ConjTrans, A, T, C, target=tg)
        assert abs(np.linalg.norm(s.to_numpy(C)) - np.linalg.norm(c)) < 100 * tol(dt) * np.linalg.norm(c)
        s.unmlq(s.Side.Left, s.Op.NoTrans, A, T, C, target=tg)
        assert relerr(s.to_numpy(C), c) < 100 * tol(dt), (m, n)
    m, n = 90, 200
    a = rnd(m, n, dt, 161)
    b = rnd(m, 3, dt, 162)
    A = s.from_numpy(a, nb=nb, target=tg)
    BX = s.from_numpy(np.vstack([b, np.zeros((n - m, 3), dt)]), nb=nb, target=tg)
    s.gels(A, BX, target=tg)
    x = s.to_numpy(BX)
    ref = np.linalg.lstsq(a, b, rcond=None)[0]
    assert relerr(x, ref) < 1e3 * tol(dt)


def ipiv_of(piv, nb):
    """Reference Pivots (per block column k: (tile index rel. to k, offset)) ->
    LAPACK-style 0-based sequential interchanges."""
    return [(k + ti) * nb + off for k, blk in enumerate(piv) for (ti, off) in blk]


def case_getrf_shapes(tg, dt, nb):
    """Distributed LU on tall / wide / square shapes, lookahead 1 and 2, every
    pivoting method: P A = L U reconstructed from the returned factors and
    pivots (covers the cross-rank tournament tree, the gathered PPLU panel and
    the device-side row-permutation slots, including left-column swaps)."""
    for (m, n) in ((190, 190), (230, 120), (120, 200)):
        a = rnd(m, n, dt, 21 + m + n)
        if m == n:
            a_np = (a + 4 * n * np.eye(n)).astype(dt)   # no-pivoting case needs a safe diagonal
        for method, mlu in (("ppiv", 1), ("tntpiv", 2), ("nopiv", 3)):
            if method == "nopiv" and m != n:
                continue
            src = a_np if method == "nopiv" else a
            for la in (1, 2):
                A = s.from_numpy(src, nb=nb, target=tg)
                info, piv = s.getrf(A, target=tg, method_lu=mlu, lookahead=la)
                assert info == 0, (method, m, n, info)
                f = s.to_numpy(A)
                k = min(m, n)
                Lf = np.tril(f[:, :k], -1) + np.eye(m, k, dtype=dt)
                Uf = np.triu(f[:k, :])
                pa = src.copy()
                for i, r in enumerate(ipiv_of(piv, nb) if method != "nopiv" else range(k)):
                    if r != i:
                        pa[[i, r]] = pa[[r, i]]
                assert relerr(Lf @ Uf, pa) < 100 * tol(dt), (method, m, n, la)


def case_geqrf(tg, dt, nb):
    m, n = 230, 120
    a = rnd(m, n, dt, 11)
    b = rnd(m, 2, dt, 12)
    A = s.from_numpy(a, nb=nb, target=tg)
    B = s.from_numpy(b, nb=nb, target=tg)
    s.gels(A, B, target=tg)
    x = s.to_numpy(B)[:n]
    ref = np.linalg.lstsq(a, b, rcond=None)[0]
    assert relerr(x, ref) < 100 * tol(dt)


def case_geqrf_shapes(tg, dt, nb):
    """Distributed QR (TSQR tree + Householder reconstruction on p > 1) on
    tall / square / wide shapes, lookahead 1 and 2: Q^H A = R through unmqr,
    |R| against numpy's, and Q (Q^H C) = C."""
    for (m, n) in ((230, 120), (150, 150), (100, 170)):
        a = rnd(m, n, dt, 31 + m + n)
        c = rnd(m, 5, dt, 32 + m)
        for la in (1, 2):
            A = s.from_numpy(a, nb=nb, target=tg)
            T = s.geqrf(A, target=tg, lookahead=la)
            f = s.to_numpy(A)
            k = min(m, n)
            r = np.triu(f[:k, :])
            rref = np.linalg.qr(a, mode="r")[:k, :]
            assert relerr(np.abs(r), np.abs(rref)) < 100 * tol(dt), ("R", m, n, la)
            Aq = s.from_numpy(a, nb=nb, target=tg)
            s.unmqr(s.Side.Left, s.Op.ConjTrans, A, T, Aq, target=tg)
            qa = s.to_numpy(Aq)
            assert relerr(np.triu(qa[:k]), r) < 100 * tol(dt), ("QhA", m, n, la)
            assert np.abs(qa[k:]).max() <= 100 * tol(dt) * np.abs(a).max() * m if m > k else True
            C = s.from_numpy(c, nb=nb, target=tg)
            s.unmqr(s.Side.Left, s.Op.ConjTrans, A, T, C, target=tg)
            s.unmqr(s.Side.Left, s.Op.NoTrans, A, T, C, target=tg)
            assert relerr(s.to_numpy(C), c) < 100 * tol(dt), ("QQh", m, n, la)


def case_rowx_bytes(tg, dt, nb):
    """Exact row exchange of the p x q LU (getrf.cc RowXPlan): the elements
    each process sends in the trailing / left row moves equal, step by step,
    the rows that change process times its local columns -- winner rows it
    owns go to the p-1 other processes of its column (every process needs the
    U block row), displaced rows only to their destination's owner, nothing
    padded -- recomputed here from the returned pivots."""
    g = parallel.current_grid()
    p, q, myrow, mycol = g.p, g.q, g.myrow, g.mycol
    m, n = 6 * nb + 9, 5 * nb + 3
    a = rnd(m, n, dt, 171)
    for fn in (s.getrf_tntpiv, s.getrf):
        A = s.from_numpy(a, nb=nb, target=tg)
        s._slate.lu_rowx_reset()
        info, piv = fn(A, target=tg)
        elems, rows = s._slate.lu_rowx_stats()
        assert info == 0
        if p == 1:
            assert elems == 0
            continue
        owner = lambda r: (r // nb) % p
        nt = (n + nb - 1) // nb
        tile_w = [min(nb, n - j * nb) for j in range(nt)]
        local_cols = lambda j0, j1: sum(tile_w[j] for j in range(j0, j1) if j % q == mycol)
        expect = 0
        exp_rows = 0
        for k, pk in enumerate(piv):
            kk, kd = k * nb, len(pk)
            content = {}
            get = lambda r: content.get(r, r)
            for t, (ti, off) in enumerate(pk):
                dst, src = kk + t, (k + ti) * nb + off
                content[dst], content[src] = get(src), get(dst)
            # trailing columns: U rows I own to every other process, my displaced rows
            u_me = sum(1 for t in range(kd) if owner(get(kk + t)) == myrow)
            d_me = sum(1 for dst, src in content.items()
                       if not (kk <= dst < kk + kd) and src != dst and owner(src) == myrow and owner(dst) != myrow)
            ncr = local_cols(k + 1, nt)
            expect += (u_me * (p - 1) + d_me) * ncr
            exp_rows += (u_me * (p - 1) + d_me) * (1 if ncr else 0)
            # left columns: every move whose source is mine and destination is not
            l_me = sum(1 for dst, src in content.items() if src != dst and owner(src) == myrow and owner(dst) != myrow)
            expect += l_me * local_cols(0, k)
        assert elems == expect, (fn.__name__, elems, expect)
        # and strictly less than the zero-padded slot all-reduce it replaces
        # (2 kd rows per column range, every process, every step)
        padded = sum(2 * len(pk) * local_cols(k + 1, nt) for k, pk in enumerate(piv))
        assert elems < padded or padded == 0, (elems, padded)


def case_geqrf_cholqr(tg, dt, nb):
    """p > 1 QR panels by shifted CholeskyQR3 + Householder reconstruction,
    with the TSQR tree as the fallback when the last Gram matrix shows a
    non-orthogonal Q: a well-conditioned matrix never falls back; a matrix
    with an all-zero block column (rank-deficient panel) does, for that panel,
    and both give a correct QR."""
    g = parallel.current_grid()
    m, n = 7 * nb + 5, 4 * nb
    for case in ("full", "zero", "illcond"):
        a = rnd(m, n, dt, 61)
        if case == "zero":
            a[:, nb:2 * nb] = 0
        if case == "illcond":
            # first block column with cond 1e10 (fp32: 1e5): beyond plain
            # CholeskyQR2, so the accept test must route it to the shifted
            # variant or the tree, and Q must still come out orthogonal
            rng = np.random.default_rng(62)
            qu, _ = np.linalg.qr(rng.standard_normal((m, nb)))
            qv, _ = np.linalg.qr(rng.standard_normal((nb, nb)))
            c = 1e5 if np.dtype(dt) in (np.float32, np.complex64) else 1e10
            a[:, :nb] = ((qu * np.logspace(0, -np.log10(c), nb)) @ qv).astype(dt)
        A = s.from_numpy(a, nb=nb, target=tg)
        s._slate.lane_log_enable(True)
        T = s.geqrf(A, target=tg)
        log = s._slate.lane_log_take()
        s._slate.lane_log_enable(False)
        labels = [label for label, _ in log]
        if g.p > 1:
            # over all ranks: some process column ran CholeskyQR panels, and
            # the TSQR tree ran only for the rank-deficient matrix
            f = g.world.allreduce_sum_i64([int("geqrf_cholqr" in labels), int("geqrf_tsqr_local" in labels)])
            assert f[0] > 0, labels
            if case != "illcond":   # (shifted CholeskyQR3 or the tree: either is fine)
                assert (f[1] == 0) if case == "full" else (f[1] > 0), (case, f)
        r = np.triu(s.to_numpy(A)[:n])
        rref = np.linalg.qr(a, mode="r")[:n]
        if case != "illcond":   # R itself is only kappa * u accurate there
            assert relerr(np.abs(r), np.abs(rref)) < 100 * tol(dt), case
        C = s.from_numpy(a, nb=nb, target=tg)
        s.unmqr(s.Side.Left, s.Op.ConjTrans, A, T, C, target=tg)
        qa = s.to_numpy(C)
        assert relerr(np.triu(qa[:n]), r) < 100 * tol(dt), case
        assert np.abs(qa[n:]).max() <= 100 * tol(dt) * np.abs(a).max() * m, case
        # explicit Q = Q E (first n columns): orthogonal to working precision
        E = s.from_numpy(np.eye(m, n, dtype=dt), nb=nb, target=tg)
        s.unmqr(s.Side.Left, s.Op.NoTrans, A, T, E, target=tg)
        q = s.to_numpy(E)
        assert np.abs(q.conj().T @ q - np.eye(n)).max() < 100 * n * tol(dt), case


def case_norm(tg, dt, nb):
    a = rnd(170, 110, dt, 13)
    A = s.from_numpy(a, nb=nb, target=tg)
    for kind, ref in [(s.Norm.One, np.linalg.norm(a, 1)), (s.Norm.Inf, np.linalg.norm(a, np.inf)),
                      (s.Norm.Fro, np.linalg.norm(a)), (s.Norm.Max, np.abs(a).max())]:
        v = s.norm(kind, A, target=tg)
        assert abs(v - ref) <= 1e-4 * ref, (kind, v, ref)


def case_norm_masked(tg, dt, nb):
    """Hermitian and unit-triangular norms (stored triangle only) on the full
    matrix, a tile-aligned sub-view and an unaligned diagonal slice."""
    n = 200
    a = rnd(n, n, dt, 19)
    # (complex: the diagonal's imaginary part is ignored, LAPACK lanhe semantics)
    A = s.from_numpy(a, nb=nb, target=tg)
    views = [(A, a), (A.sub(1, 3, 1, 3), a[nb:4 * nb, nb:4 * nb]), (A.slice(10, 149, 10, 149), a[10:150, 10:150])]
    for V, v in views:
        for uplo in (s.Uplo.Lower, s.Uplo.Upper):
            st = np.tril(v) if uplo == s.Uplo.Lower else np.triu(v)
            h = st + (np.tril(v, -1) if uplo == s.Uplo.Lower else np.triu(v, 1)).conj().T
            h[np.diag_indices_from(h)] = np.real(np.diag(v))
            t = (np.tril(v, -1) if uplo == s.Uplo.Lower else np.triu(v, 1)) + np.eye(len(v), dtype=v.dtype)
            H = s.HermitianMatrix(uplo, V)
            T = s.TriangularMatrix(uplo, s.Diag.Unit, V)
            for kind, f in [(s.Norm.One, lambda x: np.linalg.norm(x, 1)), (s.Norm.Inf, lambda x: np.linalg.norm(x, np.inf)),
                            (s.Norm.Fro, np.linalg.norm), (s.Norm.Max, lambda x: np.abs(x).max())]:
                for M, ref in ((H, f(h)), (T, f(t))):
                    val = s.norm(kind, M, target=tg)
                    assert abs(val - ref) <= 1e-4 * ref, (kind, uplo, val, ref, v.shape)


def case_mixed(tg, dt, nb):
    n = 160
    a = rnd(n, n, np.float64, 14) + n * np.eye(n)
    b = rnd(n, 2, np.float64, 15)
    A = s.from_numpy(a, nb=nb, target=tg)
    B = s.from_numpy(b, nb=nb, target=tg)
    X = s.from_numpy(np.zeros_like(b), nb=nb, target=tg)
    info, _, it = s.gesv_mixed(A, B, X, target=tg)
    assert info == 0
    assert relerr(a @ s.to_numpy(X), b) < 1e-12


def case_tile_comm(tg, dt, nb):
    """Tile-level messages (tile_comm.cc; reference Tile::send / recv / bcast,
    BaseMatrix::tileBcast / tileLayoutConvert): a tile sent point to point, a
    tile broadcast to the owners of a block row (binomial tree over the rank
    set), received into workspace and read back; row-major conversion of a
    square local tile and of a rectangular received one, and the reset."""
    g = parallel.current_grid()
    me = parallel.world_rank()
    world = g.p * g.q
    m, n = 4 * nb + 5, 3 * nb + 7
    a = rnd(m, n, dt, 181)
    A = s.from_numpy(a, nb=nb, target=tg)
    tiles = lambda i, j: a[i * nb:min(m, (i + 1) * nb), j * nb:min(n, (j + 1) * nb)]
    # point to point: the last tile (rectangular edge tile) to every other rank in turn
    i0, j0 = A.mt - 1, A.nt - 1
    own = A.tileRank(i0, j0)
    for dst in range(world):
        if dst == own:
            continue
        if me == own:
            A.tileSend(i0, j0, dst)
        elif me == dst:
            A.tileRecv(i0, j0, own)
            assert A.tileExists(i0, j0)
            np.testing.assert_array_equal(A.tileData(i0, j0), tiles(i0, j0))
            # rectangular received tile to row-major and back
            A.tileLayoutConvert(i0, j0, s.Layout.RowMajor)
            assert A.tileLayout(i0, j0) == s.Layout.RowMajor
            np.testing.assert_array_equal(A.tileData(i0, j0), tiles(i0, j0))
            A.tileErase(i0, j0)
            assert not A.tileExists(i0, j0)
    # broadcast tile (1, 0) to the owners of block row 2
    B = A.sub(2, 2, 0, A.nt - 1)
    A.tileBcast(1, 0, B)
    owners = {A.tileRank(2, j) for j in range(A.nt)} | {A.tileRank(1, 0)}
    if me in owners:
        assert A.tileExists(1, 0)
        np.testing.assert_array_equal(A.tileData(1, 0), tiles(1, 0))
    elif not A.tileIsLocal(1, 0):
        assert not A.tileExists(1, 0)
    # explicit set (every rank), received row-major
    A.tileBcastToSet(0, 1, set(range(world)), s.Layout.RowMajor)
    np.testing.assert_array_equal(A.tileData(0, 1), tiles(0, 1))
    if not A.tileIsLocal(0, 1):
        assert A.tileLayout(0, 1) == s.Layout.RowMajor
    # square local tile: row-major in place, data unchanged as a matrix; the
    # reset puts the local array back into column-major (drivers read it)
    if A.tileIsLocal(0, 0):
        A.tileLayoutConvert(0, 0, s.Layout.RowMajor)
        assert A.tileLayout(0, 0) == s.Layout.RowMajor
        np.testing.assert_array_equal(A.tileData(0, 0), tiles(0, 0))
    A.tileLayoutReset()
    assert A.tileLayout(0, 0) == s.Layout.ColMajor
    np.testing.assert_array_equal(s.to_numpy(A), a)


def case_factor_objects(tg, dt, nb):
    """Factor-once objects (models/factor.py) on the grid: LU (tournament)
    solve of two right-hand-side blocks and a mixed-precision solve that
    refines to working precision against the untouched A."""
    n = 3 * nb + 11
    a = rnd(n, n, dt, 191) + 4 * np.eye(n, dtype=dt)
    F = s.LUFactor(s.from_numpy(a.copy(), nb=nb, target=tg), target=tg)
    for seed in (192, 193):
        b = rnd(n, 2, dt, seed)
        B = s.from_numpy(b, nb=nb, target=tg)
        F.solve(B)
        assert relerr(a @ s.to_numpy(B), b) < tol(dt)
    if dt in (np.float64, np.complex128):
        A = s.from_numpy(a, nb=nb, target=tg)
        M = s.MixedLUFactor(A, target=tg)
        b = rnd(n, 1, dt, 194)
        X, it = M.solve(s.from_numpy(b, nb=nb, target=tg))
        assert 0 <= it < 30
        assert relerr(a @ s.to_numpy(X), b) < 1e-12


CASES = {k[5:]: v for k, v in globals().items() if k.startswith("case_")}
EXTRA = {}


def main():
    p, q, tg = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    names = sys.argv[4].split(",")
    dtypes = [np.float64, np.complex64] if len(sys.argv) < 6 else [getattr(np, d) for d in sys.argv[5].split(",")]
    parallel.init_grid(p, q, transport=os.environ.get("SLATE_TRANSPORT", "auto"))
    for name in names:
        fn = CASES.get(name) or EXTRA[name]
        for dt in dtypes:
            if name == "mixed" and dt != np.float64:
                continue
            for nb in (32, 48):
                fn(tg, dt, nb)
    parallel.finalize()
    if parallel.world_rank() == 0:
        print("DIST_OK", p, q, tg, names, flush=True)


if __name__ == "__main__":
    main()
