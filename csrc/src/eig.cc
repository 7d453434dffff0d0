// Two-stage Hermitian eigensolver and SVD drivers (reference src/heev.cc,
// he2hb.cc, hb2st.cc, unmtr_he2hb.cc, unmtr_hb2st.cc, hegst.cc, hegv.cc,
// svd.cc, ge2tb.cc, tb2bd.cc, bdsqr.cc, unmbr_ge2tb.cc).
//
// Stage 1 (distributed, target = Devices runs on the MFMA kernels): he2hb /
// ge2tb reduce to band form with one geqrf (and gelqf) per block column and
// two-sided block updates through unmqr / unmlq, so every flop-heavy piece is
// the same device-resident QR machinery as the geqrf headline.
// Stage 2 (host, every rank redundantly, deterministic): the band (O(n nb)
// data) is gathered, chased to tridiagonal / bidiagonal (eig_host.cc), and
// solved by divide and conquer (stedc), QR iteration (steqr/sterf) or
// Golub-Reinsch (bdsqr).  The stage-2 reflectors are applied on the host, then
// the stage-1 back-transform runs distributed (unmqr / unmlq on Z, U, VT).
#include "internal.hh"
#include "slate_amd/eig_host.hh"

#include <cmath>

namespace slate {

using namespace internal;

namespace {

/// Dense Hermitian copy (both triangles) of A in a general matrix.
template <typename T>
Matrix<T> hermitian_full(HermitianMatrix<T> const& A, Options const& opts) {
    Target target = resolve_target(opts);
    Matrix<T> Ag(A);
    Ag.set_uplo(Uplo::General);
    Matrix<T> F = Ag.emptyLike();
    F.insertLocalTiles(target);
    slate::copy<T, T>(conj_transpose(Ag), F, opts);
    BaseTrapezoidMatrix<T> At(A.uplo(), Ag, MatrixKind::Trapezoid), Ft(A.uplo(), F, MatrixKind::Trapezoid);
    slate::copy<T, T>(At, Ft, opts);
    return F;
}

/// Fill a distributed matrix from a replicated host array (column-major).
template <typename T>
void fill_from_host(Matrix<T>& M, std::vector<T> const& h, int64_t ldh) {
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) { return h[i + j * ldh]; }), M, oh);
}

template <typename T>
bool wanted(Matrix<T> const& M) { return M.m() > 0 && M.n() > 0; }

}  // namespace

//------------------------------------------------------------------------------
/// he2hb: A (dense Hermitian, general storage) -> band of width nb; the
/// reflectors stay below the band, their T factors in Ts.
template <typename T>
void he2hb(Matrix<T>& A, std::vector<TriangularFactors<T>>& Ts, Options const& opts) {
    trace::Block tb("he2hb");
    internal::DriverScope ds_;
    const int64_t nt = A.nt();
    Ts.assign(std::max<int64_t>(nt - 1, 0), {});
    for (int64_t k = 0; k + 1 < nt; ++k) {
        Matrix<T> panel = A.sub(k + 1, nt - 1, k, k);
        geqrf(panel, Ts[k], opts);
        Matrix<T> A22 = A.sub(k + 1, nt - 1, k + 1, nt - 1);
        unmqr(Side::Left, Op::ConjTrans, panel, Ts[k], A22, opts);
        unmqr(Side::Right, Op::NoTrans, panel, Ts[k], A22, opts);
    }
}

template <typename T>
void heev(HermitianMatrix<T>& A, std::vector<real_type<T>>& Lambda, Matrix<T>& Z, Options const& opts) {
    trace::Block tb("heev");
    internal::DriverScope ds_;
    using R = real_type<T>;
    const int64_t n = A.n(), nb = A.nb(), nt = A.nt();
    Lambda.assign(n, R(0));
    if (n == 0) return;
    Matrix<T> F = hermitian_full(A, opts);
    std::vector<TriangularFactors<T>> Ts;
    he2hb(F, Ts, opts);
    // stage 2 on the host: band (lower, width nb) -> tridiagonal
    std::vector<T> full;
    gather(F, full, opts);
    std::vector<T> B(size_t(n) * n, T(0));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = j; i <= std::min(n - 1, j + nb); ++i) {
            B[i + j * n] = full[i + j * n];
            B[j + i * n] = slate::conj(full[i + j * n]);
        }
    for (int64_t i = 0; i < n; ++i) B[i + i * n] = T(std::real(B[i + i * n]));
    full.clear(); full.shrink_to_fit();
    std::vector<R> d, e;
    host::Reflectors<T> Q2;
    std::vector<T> phase;
    {
        trace::Block t2("hb2st");
        host::hb2st<T>(n, nb, B.data(), n, d, e, Q2, phase);
    }
    B.clear(); B.shrink_to_fit();
    if (!wanted(Z)) {
        trace::Block t2("sterf");
        host::sterf<R>(n, d.data(), e.data());
        Lambda = d;
        return;
    }
    const int64_t me = get_option<int64_t>(opts, Option::MethodEig, int64_t(MethodEig::DC));
    const bool use_qr = (me == int64_t(MethodEig::QR) || me == 'q');
    std::vector<R> Zr(size_t(n) * n, R(0));
    {
        trace::Block t2("tridiag_eig");
        if (use_qr) {
            for (int64_t i = 0; i < n; ++i) Zr[i + i * n] = R(1);
            host::steqr<R, R>(n, d.data(), e.data(), Zr.data(), n, n);
        } else {
            host::stedc<R>(n, d.data(), e.data(), Zr.data(), n);
        }
    }
    Lambda = d;
    std::vector<T> Zc(size_t(n) * n);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) Zc[i + j * n] = phase[i] * T(Zr[i + j * n]);
    Zr.clear(); Zr.shrink_to_fit();
    {
        trace::Block t2("unmtr_hb2st");
        Q2.apply_left(false, n, Zc.data(), n);
    }
    fill_from_host(Z, Zc, n);
    Target target = resolve_target(opts);
    if (target == Target::Devices) Z.insertLocalTiles(Target::Devices);
    // stage-1 back-transform (unmtr_he2hb)
    trace::Block t3("unmtr_he2hb");
    const int64_t znt = Z.nt();
    for (int64_t k = nt - 2; k >= 0; --k) {
        Matrix<T> panel = F.sub(k + 1, nt - 1, k, k);
        Matrix<T> Zk = Z.sub(k + 1, nt - 1, 0, znt - 1);
        unmqr(Side::Left, Op::NoTrans, panel, Ts[k], Zk, opts);
    }
}

//------------------------------------------------------------------------------
/// Reduce the generalized problem to standard form with the Cholesky factor
/// in B (potrf output).  itype 1: A = L^{-1} A L^{-H} (or U^{-H} A U^{-1});
/// itype 2/3: A = L^H A L (or U A U^H).  Reference src/hegst.cc.
template <typename T>
void hegst(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T> const& B, Options const& opts) {
    trace::Block tb("hegst");
    internal::DriverScope ds_;
    slate_error_if_msg(itype < 1 || itype > 3, "hegst: itype must be 1, 2 or 3");
    Target target = resolve_target(opts);
    Matrix<T> F = hermitian_full(A, opts);
    Matrix<T> Bg(B);
    Bg.set_uplo(Uplo::General);
    const bool lower = (B.uplo() == Uplo::Lower);
    TriangularMatrix<T> L(B.uplo(), Diag::NonUnit, Bg);
    // work with the lower factor L: if B stores U (= L^H), use its conj-transpose
    TriangularMatrix<T> Lw = lower ? L : TriangularMatrix<T>(conj_transpose(L));
    if (itype == 1) {
        trsm(Side::Left, T(1), Lw, F, opts);                   // L^{-1} A
        trsm(Side::Right, T(1), conj_transpose(Lw), F, opts);  // ... L^{-H}
    } else {
        trmm(Side::Left, T(1), conj_transpose(Lw), F, opts);   // L^H A
        trmm(Side::Right, T(1), Lw, F, opts);                  // ... L
    }
    // write back A's triangle
    Matrix<T> Ag(A);
    Ag.set_uplo(Uplo::General);
    BaseTrapezoidMatrix<T> Ft(A.uplo(), F, MatrixKind::Trapezoid), At(A.uplo(), Ag, MatrixKind::Trapezoid);
    slate::copy<T, T>(Ft, At, opts);
    (void)target;
}

/// Generalized Hermitian-definite eigenproblem.  Reference src/hegv.cc.
template <typename T>
void hegv(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_type<T>>& Lambda,
          Matrix<T>& Z, Options const& opts) {
    trace::Block tb("hegv");
    internal::DriverScope ds_;
    int64_t info = potrf(B, opts);
    slate_error_if_msg(info != 0, "hegv: B is not positive definite");
    hegst(itype, A, B, opts);
    heev(A, Lambda, Z, opts);
    if (!wanted(Z)) return;
    Matrix<T> Bg(B);
    Bg.set_uplo(Uplo::General);
    TriangularMatrix<T> L(B.uplo(), Diag::NonUnit, Bg);
    TriangularMatrix<T> Lw = B.uplo() == Uplo::Lower ? L : TriangularMatrix<T>(conj_transpose(L));
    if (itype == 1 || itype == 2) trsm(Side::Left, T(1), conj_transpose(Lw), Z, opts);   // x = L^{-H} y
    else trmm(Side::Left, T(1), Lw, Z, opts);                                             // x = L y
}

//------------------------------------------------------------------------------
/// ge2tb: A (m >= n) -> upper band of width nb; Householder QR of each block
/// column, LQ of each block row.  Reference src/ge2tb.cc.
template <typename T>
void ge2tb(Matrix<T>& A, std::vector<TriangularFactors<T>>& TU, std::vector<TriangularFactors<T>>& TV,
           Options const& opts) {
    trace::Block tb("ge2tb");
    internal::DriverScope ds_;
    const int64_t mt = A.mt(), nt = A.nt();
    TU.assign(nt, {});
    TV.assign(std::max<int64_t>(nt - 1, 0), {});
    for (int64_t k = 0; k < nt; ++k) {
        Matrix<T> cp = A.sub(k, mt - 1, k, k);
        geqrf(cp, TU[k], opts);
        if (k + 1 < nt) {
            Matrix<T> A2 = A.sub(k, mt - 1, k + 1, nt - 1);
            unmqr(Side::Left, Op::ConjTrans, cp, TU[k], A2, opts);
            Matrix<T> rp = A.sub(k, k, k + 1, nt - 1);
            gelqf(rp, TV[k], opts);
            if (k + 1 < mt) {
                Matrix<T> A3 = A.sub(k + 1, mt - 1, k + 1, nt - 1);
                unmlq(Side::Right, Op::ConjTrans, rp, TV[k], A3, opts);
            }
        }
    }
}

template <typename T>
void svd(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Matrix<T>& U, Matrix<T>& VT, Options const& opts) {
    trace::Block tb("svd");
    internal::DriverScope ds_;
    using R = real_type<T>;
    Target target = resolve_target(opts);
    const int64_t m = A.m(), n = A.n();
    if (m < n) {
        // A^H = U' S V'^H  =>  A = V' S U'^H
        Matrix<T> Ah = A.emptyLike(0, 0, Op::ConjTrans);
        Ah.insertLocalTiles(target);
        slate::copy<T, T>(conj_transpose(A), Ah, opts);
        Matrix<T> Uh, VTh;
        if (wanted(VT)) { Uh = Matrix<T>(n, m, Ah.mb(), Ah.nb(), Ah.grid()); Uh.insertLocalTiles(target); }
        if (wanted(U)) { VTh = Matrix<T>(m, m, Ah.nb(), Ah.nb(), Ah.grid()); VTh.insertLocalTiles(target); }
        svd(Ah, Sigma, Uh, VTh, opts);
        if (wanted(U)) slate::copy<T, T>(conj_transpose(VTh), U, opts);
        if (wanted(VT)) slate::copy<T, T>(conj_transpose(Uh), VT, opts);
        return;
    }
    const int64_t nb = A.nb();
    Matrix<T> W = A.emptyLike();
    W.insertLocalTiles(target);
    slate::copy<T, T>(A, W, opts);
    std::vector<TriangularFactors<T>> TU, TV;
    ge2tb(W, TU, TV, opts);
    std::vector<T> full;
    gather(W, full, opts);
    std::vector<T> Bd(size_t(n) * n, T(0));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = std::max<int64_t>(0, j - nb); i <= j; ++i) Bd[i + j * n] = full[i + j * m];
    full.clear(); full.shrink_to_fit();
    std::vector<R> d, e;
    host::Reflectors<T> QU2, QV2;
    std::vector<T> pu, pv;
    {
        trace::Block t2("tb2bd");
        host::tb2bd<T>(n, n, nb, Bd.data(), n, d, e, QU2, QV2, pu, pv);
    }
    Bd.clear(); Bd.shrink_to_fit();
    const bool wu = wanted(U), wv = wanted(VT);
    std::vector<T> U2, VT2;
    if (wu) { U2.assign(size_t(n) * n, T(0)); for (int64_t i = 0; i < n; ++i) U2[i + i * n] = pu[i]; }
    if (wv) { VT2.assign(size_t(n) * n, T(0)); for (int64_t i = 0; i < n; ++i) VT2[i + i * n] = slate::conj(pv[i]); }
    {
        trace::Block t2("bdsqr");
        host::bdsqr<R, T>(n, d.data(), e.data(), wu ? U2.data() : nullptr, n, n, wv ? VT2.data() : nullptr, n, n);
    }
    Sigma = d;
    if (wu) {
        QU2.apply_left(false, n, U2.data(), n);
        std::vector<T> Uh(size_t(m) * n, T(0));
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < n; ++i) Uh[i + j * m] = U2[i + j * n];
        fill_from_host(U, Uh, m);
        if (target == Target::Devices) U.insertLocalTiles(Target::Devices);
        const int64_t mt = W.mt(), unt = U.nt();
        for (int64_t k = W.nt() - 1; k >= 0; --k) {
            Matrix<T> cp = W.sub(k, mt - 1, k, k);
            Matrix<T> Uk = U.sub(k, U.mt() - 1, 0, unt - 1);
            unmqr(Side::Left, Op::NoTrans, cp, TU[k], Uk, opts);
        }
    }
    if (wv) {
        // VT2 := VT2 QV2^H  computed as (QV2 VT2^H)^H
        std::vector<T> Vh(size_t(n) * n);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < n; ++i) Vh[i + j * n] = slate::conj(VT2[j + i * n]);
        QV2.apply_left(false, n, Vh.data(), n);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < n; ++i) VT2[i + j * n] = slate::conj(Vh[j + i * n]);
        fill_from_host(VT, VT2, n);
        if (target == Target::Devices) VT.insertLocalTiles(Target::Devices);
        const int64_t nt = W.nt(), vmt = VT.mt();
        for (int64_t k = nt - 2; k >= 0; --k) {
            Matrix<T> rp = W.sub(k, k, k + 1, nt - 1);
            Matrix<T> Vk = VT.sub(0, vmt - 1, k + 1, VT.nt() - 1);
            unmlq(Side::Right, Op::NoTrans, rp, TV[k], Vk, opts);
        }
    }
}

#define SLATE_EIG_INST(T)                                                                                   \
    template void he2hb<T>(Matrix<T>&, std::vector<TriangularFactors<T>>&, Options const&);                 \
    template void heev<T>(HermitianMatrix<T>&, std::vector<real_type<T>>&, Matrix<T>&, Options const&);     \
    template void hegst<T>(int64_t, HermitianMatrix<T>&, HermitianMatrix<T> const&, Options const&);        \
    template void hegv<T>(int64_t, HermitianMatrix<T>&, HermitianMatrix<T>&, std::vector<real_type<T>>&,    \
                          Matrix<T>&, Options const&);                                                      \
    template void ge2tb<T>(Matrix<T>&, std::vector<TriangularFactors<T>>&, std::vector<TriangularFactors<T>>&, \
                           Options const&);                                                                 \
    template void svd<T>(Matrix<T>&, std::vector<real_type<T>>&, Matrix<T>&, Matrix<T>&, Options const&);

SLATE_EIG_INST(float)
SLATE_EIG_INST(double)
SLATE_EIG_INST(std::complex<float>)
SLATE_EIG_INST(std::complex<double>)

}  // namespace slate
