// Stage-level public API of the two-stage eigenvalue and SVD reductions and
// the symmetric/real aliases (reference slate.hh:1050-1334: unmbr_ge2tb,
// tb2bd, bdsqr, unmtr_he2hb, hb2st, unmtr_hb2st, stedc + stedc_* stages,
// steqr2, sterf, unmbr_tb2bd; syev/sygv/sygst/sysv/sytrf/sytrs, gesvd,
// svd_vals, gels_qr, gels_cholqr).
//
// The bulge-chasing stages run on the host of every rank (the reference runs
// hb2st/tb2bd on one node with OpenMP tasks, hb2st.cc / tb2bd.cc); their
// reflectors are kept as BandReflectors, replicated on every rank, instead of
// the reference's V matrix.  Vector matrices are updated through replicated
// host copies and written back to each rank's local part.
#include "internal.hh"

#include <functional>

namespace slate {

using namespace internal;

namespace {

template <typename T>
std::vector<T> replicate(BaseMatrix<T> const& A, Options const& opts) {
    std::vector<T> h;
    gather(A, h, opts);
    return h;
}

template <typename T>
void write_back(Matrix<T>& M, std::vector<T> const& h, int64_t ldh) {
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) { return h[i + j * ldh]; }), M, oh);
}

template <typename T>
bool wanted(Matrix<T> const& M) { return M.m() > 0 && M.n() > 0; }

/// C (m x n, column-major) := M C  with M = Q diag(phase) (op N) or M^H (op C).
template <typename T>
void apply_band_reflectors_left(Op op, BandReflectors<T> const& V, int64_t n, T* C, int64_t ldc, int64_t m) {
    const bool have_phase = !V.phase.empty();
    if (op == Op::NoTrans) {
        if (have_phase)
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < m; ++i) C[i + j * ldc] *= V.phase[i];
        V.Q.apply_left(false, n, C, ldc);
    } else {
        V.Q.apply_left(true, n, C, ldc);
        if (have_phase)
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < m; ++i) C[i + j * ldc] *= slate::conj(V.phase[i]);
    }
}

/// Left or right application of a reflector sequence to a distributed C.
template <typename T>
void apply_band_reflectors(Side side, Op op, BandReflectors<T> const& V, Matrix<T>& C, Options const& opts) {
    const int64_t m = C.m(), n = C.n();
    std::vector<T> h = replicate(C, opts);
    if (side == Side::Left) {
        apply_band_reflectors_left(op, V, n, h.data(), m, m);
        write_back(C, h, m);
    } else {
        // C M = (M^H C^H)^H
        std::vector<T> t(size_t(n) * m);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < m; ++i) t[j + i * n] = slate::conj(h[i + j * m]);
        apply_band_reflectors_left(op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans, V, m, t.data(), n, n);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < m; ++i) h[i + j * m] = slate::conj(t[j + i * n]);
        write_back(C, h, m);
    }
}

}  // namespace

//------------------------------------------------------------------------------
template <typename T>
void hb2st(HermitianBandMatrix<T>& A, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E,
           BandReflectors<T>& V, Options const& opts) {
    trace::Block tb("hb2st");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kd = A.bandwidth();
    std::vector<T> full = replicate(A, opts);
    const bool lower = A.uplo() == Uplo::Lower;
    std::vector<T> B(size_t(n) * n, T(0));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = j; i <= std::min(n - 1, j + kd); ++i) {
            T v = lower ? full[i + j * n] : slate::conj(full[j + i * n]);
            B[i + j * n] = v;
            B[j + i * n] = slate::conj(v);
        }
    for (int64_t i = 0; i < n; ++i) B[i + i * n] = T(std::real(B[i + i * n]));
    V = BandReflectors<T>{};
    host::hb2st<T>(n, kd, B.data(), n, D, E, V.Q, V.phase);
}

template <typename T>
void unmtr_hb2st(Side side, Op op, BandReflectors<T> const& V, Matrix<T>& C, Options const& opts) {
    trace::Block tb("unmtr_hb2st");
    internal::DriverScope ds_;
    apply_band_reflectors(side, op, V, C, opts);
}

template <typename T>
void unmtr_he2hb(Side side, Op op, Matrix<T>& A, std::vector<TriangularFactors<T>>& Ts, Matrix<T>& C,
                 Options const& opts) {
    trace::Block tb("unmtr_he2hb");
    internal::DriverScope ds_;
    const int64_t nt = A.nt();
    // Q = Q_0 Q_1 ... Q_{nt-2}; Q_k acts on block rows k+1..nt-1
    auto apply = [&](int64_t k, Op o) {
        Matrix<T> panel = A.sub(k + 1, nt - 1, k, k);
        if (side == Side::Left) {
            Matrix<T> Ck = C.sub(k + 1, C.mt() - 1, 0, C.nt() - 1);
            unmqr(Side::Left, o, panel, Ts[k], Ck, opts);
        } else {
            Matrix<T> Ck = C.sub(0, C.mt() - 1, k + 1, C.nt() - 1);
            unmqr(Side::Right, o, panel, Ts[k], Ck, opts);
        }
    };
    const bool forward = (side == Side::Left) == (op != Op::NoTrans);
    if (forward) for (int64_t k = 0; k + 1 < nt; ++k) apply(k, op);
    else for (int64_t k = nt - 2; k >= 0; --k) apply(k, op);
}

template <typename T>
void tb2bd(TriangularBandMatrix<T>& A, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E,
           BandReflectors<T>& U, BandReflectors<T>& V, Options const& opts) {
    trace::Block tb("tb2bd");
    internal::DriverScope ds_;
    slate_error_if_msg(A.uplo() != Uplo::Upper, "tb2bd: A must be upper triangular band");
    const int64_t m = A.m(), n = A.n(), kd = A.bandwidth();
    std::vector<T> full = replicate(A, opts);
    std::vector<T> B(size_t(m) * n, T(0));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = std::max<int64_t>(0, j - kd); i <= std::min(j, m - 1); ++i) B[i + j * m] = full[i + j * m];
    U = BandReflectors<T>{};
    V = BandReflectors<T>{};
    host::tb2bd<T>(m, n, kd, B.data(), m, D, E, U.Q, V.Q, U.phase, V.phase);
}

template <typename T>
void unmbr_tb2bd(Side side, Op op, BandReflectors<T> const& V, Matrix<T>& C, Options const& opts) {
    trace::Block tb("unmbr_tb2bd");
    internal::DriverScope ds_;
    apply_band_reflectors(side, op, V, C, opts);
}

template <typename T>
void unmbr_ge2tb(Side side, Op op, Matrix<T>& A, std::vector<TriangularFactors<T>>& Ts, Matrix<T>& C,
                 Options const& opts) {
    trace::Block tb("unmbr_ge2tb");
    internal::DriverScope ds_;
    const int64_t mt = A.mt(), nt = A.nt();
    if (side == Side::Left) {
        // U = QU_0 ... QU_{nt-1}; QU_k = block-column k's QR reflectors
        auto apply = [&](int64_t k) {
            Matrix<T> cp = A.sub(k, mt - 1, k, k);
            Matrix<T> Ck = C.sub(k, C.mt() - 1, 0, C.nt() - 1);
            unmqr(Side::Left, op, cp, Ts[k], Ck, opts);
        };
        if (op == Op::NoTrans) for (int64_t k = nt - 1; k >= 0; --k) apply(k);
        else for (int64_t k = 0; k < nt; ++k) apply(k);
    } else {
        // V^H = ... ; QV_k = block-row k's LQ reflectors (columns k+1..)
        auto apply = [&](int64_t k) {
            Matrix<T> rp = A.sub(k, k, k + 1, nt - 1);
            Matrix<T> Ck = C.sub(0, C.mt() - 1, k + 1, C.nt() - 1);
            unmlq(Side::Right, op, rp, Ts[k], Ck, opts);
        };
        const int64_t K = int64_t(Ts.size());
        if (op == Op::NoTrans) for (int64_t k = K - 1; k >= 0; --k) apply(k);
        else for (int64_t k = 0; k < K; ++k) apply(k);
    }
}

//------------------------------------------------------------------------------
template <typename R>
void sterf(std::vector<R>& D, std::vector<R>& E, Options const&) {
    trace::Block tb("sterf");
    internal::DriverScope ds_;
    host::sterf<R>(int64_t(D.size()), D.data(), E.data());
}

template <typename T>
void steqr2(Job jobz, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E, Matrix<T>& Z,
            Options const& opts) {
    trace::Block tb("steqr2");
    internal::DriverScope ds_;
    using R = real_type<T>;
    const int64_t n = int64_t(D.size());
    if (jobz == Job::NoVec || !wanted(Z)) {
        host::sterf<R>(n, D.data(), E.data());
        return;
    }
    // Z's rows are independent under the column rotations: update the
    // replicated rows (reference steqr2 keeps them distributed per rank)
    const int64_t zm = Z.m();
    std::vector<T> h = replicate(Z, opts);
    int64_t info = host::steqr<R, T>(n, D.data(), E.data(), h.data(), zm, zm);
    slate_error_if_msg(info != 0, "steqr2: QL iteration did not converge");
    write_back(Z, h, zm);
}

template <typename R>
void stedc(std::vector<R>& D, std::vector<R>& E, Matrix<R>& Q, Options const&) {
    trace::Block tb("stedc");
    internal::DriverScope ds_;
    const int64_t n = int64_t(D.size());
    std::vector<R> h(size_t(n) * n);
    host::stedc<R>(n, D.data(), E.data(), h.data(), n);
    write_back(Q, h, n);
}

template <typename R>
void stedc_solve(std::vector<R>& D, std::vector<R>& E, Matrix<R>& Q, Options const& opts) {
    trace::Block tb("stedc_solve");
    internal::DriverScope ds_;
    const int64_t n = int64_t(D.size());
    std::vector<R> ee(E.begin(), E.end());
    ee.resize(std::max<int64_t>(n, 1), R(0));
    std::vector<R> h(size_t(n) * n);
    host::stedc_solve<R>(n, D.data(), ee.data(), h.data(), n);
    write_back(Q, h, n);
    (void)opts;
}

template <typename R>
void stedc_z_vector(Matrix<R>& Q, int64_t n1, R sgn, std::vector<R>& z, Options const& opts) {
    const int64_t n = Q.n();
    std::vector<R> h = replicate(Q, opts);
    z.resize(n);
    host::stedc_z_vector<R>(n1, n, h.data(), Q.m(), sgn, z.data());
}

template <typename R>
void stedc_sort(std::vector<R>& D, std::vector<R>& z, Matrix<R>& Q, Matrix<R>& Qout, std::vector<int64_t>& perm,
                Options const& opts) {
    const int64_t n = int64_t(D.size());
    std::vector<R> h = replicate(Q, opts), ho(size_t(n) * n);
    perm.resize(n);
    host::stedc_sort<R>(n, D.data(), z.data(), h.data(), Q.m(), ho.data(), n, perm.data());
    write_back(Qout, ho, n);
}

template <typename R>
int64_t stedc_deflate(R rho, std::vector<R>& D, std::vector<R>& z, Matrix<R>& Q, std::vector<char>& deflated,
                      Options const& opts) {
    const int64_t n = int64_t(D.size());
    std::vector<R> h = replicate(Q, opts);
    deflated.assign(n, 0);
    int64_t k = host::stedc_deflate<R>(n, rho, D.data(), z.data(), h.data(), Q.m(), deflated.data());
    write_back(Q, h, Q.m());
    return k;
}

template <typename R>
void stedc_secular(R rho, std::vector<R> const& D, std::vector<R> const& z, std::vector<R>& Lambda,
                   Matrix<R>& U, Options const&) {
    const int64_t k = int64_t(D.size());
    Lambda.resize(k);
    std::vector<R> h(size_t(k) * k);
    host::stedc_secular<R>(k, rho, D.data(), z.data(), Lambda.data(), h.data(), k);
    write_back(U, h, k);
}

template <typename R>
void stedc_merge(Matrix<R>& Q, Matrix<R>& U, Matrix<R>& Qout, Options const& opts) {
    // Qout = Q * U: the distributed GEMM of the merge step
    gemm(R(1), Q, U, R(0), Qout, opts);
}

template <typename T>
void bdsqr(Job jobu, Job jobvt, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E, Matrix<T>& U,
           Matrix<T>& VT, Options const& opts) {
    trace::Block tb("bdsqr");
    internal::DriverScope ds_;
    using R = real_type<T>;
    const int64_t n = int64_t(D.size());
    const bool wu = jobu != Job::NoVec && wanted(U), wv = jobvt != Job::NoVec && wanted(VT);
    std::vector<T> hu, hv;
    if (wu) hu = replicate(U, opts);
    if (wv) hv = replicate(VT, opts);
    const int64_t um = wu ? U.m() : 1, vn = wv ? VT.n() : 1;
    int64_t info = host::bdsqr<R, T>(n, D.data(), E.data(), wu ? hu.data() : nullptr, um, um,
                                     wv ? hv.data() : nullptr, std::max<int64_t>(n, 1), vn);
    slate_error_if_msg(info != 0, "bdsqr: QR iteration did not converge");
    if (wu) write_back(U, hu, um);
    if (wv) write_back(VT, hv, std::max<int64_t>(n, 1));
}

//------------------------------------------------------------------------------
// Real symmetric aliases (the reference enables them for real types only).
template <typename T>
void syev(SymmetricMatrix<T>& A, std::vector<real_type<T>>& Lambda, Matrix<T>& Z, Options const& opts) {
    static_assert(!is_complex_v<T>, "syev: real types only (use heev)");
    HermitianMatrix<T> H(A.uplo(), A);
    heev(H, Lambda, Z, opts);
}

template <typename T>
void sygst(int64_t itype, SymmetricMatrix<T>& A, SymmetricMatrix<T> const& B, Options const& opts) {
    static_assert(!is_complex_v<T>, "sygst: real types only (use hegst)");
    HermitianMatrix<T> HA(A.uplo(), A), HB(B.uplo(), B);
    hegst(itype, HA, HB, opts);
}

template <typename T>
void sygv(int64_t itype, SymmetricMatrix<T>& A, SymmetricMatrix<T>& B, std::vector<real_type<T>>& Lambda,
          Matrix<T>& Z, Options const& opts) {
    static_assert(!is_complex_v<T>, "sygv: real types only (use hegv)");
    HermitianMatrix<T> HA(A.uplo(), A), HB(B.uplo(), B);
    hegv(itype, HA, HB, Lambda, Z, opts);
}

template <typename T>
int64_t sytrf(SymmetricMatrix<T>& A, std::vector<int64_t>& ipiv, Options const& opts) {
    static_assert(!is_complex_v<T>, "sytrf: real types only (use hetrf)");
    HermitianMatrix<T> H(A.uplo(), A);
    return hetrf(H, ipiv, opts);
}

template <typename T>
void sytrs(SymmetricMatrix<T> const& A, std::vector<int64_t> const& ipiv, Matrix<T>& B, Options const& opts) {
    static_assert(!is_complex_v<T>, "sytrs: real types only (use hetrs)");
    HermitianMatrix<T> H(A.uplo(), A);
    hetrs(H, ipiv, B, opts);
}

template <typename T>
int64_t sysv(SymmetricMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Options const& opts) {
    static_assert(!is_complex_v<T>, "sysv: real types only (use hesv)");
    HermitianMatrix<T> H(A.uplo(), A);
    return hesv(H, ipiv, B, opts);
}

//------------------------------------------------------------------------------
template <typename T>
void svd_vals(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Options const& opts) {
    Matrix<T> U, VT;
    svd(A, Sigma, U, VT, opts);
}

template <typename T>
void gesvd(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Matrix<T>& U, Matrix<T>& VT, Options const& opts) {
    svd(A, Sigma, U, VT, opts);
}

template <typename T>
void gels_qr(Matrix<T>& A, TriangularFactors<T>& T_, Matrix<T>& BX, Options const& opts) {
    Options o = opts;
    o[Option::MethodGels] = int64_t(MethodGels::Geqrf);
    gels(A, T_, BX, o);
}

template <typename T>
void gels_cholqr(Matrix<T>& A, Matrix<T>& R, Matrix<T>& BX, Options const& opts) {
    trace::Block tb("gels_cholqr");
    internal::DriverScope ds_;
    // A = Q R with CholeskyQR; X = R^{-1} (Q^H B)   (m >= n)
    const int64_t m = A.m(), n = A.n(), nrhs = BX.n();
    slate_error_if_msg(m < n, "gels_cholqr: requires m >= n");
    int64_t info = cholqr(A, R, opts);
    slate_error_if_msg(info != 0, "gels_cholqr: Cholesky QR failed (A rank deficient?)");
    Matrix<T> B = BX.slice(0, m - 1, 0, nrhs - 1);
    Matrix<T> W(n, nrhs, BX.mb(), BX.nb(), BX.grid());
    W.insertLocalTiles(resolve_target(opts));
    gemm(T(1), conj_transpose(A), B, T(0), W, opts);
    TriangularMatrix<T> Rt(Uplo::Upper, Diag::NonUnit, R);
    trsm(Side::Left, T(1), Rt, W, opts);
    Matrix<T> X = BX.slice(0, n - 1, 0, nrhs - 1);
    slate::copy<T, T>(W, X, opts);
}

//------------------------------------------------------------------------------
#define SLATE_STAGE_INST(T)                                                                                   \
    template void hb2st<T>(HermitianBandMatrix<T>&, std::vector<real_type<T>>&, std::vector<real_type<T>>&,   \
                           BandReflectors<T>&, Options const&);                                               \
    template void unmtr_hb2st<T>(Side, Op, BandReflectors<T> const&, Matrix<T>&, Options const&);             \
    template void unmtr_he2hb<T>(Side, Op, Matrix<T>&, std::vector<TriangularFactors<T>>&, Matrix<T>&,        \
                                 Options const&);                                                             \
    template void tb2bd<T>(TriangularBandMatrix<T>&, std::vector<real_type<T>>&, std::vector<real_type<T>>&,  \
                           BandReflectors<T>&, BandReflectors<T>&, Options const&);                           \
    template void unmbr_tb2bd<T>(Side, Op, BandReflectors<T> const&, Matrix<T>&, Options const&);             \
    template void unmbr_ge2tb<T>(Side, Op, Matrix<T>&, std::vector<TriangularFactors<T>>&, Matrix<T>&,        \
                                 Options const&);                                                             \
    template void steqr2<T>(Job, std::vector<real_type<T>>&, std::vector<real_type<T>>&, Matrix<T>&,          \
                            Options const&);                                                                  \
    template void bdsqr<T>(Job, Job, std::vector<real_type<T>>&, std::vector<real_type<T>>&, Matrix<T>&,      \
                           Matrix<T>&, Options const&);                                                       \
    template void svd_vals<T>(Matrix<T>&, std::vector<real_type<T>>&, Options const&);                        \
    template void gesvd<T>(Matrix<T>&, std::vector<real_type<T>>&, Matrix<T>&, Matrix<T>&, Options const&);   \
    template void gels_qr<T>(Matrix<T>&, TriangularFactors<T>&, Matrix<T>&, Options const&);                 \
    template void gels_cholqr<T>(Matrix<T>&, Matrix<T>&, Matrix<T>&, Options const&);

#define SLATE_STAGE_REAL_INST(T)                                                                              \
    template void sterf<T>(std::vector<T>&, std::vector<T>&, Options const&);                                  \
    template void stedc<T>(std::vector<T>&, std::vector<T>&, Matrix<T>&, Options const&);                     \
    template void stedc_solve<T>(std::vector<T>&, std::vector<T>&, Matrix<T>&, Options const&);               \
    template void stedc_z_vector<T>(Matrix<T>&, int64_t, T, std::vector<T>&, Options const&);                 \
    template void stedc_sort<T>(std::vector<T>&, std::vector<T>&, Matrix<T>&, Matrix<T>&,                     \
                                std::vector<int64_t>&, Options const&);                                       \
    template int64_t stedc_deflate<T>(T, std::vector<T>&, std::vector<T>&, Matrix<T>&, std::vector<char>&,    \
                                      Options const&);                                                        \
    template void stedc_secular<T>(T, std::vector<T> const&, std::vector<T> const&, std::vector<T>&,          \
                                   Matrix<T>&, Options const&);                                               \
    template void stedc_merge<T>(Matrix<T>&, Matrix<T>&, Matrix<T>&, Options const&);                         \
    template void syev<T>(SymmetricMatrix<T>&, std::vector<T>&, Matrix<T>&, Options const&);                  \
    template void sygst<T>(int64_t, SymmetricMatrix<T>&, SymmetricMatrix<T> const&, Options const&);          \
    template void sygv<T>(int64_t, SymmetricMatrix<T>&, SymmetricMatrix<T>&, std::vector<T>&, Matrix<T>&,    \
                          Options const&);                                                                    \
    template int64_t sytrf<T>(SymmetricMatrix<T>&, std::vector<int64_t>&, Options const&);                    \
    template void sytrs<T>(SymmetricMatrix<T> const&, std::vector<int64_t> const&, Matrix<T>&, Options const&); \
    template int64_t sysv<T>(SymmetricMatrix<T>&, std::vector<int64_t>&, Matrix<T>&, Options const&);

SLATE_STAGE_INST(float)
SLATE_STAGE_INST(double)
SLATE_STAGE_INST(std::complex<float>)
SLATE_STAGE_INST(std::complex<double>)
SLATE_STAGE_REAL_INST(float)
SLATE_STAGE_REAL_INST(double)

}  // namespace slate
