// Stage-level public API of the two-stage eigenvalue and SVD reductions and
// the symmetric/real aliases (reference slate.hh:1050-1334: unmbr_ge2tb,
// tb2bd, bdsqr, unmtr_he2hb, hb2st, unmtr_hb2st, stedc + stedc_* stages,
// steqr2, sterf, unmbr_tb2bd; syev/sygv/sygst/sysv/sytrf/sytrs, gesvd,
// svd_vals, gels_qr, gels_cholqr).
//
// The bulge-chasing stages run on the host of every rank from the gathered
// band only (O(n kd) data; the reference runs hb2st/tb2bd on one node with
// OpenMP tasks, hb2st.cc / tb2bd.cc); their reflectors are kept as
// BandReflectors, replicated on every rank, instead of the reference's V
// matrix.  The vector stages keep their matrices distributed: the reflectors /
// rotations act within columns (rows), so they run on a 1-D copy in which
// every rank holds whole columns (rows) of its share; stedc is the distributed
// divide and conquer (eig_dist.cc).  The low-level stedc_* building blocks
// (z_vector, sort, deflate, secular) keep replicated host copies: they are
// test hooks for the merge steps, not the solver's path.
#include "internal.hh"
#include "eig_sinks.hh"

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

/// Left or right application of a reflector sequence to a distributed C:
/// Left acts within columns, so C is copied to a 1 x P layout (every rank
/// holds whole columns); Right acts within rows (P x 1 layout).  Each rank
/// applies the reflectors to its own share: per-rank host memory O(m n / P).
template <typename T>
void apply_band_reflectors(Side side, Op op, BandReflectors<T> const& V, Matrix<T>& C, Options const&) {
    const int64_t m = C.m(), n = C.n();
    if (m == 0 || n == 0) return;
    Options oh = {{Option::Target, Target::Host}};
    if (side == Side::Left) {
        Matrix<T> C1(m, n, m, std::max<int64_t>(1, C.nb()), row_grid(C.grid()));
        C1.insertLocalTiles(Target::Host);
        slate::copy<T, T>(C, C1, oh);
        LocalBlock<T> l = C1.local(Loc::Host, true);
        if (l.n > 0) apply_band_reflectors_left(op, V, l.n, l.ptr, l.ld, m);
        slate::copy<T, T>(C1, C, oh);
    } else {
        // C M = (M^H C^H)^H on my rows
        Matrix<T> C1(m, n, std::max<int64_t>(1, C.mb()), n, col_grid(C.grid()));
        C1.insertLocalTiles(Target::Host);
        slate::copy<T, T>(C, C1, oh);
        LocalBlock<T> l = C1.local(Loc::Host, true);
        if (l.m > 0) {
            std::vector<T> t(size_t(n) * l.m);
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < l.m; ++i) t[j + i * n] = slate::conj(l.ptr[i + j * l.ld]);
            apply_band_reflectors_left(op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans, V, l.m, t.data(), n, n);
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < l.m; ++i) l.ptr[i + j * l.ld] = slate::conj(t[j + i * n]);
        }
        slate::copy<T, T>(C1, C, oh);
    }
}

}  // namespace

//------------------------------------------------------------------------------
template <typename T>
void hb2st(HermitianBandMatrix<T>& A, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E,
           BandReflectors<T>& V, Options const& opts) {
    trace::Block tb("hb2st");
    internal::DriverScope ds_;
    (void)opts;
    const int64_t n = A.n(), kd = A.bandwidth();
    // the lower band gathered into general band storage with room for the
    // bulge (kl = ku = 2 kd), then mirrored: (i, j) at B[M + i - j + j ldb]
    const int64_t M = 2 * std::max<int64_t>(kd, 1), ldb = 2 * M + 1;
    BaseMatrix<T> Ap = A.op() == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(A.op() == Op::ConjTrans);
    const bool lower = (A.uplo_physical() == Uplo::Lower);
    std::vector<T> B = lower ? band_gather<T>(Ap, kd, 0, M, ldb) : band_gather<T>(Ap, 0, kd, M, ldb, true);
    if (A.op() != Op::NoTrans && is_complex_v<T> && A.op() == Op::Trans)
        for (auto& x : B) x = slate::conj(x);
    for (int64_t j = 0; j < n; ++j) {
        for (int64_t i = j + 1; i <= std::min(n - 1, j + kd); ++i)
            B[size_t(M + j - i + i * ldb)] = slate::conj(B[size_t(M + i - j + j * ldb)]);
        T& dd = B[size_t(M + j * ldb)];
        dd = T(std::real(dd));
    }
    V = BandReflectors<T>{};
    host::hb2st<T>(n, kd, B.data() + M, ldb - 1, D, E, V.Q, V.phase);
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
    U = BandReflectors<T>{};
    V = BandReflectors<T>{};
    if (m == n && A.op() == Op::NoTrans && !std::getenv("SLATE_TB2BD_FULL")) {
        // band only, in general band storage with room for the bulge
        // (kl = ku = 3 kd + 2, as the svd driver): (i, j) at B[M + i - j + j ldb]
        const int64_t M = 3 * std::max<int64_t>(kd, 1) + 2, ldb = 2 * M + 1;
        std::vector<T> B = band_gather<T>(A, 0, kd, M, ldb);
        host::tb2bd<T>(m, n, kd, B.data() + M, ldb - 1, D, E, U.Q, V.Q, U.phase, V.phase);
        return;
    }
    std::vector<T> full = replicate(A, opts);
    std::vector<T> B(size_t(m) * n, T(0));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = std::max<int64_t>(0, j - kd); i <= std::min(j, m - 1); ++i) B[i + j * m] = full[i + j * m];
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
    // Z's rows are independent under the column rotations: each rank applies
    // them to its own rows (reference steqr2.cc:60-74)
    slate_error_if_msg(Z.n() != n, "steqr2: Z must have n columns");
    int64_t info = internal::steqr2_dist<T>(D, E, Z, opts);
    slate_error_if_msg(info != 0, "steqr2: QL iteration did not converge");
}

/// Distributed divide and conquer into Q (eig_dist.cc); a Q that is not a
/// square-tiled block-cyclic n x n matrix gets a block-cyclic working copy.
template <typename R>
void stedc_into(std::vector<R>& D, std::vector<R> const& E, Matrix<R>& Q, Options const& opts) {
    const int64_t n = int64_t(D.size());
    slate_error_if_msg(Q.m() != n || Q.n() != n, "stedc: Q must be n x n");
    if (!Q.arbitrary_layout() && Q.op() == Op::NoTrans && Q.mb() == Q.nb() && Q.aligned()) {
        internal::stedc_dist<R>(D, E, Q, opts);
        return;
    }
    const int64_t b = std::max<int64_t>(1, std::max(Q.mb(), Q.nb()));
    Matrix<R> Qb(n, n, b, b, Q.grid());
    Qb.insertLocalTiles(resolve_target(opts));
    internal::stedc_dist<R>(D, E, Qb, opts);
    slate::copy<R, R>(Qb, Q, opts);
}

template <typename R>
void stedc(std::vector<R>& D, std::vector<R>& E, Matrix<R>& Q, Options const& opts) {
    trace::Block tb("stedc");
    internal::DriverScope ds_;
    stedc_into(D, E, Q, opts);
}

template <typename R>
void stedc_solve(std::vector<R>& D, std::vector<R>& E, Matrix<R>& Q, Options const& opts) {
    trace::Block tb("stedc_solve");
    internal::DriverScope ds_;
    stedc_into(D, E, Q, opts);
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
    if (!wu && !wv) {
        int64_t info = host::bdsqr_core<R>(n, D.data(), E.data(), nullptr);
        slate_error_if_msg(info != 0, "bdsqr: QR iteration did not converge");
        return;
    }
    // the rotations act on columns of U and rows of VT: U's rows and VT's
    // columns (rows of Vt = VT^T) are spread over the ranks (P x 1 layouts);
    // every rank rotates its own rows, on the device through the batched
    // wavefront kernel (eig_sinks.hh)
    const Target target = resolve_target(opts);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    slate_error_if_msg((wu && U.n() != n) || (wv && VT.m() != n), "bdsqr: U must be m x n and VT n x n");
    Matrix<T> Ur, Vr;
    if (wu) {
        Ur = Matrix<T>(U.m(), n, std::max<int64_t>(1, U.mb()), std::max<int64_t>(n, 1), col_grid(U.grid()));
        Ur.insertLocalTiles(target);
        slate::copy<T, T>(U, Ur, opts);
    }
    if (wv) {
        Vr = Matrix<T>(VT.n(), n, std::max<int64_t>(1, VT.nb()), std::max<int64_t>(n, 1), col_grid(VT.grid()));
        Vr.insertLocalTiles(target);
        slate::copy<T, T>(transpose(VT), Vr, opts);
    }
    int64_t info = 0;
    {
        RowRotSink<T> sink(c, n);
        LocalBlock<T> lu, lv;
        if (wu) { lu = Ur.local(loc_of(target), true); sink.U = lu.m > 0 ? lu.ptr : nullptr; sink.ldu = lu.ld; sink.urows = lu.m; }
        if (wv) { lv = Vr.local(loc_of(target), true); sink.V = lv.m > 0 ? lv.ptr : nullptr; sink.ldv = lv.ld; sink.vrows = lv.m; }
        info = host::bdsqr_core<R>(n, D.data(), E.data(), &sink);
        sink.finish();
    }
    slate_error_if_msg(info != 0, "bdsqr: QR iteration did not converge");
    if (wu) slate::copy<T, T>(Ur, U, opts);
    if (wv) slate::copy<T, T>(transpose(Vr), VT, opts);
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
