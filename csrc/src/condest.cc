// Condition-number estimators (reference src/gecondest.cc, pocondest.cc,
// trcondest.cc, internal_norm1est.cc): Higham's 1-norm estimator (LAPACK
// lacn2, Higham 1988 "FORTRAN codes for estimating the one-norm of a real or
// complex matrix") driven by distributed triangular solves with the factors.
//
// The estimator's vectors are n-long and replicated on every rank (O(n) next
// to the O(n^2) solves); each "apply" fills a distributed n x 1 right-hand
// side conforming to A's rows, runs the solves on the target (device MFMA
// trsm when target = Devices), and gathers the result back.
#include "internal.hh"

#include <cmath>

namespace slate {

using namespace internal;

namespace {

template <typename T>
TriangularMatrix<T> tri_view(Uplo u, Diag d, BaseMatrix<T> const& A) {
    Matrix<T> G(A);
    G.set_uplo(Uplo::General);
    return TriangularMatrix<T>(u, d, G);
}

/// Replicated host vector <-> distributed n x 1 column conforming to A's rows.
template <typename T>
struct VecIO {
    int64_t n, mb;
    GridPtr grid;
    Target target;
    int rsrc;
    Matrix<T> make(std::vector<T> const& x) const {
        Matrix<T> X(n, 1, mb, mb, grid, rsrc, 0);
        X.insertLocalTiles(Target::Host);
        Options o = {{Option::Target, Target::Host}};
        set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t) { return x[i]; }), X, o);
        if (target == Target::Devices) X.insertLocalTiles(Target::Devices);
        return X;
    }
    void read(Matrix<T> const& X, std::vector<T>& x) const {
        Options o = {{Option::Target, target}};
        gather<T>(X, x, o);
    }
};

template <typename T>
real_type<T> sgn_abs(T const& v) { return std::abs(v); }

/// Higham's estimator of ||M||_1 given y = M x (kase 1) and y = M^H x (kase 2).
template <typename T, typename Apply>
real_type<T> norm1est(int64_t n, Apply&& apply) {
    using R = real_type<T>;
    if (n <= 0) return R(0);
    auto nrm1 = [](std::vector<T> const& v) { R s = 0; for (auto& e : v) s += std::abs(e); return s; };
    auto sign = [](T v) -> T {
        R a = std::abs(v);
        if (a == R(0)) return T(1);
        return v / a;
    };
    auto argmax = [](std::vector<T> const& v) {
        int64_t j = 0; R mx = -1;
        for (int64_t i = 0; i < int64_t(v.size()); ++i) {
            R a = is_complex_v<T> ? std::abs(v[i]) : std::abs(std::real(v[i]));
            if (a > mx) { mx = a; j = i; }
        }
        return j;
    };
    std::vector<T> x(n, T(R(1) / R(n))), y, z;
    apply(1, x, y);
    if (n == 1) return std::abs(y[0]);
    R est = nrm1(y);
    std::vector<T> xi(n);
    for (int64_t i = 0; i < n; ++i) xi[i] = sign(y[i]);
    apply(2, xi, z);
    int64_t j = argmax(z);
    const int itmax = 5;
    for (int iter = 2; iter <= itmax; ++iter) {
        std::fill(x.begin(), x.end(), T(0));
        x[j] = T(1);
        apply(1, x, y);
        R estold = est;
        est = nrm1(y);
        bool same = true;
        for (int64_t i = 0; i < n && same; ++i) same = (sign(y[i]) == xi[i]);
        if ((!is_complex_v<T> && same) || est <= estold) { est = std::max(est, estold); break; }
        for (int64_t i = 0; i < n; ++i) xi[i] = sign(y[i]);
        apply(2, xi, z);
        int64_t jlast = j;
        j = argmax(z);
        if (std::abs(z[jlast]) == std::abs(z[j])) break;
    }
    // alternating-sign test vector (protects against special structures)
    for (int64_t i = 0; i < n; ++i) {
        R v = R(1) + R(i) / R(n - 1);
        x[i] = T((i % 2) ? -v : v);
    }
    apply(1, x, y);
    R temp = R(2) * nrm1(y) / R(3 * n);
    return std::max(est, temp);
}

template <typename T>
int row0_src(BaseMatrix<T> const& A) { return A.srow_owner(0); }

}  // namespace

/// rcond of A from its LU factors (getrf output; pivots do not change the
/// 1- or inf-norm of A^{-1}).  Reference src/gecondest.cc.
template <typename T>
real_type<T> gecondest(Norm in_norm, Matrix<T>& A, real_type<T> Anorm, Options const& opts) {
    trace::Block tb("gecondest");
    internal::DriverScope ds_;
    using R = real_type<T>;
    slate_error_if_msg(in_norm != Norm::One && in_norm != Norm::Inf, "gecondest: norm must be One or Inf");
    const int64_t n = A.n();
    if (n == 0) return R(1);
    if (Anorm == R(0)) return R(0);
    Target target = resolve_target(opts);
    VecIO<T> io{n, A.mb(), A.grid(), target, row0_src(A)};
    auto L = tri_view<T>(Uplo::Lower, Diag::Unit, A);
    auto U = tri_view<T>(Uplo::Upper, Diag::NonUnit, A);
    // kase 1 applies M, kase 2 applies M^H; M = A^{-1} (One) or A^{-H} (Inf)
    auto apply = [&](int kase, std::vector<T> const& x, std::vector<T>& y) {
        Matrix<T> X = io.make(x);
        bool inv = (kase == 1) == (in_norm == Norm::One);
        if (inv) {      // A^{-1} x = U^{-1} L^{-1} x
            trsm(Side::Left, T(1), L, X, opts);
            trsm(Side::Left, T(1), U, X, opts);
        } else {        // A^{-H} x = L^{-H} U^{-H} x
            trsm(Side::Left, T(1), conj_transpose(U), X, opts);
            trsm(Side::Left, T(1), conj_transpose(L), X, opts);
        }
        io.read(X, y);
    };
    R ainv = norm1est<T>(n, apply);
    return ainv == R(0) ? R(0) : (R(1) / ainv) / Anorm;
}

/// rcond of a Hermitian positive definite A from its Cholesky factor.
/// Reference src/pocondest.cc.
template <typename T>
real_type<T> pocondest(Norm in_norm, HermitianMatrix<T>& A, real_type<T> Anorm, Options const& opts) {
    trace::Block tb("pocondest");
    internal::DriverScope ds_;
    using R = real_type<T>;
    slate_error_if_msg(in_norm != Norm::One && in_norm != Norm::Inf, "pocondest: norm must be One or Inf");
    const int64_t n = A.n();
    if (n == 0) return R(1);
    if (Anorm == R(0)) return R(0);
    Target target = resolve_target(opts);
    VecIO<T> io{n, A.mb(), A.grid(), target, row0_src(BaseMatrix<T>(A))};
    // A^{-1} is Hermitian: both kases apply potrs
    auto apply = [&](int, std::vector<T> const& x, std::vector<T>& y) {
        Matrix<T> X = io.make(x);
        potrs(A, X, opts);
        io.read(X, y);
    };
    R ainv = norm1est<T>(n, apply);
    return ainv == R(0) ? R(0) : (R(1) / ainv) / Anorm;
}

/// rcond of a triangular matrix (its norm computed here).
/// Reference src/trcondest.cc.
template <typename T>
real_type<T> trcondest(Norm in_norm, TriangularMatrix<T>& A, Options const& opts) {
    trace::Block tb("trcondest");
    internal::DriverScope ds_;
    using R = real_type<T>;
    slate_error_if_msg(in_norm != Norm::One && in_norm != Norm::Inf, "trcondest: norm must be One or Inf");
    const int64_t n = A.n();
    if (n == 0) return R(1);
    R Anorm = norm(in_norm, A, opts);
    if (Anorm == R(0)) return R(0);
    Target target = resolve_target(opts);
    VecIO<T> io{n, A.mb(), A.grid(), target, row0_src(BaseMatrix<T>(A))};
    auto apply = [&](int kase, std::vector<T> const& x, std::vector<T>& y) {
        Matrix<T> X = io.make(x);
        bool inv = (kase == 1) == (in_norm == Norm::One);
        if (inv) trsm(Side::Left, T(1), A, X, opts);
        else     trsm(Side::Left, T(1), conj_transpose(A), X, opts);
        io.read(X, y);
    };
    R ainv = norm1est<T>(n, apply);
    return ainv == R(0) ? R(0) : (R(1) / ainv) / Anorm;
}

#define SLATE_CONDEST_INST(T)                                                                   \
    template real_type<T> gecondest<T>(Norm, Matrix<T>&, real_type<T>, Options const&);         \
    template real_type<T> pocondest<T>(Norm, HermitianMatrix<T>&, real_type<T>, Options const&); \
    template real_type<T> trcondest<T>(Norm, TriangularMatrix<T>&, Options const&);

SLATE_CONDEST_INST(float)
SLATE_CONDEST_INST(double)
SLATE_CONDEST_INST(std::complex<float>)
SLATE_CONDEST_INST(std::complex<double>)

}  // namespace slate
