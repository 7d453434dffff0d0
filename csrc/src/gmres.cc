// GMRES-based iterative refinement with a low-precision factorization as the
// right preconditioner (reference src/gesv_mixed_gmres.cc, posv_mixed_gmres.cc;
// Carson & Higham, "Accelerating the solution of linear systems by iterative
// refinement in three precisions", 2018).
//
// The factorization runs in fp32 on the device MFMA kernels; the matrix-vector
// products with A and the preconditioner solves are distributed operations;
// the Krylov basis (restart vectors of length n) and the small Hessenberg
// least-squares problem are replicated on every rank (O(n * restart) memory,
// negligible next to A).  One right-hand side, as in the reference.
#include "internal.hh"
#include "spread.hh"

#include <cmath>

namespace slate {

using namespace internal;

namespace {

template <typename T>
struct Vec {
    int64_t n, mb;
    GridPtr grid;
    Target target;
    int rsrc;
    template <typename U>
    Matrix<U> make(std::vector<T> const& x) const {
        Matrix<U> X(n, 1, mb, mb, grid, rsrc, 0);
        X.insertLocalTiles(Target::Host);
        Options o = {{Option::Target, Target::Host}};
        set<U>(std::function<U(int64_t, int64_t)>([&](int64_t i, int64_t) { return U(x[i]); }), X, o);
        if (target == Target::Devices) X.insertLocalTiles(Target::Devices);
        return X;
    }
    template <typename U>
    void read(Matrix<U> const& X, std::vector<T>& x) const {
        std::vector<U> t;
        Options o = {{Option::Target, target}};
        gather<U>(X, t, o);
        x.resize(n);
        for (int64_t i = 0; i < n; ++i) x[i] = T(t[i]);
    }
};

template <typename T>
real_type<T> nrm2(std::vector<T> const& v) {
    real_type<T> s = 0;
    for (auto& e : v) s += std::norm(e);
    return std::sqrt(s);
}

template <typename T>
real_type<T> nrmmax(std::vector<T> const& v) {
    real_type<T> s = 0;
    for (auto& e : v) s = std::max(s, real_type<T>(std::abs(e)));
    return s;
}

template <typename T>
T dotc(std::vector<T> const& a, std::vector<T> const& b) {
    T s = 0;
    for (size_t i = 0; i < a.size(); ++i) s += slate::conj(a[i]) * b[i];
    return s;
}

// Complex/real Givens rotation (LAPACK lartg semantics, simplified)
template <typename T>
void givens(T f, T g, real_type<T>& c, T& s, T& r) {
    using R = real_type<T>;
    R af = std::abs(f), ag = std::abs(g);
    if (ag == R(0)) { c = 1; s = 0; r = f; return; }
    if (af == R(0)) { c = 0; s = slate::conj(g) / ag; r = T(ag); return; }
    R nrm = std::hypot(af, ag);
    c = af / nrm;
    T fs = f / af;
    s = fs * slate::conj(g) / nrm;
    r = fs * nrm;
}

/// GMRES-IR core.  matvec(x, y): y = A x (distributed); precond(v, z): z = M^{-1} v.
template <typename T, typename MatVec, typename Precond>
bool gmres_ir(int64_t n, std::vector<T> const& b, std::vector<T>& x, real_type<T> Anorm, int itermax,
              int restart, MatVec&& matvec, Precond&& precond, int& iter) {
    using R = real_type<T>;
    const R eps = std::numeric_limits<R>::epsilon();
    const R cte = Anorm * eps * std::sqrt(R(n));
    std::vector<T> r(n), w(n), Ax(n);
    iter = 0;
    std::vector<std::vector<T>> V(restart + 1, std::vector<T>(n)), Z(restart, std::vector<T>(n));
    std::vector<T> H((restart + 1) * restart), g(restart + 1), sn(restart);
    std::vector<R> cs(restart);
    while (iter <= itermax) {
        matvec(x, Ax);
        for (int64_t i = 0; i < n; ++i) r[i] = b[i] - Ax[i];
        R rmax = nrmmax(r), xmax = nrmmax(x);
        if (rmax <= xmax * cte) return true;
        if (iter == itermax) break;
        R beta = nrm2(r);
        if (beta == R(0)) return true;
        for (int64_t i = 0; i < n; ++i) V[0][i] = r[i] / beta;
        std::fill(g.begin(), g.end(), T(0));
        g[0] = T(beta);
        int k = 0;
        for (; k < restart && iter < itermax; ++k) {
            ++iter;
            precond(V[k], Z[k]);
            matvec(Z[k], w);
            // modified Gram-Schmidt, twice ("twice is enough")
            for (int pass = 0; pass < 2; ++pass)
                for (int i = 0; i <= k; ++i) {
                    T h = dotc(V[i], w);
                    H[i + k * (restart + 1)] += h;
                    for (int64_t t = 0; t < n; ++t) w[t] -= h * V[i][t];
                }
            R hn = nrm2(w);
            H[k + 1 + k * (restart + 1)] = T(hn);
            if (hn > R(0)) for (int64_t t = 0; t < n; ++t) V[k + 1][t] = w[t] / hn;
            // apply previous rotations to column k, then a new one
            for (int i = 0; i < k; ++i) {
                T& h0 = H[i + k * (restart + 1)];
                T& h1 = H[i + 1 + k * (restart + 1)];
                T t0 = cs[i] * h0 + sn[i] * h1;
                h1 = -slate::conj(sn[i]) * h0 + cs[i] * h1;
                h0 = t0;
            }
            T rr;
            givens(H[k + k * (restart + 1)], H[k + 1 + k * (restart + 1)], cs[k], sn[k], rr);
            H[k + k * (restart + 1)] = rr;
            H[k + 1 + k * (restart + 1)] = T(0);
            g[k + 1] = -slate::conj(sn[k]) * g[k];
            g[k] = cs[k] * g[k];
            if (std::abs(g[k + 1]) <= cte * std::max(xmax, R(1)) * R(0.5) || hn == R(0)) { ++k; break; }
        }
        // y = H(0:k,0:k)^{-1} g(0:k); x += Z y
        std::vector<T> y(k);
        for (int i = k - 1; i >= 0; --i) {
            T s = g[i];
            for (int j = i + 1; j < k; ++j) s -= H[i + j * (restart + 1)] * y[j];
            y[i] = s / H[i + i * (restart + 1)];
        }
        for (int j = 0; j < k; ++j)
            for (int64_t t = 0; t < n; ++t) x[t] += Z[j][t] * y[j];
        std::fill(H.begin(), H.end(), T(0));
    }
    return false;
}

}  // namespace

namespace internal {

template <typename T>
bool gmres_refine(Matrix<T>& B, Matrix<T>& X, real_type<T> Anorm, int itermax, int& iters,
                  std::function<void(Matrix<T>&, Matrix<T>&)> const& residual,
                  std::function<void(Matrix<typename lower_prec<T>::type>&)> const& solve_lo, Options const& opts) {
    trace::Block tb("gmres_refine");
    using Lo = typename lower_prec<T>::type;
    Target target = resolve_target(opts);
    const int64_t n = B.m(), nrhs = B.n();
    const int restart = std::max(1, std::min(30, itermax));
    Vec<T> io{n, B.mb(), B.grid(), target, B.srow_owner(0)};
    std::vector<T> bh, xh;
    gather<T>(B, bh, opts);
    gather<T>(X, xh, opts);
    auto precond = [&](std::vector<T> const& v, std::vector<T>& z) {
        Matrix<Lo> Vm = io.template make<Lo>(v);
        solve_lo(Vm);
        io.read(Vm, z);
    };
    auto matvec = [&](std::vector<T> const& v, std::vector<T>& y) {
        Matrix<T> Vm = io.template make<T>(v);
        Matrix<T> Y = io.template make<T>(std::vector<T>(n, T(0)));
        residual(Y, Vm);                          // Y = -A v
        io.read(Y, y);
        for (auto& e : y) e = -e;
    };
    bool ok = true;
    iters = 0;
    for (int64_t j = 0; j < nrhs; ++j) {
        std::vector<T> b(bh.begin() + j * n, bh.begin() + (j + 1) * n), x(xh.begin() + j * n, xh.begin() + (j + 1) * n);
        int it = 0;
        ok = gmres_ir<T>(n, b, x, Anorm, itermax, restart, matvec, precond, it) && ok;
        iters = std::max(iters, it);
        std::copy(x.begin(), x.end(), xh.begin() + j * n);
    }
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) { return xh[i + j * n]; }), X, oh);
    return ok;
}

template bool gmres_refine<double>(Matrix<double>&, Matrix<double>&, double, int, int&,
                                   std::function<void(Matrix<double>&, Matrix<double>&)> const&,
                                   std::function<void(Matrix<float>&)> const&, Options const&);
template bool gmres_refine<std::complex<double>>(
    Matrix<std::complex<double>>&, Matrix<std::complex<double>>&, double, int, int&,
    std::function<void(Matrix<std::complex<double>>&, Matrix<std::complex<double>>&)> const&,
    std::function<void(Matrix<std::complex<float>>&)> const&, Options const&);

}  // namespace internal

template <typename T>
int64_t gesv_mixed_gmres(Matrix<T>& A, Pivots& pivots, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts) {
    {
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}, {&B, false}, {&X, true}}, [&](std::vector<Matrix<T>>& M, int r) {
                Pivots P;
                int it = 0;
                const int64_t i = gesv_mixed_gmres(M[0], P, M[1], M[2], it, opts);
                if (r == 0) { info = i; pivots = P; iter = it; }
            }))
            return info;
    }
    trace::Block tb("gesv_mixed_gmres");
    internal::DriverScope ds_;
    using Lo = typename lower_prec<T>::type;
    slate_error_if_msg(B.n() != 1, "gesv_mixed_gmres: one right-hand side");
    Target target = resolve_target(opts);
    const int itermax = int(get_option<int64_t>(opts, Option::MaxIterations, 30));
    const bool fallback = get_option<int64_t>(opts, Option::UseFallbackSolver, 1) != 0;
    const int restart = std::max(1, std::min(30, itermax));
    const int64_t n = A.n();
    Vec<T> io{n, A.mb(), A.grid(), target, A.srow_owner(0)};
    Matrix<Lo> A_lo(A.m(), A.n(), A.mb(), A.nb(), A.grid());
    A_lo.insertLocalTiles(target);
    slate::copy<T, Lo>(A, A_lo, opts);
    Pivots piv_lo;
    int64_t info = getrf(A_lo, piv_lo, opts);
    iter = 0;
    if (info == 0) {
        std::vector<T> b, x;
        io.read(B, b);
        auto precond = [&](std::vector<T> const& v, std::vector<T>& z) {
            Matrix<Lo> Vm = io.template make<Lo>(v);
            getrs(A_lo, piv_lo, Vm, opts);
            io.read(Vm, z);
        };
        auto matvec = [&](std::vector<T> const& v, std::vector<T>& y) {
            Matrix<T> Vm = io.template make<T>(v);
            Matrix<T> Y = io.template make<T>(std::vector<T>(n, T(0)));
            gemm(T(1), A, Vm, T(0), Y, opts);
            io.read(Y, y);
        };
        precond(b, x);
        real_type<T> Anorm = norm(Norm::Inf, A, opts);
        if (gmres_ir<T>(n, b, x, Anorm, itermax, restart, matvec, precond, iter)) {
            Options oh = {{Option::Target, Target::Host}};
            set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t) { return x[i]; }), X, oh);
            return 0;
        }
        iter = -iter - 1;
    } else {
        iter = -3;
    }
    if (!fallback) return info;
    slate::copy<T, T>(B, X, opts);
    return gesv(A, pivots, X, opts);
}

template <typename T>
int64_t posv_mixed_gmres(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts) {
    {
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}, {&B, false}, {&X, true}}, [&](std::vector<Matrix<T>>& M, int r) {
                auto H = internal::rewrap(A, M[0]);
                int it = 0;
                const int64_t i = posv_mixed_gmres(H, M[1], M[2], it, opts);
                if (r == 0) { info = i; iter = it; }
            }))
            return info;
    }
    trace::Block tb("posv_mixed_gmres");
    internal::DriverScope ds_;
    using Lo = typename lower_prec<T>::type;
    slate_error_if_msg(B.n() != 1, "posv_mixed_gmres: one right-hand side");
    Target target = resolve_target(opts);
    const int itermax = int(get_option<int64_t>(opts, Option::MaxIterations, 30));
    const bool fallback = get_option<int64_t>(opts, Option::UseFallbackSolver, 1) != 0;
    const int restart = std::max(1, std::min(30, itermax));
    const int64_t n = A.n();
    Vec<T> io{n, A.mb(), A.grid(), target, A.srow_owner(0)};
    Matrix<T> Ag(A);
    Ag.set_uplo(Uplo::General);
    const Uplo u = A.uplo();
    // dense Hermitian copy for the products, fp32 copy for the factorization
    Matrix<T> Afull = Ag.emptyLike();
    Afull.insertLocalTiles(target);
    {
        slate::copy<T, T>(conj_transpose(Ag), Afull, opts);
        BaseTrapezoidMatrix<T> At(u, Ag, MatrixKind::Trapezoid), Ft(u, Afull, MatrixKind::Trapezoid);
        slate::copy<T, T>(At, Ft, opts);
    }
    Matrix<Lo> A_lo(A.m(), A.n(), A.mb(), A.nb(), A.grid());
    A_lo.insertLocalTiles(target);
    slate::copy<T, Lo>(Afull, A_lo, opts);
    HermitianMatrix<Lo> H_lo(u, A_lo);
    int64_t info = potrf(H_lo, opts);
    iter = 0;
    if (info == 0) {
        std::vector<T> b, x;
        io.read(B, b);
        auto precond = [&](std::vector<T> const& v, std::vector<T>& z) {
            Matrix<Lo> Vm = io.template make<Lo>(v);
            potrs(H_lo, Vm, opts);
            io.read(Vm, z);
        };
        auto matvec = [&](std::vector<T> const& v, std::vector<T>& y) {
            Matrix<T> Vm = io.template make<T>(v);
            Matrix<T> Y = io.template make<T>(std::vector<T>(n, T(0)));
            gemm(T(1), Afull, Vm, T(0), Y, opts);
            io.read(Y, y);
        };
        precond(b, x);
        real_type<T> Anorm = norm(Norm::Inf, Afull, opts);
        if (gmres_ir<T>(n, b, x, Anorm, itermax, restart, matvec, precond, iter)) {
            Options oh = {{Option::Target, Target::Host}};
            set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t) { return x[i]; }), X, oh);
            return 0;
        }
        iter = -iter - 1;
    } else {
        iter = -3;
    }
    if (!fallback) return info;
    slate::copy<T, T>(B, X, opts);
    return posv(A, X, opts);
}

template int64_t gesv_mixed_gmres<double>(Matrix<double>&, Pivots&, Matrix<double>&, Matrix<double>&, int&,
                                          Options const&);
template int64_t gesv_mixed_gmres<std::complex<double>>(Matrix<std::complex<double>>&, Pivots&,
                                                        Matrix<std::complex<double>>&,
                                                        Matrix<std::complex<double>>&, int&, Options const&);
template int64_t posv_mixed_gmres<double>(HermitianMatrix<double>&, Matrix<double>&, Matrix<double>&, int&,
                                          Options const&);
template int64_t posv_mixed_gmres<std::complex<double>>(HermitianMatrix<std::complex<double>>&,
                                                        Matrix<std::complex<double>>&,
                                                        Matrix<std::complex<double>>&, int&, Options const&);

}  // namespace slate
