// Solvers built on the factorizations (reference src/getrs.cc, gesv.cc,
// getrs_nopiv.cc, gesv_nopiv.cc, potrs.cc, posv.cc, potri.cc, getri.cc,
// trtri.cc, trtrm.cc, gesv_mixed.cc, posv_mixed.cc, gesv_mixed_gmres.cc,
// posv_mixed_gmres.cc).
//
// Mixed precision (gesv_mixed / posv_mixed, reference gesv_mixed.cc:106-290):
// factor an fp32 copy with the fp32 MFMA kernels, solve in fp32, then refine
// in fp64: R = B - A X with the fp64 MFMA GEMM, correction solved with the
// fp32 factors, convergence by the reference's criterion
// ||R||_max < ||X||_max * ||A||_inf * eps * sqrt(n) (iterRefConverged);
// fall back to a full-precision factorization if it does not converge.
#include "internal.hh"
#include "spread.hh"

#include <cmath>

namespace slate {

using namespace internal;

namespace {
template <typename T>
TriangularMatrix<T> tri(Uplo u, Diag d, BaseMatrix<T> const& A) {
    Matrix<T> G(A);
    G.set_uplo(Uplo::General);
    return TriangularMatrix<T>(u, d, G);
}
}  // namespace

//------------------------------------------------------------------------------
template <typename T>
void getrs(Matrix<T> const& A, Pivots const& pivots, Matrix<T>& B, Options const& opts) {
    if (internal::spread<T>(opts, {{&A, false}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int) {
            getrs(M[0], pivots, M[1], opts);
        }))
        return;
    if (needs_bc(A, B)) {
        // factors of an arbitrary-layout A live in its block-cyclic tiling
        Matrix<T> Ab = bc_operand(A, opts);
        Matrix<T> Bb = block_cyclic_rows_of(Ab, B, opts);
        getrs(Ab, pivots, Bb, opts);
        slate::copy<T, T>(Bb, B, opts);
        return;
    }
    trace::Block tb("getrs");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    apply_pivots(pivots, A, B, target, true);
    trsm(Side::Left, T(1), tri<T>(Uplo::Lower, Diag::Unit, A), B, opts);
    trsm(Side::Left, T(1), tri<T>(Uplo::Upper, Diag::NonUnit, A), B, opts);
}

/// op(A) X = B with the getrf factors; op = Trans / ConjTrans:
/// A^H = U^H L^H P  =>  X = P^T L^{-H} U^{-H} B.
template <typename T>
void getrs(Op trans, Matrix<T> const& A, Pivots const& pivots, Matrix<T>& B, Options const& opts) {
    if (trans == Op::NoTrans) { getrs(A, pivots, B, opts); return; }
    if (internal::spread<T>(opts, {{&A, false}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int) {
            getrs(trans, M[0], pivots, M[1], opts);
        }))
        return;
    if (needs_bc(A, B)) {
        Matrix<T> Ab = bc_operand(A, opts);
        Matrix<T> Bb = block_cyclic_rows_of(Ab, B, opts);
        getrs(trans, Ab, pivots, Bb, opts);
        slate::copy<T, T>(Bb, B, opts);
        return;
    }
    trace::Block tb("getrs_trans");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    auto L = tri<T>(Uplo::Lower, Diag::Unit, A);
    auto U = tri<T>(Uplo::Upper, Diag::NonUnit, A);
    if (trans == Op::Trans) {
        trsm(Side::Left, T(1), transpose(U), B, opts);
        trsm(Side::Left, T(1), transpose(L), B, opts);
    } else {
        trsm(Side::Left, T(1), conj_transpose(U), B, opts);
        trsm(Side::Left, T(1), conj_transpose(L), B, opts);
    }
    apply_pivots(pivots, A, B, target, false);
}

template <typename T>
void getrs_nopiv(Matrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("getrs_nopiv");
    internal::DriverScope ds_;
    trsm(Side::Left, T(1), tri<T>(Uplo::Lower, Diag::Unit, A), B, opts);
    trsm(Side::Left, T(1), tri<T>(Uplo::Upper, Diag::NonUnit, A), B, opts);
}

template <typename T>
int64_t gesv(Matrix<T>& A, Pivots& pivots, Matrix<T>& B, Options const& opts) {
    {   // one process, several GPUs: factor and solve on the same in-process ranks
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
                Pivots P;
                const int64_t i = gesv(M[0], P, M[1], opts);
                if (rank == 0) { info = i; pivots = P; }
            }))
            return info;
    }
    if (A.arbitrary_layout() || B.arbitrary_layout()) {
        Matrix<T> Ab = internal::block_cyclic(A, opts), Bb = internal::block_cyclic(B, opts);
        int64_t info = gesv(Ab, pivots, Bb, opts);
        slate::copy<T, T>(Ab, A, opts);
        slate::copy<T, T>(Bb, B, opts);
        return info;
    }
    trace::Block tb("gesv");
    internal::DriverScope ds_;
    int64_t info = getrf(A, pivots, opts);
    if (info == 0) getrs(A, pivots, B, opts);
    return info;
}

template <typename T>
int64_t gesv_nopiv(Matrix<T>& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("gesv_nopiv");
    internal::DriverScope ds_;
    int64_t info = getrf_nopiv(A, opts);
    if (info == 0) getrs_nopiv(A, B, opts);
    return info;
}

template <typename T>
void potrs(HermitianMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    {
        const Uplo u = A.uplo();
        if (internal::spread<T>(opts, {{&A, false}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int) {
                HermitianMatrix<T> H(u, M[0]);
                potrs(H, M[1], opts);
            }))
            return;
    }
    trace::Block tb("potrs");
    internal::DriverScope ds_;
    // A = L L^H (lower) or U^H U (upper) in the physical triangle
    BaseMatrix<T> Ap = A.op() == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(A.op() == Op::ConjTrans);
    Uplo u = A.uplo_physical();
    auto Tm = tri<T>(u, Diag::NonUnit, Ap);
    if (u == Uplo::Lower) {
        trsm(Side::Left, T(1), Tm, B, opts);
        trsm(Side::Left, T(1), conj_transpose(Tm), B, opts);
    } else {
        trsm(Side::Left, T(1), conj_transpose(Tm), B, opts);
        trsm(Side::Left, T(1), Tm, B, opts);
    }
}

template <typename T>
int64_t posv(HermitianMatrix<T>& A, Matrix<T>& B, Options const& opts) {
    {
        int64_t info = 0;
        const Uplo u = A.uplo();
        if (internal::spread<T>(opts, {{&A, true}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
                HermitianMatrix<T> H(u, M[0]);
                const int64_t i = posv(H, M[1], opts);
                if (rank == 0) info = i;
            }))
            return info;
    }
    if (A.arbitrary_layout() || B.arbitrary_layout()) {
        HermitianMatrix<T> Ab(A.uplo(), internal::block_cyclic(A, opts));
        Matrix<T> Bb = internal::block_cyclic(B, opts);
        int64_t info = posv(Ab, Bb, opts);
        slate::copy<T, T>(Ab, A, opts);
        slate::copy<T, T>(Bb, B, opts);
        return info;
    }
    trace::Block tb("posv");
    internal::DriverScope ds_;
    int64_t info = potrf(A, opts);
    if (info == 0) potrs(A, B, opts);
    return info;
}

//------------------------------------------------------------------------------
// inverses
template <typename T>
int64_t trtri(TriangularMatrix<T>& A, Options const& opts) {
    trace::Block tb("trtri");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (A.grid()->size() == 1 && A.op() == Op::NoTrans) {
        lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
        LocalBlock<T> la = A.local(loc, true);
        lb::trtri(c, A.uplo(), A.diag(), la.m, la.ptr, la.ld);
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        internal::finish_origin(A, opts);
        return 0;
    }
    // distributed: solve A X = I
    Matrix<T> X = Matrix<T>(BaseMatrix<T>(A)).emptyLike();
    X.insertLocalTiles(target);
    set(T(0), T(1), X, opts);
    trsm(Side::Left, T(1), A, X, opts);
    BaseTrapezoidMatrix<T> Xt(A.uplo(), X, MatrixKind::Trapezoid);
    slate::copy<T, T>(Xt, A, opts);
    return 0;
}

template <typename T>
void trtrm(TriangularMatrix<T>& A, Options const& opts) {
    trace::Block tb("trtrm");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (A.grid()->size() == 1 && A.op() == Op::NoTrans) {
        lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
        LocalBlock<T> la = A.local(loc, true);
        lb::lauum(c, A.uplo(), la.m, la.ptr, la.ld);
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        internal::finish_origin(A, opts);
        return;
    }
    // distributed: L^H L via a dense copy of L and herk-style gemm
    Matrix<T> F = Matrix<T>(BaseMatrix<T>(A)).emptyLike();
    F.insertLocalTiles(target);
    set(T(0), T(0), F, opts);
    BaseTrapezoidMatrix<T> Ft(A.uplo(), F, MatrixKind::Trapezoid);
    slate::copy<T, T>(A, Ft, opts);
    Matrix<T> G = F.emptyLike();
    G.insertLocalTiles(target);
    if (A.uplo() == Uplo::Lower) gemm(T(1), conj_transpose(F), F, T(0), G, opts);
    else gemm(T(1), F, conj_transpose(F), T(0), G, opts);
    BaseTrapezoidMatrix<T> Gt(A.uplo(), G, MatrixKind::Trapezoid);
    slate::copy<T, T>(Gt, A, opts);
}

template <typename T>
int64_t potri(HermitianMatrix<T>& A, Options const& opts) {
    {
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}}, [&](std::vector<Matrix<T>>& M, int r) {
                auto H = internal::rewrap(A, M[0]);
                const int64_t i = potri(H, opts);
                if (r == 0) info = i;
            }, false))
            return info;
    }
    trace::Block tb("potri");
    internal::DriverScope ds_;
    int64_t info = 0;
    BaseMatrix<T> Ap = A.op() == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(A.op() == Op::ConjTrans);
    TriangularMatrix<T> Tm = tri<T>(A.uplo_physical(), Diag::NonUnit, Ap);
    info = trtri(Tm, opts);
    if (info == 0) trtrm(Tm, opts);
    return info;
}

template <typename T>
int64_t getri(Matrix<T>& A, Pivots const& pivots, Options const& opts) {
    {
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}}, [&](std::vector<Matrix<T>>& M, int r) {
                const int64_t i = getri(M[0], pivots, opts);
                if (r == 0) info = i;
            }, false))
            return info;
    }
    if (A.arbitrary_layout()) {
        Matrix<T> Ab = internal::block_cyclic(A, opts);
        int64_t info = getri(Ab, pivots, opts);
        slate::copy<T, T>(Ab, A, opts);
        return info;
    }
    trace::Block tb("getri");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    // A^{-1} = U^{-1} L^{-1} P: solve (L U) X = P^T ... via X = A^{-1} I
    Matrix<T> X = A.emptyLike();
    X.insertLocalTiles(target);
    set(T(0), T(1), X, opts);
    getrs(A, pivots, X, opts);
    slate::copy<T, T>(X, A, opts);
    return 0;
}

//------------------------------------------------------------------------------
// mixed precision iterative refinement
namespace {

template <typename T> using R_of = real_type<T>;

/// SLATE_MIXED_VERBOSE=1: per-iteration refinement distance / contraction on rank 0
bool mixed_verbose() {
    static const bool v = [] {
        const char* e = std::getenv("SLATE_MIXED_VERBOSE");
        return e && std::atoi(e) != 0;
    }();
    return v;
}

template <typename T>
bool iter_ref_converged(std::vector<real_type<T>> const& rnorm, std::vector<real_type<T>> const& xnorm,
                        real_type<T> cte) {
    for (size_t j = 0; j < rnorm.size(); ++j)
        if (!(rnorm[j] < xnorm[j] * cte)) return false;
    return true;
}

/// Mixed-precision iterative refinement.  A is the working-precision matrix
/// as a general view of its storage (for posv_mixed only its stored triangle
/// is valid); residual(Rm, X) computes Rm = Rm - A X.
template <typename T, typename Fac, typename Slv, typename FullSolve, typename Resid>
int64_t mixed_refine(Matrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts,
                     Fac&& factor_lo, Slv&& solve_lo, FullSolve&& full_solve, Resid&& residual, R_of<T> Anorm,
                     char const* name) {
    using Lo = typename lower_prec<T>::type;
    using R = real_type<T>;
    Target target = resolve_target(opts);
    const int itermax = int(get_option<int64_t>(opts, Option::MaxIterations, 30));
    const bool fallback = get_option<int64_t>(opts, Option::UseFallbackSolver, 1) != 0;
    const bool escalate = get_option<int64_t>(opts, Option::EscalateGmres, 0) != 0;
    const R eps = std::numeric_limits<R>::epsilon();
    Timer timer;
    iter = 0;
    const int64_t n = A.n(), nrhs = B.n();
    const R cte = Anorm * eps * std::sqrt(R(n));
    // low-precision copies (A_lo is the one n x n temporary, in fp32)
    Matrix<Lo> A_lo(A.m(), A.n(), A.mb(), A.nb(), A.grid());
    A_lo.insertLocalTiles(target);
    Matrix<Lo> X_lo(B.m(), B.n(), B.mb(), B.nb(), B.grid());
    X_lo.insertLocalTiles(target);
    slate::copy<T, Lo>(A, A_lo, opts);
    slate::copy<T, Lo>(B, X_lo, opts);
    timer.reset();
    int64_t info = factor_lo(A_lo);
    timers()[std::string(name) + "::factor_lo"] = timer.elapsed();
    if (info != 0) {
        iter = -3;
    } else {
        solve_lo(A_lo, X_lo);
        slate::copy<Lo, T>(X_lo, X, opts);
        Matrix<T> Rm = B.emptyLike();
        Rm.insertLocalTiles(target);
        Matrix<T> D = X.emptyLike();      // correction, allocated once
        D.insertLocalTiles(target);
        std::vector<R> rnorm(nrhs), xnorm(nrhs);
        timer.reset();
        // distance to convergence max_j rnorm_j / (xnorm_j cte) per iteration:
        // its ratio is the refinement's contraction factor
        std::vector<double> dist;
        bool stalled = false;
        for (int it = 0; it <= itermax; ++it) {
            // R = B - A X
            slate::copy<T, T>(B, Rm, opts);
            residual(Rm, X);
            colNorms(Norm::Max, X, xnorm.data(), opts);
            colNorms(Norm::Max, Rm, rnorm.data(), opts);
            double dmax = 0;
            for (int64_t j = 0; j < nrhs; ++j)
                dmax = std::max(dmax, double(rnorm[j]) / std::max(double(xnorm[j]) * double(cte), 1e-300));
            dist.push_back(dmax);
            if (mixed_verbose() && A.grid()->rank() == 0)
                std::fprintf(stderr, "# %s it %d: max_j |r_j|/(|x_j| n^1/2 eps |A|) = %.3e%s\n", name, it, dmax,
                             it > 0 ? (" contraction " + std::to_string(dmax / dist[it - 1])).c_str() : "");
            if (iter_ref_converged<T>(rnorm, xnorm, cte)) {
                iter = it;
                timers()[std::string(name) + "::iter_ref"] = timer.elapsed();
                return 0;
            }
            if (it == itermax) break;
            // stagnation / projected miss (escalation only): with contraction
            // rho the remaining log(d) / -log(rho) iterations exceed the budget
            if (escalate && it >= 3) {
                const double rho = dist[it] / dist[it - 1], rho2 = dist[it - 1] / dist[it - 2];
                const double r = std::max(rho, rho2);
                if (r >= 0.9 || (r < 1 && it + std::log(dmax) / -std::log(r) > 1.2 * itermax)) {
                    stalled = true;
                    break;
                }
            }
            // correction in low precision: X += A_lo^{-1} R
            slate::copy<T, Lo>(Rm, X_lo, opts);
            solve_lo(A_lo, X_lo);
            slate::copy<Lo, T>(X_lo, D, opts);
            add(T(1), D, T(1), X, opts);
        }
        timers()[std::string(name) + "::iter_ref"] = timer.elapsed();
        const int it_ir = int(dist.size()) - 1;
        iter = -itermax - 1;
        if (escalate) {
            // GMRES-IR from the current X with the same low-precision factors
            timer.reset();
            int it_g = 0;
            const bool ok = internal::gmres_refine<T>(B, X, Anorm, itermax, it_g, residual,
                                                      [&](Matrix<Lo>& V) { solve_lo(A_lo, V); }, opts);
            timers()[std::string(name) + "::gmres"] = timer.elapsed();
            if (mixed_verbose() && A.grid()->rank() == 0)
                std::fprintf(stderr, "# %s: classical IR %s after %d iterations, GMRES-IR %s in %d\n", name,
                             stalled ? "stalled" : "did not converge", it_ir, ok ? "converged" : "failed", it_g);
            if (ok) {
                iter = it_ir + it_g;
                return 0;
            }
            iter = -(it_ir + it_g) - 1;
        }
    }
    if (!fallback) return info;
    // fall back to a full precision solve
    timer.reset();
    slate::copy<T, T>(B, X, opts);
    info = full_solve(A, X);
    timers()[std::string(name) + "::fallback"] = timer.elapsed();
    return info;
}

}  // namespace

template <typename T>
int64_t gesv_mixed(Matrix<T>& A, Pivots& pivots, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts) {
    {   // one process, several GPUs: the whole refinement on the in-process ranks
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}, {&B, false}, {&X, true}}, [&](std::vector<Matrix<T>>& M, int r) {
                Pivots P;
                int it = 0;
                const int64_t i = gesv_mixed(M[0], P, M[1], M[2], it, opts);
                if (r == 0) { info = i; pivots = P; iter = it; }
            }))
            return info;
    }
    trace::Block tb("gesv_mixed");
    internal::DriverScope ds_;
    using Lo = typename lower_prec<T>::type;
    if constexpr (std::is_same_v<Lo, T>) {
        slate_error("gesv_mixed requires a double-precision type");
    } else {
        Pivots piv_lo;
        Matrix<T> Acopy;  // original A is needed for residuals; factorization works on A_lo
        return mixed_refine<T>(A, B, X, iter, opts,
            [&](Matrix<Lo>& A_lo) { return getrf(A_lo, piv_lo, opts); },
            [&](Matrix<Lo>& A_lo, Matrix<Lo>& X_lo) { getrs(A_lo, piv_lo, X_lo, opts); },
            [&](Matrix<T>& Af, Matrix<T>& Xf) { return gesv(Af, pivots, Xf, opts); },
            [&](Matrix<T>& Rm, Matrix<T>& Xc) { gemm(T(-1), A, Xc, T(1), Rm, opts); },
            norm(Norm::Inf, A, opts), "gesv_mixed");
    }
    return 0;
}

template <typename T>
int64_t posv_mixed(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts) {
    {
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}, {&B, false}, {&X, true}}, [&](std::vector<Matrix<T>>& M, int r) {
                auto H = internal::rewrap(A, M[0]);
                int it = 0;
                const int64_t i = posv_mixed(H, M[1], M[2], it, opts);
                if (r == 0) { info = i; iter = it; }
            }))
            return info;
    }
    trace::Block tb("posv_mixed");
    internal::DriverScope ds_;
    using Lo = typename lower_prec<T>::type;
    if constexpr (std::is_same_v<Lo, T>) {
        slate_error("posv_mixed requires a double-precision type");
    } else {
        // the stored triangle only: the residual is a distributed hemm and
        // the fp32 copy takes the triangle (no dense fp64 n x n temporary)
        Matrix<T> Ag(A);
        Ag.set_uplo(Uplo::General);
        Uplo u = A.uplo();
        return mixed_refine<T>(Ag, B, X, iter, opts,
            [&](Matrix<Lo>& A_lo) { HermitianMatrix<Lo> H(u, A_lo); return potrf(H, opts); },
            [&](Matrix<Lo>& A_lo, Matrix<Lo>& X_lo) { HermitianMatrix<Lo> H(u, A_lo); potrs(H, X_lo, opts); },
            [&](Matrix<T>&, Matrix<T>& Xf) { return posv(A, Xf, opts); },
            [&](Matrix<T>& Rm, Matrix<T>& Xc) { hemm(Side::Left, T(-1), A, Xc, T(1), Rm, opts); },
            norm(Norm::Inf, A, opts), "posv_mixed");
    }
    return 0;
}

/// Out-of-place inverse from the LU factors: B = A^{-1} (reference getriOOP.cc).
template <typename T>
int64_t getri(Matrix<T>& A, Pivots const& pivots, Matrix<T>& B, Options const& opts) {
    trace::Block tb("getriOOP");
    internal::DriverScope ds_;
    set(T(0), T(1), B, opts);
    getrs(A, pivots, B, opts);
    return 0;
}

//------------------------------------------------------------------------------
#define SLATE_SOLVE_INST(T)                                                                     \
    template void getrs<T>(Matrix<T> const&, Pivots const&, Matrix<T>&, Options const&);       \
    template void getrs<T>(Op, Matrix<T> const&, Pivots const&, Matrix<T>&, Options const&);   \
    template void getrs_nopiv<T>(Matrix<T> const&, Matrix<T>&, Options const&);                \
    template int64_t gesv<T>(Matrix<T>&, Pivots&, Matrix<T>&, Options const&);                 \
    template int64_t gesv_nopiv<T>(Matrix<T>&, Matrix<T>&, Options const&);                    \
    template void potrs<T>(HermitianMatrix<T> const&, Matrix<T>&, Options const&);             \
    template int64_t posv<T>(HermitianMatrix<T>&, Matrix<T>&, Options const&);                 \
    template int64_t trtri<T>(TriangularMatrix<T>&, Options const&);                           \
    template void trtrm<T>(TriangularMatrix<T>&, Options const&);                              \
    template int64_t potri<T>(HermitianMatrix<T>&, Options const&);                            \
    template int64_t getri<T>(Matrix<T>&, Pivots const&, Options const&);                         \
    template int64_t getri<T>(Matrix<T>&, Pivots const&, Matrix<T>&, Options const&);

SLATE_SOLVE_INST(float)
SLATE_SOLVE_INST(double)
SLATE_SOLVE_INST(std::complex<float>)
SLATE_SOLVE_INST(std::complex<double>)

template int64_t gesv_mixed<double>(Matrix<double>&, Pivots&, Matrix<double>&, Matrix<double>&, int&, Options const&);
template int64_t gesv_mixed<std::complex<double>>(Matrix<std::complex<double>>&, Pivots&, Matrix<std::complex<double>>&,
                                                  Matrix<std::complex<double>>&, int&, Options const&);
template int64_t posv_mixed<double>(HermitianMatrix<double>&, Matrix<double>&, Matrix<double>&, int&, Options const&);
template int64_t posv_mixed<std::complex<double>>(HermitianMatrix<std::complex<double>>&, Matrix<std::complex<double>>&,
                                                  Matrix<std::complex<double>>&, int&, Options const&);

}  // namespace slate
