// ex06: LU solvers (reference examples/ex06_linear_system_lu.cc): lu_solve
// (gesv), factor + solve_using_factor, tournament pivoting (CALU), no
// pivoting, out-of-place inverse, condition estimate, mixed precision.
#include "util.hh"

int main() {
    slate::init_grid();
    ex::banner("ex06_linear_system_lu");
    int fails = 0;
    const int64_t n = 400, nrhs = 5, nb = 64;
    auto o = ex::opts();
    slate::Matrix<double> A(n, n, nb), B(n, nrhs, nb);
    ex::random_fill(A, 11); ex::random_fill(B, 12);
    auto A0 = ex::copy_of(A), B0 = ex::copy_of(B);

    int64_t info = slate::lu_solve(A, B, o);
    fails += ex::check("lu_solve", info ? 1.0 : ex::solve_residual(A0, B, B0), 1e-15);

    // factor once, solve twice; CALU (tournament pivoting) via MethodLU
    for (int method : {1, 2}) {
        auto F = ex::copy_of(A0), X = ex::copy_of(B0);
        slate::Pivots piv;
        slate::Options om = o;
        om[slate::Option::MethodLU] = int64_t(method);
        info = slate::lu_factor(F, piv, om);
        slate::lu_solve_using_factor(F, piv, X, o);
        fails += ex::check(method == 1 ? "lu_factor + solve (partial pivoting)" : "lu_factor + solve (CALU)",
                           info ? 1.0 : ex::solve_residual(A0, X, B0), 1e-15);
        if (method == 1) {
            double anorm = slate::norm(slate::Norm::One, A0, o);
            double rcond = slate::lu_rcondest_using_factor(slate::Norm::One, F, anorm, o);
            fails += ex::check("lu_rcondest in (0, 1]", (rcond > 0 && rcond <= 1) ? 0.0 : 1.0, 0);
            slate::Matrix<double> Ainv = A0.emptyLike();
            Ainv.insertLocalTiles(ex::target());
            slate::lu_inverse_using_factor_out_of_place(F, piv, Ainv, o);
            slate::Matrix<double> I = A0.emptyLike();
            I.insertLocalTiles(ex::target());
            slate::set(0.0, 1.0, I, o);
            slate::multiply(1.0, A0, Ainv, -1.0, I, o);
            fails += ex::check("A * inv(A) - I", slate::norm(slate::Norm::One, I, o) * rcond / n, 1e-14);
        }
    }
    // mixed precision: fp32 factorization + fp64 iterative refinement
    {
        auto F = ex::copy_of(A0), X = B0.emptyLike();
        X.insertLocalTiles(ex::target());
        slate::Pivots piv;
        int iter = 0;
        info = slate::gesv_mixed(F, piv, B0, X, iter, o);
        fails += ex::check("gesv_mixed (fp32 LU + fp64 refinement)", info ? 1.0 : ex::solve_residual(A0, X, B0), 1e-15);
        if (ex::rank() == 0) std::printf("  gesv_mixed iterations: %d\n", iter);
    }
    return ex::finish(fails);
}
