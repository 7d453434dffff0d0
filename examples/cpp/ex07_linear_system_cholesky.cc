// ex07: Cholesky solvers (reference examples/ex07_linear_system_cholesky.cc):
// chol_solve (posv), chol_factor + solve_using_factor, inverse, condition
// estimate, and the mixed-precision posv_mixed.
#include "util.hh"

int main() {
    slate::init_grid();
    ex::banner("ex07_linear_system_cholesky");
    int fails = 0;
    const int64_t n = 400, nrhs = 4, nb = 64;
    auto o = ex::opts();
    slate::Matrix<double> Ag(n, n, nb), B(n, nrhs, nb);
    Ag.insertLocalTiles(ex::target());
    {
        slate::BaseMatrix<double>& bA = Ag;
        slate::generate_matrix(std::string("spd"), bA, 13, -1, o);   // Hermitian rands + n I
    }
    ex::random_fill(B, 14);
    auto A0 = ex::copy_of(Ag), B0 = ex::copy_of(B);
    slate::HermitianMatrix<double> A(slate::Uplo::Lower, Ag);
    int64_t info = slate::chol_solve(A, B, o);
    fails += ex::check("chol_solve", info ? 1.0 : ex::solve_residual(A0, B, B0), 1e-15);

    auto Fg = ex::copy_of(A0);
    slate::HermitianMatrix<double> F(slate::Uplo::Lower, Fg);
    info = slate::chol_factor(F, o);
    auto X = ex::copy_of(B0);
    slate::chol_solve_using_factor(F, X, o);
    fails += ex::check("chol_factor + chol_solve_using_factor", info ? 1.0 : ex::solve_residual(A0, X, B0), 1e-15);
    double rcond = slate::chol_rcondest_using_factor(slate::Norm::One, F, slate::norm(slate::Norm::One, A0, o), o);
    fails += ex::check("chol_rcondest in (0, 1]", (rcond > 0 && rcond <= 1) ? 0.0 : 1.0, 0);

    auto Mg = ex::copy_of(A0), Xm = B0.emptyLike();
    Xm.insertLocalTiles(ex::target());
    slate::HermitianMatrix<double> M(slate::Uplo::Lower, Mg);
    int iter = 0;
    info = slate::posv_mixed(M, B0, Xm, iter, o);
    fails += ex::check("posv_mixed", info ? 1.0 : ex::solve_residual(A0, Xm, B0), 1e-15);
    return ex::finish(fails);
}
