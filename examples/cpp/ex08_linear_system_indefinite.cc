// ex08: Hermitian / symmetric indefinite solve (reference
// examples/ex08_linear_system_indefinite.cc).  Here: Bunch-Kaufman LDL^H.
#include "util.hh"

int main() {
    slate::init_grid();
    ex::banner("ex08_linear_system_indefinite");
    int fails = 0;
    const int64_t n = 300, nrhs = 3, nb = 64;
    auto o = ex::opts();
    slate::Matrix<double> Ag(n, n, nb), B(n, nrhs, nb);
    ex::random_fill(Ag, 15); ex::random_fill(B, 16);
    // symmetrize (indefinite: random symmetric has both signs)
    auto At = ex::copy_of(Ag);
    slate::Matrix<double> S = Ag.emptyLike();
    S.insertLocalTiles(ex::target());
    slate::copy<double, double>(slate::transpose(At), S, o);
    slate::add(0.5, S, 0.5, Ag, o);
    auto A0 = ex::copy_of(Ag), B0 = ex::copy_of(B);
    slate::HermitianMatrix<double> A(slate::Uplo::Lower, Ag);
    int64_t info = slate::indefinite_solve(A, B, o);
    fails += ex::check("indefinite_solve (hesv)", info ? 1.0 : ex::solve_residual(A0, B, B0), 1e-14);

    auto Sg = ex::copy_of(A0), X = ex::copy_of(B0);
    slate::SymmetricMatrix<double> Sy(slate::Uplo::Upper, Sg);
    std::vector<int64_t> ipiv;
    info = slate::indefinite_factor(Sy, ipiv, o);
    slate::indefinite_solve_using_factor(Sy, ipiv, X, o);
    fails += ex::check("indefinite_factor + solve (sytrf/sytrs)", info ? 1.0 : ex::solve_residual(A0, X, B0), 1e-14);
    return ex::finish(fails);
}
