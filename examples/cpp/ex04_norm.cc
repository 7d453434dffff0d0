// ex04: matrix norms (reference examples/ex04_norm.cc): one, inf, max, Frobenius
// for general, triangular, symmetric/Hermitian views, and column norms.
#include "util.hh"
#include <vector>

int main() {
    slate::init_grid();
    ex::banner("ex04_norm");
    int fails = 0;
    const int64_t n = 256, nb = 48;
    slate::Matrix<double> A(n, n, nb);
    A.insertLocalTiles(ex::target());
    auto o = ex::opts();
    slate::set(1.0, 1.0, A, o);                   // all ones
    fails += ex::check("one-norm of ones", std::abs(slate::norm(slate::Norm::One, A, o) - n), 1e-12);
    fails += ex::check("inf-norm of ones", std::abs(slate::norm(slate::Norm::Inf, A, o) - n), 1e-12);
    fails += ex::check("max-norm of ones", std::abs(slate::norm(slate::Norm::Max, A, o) - 1), 1e-12);
    fails += ex::check("fro-norm of ones", std::abs(slate::norm(slate::Norm::Fro, A, o) - double(n)), 1e-9);
    slate::TriangularMatrix<double> L(slate::Uplo::Lower, slate::Diag::NonUnit, A);
    fails += ex::check("one-norm of lower(ones)", std::abs(slate::norm(slate::Norm::One, L, o) - n), 1e-12);
    fails += ex::check("inf-norm of lower(ones)", std::abs(slate::norm(slate::Norm::Inf, L, o) - n), 1e-12);
    slate::HermitianMatrix<double> H(slate::Uplo::Lower, A);
    fails += ex::check("fro-norm of Hermitian(ones)", std::abs(slate::norm(slate::Norm::Fro, H, o) - double(n)), 1e-9);
    std::vector<double> cn(n);
    slate::colNorms(slate::Norm::Max, A, cn.data(), o);
    double e = 0;
    for (double v : cn) e = std::max(e, std::abs(v - 1));
    fails += ex::check("column max-norms", e, 0);
    return ex::finish(fails);
}
