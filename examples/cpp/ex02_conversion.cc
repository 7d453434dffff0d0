// ex02: views and conversions (reference examples/ex02_conversion.cc):
// general -> triangular / trapezoid / symmetric / Hermitian views sharing
// storage, shallow transposes, and deep copies with precision conversion.
#include "util.hh"

int main() {
    slate::init_grid();
    ex::banner("ex02_conversion");
    int fails = 0;
    const int64_t n = 300, nb = 64;
    slate::Matrix<double> A(n, n, nb);
    ex::random_fill(A, 2);
    auto o = ex::opts();

    slate::TriangularMatrix<double> L(slate::Uplo::Lower, slate::Diag::NonUnit, A);
    slate::TrapezoidMatrix<double> Z(slate::Uplo::Upper, slate::Diag::Unit, A);
    slate::SymmetricMatrix<double> Sy(slate::Uplo::Lower, A);
    slate::HermitianMatrix<double> He(slate::Uplo::Upper, A);
    fails += ex::check("views share storage", double(L.storage() != A.storage() || He.storage() != A.storage()), 0);

    auto AT = slate::transpose(A);              // shallow: no data moved
    fails += ex::check("transpose is a view", double(AT.op() != slate::Op::Trans || AT.m() != n), 0);

    // deep copy with precision conversion (the mixed-precision building block)
    slate::Matrix<float> Af(n, n, nb);
    Af.insertLocalTiles(ex::target());
    slate::copy<double, float>(A, Af, o);
    slate::Matrix<double> Ad = A.emptyLike();
    Ad.insertLocalTiles(ex::target());
    slate::copy<float, double>(Af, Ad, o);
    slate::add(-1.0, A, 1.0, Ad, o);
    double rel = slate::norm(slate::Norm::Max, Ad, o) / slate::norm(slate::Norm::Max, A, o);
    fails += ex::check("d -> s -> d round trip", rel, 1e-7);

    // materialize A^T (deep transpose through copy of the transposed view)
    slate::Matrix<double> T = AT.emptyLike();
    T.insertLocalTiles(ex::target());
    slate::copy<double, double>(AT, T, o);
    fails += ex::check("norm_one(A) == norm_inf(A^T)",
                       std::abs(slate::norm(slate::Norm::One, A, o) - slate::norm(slate::Norm::Inf, T, o)), 1e-9);
    return ex::finish(fails);
}
