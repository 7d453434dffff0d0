// ex05: level-3 BLAS through the simplified API (reference
// examples/ex05_blas.cc): multiply (gemm/hemm/symm), rank_k_update (herk),
// rank_2k_update (her2k), triangular_multiply / triangular_solve (trmm/trsm).
#include "util.hh"

int main() {
    slate::init_grid();
    ex::banner("ex05_blas");
    int fails = 0;
    const int64_t m = 384, n = 256, k = 320, nb = 64;
    auto o = ex::opts();
    slate::Matrix<double> A(m, k, nb), B(k, n, nb), C(m, n, nb);
    ex::random_fill(A, 5); ex::random_fill(B, 6); ex::random_fill(C, 7);
    // gemm checked by multiplying with a random X: C X = A (B X) + C0 X (reference test_gemm.cc)
    slate::Matrix<double> X(n, 8, nb), CX(m, 8, nb), BX(k, 8, nb), R(m, 8, nb);
    ex::random_fill(X, 8);
    for (auto* M : {&CX, &BX, &R}) M->insertLocalTiles(ex::target());
    slate::multiply(1.0, C, X, 0.0, R, o);                       // R = C0 X
    slate::multiply(2.0, A, B, -1.0, C, o);                      // C = 2 A B - C0
    slate::multiply(1.0, C, X, 0.0, CX, o);
    slate::multiply(1.0, B, X, 0.0, BX, o);
    slate::multiply(2.0, A, BX, -1.0, R, o);                     // R = 2 A B X - C0 X
    slate::add(-1.0, CX, 1.0, R, o);
    fails += ex::check("multiply (gemm)", slate::norm(slate::Norm::One, R, o) / slate::norm(slate::Norm::One, CX, o), 1e-13);

    // herk C = A A^T, compare with gemm
    slate::Matrix<double> Cg(m, m, nb), Ch(m, m, nb);
    Cg.insertLocalTiles(ex::target()); Ch.insertLocalTiles(ex::target());
    slate::set(0.0, 0.0, Ch, o);
    slate::HermitianMatrix<double> H(slate::Uplo::Lower, Ch);
    slate::rank_k_update(1.0, A, 0.0, H, o);
    slate::multiply(1.0, A, slate::transpose(A), 0.0, Cg, o);
    slate::TriangularMatrix<double> Lh(slate::Uplo::Lower, slate::Diag::NonUnit, Ch), Lg(slate::Uplo::Lower, slate::Diag::NonUnit, Cg);
    slate::BaseTrapezoidMatrix<double> Th(slate::Uplo::Lower, Ch, slate::MatrixKind::Trapezoid),
                                       Tg(slate::Uplo::Lower, Cg, slate::MatrixKind::Trapezoid);
    slate::add(-1.0, Tg, 1.0, Th, o);
    fails += ex::check("rank_k_update (herk)", slate::norm(slate::Norm::Max, Lh, o) / slate::norm(slate::Norm::Max, Lg, o), 1e-13);

    // trsm(trmm(B)) == B with a well-conditioned triangle
    slate::Matrix<double> T(k, k, nb);
    T.insertLocalTiles(ex::target());
    slate::set(0.0, double(k), T, o);                            // k I + random: well conditioned
    slate::Matrix<double> T2(k, k, nb);
    ex::random_fill(T2, 10);
    slate::add(1.0, T2, 1.0, T, o);
    slate::TriangularMatrix<double> U(slate::Uplo::Upper, slate::Diag::NonUnit, T);
    auto B0 = ex::copy_of(B);
    slate::triangular_multiply(1.0, U, B, o);
    slate::triangular_solve(1.0, U, B, o);
    slate::add(-1.0, B0, 1.0, B, o);
    fails += ex::check("triangular_solve(triangular_multiply(B))",
                       slate::norm(slate::Norm::Max, B, o) / slate::norm(slate::Norm::Max, B0, o), 1e-12);
    return ex::finish(fails);
}
