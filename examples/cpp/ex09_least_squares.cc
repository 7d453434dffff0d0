// ex09: least squares (reference examples/ex09_least_squares.cc):
// overdetermined (QR and CholeskyQR) and underdetermined (LQ, minimum norm).
#include "util.hh"

int main() {
    slate::init_grid();
    ex::banner("ex09_least_squares");
    int fails = 0;
    const int64_t m = 500, n = 200, nrhs = 2, nb = 50;
    auto o = ex::opts();
    // overdetermined: residual r = b - A x must be orthogonal to range(A)
    for (int method : {1, 2}) {
        slate::Matrix<double> A(m, n, nb), BX(m, nrhs, nb);
        ex::random_fill(A, 17); ex::random_fill(BX, 18);
        auto A0 = ex::copy_of(A), B0 = ex::copy_of(BX);
        slate::Options om = o;
        om[slate::Option::MethodGels] = int64_t(method);
        slate::least_squares_solve(A, BX, om);
        auto X = BX.slice(0, n - 1, 0, nrhs - 1);
        slate::Matrix<double> R = ex::copy_of(B0), G(n, nrhs, nb);
        G.insertLocalTiles(ex::target());
        slate::multiply(-1.0, A0, X, 1.0, R, o);                          // r = b - A x
        slate::multiply(1.0, slate::transpose(A0), R, 0.0, G, o);        // A^T r = 0
        double rel = slate::norm(slate::Norm::One, G, o) /
                     (slate::norm(slate::Norm::One, A0, o) * slate::norm(slate::Norm::One, B0, o));
        fails += ex::check(method == 1 ? "least squares, QR" : "least squares, CholeskyQR", rel, 1e-13);
    }
    // underdetermined: A x = b exactly (minimum-norm solution)
    {
        slate::Matrix<double> A(n, m, nb), BX(m, nrhs, nb);
        ex::random_fill(A, 19);
        ex::random_fill(BX, 20);
        auto A0 = ex::copy_of(A);
        auto Bv = BX.slice(0, n - 1, 0, nrhs - 1);
        slate::Matrix<double> B0(n, nrhs, nb);
        B0.insertLocalTiles(ex::target());
        slate::copy<double, double>(Bv, B0, o);
        slate::least_squares_solve(A, BX, o);
        fails += ex::check("underdetermined (LQ) A x = b", ex::solve_residual(A0, BX, B0), 1e-14);
    }
    return ex::finish(fails);
}
