// ex15: setting matrix entries (reference examples/ex15_set_matrix.cc):
// constant off-diagonal / diagonal values, and an element-wise lambda of the
// global indices.
#include "util.hh"

int main() {
    slate::init_grid();
    ex::banner("ex15_set_matrix");
    int fails = 0;
    const int64_t m = 200, n = 150, nb = 32;
    auto o = ex::opts();
    slate::Matrix<double> A(m, n, nb);
    A.insertLocalTiles(ex::target());
    slate::set(2.0, 5.0, A, o);                                   // 2 off the diagonal, 5 on it
    fails += ex::check("set(offdiag, diag): max", std::abs(slate::norm(slate::Norm::Max, A, o) - 5), 0);
    slate::set<double>([](int64_t i, int64_t j) { return double(i) - 0.5 * double(j); }, A, o);
    double err = 0;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i)
            if (A.tileIsLocal(i / nb, j / nb)) {
                A.tileGetAllForReading(slate::Loc::Host);
                err = std::max(err, std::abs(A.elem(i, j) - (double(i) - 0.5 * double(j))));
            }
    fails += ex::check("set(lambda of global indices)", err, 0);
    slate::TriangularMatrix<double> L(slate::Uplo::Lower, slate::Diag::NonUnit, A.slice(0, n - 1, 0, n - 1));
    slate::set(0.0, 1.0, L, o);                                  // only the lower triangle changes
    fails += ex::check("set on a triangular view keeps the upper part",
                       std::abs(slate::norm(slate::Norm::Max, A.slice(0, 0, n - 1, n - 1), o) - 0.5 * double(n - 1)), 0);
    slate::print("A", A, {{slate::Option::PrintEdgeItems, int64_t(3)}, {slate::Option::PrintPrecision, int64_t(1)}});
    return ex::finish(fails);
}
