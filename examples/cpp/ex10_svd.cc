// ex10: singular value decomposition (reference examples/ex10_svd.cc):
// values only, then thin U / V^T with the reconstruction A = U S V^T.
#include "util.hh"
#include <vector>

int main() {
    slate::init_grid();
    ex::banner("ex10_svd");
    int fails = 0;
    const int64_t m = 300, n = 200, nb = 50;
    auto o = ex::opts();
    slate::Matrix<double> A(m, n, nb);
    ex::random_fill(A, 21);
    auto A0 = ex::copy_of(A), A1 = ex::copy_of(A);
    std::vector<double> S0, S;
    slate::svd_vals(A1, S0, o);
    slate::Matrix<double> U(m, n, nb), VT(n, n, nb);
    U.insertLocalTiles(ex::target()); VT.insertLocalTiles(ex::target());
    slate::svd(A, S, U, VT, o);
    double dv = 0;
    for (size_t i = 0; i < S.size(); ++i) dv = std::max(dv, std::abs(S[i] - S0[i]));
    fails += ex::check("singular values with / without vectors", dv / S[0], 1e-13);
    // U diag(S) V^T - A
    slate::Matrix<double> US = ex::copy_of(U);
    std::vector<double> ones(m, 1.0);
    slate::scale_row_col(slate::Equed::Col, ones, S, US, o);
    slate::multiply(1.0, US, VT, -1.0, A0, o);
    fails += ex::check("A - U S V^T", slate::norm(slate::Norm::One, A0, o) / (S[0] * m), 1e-14);
    if (ex::rank() == 0) slate::print("Sigma", int64_t(S.size()), S.data(), 1, {{slate::Option::PrintEdgeItems, int64_t(4)}});
    return ex::finish(fails);
}
