// ex12: generalized Hermitian-definite eigenproblem A x = lambda B x
// (reference examples/ex12_generalized_hermitian_eig.cc).
#include "util.hh"
#include <vector>

int main() {
    slate::init_grid();
    ex::banner("ex12_generalized_hermitian_eig");
    int fails = 0;
    const int64_t n = 200, nb = 40;
    auto o = ex::opts();
    slate::Matrix<double> Ag(n, n, nb), Bg(n, n, nb);
    Ag.insertLocalTiles(ex::target()); Bg.insertLocalTiles(ex::target());
    {
        slate::BaseMatrix<double>& a = Ag;
        slate::BaseMatrix<double>& b = Bg;
        slate::generate_matrix(std::string("spd"), a, 23, 0.0, o);
        slate::generate_matrix(std::string("spd"), b, 24, -1, o);   // + n I: positive definite
    }
    auto A0 = ex::copy_of(Ag), B0 = ex::copy_of(Bg);
    slate::HermitianMatrix<double> A(slate::Uplo::Lower, Ag), B(slate::Uplo::Lower, Bg);
    std::vector<double> L;
    slate::Matrix<double> Z(n, n, nb);
    Z.insertLocalTiles(ex::target());
    slate::eig(1, A, B, L, Z, o);
    // A Z - B Z Lambda
    slate::Matrix<double> AZ(n, n, nb), BZ(n, n, nb);
    AZ.insertLocalTiles(ex::target()); BZ.insertLocalTiles(ex::target());
    slate::multiply(1.0, A0, Z, 0.0, AZ, o);
    slate::multiply(1.0, B0, Z, 0.0, BZ, o);
    std::vector<double> ones(n, 1.0);
    slate::scale_row_col(slate::Equed::Col, ones, L, BZ, o);
    slate::add(-1.0, BZ, 1.0, AZ, o);
    double lmax = 0;
    for (double v : L) lmax = std::max(lmax, std::abs(v));
    fails += ex::check("A Z - B Z Lambda", slate::norm(slate::Norm::One, AZ, o) /
                       (slate::norm(slate::Norm::One, A0, o) + lmax * slate::norm(slate::Norm::One, B0, o)) / n, 1e-13);
    return ex::finish(fails);
}
