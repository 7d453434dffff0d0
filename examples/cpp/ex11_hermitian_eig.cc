// ex11: Hermitian / symmetric eigenvalues (reference
// examples/ex11_hermitian_eig.cc): values only, then vectors (A Z = Z Lambda).
#include "util.hh"
#include <complex>
#include <vector>

template <typename T>
int run(const char* name, int64_t n, int64_t nb) {
    auto o = ex::opts();
    slate::Matrix<T> Ag(n, n, nb);
    Ag.insertLocalTiles(ex::target());
    {
        slate::BaseMatrix<T>& b = Ag;
        slate::generate_matrix(std::string("spd"), b, 22, 0.0, o);   // Hermitian rands (shift 0)
    }
    auto A0 = ex::copy_of(Ag), A1 = ex::copy_of(Ag);
    using R = slate::real_type<T>;
    std::vector<R> L0, L;
    slate::HermitianMatrix<T> H1(slate::Uplo::Lower, A1), H(slate::Uplo::Lower, Ag);
    slate::eig_vals(H1, L0, o);
    slate::Matrix<T> Z(n, n, nb);
    Z.insertLocalTiles(ex::target());
    slate::eig(H, L, Z, o);
    double dv = 0, amax = 0;
    for (size_t i = 0; i < L.size(); ++i) { dv = std::max(dv, double(std::abs(L[i] - L0[i]))); amax = std::max(amax, double(std::abs(L[i]))); }
    int fails = ex::check((std::string(name) + ": eig_vals == eig values").c_str(), dv / amax, 1e-13);
    // A Z - Z Lambda
    slate::Matrix<T> AZ(n, n, nb), ZL = ex::copy_of(Z);
    AZ.insertLocalTiles(ex::target());
    slate::multiply(T(1), A0, Z, T(0), AZ, o);
    std::vector<R> ones(n, R(1));
    slate::scale_row_col(slate::Equed::Col, ones, L, ZL, o);
    slate::add(T(-1), ZL, T(1), AZ, o);
    fails += ex::check((std::string(name) + ": A Z - Z Lambda").c_str(),
                       slate::norm(slate::Norm::One, AZ, o) / (amax * n), 1e-13);
    return fails;
}

int main() {
    slate::init_grid();
    ex::banner("ex11_hermitian_eig");
    int fails = run<double>("double", 256, 32);
    fails += run<std::complex<double>>("complex<double>", 192, 32);
    return ex::finish(fails);
}
