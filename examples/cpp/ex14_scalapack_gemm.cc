// ex14: computing on ScaLAPACK-distributed data in place (reference
// examples/ex14_scalapack_gemm.cc): wrap each rank's local block-cyclic
// arrays with fromScaLAPACK, call the driver, read the result in place.
#include "util.hh"
#include <vector>

int main() {
    auto g = slate::init_grid();
    ex::banner("ex14_scalapack_gemm");
    int fails = 0;
    const int64_t m = 300, n = 260, k = 280, nb = 32;
    auto loc = [&](int64_t rows, int64_t cols, std::vector<double>& v, int64_t& lld) {
        int64_t ml = slate::numroc(rows, nb, g->myrow(), g->p()), nl = slate::numroc(cols, nb, g->mycol(), g->q());
        lld = std::max<int64_t>(ml, 1);
        v.assign(size_t(lld) * std::max<int64_t>(nl, 1), 0.0);
        // global (i, j) -> value: a smooth function, so every rank can check
        for (int64_t jl = 0; jl < nl; ++jl)
            for (int64_t il = 0; il < ml; ++il) {
                int64_t i = slate::l2g(il, nb, g->myrow(), g->p()), j = slate::l2g(jl, nb, g->mycol(), g->q());
                v[il + jl * lld] = std::sin(0.01 * double(i + 1)) * std::cos(0.02 * double(j + 1));
            }
    };
    std::vector<double> a, b, c;
    int64_t lda, ldb, ldc;
    loc(m, k, a, lda); loc(k, n, b, ldb); loc(m, n, c, ldc);
    auto A = slate::Matrix<double>::fromScaLAPACK(m, k, a.data(), lda, nb, nb, g);
    auto B = slate::Matrix<double>::fromScaLAPACK(k, n, b.data(), ldb, nb, nb, g);
    auto C = slate::Matrix<double>::fromScaLAPACK(m, n, c.data(), ldc, nb, nb, g);
    slate::gemm(1.0, A, B, 0.0, C, ex::opts());
    C.tileUpdateAllOrigin();
    // C(i, j) = sum_l sin(.01(i+1)) cos(.02(l+1)) sin(.01(l+1)) cos(.02(j+1))
    double s = 0;
    for (int64_t l = 0; l < k; ++l) s += std::cos(0.02 * double(l + 1)) * std::sin(0.01 * double(l + 1));
    double err = 0;
    int64_t ml = slate::numroc(m, nb, g->myrow(), g->p()), nl = slate::numroc(n, nb, g->mycol(), g->q());
    for (int64_t jl = 0; jl < nl; ++jl)
        for (int64_t il = 0; il < ml; ++il) {
            int64_t i = slate::l2g(il, nb, g->myrow(), g->p()), j = slate::l2g(jl, nb, g->mycol(), g->q());
            double ref = std::sin(0.01 * double(i + 1)) * std::cos(0.02 * double(j + 1)) * s;
            err = std::max(err, std::abs(c[il + jl * ldc] - ref));
        }
    fails += ex::check("gemm on ScaLAPACK local arrays", err, 1e-12);
    return ex::finish(fails);
}
