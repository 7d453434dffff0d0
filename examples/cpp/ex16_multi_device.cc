// ex16: one process, its matrices spread over several GPUs (reference: an
// MPI rank gives its tiles to all of its GPUs, MatrixStorage.hh:503-506, and
// Matrix::fromDevices(Aarray, num_devices), Matrix.hh:396-404).
//
// Matrix::multiDevice places a matrix 2-D block-cyclic over the in-process
// ranks of this process (one per GPU; SLATE_INPROC_RANKS overrides the count,
// e.g. 4 ranks sharing one GPU); the drivers run on those ranks in place.
// Factor once and solve twice: the copy counter (inproc_copy_bytes) shows
// that no matrix data moves between the caller and the devices after the
// one-time load -- unlike calls on one-GPU matrices, which are scattered to
// the ranks and gathered back on every call.
#include "util.hh"

#include <vector>

int main() {
    ex::banner("ex16_multi_device");
    int fails = 0;
    const int64_t n = 1000, nrhs = 4, nb = 96;
    const int nd = slate::inproc_ranks() > 1 ? 0 : 4;   // every usable GPU, else 4 ranks on this one
    // host data, loaded once
    std::vector<double> a(size_t(n) * n), b(size_t(n) * nrhs);
    uint64_t x = 12345;
    auto rnd = [&] { x = x * 6364136223846793005ull + 1442695040888963407ull; return double(x >> 11) * 0x1p-53 - 0.5; };
    for (auto& v : a) v = rnd();
    for (int64_t i = 0; i < n; ++i) a[size_t(i) + size_t(i) * n] += 4.0;
    for (auto& v : b) v = rnd();
    auto Ah = slate::Matrix<double>::fromLAPACK(n, n, a.data(), n, nb);
    auto Bh = slate::Matrix<double>::fromLAPACK(n, nrhs, b.data(), n, nb);

    auto A = slate::Matrix<double>::multiDevice(n, n, nb, nb, nd);
    auto B1 = slate::Matrix<double>::multiDevice(n, nrhs, nb, nb, nd);
    auto B2 = slate::Matrix<double>::multiDevice(n, nrhs, nb, nb, nd);
    slate::copy<double, double>(Ah, A);      // the one-time load (scatter)
    slate::copy<double, double>(Bh, B1);
    slate::copy<double, double>(Bh, B2);
    slate::scale(2.0, 1.0, B2);              // second right-hand side: 2 b

    const int64_t bytes0 = slate::inproc_copy_bytes(), runs0 = slate::inproc_run_count();
    slate::Pivots piv;
    int64_t info = slate::lu_factor(A, piv);
    slate::lu_solve_using_factor(A, piv, B1);
    slate::lu_solve_using_factor(A, piv, B2);
    const int64_t moved = slate::inproc_copy_bytes() - bytes0, runs = slate::inproc_run_count() - runs0;
    if (ex::rank() == 0)
        std::printf("  factor + 2 solves on %d devices: %lld driver runs, %lld bytes copied in / out\n",
                    int(A.storage()->parts.size()), (long long)runs, (long long)moved);
    fails += ex::check("no re-scatter between factor and solves", double(moved), 0);

    // residuals on the host: gather X, compare A X with b and 2 b
    std::vector<double> x1(size_t(n) * nrhs), x2(size_t(n) * nrhs);
    B1.gather(x1.data(), n);
    B2.gather(x2.data(), n);
    double r1 = 0, r2 = 0, bn = 0;
    for (int64_t j = 0; j < nrhs; ++j)
        for (int64_t i = 0; i < n; ++i) {
            double s1 = 0, s2 = 0;
            for (int64_t k = 0; k < n; ++k) {
                s1 += a[size_t(i) + size_t(k) * n] * x1[size_t(k) + size_t(j) * n];
                s2 += a[size_t(i) + size_t(k) * n] * x2[size_t(k) + size_t(j) * n];
            }
            r1 = std::max(r1, std::abs(s1 - b[size_t(i) + size_t(j) * n]));
            r2 = std::max(r2, std::abs(s2 - 2 * b[size_t(i) + size_t(j) * n]));
            bn = std::max(bn, std::abs(b[size_t(i) + size_t(j) * n]));
        }
    fails += ex::check("multi-device LU solve 1", info ? 1.0 : r1 / (bn * n), 1e-12);
    fails += ex::check("multi-device LU solve 2", info ? 1.0 : r2 / (2 * bn * n), 1e-12);

    // Cholesky and QR least squares on the same devices
    {
        auto H = slate::Matrix<double>::multiDevice(n, n, nb, nb, nd);
        slate::Matrix<double> At = Ah.emptyLike();   // a^T + a + 2 n I on the host
        At.insertLocalTiles(slate::Target::HostTask);
        std::vector<double> h(size_t(n) * n);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < n; ++i)
                h[size_t(i) + size_t(j) * n] = a[size_t(i) + size_t(j) * n] + a[size_t(j) + size_t(i) * n] +
                                               (i == j ? 2.0 * n : 0.0);
        auto Hh = slate::Matrix<double>::fromLAPACK(n, n, h.data(), n, nb);
        slate::copy<double, double>(Hh, H);
        slate::HermitianMatrix<double> HL(slate::Uplo::Lower, H);
        auto X = slate::Matrix<double>::multiDevice(n, nrhs, nb, nb, nd);
        slate::copy<double, double>(Bh, X);
        const int64_t c0 = slate::inproc_copy_bytes();
        info = slate::chol_solve(HL, X);
        fails += ex::check("multi-device Cholesky solve: no copies",
                           double(slate::inproc_copy_bytes() - c0), 0);
        std::vector<double> xs(size_t(n) * nrhs);
        X.gather(xs.data(), n);
        double r = 0;
        for (int64_t i = 0; i < n; ++i) {
            double s = 0;
            for (int64_t k = 0; k < n; ++k) s += h[size_t(i) + size_t(k) * n] * xs[size_t(k)];
            r = std::max(r, std::abs(s - b[size_t(i)]));
        }
        fails += ex::check("multi-device Cholesky residual", info ? 1.0 : r / (bn * n), 1e-12);
    }
    return ex::finish(fails);
}
