// Hermitian indefinite factorization and solve (reference src/hetrf.cc,
// hetrs.cc, hesv.cc).  The reference factors with Aasen's algorithm on the
// host ("GPU version not yet implemented", hetrf.cc) and then band-LU's the
// block-tridiagonal T; here the factorization is Bunch-Kaufman diagonal
// pivoting, A = P L D L^H P^T with 1x1 and 2x2 pivots (LAPACK hetf2
// semantics), computed on the host copy of the matrix (every rank, replicated
// and deterministic) and written back into A's triangle.  ipiv follows the
// LAPACK convention (1-based; negative pairs mark 2x2 blocks).
#include "internal.hh"

#include <cmath>

namespace slate {

using namespace internal;

namespace {

template <typename T> inline real_type<T> cabs1(T x) { return std::abs(std::real(x)) + std::abs(std::imag(x)); }

/// Lower Bunch-Kaufman on a dense column-major n x n array.
template <typename T>
int64_t hetf2_lower(int64_t n, T* a, int64_t lda, int64_t* ipiv) {
    using R = real_type<T>;
    auto A = [&](int64_t i, int64_t j) -> T& { return a[i + j * lda]; };
    const R alpha = (R(1) + std::sqrt(R(17))) / R(8);
    int64_t info = 0, k = 0;
    while (k < n) {
        int64_t kstep = 1, kp = k;
        R absakk = std::abs(std::real(A(k, k)));
        int64_t imax = k;
        R colmax = 0;
        for (int64_t i = k + 1; i < n; ++i) if (cabs1(A(i, k)) > colmax) { colmax = cabs1(A(i, k)); imax = i; }
        if (std::max(absakk, colmax) == R(0)) {
            if (info == 0) info = k + 1;
            kp = k;
            A(k, k) = T(std::real(A(k, k)));
        } else {
            if (absakk >= alpha * colmax) {
                kp = k;
            } else {
                R rowmax = 0;
                for (int64_t j = k; j < imax; ++j) rowmax = std::max(rowmax, cabs1(A(imax, j)));
                for (int64_t i = imax + 1; i < n; ++i) rowmax = std::max(rowmax, cabs1(A(i, imax)));
                if (absakk >= alpha * colmax * (colmax / rowmax)) kp = k;
                else if (std::abs(std::real(A(imax, imax))) >= alpha * rowmax) kp = imax;
                else { kp = imax; kstep = 2; }
            }
            const int64_t kk = k + kstep - 1;
            if (kp != kk) {
                for (int64_t i = kp + 1; i < n; ++i) std::swap(A(i, kk), A(i, kp));
                for (int64_t j = kk + 1; j < kp; ++j) {
                    T t = slate::conj(A(j, kk));
                    A(j, kk) = slate::conj(A(kp, j));
                    A(kp, j) = t;
                }
                A(kp, kk) = slate::conj(A(kp, kk));
                R r1 = std::real(A(kk, kk));
                A(kk, kk) = T(std::real(A(kp, kp)));
                A(kp, kp) = T(r1);
                if (kstep == 2) {
                    A(k, k) = T(std::real(A(k, k)));
                    std::swap(A(k + 1, k), A(kp, k));
                }
            } else {
                A(k, k) = T(std::real(A(k, k)));
                if (kstep == 2) A(k + 1, k + 1) = T(std::real(A(k + 1, k + 1)));
            }
            if (kstep == 1) {
                R r1 = R(1) / std::real(A(k, k));
                #pragma omp parallel for schedule(static) if (n - k > 256)
                for (int64_t j = k + 1; j < n; ++j) {
                    T xj = slate::conj(A(j, k)) * r1;
                    for (int64_t i = j; i < n; ++i) A(i, j) -= A(i, k) * xj;
                    A(j, j) = T(std::real(A(j, j)));
                }
                for (int64_t i = k + 1; i < n; ++i) A(i, k) *= r1;
            } else if (k + 2 < n) {
                R d = std::abs(A(k + 1, k));
                R d11 = std::real(A(k + 1, k + 1)) / d;
                R d22 = std::real(A(k, k)) / d;
                R tt = R(1) / (d11 * d22 - R(1));
                T d21 = A(k + 1, k) / d;
                R dd = tt / d;
                std::vector<T> wk(n), wkp1(n);
                for (int64_t j = k + 2; j < n; ++j) {
                    wk[j] = dd * (d11 * A(j, k) - d21 * A(j, k + 1));
                    wkp1[j] = dd * (d22 * A(j, k + 1) - slate::conj(d21) * A(j, k));
                }
                #pragma omp parallel for schedule(static) if (n - k > 256)
                for (int64_t j = k + 2; j < n; ++j) {
                    T cw = slate::conj(wk[j]), cw1 = slate::conj(wkp1[j]);
                    for (int64_t i = j; i < n; ++i) A(i, j) -= A(i, k) * cw + A(i, k + 1) * cw1;
                    A(j, j) = T(std::real(A(j, j)));
                }
                for (int64_t j = k + 2; j < n; ++j) { A(j, k) = wk[j]; A(j, k + 1) = wkp1[j]; }
            }
        }
        if (kstep == 1) ipiv[k] = kp + 1;
        else ipiv[k] = ipiv[k + 1] = -(kp + 1);
        k += kstep;
    }
    return info;
}

template <typename T>
void hetrs_lower(int64_t n, int64_t nrhs, T const* a, int64_t lda, int64_t const* ipiv, T* b, int64_t ldb) {
    auto A = [&](int64_t i, int64_t j) { return a[i + j * lda]; };
    #pragma omp parallel for schedule(static) if (nrhs > 1)
    for (int64_t c = 0; c < nrhs; ++c) {
        T* x = b + c * ldb;
        int64_t k = 0;
        while (k < n) {
            if (ipiv[k] > 0) {
                int64_t kp = ipiv[k] - 1;
                if (kp != k) std::swap(x[k], x[kp]);
                for (int64_t i = k + 1; i < n; ++i) x[i] -= A(i, k) * x[k];
                x[k] /= std::real(A(k, k));
                k += 1;
            } else {
                int64_t kp = -ipiv[k] - 1;
                if (kp != k + 1) std::swap(x[k + 1], x[kp]);
                for (int64_t i = k + 2; i < n; ++i) x[i] -= A(i, k) * x[k] + A(i, k + 1) * x[k + 1];
                T akm1k = A(k + 1, k);
                T akm1 = A(k, k) / slate::conj(akm1k);
                T ak = A(k + 1, k + 1) / akm1k;
                T denom = akm1 * ak - T(1);
                T bkm1 = x[k] / slate::conj(akm1k);
                T bk = x[k + 1] / akm1k;
                x[k] = (ak * bkm1 - bk) / denom;
                x[k + 1] = (akm1 * bk - bkm1) / denom;
                k += 2;
            }
        }
        k = n - 1;
        while (k >= 0) {
            if (ipiv[k] > 0) {
                T s = x[k];
                for (int64_t i = k + 1; i < n; ++i) s -= slate::conj(A(i, k)) * x[i];
                x[k] = s;
                int64_t kp = ipiv[k] - 1;
                if (kp != k) std::swap(x[k], x[kp]);
                k -= 1;
            } else {
                T s = x[k], s1 = x[k - 1];
                for (int64_t i = k + 1; i < n; ++i) {
                    s -= slate::conj(A(i, k)) * x[i];
                    s1 -= slate::conj(A(i, k - 1)) * x[i];
                }
                x[k] = s;
                x[k - 1] = s1;
                int64_t kp = -ipiv[k] - 1;
                if (kp != k) std::swap(x[k], x[kp]);
                k -= 2;
            }
        }
    }
}

/// Replicated lower-triangle copy of a Hermitian matrix (Upper read as L^H).
template <typename T>
std::vector<T> gather_lower(HermitianMatrix<T> const& A, Options const& opts) {
    Matrix<T> G(A);
    G.set_uplo(Uplo::General);
    std::vector<T> full;
    gather(G, full, opts);
    const int64_t n = A.n();
    if (A.uplo() == Uplo::Upper)
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = j; i < n; ++i) full[i + j * n] = slate::conj(full[j + i * n]);
    return full;
}

}  // namespace

template <typename T>
int64_t hetrf(HermitianMatrix<T>& A, std::vector<int64_t>& ipiv, Options const& opts) {
    trace::Block tb("hetrf");
    internal::DriverScope ds_;
    const int64_t n = A.n();
    std::vector<T> a = gather_lower(A, opts);
    ipiv.assign(n, 0);
    int64_t info = hetf2_lower<T>(n, a.data(), n, ipiv.data());
    // write back the factor into A's stored triangle
    Matrix<T> G(A);
    G.set_uplo(Uplo::General);
    const bool upper = A.uplo() == Uplo::Upper;
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) {
        if (!upper) return i >= j ? a[i + j * n] : T(0);
        return i <= j ? slate::conj(a[j + i * n]) : T(0);
    }), G, oh);
    if (resolve_target(opts) == Target::Devices) G.storage()->get(Loc::Device, false);
    return info;
}

template <typename T>
void hetrs(HermitianMatrix<T> const& A, std::vector<int64_t> const& ipiv, Matrix<T>& B, Options const& opts) {
    trace::Block tb("hetrs");
    internal::DriverScope ds_;
    const int64_t n = A.n(), nrhs = B.n();
    std::vector<T> a = gather_lower(A, opts);
    std::vector<T> b;
    gather(B, b, opts);
    hetrs_lower<T>(n, nrhs, a.data(), n, ipiv.data(), b.data(), n);
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) { return b[i + j * n]; }), B, oh);
    if (resolve_target(opts) == Target::Devices) B.storage()->get(Loc::Device, false);
}

template <typename T>
int64_t hesv(HermitianMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Options const& opts) {
    trace::Block tb("hesv");
    internal::DriverScope ds_;
    int64_t info = hetrf(A, ipiv, opts);
    if (info == 0) hetrs(A, ipiv, B, opts);
    return info;
}

#define SLATE_HE_INST(T)                                                                              \
    template int64_t hetrf<T>(HermitianMatrix<T>&, std::vector<int64_t>&, Options const&);           \
    template void hetrs<T>(HermitianMatrix<T> const&, std::vector<int64_t> const&, Matrix<T>&,       \
                           Options const&);                                                           \
    template int64_t hesv<T>(HermitianMatrix<T>&, std::vector<int64_t>&, Matrix<T>&, Options const&);

SLATE_HE_INST(float)
SLATE_HE_INST(double)
SLATE_HE_INST(std::complex<float>)
SLATE_HE_INST(std::complex<double>)

}  // namespace slate
