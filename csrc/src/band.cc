// Band drivers (reference src/gbtrf.cc, gbtrs.cc, gbsv.cc, pbtrf.cc, pbtrs.cc,
// pbsv.cc, gbmm.cc, hbmm.cc, tbsm.cc, internal_gbnorm.cc / hbnorm.cc).
//
// The band factorizations are O(n kl (kl+ku)) and latency-bound per column,
// so (like the reference's host panels) they run on the host: the band
// entries (O(n * bandwidth), not O(n^2)) are reduced into replicated LAPACK
// band storage on every rank, factored with the unblocked band kernels below,
// and each rank writes its own entries back.  The band multiplies / solves
// (gbmm, hbmm, tbsm) run distributed on a band-masked dense operand so the
// flops land on the device GEMM/TRSM.
#include "internal.hh"

#include <cmath>

namespace slate {

using namespace internal;

namespace {

/// Visit every local element of A (NoTrans view) with its global (i, j)
/// relative to the view; f(i, j, T& value).  Host instance, optionally for write.
template <typename T, typename F>
void for_each_local(BaseMatrix<T> const& A, bool write, F&& f) {
    slate_error_if_msg(A.op() != Op::NoTrans, "band: NoTrans view required");
    auto& s = *A.storage();
    s.get(Loc::Host, write);
    const int64_t ld = s.ld(Loc::Host);
    LocalBlock<T> la = A.local_raw(Loc::Host);
    std::vector<int64_t> gr(la.m);
    for (int64_t il = 0; il < la.m; ++il)
        gr[il] = l2g(A.lrow_begin() + il, s.mb, s.rrel(), s.grid->p()) - A.row0();
    for (int64_t jl = 0; jl < la.n; ++jl) {
        int64_t gc = l2g(A.lcol_begin() + jl, s.nb, s.crel(), s.grid->q()) - A.col0();
        for (int64_t il = 0; il < la.m; ++il) f(gr[il], gc, la.ptr[il + jl * ld]);
    }
}

/// Replicated LAPACK band storage: AB(r0 + i - j, j) = A(i, j) for
/// -ku <= i - j <= kl; ldab >= r0 + kl + 1.  conj_upper: read A's upper
/// band (i < j) as the conj-transposed lower band (Hermitian band, Upper).
template <typename T>
std::vector<T> gather_band(BaseMatrix<T> const& A, int64_t kl, int64_t ku, int64_t r0, int64_t ldab,
                           bool upper_as_lower = false) {
    const int64_t n = A.n();
    std::vector<T> ab(size_t(ldab) * n, T(0));
    for_each_local(A, false, [&](int64_t i, int64_t j, T& v) {
        if (upper_as_lower) {
            if (j >= i && j - i <= ku) ab[(r0 + j - i) + i * ldab] = slate::conj(v);   // (j, i) of the lower band
        } else if (i - j <= kl && j - i <= ku) {
            ab[(r0 + i - j) + j * ldab] = v;
        }
    });
    // every band entry is owned by exactly one rank
    Comm& w = A.grid()->world();
    if (w.size() > 1) {
        using R = real_type<T>;
        size_t mult = is_complex_v<T> ? 2 : 1;
        allreduce_host<R>(w, reinterpret_cast<R*>(ab.data()), ab.size() * mult, ReduceOp::Sum);
    }
    return ab;
}

template <typename T>
void scatter_band(BaseMatrix<T>& A, std::vector<T> const& ab, int64_t kl, int64_t ku, int64_t r0, int64_t ldab,
                  bool upper_as_lower = false) {
    for_each_local(A, true, [&](int64_t i, int64_t j, T& v) {
        if (upper_as_lower) {
            if (j >= i && j - i <= ku) v = slate::conj(ab[(r0 + j - i) + i * ldab]);
        } else if (i - j <= kl && j - i <= ku) {
            v = ab[(r0 + i - j) + j * ldab];
        }
    });
}

/// Dense (replicated, column-major) copy of a distributed matrix.
template <typename T>
std::vector<T> gather_dense(BaseMatrix<T> const& B, Options const& opts) {
    std::vector<T> b;
    gather(B, b, opts);
    return b;
}

template <typename T>
void scatter_dense(Matrix<T>& B, std::vector<T> const& b, int64_t ldb) {
    for_each_local(B, true, [&](int64_t i, int64_t j, T& v) { v = b[i + j * ldb]; });
}

//------------------------------------------------------------------------------
// host band kernels (LAPACK gbtf2 / gbtrs / pbtf2 / pbtrs semantics)
template <typename T>
int64_t gbtf2(int64_t n, int64_t kl, int64_t ku, T* ab, int64_t ldab, int64_t* ipiv) {
    const int64_t kv = ku + kl;
    auto A = [&](int64_t i, int64_t j) -> T& { return ab[(kv + i - j) + j * ldab]; };
    int64_t info = 0, ju = 0;
    for (int64_t j = 0; j < n; ++j) {
        const int64_t km = std::min(kl, n - 1 - j);
        int64_t jp = 0;
        real_type<T> mx = -1;
        for (int64_t i = 0; i <= km; ++i) {
            real_type<T> a = std::abs(std::real(A(j + i, j))) + std::abs(std::imag(A(j + i, j)));
            if (a > mx) { mx = a; jp = i; }
        }
        ipiv[j] = j + jp;
        if (A(j + jp, j) != T(0)) {
            ju = std::max(ju, std::min(j + ku + jp, n - 1));
            if (jp != 0)
                for (int64_t c = j; c <= ju; ++c) std::swap(A(j + jp, c), A(j, c));
            if (km > 0) {
                T r = T(1) / A(j, j);
                for (int64_t i = 1; i <= km; ++i) A(j + i, j) *= r;
                for (int64_t c = j + 1; c <= ju; ++c) {
                    T t = A(j, c);
                    if (t == T(0)) continue;
                    for (int64_t i = 1; i <= km; ++i) A(j + i, c) -= A(j + i, j) * t;
                }
            }
        } else if (info == 0) {
            info = j + 1;
        }
    }
    return info;
}

template <typename T>
void gbtrs_host(int64_t n, int64_t kl, int64_t ku, int64_t nrhs, T const* ab, int64_t ldab, int64_t const* ipiv,
                T* b, int64_t ldb) {
    const int64_t kv = ku + kl;
    auto A = [&](int64_t i, int64_t j) { return ab[(kv + i - j) + j * ldab]; };
    #pragma omp parallel for schedule(static) if (nrhs > 1)
    for (int64_t c = 0; c < nrhs; ++c) {
        T* x = b + c * ldb;
        for (int64_t j = 0; j < n; ++j) {
            if (ipiv[j] != j) std::swap(x[j], x[ipiv[j]]);
            int64_t km = std::min(kl, n - 1 - j);
            for (int64_t i = 1; i <= km; ++i) x[j + i] -= A(j + i, j) * x[j];
        }
        for (int64_t j = n - 1; j >= 0; --j) {
            x[j] /= A(j, j);
            int64_t lo = std::max<int64_t>(0, j - kv);
            for (int64_t i = lo; i < j; ++i) x[i] -= A(i, j) * x[j];
        }
    }
}

/// Lower band Cholesky: ab(i - j, j) = A(i, j), ldab >= kd + 1.
template <typename T>
int64_t pbtf2(int64_t n, int64_t kd, T* ab, int64_t ldab) {
    auto L = [&](int64_t i, int64_t j) -> T& { return ab[(i - j) + j * ldab]; };
    for (int64_t j = 0; j < n; ++j) {
        real_type<T> ajj = std::real(L(j, j));
        if (!(ajj > 0)) return j + 1;
        ajj = std::sqrt(ajj);
        L(j, j) = T(ajj);
        int64_t kn = std::min(kd, n - 1 - j);
        for (int64_t i = 1; i <= kn; ++i) L(j + i, j) /= T(ajj);
        for (int64_t c = 1; c <= kn; ++c) {
            T lc = slate::conj(L(j + c, j));
            for (int64_t r = c; r <= kn; ++r) L(j + r, j + c) -= L(j + r, j) * lc;
        }
    }
    return 0;
}

template <typename T>
void pbtrs_host(int64_t n, int64_t kd, int64_t nrhs, T const* ab, int64_t ldab, T* b, int64_t ldb) {
    auto L = [&](int64_t i, int64_t j) { return ab[(i - j) + j * ldab]; };
    #pragma omp parallel for schedule(static) if (nrhs > 1)
    for (int64_t c = 0; c < nrhs; ++c) {
        T* x = b + c * ldb;
        for (int64_t j = 0; j < n; ++j) {
            x[j] /= L(j, j);
            int64_t kn = std::min(kd, n - 1 - j);
            for (int64_t i = 1; i <= kn; ++i) x[j + i] -= L(j + i, j) * x[j];
        }
        for (int64_t j = n - 1; j >= 0; --j) {
            int64_t kn = std::min(kd, n - 1 - j);
            T s = x[j];
            for (int64_t i = 1; i <= kn; ++i) s -= slate::conj(L(j + i, j)) * x[j + i];
            x[j] = s / slate::conj(L(j, j));
        }
    }
}

/// Pivots (reference layout: per tile column, (tile offset from k, row offset))
template <typename T>
void pivots_from_ipiv(BaseMatrix<T> const& A, std::vector<int64_t> const& ipiv, Pivots& pivots) {
    const int64_t kt = std::min(A.mt(), A.nt());
    pivots.assign(kt, {});
    for (int64_t k = 0; k < kt; ++k) {
        int64_t kk = grow_of(A, k), kd = std::min(A.tileNb(k), int64_t(ipiv.size()) - kk);
        for (int64_t t = 0; t < kd; ++t) {
            int64_t r = ipiv[kk + t];
            int64_t ti = 0;
            while (ti + k + 1 < A.mt() && grow_of(A, k + ti + 1) <= r) ++ti;
            pivots[k].push_back(Pivot(ti, r - grow_of(A, k + ti)));
        }
    }
}

template <typename T>
std::vector<int64_t> ipiv_from_pivots(BaseMatrix<T> const& A, Pivots const& pivots) {
    std::vector<int64_t> ipiv;
    for (int64_t k = 0; k < int64_t(pivots.size()); ++k)
        for (auto const& p : pivots[k]) ipiv.push_back(grow_of(A, k + p.tileIndex()) + p.elementOffset());
    return ipiv;
}

/// General copy of a band matrix with out-of-band entries zeroed.
template <typename T>
Matrix<T> band_dense(BaseMatrix<T> const& A, int64_t kl, int64_t ku, Options const& opts, bool herm = false,
                     Uplo uplo = Uplo::General) {
    Target target = resolve_target(opts);
    Matrix<T> G(A);
    G.set_uplo(Uplo::General);
    Matrix<T> D = G.emptyLike();
    D.insertLocalTiles(Target::Host);
    Options oh = {{Option::Target, Target::Host}};
    slate::copy<T, T>(G, D, oh);
    if (herm) {
        // Hermitian band stored in one triangle: mirror it
        Matrix<T> Dh = D.emptyLike();
        Dh.insertLocalTiles(Target::Host);
        slate::copy<T, T>(conj_transpose(D), Dh, oh);
        D.storage()->get(Loc::Host, true);
        // combine: D(i,j) = stored-triangle value, other triangle from Dh
        LocalBlock<T> ld = D.local_raw(Loc::Host), lh = Dh.local_raw(Loc::Host);
        auto& s = *D.storage();
        for (int64_t jl = 0; jl < ld.n; ++jl) {
            int64_t gc = l2g(D.lcol_begin() + jl, s.nb, s.crel(), s.grid->q()) - D.col0();
            for (int64_t il = 0; il < ld.m; ++il) {
                int64_t gr = l2g(D.lrow_begin() + il, s.mb, s.rrel(), s.grid->p()) - D.row0();
                bool stored = (uplo == Uplo::Lower) ? gr >= gc : gr <= gc;
                T v = stored ? ld.ptr[il + jl * ld.ld] : lh.ptr[il + jl * lh.ld];
                if (gr == gc) v = T(std::real(v));
                ld.ptr[il + jl * ld.ld] = v;
            }
        }
    }
    for_each_local(D, true, [&](int64_t i, int64_t j, T& v) {
        if (i - j > kl || j - i > ku) v = T(0);
    });
    if (target == Target::Devices) D.insertLocalTiles(Target::Devices);
    return D;
}

}  // namespace

//------------------------------------------------------------------------------
template <typename T>
int64_t gbtrf(BandMatrix<T>& A, Pivots& pivots, Options const& opts) {
    trace::Block tb("gbtrf");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kl = A.lowerBandwidth(), ku = A.upperBandwidth();
    slate_error_if_msg(A.m() != n, "gbtrf: square band matrix required");
    const int64_t ldab = 2 * kl + ku + 1, kv = kl + ku;
    // AB(kv + i - j, j) = A(i, j); rows [0, kl) receive the fill
    std::vector<T> ab = gather_band<T>(A, kl, ku, kv, ldab);
    std::vector<int64_t> ipiv(n);
    int64_t info = gbtf2<T>(n, kl, ku, ab.data(), ldab, ipiv.data());
    // factors: L (kl below) and U (kl + ku above); the matrix's storage holds the fill
    scatter_band<T>(A, ab, kl, kv, kv, ldab);
    A.set_band(kl, kl + ku);
    pivots_from_ipiv(A, ipiv, pivots);
    Target target = resolve_target(opts);
    if (target == Target::Devices) A.storage()->get(Loc::Device, false);
    return info;
}

template <typename T>
void gbtrs(BandMatrix<T> const& A, Pivots const& pivots, Matrix<T>& B, Options const& opts) {
    trace::Block tb("gbtrs");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kl = A.lowerBandwidth(), ku_f = A.upperBandwidth();
    // after gbtrf the stored upper bandwidth is kl + ku (fill)
    const int64_t ku = std::max<int64_t>(ku_f - kl, 0);
    const int64_t ldab = 2 * kl + ku + 1;
    std::vector<T> ab = gather_band<T>(A, kl, kl + ku, kl + ku, ldab);
    std::vector<int64_t> ipiv = ipiv_from_pivots(A, pivots);
    std::vector<T> b = gather_dense(B, opts);
    gbtrs_host<T>(n, kl, ku, B.n(), ab.data(), ldab, ipiv.data(), b.data(), n);
    scatter_dense(B, b, n);
    if (resolve_target(opts) == Target::Devices) B.storage()->get(Loc::Device, false);
}

template <typename T>
int64_t gbsv(BandMatrix<T>& A, Pivots& pivots, Matrix<T>& B, Options const& opts) {
    trace::Block tb("gbsv");
    internal::DriverScope ds_;
    int64_t info = gbtrf(A, pivots, opts);
    if (info == 0) gbtrs(A, pivots, B, opts);
    return info;
}

template <typename T>
int64_t pbtrf(HermitianBandMatrix<T>& A, Options const& opts) {
    trace::Block tb("pbtrf");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kd = A.bandwidth();
    const bool upper = A.uplo() == Uplo::Upper;
    // lower band storage ab(i - j, j) = L(i, j); an Upper matrix is read as U^H
    std::vector<T> ab = upper ? gather_band<T>(A, 0, kd, 0, kd + 1, true) : gather_band<T>(A, kd, 0, 0, kd + 1);
    int64_t info = pbtf2<T>(n, kd, ab.data(), kd + 1);
    if (upper) scatter_band<T>(A, ab, 0, kd, 0, kd + 1, true);
    else scatter_band<T>(A, ab, kd, 0, 0, kd + 1);
    if (resolve_target(opts) == Target::Devices) A.storage()->get(Loc::Device, false);
    return info;
}

template <typename T>
void pbtrs(HermitianBandMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("pbtrs");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kd = A.bandwidth();
    const bool upper = A.uplo() == Uplo::Upper;
    std::vector<T> ab = upper ? gather_band<T>(A, 0, kd, 0, kd + 1, true) : gather_band<T>(A, kd, 0, 0, kd + 1);
    std::vector<T> b = gather_dense(B, opts);
    pbtrs_host<T>(n, kd, B.n(), ab.data(), kd + 1, b.data(), n);
    scatter_dense(B, b, n);
    if (resolve_target(opts) == Target::Devices) B.storage()->get(Loc::Device, false);
}

template <typename T>
int64_t pbsv(HermitianBandMatrix<T>& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("pbsv");
    internal::DriverScope ds_;
    int64_t info = pbtrf(A, opts);
    if (info == 0) pbtrs(A, B, opts);
    return info;
}

//------------------------------------------------------------------------------
template <typename T>
void gbmm(T alpha, BandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts) {
    trace::Block tb("gbmm");
    internal::DriverScope ds_;
    Matrix<T> D = band_dense<T>(A, A.lowerBandwidth(), A.upperBandwidth(), opts);
    gemm(alpha, D, B, beta, C, opts);
}

template <typename T>
void hbmm(Side side, T alpha, HermitianBandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts) {
    trace::Block tb("hbmm");
    internal::DriverScope ds_;
    const int64_t kd = A.bandwidth();
    Matrix<T> D = band_dense<T>(A, kd, kd, opts, true, A.uplo());
    if (side == Side::Left) gemm(alpha, D, B, beta, C, opts);
    else gemm(alpha, B, D, beta, C, opts);
}

template <typename T>
void tbsm(Side side, T alpha, TriangularBandMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("tbsm");
    internal::DriverScope ds_;
    Matrix<T> D = band_dense<T>(A, A.kl(), A.ku(), opts);
    TriangularMatrix<T> Tm(A.uplo(), A.diag(), D);
    trsm(side, alpha, Tm, B, opts);
}

#define SLATE_BAND_INST(T)                                                                                 \
    template int64_t gbtrf<T>(BandMatrix<T>&, Pivots&, Options const&);                                   \
    template void gbtrs<T>(BandMatrix<T> const&, Pivots const&, Matrix<T>&, Options const&);              \
    template int64_t gbsv<T>(BandMatrix<T>&, Pivots&, Matrix<T>&, Options const&);                        \
    template int64_t pbtrf<T>(HermitianBandMatrix<T>&, Options const&);                                   \
    template void pbtrs<T>(HermitianBandMatrix<T> const&, Matrix<T>&, Options const&);                    \
    template int64_t pbsv<T>(HermitianBandMatrix<T>&, Matrix<T>&, Options const&);                        \
    template void gbmm<T>(T, BandMatrix<T> const&, Matrix<T> const&, T, Matrix<T>&, Options const&);      \
    template void hbmm<T>(Side, T, HermitianBandMatrix<T> const&, Matrix<T> const&, T, Matrix<T>&,        \
                          Options const&);                                                                 \
    template void tbsm<T>(Side, T, TriangularBandMatrix<T> const&, Matrix<T>&, Options const&);

SLATE_BAND_INST(float)
SLATE_BAND_INST(double)
SLATE_BAND_INST(std::complex<float>)
SLATE_BAND_INST(std::complex<double>)

}  // namespace slate
