// Random butterfly transforms (reference src/gerbt.cc, gesv_rbt.cc,
// internal_gerbt.cc, internal_rbt_generate.cc; Parker 1995, Baboulin, Dongarra,
// Herrmann & Tomov 2013): A' = U^T A V with recursive butterflies U, V of
// depth d, so that LU WITHOUT pivoting of A' is stable with high probability;
// x = V y, then iterative refinement against the original A.
//
// A depth-d butterfly has 2^d nonzeros per row.  The transform is applied as
// two distributed GEMMs with the explicitly generated (sparse-valued, dense
// stored) butterflies so it runs on the MFMA kernels; the generator is the
// counter-based hash of the matgen library, so U and V depend only on
// (seed, n, depth) and never on the process grid.
#include "internal.hh"

#include <cmath>
#include <map>

namespace slate {

using namespace internal;

namespace {

inline double rbt_rand(uint64_t seed, uint64_t level, uint64_t idx) {
    // SplitMix64 on (seed, level, idx) -> r in [-0.5, 0.5]; entry exp(r / 10)
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + level * 0xBF58476D1CE4E5B9ull + idx * 0x94D049BB133111EBull;
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    double r = double(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    return std::exp(r / 10.0);
}

/// Sparse rows of W = L_d ... L_1, each L a block-diagonal of butterflies
/// B = 1/sqrt(2) [R0 R1; R0 -R1] on blocks of size n / 2^(level).
std::vector<std::map<int64_t, double>> butterfly_rows(int64_t n, int depth, uint64_t seed) {
    std::vector<std::map<int64_t, double>> W(n);
    for (int64_t i = 0; i < n; ++i) W[i][i] = 1.0;
    const double s2 = 1.0 / std::sqrt(2.0);
    for (int lev = 0; lev < depth; ++lev) {
        // L_lev: blocks of size bs = ceil(n / 2^lev); within a block of length L,
        // pair row r < h with r + h (h = L / 2); a middle leftover row stays
        int64_t nblk = int64_t(1) << lev;
        std::vector<std::map<int64_t, double>> Wn(n);
        for (int64_t b = 0; b < nblk; ++b) {
            int64_t r0 = n * b / nblk, r1 = n * (b + 1) / nblk, L = r1 - r0, h = L / 2;
            for (int64_t r = 0; r < L; ++r) {
                int64_t i = r0 + r;
                // row i of L_lev times W (W := L_lev W)
                auto axpy = [&](double a, int64_t src) { for (auto& kv : W[src]) Wn[i][kv.first] += a * kv.second; };
                if (r < h) {
                    double R0 = rbt_rand(seed, lev, 2 * i), R1 = rbt_rand(seed, lev, 2 * i + 1);
                    axpy(s2 * R0, i);
                    axpy(s2 * R1, i + h);
                } else if (r < 2 * h) {
                    int64_t ip = i - h;
                    double R0 = rbt_rand(seed, lev, 2 * ip), R1 = rbt_rand(seed, lev, 2 * ip + 1);
                    axpy(s2 * R0, ip);
                    axpy(-s2 * R1, i);
                } else {
                    axpy(1.0, i);
                }
            }
        }
        W.swap(Wn);
    }
    return W;
}

template <typename T>
Matrix<T> butterfly_matrix(int64_t n, int64_t nb, GridPtr grid, int depth, uint64_t seed, Target target) {
    auto rows = butterfly_rows(n, depth, seed);
    Matrix<T> W(n, n, nb, nb, grid);
    W.insertLocalTiles(Target::Host);
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) {
        auto it = rows[i].find(j);
        return it == rows[i].end() ? T(0) : T(it->second);
    }), W, oh);
    if (target == Target::Devices) W.insertLocalTiles(Target::Devices);
    return W;
}

}  // namespace

/// A := U^T A V (reference gerbt(U, A, V)); U and V from (seed, depth).
template <typename T>
void gerbt(Matrix<T>& A, int depth, uint64_t seed_u, uint64_t seed_v, Options const& opts) {
    trace::Block tb("gerbt");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const int64_t n = A.n();
    Matrix<T> U = butterfly_matrix<T>(A.m(), A.mb(), A.grid(), depth, seed_u, target);
    Matrix<T> V = butterfly_matrix<T>(n, A.nb(), A.grid(), depth, seed_v, target);
    Matrix<T> W = A.emptyLike();
    W.insertLocalTiles(target);
    gemm(T(1), transpose(U), A, T(0), W, opts);
    gemm(T(1), W, V, T(0), A, opts);
}

template <typename T>
int64_t gesv_rbt(Matrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts) {
    trace::Block tb("gesv_rbt");
    internal::DriverScope ds_;
    using R = real_type<T>;
    Target target = resolve_target(opts);
    const int depth = int(get_option<int64_t>(opts, Option::Depth, 2));
    const int itermax = int(get_option<int64_t>(opts, Option::MaxIterations, 10));
    const bool fallback = get_option<int64_t>(opts, Option::UseFallbackSolver, 1) != 0;
    const int64_t n = A.n();
    const uint64_t su = 0x5eed0001, sv = 0x5eed0002;
    R Anorm = norm(Norm::Inf, A, opts);
    const R cte = Anorm * std::numeric_limits<R>::epsilon() * std::sqrt(R(n));
    Matrix<T> U = butterfly_matrix<T>(n, A.mb(), A.grid(), depth, su, target);
    Matrix<T> V = butterfly_matrix<T>(n, A.nb(), A.grid(), depth, sv, target);
    // A' = U^T A V (A is kept for the residuals)
    Matrix<T> Ap = A.emptyLike();
    Ap.insertLocalTiles(target);
    {
        Matrix<T> W = A.emptyLike();
        W.insertLocalTiles(target);
        gemm(T(1), transpose(U), A, T(0), W, opts);
        gemm(T(1), W, V, T(0), Ap, opts);
    }
    int64_t info = getrf_nopiv(Ap, opts);
    iter = 0;
    auto solve = [&](Matrix<T> const& Rhs, Matrix<T>& Out) {
        // Out = V (A')^{-1} U^T Rhs
        Matrix<T> Y = Rhs.emptyLike();
        Y.insertLocalTiles(target);
        gemm(T(1), transpose(U), Rhs, T(0), Y, opts);
        getrs_nopiv(Ap, Y, opts);
        gemm(T(1), V, Y, T(0), Out, opts);
    };
    if (info == 0) {
        solve(B, X);
        Matrix<T> Rm = B.emptyLike();
        Rm.insertLocalTiles(target);
        Matrix<T> D = X.emptyLike();
        D.insertLocalTiles(target);
        const int64_t nrhs = B.n();
        std::vector<R> rnorm(nrhs), xnorm(nrhs);
        for (int it = 0; it <= itermax; ++it) {
            slate::copy<T, T>(B, Rm, opts);
            gemm(T(-1), A, X, T(1), Rm, opts);
            colNorms(Norm::Max, X, xnorm.data(), opts);
            colNorms(Norm::Max, Rm, rnorm.data(), opts);
            bool ok = true;
            for (int64_t j = 0; j < nrhs; ++j) ok = ok && rnorm[j] <= xnorm[j] * cte;
            if (ok) { iter = it; return 0; }
            if (it == itermax) break;
            solve(Rm, D);
            add(T(1), D, T(1), X, opts);
        }
        iter = -itermax - 1;
    } else {
        iter = -3;
    }
    if (!fallback) return info;
    slate::copy<T, T>(B, X, opts);
    Pivots piv;
    return gesv(A, piv, X, opts);
}

#define SLATE_RBT_INST(T)                                                                         \
    template void gerbt<T>(Matrix<T>&, int, uint64_t, uint64_t, Options const&);                 \
    template int64_t gesv_rbt<T>(Matrix<T>&, Matrix<T>&, Matrix<T>&, int&, Options const&);

SLATE_RBT_INST(float)
SLATE_RBT_INST(double)
SLATE_RBT_INST(std::complex<float>)
SLATE_RBT_INST(std::complex<double>)

}  // namespace slate
