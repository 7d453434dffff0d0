// Host tile kernels: C++/OpenMP BLAS-3 and LAPACK-style routines.
//
// The reference calls vendor host BLAS/LAPACK through BLAS++/LAPACK++
// (Tile_blas.hh:30-944, Tile_lapack.hh:23-331).  No host BLAS exists on this
// platform, so these are our own column-major implementations; they back
// Target::Host* and serve as numerical oracles in tests.  Indices are 0-based;
// ipiv entries are 0-based absolute row indices.
#pragma once

#include "types.hh"
#include "util.hh"

#include <algorithm>
#include <cmath>
#include <limits>
#include <complex>
#include <cstring>
#include <vector>
#include <type_traits>

namespace slate {
namespace host {

template <typename T>
inline T opval(Op op, T const* A, int64_t lda, int64_t i, int64_t j) {
    // element (i, j) of op(A)
    if (op == Op::NoTrans) return A[i + j * lda];
    T v = A[j + i * lda];
    return op == Op::ConjTrans ? slate::conj(v) : v;
}

/// Copy op(A) (m x n) into dense B (ld m).
template <typename T>
void pack(Op op, int64_t m, int64_t n, T const* A, int64_t lda, T* B) {
    #pragma omp parallel for schedule(static) if (m * n > 65536)
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i)
            B[i + j * m] = opval(op, A, lda, i, j);
}

//------------------------------------------------------------------------------
/// Packed, register-blocked GEMM for real types (the host target's compute
/// path: BASELINE config 1 and every host-task driver).  Goto-style: B is
/// packed into NR-column panels per (jc, pc) block, A into MR-row panels per
/// thread, and an MR x NR micro-tile of C lives in 12 AVX2 registers (GCC
/// vector extensions; -march=x86-64-v3 turns them into FMA ymm code).
namespace gemm_detail {

template <typename T> struct VecT;
template <> struct VecT<double> { typedef double v __attribute__((vector_size(32))); static constexpr int W = 4; };
template <> struct VecT<float> { typedef float v __attribute__((vector_size(32))); static constexpr int W = 8; };

template <typename T>
struct Blk {
    static constexpr int W = VecT<T>::W, MR = 2 * W, NR = 6;
    static constexpr int64_t KC = 256, MC = 16 * MR, NC = 6 * 512;
};

/// Ap[p][l][r] = op(A)(i0 + p MR + r, l0 + l), zero-padded rows
template <typename T>
inline void pack_a(Op op, T const* A, int64_t lda, int64_t i0, int64_t mc, int64_t l0, int64_t kc, T* Ap) {
    constexpr int MR = Blk<T>::MR;
    for (int64_t p = 0; p * MR < mc; ++p) {
        T* dst = Ap + p * MR * kc;
        const int64_t rv = std::min<int64_t>(MR, mc - p * MR);
        for (int64_t l = 0; l < kc; ++l) {
            for (int r = 0; r < rv; ++r) dst[l * MR + r] = opval(op, A, lda, i0 + p * MR + r, l0 + l);
            for (int r = int(rv); r < MR; ++r) dst[l * MR + r] = T(0);
        }
    }
}

/// Bp[q][l][c] = op(B)(l0 + l, j0 + q NR + c), zero-padded columns
template <typename T>
inline void pack_b(Op op, T const* B, int64_t ldb, int64_t l0, int64_t kc, int64_t j0, int64_t nc, T* Bp) {
    constexpr int NR = Blk<T>::NR;
    const int64_t nq = (nc + NR - 1) / NR;
    #pragma omp parallel for schedule(static) if (kc * nc > 32768)
    for (int64_t q = 0; q < nq; ++q) {
        T* dst = Bp + q * NR * kc;
        const int64_t cv = std::min<int64_t>(NR, nc - q * NR);
        for (int64_t l = 0; l < kc; ++l) {
            for (int c = 0; c < cv; ++c) dst[l * NR + c] = opval(op, B, ldb, l0 + l, j0 + q * NR + c);
            for (int c = int(cv); c < NR; ++c) dst[l * NR + c] = T(0);
        }
    }
}

/// C(mr x nr) += alpha Ap_panel Bp_panel over kc
template <typename T>
inline void micro(int64_t kc, T const* __restrict__ Ap, T const* __restrict__ Bp, T alpha, T* C, int64_t ldc,
                  int mr, int nr) {
    typedef typename VecT<T>::v V;
    constexpr int W = VecT<T>::W, MR = Blk<T>::MR, NR = Blk<T>::NR;
    V acc[2][NR];
    for (int c = 0; c < NR; ++c) { acc[0][c] = V{} ; acc[1][c] = V{}; }
    for (int64_t l = 0; l < kc; ++l) {
        V a0, a1;
        __builtin_memcpy(&a0, Ap + l * MR, sizeof(V));
        __builtin_memcpy(&a1, Ap + l * MR + W, sizeof(V));
        #pragma GCC unroll 6
        for (int c = 0; c < NR; ++c) {
            const T bv = Bp[l * NR + c];
            V b;
            for (int t = 0; t < W; ++t) b[t] = bv;
            acc[0][c] += a0 * b;
            acc[1][c] += a1 * b;
        }
    }
    if (mr == MR && nr == NR) {
        for (int c = 0; c < NR; ++c) {
            T* cc = C + c * ldc;
            for (int t = 0; t < W; ++t) { cc[t] += alpha * acc[0][c][t]; cc[W + t] += alpha * acc[1][c][t]; }
        }
        return;
    }
    for (int c = 0; c < nr; ++c) {
        T* cc = C + c * ldc;
        for (int r = 0; r < mr; ++r) cc[r] += alpha * (r < W ? acc[0][c][r] : acc[1][c][r - W]);
    }
}

template <typename T>
void gemm_packed(Op opA, Op opB, int64_t m, int64_t n, int64_t k, T alpha, T const* A, int64_t lda, T const* B,
                 int64_t ldb, T* C, int64_t ldc) {
    using Bk = Blk<T>;
    constexpr int MR = Bk::MR, NR = Bk::NR;
    std::vector<T> Bp(size_t(Bk::KC) * size_t(((Bk::NC + NR - 1) / NR) * NR));
    for (int64_t jc = 0; jc < n; jc += Bk::NC) {
        const int64_t nc = std::min(Bk::NC, n - jc);
        for (int64_t pc = 0; pc < k; pc += Bk::KC) {
            const int64_t kc = std::min(Bk::KC, k - pc);
            pack_b(opB, B, ldb, pc, kc, jc, nc, Bp.data());
            const int64_t nic = (m + Bk::MC - 1) / Bk::MC;
            #pragma omp parallel if (double(m) * nc * kc > 2e6)
            {
                std::vector<T> Ap(size_t(Bk::MC) * size_t(kc));
                #pragma omp for schedule(dynamic)
                for (int64_t ib = 0; ib < nic; ++ib) {
                    const int64_t ic = ib * Bk::MC, mc = std::min(Bk::MC, m - ic);
                    pack_a(opA, A, lda, ic, mc, pc, kc, Ap.data());
                    for (int64_t jr = 0; jr < nc; jr += NR) {
                        const int nr = int(std::min<int64_t>(NR, nc - jr));
                        T const* bp = Bp.data() + (jr / NR) * NR * kc;
                        for (int64_t ir = 0; ir < mc; ir += MR) {
                            const int mr = int(std::min<int64_t>(MR, mc - ir));
                            micro(kc, Ap.data() + (ir / MR) * MR * kc, bp, alpha, C + (ic + ir) + (jc + jr) * ldc,
                                  ldc, mr, nr);
                        }
                    }
                }
            }
        }
    }
}

}  // namespace gemm_detail

/// C = alpha op(A) op(B) + beta C
template <typename T>
void gemm(Op opA, Op opB, int64_t m, int64_t n, int64_t k, T alpha,
          T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc)
{
    if (m <= 0 || n <= 0) return;
    if constexpr (std::is_same<T, double>::value || std::is_same<T, float>::value) {
        if (double(m) * n * k >= 32768.0 && m >= 8 && n >= 6) {
            #pragma omp parallel for schedule(static) if (m * n > 65536)
            for (int64_t j = 0; j < n; ++j) {
                T* c = C + j * ldc;
                if (beta == T(0)) for (int64_t i = 0; i < m; ++i) c[i] = T(0);
                else if (beta != T(1)) for (int64_t i = 0; i < m; ++i) c[i] *= beta;
            }
            if (alpha != T(0) && k > 0) gemm_detail::gemm_packed(opA, opB, m, n, k, alpha, A, lda, B, ldb, C, ldc);
            return;
        }
    }
    std::vector<T> Ap, Bp;
    if (opA != Op::NoTrans && k > 0) { Ap.resize(size_t(m) * k); pack(opA, m, k, A, lda, Ap.data()); A = Ap.data(); lda = m; }
    if (opB != Op::NoTrans && k > 0) { Bp.resize(size_t(k) * n); pack(opB, k, n, B, ldb, Bp.data()); B = Bp.data(); ldb = k; }
    const int64_t MB = 256, KB = 128, NB = 32;
    int64_t nblk = ceildiv(n, NB);
    #pragma omp parallel for schedule(dynamic) if (double(m) * n * std::max<int64_t>(k, 1) > 1e6)
    for (int64_t jb = 0; jb < nblk; ++jb) {
        int64_t j0 = jb * NB, j1 = std::min(n, j0 + NB);
        for (int64_t j = j0; j < j1; ++j) {
            T* c = C + j * ldc;
            if (beta == T(0)) for (int64_t i = 0; i < m; ++i) c[i] = T(0);
            else if (beta != T(1)) for (int64_t i = 0; i < m; ++i) c[i] *= beta;
        }
        if (alpha == T(0)) continue;
        for (int64_t l0 = 0; l0 < k; l0 += KB) {
            int64_t l1 = std::min(k, l0 + KB);
            for (int64_t i0 = 0; i0 < m; i0 += MB) {
                int64_t i1 = std::min(m, i0 + MB);
                for (int64_t j = j0; j < j1; ++j) {
                    T* __restrict__ c = C + j * ldc;
                    for (int64_t l = l0; l < l1; ++l) {
                        T b = alpha * B[l + j * ldb];
                        T const* __restrict__ a = A + l * lda;
                        for (int64_t i = i0; i < i1; ++i) c[i] += a[i] * b;
                    }
                }
            }
        }
    }
}

/// C = alpha A op(A) ... : herk/syrk on the uplo triangle of C (n x n):
/// C = alpha op(A) op(A)^{H or T} + beta C, op(A) is n x k.
template <typename T>
void rankk(bool herm, Uplo uplo, Op op, int64_t n, int64_t k, T alpha, T const* A, int64_t lda,
           T beta, T* C, int64_t ldc)
{
    if (n <= 0) return;
    // X = op(A) (n x k)
    std::vector<T> X(size_t(n) * std::max<int64_t>(k, 1));
    if (k > 0) pack(op, n, k, A, lda, X.data());
    #pragma omp parallel for schedule(dynamic) if (n * n * k > 1000000)
    for (int64_t j = 0; j < n; ++j) {
        int64_t i0 = uplo == Uplo::Lower ? j : 0, i1 = uplo == Uplo::Lower ? n : j + 1;
        for (int64_t i = i0; i < i1; ++i) {
            T s = T(0);
            for (int64_t l = 0; l < k; ++l)
                s += X[i + l * n] * (herm ? slate::conj(X[j + l * n]) : X[j + l * n]);
            T c = beta == T(0) ? T(0) : beta * C[i + j * ldc];
            C[i + j * ldc] = alpha * s + c;
            if (herm && i == j) C[i + j * ldc] = real(C[i + j * ldc]);
        }
    }
}

/// rank-2k: C = alpha X Y^{H/T} + conj(alpha) Y X^{H/T} + beta C  (X = op(A), Y = op(B))
template <typename T>
void rank2k(bool herm, Uplo uplo, Op op, int64_t n, int64_t k, T alpha, T const* A, int64_t lda,
            T const* B, int64_t ldb, T beta, T* C, int64_t ldc)
{
    if (n <= 0) return;
    std::vector<T> X(size_t(n) * std::max<int64_t>(k, 1)), Y(size_t(n) * std::max<int64_t>(k, 1));
    if (k > 0) { pack(op, n, k, A, lda, X.data()); pack(op, n, k, B, ldb, Y.data()); }
    T alpha2 = herm ? slate::conj(alpha) : alpha;
    #pragma omp parallel for schedule(dynamic) if (n * n * k > 1000000)
    for (int64_t j = 0; j < n; ++j) {
        int64_t i0 = uplo == Uplo::Lower ? j : 0, i1 = uplo == Uplo::Lower ? n : j + 1;
        for (int64_t i = i0; i < i1; ++i) {
            T s1 = T(0), s2 = T(0);
            for (int64_t l = 0; l < k; ++l) {
                s1 += X[i + l * n] * (herm ? slate::conj(Y[j + l * n]) : Y[j + l * n]);
                s2 += Y[i + l * n] * (herm ? slate::conj(X[j + l * n]) : X[j + l * n]);
            }
            T c = beta == T(0) ? T(0) : beta * C[i + j * ldc];
            C[i + j * ldc] = alpha * s1 + alpha2 * s2 + c;
            if (herm && i == j) C[i + j * ldc] = real(C[i + j * ldc]);
        }
    }
}

/// Expand a symmetric/Hermitian matrix stored in `uplo` into a full dense copy.
template <typename T>
std::vector<T> expand_sym(bool herm, Uplo uplo, int64_t n, T const* A, int64_t lda) {
    std::vector<T> F(size_t(n) * n);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) {
            bool stored = uplo == Uplo::Lower ? i >= j : i <= j;
            T v = stored ? A[i + j * lda] : A[j + i * lda];
            if (!stored && herm) v = slate::conj(v);
            if (herm && i == j) v = real(v);
            F[i + j * n] = v;
        }
    return F;
}

/// hemm/symm: C = alpha A B + beta C (Left) or alpha B A + beta C (Right)
template <typename T>
void symm(bool herm, Side side, Uplo uplo, int64_t m, int64_t n, T alpha, T const* A, int64_t lda,
          T const* B, int64_t ldb, T beta, T* C, int64_t ldc)
{
    int64_t na = side == Side::Left ? m : n;
    auto F = expand_sym(herm, uplo, na, A, lda);
    if (side == Side::Left) gemm(Op::NoTrans, Op::NoTrans, m, n, m, alpha, F.data(), m, B, ldb, beta, C, ldc);
    else gemm(Op::NoTrans, Op::NoTrans, m, n, n, alpha, B, ldb, F.data(), n, beta, C, ldc);
}

/// Dense copy of op(triangle) with unit/zero fill (n x n).
template <typename T>
std::vector<T> expand_tri(Uplo uplo, Diag diag, int64_t n, T const* A, int64_t lda) {
    std::vector<T> F(size_t(n) * n, T(0));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) {
            bool in = uplo == Uplo::Lower ? i >= j : i <= j;
            if (!in) continue;
            F[i + j * n] = (i == j && diag == Diag::Unit) ? T(1) : A[i + j * lda];
        }
    return F;
}

/// B = alpha op(A) B (Left) or alpha B op(A) (Right), A triangular
template <typename T>
void trmm(Side side, Uplo uplo, Op op, Diag diag, int64_t m, int64_t n, T alpha,
          T const* A, int64_t lda, T* B, int64_t ldb)
{
    if (m <= 0 || n <= 0) return;
    int64_t na = side == Side::Left ? m : n;
    auto F = expand_tri(uplo, diag, na, A, lda);
    std::vector<T> Bc(size_t(m) * n);
    for (int64_t j = 0; j < n; ++j) for (int64_t i = 0; i < m; ++i) Bc[i + j * m] = B[i + j * ldb];
    if (side == Side::Left) gemm(op, Op::NoTrans, m, n, m, alpha, F.data(), m, Bc.data(), m, T(0), B, ldb);
    else gemm(Op::NoTrans, op, m, n, n, alpha, Bc.data(), m, F.data(), n, T(0), B, ldb);
}

/// Solve op(A) X = alpha B (Left) or X op(A) = alpha B (Right); X overwrites B.
template <typename T>
void trsm(Side side, Uplo uplo, Op op, Diag diag, int64_t m, int64_t n, T alpha,
          T const* A, int64_t lda, T* B, int64_t ldb)
{
    if (m <= 0 || n <= 0) return;
    if (alpha != T(1))
        for (int64_t j = 0; j < n; ++j) for (int64_t i = 0; i < m; ++i) B[i + j * ldb] *= alpha;
    // Reduce Right to Left by transposition: X op(A) = B  <=>  op(A)^T X^T = B^T
    if (side == Side::Right) {
        std::vector<T> Bt(size_t(n) * m);
        for (int64_t j = 0; j < n; ++j) for (int64_t i = 0; i < m; ++i) Bt[j + i * n] = B[i + j * ldb];
        // op(A)^T: NoTrans->Trans, Trans->NoTrans, ConjTrans -> conj(A) untransposed
        if (op == Op::ConjTrans) {
            // X A^H = B  <=>  conj(A) X^T... use conj: (X A^H)^T = conj(A) X^T
            std::vector<T> Ac(size_t(n) * n);
            for (int64_t j = 0; j < n; ++j) for (int64_t i = 0; i < n; ++i) Ac[i + j * n] = slate::conj(A[i + j * lda]);
            trsm(Side::Left, uplo, Op::NoTrans, diag, n, m, T(1), Ac.data(), n, Bt.data(), n);
        } else {
            trsm(Side::Left, uplo, op == Op::NoTrans ? Op::Trans : Op::NoTrans, diag, n, m, T(1), A, lda, Bt.data(), n);
        }
        for (int64_t j = 0; j < n; ++j) for (int64_t i = 0; i < m; ++i) B[i + j * ldb] = Bt[j + i * n];
        return;
    }
    // Left: effective lower if (Lower, NoTrans) or (Upper, Trans)
    bool lower_eff = (uplo == Uplo::Lower) == (op == Op::NoTrans);
    #pragma omp parallel for schedule(static) if (m * m * n > 1000000)
    for (int64_t j = 0; j < n; ++j) {
        T* b = B + j * ldb;
        if (lower_eff) {
            for (int64_t i = 0; i < m; ++i) {
                T s = b[i];
                for (int64_t l = 0; l < i; ++l) s -= opval(op, A, lda, i, l) * b[l];
                b[i] = diag == Diag::Unit ? s : s / opval(op, A, lda, i, i);
            }
        } else {
            for (int64_t i = m - 1; i >= 0; --i) {
                T s = b[i];
                for (int64_t l = i + 1; l < m; ++l) s -= opval(op, A, lda, i, l) * b[l];
                b[i] = diag == Diag::Unit ? s : s / opval(op, A, lda, i, i);
            }
        }
    }
}

//------------------------------------------------------------------------------
/// Cholesky of the uplo triangle; returns info (0 or 1-based failing column).
template <typename T>
int64_t potrf(Uplo uplo, int64_t n, T* A, int64_t lda) {
    using R = real_type<T>;
    if (uplo == Uplo::Upper) {
        // A = U^H U : work on conj-transpose as lower
        for (int64_t j = 0; j < n; ++j) {
            R d = real(A[j + j * lda]);
            for (int64_t l = 0; l < j; ++l) d -= std::norm(A[l + j * lda]);
            if (!(d > 0)) return j + 1;
            R s = std::sqrt(d);
            A[j + j * lda] = s;
            #pragma omp parallel for if (n - j > 256)
            for (int64_t i = j + 1; i < n; ++i) {
                T v = A[j + i * lda];
                for (int64_t l = 0; l < j; ++l) v -= slate::conj(A[l + j * lda]) * A[l + i * lda];
                A[j + i * lda] = v / s;
            }
        }
        return 0;
    }
    for (int64_t j = 0; j < n; ++j) {
        R d = real(A[j + j * lda]);
        for (int64_t l = 0; l < j; ++l) d -= std::norm(A[j + l * lda]);
        if (!(d > 0)) return j + 1;
        R s = std::sqrt(d);
        A[j + j * lda] = s;
        #pragma omp parallel for if (n - j > 256)
        for (int64_t i = j + 1; i < n; ++i) {
            T v = A[i + j * lda];
            for (int64_t l = 0; l < j; ++l) v -= A[i + l * lda] * slate::conj(A[j + l * lda]);
            A[i + j * lda] = v / s;
        }
    }
    return 0;
}

/// LU with partial pivoting (right-looking, rank-1 updates, OpenMP over columns).
/// ipiv[j] = 0-based row swapped with row j.  Returns info (1-based first zero pivot).
/// thresh < 1: threshold pivoting, the diagonal stays pivot while |a_jj| >= thresh * max.
template <typename T>
int64_t getrf(int64_t m, int64_t n, T* A, int64_t lda, int64_t* ipiv, bool pivot = true, double thresh = 1.0) {
    int64_t info = 0;
    int64_t mn = std::min(m, n);
    for (int64_t j = 0; j < mn; ++j) {
        int64_t p = j;
        if (pivot) {
            real_type<T> best = -1;
            for (int64_t i = j; i < m; ++i) {
                real_type<T> v = cabs1(A[i + j * lda]);
                if (v > best) { best = v; p = i; }
            }
            if (thresh < 1.0 && p != j && cabs1(A[j + j * lda]) >= real_type<T>(thresh) * best) p = j;
        }
        ipiv[j] = p;
        if (p != j)
            for (int64_t c = 0; c < n; ++c) std::swap(A[j + c * lda], A[p + c * lda]);
        T d = A[j + j * lda];
        if (d == T(0)) { if (info == 0) info = j + 1; continue; }
        T rd = T(1) / d;
        for (int64_t i = j + 1; i < m; ++i) A[i + j * lda] *= rd;
        #pragma omp parallel for schedule(static) if ((m - j) * (n - j) > 65536)
        for (int64_t c = j + 1; c < n; ++c) {
            T u = A[j + c * lda];
            if (u == T(0)) continue;
            T* ac = A + c * lda;
            T const* aj = A + j * lda;
            for (int64_t i = j + 1; i < m; ++i) ac[i] -= aj[i] * u;
        }
    }
    return info;
}

/// Apply row interchanges ipiv[k1..k2) (0-based absolute rows) to n columns.
template <typename T>
void laswp(int64_t n, T* A, int64_t lda, int64_t k1, int64_t k2, int64_t const* ipiv, bool forward = true) {
    if (forward) {
        for (int64_t k = k1; k < k2; ++k)
            if (ipiv[k] != k) for (int64_t c = 0; c < n; ++c) std::swap(A[k + c * lda], A[ipiv[k] + c * lda]);
    } else {
        for (int64_t k = k2 - 1; k >= k1; --k)
            if (ipiv[k] != k) for (int64_t c = 0; c < n; ++c) std::swap(A[k + c * lda], A[ipiv[k] + c * lda]);
    }
}

//------------------------------------------------------------------------------
/// Householder reflector (LAPACK larfg): given alpha and x (n-1), produce
/// beta, tau, v (v(0)=1 implicit) with H^H [alpha; x] = [beta; 0].
template <typename T>
void larfg(int64_t n, T& alpha, T* x, int64_t incx, T& tau) {
    using R = real_type<T>;
    if (n <= 0) { tau = T(0); return; }
    R xnorm = 0, scale = 0, ssq = 1;
    for (int64_t i = 0; i < n - 1; ++i) {
        R a = std::abs(x[i * incx]);
        if (a != 0) add_sumsq(scale, ssq, a);
    }
    xnorm = scale * std::sqrt(ssq);
    R alphr = real(alpha), alphi = imag(alpha);
    if (xnorm == 0 && alphi == 0) { tau = T(0); return; }
    R beta = -std::copysign(std::hypot(std::hypot(alphr, alphi), xnorm), alphr);
    // |beta| below the safe minimum (bulge chasing drives entries toward
    // denormals): rescale x and alpha by 1/safmin until it is not, as LAPACK
    // larfg does, so 1 / (alpha - beta) cannot overflow
    const R safmin = std::numeric_limits<R>::min() / std::numeric_limits<R>::epsilon();
    int knt = 0;
    if (std::abs(beta) < safmin) {
        const R rsafmn = R(1) / safmin;
        do {
            ++knt;
            for (int64_t i = 0; i < n - 1; ++i) x[i * incx] *= rsafmn;
            beta *= rsafmn;
            alpha *= rsafmn;
        } while (std::abs(beta) < safmin && knt < 20);
        scale = 0; ssq = 1;
        for (int64_t i = 0; i < n - 1; ++i) {
            R a = std::abs(x[i * incx]);
            if (a != 0) add_sumsq(scale, ssq, a);
        }
        xnorm = scale * std::sqrt(ssq);
        alphr = real(alpha);
        alphi = imag(alpha);
        beta = -std::copysign(std::hypot(std::hypot(alphr, alphi), xnorm), alphr);
    }
    T t;
    if constexpr (is_complex_v<T>) t = T((beta - alphr) / beta, -alphi / beta);
    else t = T((beta - alphr) / beta);
    T scal = T(1) / (alpha - T(beta));
    for (int64_t i = 0; i < n - 1; ++i) x[i * incx] *= scal;
    for (int k = 0; k < knt; ++k) beta *= safmin;
    tau = t;
    alpha = T(beta);
}

/// Unblocked QR (geqr2): A = Q R, V below the diagonal, tau[min(m,n)].
template <typename T>
void geqr2(int64_t m, int64_t n, T* A, int64_t lda, T* tau) {
    int64_t k = std::min(m, n);
    for (int64_t j = 0; j < k; ++j) {
        larfg(m - j, A[j + j * lda], A + (j + 1) + j * lda, 1, tau[j]);
        if (j + 1 < n && tau[j] != T(0)) {
            T ajj = A[j + j * lda];
            A[j + j * lda] = T(1);
            T tc = slate::conj(tau[j]);
            #pragma omp parallel for if ((m - j) * (n - j) > 65536)
            for (int64_t c = j + 1; c < n; ++c) {
                T w = T(0);
                for (int64_t i = j; i < m; ++i) w += slate::conj(A[i + j * lda]) * A[i + c * lda];
                w *= tc;
                for (int64_t i = j; i < m; ++i) A[i + c * lda] -= A[i + j * lda] * w;
            }
            A[j + j * lda] = ajj;
        }
    }
}

/// Form the upper-triangular T (k x k) of a forward, columnwise block
/// reflector H = I - V T V^H (LAPACK larft), V m x k unit lower.
template <typename T>
void larft(int64_t m, int64_t k, T const* V, int64_t ldv, T const* tau, T* Tm, int64_t ldt) {
    for (int64_t i = 0; i < k; ++i) {
        for (int64_t r = 0; r < k; ++r) if (r > i) Tm[r + i * ldt] = T(0);
        if (tau[i] == T(0)) {
            for (int64_t r = 0; r <= i; ++r) Tm[r + i * ldt] = T(0);
            continue;
        }
        // T(0:i, i) = -tau(i) V(i:m, 0:i)^H V(i:m, i)
        for (int64_t r = 0; r < i; ++r) {
            T s = slate::conj(V[i + r * ldv]);  // V(i,i) = 1
            for (int64_t l = i + 1; l < m; ++l) s += slate::conj(V[l + r * ldv]) * V[l + i * ldv];
            Tm[r + i * ldt] = -tau[i] * s;
        }
        // T(0:i, i) = T(0:i, 0:i) T(0:i, i)
        for (int64_t r = 0; r < i; ++r) {
            T s = T(0);
            for (int64_t l = r; l < i; ++l) s += Tm[r + l * ldt] * Tm[l + i * ldt];
            Tm[r + i * ldt] = s;
        }
        Tm[i + i * ldt] = tau[i];
    }
}

/// Apply H = I - V T V^H (or H^H) from the left or right to C (larfb,
/// forward columnwise).  V is m_v x k unit lower-trapezoidal (diag implicit).
template <typename T>
void larfb(Side side, Op op, int64_t m, int64_t n, int64_t k, T const* V, int64_t ldv,
           T const* Tm, int64_t ldt, T* C, int64_t ldc)
{
    if (m <= 0 || n <= 0 || k <= 0) return;
    int64_t mv = side == Side::Left ? m : n;
    // explicit V with unit diagonal and zeros above
    std::vector<T> Vf(size_t(mv) * k, T(0));
    for (int64_t j = 0; j < k; ++j)
        for (int64_t i = j; i < mv; ++i) Vf[i + j * mv] = (i == j) ? T(1) : V[i + j * ldv];
    std::vector<T> Tf(size_t(k) * k, T(0));
    for (int64_t j = 0; j < k; ++j) for (int64_t i = 0; i <= j; ++i) Tf[i + j * k] = Tm[i + j * ldt];
    if (side == Side::Left) {
        // C = H^op C = C - V op(T) (V^H C)
        std::vector<T> W(size_t(k) * n), W2(size_t(k) * n);
        gemm(Op::ConjTrans, Op::NoTrans, k, n, m, T(1), Vf.data(), mv, C, ldc, T(0), W.data(), k);
        gemm(op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans, Op::NoTrans, k, n, k, T(1), Tf.data(), k, W.data(), k, T(0), W2.data(), k);
        gemm(Op::NoTrans, Op::NoTrans, m, n, k, T(-1), Vf.data(), mv, W2.data(), k, T(1), C, ldc);
    } else {
        // C = C H^op = C - (C V) op(T) V^H
        std::vector<T> W(size_t(m) * k), W2(size_t(m) * k);
        gemm(Op::NoTrans, Op::NoTrans, m, k, n, T(1), C, ldc, Vf.data(), mv, T(0), W.data(), m);
        gemm(Op::NoTrans, op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans, m, k, k, T(1), W.data(), m, Tf.data(), k, T(0), W2.data(), m);
        gemm(Op::NoTrans, Op::ConjTrans, m, n, k, T(-1), W2.data(), m, Vf.data(), mv, T(1), C, ldc);
    }
}

/// Blocked QR: A = Q R with T factors per ib-block stored in Tm (ib x n).
template <typename T>
void geqrf(int64_t m, int64_t n, T* A, int64_t lda, T* tau, int64_t ib = 32) {
    int64_t k = std::min(m, n);
    std::vector<T> Tb(size_t(ib) * ib);
    for (int64_t j = 0; j < k; j += ib) {
        int64_t jb = std::min(ib, k - j);
        geqr2(m - j, jb, A + j + j * lda, lda, tau + j);
        if (j + jb < n) {
            larft(m - j, jb, A + j + j * lda, lda, tau + j, Tb.data(), ib);
            larfb(Side::Left, Op::ConjTrans, m - j, n - j - jb, jb, A + j + j * lda, lda,
                  Tb.data(), ib, A + j + (j + jb) * lda, lda);
        }
    }
}

/// Triangular inverse in place.
template <typename T>
void trtri(Uplo uplo, Diag diag, int64_t n, T* A, int64_t lda) {
    // column-by-column (LAPACK trti2 style)
    if (uplo == Uplo::Upper) {
        for (int64_t j = 0; j < n; ++j) {
            T ajj;
            if (diag == Diag::NonUnit) { A[j + j * lda] = T(1) / A[j + j * lda]; ajj = -A[j + j * lda]; }
            else ajj = T(-1);
            // x = A(0:j,0:j) * A(0:j, j)  (upper triangular matvec, already inverted part)
            for (int64_t i = 0; i < j; ++i) {
                T s = T(0);
                for (int64_t l = i; l < j; ++l) {
                    T a = (l == i && diag == Diag::Unit) ? T(1) : A[i + l * lda];
                    s += a * A[l + j * lda];
                }
                A[i + j * lda] = s;
            }
            for (int64_t i = 0; i < j; ++i) A[i + j * lda] *= ajj;
        }
    } else {
        for (int64_t j = n - 1; j >= 0; --j) {
            T ajj;
            if (diag == Diag::NonUnit) { A[j + j * lda] = T(1) / A[j + j * lda]; ajj = -A[j + j * lda]; }
            else ajj = T(-1);
            if (j < n - 1) {
                for (int64_t i = n - 1; i > j; --i) {
                    T s = T(0);
                    for (int64_t l = j + 1; l <= i; ++l) {
                        T a = (l == i && diag == Diag::Unit) ? T(1) : A[i + l * lda];
                        s += a * A[l + j * lda];
                    }
                    A[i + j * lda] = s;
                }
                for (int64_t i = j + 1; i < n; ++i) A[i + j * lda] *= ajj;
            }
        }
    }
}

/// L^H L (Lower) or U U^H (Upper) in place (LAPACK lauum).
template <typename T>
void lauum(Uplo uplo, int64_t n, T* A, int64_t lda) {
    std::vector<T> F(size_t(n) * n, T(0)), R(size_t(n) * n);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i)
            if (uplo == Uplo::Lower ? i >= j : i <= j) F[i + j * n] = A[i + j * lda];
    if (uplo == Uplo::Lower) gemm(Op::ConjTrans, Op::NoTrans, n, n, n, T(1), F.data(), n, F.data(), n, T(0), R.data(), n);
    else gemm(Op::NoTrans, Op::ConjTrans, n, n, n, T(1), F.data(), n, F.data(), n, T(0), R.data(), n);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i)
            if (uplo == Uplo::Lower ? i >= j : i <= j) A[i + j * lda] = R[i + j * n];
}

}  // namespace host
}  // namespace slate
