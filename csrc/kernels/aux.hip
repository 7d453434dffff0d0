// Auxiliary gfx950 kernels: set / copy+convert / add / scale / transpose /
// diagonal-block triangular inverse / small Cholesky / row permutation.
//
// Reference counterparts: src/cuda/device_{geset,tzset,gecopy,tzcopy,geadd,
// tzadd,gescale,tzscale,gescale_row_col,transpose}.cu.  The reference launches
// one thread block per tile with one thread per row; here the local array is
// one strided block, so kernels use a 2-D grid of 64x4 thread tiles where
// consecutive lanes walk consecutive rows (coalesced column-major access) and
// each thread handles several columns.
#include "device_common.hh"
#include "kernels.hh"
#include "slate_amd/device.hh"
#include "leaf_common.hh"

#include <cstdlib>
#include <stdexcept>
#include <type_traits>

namespace slate_amd {
namespace dev {

namespace {

constexpr int TX = 64, TY = 4, COLS_PER_THREAD = 8;

inline dim3 grid2d(int64_t m, int64_t n) {
    int64_t gx = (m + TX - 1) / TX;
    int64_t gy = (n + TY * COLS_PER_THREAD - 1) / (TY * COLS_PER_THREAD);
    return dim3((unsigned)gx, (unsigned)std::min<int64_t>(gy, 65535));
}

// in-triangle test: uplo 'L' keeps i >= j (+ offset), 'U' keeps i <= j, 'G' all
__device__ inline bool in_tri(char uplo, int64_t i, int64_t j) {
    return uplo == 'G' || (uplo == 'L' ? i >= j : i <= j);
}

template <typename T>
__global__ void set_kernel(char uplo, int64_t m, int64_t n, T offdiag, T diag, T* A, int64_t lda) {
    int64_t i = blockIdx.x * (int64_t)TX + threadIdx.x;
    if (i >= m) return;
    for (int64_t j = blockIdx.y * (int64_t)TY * COLS_PER_THREAD + threadIdx.y; j < n;
         j += (int64_t)gridDim.y * TY * COLS_PER_THREAD) {
        #pragma unroll
        for (int c = 0; c < COLS_PER_THREAD; ++c) {
            int64_t jj = j + c * TY;
            if (jj < n && in_tri(uplo, i, jj))
                A[i + jj * lda] = (i == jj) ? diag : offdiag;
        }
    }
}

template <typename Ts, typename Td>
__device__ inline Td convert(Ts v) {
    if constexpr (is_cplx<Ts>::value && is_cplx<Td>::value)
        return Td((real_t<Td>)v.re, (real_t<Td>)v.im);
    else if constexpr (is_cplx<Td>::value)
        return Td((real_t<Td>)v, 0);
    else if constexpr (is_cplx<Ts>::value)
        return Td(v.re);
    else
        return Td(v);
}

// B = op(A) with precision conversion; trans: 'N', 'T', 'C'.
// For op != N, reads A[j + i*lda] (uncoalesced on one side; transposes of
// large matrices go through transpose_kernel instead).
template <typename Ts, typename Td>
__global__ void copy_kernel(char uplo, char trans, int64_t m, int64_t n,
                            const Ts* A, int64_t lda, Td* B, int64_t ldb) {
    int64_t i = blockIdx.x * (int64_t)TX + threadIdx.x;
    if (i >= m) return;
    for (int64_t j = blockIdx.y * (int64_t)TY * COLS_PER_THREAD + threadIdx.y; j < n;
         j += (int64_t)gridDim.y * TY * COLS_PER_THREAD) {
        #pragma unroll
        for (int c = 0; c < COLS_PER_THREAD; ++c) {
            int64_t jj = j + c * TY;
            if (jj < n && in_tri(uplo, i, jj)) {
                Ts v = trans == 'N' ? A[i + jj * lda] : A[jj + i * lda];
                if (trans == 'C') v = conj(v);
                B[i + jj * ldb] = convert<Ts, Td>(v);
            }
        }
    }
}

// B = alpha A + beta B
template <typename T>
__global__ void add_kernel(char uplo, int64_t m, int64_t n, T alpha, const T* A, int64_t lda,
                           T beta, T* B, int64_t ldb) {
    int64_t i = blockIdx.x * (int64_t)TX + threadIdx.x;
    if (i >= m) return;
    bool bz = is_zero(beta);
    for (int64_t j = blockIdx.y * (int64_t)TY * COLS_PER_THREAD + threadIdx.y; j < n;
         j += (int64_t)gridDim.y * TY * COLS_PER_THREAD) {
        #pragma unroll
        for (int c = 0; c < COLS_PER_THREAD; ++c) {
            int64_t jj = j + c * TY;
            if (jj < n && in_tri(uplo, i, jj)) {
                T v = alpha * A[i + jj * lda];
                if (!bz) v += beta * B[i + jj * ldb];
                B[i + jj * ldb] = v;
            }
        }
    }
}

// A *= numer/denom  (computed as one multiplier, overflow-safe split as in
// LAPACK lascl is done on the host side by choosing mul)
template <typename T>
__global__ void scale_kernel(char uplo, int64_t m, int64_t n, real_t<T> mul, T* A, int64_t lda) {
    int64_t i = blockIdx.x * (int64_t)TX + threadIdx.x;
    if (i >= m) return;
    for (int64_t j = blockIdx.y * (int64_t)TY * COLS_PER_THREAD + threadIdx.y; j < n;
         j += (int64_t)gridDim.y * TY * COLS_PER_THREAD) {
        #pragma unroll
        for (int c = 0; c < COLS_PER_THREAD; ++c) {
            int64_t jj = j + c * TY;
            if (jj < n && in_tri(uplo, i, jj)) A[i + jj * lda] = A[i + jj * lda] * mul;
        }
    }
}

// A = diag(R) A diag(C)  (equilibration); R or C may be null
// B(i, j) = s[i] * A(i, j) with A real: a real eigenvector matrix into the
// (complex) working precision with a row phase (heev / svd stage 2)
template <typename T>
__global__ void real_rowscale_kernel(int64_t m, int64_t n, const real_t<T>* A, int64_t lda, const T* sc, T* B,
                                     int64_t ldb) {
    int64_t i = blockIdx.x * (int64_t)TX + threadIdx.x;
    if (i >= m) return;
    const T si = sc ? sc[i] : T(real_t<T>(1));
    for (int64_t j = blockIdx.y * (int64_t)TY * COLS_PER_THREAD + threadIdx.y; j < n;
         j += (int64_t)gridDim.y * TY * COLS_PER_THREAD) {
        #pragma unroll
        for (int c = 0; c < COLS_PER_THREAD; ++c) {
            int64_t jj = j + c * TY;
            if (jj < n) B[i + jj * ldb] = si * T(A[i + jj * lda]);
        }
    }
}

template <typename T>
__global__ void scale_row_col_kernel(int64_t m, int64_t n, const real_t<T>* R, const real_t<T>* C,
                                     T* A, int64_t lda) {
    int64_t i = blockIdx.x * (int64_t)TX + threadIdx.x;
    if (i >= m) return;
    real_t<T> r = R ? R[i] : real_t<T>(1);
    for (int64_t j = blockIdx.y * (int64_t)TY * COLS_PER_THREAD + threadIdx.y; j < n;
         j += (int64_t)gridDim.y * TY * COLS_PER_THREAD) {
        #pragma unroll
        for (int c = 0; c < COLS_PER_THREAD; ++c) {
            int64_t jj = j + c * TY;
            if (jj < n) A[i + jj * lda] = A[i + jj * lda] * (r * (C ? C[jj] : real_t<T>(1)));
        }
    }
}

// Out-of-place transpose through an LDS tile (reference device_transpose.cu
// :242-506 uses NB=32 tiles with an [NB][NX+1] pad; same idea, 64-wide rows).
template <typename T>
__global__ void transpose_kernel(bool conjugate, int64_t m, int64_t n, const T* A, int64_t lda, T* B, int64_t ldb) {
    constexpr int NBT = 64;
    __shared__ T tile[NBT][NBT + 1];
    int64_t i0 = blockIdx.x * (int64_t)NBT, j0 = blockIdx.y * (int64_t)NBT;
    int tx = threadIdx.x, ty = threadIdx.y;  // 64 x 4
    for (int jj = ty; jj < NBT; jj += 4) {
        int64_t i = i0 + tx, j = j0 + jj;
        if (i < m && j < n) tile[jj][tx] = A[i + j * lda];
    }
    __syncthreads();
    for (int ii = ty; ii < NBT; ii += 4) {
        int64_t j = j0 + tx, i = i0 + ii;   // B is n x m: B[j, i] = A[i, j]
        if (i < m && j < n) {
            T v = tile[tx][ii];
            B[j + i * ldb] = conjugate ? conj(v) : v;
        }
    }
}

//------------------------------------------------------------------------------
// Small triangular solve on one wave: X := A^{-1} B for the m x m (m <= MM,
// MM = 32 or 64) lower or upper triangle A and ncol <= 64 right-hand-side
// columns (B == nullptr: the identity, i.e. the inverse; then X may be null
// and S, (MM + 1) x 64 at least, carries the result), result into Out.
// One lane per column; the triangle in LDS as the row stream of leaf_solve
// (column c of the triangle as row c, reciprocal pivots on the diagonal; an
// upper triangle is solved as the lower one of the index-reversed system);
// the columns transposed through LDS so that global loads and stores stay
// coalesced.  Right-looking: a step's updates are independent FMAs (the
// dot-product form measured 42.7 / 18.1 us per 64 / 32 rows).  All global
// loads are unconditional (clamped row, column offsets in SGPRs) and
// unrolled so that they issue back to back: a rolled loop of guarded loads
// waited ~800 cycles per column.
template <typename T, int MM>
__device__ __forceinline__ void tri_solve_cols(bool lower, bool unit, int m, const T* A, int64_t lda, const T* B,
                                               int64_t ldb, T* Out, int64_t ldo, int ncol, T* S, T* X) {
    constexpr int LS = kLeafLS, XS = MM + 1;
    const int lane = threadIdx.x;
    const int lp = lower ? lane : MM - 1 - lane;     // lane = row l of the triangle
    const int lr = min(lane, m - 1);
    LEAF_STAMP(0);
    // (loads into registers first, LDS stores after: a load feeding the
    // LDS store of the same iteration waited alone, ~750 cycles per column)
    {
        const T* Al = A + lr;
        int64_t off = 0;
        const T dg = A[lr + (int64_t)lr * lda];
        T t[MM];
        #pragma unroll
        for (int c = 0; c < MM; ++c) {
            t[c] = Al[off];
            if (c + 1 < m) off += lda;
        }
        const T rdg = (unit || lane >= m) ? one<T>() : one<T>() / dg;
        #pragma unroll
        for (int c = 0; c < MM; ++c) {
            const T w = (lane == c) ? rdg : ((lane < m && c < m) ? t[c] : zero<T>());
            if (lane < MM) S[(lower ? c : MM - 1 - c) * LS + lp] = w;
        }
    }
    LEAF_STAMP(1);
    T y[MM];
    if (B) {
        const T* Bl = B + lr;
        int64_t off = 0;
        T t[64];
        #pragma unroll
        for (int e = 0; e < 64; ++e) {
            t[e] = Bl[off];
            if (e + 1 < ncol) off += ldb;
        }
        #pragma unroll
        for (int e = 0; e < 64; ++e)
            if (lane < MM) X[e * XS + lp] = (lane < m && e < ncol) ? t[e] : zero<T>();
        __syncthreads();
        LEAF_STAMP(2);
        #pragma unroll
        for (int c = 0; c < MM; ++c) y[c] = X[lane * XS + c];
    } else {
        // the identity: lane j's column has its one at solve index lp(j)
        __syncthreads();
        LEAF_STAMP(2);
        #pragma unroll
        for (int c = 0; c < MM; ++c) y[c] = (c == lp && lane < m) ? one<T>() : zero<T>();
    }
    LEAF_STAMP(3);
    leaf_solve<T, false, false, MM>(y, S);
    LEAF_STAMP(4);
    // the result goes back through LDS (X, or S once the solve has read it
    // when there is no X: the inverse needs no right-hand side)
    T* R = X ? X : S;
    constexpr int RS = XS;
    __syncthreads();
    #pragma unroll
    for (int c = 0; c < MM; ++c) R[lane * RS + c] = y[c];
    __syncthreads();
    if (lane < m) {
        T* Ol = Out + lane;
        int64_t off = 0;
        #pragma unroll
        for (int e = 0; e < 64; ++e) {
            if (e < ncol) Ol[off] = R[e * RS + lp];
            off += ldo;
        }
    }
    LEAF_STAMP(5);
}

//------------------------------------------------------------------------------
// Inverse of the diagonal nbs x nbs blocks of a triangular matrix (nbs <= 64).
// Block b of A (at A + b*nbs*(1+lda)) is inverted into W (same position in W,
// ld ldw); the full square block is written (zeros outside the triangle).
// One 64-lane wave per block: tri_solve_cols against the identity.
template <typename T>
__global__ __launch_bounds__(64)
void trtri_diag_kernel(char uplo, char diag, int64_t n, int nbs,
                       const T* A, int64_t lda, T* W, int64_t ldw, int64_t wrap) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ __attribute__((aligned(16))) T S[64 * kLeafLS];
    const int b = blockIdx.x;
    const int64_t off = (int64_t)b * nbs;
    const int nb = (int)min<int64_t>(nbs, n - off);
    const T* Ab = A + off + off * lda;
    // wrap > 0: W is a stack of wrap x wrap blocks (block t at W + t wrap^2,
    // ld = wrap), each holding the inverse of A's t-th diagonal wrap-block
    T* Wb = wrap > 0 ? W + (off / wrap) * wrap * wrap + (off % wrap) * (1 + ldw) : W + off + off * ldw;
    // the inverse = the solve against the identity (exact zeros outside the
    // triangle: the full square block is written)
    tri_solve_cols<T, 64>(uplo == 'L', diag == 'U', nb, Ab, lda, nullptr, 0, Wb, ldw, nb, S, nullptr);
}

//------------------------------------------------------------------------------
// Cholesky of a small (n <= 64) diagonal block: one wave, lane i owns row i
// of the lower factor in registers (left-looking, fully unrolled); row j's
// finished entries are broadcast with v_readlane.  Upper is handled as the
// conjugate transpose.  info (if non-null) receives info_offset + first
// failing column (1-based) when *info is still 0.
template <typename T>
__global__ __launch_bounds__(64)
void potrf_small_kernel(char uplo, int n, T* A, int64_t lda, int* info, int info_offset) {
    SLATE_PANEL_WAVE_PRIO();
    const int i = threadIdx.x;
    T a[64];
    #pragma unroll
    for (int l = 0; l < 64; ++l) {
        T v = zero<T>();
        if (i < n && l < n && i >= l)
            v = (uplo == 'L') ? A[i + (int64_t)l * lda] : conj(A[l + (int64_t)i * lda]);
        a[l] = v;
    }
    int fail = 0;
    #pragma unroll
    for (int j = 0; j < 64; ++j) {
        if (j < n) {
            T s = a[j];
            #pragma unroll
            for (int l = 0; l < j; ++l) s -= a[l] * conj(bcast_lane(a[l], j));
            real_t<T> d = real(bcast_lane(s, j));
            if (!(d > real_t<T>(0)) && fail == 0) fail = j + 1;
            real_t<T> sd = sqrt(d);
            if (i == j) a[j] = make_val<T>((double)sd);
            else if (i > j) a[j] = s * (real_t<T>(1) / sd);
        }
    }
    if (fail && info && i == 0 && *info == 0) *info = info_offset + fail;
    if (i < n) {
        #pragma unroll
        for (int l = 0; l < 64; ++l) {
            if (l <= i && l < n) {
                if (uplo == 'L') A[i + (int64_t)l * lda] = a[l];
                else A[l + (int64_t)i * lda] = conj(a[l]);
            }
        }
    }
}

//------------------------------------------------------------------------------
// Lower Cholesky of a small (n <= 64) diagonal block AND the inverse of its
// factor in one launch: the factorization as potrf_small (lane i owns row i),
// then the factor goes through LDS and lane j computes column j of L^{-1} by
// substitution as trtri_diag does.  A receives L (lower triangle only), W
// (ld ldw) the full 64 x 64 inverse (zero above the diagonal; identity
// padding beyond n).  One launch instead of potrf_small + set + trtri_diag
// on the blocked device potrf's critical path.
template <typename T>
__global__ __launch_bounds__(64)
void potrf_inv_small_kernel(int n, T* A, int64_t lda, T* W, int64_t ldw, int* info, int info_offset) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ T L[64][65];
    __shared__ T rd[64];
    const int i = threadIdx.x;
    T a[64];
    #pragma unroll
    for (int l = 0; l < 64; ++l)
        a[l] = (i < n && l < n && i >= l) ? A[i + (int64_t)l * lda] : zero<T>();
    int fail = 0;
    #pragma unroll
    for (int j = 0; j < 64; ++j) {
        if (j < n) {
            T s = a[j];
            #pragma unroll
            for (int l = 0; l < j; ++l) s -= a[l] * conj(bcast_lane(a[l], j));
            real_t<T> d = real(bcast_lane(s, j));
            if (!(d > real_t<T>(0)) && fail == 0) fail = j + 1;
            real_t<T> sd = sqrt(d);
            if (i == j) a[j] = make_val<T>((double)sd);
            else if (i > j) a[j] = s * (real_t<T>(1) / sd);
        }
    }
    if (fail && info && i == 0 && *info == 0) *info = info_offset + fail;
    #pragma unroll
    for (int l = 0; l < 64; ++l) {
        // identity padding keeps the substitution below well defined
        L[i][l] = (i < n && l < n) ? a[l] : ((i == l) ? one<T>() : zero<T>());
        if (i < n && l < n && l <= i) A[i + (int64_t)l * lda] = a[l];
    }
    __syncthreads();
    rd[i] = one<T>() / L[i][i];
    __syncthreads();
    const int j = i;
    T x[64];
    #pragma unroll
    for (int r = 0; r < 64; ++r) {
        T s = zero<T>();
        #pragma unroll
        for (int l = 0; l < r; ++l) s += L[r][l] * x[l];
        x[r] = (r < j) ? zero<T>() : ((r == j) ? rd[r] : -(s * rd[r]));
    }
    #pragma unroll
    for (int r = 0; r < 64; ++r) W[r + (int64_t)j * ldw] = x[r];
}

//------------------------------------------------------------------------------
// Leaf of the blocked device potrf (lower): the Cholesky factor of the b x b
// (b <= 64) diagonal block at A AND the rows below it, A21 := A21 L11^{-H}, in
// ONE launch of single-wave workgroups.  Replaces the factor + inverse kernel,
// the A21 * inv GEMM and the copy back per 64 columns (50 + 22 + 5 us per leaf
// on an idle MI355X).
//  * Every workgroup factors the diagonal block, right-looking, lane i owning
//    row i in registers: step j takes the pivot by v_readlane, writes column j
//    of L to LDS (diagonal as its reciprocal), updates element j+1 at once
//    from lane j+1 (the next step's pivot: the only update on the step-to-step
//    chain) and applies the rest of column j-1's rank-1 update from LDS
//    broadcast reads one step late, so those reads are in flight behind the
//    pivot chain.  Workgroup 0 writes L11; workgroup w >= 1 solves rows
//    (w-1)*64 .. +63 of A21 (right-looking substitution: the updates of a
//    step are independent FMAs).
//  * LDS columns stream in 16-row groups with the next group's reads issued
//    before the current group's FMAs, each group ending in an empty volatile
//    asm on its registers plus a scheduling barrier (left alone, the
//    scheduler sank the FMAs below every read and spilled 15 KB per lane).
//  * A partial leaf (b < 64) is factored as diag(A11, I), so every step is
//    unconditional; loads use wave-uniform column pointers and clamped rows
//    (no per-load branches or 64-bit address math per lane).
//  * rsqrt by v_rsq plus one Newton step instead of sqrt and a division.
template <typename T>
__global__ __launch_bounds__(64)
void potrf_leaf_kernel(int b, int r, T* A, int64_t lda, int* info, int info_offset, T* W, const T* Wprev, T* Aprev,
                       int bprev) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    constexpr int LS = kLeafLS;
    __shared__ __attribute__((aligned(16))) T LT[64 * LS];   // LT[j*LS + l] = L(l, j)
    const int i = threadIdx.x;
    LEAF_STAMP(0);
    {
        T a[64];
        {
            // columns past b re-read column b-1 (their values are not used:
            // i >= l >= b fails i < b); the column offset runs in SGPRs
            const T* Ai = A + min(i, b - 1);
            int64_t off = 0;
            #pragma unroll
            for (int l = 0; l < 64; ++l) {
                const T v = Ai[off];
                a[l] = (i >= l && i < b) ? v : ((i == l) ? one<T>() : zero<T>());
                if (l + 1 < b) off += lda;
            }
        }
        LEAF_STAMP(1);
        int fail = 0;
        T buf[2][kLeafG];
        auto step = [&](auto jc) __attribute__((always_inline)) {
            constexpr int j = decltype(jc)::value;
            // pivot: all earlier columns' updates of element j are in
            const R d = real(bcast_lane(a[j], j));
            if (!(d > R(0)) && fail == 0) fail = j + 1;
            const R rs = leaf_rsqrt(d);
            const R sd = d * rs;
            const T Lij = (i == j) ? make_val<T>((double)sd) : ((i > j) ? a[j] * rs : zero<T>());
            a[j] = Lij;
            LT[j * LS + i] = (i == j) ? make_val<T>((double)rs) : Lij;
            if constexpr (j + 1 < 64) {
                a[j + 1] -= Lij * conj(bcast_lane(Lij, j + 1));
                leaf_pin1(a[j + 1]);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (j == 0) {
                // prime the stream: column 0's first group (rows >= 2)
                #pragma unroll
                for (int e = 0; e < kLeafG; ++e) buf[0][e] = LT[leaf_g0(2) * kLeafG + e];
            }
            // column k = j - 1's update of rows >= j + 1, prefetching one group ahead
            constexpr int k = j - 1;
            if constexpr (k >= 0 && k + 2 < 64) {
                constexpr int q0 = leaf_fq0(k), g0 = leaf_g0(k + 2);
                const T Lk = a[k];           // L(i, k)
                #pragma unroll
                for (int g = g0; g < 64 / kLeafG; ++g) {
                    const int q = q0 + g - g0;
                    const int nk = (g + 1 < 64 / kLeafG) ? k : k + 1;
                    const int ng = (g + 1 < 64 / kLeafG) ? g + 1 : leaf_g0(k + 3);
                    if (nk + 2 < 64) {
                        #pragma unroll
                        for (int e = 0; e < kLeafG; ++e) buf[(q + 1) & 1][e] = LT[nk * LS + ng * kLeafG + e];
                    }
                    #pragma unroll
                    for (int e = 0; e < kLeafG; ++e)
                        if (g * kLeafG + e >= k + 2) a[g * kLeafG + e] -= Lk * conj(buf[q & 1][e]);
                    #pragma unroll
                    for (int e = 0; e < kLeafG; ++e)
                        if (g * kLeafG + e >= k + 2) leaf_pin1(a[g * kLeafG + e]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        };
#define LEAF_FSTEP(x) step(std::integral_constant<int, (x)>{});
        LEAF_REP64(LEAF_FSTEP)
#undef LEAF_FSTEP
        LEAF_STAMP(2);
        if (blockIdx.x == 0) {
            if (fail && fail <= b && info && i == 0 && *info == 0) *info = info_offset + fail;
            // With r > 0 the other workgroups may not have read A11 yet (they
            // can start late behind a concurrent GEMM): L11 goes to W and the
            // next leaf's workgroup 0 copies it into place (Wprev -> Aprev),
            // when every reader of that block has finished.
            const bool direct = (r == 0);
            T* Ai = direct ? A + i : W + i;
            const int64_t ld = direct ? lda : 64;
            int64_t off = 0;
            #pragma unroll
            for (int l = 0; l < 64; ++l) {      // predicated, not `break`: an early
                if (l <= i && i < b) Ai[off] = a[l];   // exit can leave the loop
                off += ld;                      // rolled and a[] in scratch
            }
        }
    }
    if (blockIdx.x == 0 && Aprev) {
        // all loads, then all stores (a load feeding the same iteration's
        // store waited alone: ~24 us on the leaf's workgroup 0)
        T* Ap = Aprev + i;
        const T* Wp = Wprev + i;
        T t[64];
        #pragma unroll
        for (int l = 0; l < 64; ++l) t[l] = Wp[l * 64];
        int64_t off = 0;
        #pragma unroll
        for (int l = 0; l < 64; ++l) {
            if (l < bprev && l <= i && i < bprev) Ap[off] = t[l];
            off += lda;
        }
    }
    if (blockIdx.x == 0) return;
    __syncthreads();
    const int64_t row = b + (int64_t)(blockIdx.x - 1) * 64 + i;
    const bool live = row < b + (int64_t)r;
    const int64_t rr = live ? row : b;      // r > 0 here: row b exists
    T y[64];
    {
        const T* Ar = A + rr;
        int64_t off = 0;
        #pragma unroll
        for (int c = 0; c < 64; ++c) {
            const T v = Ar[off];
            y[c] = (live && c < b) ? v : zero<T>();
            if (c + 1 < b) off += lda;
        }
    }
    LEAF_STAMP(3);
    leaf_solve<T, true, false>(y, LT);
    LEAF_STAMP(4);
    if (live) {
        T* Ar = A + row;
        int64_t off = 0;
        #pragma unroll
        for (int c = 0; c < 64; ++c) {
            if (c < b) Ar[off] = y[c];
            off += lda;
        }
    }
    LEAF_STAMP(5);
}

//------------------------------------------------------------------------------
// Left triangular solve A X = B (NoTrans) with a small triangle (m <= MM,
// MM = 32 or 64), one launch (the LU panel recursion's U12 = L11^{-1} A12 at
// its narrowest levels, on the critical path): tri_solve_cols per 64 columns.
template <typename T, int MM>
__global__ __launch_bounds__(64)
void trsm_small_kernel(char uplo, char diag, int m, int64_t n, const T* A, int64_t lda, T* B, int64_t ldb) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ __attribute__((aligned(16))) T S[MM * kLeafLS];
    __shared__ T X[64 * (MM + 1)];
    const int64_t col0 = (int64_t)blockIdx.x * 64;
    tri_solve_cols<T, MM>(uplo == 'L', diag == 'U', m, A, lda, B + col0 * ldb, ldb, B + col0 * ldb, ldb,
                          (int)min<int64_t>(64, n - col0), S, X);
}

// Round-4 forms (dot-product substitution, triangle in LDS): the default
// (see small_solve_v1: slower alone, faster beside the concurrent trailing GEMM).
template <typename T, int MM>
__global__ __launch_bounds__(64)
void trsm_small_v1_kernel(char uplo, char diag, int m, int64_t n, const T* A, int64_t lda, T* B, int64_t ldb) {
    SLATE_PANEL_WAVE_PRIO();
    // MM = 32 or 64 (m <= MM): the padded triangle, and the workgroup's 64
    // right-hand-side columns staged through LDS so that global loads and
    // stores run along the columns (a lane-per-column access would touch a
    // different cache line in every lane)
    __shared__ T L[MM][MM + 1];
    __shared__ T X[64][MM + 1];
    __shared__ T rd[MM];
    const int lane = threadIdx.x;
    const int64_t col0 = (int64_t)blockIdx.x * 64;
    const int ncol = (int)min<int64_t>(64, n - col0);
    for (int j = 0; j < MM; ++j)
        if (lane < MM)
            L[lane][j] = (lane < m && j < m) ? A[lane + (int64_t)j * lda] : (lane == j ? one<T>() : zero<T>());
    for (int c = 0; c < ncol; ++c)
        if (lane < m) X[c][lane] = B[lane + (col0 + c) * ldb];
    __syncthreads();
    if (lane < MM) rd[lane] = (diag == 'U') ? one<T>() : one<T>() / L[lane][lane];
    __syncthreads();
    const bool live = lane < ncol;
    T x[MM];
    #pragma unroll
    for (int i = 0; i < MM; ++i) x[i] = (live && i < m) ? X[lane][i] : zero<T>();
    if (uplo == 'L') {
        #pragma unroll
        for (int i = 0; i < MM; ++i) {
            T s = x[i];
            #pragma unroll
            for (int l = 0; l < i; ++l) s -= L[i][l] * x[l];
            x[i] = s * rd[i];
        }
    } else {
        #pragma unroll
        for (int i = MM - 1; i >= 0; --i) {
            T s = x[i];
            #pragma unroll
            for (int l = i + 1; l < MM; ++l) s -= L[i][l] * x[l];
            x[i] = s * rd[i];
        }
    }
    if (live) {
        #pragma unroll
        for (int i = 0; i < MM; ++i) X[lane][i] = x[i];
    }
    __syncthreads();
    for (int c = 0; c < ncol; ++c)
        if (lane < m) B[lane + (col0 + c) * ldb] = X[c][lane];
}

template <typename T>
__global__ __launch_bounds__(64)
void trtri_diag_v1_kernel(char uplo, char diag, int64_t n, int nbs,
                       const T* A, int64_t lda, T* W, int64_t ldw, int64_t wrap) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ T L[64][64];
    __shared__ T rd[64];
    const int b = blockIdx.x;
    const int64_t off = (int64_t)b * nbs;
    const int nb = (int)min<int64_t>(nbs, n - off);
    const int lane = threadIdx.x;
    const T* Ab = A + off + off * lda;
    // wrap > 0: W is a stack of wrap x wrap blocks (block t at W + t wrap^2,
    // ld = wrap), each holding the inverse of A's t-th diagonal wrap-block
    T* Wb = wrap > 0 ? W + (off / wrap) * wrap * wrap + (off % wrap) * (1 + ldw) : W + off + off * ldw;
    const bool unit = (diag == 'U');
    const bool lower = (uplo == 'L');
    for (int j = 0; j < 64; ++j)
        L[lane][j] = (lane < nb && j < nb) ? Ab[lane + j * lda] : (lane == j ? one<T>() : zero<T>());
    __syncthreads();
    rd[lane] = unit ? one<T>() : one<T>() / L[lane][lane];
    __syncthreads();
    const int j = lane;
    T x[64];
    if (lower) {
        #pragma unroll
        for (int i = 0; i < 64; ++i) {
            T s = zero<T>();
            #pragma unroll
            for (int l = 0; l < i; ++l) s += L[i][l] * x[l];
            x[i] = (i < j) ? zero<T>() : ((i == j) ? rd[i] : -(s * rd[i]));
        }
    } else {
        #pragma unroll
        for (int i = 63; i >= 0; --i) {
            T s = zero<T>();
            #pragma unroll
            for (int l = i + 1; l < 64; ++l) s += L[i][l] * x[l];
            x[i] = (i > j) ? zero<T>() : ((i == j) ? rd[i] : -(s * rd[i]));
        }
    }
    if (lane < nb) {
        #pragma unroll
        for (int i = 0; i < 64; ++i)
            if (i < nb) Wb[i + (int64_t)j * ldw] = x[i];
    }
}

//------------------------------------------------------------------------------
// Row permutation: for each pair p, row dst[p] of every column receives the
// value of row src[p] (all reads happen before any write within a column).
// One 256-thread workgroup per column strip of COLS columns.
template <typename T, int PER>
__global__ void permute_rows_kernel(int64_t n, T* A, int64_t lda, const int64_t* dst,
                                    const int64_t* src, const int* npairs_ptr, int max_pairs) {
    const int npairs = npairs_ptr ? min(*npairs_ptr, max_pairs) : max_pairs;
    const int64_t j = blockIdx.x;
    if (j >= n) return;
    T* col = A + j * lda;
    for (int base = 0; base < npairs; base += 256 * PER) {
        T v[PER];
        #pragma unroll
        for (int r = 0; r < PER; ++r) {
            int p = base + threadIdx.x + r * 256;
            if (p < npairs) v[r] = col[src[p]];
        }
        __syncthreads();
        #pragma unroll
        for (int r = 0; r < PER; ++r) {
            int p = base + threadIdx.x + r * 256;
            if (p < npairs) col[dst[p]] = v[r];
        }
        __syncthreads();
    }
}

// V = unit-lower part of A (one launch instead of a copy plus a triangle set)
// (diagonal of column j at row j + off)
template <typename T>
__global__ void form_v_kernel(int64_t m, int64_t k, int64_t off, const T* A, int64_t lda, T* V, int64_t ldv) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t j = blockIdx.y;
    if (i >= m) return;
    const int64_t d = j + off;
    V[i + j * ldv] = i < d ? zero<T>() : (i == d ? one<T>() : A[i + j * lda]);
}

// More pairs than one register pass holds (2 * nb > 2048, i.e. nb > 1024):
// every source value of the column is staged in LDS before any write (the
// register kernel's second pass would read rows its first pass overwrote).
template <typename T>
__global__ void permute_rows_lds_kernel(int64_t n, T* A, int64_t lda, const int64_t* dst, const int64_t* src,
                                        const int* npairs_ptr, int max_pairs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char perm_smem[];
    T* v = reinterpret_cast<T*>(perm_smem);
    const int npairs = npairs_ptr ? min(*npairs_ptr, max_pairs) : max_pairs;
    const int64_t j = blockIdx.x;
    if (j >= n) return;
    T* col = A + j * lda;
    for (int p = threadIdx.x; p < npairs; p += blockDim.x) v[p] = col[src[p]];
    __syncthreads();
    for (int p = threadIdx.x; p < npairs; p += blockDim.x) col[dst[p]] = v[p];
}

// Row gather / scatter between a column strip of A and a packed buffer
// (buf is count x n, column-major, ld = count): gather buf(t, :) = A(idx[t], :),
// scatter A(idx[t], :) = buf(t, :).  Used by the distributed row exchange.
template <typename T>
__global__ void rows_pack_kernel(int64_t n, T* A, int64_t lda, const int64_t* idx, int count, T* buf,
                                 int scatter) {
    const int64_t j = blockIdx.y;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count || j >= n) return;
    T* a = A + idx[t] + j * lda;
    T* b = buf + t + j * (int64_t)count;
    if (scatter) *a = *b; else *b = *a;
}

// Sequential interchanges applied to a column strip (LAPACK laswp semantics,
// ipiv 0-based absolute rows), used when the pivot count is tiny.
template <typename T>
__global__ void laswp_kernel(int64_t n, T* A, int64_t lda, int64_t k1, int64_t k2,
                             const int64_t* ipiv, int64_t ipiv_offset) {
    int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= n) return;
    T* col = A + j * lda;
    for (int64_t k = k1; k < k2; ++k) {
        int64_t p = ipiv[k - ipiv_offset];
        if (p != k) { T t = col[k]; col[k] = col[p]; col[p] = t; }
    }
}

}  // namespace

//------------------------------------------------------------------------------
// launchers
template <typename T>
void geset(char uplo, int64_t m, int64_t n, T offdiag, T diag, T* A, int64_t lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(set_kernel<T>, grid2d(m, n), dim3(TX, TY), 0, s, uplo, m, n, offdiag, diag, A, lda);
}

template <typename Ts, typename Td>
void gecopy(char uplo, char trans, int64_t m, int64_t n, const Ts* A, int64_t lda, Td* B, int64_t ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (trans != 'N' && uplo == 'G' && std::is_same<Ts, Td>::value) {
        // B (m x n) = op(A), A is n x m: tile transpose over A's (n x m) index space
        dim3 g((unsigned)((n + 63) / 64), (unsigned)((m + 63) / 64));
        hipLaunchKernelGGL(transpose_kernel<Ts>, g, dim3(64, 4), 0, s, trans == 'C',
                           n, m, A, lda, reinterpret_cast<Ts*>(B), ldb);
        return;
    }
    hipLaunchKernelGGL((copy_kernel<Ts, Td>), grid2d(m, n), dim3(TX, TY), 0, s, uplo, trans, m, n, A, lda, B, ldb);
}

template <typename T>
void geadd(char uplo, int64_t m, int64_t n, T alpha, const T* A, int64_t lda, T beta, T* B, int64_t ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(add_kernel<T>, grid2d(m, n), dim3(TX, TY), 0, s, uplo, m, n, alpha, A, lda, beta, B, ldb);
}

template <typename T>
void gescale(char uplo, int64_t m, int64_t n, real_t<T> mul, T* A, int64_t lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(scale_kernel<T>, grid2d(m, n), dim3(TX, TY), 0, s, uplo, m, n, mul, A, lda);
}

template <typename T>
void real_rowscale(int64_t m, int64_t n, const real_t<T>* A, int64_t lda, const T* sc, T* B, int64_t ldb,
                   hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(real_rowscale_kernel<T>, grid2d(m, n), dim3(TX, TY), 0, s, m, n, A, lda, sc, B, ldb);
}

template <typename T>
void gescale_row_col(int64_t m, int64_t n, const real_t<T>* R, const real_t<T>* C, T* A, int64_t lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(scale_row_col_kernel<T>, grid2d(m, n), dim3(TX, TY), 0, s, m, n, R, C, A, lda);
}

// Small triangular solves: the dot-product kernels (default) or the
// solve-stream ones (SLATE_SMALL_SOLVE=2).  The stream kernels are 2x faster
// alone (trsm_small 64 x 448: 41 -> 22 us, trtri_diag 33 -> 20 us; the
// 32768 x 512 tournament panel 2.88 -> 2.66 ms) but the 1-GPU dgetrf, whose
// panel runs beside the trailing GEMM, measured 55.9 against 59.0-59.1
// TFLOP/s with them (same box, interleaved runs, profiles/r5_small_solve_ab.txt).
// With CUs reserved for the panel queues (the one-process-per-GPU default)
// the panel no longer waits for GEMM slots and the stream kernels win: 2 x 4
// LU model 170.8 / 173.4 -> 174.1 / 177.6 TFLOP/s (profiles/r6_redecide.txt),
// so they are the default there.
inline bool small_solve_v1() {
    static const bool v = [] {
        const char* e = std::getenv("SLATE_SMALL_SOLVE");
        if (e) return std::atoi(e) != 2;
        return slate::device::reserved_cus() == 0;
    }();
    return v;
}

template <typename T>
void trtri_diag(char uplo, char diag, int64_t n, int nbs, const T* A, int64_t lda, T* W, int64_t ldw, hipStream_t s) {
    if (n <= 0) return;
    int nblk = (int)((n + nbs - 1) / nbs);
    if (small_solve_v1())
        hipLaunchKernelGGL(trtri_diag_v1_kernel<T>, dim3(nblk), dim3(64), 0, s, uplo, diag, n, nbs, A, lda, W, ldw,
                           int64_t(0));
    else
        hipLaunchKernelGGL(trtri_diag_kernel<T>, dim3(nblk), dim3(64), 0, s, uplo, diag, n, nbs, A, lda, W, ldw,
                           int64_t(0));
}

template <typename T>
void trtri_diag_stack(char uplo, char diag, int64_t n, int nbs, const T* A, int64_t lda, T* W, int64_t bs, hipStream_t s) {
    if (n <= 0) return;
    int nblk = (int)((n + nbs - 1) / nbs);
    if (small_solve_v1())
        hipLaunchKernelGGL(trtri_diag_v1_kernel<T>, dim3(nblk), dim3(64), 0, s, uplo, diag, n, nbs, A, lda, W, bs, bs);
    else
        hipLaunchKernelGGL(trtri_diag_kernel<T>, dim3(nblk), dim3(64), 0, s, uplo, diag, n, nbs, A, lda, W, bs, bs);
}

template <typename T>
void potrf_small(char uplo, int n, T* A, int64_t lda, int* info, int info_offset, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(potrf_small_kernel<T>, dim3(1), dim3(64), 0, s, uplo, n, A, lda, info, info_offset);
}

template <typename T>
void potrf_inv_small(int n, T* A, int64_t lda, T* W, int64_t ldw, int* info, int info_offset, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(potrf_inv_small_kernel<T>, dim3(1), dim3(64), 0, s, n, A, lda, W, ldw, info, info_offset);
}

template <typename T>
void potrf_leaf(int b, int64_t r, T* A, int64_t lda, int* info, int info_offset, T* W, const T* Wprev, T* Aprev,
                int bprev, hipStream_t s) {
    if (b <= 0) return;
    if (b > 64 || r < 0 || bprev > 64) throw std::invalid_argument("potrf_leaf: b, bprev must be <= 64 and r >= 0");
    if (r > 0 && !W) throw std::invalid_argument("potrf_leaf: r > 0 needs the 64 x 64 staging block W");
    if (Aprev && !Wprev) throw std::invalid_argument("potrf_leaf: Aprev needs Wprev");
    if constexpr (sizeof(T) > 8) {
        // complex<double>: the per-lane rows need 256 VGPRs each; the
        // blocked potrf keeps the inverse-based leaf for it
        throw std::invalid_argument("potrf_leaf: complex<double> is not supported");
    } else {
        const unsigned nblk = 1 + (unsigned)((r + 63) / 64);
        hipLaunchKernelGGL(potrf_leaf_kernel<T>, dim3(nblk), dim3(64), 0, s, b, (int)r, A, lda, info, info_offset, W,
                           Wprev, Aprev, bprev);
    }
}

template <typename T>
void trsm_small(char uplo, char diag, int m, int64_t n, const T* A, int64_t lda, T* B, int64_t ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    const dim3 grid((unsigned)((n + 63) / 64));
    if (small_solve_v1()) {
        if (m <= 32)
            hipLaunchKernelGGL((trsm_small_v1_kernel<T, 32>), grid, dim3(64), 0, s, uplo, diag, m, n, A, lda, B, ldb);
        else
            hipLaunchKernelGGL((trsm_small_v1_kernel<T, 64>), grid, dim3(64), 0, s, uplo, diag, m, n, A, lda, B, ldb);
    } else {
        if (m <= 32)
            hipLaunchKernelGGL((trsm_small_kernel<T, 32>), grid, dim3(64), 0, s, uplo, diag, m, n, A, lda, B, ldb);
        else
            hipLaunchKernelGGL((trsm_small_kernel<T, 64>), grid, dim3(64), 0, s, uplo, diag, m, n, A, lda, B, ldb);
    }
}

template <typename T>
void form_v(int64_t m, int64_t k, int64_t off, const T* A, int64_t lda, T* V, int64_t ldv, hipStream_t s) {
    if (m <= 0 || k <= 0) return;
    hipLaunchKernelGGL(form_v_kernel<T>, dim3((unsigned)((m + 255) / 256), (unsigned)k), dim3(256), 0, s, m, k, off,
                       A, lda, V, ldv);
}

template <typename T>
void permute_rows(int64_t n, T* A, int64_t lda, const int64_t* dst, const int64_t* src,
                  const int* npairs, int max_pairs, hipStream_t s) {
    if (n <= 0 || max_pairs <= 0) return;
    // one register pass: every gather of the column in flight before the
    // barrier (a second pass would read rows the first had overwritten)
    if (max_pairs <= 256 * 8) {
        hipLaunchKernelGGL((permute_rows_kernel<T, 8>), dim3((unsigned)n), dim3(256), 0, s, n, A, lda, dst, src,
                           npairs, max_pairs);
        return;
    }
    // (> 2048 pairs: the LDS-staged kernel measured equal-or-faster than a
    // 16-per-thread register pass, 3306-3334 vs 3344-3352 ms for dgetrf at
    // nb = 2048; SLATE_PERM_LDS=0 selects the register pass)
    static const bool force_lds = [] { const char* e = std::getenv("SLATE_PERM_LDS"); return !e || std::atoi(e); }();
    if (max_pairs <= 256 * 16 && sizeof(T) <= 8 && !force_lds) {
        hipLaunchKernelGGL((permute_rows_kernel<T, 16>), dim3((unsigned)n), dim3(256), 0, s, n, A, lda, dst, src,
                           npairs, max_pairs);
        return;
    }
    const size_t shm = size_t(max_pairs) * sizeof(T);
    if (shm > 65536) throw std::runtime_error("permute_rows: more row pairs than one LDS pass holds");
    hipLaunchKernelGGL(permute_rows_lds_kernel<T>, dim3((unsigned)n), dim3(256), shm, s, n, A, lda, dst, src, npairs,
                       max_pairs);
}

template <typename T>
void rows_pack(int64_t n, T* A, int64_t lda, const int64_t* idx, int count, T* buf, bool scatter, hipStream_t s) {
    if (n <= 0 || count <= 0) return;
    dim3 grid((unsigned)((count + 63) / 64), (unsigned)n);
    hipLaunchKernelGGL(rows_pack_kernel<T>, grid, dim3(64), 0, s, n, A, lda, idx, count, buf, scatter ? 1 : 0);
}

template <typename T>
void laswp(int64_t n, T* A, int64_t lda, int64_t k1, int64_t k2, const int64_t* ipiv, int64_t ipiv_offset, hipStream_t s) {
    if (n <= 0 || k2 <= k1) return;
    hipLaunchKernelGGL(laswp_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, A, lda, k1, k2, ipiv, ipiv_offset);
}

#define SLATE_INST_AUX(T)                                                                                  \
    template void geset<T>(char, int64_t, int64_t, T, T, T*, int64_t, hipStream_t);                       \
    template void geadd<T>(char, int64_t, int64_t, T, const T*, int64_t, T, T*, int64_t, hipStream_t);   \
    template void gescale<T>(char, int64_t, int64_t, real_t<T>, T*, int64_t, hipStream_t);                \
    template void gescale_row_col<T>(int64_t, int64_t, const real_t<T>*, const real_t<T>*, T*, int64_t, hipStream_t); \
    template void real_rowscale<T>(int64_t, int64_t, const real_t<T>*, int64_t, const T*, T*, int64_t, hipStream_t); \
    template void trtri_diag<T>(char, char, int64_t, int, const T*, int64_t, T*, int64_t, hipStream_t);   \
    template void trtri_diag_stack<T>(char, char, int64_t, int, const T*, int64_t, T*, int64_t, hipStream_t); \
    template void potrf_small<T>(char, int, T*, int64_t, int*, int, hipStream_t);                          \
    template void potrf_inv_small<T>(int, T*, int64_t, T*, int64_t, int*, int, hipStream_t);                 \
    template void potrf_leaf<T>(int, int64_t, T*, int64_t, int*, int, T*, const T*, T*, int, hipStream_t);   \
    template void trsm_small<T>(char, char, int, int64_t, const T*, int64_t, T*, int64_t, hipStream_t);     \
    template void permute_rows<T>(int64_t, T*, int64_t, const int64_t*, const int64_t*, const int*, int, hipStream_t); \
    template void form_v<T>(int64_t, int64_t, int64_t, const T*, int64_t, T*, int64_t, hipStream_t);                     \
    template void laswp<T>(int64_t, T*, int64_t, int64_t, int64_t, const int64_t*, int64_t, hipStream_t);  \
    template void rows_pack<T>(int64_t, T*, int64_t, const int64_t*, int, T*, bool, hipStream_t);

SLATE_INST_AUX(float)
SLATE_INST_AUX(double)
SLATE_INST_AUX(cplx<float>)
SLATE_INST_AUX(cplx<double>)

#define SLATE_INST_COPY(Ts, Td) \
    template void gecopy<Ts, Td>(char, char, int64_t, int64_t, const Ts*, int64_t, Td*, int64_t, hipStream_t);
SLATE_INST_COPY(float, float)
SLATE_INST_COPY(double, double)
SLATE_INST_COPY(float, double)
SLATE_INST_COPY(double, float)
SLATE_INST_COPY(cplx<float>, cplx<float>)
SLATE_INST_COPY(cplx<double>, cplx<double>)
SLATE_INST_COPY(cplx<float>, cplx<double>)
SLATE_INST_COPY(cplx<double>, cplx<float>)

}  // namespace dev
}  // namespace slate_amd
