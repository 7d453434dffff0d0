// Skinny products and the batched diagonal-block inverse behind the
// few-right-hand-side triangular solve (gfx950).
//
// Iterative refinement (gesv_mixed / posv_mixed, reference src/gesv_mixed.cc
// and src/gesv_mixed_gmres.cc) spends its iterations in  r = b - A x  and in
// getrs / potrs with 1..16 right-hand sides.  On the MFMA GEMM those are
// 128-column tiles with one live column, and the blocked trsm re-inverted every
// diagonal block with ~20 small dependent launches: ~4,000 launches and
// ~150 ms per refinement step at n = 65536.  Here:
//
//   gemv_n   y = alpha A x + beta y,   A m x k column-major (M-contiguous):
//            a 2-D grid of (256-row block) x (K chunk) workgroups, one row per
//            lane, 4 columns in flight per lane; x is wave-uniform (scalar
//            loads).  With more than one K chunk the chunk sums go to a
//            partial buffer reduced in chunk order (deterministic).
//   gemv_t   y = alpha op(A) x + beta y,  op = T / C, A k x m: one wave per
//            output row (a contiguous column of A), 16-byte loads along K,
//            DPP wave reduction.  K-chunked the same way for short outputs.
//   trtri    all full BS x BS diagonal blocks of a triangle inverted at once
//            into a stack (block t at W + t BS^2, ld BS): one 64 x 64 diagonal
//            launch over every block, then each doubling level as strided
//            batched MFMA GEMMs (the batch runs over the blocks).
#include "device_common.hh"
#include "kernels.hh"

#include <algorithm>

namespace slate_amd {
namespace dev {

namespace {

constexpr int GV_THREADS = 256;
constexpr int GV_MAXR = 16;   // right-hand sides per launch

template <typename T, bool CONJ>
__device__ inline T cj(T v) {
    if constexpr (CONJ) return conj(v);
    else return v;
}

// ---- y (or partial) = sum over this chunk of A(:, l) x(l, :)
template <typename T, int NR>
__global__ void __launch_bounds__(GV_THREADS)
gemv_n_kernel(int64_t m, int64_t k, int64_t kc, int nr, T alpha, const T* __restrict__ A, int64_t lda,
              const T* __restrict__ X, int64_t ldx, T beta, T* __restrict__ Y, int64_t ldy,
              T* __restrict__ P) {
    const int64_t i = blockIdx.x * (int64_t)GV_THREADS + threadIdx.x;
    const int64_t l0 = blockIdx.y * kc;
    const int64_t l1 = min(k, l0 + kc);
    T acc[NR];
    #pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = zero<T>();
    if (i < m) {
        const T* a = A + i;
        int64_t l = l0;
        for (; l + 4 <= l1; l += 4) {
            // four independent column loads in flight per lane
            T a0 = a[(l + 0) * lda], a1 = a[(l + 1) * lda], a2 = a[(l + 2) * lda], a3 = a[(l + 3) * lda];
            #pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (r >= nr) break;
                const T* x = X + l + r * ldx;
                acc[r] += a0 * x[0];
                acc[r] += a1 * x[1];
                acc[r] += a2 * x[2];
                acc[r] += a3 * x[3];
            }
        }
        for (; l < l1; ++l) {
            T av = a[l * lda];
            #pragma unroll
            for (int r = 0; r < NR; ++r) if (r < nr) acc[r] += av * X[l + r * ldx];
        }
        if (P) {
            T* p = P + (int64_t)blockIdx.y * m * nr + i;
            #pragma unroll
            for (int r = 0; r < NR; ++r) if (r < nr) p[r * m] = acc[r];
        } else {
            #pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (r >= nr) break;
                T* y = Y + i + r * ldy;
                *y = is_zero(beta) ? alpha * acc[r] : alpha * acc[r] + beta * (*y);
            }
        }
    }
}

// ---- one wave per output row i: dot of A(:, i) (length k, contiguous) with x
template <typename T, int NR, bool CONJ>
__global__ void __launch_bounds__(GV_THREADS)
gemv_t_kernel(int64_t m, int64_t k, int64_t kc, int nr, T alpha, const T* __restrict__ A, int64_t lda,
              const T* __restrict__ X, int64_t ldx, T beta, T* __restrict__ Y, int64_t ldy,
              T* __restrict__ P) {
    const int lane = threadIdx.x & 63;
    const int64_t i = blockIdx.x * (int64_t)(GV_THREADS / 64) + (threadIdx.x >> 6);
    const int64_t l0 = blockIdx.y * kc;
    const int64_t l1 = min(k, l0 + kc);
    T acc[NR];
    #pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = zero<T>();
    if (i < m) {   // wave-uniform
        const T* a = A + i * lda;
        int64_t l = l0 + lane;
        for (; l + 64 < l1; l += 128) {
            T a0 = cj<T, CONJ>(a[l]), a1 = cj<T, CONJ>(a[l + 64]);
            #pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (r >= nr) break;
                acc[r] += a0 * X[l + r * ldx];
                acc[r] += a1 * X[l + 64 + r * ldx];
            }
        }
        for (; l < l1; l += 64) {
            T av = cj<T, CONJ>(a[l]);
            #pragma unroll
            for (int r = 0; r < NR; ++r) if (r < nr) acc[r] += av * X[l + r * ldx];
        }
        #pragma unroll
        for (int r = 0; r < NR; ++r) {
            if constexpr (is_cplx<T>::value) {
                using R = real_t<T>;
                R re = wave_reduce(acc[r].re, [](R u, R v) { return u + v; });
                R im = wave_reduce(acc[r].im, [](R u, R v) { return u + v; });
                acc[r] = T(re, im);
            } else {
                acc[r] = wave_reduce(acc[r], [](T u, T v) { return u + v; });
            }
        }
        if (lane == 0) {
            if (P) {
                T* p = P + (int64_t)blockIdx.y * m * nr + i;
                #pragma unroll
                for (int r = 0; r < NR; ++r) if (r < nr) p[r * m] = acc[r];
            } else {
                #pragma unroll
                for (int r = 0; r < NR; ++r) {
                    if (r >= nr) break;
                    T* y = Y + i + r * ldy;
                    *y = is_zero(beta) ? alpha * acc[r] : alpha * acc[r] + beta * (*y);
                }
            }
        }
    }
}

// y(:, r) = alpha sum_c P[c](:, r) + beta y(:, r), chunks summed in order
template <typename T>
__global__ void gemv_reduce_kernel(int64_t m, int nr, int chunks, const T* __restrict__ P, T alpha, T beta,
                                   T* __restrict__ Y, int64_t ldy) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    if (i >= m) return;
    const int64_t stride = m * nr;
    const T* p = P + i + r * m;
    T s0 = zero<T>(), s1 = zero<T>();
    int c = 0;
    for (; c + 2 <= chunks; c += 2) { s0 += p[c * stride]; s1 += p[(c + 1) * stride]; }
    if (c < chunks) s0 += p[c * stride];
    T s = s0 + s1;
    T* y = Y + i + r * ldy;
    *y = is_zero(beta) ? alpha * s : alpha * s + beta * (*y);
}

template <typename T, int NR>
void gemv_n_launch(int64_t m, int64_t k, int nr, T alpha, const T* A, int64_t lda, const T* X, int64_t ldx, T beta,
                   T* Y, int64_t ldy, T* P, int chunks, hipStream_t s) {
    const int64_t kc = (k + chunks - 1) / chunks;
    dim3 grid((unsigned)((m + GV_THREADS - 1) / GV_THREADS), (unsigned)chunks);
    hipLaunchKernelGGL((gemv_n_kernel<T, NR>), grid, dim3(GV_THREADS), 0, s, m, k, kc, nr, alpha, A, lda, X, ldx,
                       beta, Y, ldy, chunks > 1 ? P : nullptr);
}

template <typename T, int NR, bool CONJ>
void gemv_t_launch(int64_t m, int64_t k, int nr, T alpha, const T* A, int64_t lda, const T* X, int64_t ldx, T beta,
                   T* Y, int64_t ldy, T* P, int chunks, hipStream_t s) {
    const int64_t kc = ((k + chunks - 1) / chunks + 63) / 64 * 64;
    dim3 grid((unsigned)((m + GV_THREADS / 64 - 1) / (GV_THREADS / 64)), (unsigned)chunks);
    hipLaunchKernelGGL((gemv_t_kernel<T, NR, CONJ>), grid, dim3(GV_THREADS), 0, s, m, k, kc, nr, alpha, A, lda, X,
                       ldx, beta, Y, ldy, chunks > 1 ? P : nullptr);
}

}  // namespace

// About 2048 workgroups in flight (8 per CU) unless the rows alone give that;
// chunks of at least 256 columns for the transposed form (a wave per row),
// 32 for the row-per-lane form: the few-right-hand-side triangular solves of
// mixed-precision refinement run it on tall m x 256 blocks (m = 32768: 128
// workgroups walking 256 columns each, ~0.9 TB/s), where 8 column chunks
// give 1024 workgroups.
int gemv_chunks(char trans, int64_t m, int64_t k) {
    const int64_t row_blocks = trans == 'N' ? (m + GV_THREADS - 1) / GV_THREADS : (m + 3) / 4;
    int64_t want = (2048 + row_blocks - 1) / row_blocks;
    want = std::min<int64_t>(want, std::max<int64_t>(1, k / (trans == 'N' ? 32 : 256)));
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, 64));
}

template <typename T>
void gemv(char trans, int64_t m, int64_t k, int nr, T alpha, const T* A, int64_t lda, const T* X, int64_t ldx,
          T beta, T* Y, int64_t ldy, T* P, int chunks, hipStream_t s) {
    if (m <= 0 || nr <= 0) return;
    if (k <= 0) { geadd<T>('G', m, nr, zero<T>(), Y, ldy, beta, Y, ldy, s); return; }
    for (int r0 = 0; r0 < nr; r0 += GV_MAXR) {
        const int nn = std::min(GV_MAXR, nr - r0);
        const T* Xr = X + r0 * ldx;
        T* Yr = Y + r0 * ldy;
#define SLATE_GV_CASE(NR)                                                                                 \
        case NR:                                                                                          \
            if (trans == 'N') gemv_n_launch<T, NR>(m, k, nn, alpha, A, lda, Xr, ldx, beta, Yr, ldy, P, chunks, s); \
            else if (trans == 'C' && is_cplx<T>::value)                                                   \
                gemv_t_launch<T, NR, true>(m, k, nn, alpha, A, lda, Xr, ldx, beta, Yr, ldy, P, chunks, s);    \
            else gemv_t_launch<T, NR, false>(m, k, nn, alpha, A, lda, Xr, ldx, beta, Yr, ldy, P, chunks, s);  \
            break;
        switch (nn <= 1 ? 1 : nn <= 2 ? 2 : nn <= 4 ? 4 : nn <= 8 ? 8 : 16) {
            SLATE_GV_CASE(1)
            SLATE_GV_CASE(2)
            SLATE_GV_CASE(4)
            SLATE_GV_CASE(8)
            SLATE_GV_CASE(16)
        }
#undef SLATE_GV_CASE
        if (chunks > 1) {
            dim3 grid((unsigned)((m + 255) / 256), (unsigned)nn);
            hipLaunchKernelGGL(gemv_reduce_kernel<T>, grid, dim3(256), 0, s, m, nn, chunks, P, alpha, beta, Yr, ldy);
        }
    }
}

//------------------------------------------------------------------------------
// Batched inverse of the nblk full BS x BS diagonal blocks of a triangle:
// block t = A(t BS : +BS, t BS : +BS) -> W + t BS^2 (ld BS).  work holds
// nblk * BS^2 / 2 scalars.
template <typename T>
void trtri_blocks(char uplo, char diag, int64_t BS, int64_t nblk, const T* A, int64_t lda, T* W, T* work,
                  hipStream_t s) {
    if (nblk <= 0) return;
    constexpr int NBS = 64;
    geset<T>('G', BS, BS * nblk, zero<T>(), zero<T>(), W, BS, s);
    trtri_diag_stack<T>(uplo, diag, BS * nblk, NBS, A, lda, W, BS, s);
    const int64_t sA = BS * (lda + 1), sW = BS * BS;
    for (int64_t sz = NBS; sz < BS; sz *= 2) {
        for (int64_t p = 0; p + sz < BS; p += 2 * sz) {
            const int64_t s2 = std::min(sz, BS - p - sz);
            T* X11 = W + p + p * BS;
            T* X22 = W + (p + sz) + (p + sz) * BS;
            if (uplo == 'L') {
                // X21 = -X22 A21 X11,  A21 = A(p+sz : +s2, p : +sz)
                T* X21 = W + (p + sz) + p * BS;
                const T* A21 = A + (p + sz) + p * lda;
                gemm_real<T>('N', 'N', s2, sz, sz, one<T>(), A21, lda, sA, X11, BS, sW, zero<T>(), work, s2, s2 * sz,
                             nblk, s);
                gemm_real<T>('N', 'N', s2, sz, s2, make_val<T>(-1.0), X22, BS, sW, work, s2, s2 * sz, zero<T>(), X21,
                             BS, sW, nblk, s);
            } else {
                // X12 = -X11 A12 X22,  A12 = A(p : +sz, p+sz : +s2)
                T* X12 = W + p + (p + sz) * BS;
                const T* A12 = A + p + (p + sz) * lda;
                gemm_real<T>('N', 'N', sz, s2, s2, one<T>(), A12, lda, sA, X22, BS, sW, zero<T>(), work, sz, sz * s2,
                             nblk, s);
                gemm_real<T>('N', 'N', sz, s2, sz, make_val<T>(-1.0), X11, BS, sW, work, sz, sz * s2, zero<T>(), X12,
                             BS, sW, nblk, s);
            }
        }
    }
}

#define SLATE_INST_SKINNY(T)                                                                                    \
    template void gemv<T>(char, int64_t, int64_t, int, T, const T*, int64_t, const T*, int64_t, T, T*, int64_t,  \
                          T*, int, hipStream_t);
SLATE_INST_SKINNY(float)
SLATE_INST_SKINNY(double)
SLATE_INST_SKINNY(cplx<float>)
SLATE_INST_SKINNY(cplx<double>)
template void trtri_blocks<float>(char, char, int64_t, int64_t, const float*, int64_t, float*, float*, hipStream_t);
template void trtri_blocks<double>(char, char, int64_t, int64_t, const double*, int64_t, double*, double*, hipStream_t);

}  // namespace dev
}  // namespace slate_amd
