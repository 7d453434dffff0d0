// Complex GEMM for gfx950 (c/z precisions): C = alpha op(A) op(B) + beta C,
// optional triangular store mask (uplo 'L'/'U') for herk/her2k/syrk.
// LDS-tiled 64x64 outputs per 256-thread workgroup, 4x4 per thread, with the
// real and imaginary parts kept in separate accumulators (4 real FMAs per
// complex multiply-add).  The real precisions use the MFMA kernel instead.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

constexpr int CB = 64, CK = 16;

template <typename T>
__device__ inline T ld_op(const T* X, int64_t ld, char trans, int64_t i, int64_t j, int64_t mi, int64_t nj) {
    // element (i, j) of op(X), zero outside [0,mi) x [0,nj)
    if (i >= mi || j >= nj) return zero<T>();
    if (trans == 'N') return X[i + j * ld];
    T v = X[j + i * ld];
    return trans == 'C' ? conj(v) : v;
}

template <typename T>
__global__ __launch_bounds__(256)
void gemm_cplx_kernel(char uplo, char ta, char tb, int64_t m, int64_t n, int64_t k, T alpha,
                      const T* A, int64_t lda, const T* B, int64_t ldb, T beta, T* C, int64_t ldc) {
    using R = real_t<T>;
    __shared__ T As[CK][CB + 1];
    __shared__ T Bs[CK][CB + 1];
    const int64_t m0 = blockIdx.x * (int64_t)CB, n0 = blockIdx.y * (int64_t)CB;
    if (uplo == 'L' && m0 + CB <= n0) return;
    if (uplo == 'U' && n0 + CB <= m0) return;
    const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
    R cr[4][4] = {}, ci[4][4] = {};
    for (int64_t k0 = 0; k0 < k; k0 += CK) {
        for (int e = threadIdx.x; e < CK * CB; e += 256) {
            int kk = e / CB, x = e % CB;
            As[kk][x] = ld_op(A, lda, ta, m0 + x, k0 + kk, m, k);
            Bs[kk][x] = ld_op(B, ldb, tb, k0 + kk, n0 + x, k, n);
        }
        __syncthreads();
        #pragma unroll
        for (int kk = 0; kk < CK; ++kk) {
            T a[4], b[4];
            #pragma unroll
            for (int r = 0; r < 4; ++r) { a[r] = As[kk][tx + 16 * r]; b[r] = Bs[kk][ty + 16 * r]; }
            #pragma unroll
            for (int r = 0; r < 4; ++r)
                #pragma unroll
                for (int c = 0; c < 4; ++c) {
                    cr[r][c] += a[r].re * b[c].re - a[r].im * b[c].im;
                    ci[r][c] += a[r].re * b[c].im + a[r].im * b[c].re;
                }
        }
        __syncthreads();
    }
    bool bz = is_zero(beta);
    #pragma unroll
    for (int r = 0; r < 4; ++r)
        #pragma unroll
        for (int c = 0; c < 4; ++c) {
            int64_t i = m0 + tx + 16 * r, j = n0 + ty + 16 * c;
            if (i >= m || j >= n) continue;
            if (uplo == 'L' && i < j) continue;
            if (uplo == 'U' && i > j) continue;
            T v = alpha * T(cr[r][c], ci[r][c]);
            if (!bz) v += beta * C[i + j * ldc];
            C[i + j * ldc] = v;
        }
}

}  // namespace

template <typename T>
void gemm_cplx(char uplo, char transA, char transB, int64_t m, int64_t n, int64_t k,
               T alpha, const T* A, int64_t lda, const T* B, int64_t ldb,
               T beta, T* C, int64_t ldc, hipStream_t stream) {
    if (m <= 0 || n <= 0) return;
    dim3 grid((unsigned)((m + CB - 1) / CB), (unsigned)((n + CB - 1) / CB));
    hipLaunchKernelGGL(gemm_cplx_kernel<T>, grid, dim3(256), 0, stream, uplo, transA, transB, m, n, k,
                       alpha, A, lda, B, ldb, beta, C, ldc);
}

template void gemm_cplx<cplx<float>>(char, char, char, int64_t, int64_t, int64_t, cplx<float>, const cplx<float>*,
                                     int64_t, const cplx<float>*, int64_t, cplx<float>, cplx<float>*, int64_t, hipStream_t);
template void gemm_cplx<cplx<double>>(char, char, char, int64_t, int64_t, int64_t, cplx<double>, const cplx<double>*,
                                      int64_t, const cplx<double>*, int64_t, cplx<double>, cplx<double>*, int64_t, hipStream_t);

}  // namespace dev
}  // namespace slate_amd
