// Matrix-norm partial kernels (reference src/cuda/device_{genorm,henorm,
// synorm,trnorm}.cu).  The reference computes per-tile partial norms with one
// thread per row; here one 64-lane wave reduces one column of the local block
// (coalesced along rows) and the row-sum kernel uses one thread per row.
// Results are per-column (or per-row) values; drivers finish the reduction
// on the host and across ranks (allreduce), as the reference does.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

// include element (gi, gj)? with uplo 'G','L','U' on global indices
__device__ inline bool included(char uplo, int64_t gi, int64_t gj) {
    return uplo == 'G' || (uplo == 'L' ? gi >= gj : gi <= gj);
}

template <typename T>
__global__ void colnorm_kernel(char kind, char uplo, char diag, int64_t m, int64_t n, const T* A, int64_t lda,
                               int64_t gr, int64_t gc, real_t<T>* out) {
    using R = real_t<T>;
    const int lane = threadIdx.x & 63;
    const int64_t j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= n) return;
    const T* col = A + j * lda;
    if (kind == 'F') {
        // two-pass scaled sum of squares: max, then sum (|x|/max)^2
        R mx = 0;
        for (int64_t i = lane; i < m; i += 64) {
            if (!included(uplo, gr + i, gc + j)) continue;
            R a = (diag == 'U' && gr + i == gc + j) ? R(1) : absval(col[i]);
            mx = max_nan(mx, a);
        }
        mx = wave_max_nan(mx);
        R s = 0;
        if (mx > 0 && !isinf(mx)) {
            for (int64_t i = lane; i < m; i += 64) {
                if (!included(uplo, gr + i, gc + j)) continue;
                R a = (diag == 'U' && gr + i == gc + j) ? R(1) : absval(col[i]);
                R t = a / mx;
                s += t * t;
            }
            s = wave_sum(s);
        }
        if (lane == 0) { out[2 * j] = mx; out[2 * j + 1] = (mx > 0 && !isinf(mx)) ? s : (isinf(mx) ? R(1) : R(0)); }
        return;
    }
    R v = 0;
    for (int64_t i = lane; i < m; i += 64) {
        if (!included(uplo, gr + i, gc + j)) continue;
        R a = (diag == 'U' && gr + i == gc + j) ? R(1) : absval(col[i]);
        if (kind == 'M') v = max_nan(v, a);
        else v += a;
    }
    v = (kind == 'M') ? wave_max_nan(v) : wave_sum(v);
    if (lane == 0) out[j] = v;
}

template <typename T>
__global__ void rownorm_kernel(char uplo, char diag, int64_t m, int64_t n, const T* A, int64_t lda,
                               int64_t gr, int64_t gc, real_t<T>* out) {
    using R = real_t<T>;
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= m) return;
    R v = 0;
    for (int64_t j = 0; j < n; ++j) {
        if (!included(uplo, gr + i, gc + j)) continue;
        v += (diag == 'U' && gr + i == gc + j) ? R(1) : absval(A[i + j * lda]);
    }
    out[i] = v;
}

}  // namespace

template <typename T>
void genorm_partial(char kind, char uplo, char diag, int64_t m, int64_t n, const T* A, int64_t lda,
                    int64_t goff_row, int64_t goff_col, real_t<T>* out, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (kind == 'I') {
        hipLaunchKernelGGL(rownorm_kernel<T>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s,
                           uplo, diag, m, n, A, lda, goff_row, goff_col, out);
    } else {
        hipLaunchKernelGGL(colnorm_kernel<T>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s,
                           kind, uplo, diag, m, n, A, lda, goff_row, goff_col, out);
    }
}

#define SLATE_INST_NORM(T) \
    template void genorm_partial<T>(char, char, char, int64_t, int64_t, const T*, int64_t, int64_t, int64_t, real_t<T>*, hipStream_t);
SLATE_INST_NORM(float)
SLATE_INST_NORM(double)
SLATE_INST_NORM(cplx<float>)
SLATE_INST_NORM(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
