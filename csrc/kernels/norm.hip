// Matrix-norm partial kernels (reference src/cuda/device_{genorm,henorm,
// synorm,trnorm}.cu).  The reference computes per-tile partial norms with one
// thread per row; here one 64-lane wave reduces one column of the local block
// (coalesced along rows) and the row-sum kernel uses one thread per row over
// column chunks (2-D grid) followed by an in-order chunk reduction.
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

// Row sums over one column chunk: grid (row blocks, column chunks), one thread
// per row, consecutive lanes on consecutive rows (coalesced column reads).
// Chunk partials land in part[chunk * m + i] and rowsum_reduce_kernel adds
// them in chunk order, so the result is deterministic.
template <typename T>
__global__ void rownorm_kernel(char uplo, char diag, int64_t m, int64_t n, const T* A, int64_t lda,
                               int64_t gr, int64_t gc, int64_t cols_per_chunk, real_t<T>* part) {
    using R = real_t<T>;
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int64_t j0 = blockIdx.y * cols_per_chunk;
    const int64_t j1 = j0 + cols_per_chunk < n ? j0 + cols_per_chunk : n;
    R v = 0;
    if (uplo == 'G' && diag != 'U') {
        const T* a = A + i + j0 * lda;
        int64_t j = j0;
        R v1 = 0;
        for (; j + 1 < j1; j += 2, a += 2 * lda) { v += absval(a[0]); v1 += absval(a[lda]); }
        if (j < j1) v += absval(a[0]);
        v += v1;
    } else {
        for (int64_t j = j0; j < j1; ++j) {
            if (!included(uplo, gr + i, gc + j)) continue;
            v += (diag == 'U' && gr + i == gc + j) ? R(1) : absval(A[i + j * lda]);
        }
    }
    part[blockIdx.y * m + i] = v;
}

template <typename R>
__global__ void rowsum_reduce_kernel(int64_t m, int64_t nch, const R* part, R* out) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= m) return;
    R v = 0;
    for (int64_t c = 0; c < nch; ++c) v += part[c * m + i];
    out[i] = v;
}

// column chunks for the row-sum kernel: enough workgroups to fill 256 CUs for
// tall-and-wide local blocks, bounded partial storage (<= 64 * m).
inline int64_t row_chunks(int64_t n) {
    int64_t c = (n + 511) / 512;
    return c < 1 ? 1 : (c > 64 ? 64 : c);
}

}  // namespace

template <typename T>
void genorm_partial(char kind, char uplo, char diag, int64_t m, int64_t n, const T* A, int64_t lda,
                    int64_t goff_row, int64_t goff_col, real_t<T>* out, hipStream_t s, real_t<T>* work) {
    if (m <= 0 || n <= 0) return;
    if (kind == 'I') {
        const int64_t nch = work ? row_chunks(n) : 1;
        const int64_t cpc = (n + nch - 1) / nch;
        const unsigned gx = (unsigned)((m + 255) / 256);
        hipLaunchKernelGGL(rownorm_kernel<T>, dim3(gx, (unsigned)nch), dim3(256), 0, s,
                           uplo, diag, m, n, A, lda, goff_row, goff_col, cpc, nch > 1 ? work : out);
        if (nch > 1)
            hipLaunchKernelGGL(rowsum_reduce_kernel<real_t<T>>, dim3(gx), dim3(256), 0, s, m, nch,
                               (const real_t<T>*)work, out);
    } else {
        hipLaunchKernelGGL(colnorm_kernel<T>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s,
                           kind, uplo, diag, m, n, A, lda, goff_row, goff_col, out);
    }
}

int64_t genorm_work_size(char kind, int64_t m, int64_t n) {
    if (kind != 'I' || m <= 0 || n <= 0) return 0;
    int64_t nch = row_chunks(n);
    return nch > 1 ? nch * m : 0;
}

#define SLATE_INST_NORM(T) \
    template void genorm_partial<T>(char, char, char, int64_t, int64_t, const T*, int64_t, int64_t, int64_t, real_t<T>*, hipStream_t, real_t<T>*);
SLATE_INST_NORM(float)
SLATE_INST_NORM(double)
SLATE_INST_NORM(cplx<float>)
SLATE_INST_NORM(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
