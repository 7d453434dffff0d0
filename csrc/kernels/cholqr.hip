// Helpers of the CholeskyQR panel (qr.cc TsqrPanel, shifted CholeskyQR3 +
// Householder reconstruction): the Gram-matrix shift of the first pass and
// the orthogonality check of the last one.  One 256-thread workgroup: the
// Gram matrix is nb x nb (<= 1024), the work is a trace and a max.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

template <typename R>
__device__ inline R block_sum(R v, R* sh) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (tid < s) sh[tid] += sh[tid + s];
        __syncthreads();
    }
    R r = sh[0];
    __syncthreads();
    return r;
}

template <typename R>
[[maybe_unused]] __device__ inline R block_max(R v, R* sh) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (tid < s) { R o = sh[tid + s]; sh[tid] = (o > sh[tid] || isnan(o)) ? o : sh[tid]; }
        __syncthreads();
    }
    R r = sh[0];
    __syncthreads();
    return r;
}

template <typename T>
__device__ inline real_t<T> re_of(T x) {
    if constexpr (is_cplx<T>::value) return x.re; else return x;
}

/// G(i, i) += c * trace(G)   (real shift on the diagonal)
template <typename T>
__global__ __launch_bounds__(256) void cholqr_shift_kernel(T* G, int64_t ldg, int n, double c) {
    using R = real_t<T>;
    __shared__ R sh[256];
    R t = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) t += re_of(G[i + i * ldg]);
    const R tr = block_sum(t, sh);
    const R add = R(c) * tr;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if constexpr (is_cplx<T>::value) G[i + i * ldg].re += add; else G[i + i * ldg] += add;
    }
}

/// flag = 1 if the lower triangle of G is not within tol of I (or not
/// finite).  One wave per column (4 per workgroup), so the check costs one
/// pass over nb^2 / 2 entries spread over the chip instead of a single
/// workgroup's loop (which took ~0.9 ms at nb = 512 beside the trailing GEMM).
/// The flag is cleared by the launcher; only failing lanes store 1.
template <typename T>
__global__ __launch_bounds__(256) void cholqr_check_kernel(const T* G, int64_t ldg, int n, double* ssq) {
    // ||G - I||_F^2 from the lower triangle (off-diagonal terms twice); a
    // wave per column, one f64 atomic add per wave.  NaN / Inf propagate.
    using R = real_t<T>;
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (j >= n) return;
    double acc = 0;
    for (int i = j + lane; i < n; i += 64) {
        T g = G[i + int64_t(j) * ldg];
        double d2;
        if constexpr (is_cplx<T>::value) {
            const double re = double(g.re) - (i == j ? 1.0 : 0.0), im = double(g.im);
            d2 = re * re + im * im;
        } else {
            const double d = double(g) - (i == j ? 1.0 : 0.0);
            d2 = d * d;
        }
        acc += (i == j ? 1.0 : 2.0) * d2;
    }
    acc = wave_sum(acc);
    if (lane == 0) atomicAdd(ssq, acc);
}

__global__ void cholqr_verdict_kernel(const double* ssq, double tol, int* flag) {
    *flag = (*ssq <= tol * tol) ? 0 : 1;   // NaN fails
}

}  // namespace

template <typename T>
void cholqr_shift(T* G, int64_t ldg, int n, double c, hipStream_t s) {
    if (n <= 0) return;
    cholqr_shift_kernel<T><<<1, 256, 0, s>>>(G, ldg, n, c);
}

template <typename T>
void cholqr_check(const T* G, int64_t ldg, int n, double tol, int* flag, double* ssq, hipStream_t s) {
    (void)hipMemsetAsync(ssq, 0, sizeof(double), s);
    if (n > 0) cholqr_check_kernel<T><<<(n + 3) / 4, 256, 0, s>>>(G, ldg, n, ssq);
    cholqr_verdict_kernel<<<1, 1, 0, s>>>(ssq, tol, flag);
}

#define SLATE_INST_CHOLQR(T)                                                            \
    template void cholqr_shift<T>(T*, int64_t, int, double, hipStream_t);              \
    template void cholqr_check<T>(const T*, int64_t, int, double, int*, double*, hipStream_t);

SLATE_INST_CHOLQR(float)
SLATE_INST_CHOLQR(double)
SLATE_INST_CHOLQR(cplx<float>)
SLATE_INST_CHOLQR(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
