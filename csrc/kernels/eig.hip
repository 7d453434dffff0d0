// Device helpers of the two-stage eigensolver back-transform (unmtr_hb2st).
//
// The hb2st reflectors of kd consecutive sweeps at one bulge step form a block
// V (2 kd x kd) with H_1 ... H_kd = I - V T V^H.  T^{-1} = striu(V^H V) +
// diag(1 / tau) (the UT-transform identity behind LAPACK larft), so the
// application only needs the Gram matrix V^H V (one GEMM) turned into T^{-1}
// in place by this kernel, and a triangular solve.  A zero reflector (tau = 0,
// v = 0) gets a unit diagonal: its column of V is zero, so it contributes
// nothing.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

template <typename T>
__global__ __launch_bounds__(256) void tinv_from_gram_kernel(int64_t k, T* G, int64_t ldg, const T* tau) {
    for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < k * k; idx += 256 * (int64_t)gridDim.x) {
        const int64_t i = idx % k, j = idx / k;
        if (i > j) G[i + j * ldg] = T();
        else if (i == j) {
            const T t = tau[i];
            G[i + j * ldg] = is_zero(t) ? make_val<T>(1.0) : make_val<T>(1.0) / t;
        }
    }
}

// ---- bdsqr rotations on the device.  Every row of M is independent; one
// thread owns one row and walks the columns once per batch of K QR sweeps
// with a register window of 2K columns: at step tau, sweep s applies its
// rotation at column pair (j, j + 1), j = tau - 2 s.  Sweep s at j only needs
// sweep s - 1 to be done with column j + 1, which happened at step tau - 1,
// so the K rotations of one step touch disjoint pairs and are independent
// (ILP instead of a K-long dependency chain).  Each column is read and
// written once per batch instead of once per sweep.  D holds the rotations in
// step order: D[2 (tau - p0) K + 2 s + {0, 1}] = (c, s) of sweep s at step
// tau (identity where sweep s has no rotation), so a step reads 2K
// consecutive reals (prefetched one step ahead).  [x y] <- [c x - s y,
// s x + c y] on columns [p0, p1).
template <typename T, typename R, int K>
__global__ __launch_bounds__(64) void rot_sweeps_kernel(int64_t rows, T* M, int64_t ld, int64_t p0, int64_t p1,
                                                        const R* D) {
    const int64_t r = blockIdx.x * 64 + threadIdx.x;
    if (r >= rows) return;
    T* row = M + r;
    T w[2 * K];
    #pragma unroll
    for (int i = 0; i < 2 * K; ++i) w[i] = T();
    w[2 * K - 2] = row[p0 * ld];
    w[2 * K - 1] = (p0 + 1 < p1) ? row[(p0 + 1) * ld] : T();
    const int64_t tend = p1 - 2 + 2 * (K - 1);
    R cs[2 * K], nx[2 * K];
    #pragma unroll
    for (int i = 0; i < 2 * K; ++i) cs[i] = D[i];
    for (int64_t tau = p0; tau <= tend; ++tau) {
        const R* Dn = D + 2 * K * (tau + 1 - p0);
        if (tau < tend) {
            #pragma unroll
            for (int i = 0; i < 2 * K; ++i) nx[i] = Dn[i];
        }
        #pragma unroll
        for (int s = 0; s < K; ++s) {
            const R c = cs[2 * s], sn = cs[2 * s + 1];
            const T x = w[2 * K - 2 - 2 * s], y = w[2 * K - 1 - 2 * s];
            w[2 * K - 2 - 2 * s] = x * c - y * sn;
            w[2 * K - 1 - 2 * s] = x * sn + y * c;
        }
        const int64_t cr = tau - 2 * K + 2;
        if (cr >= p0) row[cr * ld] = w[0];
        #pragma unroll
        for (int i = 0; i < 2 * K - 1; ++i) w[i] = w[i + 1];
        const int64_t cn = tau + 2;
        w[2 * K - 1] = (cn < p1) ? row[cn * ld] : T();
        #pragma unroll
        for (int i = 0; i < 2 * K; ++i) cs[i] = nx[i];
    }
    if (p1 - 1 >= p0) row[(p1 - 1) * ld] = w[0];
}

// one rotation on columns (a, b): [x y] <- [x c + y s, y c - x s]
template <typename T, typename R>
__global__ __launch_bounds__(256) void rot_cols_kernel(int64_t rows, T* M, int64_t ld, int64_t a, int64_t b, R c,
                                                       R s) {
    const int64_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const T x = M[r + a * ld], y = M[r + b * ld];
    M[r + a * ld] = x * c + y * s;
    M[r + b * ld] = y * c - x * s;
}

}  // namespace

template <typename T>
void rot_sweeps(int64_t rows, T* M, int64_t ld, int64_t p0, int64_t p1, const rt<T>* D, hipStream_t s) {
    if (rows <= 0 || p1 - p0 < 2) return;
    hipLaunchKernelGGL((rot_sweeps_kernel<T, rt<T>, kRotBatch>), dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, s,
                       rows, M, ld, p0, p1, D);
}

template <typename T>
void rot_cols(int64_t rows, T* M, int64_t ld, int64_t a, int64_t b, rt<T> c, rt<T> sn, hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL((rot_cols_kernel<T, rt<T>>), dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, rows, M,
                       ld, a, b, c, sn);
}

template <typename T>
void tinv_from_gram(int64_t k, T* G, int64_t ldg, const T* tau, hipStream_t s) {
    if (k <= 0) return;
    const unsigned nb = (unsigned)std::min<int64_t>((k * k + 255) / 256, 256);
    hipLaunchKernelGGL(tinv_from_gram_kernel<T>, dim3(nb), dim3(256), 0, s, k, G, ldg, tau);
}

#define SLATE_INST_EIG(T)                                                                                          \
    template void tinv_from_gram<T>(int64_t, T*, int64_t, const T*, hipStream_t);                                 \
    template void rot_sweeps<T>(int64_t, T*, int64_t, int64_t, int64_t, const rt<T>*, hipStream_t);             \
    template void rot_cols<T>(int64_t, T*, int64_t, int64_t, int64_t, rt<T>, rt<T>, hipStream_t);

SLATE_INST_EIG(float)
SLATE_INST_EIG(double)
SLATE_INST_EIG(cplx<float>)
SLATE_INST_EIG(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
