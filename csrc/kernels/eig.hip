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

}  // namespace

template <typename T>
void tinv_from_gram(int64_t k, T* G, int64_t ldg, const T* tau, hipStream_t s) {
    if (k <= 0) return;
    const unsigned nb = (unsigned)std::min<int64_t>((k * k + 255) / 256, 256);
    hipLaunchKernelGGL(tinv_from_gram_kernel<T>, dim3(nb), dim3(256), 0, s, k, G, ldg, tau);
}

#define SLATE_INST_EIG(T) template void tinv_from_gram<T>(int64_t, T*, int64_t, const T*, hipStream_t);

SLATE_INST_EIG(float)
SLATE_INST_EIG(double)
SLATE_INST_EIG(cplx<float>)
SLATE_INST_EIG(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
