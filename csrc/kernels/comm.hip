// Reduction kernel of the in-process (thread) communicator: the buffers of
// all ranks have been copied (peer copies over xGMI / SDMA) into one staging
// array, nbuf slabs of `count` elements `stride` apart; out = op over slabs.
// Memory-bound: 64-wide waves, 4 elements per thread per grid-stride step,
// enough workgroups to cover all 256 CUs.
#include "kernels.hh"
#include "device_common.hh"

namespace slate_amd {
namespace dev {

namespace {

template <typename T, int OP>
__global__ void __launch_bounds__(256) reduce_slabs_kernel(T* __restrict__ out, const T* __restrict__ in, int nbuf,
                                                           int64_t count, int64_t stride) {
    const int64_t step = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < count; i += step) {
        T acc = in[i];
        for (int b = 1; b < nbuf; ++b) {
            const T x = in[i + b * stride];
            if (OP == 0) acc += x;
            else if (OP == 1) acc = x > acc ? x : acc;
            else acc = x < acc ? x : acc;
        }
        out[i] = acc;
    }
}

template <typename T>
void launch(int op, T* out, const T* in, int nbuf, int64_t count, int64_t stride, hipStream_t s) {
    if (count <= 0) return;
    const int threads = 256;
    const int64_t want = (count + threads - 1) / threads;
    const int blocks = int(want < 4096 ? want : 4096);
    if (op == 0) reduce_slabs_kernel<T, 0><<<blocks, threads, 0, s>>>(out, in, nbuf, count, stride);
    else if (op == 1) reduce_slabs_kernel<T, 1><<<blocks, threads, 0, s>>>(out, in, nbuf, count, stride);
    else reduce_slabs_kernel<T, 2><<<blocks, threads, 0, s>>>(out, in, nbuf, count, stride);
}

}  // namespace

void reduce_slabs(char type, int op, void* out, const void* in, int nbuf, int64_t count, int64_t stride,
                  hipStream_t s) {
    switch (type) {
        case 'f': launch(op, static_cast<float*>(out), static_cast<const float*>(in), nbuf, count, stride, s); break;
        case 'd': launch(op, static_cast<double*>(out), static_cast<const double*>(in), nbuf, count, stride, s); break;
        case 'i': launch(op, static_cast<int32_t*>(out), static_cast<const int32_t*>(in), nbuf, count, stride, s); break;
        case 'l': launch(op, static_cast<int64_t*>(out), static_cast<const int64_t*>(in), nbuf, count, stride, s); break;
        case 'b': launch(op, static_cast<int8_t*>(out), static_cast<const int8_t*>(in), nbuf, count, stride, s); break;
        default: break;
    }
}

}  // namespace dev
}  // namespace slate_amd
