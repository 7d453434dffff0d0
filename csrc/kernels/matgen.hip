// Device-side test-matrix generation (reference matgen/generate_matrix_ge.cc
// and matgen/random.cc).  Element values are a counter-based hash of
// (global i, global j, seed) -- like the reference's Philox-2x64 keyed
// generator -- so a matrix is identical for every process grid.  Each thread
// computes the global indices of its local element from the block-cyclic map.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

__device__ inline double unit(uint64_t i, uint64_t j, uint64_t seed) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull ^ (j + 0x632BE59BD9B4E019ull) * 0xD1B54A32D192ED03ull
               ^ seed * 0x94D049BB133111EBull;
    return (double)(mix64(x) >> 11) * (1.0 / 9007199254740992.0);
}

// kind: 'r' rands [-1,1), 'u' rand [0,1), 's' symmetric rands + shift*I,
//       'd' rands + shift*I, 'i' identity, 'z' zeros
template <typename T>
__global__ void generate_kernel(char kind, int64_t mloc, int64_t nloc, T* A, int64_t lda,
                                int64_t mb, int p, int rrel, int64_t row0,
                                int64_t nb, int q, int crel, int64_t col0,
                                uint64_t seed, double shift) {
    int64_t il = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (il >= mloc) return;
    int64_t gi = ((il / mb) * p + rrel) * mb + il % mb - row0;
    for (int64_t jl = blockIdx.y; jl < nloc; jl += gridDim.y) {
        int64_t gj = ((jl / nb) * q + crel) * nb + jl % nb - col0;
        uint64_t a = gi, b = gj;
        if (kind == 's' && a > b) { uint64_t t = a; a = b; b = t; }
        double v;
        if (kind == 'i') v = (gi == gj) ? 1.0 : 0.0;
        else if (kind == 'z') v = 0.0;
        else if (kind == 'u') v = unit(a, b, seed);
        else v = 2.0 * unit(a, b, seed) - 1.0;
        if ((kind == 's' || kind == 'd') && gi == gj) v += shift;
        T out;
        if constexpr (is_cplx<T>::value) {
            double w = (kind == 'i' || kind == 'z') ? 0.0 : 2.0 * unit(a, b, seed + 7919) - 1.0;
            if (kind == 's') { if (gi == gj) w = 0.0; else if (gi < gj) w = -w; }
            out = T((real_t<T>)v, (real_t<T>)w);
        } else {
            out = (T)v;
        }
        A[il + jl * lda] = out;
    }
}

}  // namespace

template <typename T>
void generate(char kind, int64_t mloc, int64_t nloc, T* A, int64_t lda, int64_t mb, int p, int rrel, int64_t row0,
              int64_t nb, int q, int crel, int64_t col0, uint64_t seed, double shift, hipStream_t s) {
    if (mloc <= 0 || nloc <= 0) return;
    dim3 grid((unsigned)((mloc + 255) / 256), (unsigned)std::min<int64_t>(nloc, 8192));
    hipLaunchKernelGGL(generate_kernel<T>, grid, dim3(256), 0, s, kind, mloc, nloc, A, lda, mb, p, rrel, row0,
                       nb, q, crel, col0, seed, shift);
}

#define SLATE_INST_GEN(T) \
    template void generate<T>(char, int64_t, int64_t, T*, int64_t, int64_t, int, int, int64_t, int64_t, int, int, int64_t, uint64_t, double, hipStream_t);
SLATE_INST_GEN(float)
SLATE_INST_GEN(double)
SLATE_INST_GEN(cplx<float>)
SLATE_INST_GEN(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
