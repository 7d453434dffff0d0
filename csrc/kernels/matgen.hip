// Device-side test-matrix generation (reference matgen/generate_matrix_ge.cc
// and matgen/random.cc).  Element values come from matgen_entry.hh, shared
// with the host path, so a matrix is identical for every process grid and
// target.  Each thread computes the global indices of its local elements from
// the block-cyclic map; columns are strided over grid.y so one launch covers
// any local width.
#include "device_common.hh"
#include "kernels.hh"
#include "matgen_entry.hh"

namespace slate_amd {
namespace dev {

namespace {

struct BcMap {
    int64_t mb, nb;
    int p, q, rrel, crel;
    int64_t rb, cb;      // absolute local row / col of the view block's (0, 0)
    int64_t row0, col0;  // global offset of the view
};

__device__ inline int64_t gl_row(BcMap const& g, int64_t il) {
    int64_t l = g.rb + il;
    return ((l / g.mb) * g.p + g.rrel) * g.mb + l % g.mb - g.row0;
}
__device__ inline int64_t gl_col(BcMap const& g, int64_t jl) {
    int64_t l = g.cb + jl;
    return ((l / g.nb) * g.q + g.crel) * g.nb + l % g.nb - g.col0;
}

template <typename T>
__global__ void generate_kernel(gen::Spec spec, BcMap g, int64_t mloc, int64_t nloc, T* A, int64_t lda) {
    int64_t il = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (il >= mloc) return;
    const int64_t gi = gl_row(g, il);
    for (int64_t jl = blockIdx.y; jl < nloc; jl += gridDim.y) {
        const int64_t gj = gl_col(g, jl);
        double re, im;
        gen::entry(spec, gi, gj, is_cplx<T>::value, re, im);
        if constexpr (is_cplx<T>::value) A[il + jl * lda] = T((real_t<T>)re, (real_t<T>)im);
        else A[il + jl * lda] = (T)re;
    }
}

// Diagonal post-processing on local elements with gi == gj:
// op 'R' drop the imaginary part, op 'S' add shift.
template <typename T>
__global__ void diag_kernel(char op, double shift, BcMap g, int64_t mloc, int64_t nloc, T* A, int64_t lda) {
    int64_t il = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (il >= mloc) return;
    const int64_t gi = gl_row(g, il);
    // the diagonal element of global row gi lives in global column gi
    int64_t gc = gi + g.col0;
    if (gc < 0 || (gc / g.nb) % g.q != g.crel) return;
    int64_t jl = (gc / g.nb / g.q) * g.nb + gc % g.nb - g.cb;
    if (jl < 0 || jl >= nloc) return;
    T& a = A[il + jl * lda];
    if constexpr (is_cplx<T>::value) {
        if (op == 'R') a = T(a.re, (real_t<T>)0);
        else a = T(a.re + (real_t<T>)shift, a.im);
    } else {
        if (op == 'S') a = a + (T)shift;
    }
}

}  // namespace

template <typename T>
void generate(gen::Spec const& spec, int64_t mloc, int64_t nloc, T* A, int64_t lda, int64_t mb, int p, int rrel,
              int64_t rb, int64_t row0, int64_t nb, int q, int crel, int64_t cb, int64_t col0, hipStream_t s) {
    if (mloc <= 0 || nloc <= 0) return;
    BcMap g{mb, nb, p, q, rrel, crel, rb, cb, row0, col0};
    dim3 grid((unsigned)((mloc + 255) / 256), (unsigned)std::min<int64_t>(nloc, 8192));
    hipLaunchKernelGGL(generate_kernel<T>, grid, dim3(256), 0, s, spec, g, mloc, nloc, A, lda);
}

template <typename T>
void gen_diag(char op, double shift, int64_t mloc, int64_t nloc, T* A, int64_t lda, int64_t mb, int p, int rrel,
              int64_t rb, int64_t row0, int64_t nb, int q, int crel, int64_t cb, int64_t col0, hipStream_t s) {
    if (mloc <= 0 || nloc <= 0) return;
    BcMap g{mb, nb, p, q, rrel, crel, rb, cb, row0, col0};
    hipLaunchKernelGGL(diag_kernel<T>, dim3((unsigned)((mloc + 255) / 256)), dim3(256), 0, s, op, shift, g,
                       mloc, nloc, A, lda);
}

#define SLATE_INST_GEN(T)                                                                                      \
    template void generate<T>(gen::Spec const&, int64_t, int64_t, T*, int64_t, int64_t, int, int, int64_t,     \
                              int64_t, int64_t, int, int, int64_t, int64_t, hipStream_t);                      \
    template void gen_diag<T>(char, double, int64_t, int64_t, T*, int64_t, int64_t, int, int, int64_t, int64_t, \
                              int64_t, int, int, int64_t, int64_t, hipStream_t);
SLATE_INST_GEN(float)
SLATE_INST_GEN(double)
SLATE_INST_GEN(cplx<float>)
SLATE_INST_GEN(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
