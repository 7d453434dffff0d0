// Butterfly transforms (random butterfly transform, RBT) applied in O(n^2)
// per level instead of as dense GEMMs.
//
// Reference behaviour: src/gerbt.cc + src/internal/internal_gerbt.cc apply
// each 2x2 butterfly block tile by tile (Tile_gerbt.hh), sending tiles between
// the ranks that hold the two halves.
//
// MI355X design: one butterfly level pairs index i with i + h inside each
// block and is a per-index linear combination  x_i <- ca_i x_i + cp_i x_pi.
// The partner rows/columns of a process's local block are collected into one
// partner buffer P (a gather for partners held locally, one grouped exchange
// over the column / row communicator for the rest), then a single fused,
// memory-bound pass  A <- ca .* A + cp .* P  (per-row or per-column real
// coefficients) updates the local block: one read of A and P and one write of
// A per level -- HBM-bound, no MFMA needed, 2^d-fold less traffic than the
// dense product the butterfly would otherwise be.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

// by_rows: out(t, j) = A(idx[t], j)  (t < cnt, j < len), scatter: A(idx[t], j) = out(t, j)
// by cols: out(i, t) = A(i, idx[t])  (i < len, t < cnt)
template <typename T>
__global__ __launch_bounds__(256) void rbt_gather_kernel(int by_rows, int scatter, int64_t cnt, int64_t len,
                                                         const int64_t* idx, T* A, int64_t lda, T* buf,
                                                         int64_t ldb) {
    if (by_rows) {
        // 64 rows x 4 column lanes per block; loop over columns
        const int64_t t = blockIdx.x * 64 + (threadIdx.x & 63);
        if (t >= cnt) return;
        const int64_t r = idx[t];
        for (int64_t j = blockIdx.y * 4 + (threadIdx.x >> 6); j < len; j += 4 * (int64_t)gridDim.y) {
            if (scatter) A[r + j * lda] = buf[t + j * ldb];
            else buf[t + j * ldb] = A[r + j * lda];
        }
    } else {
        // one column per block.y, contiguous rows over threads
        for (int64_t t = blockIdx.y; t < cnt; t += gridDim.y) {
            const int64_t c = idx[t];
            for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < len; i += 256 * (int64_t)gridDim.x) {
                if (scatter) A[i + c * lda] = buf[i + t * ldb];
                else buf[i + t * ldb] = A[i + c * lda];
            }
        }
    }
}

// A(i, j) = ca[r] A(i, j) + cp[r] P(i, j),  r = i (by_rows) or j
template <typename T>
__global__ __launch_bounds__(256) void rbt_combine_kernel(int by_rows, int64_t m, int64_t n, T* A, int64_t lda,
                                                          const T* P, int64_t ldp, const real_t<T>* ca,
                                                          const real_t<T>* cp) {
    const int64_t j = blockIdx.y;
    if (j >= n) return;
    const real_t<T> cj_a = by_rows ? real_t<T>(0) : ca[j], cj_p = by_rows ? real_t<T>(0) : cp[j];
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < m; i += 256 * (int64_t)gridDim.x) {
        const real_t<T> a = by_rows ? ca[i] : cj_a, p = by_rows ? cp[i] : cj_p;
        T x = A[i + j * lda], y = P[i + j * ldp];
        A[i + j * lda] = x * a + y * p;
    }
}

// dst[rdst[a] + cdst[b] ldd] = src[ridx[a] + cidx[b] lds] for a < nr, b < nc
template <typename T>
__global__ __launch_bounds__(256) void gather2d_kernel(int64_t nr, int64_t nc, const T* src, int64_t lds,
                                                       const int64_t* ridx, const int64_t* cidx, T* dst, int64_t ldd,
                                                       const int64_t* rdst, const int64_t* cdst) {
    for (int64_t b = blockIdx.y; b < nc; b += gridDim.y) {
        const int64_t cs = cidx[b], cd = cdst[b];
        for (int64_t a = blockIdx.x * 256 + threadIdx.x; a < nr; a += 256 * (int64_t)gridDim.x)
            dst[rdst[a] + cd * ldd] = src[ridx[a] + cs * lds];
    }
}

inline unsigned grid_cap(int64_t v, int64_t cap) { return (unsigned)std::max<int64_t>(1, std::min(v, cap)); }

}  // namespace

template <typename T>
void gather2d(int64_t nr, int64_t nc, const T* src, int64_t lds, const int64_t* ridx, const int64_t* cidx, T* dst,
              int64_t ldd, const int64_t* rdst, const int64_t* cdst, hipStream_t s) {
    if (nr <= 0 || nc <= 0) return;
    dim3 g(grid_cap((nr + 255) / 256, 64), grid_cap(nc, 65535));
    hipLaunchKernelGGL(gather2d_kernel<T>, g, dim3(256), 0, s, nr, nc, src, lds, ridx, cidx, dst, ldd, rdst, cdst);
}

template <typename T>
void rbt_gather(bool by_rows, bool scatter, int64_t cnt, int64_t len, const int64_t* idx, T* A, int64_t lda, T* buf,
                int64_t ldb, hipStream_t s) {
    if (cnt <= 0 || len <= 0) return;
    dim3 g = by_rows ? dim3(grid_cap((cnt + 63) / 64, 1 << 20), grid_cap((len + 3) / 4, 256))
                     : dim3(grid_cap((len + 255) / 256, 64), grid_cap(cnt, 65535));
    hipLaunchKernelGGL(rbt_gather_kernel<T>, g, dim3(256), 0, s, int(by_rows), int(scatter), cnt, len, idx, A, lda,
                       buf, ldb);
}

template <typename T>
void rbt_combine(bool by_rows, int64_t m, int64_t n, T* A, int64_t lda, const T* P, int64_t ldp, const real_t<T>* ca,
                 const real_t<T>* cp, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    for (int64_t j0 = 0; j0 < n; j0 += 65535) {
        const int64_t nn = std::min<int64_t>(65535, n - j0);
        dim3 g(grid_cap((m + 255) / 256, 16), (unsigned)nn);
        hipLaunchKernelGGL(rbt_combine_kernel<T>, g, dim3(256), 0, s, int(by_rows), m, nn, A + j0 * lda, lda,
                           P + j0 * ldp, ldp, by_rows ? ca : ca + j0, by_rows ? cp : cp + j0);
    }
}

#define SLATE_INST_RBT(T)                                                                                          \
    template void rbt_gather<T>(bool, bool, int64_t, int64_t, const int64_t*, T*, int64_t, T*, int64_t,           \
                                hipStream_t);                                                                      \
    template void rbt_combine<T>(bool, int64_t, int64_t, T*, int64_t, const T*, int64_t, const real_t<T>*,        \
                                 const real_t<T>*, hipStream_t);                                                   \
    template void gather2d<T>(int64_t, int64_t, const T*, int64_t, const int64_t*, const int64_t*, T*, int64_t,     \
                              const int64_t*, const int64_t*, hipStream_t);

SLATE_INST_RBT(float)
SLATE_INST_RBT(double)
SLATE_INST_RBT(cplx<float>)
SLATE_INST_RBT(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
