// Householder reconstruction for the TSQR panel of distributed geqrf (p > 1).
//
// Reference behaviour: SLATE factors a p > 1 panel as a TSQR tree (local
// geqrf, then ttqrt between pairs of ranks, src/internal/internal_ttqrt.cc:
// 91-124) and keeps the tree's reflectors, so every later application needs
// the tree again (ttmqr, internal_ttmqr.cc).
//
// MI355X design: after the TSQR tree we rebuild the ordinary compact-WY
// factor of the panel (Ballard et al., "Reconstructing Householder vectors
// from Tall-Skinny QR"): with Q (M x kd) the TSQR orthonormal factor,
//     [S; 0] - Q = Y U'           (LU without pivoting, S = diag of unit-modulus
//                                  signs chosen on the fly so |U'(j,j)| >= 1)
//     V = Y,  T = U' S^H Y1^{-H},  R = S R_tsqr.
// The panel then has exactly the (V, T) form of the one-process QR, so the
// trailing update stays a 2-D larfb (one column all-reduce) and unmqr / gels /
// he2hb need no tree.  This file holds the narrow-block kernel of the
// sign-modified LU: one launch per 32 columns, every workgroup's wave 0
// factors the 32 x 32 top block in registers (lane = row, v_readlane
// broadcasts) and inverts U11; the workgroup's 256 rows of L21 = A21 U11^{-1}
// are FMAs against U11^{-1} in LDS.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

constexpr int TW = 32;

__device__ inline float unit_phase(float b) { return b < 0.f ? -1.f : 1.f; }
__device__ inline double unit_phase(double b) { return b < 0.0 ? -1.0 : 1.0; }
template <typename R>
__device__ inline cplx<R> unit_phase(cplx<R> b) {
    R a = absval(b);
    return a == R(0) ? cplx<R>(R(1), R(0)) : cplx<R>(b.re / a, b.im / a);
}

template <typename T>
__global__ __launch_bounds__(256) void lu_sign_narrow_kernel(int64_t m, int64_t r, int nn, T* A, int64_t lda,
                                                             const T* Utop, T* sgn) {
    __shared__ T Uinv[TW * TW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (w == 0) {
        const bool live = lane < nn;
        T a[TW];
        #pragma unroll
        for (int j = 0; j < TW; ++j) a[j] = (live && j < nn) ? Utop[j * TW + lane] : zero<T>();
        T s_mine = one<T>();
        #pragma unroll
        for (int k = 0; k < TW; ++k) {
            if (k < nn) {
                // diagonal: b + s with s = b / |b|  ->  |pivot| = 1 + |b| >= 1
                T b = bcast_lane(a[k], k);
                T s = unit_phase(b);
                T d = b + s;
                if (lane == k) { a[k] = d; s_mine = s; }
                T rd = one<T>() / d;
                T lk = a[k] * rd;
                #pragma unroll
                for (int j = k + 1; j < TW; ++j) {
                    T ukj = bcast_lane(a[j], k);
                    if (lane > k) a[j] -= lk * ukj;
                }
                if (lane > k) a[k] = lk;
            }
        }
        // U11^{-1}: lane j = column j (back substitution)
        T x[TW];
        #pragma unroll
        for (int i = TW - 1; i >= 0; --i) {
            x[i] = zero<T>();
            if (i < nn) {
                T sum = (i == lane) ? one<T>() : zero<T>();
                #pragma unroll
                for (int k = i + 1; k < TW; ++k)
                    if (k < nn) sum -= bcast_lane(a[k], i) * x[k];
                x[i] = sum / bcast_lane(a[i], i);
            }
        }
        if (lane < TW) {
            #pragma unroll
            for (int i = 0; i < TW; ++i) Uinv[i * TW + lane] = x[i];
        }
        if (blockIdx.x == 0 && live) {
            #pragma unroll
            for (int j = 0; j < TW; ++j) if (j < nn) A[r + lane + (r + j) * lda] = a[j];
            sgn[r + lane] = s_mine;
        }
    }
    __syncthreads();
    const int64_t row = r + nn + blockIdx.x * (int64_t)256 + tid;
    if (row < m) {
        T av[TW];
        #pragma unroll
        for (int k = 0; k < TW; ++k) av[k] = k < nn ? A[row + (r + k) * lda] : zero<T>();
        #pragma unroll 1
        for (int j = 0; j < nn; ++j) {
            T sum = zero<T>();
            #pragma unroll
            for (int k = 0; k < TW; ++k) sum += av[k] * Uinv[k * TW + j];
            A[row + (r + j) * lda] = sum;
        }
    }
}

}  // namespace

template <typename T>
void lu_sign_narrow(int64_t m, int64_t r, int nn, T* A, int64_t lda, const T* Utop, T* sgn, hipStream_t s) {
    if (nn <= 0 || r >= m) return;
    const int grid = (int)std::max<int64_t>(1, (m - r - nn + 255) / 256);
    hipLaunchKernelGGL(lu_sign_narrow_kernel<T>, dim3(grid), dim3(256), 0, s, m, r, nn, A, lda, Utop, sgn);
}

#define SLATE_INST_TSQR(T) \
    template void lu_sign_narrow<T>(int64_t, int64_t, int, T*, int64_t, const T*, T*, hipStream_t);

SLATE_INST_TSQR(float)
SLATE_INST_TSQR(double)
SLATE_INST_TSQR(cplx<float>)
SLATE_INST_TSQR(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
