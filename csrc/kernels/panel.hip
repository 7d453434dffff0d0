// Panel-factorization kernels for gfx950: LU with partial pivoting and
// Householder QR on tall-skinny column panels, entirely on the device (no
// host round trip per column, no vendor LAPACK).
//
// Reference: the CPU PPLU panel (src/internal/Tile_getrf.hh:162-450: per
// column max search + MPI_Allreduce(MAXLOC), swap, scal, geru, ib-blocked
// trsm/gemm), the vendor getrf in the CALU panel
// (internal_getrf_tntpiv.cc:325) and the vendor geqrf + larft-by-gemm panel
// (internal_geqrf.cc:226-330, Tile_geqrf.hh:67-490).
//
// Structure (per narrow column block, driven from device_blas.cc):
//   LU:  colmax -> [pivot -> update(j) (+partial max of j+1)]*   2 launches/col
//   QR:  [reflect+scale+dots -> update(j) (+partial norm of j+1)]*  2 launches/col
// Reductions across workgroups go through small partial arrays that the next
// (stream-ordered) kernel reduces redundantly, so no grid-wide barrier or
// inter-workgroup hand-off is needed inside a launch.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

constexpr int PT = 256;   // threads per workgroup; one row per thread

template <typename R>
__device__ inline void block_argmax(R& v, int64_t& idx) {
    // wave reduce: max |v|, ties -> smaller index (LAPACK i?amax picks first)
    #pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        R ov = __shfl_xor(v, off, 64);
        int64_t oi = __shfl_xor(idx, off, 64);
        if (ov > v || (ov == v && oi < idx) || (isnan(ov) && !isnan(v))) { v = ov; idx = oi; }
    }
    __shared__ R sv[PT / 64];
    __shared__ int64_t si[PT / 64];
    int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) { sv[w] = v; si[w] = idx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < PT / 64; ++k)
            if (sv[k] > v || (sv[k] == v && si[k] < idx) || (isnan(sv[k]) && !isnan(v))) { v = sv[k]; idx = si[k]; }
    }
}

//------------------------------------------------------------------------------
// LU: partial max of |A[i, c]| over rows i in [r, m)
template <typename T>
__global__ void lu_colmax_kernel(int64_t m, int64_t r, const T* A, int64_t lda, int64_t c,
                                 real_t<T>* pval, int64_t* pidx) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    int64_t i = r + blockIdx.x * (int64_t)PT + threadIdx.x;
    R v = -1; int64_t idx = INT64_MAX;
    if (i < m) { v = abs1(A[i + c * lda]); idx = i; }
    block_argmax(v, idx);
    if (threadIdx.x == 0) { pval[blockIdx.x] = v; pidx[blockIdx.x] = idx; }
}

// LU: reduce partials -> pivot row p for column c (row r); record ipiv,
// swap rows r and p over panel columns [0, ncols), track the permutation.
template <typename T>
__global__ void lu_pivot_kernel(int nparts, const real_t<T>* pval, const int64_t* pidx,
                                int64_t r, int64_t c, T* A, int64_t lda, int64_t ncols,
                                int64_t* ipiv, int64_t ipiv_base, int64_t* perm,
                                int* info, int64_t info_offset, int64_t* piv_out, real_t<T> thresh) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    R v = -1; int64_t idx = INT64_MAX;
    for (int k = threadIdx.x; k < nparts; k += PT) {
        R ov = pval[k]; int64_t oi = pidx[k];
        if (ov > v || (ov == v && oi < idx) || (isnan(ov) && !isnan(v))) { v = ov; idx = oi; }
    }
    block_argmax(v, idx);
    __shared__ int64_t p_sh;
    if (threadIdx.x == 0) {
        int64_t p = (idx == INT64_MAX) ? r : idx;
        // threshold pivoting: keep the diagonal when |a_rc| >= thresh * max
        if (thresh < R(1) && p != r && abs1(A[r + c * lda]) >= thresh * v) p = r;
        p_sh = p;
        ipiv[r] = ipiv_base + p;
        if (piv_out) *piv_out = p;
        if (perm && p != r) { int64_t t = perm[r]; perm[r] = perm[p]; perm[p] = t; }
        if (info && (v == R(0)) && *info == 0) *info = (int)(info_offset + c + 1);
    }
    __syncthreads();
    int64_t p = p_sh;
    if (p != r) {
        for (int64_t j = threadIdx.x; j < ncols; j += PT) {
            T a = A[r + j * lda], b = A[p + j * lda];
            A[r + j * lda] = b; A[p + j * lda] = a;
        }
    }
}

// LU: rows i in (r, m): l = A[i,c]/A[r,c]; A[i,c] = l; A[i, c+1:cend] -= l*A[r, c+1:cend];
// then partial max of the updated column c+1 (if c+1 < cend).
template <typename T>
__global__ void lu_update_kernel(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda,
                                 real_t<T>* pval, int64_t* pidx) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    __shared__ T urow[64];
    const int64_t nc = cend - c - 1;            // columns right of c in the block (<= 63)
    for (int k = threadIdx.x; k < nc; k += PT) urow[k] = A[r + (c + 1 + k) * lda];
    __syncthreads();
    T d = A[r + c * lda];
    T rd = is_zero(d) ? zero<T>() : one<T>() / d;
    int64_t i = r + 1 + blockIdx.x * (int64_t)PT + threadIdx.x;
    R v = -1; int64_t idx = INT64_MAX;
    if (i < m) {
        T l = A[i + c * lda] * rd;
        A[i + c * lda] = l;
        for (int k = 0; k < nc; ++k) {
            T a = A[i + (c + 1 + k) * lda] - l * urow[k];
            A[i + (c + 1 + k) * lda] = a;
            if (k == 0) { v = abs1(a); idx = i; }
        }
    }
    if (nc > 0) {
        block_argmax(v, idx);
        if (threadIdx.x == 0) { pval[blockIdx.x] = v; pidx[blockIdx.x] = idx; }
    }
}

// LU, 2-D parallel column step: grid.x = row blocks over [r, m),
// grid.y = 1 + nc.  y = 0 applies the DEFERRED scaling of column c-1 (its
// multipliers are only finalized here so that no block of step c-1 raced
// with readers of the unscaled column); y = j >= 1 updates column c + j with
// multipliers recomputed on the fly from the unscaled column c, and y = 1 also
// produces the partial pivot search of column c + 1.
template <typename T>
__global__ void lu_update2d_kernel(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda,
                                   real_t<T>* pval, int64_t* pidx, int scale_prev) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    const int j = blockIdx.y;
    const int64_t i = r + blockIdx.x * (int64_t)PT + threadIdx.x;
    if (j == 0) {
        if (scale_prev && i < m) {
            T d = A[(c - 1) + (c - 1) * lda];
            T rd = is_zero(d) ? zero<T>() : one<T>() / d;
            A[i + (c - 1) * lda] = A[i + (c - 1) * lda] * rd;
        }
        return;
    }
    const int64_t cc = c + j;
    T d = A[r + c * lda];
    T rd = is_zero(d) ? zero<T>() : one<T>() / d;
    T u = A[r + cc * lda];
    R v = -1; int64_t idx = INT64_MAX;
    if (i > r && i < m) {
        T l = A[i + c * lda] * rd;
        T a = A[i + cc * lda] - l * u;
        A[i + cc * lda] = a;
        if (j == 1) { v = abs1(a); idx = i; }
    }
    if (j == 1) {
        block_argmax(v, idx);
        if (threadIdx.x == 0) { pval[blockIdx.x] = v; pidx[blockIdx.x] = idx; }
    }
}

// scale rows (c, m) of column c by 1 / A[c, c]
template <typename T>
__global__ void lu_scale_col_kernel(int64_t m, int64_t c, T* A, int64_t lda) {
    SLATE_PANEL_WAVE_PRIO();
    int64_t i = c + 1 + blockIdx.x * (int64_t)PT + threadIdx.x;
    if (i >= m) return;
    T d = A[c + c * lda];
    T rd = is_zero(d) ? zero<T>() : one<T>() / d;
    A[i + c * lda] = A[i + c * lda] * rd;
}

template <typename T>
__global__ void iota_kernel(int64_t n, int64_t* p) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) p[i] = i;
}

// pairs (dst, src) from the tracked permutation: rows [0, k) and pivot rows
template <typename T>
__global__ void perm_pairs_kernel(int64_t k, const int64_t* perm, const int64_t* ipiv_local,
                                  int64_t* dst, int64_t* src) {
    int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t < k) { dst[t] = t; src[t] = perm[t]; }
    else if (t < 2 * k) {
        int64_t r = ipiv_local[t - k];
        dst[t] = r; src[t] = perm[r];
    }
}

//------------------------------------------------------------------------------
// QR.  Column c, diagonal row r.  Partial sums of |A[i,c]|^2 over i in (r, m)
template <typename T>
__global__ void qr_colnorm_kernel(int64_t m, int64_t r, const T* A, int64_t lda, int64_t c,
                                  real_t<T>* psum, T* alpha_out) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    int64_t i = r + 1 + blockIdx.x * (int64_t)PT + threadIdx.x;
    R s = 0;
    if (i < m) { T a = A[i + c * lda]; s = real(a) * real(a) + imag(a) * imag(a); }
    s = wave_sum(s);
    __shared__ R sh[PT / 64];
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        R t = 0;
        for (int k = 0; k < PT / 64; ++k) t += sh[k];
        psum[blockIdx.x] = t;
        if (blockIdx.x == 0 && alpha_out) *alpha_out = A[r + c * lda];
    }
}

// Reflector from (alpha, xnorm^2): beta, tau, scal (LAPACK larfg).
template <typename T>
__device__ inline void make_reflector(T alpha, real_t<T> xnorm2, T& beta_o, T& tau, T& scal) {
    using R = real_t<T>;
    R ar = real(alpha), ai = imag(alpha);
    if (xnorm2 == R(0) && ai == R(0)) { beta_o = alpha; tau = zero<T>(); scal = one<T>(); return; }
    R nrm = sqrt((double)ar * ar + (double)ai * ai + (double)xnorm2);
    R beta = ar >= 0 ? -nrm : nrm;
    if constexpr (is_cplx<T>::value) {
        tau = T((beta - ar) / beta, -ai / beta);
        scal = one<T>() / (alpha - T(beta, 0));
        beta_o = T(beta, 0);
    } else {
        tau = (beta - ar) / beta;
        scal = one<T>() / (alpha - beta);
        beta_o = beta;
    }
}

// QR: every workgroup reduces the norm partials redundantly, forms the
// reflector; scales v = x*scal in its rows (v_r = 1 implicit) and writes
// partial dots w[cc] = sum_i conj(v_i) A[i, cc] for cc in (c, cend).
// Block 0 stores tau and beta (A[r,c]).
template <typename T>
__global__ void qr_reflect_dots_kernel(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda,
                                       int nparts, const real_t<T>* psum, const T* alpha_in,
                                       T* tau_out, T* pdots /* [gridDim.x][nc] */) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    __shared__ R red[PT];
    __shared__ T sh_scal;
    R s = 0;
    for (int k = threadIdx.x; k < nparts; k += PT) s += psum[k];
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        R t = 0;
        for (int k = 0; k < PT; ++k) t += red[k];
        T beta, tau, scal;
        make_reflector(*alpha_in, t, beta, tau, scal);
        sh_scal = scal;
        if (blockIdx.x == 0) { *tau_out = tau; A[r + c * lda] = beta; }
    }
    __syncthreads();
    const T scal = sh_scal;
    const int64_t nc = cend - c - 1;
    // rows of this block: block b covers i in [r + b*PT, r + (b+1)*PT)
    int64_t i = r + blockIdx.x * (int64_t)PT + threadIdx.x;
    T v = zero<T>();
    if (i == r) v = one<T>();
    else if (i < m) { v = A[i + c * lda] * scal; A[i + c * lda] = v; }
    __shared__ T wsum[PT / 64][64];
    for (int k = 0; k < nc; ++k) {
        T prod = (i < m) ? conj(v) * A[i + (c + 1 + k) * lda] : zero<T>();
        // wave reduction (real and imaginary parts)
        R pr = wave_sum(real(prod)), pi_ = wave_sum(imag(prod));
        if ((threadIdx.x & 63) == 0) {
            if constexpr (is_cplx<T>::value) wsum[threadIdx.x >> 6][k] = T(pr, pi_);
            else wsum[threadIdx.x >> 6][k] = pr;
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nc; k += PT) {
        T t = zero<T>();
        for (int w = 0; w < PT / 64; ++w) t += wsum[w][k];
        pdots[(int64_t)blockIdx.x * 64 + k] = t;
    }
}

// QR: A[i, cc] -= v_i * conj(tau) * w[cc] for rows i >= r, cc in (c, cend);
// every block reduces the dot partials redundantly.  Then partial norm of
// the updated column c+1 over rows (r+1, m) and alpha for it.
template <typename T>
__global__ void qr_update_kernel(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda,
                                 int nparts, const T* pdots, const T* tau_in,
                                 real_t<T>* psum_next, T* alpha_next) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    __shared__ T z[64];
    const int64_t nc = cend - c - 1;
    const T ctau = conj(*tau_in);
    for (int k = threadIdx.x; k < nc; k += PT) {
        T t = zero<T>();
        for (int b = 0; b < nparts; ++b) t += pdots[(int64_t)b * 64 + k];
        z[k] = ctau * t;
    }
    __syncthreads();
    int64_t i = r + blockIdx.x * (int64_t)PT + threadIdx.x;
    R s = 0;
    if (i < m) {
        T v = (i == r) ? one<T>() : A[i + c * lda];
        for (int k = 0; k < nc; ++k) {
            T a = A[i + (c + 1 + k) * lda] - v * z[k];
            A[i + (c + 1 + k) * lda] = a;
            if (k == 0) {
                if (i > r + 1) s = real(a) * real(a) + imag(a) * imag(a);
                if (i == r + 1 && alpha_next) *alpha_next = a;
            }
        }
    }
    if (nc > 0 && psum_next) {
        s = wave_sum(s);
        __shared__ R sh[PT / 64];
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            R t = 0;
            for (int k = 0; k < PT / 64; ++k) t += sh[k];
            psum_next[blockIdx.x] = t;
        }
    }
}

//------------------------------------------------------------------------------
// QR, 2-D parallel column step (grid.x = row blocks over [r, m), grid.y = 1+nc).
// Every block reduces the norm partials and forms the reflector redundantly;
// v is recomputed on the fly as x * scal (v_r = 1) so the stored column c is
// scaled only in the NEXT step (y = 0 block), avoiding a race with readers.
template <typename T>
__device__ inline void qr_block_reflector(int nparts, const real_t<T>* psum, const T* alpha_in,
                                          T& beta, T& tau, T& scal) {
    using R = real_t<T>;
    __shared__ R red[PT / 64];
    __shared__ T sh[3];
    R s = 0;
    for (int k = threadIdx.x; k < nparts; k += PT) s += psum[k];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        R t = 0;
        #pragma unroll
        for (int k = 0; k < PT / 64; ++k) t += red[k];
        T b, ta, sc;
        make_reflector(*alpha_in, t, b, ta, sc);
        sh[0] = b; sh[1] = ta; sh[2] = sc;
    }
    __syncthreads();
    beta = sh[0]; tau = sh[1]; scal = sh[2];
}

// Each (row block, column group) workgroup handles QR_CPB trailing columns:
// the reflector (a reduction over the norm partials, done redundantly by every
// workgroup) and the v column are then read once per QR_CPB columns instead
// of once per column.  Still thousands of short workgroups per launch, which
// is what lets the panel slot into the CUs a concurrent trailing GEMM frees
// (one workgroup per 256 rows looping over all columns measured 20% slower
// at n = 65536).
constexpr int QR_CPB = 4;

template <typename T>
__global__ void qr_dots2d_kernel(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda,
                                 int nparts_norm, const real_t<T>* psum, const T* alpha_in,
                                 T* tau_out, T* scal_buf, T* pdots, int scale_prev) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    T beta, tau, scal;
    qr_block_reflector(nparts_norm, psum, alpha_in, beta, tau, scal);
    const int y = blockIdx.y;
    const int64_t i = r + blockIdx.x * (int64_t)PT + threadIdx.x;
    if (y == 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) { tau_out[c] = tau; scal_buf[c] = scal; A[r + c * lda] = beta; }
        if (scale_prev && i < m) {
            T sp = scal_buf[c - 1];
            A[i + (c - 1) * lda] = A[i + (c - 1) * lda] * sp;   // rows >= r are below row c-1
        }
        return;
    }
    const int j0 = 1 + (y - 1) * QR_CPB;                 // first column offset of this group
    const int ncol = (int)min<int64_t>(QR_CPB, cend - c - j0);
    T v = zero<T>();
    if (i < m) v = (i == r) ? one<T>() : A[i + c * lda] * scal;
    __shared__ R wr[QR_CPB][PT / 64], wi[QR_CPB][PT / 64];
    #pragma unroll
    for (int t = 0; t < QR_CPB; ++t) {
        if (t >= ncol) break;
        T prod = (i < m) ? conj(v) * A[i + (c + j0 + t) * lda] : zero<T>();
        R pr = wave_sum(real(prod));
        R pim = 0;
        if constexpr (is_cplx<T>::value) pim = wave_sum(imag(prod));
        if ((threadIdx.x & 63) == 0) { wr[t][threadIdx.x >> 6] = pr; wi[t][threadIdx.x >> 6] = pim; }
    }
    __syncthreads();
    if (threadIdx.x < ncol) {
        const int t = threadIdx.x;
        R a = 0, bi = 0;
        for (int w = 0; w < PT / 64; ++w) { a += wr[t][w]; bi += wi[t][w]; }
        T tt;
        if constexpr (is_cplx<T>::value) tt = T(a, bi); else tt = a;
        pdots[(int64_t)blockIdx.x * 64 + (j0 - 1 + t)] = tt;
    }
}

template <typename T>
__global__ void qr_update2d_kernel(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda,
                                   int nparts, const T* pdots, const T* tau_buf, const T* scal_buf,
                                   real_t<T>* psum_next, T* alpha_next) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    const int j0 = 1 + blockIdx.y * QR_CPB;
    const int ncol = (int)min<int64_t>(QR_CPB, cend - c - j0);
    __shared__ T zsh[QR_CPB];
    {
        // wave t reduces the dot partials of column j0 + t (lane-strided)
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        if (w < ncol) {
            R tr = 0, ti = 0;
            for (int b = lane; b < nparts; b += 64) {
                T t = pdots[(int64_t)b * 64 + (j0 - 1 + w)];
                tr += real(t); ti += imag(t);
            }
            tr = wave_sum(tr);
            if constexpr (is_cplx<T>::value) ti = wave_sum(ti);
            if (lane == 0) {
                T t;
                if constexpr (is_cplx<T>::value) t = T(tr, ti); else t = tr;
                zsh[w] = conj(tau_buf[c]) * t;
            }
        }
    }
    __syncthreads();
    const T scal = scal_buf[c];
    const int64_t i = r + blockIdx.x * (int64_t)PT + threadIdx.x;
    R s = 0;
    if (i < m) {
        const T v = (i == r) ? one<T>() : A[i + c * lda] * scal;
        #pragma unroll
        for (int t = 0; t < QR_CPB; ++t) {
            if (t >= ncol) break;
            const int64_t cc = c + j0 + t;
            T a = A[i + cc * lda] - v * zsh[t];
            A[i + cc * lda] = a;
            if (j0 + t == 1) {
                if (i > r + 1) s = real(a) * real(a) + imag(a) * imag(a);
                if (i == r + 1) *alpha_next = a;
            }
        }
    }
    if (blockIdx.y == 0) {
        s = wave_sum(s);
        __shared__ R sh[PT / 64];
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            R t = 0;
            for (int k = 0; k < PT / 64; ++k) t += sh[k];
            psum_next[blockIdx.x] = t;
        }
    }
}

// scale rows (c, m) of column c by scal_buf[c]
template <typename T>
__global__ void qr_scale_col_kernel(int64_t m, int64_t c, T* A, int64_t lda, const T* scal_buf) {
    SLATE_PANEL_WAVE_PRIO();
    int64_t i = c + 1 + blockIdx.x * (int64_t)PT + threadIdx.x;
    if (i >= m) return;
    A[i + c * lda] = A[i + c * lda] * scal_buf[c];
}

//------------------------------------------------------------------------------
// Tall-skinny inner product with split-K: P[b] = op(A)(k-chunk b)^op * B(k-chunk b)
// C (m x n, small) = alpha * A^H B + beta C, A is K x m, B is K x n (both
// column-major, K long).  Used for V^H V (larft) and V^H C on narrow panels.
template <typename T>
__global__ void tsip_partial_kernel(int64_t K, int m, int n, const T* A, int64_t lda,
                                    const T* B, int64_t ldb, int64_t kchunk, T* part) {
    SLATE_PANEL_WAVE_PRIO();
    // each block: one k-chunk; thread (tx) handles output entries
    const int64_t k0 = blockIdx.x * kchunk, k1 = min(K, k0 + kchunk);
    __shared__ T As[64][33];
    __shared__ T Bs[64][33];
    // outputs handled by this thread: e = tid + t*PT over m*n (m,n <= 32)
    T acc[4] = {zero<T>(), zero<T>(), zero<T>(), zero<T>()};
    for (int64_t kb = k0; kb < k1; kb += 64) {
        int kl = (int)min<int64_t>(64, k1 - kb);
        for (int e = threadIdx.x; e < 64 * 32; e += PT) {
            int kk = e % 64, j = e / 64;
            As[kk][j] = (kk < kl && j < m) ? A[(kb + kk) + j * lda] : zero<T>();
            Bs[kk][j] = (kk < kl && j < n) ? B[(kb + kk) + j * ldb] : zero<T>();
        }
        __syncthreads();
        #pragma unroll
        for (int t = 0; t < 4; ++t) {
            int e = threadIdx.x + t * PT;
            if (e < m * n) {
                int i = e % m, j = e / m;
                T s = acc[t];
                for (int kk = 0; kk < kl; ++kk) s += conj(As[kk][i]) * Bs[kk][j];
                acc[t] = s;
            }
        }
        __syncthreads();
    }
    #pragma unroll
    for (int t = 0; t < 4; ++t) {
        int e = threadIdx.x + t * PT;
        if (e < m * n) part[(int64_t)blockIdx.x * m * n + e] = acc[t];
    }
}

template <typename T>
__global__ void tsip_reduce_kernel(int nparts, int m, int n, const T* part, T alpha, T beta, T* C, int64_t ldc) {
    SLATE_PANEL_WAVE_PRIO();
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m * n) return;
    T s = zero<T>();
    for (int b = 0; b < nparts; ++b) s += part[(int64_t)b * m * n + e];
    int i = e % m, j = e / m;
    T c = is_zero(beta) ? zero<T>() : beta * C[i + (int64_t)j * ldc];
    C[i + (int64_t)j * ldc] = alpha * s + c;
}

// larft recurrence on a k x k block: given S = V^H V (strictly upper part
// used) and tau, form upper-triangular T in place of S (k <= 64, one block).
template <typename T>
__global__ void larft_kernel(int k, const T* tau, T* Tm, int64_t ldt) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ T S[64][65];
    __shared__ T tv[64];
    for (int e = threadIdx.x; e < k * k; e += blockDim.x) {
        int i = e % k, j = e / k;
        S[i][j] = Tm[i + (int64_t)j * ldt];
    }
    for (int e = threadIdx.x; e < k; e += blockDim.x) tv[e] = tau[e];
    __syncthreads();
    // column i: T(0:i, i) = -tau_i * T(0:i,0:i) * S(0:i, i); T(i,i) = tau_i
    for (int i = 0; i < k; ++i) {
        T col = zero<T>();
        int r = threadIdx.x;
        if (r < i) {
            T s = zero<T>();
            for (int l = r; l < i; ++l) s += S[r][l] * S[l][i];   // S(r,l) holds T(r,l) for l < i (already formed)
            col = -tv[i] * s;
        }
        __syncthreads();
        if (r < i) S[r][i] = col;
        if (r == 0) S[i][i] = tv[i];
        __syncthreads();
    }
    for (int e = threadIdx.x; e < k * k; e += blockDim.x) {
        int i = e % k, j = e / k;
        Tm[i + (int64_t)j * ldt] = (i <= j) ? S[i][j] : zero<T>();
    }
}

}  // namespace

//------------------------------------------------------------------------------
template <typename T>
void lu_colmax(int64_t m, int64_t r, const T* A, int64_t lda, int64_t c, real_t<T>* pval, int64_t* pidx,
               int nparts, hipStream_t s) {
    hipLaunchKernelGGL(lu_colmax_kernel<T>, dim3(nparts), dim3(PT), 0, s, m, r, A, lda, c, pval, pidx);
}
template <typename T>
void lu_pivot(int nparts, const real_t<T>* pval, const int64_t* pidx, int64_t r, int64_t c, T* A, int64_t lda,
              int64_t ncols, int64_t* ipiv, int64_t ipiv_base, int64_t* perm, int* info, int64_t info_offset,
              int64_t* piv_out, hipStream_t s, double thresh) {
    hipLaunchKernelGGL(lu_pivot_kernel<T>, dim3(1), dim3(PT), 0, s, nparts, pval, pidx, r, c, A, lda, ncols,
                       ipiv, ipiv_base, perm, info, info_offset, piv_out, real_t<T>(thresh));
}
template <typename T>
void lu_update(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, real_t<T>* pval, int64_t* pidx,
               hipStream_t s) {
    int64_t rows = m - r - 1;
    if (rows <= 0) return;
    int g = (int)((rows + PT - 1) / PT);
    hipLaunchKernelGGL(lu_update_kernel<T>, dim3(g), dim3(PT), 0, s, m, r, c, cend, A, lda, pval, pidx);
}
template <typename T>
void lu_update2d(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, rt<T>* pval, int64_t* pidx,
                 int scale_prev, hipStream_t s) {
    int64_t rows = m - r;
    int64_t nc = cend - c - 1;
    if (rows <= 0) return;
    int g = (int)((rows + PT - 1) / PT);
    hipLaunchKernelGGL(lu_update2d_kernel<T>, dim3(g, (unsigned)(1 + nc)), dim3(PT), 0, s, m, r, c, cend, A, lda,
                       pval, pidx, scale_prev);
}
template <typename T>
void lu_scale_col(int64_t m, int64_t c, T* A, int64_t lda, hipStream_t s) {
    int64_t rows = m - c - 1;
    if (rows <= 0) return;
    hipLaunchKernelGGL(lu_scale_col_kernel<T>, dim3((unsigned)((rows + PT - 1) / PT)), dim3(PT), 0, s, m, c, A, lda);
}
template <typename T>
void qr_dots2d(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, int nparts_norm, const rt<T>* psum,
               const T* alpha_in, T* tau_out, T* scal_buf, T* pdots, int scale_prev, hipStream_t s) {
    int64_t rows = m - r;
    if (rows <= 0) return;
    int g = (int)((rows + PT - 1) / PT);
    int64_t nc = cend - c - 1;
    hipLaunchKernelGGL(qr_dots2d_kernel<T>, dim3(g, (unsigned)(1 + (nc + QR_CPB - 1) / QR_CPB)), dim3(PT), 0, s, m, r,
                       c, cend, A, lda,
                       nparts_norm, psum, alpha_in, tau_out, scal_buf, pdots, scale_prev);
}
template <typename T>
void qr_update2d(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, int nparts, const T* pdots,
                 const T* tau_buf, const T* scal_buf, rt<T>* psum_next, T* alpha_next, hipStream_t s) {
    int64_t rows = m - r;
    int64_t nc = cend - c - 1;
    if (rows <= 0 || nc <= 0) return;
    int g = (int)((rows + PT - 1) / PT);
    hipLaunchKernelGGL(qr_update2d_kernel<T>, dim3(g, (unsigned)((nc + QR_CPB - 1) / QR_CPB)), dim3(PT), 0, s, m, r,
                       c, cend, A, lda,
                       nparts, pdots, tau_buf, scal_buf, psum_next, alpha_next);
}
template <typename T>
void qr_scale_col(int64_t m, int64_t c, T* A, int64_t lda, const T* scal_buf, hipStream_t s) {
    int64_t rows = m - c - 1;
    if (rows <= 0) return;
    hipLaunchKernelGGL(qr_scale_col_kernel<T>, dim3((unsigned)((rows + PT - 1) / PT)), dim3(PT), 0, s, m, c, A, lda,
                       scal_buf);
}

void iota(int64_t n, int64_t* p, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(iota_kernel<int>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, p);
}
void perm_pairs(int64_t k, const int64_t* perm, const int64_t* ipiv_local, int64_t* dst, int64_t* src, hipStream_t s) {
    if (k <= 0) return;
    hipLaunchKernelGGL(perm_pairs_kernel<int>, dim3((unsigned)((2 * k + 255) / 256)), dim3(256), 0, s,
                       k, perm, ipiv_local, dst, src);
}

template <typename T>
void qr_colnorm(int64_t m, int64_t r, const T* A, int64_t lda, int64_t c, real_t<T>* psum, T* alpha_out,
                int nparts, hipStream_t s) {
    hipLaunchKernelGGL(qr_colnorm_kernel<T>, dim3(nparts), dim3(PT), 0, s, m, r, A, lda, c, psum, alpha_out);
}
template <typename T>
void qr_reflect_dots(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, int nparts_norm,
                     const real_t<T>* psum, const T* alpha_in, T* tau_out, T* pdots, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL(qr_reflect_dots_kernel<T>, dim3(nblocks), dim3(PT), 0, s, m, r, c, cend, A, lda,
                       nparts_norm, psum, alpha_in, tau_out, pdots);
}
template <typename T>
void qr_update(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, int nparts, const T* pdots,
               const T* tau_in, real_t<T>* psum_next, T* alpha_next, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL(qr_update_kernel<T>, dim3(nblocks), dim3(PT), 0, s, m, r, c, cend, A, lda, nparts, pdots,
                       tau_in, psum_next, alpha_next);
}
template <typename T>
void tsip(int64_t K, int m, int n, T alpha, const T* A, int64_t lda, const T* B, int64_t ldb, T beta,
          T* C, int64_t ldc, T* work, int64_t work_elems, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    int64_t per = (int64_t)m * n;
    int64_t maxparts = std::max<int64_t>(1, std::min<int64_t>(1024, work_elems / per));
    int64_t kchunk = std::max<int64_t>(256, (K + maxparts - 1) / maxparts);
    kchunk = (kchunk + 63) / 64 * 64;
    int nparts = (int)std::max<int64_t>(1, (K + kchunk - 1) / kchunk);
    hipLaunchKernelGGL(tsip_partial_kernel<T>, dim3(nparts), dim3(PT), 0, s, K, m, n, A, lda, B, ldb, kchunk, work);
    hipLaunchKernelGGL(tsip_reduce_kernel<T>, dim3((unsigned)((per + 255) / 256)), dim3(256), 0, s,
                       nparts, m, n, work, alpha, beta, C, ldc);
}
template <typename T>
void larft_small(int k, const T* tau, T* Tm, int64_t ldt, hipStream_t s) {
    if (k <= 0) return;
    hipLaunchKernelGGL(larft_kernel<T>, dim3(1), dim3(64), 0, s, k, tau, Tm, ldt);
}

#define SLATE_INST_PANEL(T)                                                                                 \
    template void lu_colmax<T>(int64_t, int64_t, const T*, int64_t, int64_t, real_t<T>*, int64_t*, int, hipStream_t); \
    template void lu_pivot<T>(int, const real_t<T>*, const int64_t*, int64_t, int64_t, T*, int64_t, int64_t,  \
                              int64_t*, int64_t, int64_t*, int*, int64_t, int64_t*, hipStream_t, double);     \
    template void lu_update<T>(int64_t, int64_t, int64_t, int64_t, T*, int64_t, real_t<T>*, int64_t*, hipStream_t); \
    template void qr_colnorm<T>(int64_t, int64_t, const T*, int64_t, int64_t, real_t<T>*, T*, int, hipStream_t); \
    template void qr_reflect_dots<T>(int64_t, int64_t, int64_t, int64_t, T*, int64_t, int, const real_t<T>*,  \
                                     const T*, T*, T*, int, hipStream_t);                                     \
    template void qr_update<T>(int64_t, int64_t, int64_t, int64_t, T*, int64_t, int, const T*, const T*,     \
                               real_t<T>*, T*, int, hipStream_t);                                             \
    template void tsip<T>(int64_t, int, int, T, const T*, int64_t, const T*, int64_t, T, T*, int64_t, T*,    \
                          int64_t, hipStream_t);                                                               \
    template void larft_small<T>(int, const T*, T*, int64_t, hipStream_t);                             \
    template void lu_update2d<T>(int64_t, int64_t, int64_t, int64_t, T*, int64_t, rt<T>*, int64_t*, int, hipStream_t); \
    template void lu_scale_col<T>(int64_t, int64_t, T*, int64_t, hipStream_t);                          \
    template void qr_dots2d<T>(int64_t, int64_t, int64_t, int64_t, T*, int64_t, int, const rt<T>*, const T*, T*, T*, T*, int, hipStream_t); \
    template void qr_update2d<T>(int64_t, int64_t, int64_t, int64_t, T*, int64_t, int, const T*, const T*, const T*, rt<T>*, T*, hipStream_t); \
    template void qr_scale_col<T>(int64_t, int64_t, T*, int64_t, const T*, hipStream_t);

SLATE_INST_PANEL(float)
SLATE_INST_PANEL(double)
SLATE_INST_PANEL(cplx<float>)
SLATE_INST_PANEL(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
