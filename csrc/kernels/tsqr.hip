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
#include "leaf_common.hh"

#include <stdexcept>

// the many-workgroup tree kernels (qr_node / qr_node_q) may opt out of the
// panel wave priority (A/B builds: SLATE_QR_NODE_PRIO=0)
#ifndef SLATE_QR_NODE_PRIO
#define SLATE_QR_NODE_PRIO 1
#endif

namespace slate_amd {
namespace dev {

namespace {

constexpr int TW = 32;

__device__ inline float unit_phase(float b) { return b < 0.f ? -1.f : 1.f; }
__device__ inline double unit_phase(double b) { return b < 0.0 ? -1.0 : 1.0; }
// complex: a real +-1 from the real part, so S R keeps R's diagonal real with
// LAPACK's sign (beta = -sign(Re alpha) * norm) and |pivot| >= 1 + |Re b|
template <typename R>
__device__ inline cplx<R> unit_phase(cplx<R> b) { return cplx<R>(b.re < R(0) ? R(-1) : R(1), R(0)); }

__device__ inline double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}
__device__ inline float rcp_nr(float d) { return 1.0f / d; }
template <typename R>
__device__ inline cplx<R> rcp_nr(cplx<R> d) { return one<cplx<R>>() / d; }

template <typename T>
__global__ __launch_bounds__(256) void lu_sign_narrow_kernel(int64_t m, int64_t r, int nn, const T* Ain,
                                                             int64_t ldi, T* Aout, int64_t ldo, const T* Utop,
                                                             int64_t ldu, T in_scale, T* top, int64_t ldt, T* sgn) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ T Uinv[TW * TW];
    __shared__ T Us[TW][TW + 1];
    __shared__ T Rd[TW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (w == 0) {
        const bool live = lane < nn;
        T a[TW];
        #pragma unroll
        for (int j = 0; j < TW; ++j) a[j] = (live && j < nn) ? in_scale * Utop[lane + j * ldu] : zero<T>();
        T s_mine = one<T>();
        #pragma unroll
        for (int k = 0; k < TW; ++k) {
            if (k < nn) {
                // diagonal: b + s with s = b / |b|  ->  |pivot| = 1 + |b| >= 1
                T b = bcast_lane(a[k], k);
                T s = unit_phase(b);
                T d = b + s;
                if (lane == k) { a[k] = d; s_mine = s; }
                T rd = rcp_nr(d);
                T lk = a[k] * rd;
                #pragma unroll
                for (int j = k + 1; j < TW; ++j) {
                    T ukj = bcast_lane(a[j], k);
                    if (lane > k) a[j] -= lk * ukj;
                }
                if (lane > k) a[k] = lk;
            }
        }
        // U11^{-1}, lane j = column j, axpy-form back substitution against
        // U's columns in LDS (independent FMAs per step)
        if (lane < TW) {
            T dg = zero<T>();
            #pragma unroll
            for (int j = 0; j < TW; ++j) {
                Us[lane][j] = a[j];
                if (j == lane) dg = a[j];
            }
            Rd[lane] = live ? rcp_nr(dg) : zero<T>();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        T x[TW];
        #pragma unroll
        for (int i = 0; i < TW; ++i) x[i] = (i == lane && live) ? one<T>() : zero<T>();
        #pragma unroll
        for (int k = TW - 1; k >= 0; --k) {
            if (k < nn) {
                const T xk = x[k] * Rd[k];
                x[k] = xk;
                #pragma unroll
                for (int i = 0; i < k; ++i) x[i] -= Us[i][k] * xk;
            }
        }
        if (lane < TW) {
            #pragma unroll
            for (int i = 0; i < TW; ++i) Uinv[i * TW + lane] = x[i];
        }
        if (blockIdx.x == 0 && live) {
            #pragma unroll
            for (int j = 0; j < TW; ++j) if (j < nn) top[lane + j * ldt] = a[j];
            sgn[r + lane] = s_mine;
        }
    }
    __syncthreads();
    const int64_t row = r + nn + blockIdx.x * (int64_t)256 + tid;
    if (row < m) {
        // row of L21 = A21 U11^{-1}: 32 independent accumulators (one serial
        // dot product per output would chain 32 dependent FMAs 32 times)
        T acc[TW];
        #pragma unroll
        for (int j = 0; j < TW; ++j) acc[j] = zero<T>();
        #pragma unroll
        for (int k = 0; k < TW; ++k) {
            if (k < nn) {
                const T av = in_scale * Ain[row + (r + k) * ldi];
                #pragma unroll
                for (int j = 0; j < TW; ++j) acc[j] += av * Uinv[k * TW + j];
            }
        }
        #pragma unroll
        for (int j = 0; j < TW; ++j)
            if (j < nn) Aout[row + (r + j) * ldo] = acc[j];
    }
}

//------------------------------------------------------------------------------
// On-chip TSQR of one narrow panel block (nn <= 32 columns).
//
// Every node of the reduction tree is a workgroup-sized Householder QR: 256
// rows x nn columns held in VGPRs (one row per thread).  Per column: a block
// reduction of the column norm, the reflector (LAPACK larfg), ONE block
// reduction of a 32-vector carrying both the dots v^H A(:, l > k) for the
// update and the Gram entries V(:, i < k)^H v for the larft recurrence of T,
// then the rank-1 update in registers.  Leaves factor 256-row slices of the
// panel; tree nodes factor 8 stacked 32 x nn R factors of their children.
template <typename R>
__device__ inline R rsq(R x) { return x * x; }

template <typename T>
__device__ inline void larfg_dev(T alpha, real_t<T> xnorm2, T& beta_o, T& tau, T& scal) {
    using R = real_t<T>;
    R ar = real(alpha), ai = imag(alpha);
    if (xnorm2 == R(0) && ai == R(0)) { beta_o = alpha; tau = zero<T>(); scal = zero<T>(); return; }
    R nrm = sqrt(ar * ar + ai * ai + xnorm2);
    R beta = ar >= 0 ? -nrm : nrm;
    if constexpr (is_cplx<T>::value) {
        tau = T((beta - ar) / beta, -ai / beta);
        scal = one<T>() / (alpha - T(beta, R(0)));
        beta_o = T(beta, R(0));
    } else {
        tau = (beta - ar) / beta;
        scal = one<T>() / (alpha - beta);
        beta_o = beta;
    }
}

template <typename T>
__device__ inline T block_sum256(T v, T* red /* [4] */) {
    using R = real_t<T>;
    T s;
    if constexpr (is_cplx<T>::value) s = T(wave_sum(v.re), wave_sum(v.im));
    else s = wave_sum(v);
    (void)sizeof(R);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = s;
    __syncthreads();
    T t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
}

// Reduce-scatter of 32 per-lane values over a wave, without LDS: strides 32
// and 16 use v_permlane32_swap / v_permlane16_swap with vdst = the lower-index
// value and src = the upper-index value, after which (vdst + src) is, in
// every lane, its kept index plus the partner's copy of it; strides 8, 4-ish
// (row_half_mirror: i <-> 7-i) and 2 use DPP moves; a final quad_perm xor 1
// completes the sum.  Lane L ends with the wave sum of index bfly_idx(L).
__device__ inline int bfly_idx(int L) {
    return ((L >> 5) & 1) * 16 + ((L >> 4) & 1) * 8 + ((L >> 3) & 1) * 4 + ((L >> 2) & 1) * 2 + ((L >> 1) & 1);
}
template <bool SW32>
__device__ inline float swap_sum(float lo, float hi) {
    auto r = SW32 ? __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi),
                                                     false, false)
                  : __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi),
                                                     false, false);
    return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
template <bool SW32>
__device__ inline double swap_sum(double lo, double hi) {
    uint2 a = __builtin_bit_cast(uint2, lo), b = __builtin_bit_cast(uint2, hi);
    auto rx = SW32 ? __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false)
                   : __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
    auto ry = SW32 ? __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false)
                   : __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
    uint2 v = {(unsigned)rx[0], (unsigned)ry[0]}, w = {(unsigned)rx[1], (unsigned)ry[1]};
    return __builtin_bit_cast(double, v) + __builtin_bit_cast(double, w);
}
template <bool SW32, typename R>
__device__ inline cplx<R> swap_sum(cplx<R> lo, cplx<R> hi) {
    return cplx<R>(swap_sum<SW32>(lo.re, hi.re), swap_sum<SW32>(lo.im, hi.im));
}
template <int CTRL>
__device__ inline float dppv(float x) { return dpp_r<CTRL>(x); }
template <int CTRL>
__device__ inline double dppv(double x) { return dpp_r<CTRL>(x); }
template <int CTRL, typename R>
__device__ inline cplx<R> dppv(cplx<R> x) { return cplx<R>(dpp_r<CTRL>(x.re), dpp_r<CTRL>(x.im)); }

// one DPP split stage: lanes with `hi` keep index i + H, the others index i
template <int CTRL, int H, typename T>
__device__ inline void dpp_split(T (&q)[TW], bool hi) {
    #pragma unroll
    for (int i = 0; i < H; ++i) {
        T s0 = q[i] + dppv<CTRL>(q[i]);
        T s1 = q[i + H] + dppv<CTRL>(q[i + H]);
        q[i] = hi ? s1 : s0;
    }
}

template <typename T>
__device__ inline T wave_reduce_scatter32(T (&q)[TW]) {
    const int lane = threadIdx.x & 63;
    #pragma unroll
    for (int i = 0; i < 16; ++i) q[i] = swap_sum<true>(q[i], q[i + 16]);
    #pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = swap_sum<false>(q[i], q[i + 8]);
    dpp_split<0x128, 4>(q, (lane & 8) != 0);     // row_ror:8 == xor 8 inside a 16-lane row
    dpp_split<0x141, 2>(q, (lane & 4) != 0);     // row_half_mirror: i <-> 7 - i
    dpp_split<0x4E, 1>(q, (lane & 2) != 0);      // quad_perm [2,3,0,1]: xor 2
    return q[0] + dppv<0xB1>(q[0]);              // quad_perm [1,0,3,2]: xor 1
}

template <typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void qr_node_kernel(
        int64_t rows, int nn, const T* In, int64_t ldi, T* Vout, int64_t ldv, T* Rout, int64_t ldr, T* Tout) {
    if (SLATE_QR_NODE_PRIO) SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    __shared__ R red[2][4];
    __shared__ T wred[4][TW];
    __shared__ T wv[TW];
    __shared__ T s_alpha[2];
    __shared__ T Z[TW][TW + 1];     // Z(j, k) = V(:, j)^H v_k (j < k), for T after the loop
    __shared__ T Rs[TW][TW + 1];    // R(i, j), i <= j
    __shared__ T s_tau[TW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t row0 = blockIdx.x * (int64_t)256;
    const int64_t nb_rows = rows - row0 < 256 ? rows - row0 : 256;
    const bool live = tid < nb_rows;
    // Rotating register block: at step k, a[0] is column k, a[1 .. 31-k] the
    // columns still to factor, a[32-k ..] the finished reflectors V_0 .. V_{k-1}
    // (explicit: 1 on the diagonal, 0 above).  Each step ends with a shift, so
    // every index is a compile-time constant (no per-element selects on k) and
    // all 32 steps run (columns >= nn are zero: tau = 0, v = e_k).
    T a[TW];
    #pragma unroll
    for (int j = 0; j < TW; ++j) a[j] = (live && j < nn) ? In[row0 + tid + j * ldi] : zero<T>();
    for (int i = tid; i < TW * (TW + 1); i += 256) (&Rs[0][0])[i] = zero<T>();
    #pragma unroll 1
    for (int k = 0; k < TW; ++k) {
        const T ak = a[0];
        // column norm below the diagonal and alpha
        R x2 = (tid > k) ? real(ak) * real(ak) + imag(ak) * imag(ak) : R(0);
        R xs = wave_sum(x2);
        if (lane == 0) red[k & 1][w] = xs;
        if (tid == k) s_alpha[k & 1] = ak;
        __syncthreads();
        const R xnorm2 = red[k & 1][0] + red[k & 1][1] + red[k & 1][2] + red[k & 1][3];
        T beta, tau, scal;
        larfg_dev(s_alpha[k & 1], xnorm2, beta, tau, scal);
        const T v = (tid > k) ? ak * scal : (tid == k ? one<T>() : zero<T>());
        // R column k: rows < k keep their values, row k gets beta
        if (tid <= k) Rs[tid][k] = (tid == k) ? beta : ak;
        // one 32-vector reduction, same formula for every slot:
        // slots 1..31-k: v^H A(:, l) (update); slots 32-k..31: v^H V_j (Gram, conj)
        T q[TW];
        #pragma unroll
        for (int p = 0; p < TW; ++p) q[p] = conj(v) * a[p];
        T sm = wave_reduce_scatter32(q);
        if ((lane & 1) == 0) wred[w][bfly_idx(lane)] = sm;
        __syncthreads();
        if (tid < TW) {
            T t = wred[0][tid] + wred[1][tid] + wred[2][tid] + wred[3][tid];
            const bool vslot = tid >= TW - k;        // a finished reflector V_j, j = tid - (32 - k)
            if (vslot) Z[tid - (TW - k)][k] = conj(t);
            wv[tid] = (vslot || tid == 0) ? zero<T>() : t;
            if (tid == 0) s_tau[k] = tau;
        }
        __syncthreads();
        // rank-1 update of the remaining columns (v = 0 above row k leaves R alone),
        // then rotate: drop column k, append v as V_k
        const T ctv = conj(tau) * v;
        #pragma unroll
        for (int p = 1; p < TW; ++p) a[p - 1] = a[p] - ctv * wv[p];
        a[TW - 1] = v;
    }
    __syncthreads();
    // a[j] = V_j (explicit); V below the diagonal + R on/above into Vout, R into Rout
    if (live) {
        #pragma unroll
        for (int j = 0; j < TW; ++j) if (j < nn) Vout[row0 + tid + j * ldv] = (tid > j) ? a[j] : Rs[tid][j];
    }
    if (tid < TW) {
        #pragma unroll
        for (int j = 0; j < TW; ++j)
            if (j < nn) Rout[blockIdx.x * (int64_t)TW + tid + j * ldr] = (tid <= j && live) ? Rs[tid][j] : zero<T>();
    }
    // T by the larft recurrence, lane i = row i in registers:
    // T(i, k) = -tau_k sum_{j=i}^{k-1} T(i, j) Z(j, k),  T(k, k) = tau_k
    if (tid < TW) {
        const int i = tid;
        T t[TW];
        #pragma unroll
        for (int k = 0; k < TW; ++k) {
            T val = zero<T>();
            if (k < nn) {
                if (i == k) val = s_tau[k];
                else if (i < k) {
                    T sum = zero<T>();
                    #pragma unroll
                    for (int j = 0; j < k; ++j) if (j >= i) sum += t[j] * Z[j][k];
                    val = -s_tau[k] * sum;
                }
            }
            t[k] = val;
        }
        #pragma unroll
        for (int k = 0; k < TW; ++k) Tout[blockIdx.x * (int64_t)(TW * TW) + i + k * TW] = t[k];
    }
}

// Q_b [E_b; 0] for every tree node b: rows [256 b, ...) of V (unit lower top),
// T_b (32 x 32), E_b = rows [32 b, 32 b + 32) of E (identity when E == null).
// Out = [E_b; 0] - V_b T_b (V_b1^H E_b), written to rows [256 b, ...) of Q.
template <typename T>
__global__ __launch_bounds__(256) void qr_node_q_kernel(int64_t rows, int nn, const T* V, int64_t ldv,
                                                        const T* Tin, const T* E, int64_t lde, T* Q, int64_t ldq) {
    if (SLATE_QR_NODE_PRIO) SLATE_PANEL_WAVE_PRIO();
    __shared__ T sE[TW][TW + 1], sV1[TW][TW + 1], sW[TW][TW + 1], sT[TW][TW + 1];
    const int tid = threadIdx.x;
    const int64_t row0 = blockIdx.x * (int64_t)256;
    const int64_t nb_rows = rows - row0 < 256 ? rows - row0 : 256;
    for (int i = tid; i < TW * TW; i += 256) {
        int r = i % TW, c = i / TW;
        T e = zero<T>();
        if (c < nn) e = E ? E[blockIdx.x * (int64_t)TW + r + c * lde] : (r == c ? one<T>() : zero<T>());
        sE[r][c] = e;
        T v1 = zero<T>();
        if (c < nn && r < nb_rows) v1 = (r == c) ? one<T>() : (r > c ? V[row0 + r + c * ldv] : zero<T>());
        sV1[r][c] = v1;
        sT[r][c] = (c < nn && r < nn) ? Tin[blockIdx.x * (int64_t)(TW * TW) + i] : zero<T>();
    }
    __syncthreads();
    // W = V1^H E
    for (int i = tid; i < TW * TW; i += 256) {
        int r = i % TW, c = i / TW;
        T sum = zero<T>();
        #pragma unroll 8
        for (int k = 0; k < TW; ++k) sum += conj(sV1[k][r]) * sE[k][c];
        sW[r][c] = sum;
    }
    __syncthreads();
    // W2 = T W (T upper triangular) -> reuse sV1? no: write into sE's partner sT-free space
    T w2[4];
    #pragma unroll
    for (int q = 0; q < 4; ++q) {
        int i = tid + q * 256, r = i % TW, c = i / TW;
        T sum = zero<T>();
        for (int k = r; k < TW; ++k) sum += sT[r][k] * sW[k][c];
        w2[q] = sum;
    }
    __syncthreads();
    #pragma unroll
    for (int q = 0; q < 4; ++q) {
        int i = tid + q * 256, r = i % TW, c = i / TW;
        sW[r][c] = w2[q];
    }
    __syncthreads();
    if (tid < nb_rows) {
        T vr[TW];
        #pragma unroll
        for (int k = 0; k < TW; ++k)
            vr[k] = (k < nn) ? (tid > k ? V[row0 + tid + k * ldv] : (tid == k ? one<T>() : zero<T>())) : zero<T>();
        #pragma unroll 1
        for (int c = 0; c < nn; ++c) {
            T sum = tid < TW ? sE[tid][c] : zero<T>();
            #pragma unroll
            for (int k = 0; k < TW; ++k) sum -= vr[k] * sW[k][c];
            Q[row0 + tid + c * ldq] = sum;
        }
    }
}

// Finish the reconstruction of one narrow block (one wave): A's top block
// gets S R (upper) and Y1 (strictly lower); T = triu(U') S^H Y1^{-H}; tau = diag(T).
template <typename T>
__global__ __launch_bounds__(64) void qr_hr_finish_kernel(int nn, const T* LU, int64_t ldl, const T* sgn,
                                                          const T* Rr, int64_t ldr, T* A, int64_t lda, T* Tm,
                                                          int64_t ldt, T* tau) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ T sL[TW][TW + 1], sX[TW][TW + 1], sS[TW];
    const int i = threadIdx.x;
    for (int e = i; e < TW * TW; e += 64) {
        int r = e % TW, c = e / TW;
        sL[r][c] = (r < nn && c < nn) ? LU[r + c * ldl] : zero<T>();
    }
    if (i < TW) sS[i] = i < nn ? sgn[i] : one<T>();
    __syncthreads();
    if (i >= nn) return;
    const T si = sS[i];
    // row i of the top block: S R above/on the diagonal, Y1 strictly below
    for (int j = 0; j < nn; ++j) A[i + j * lda] = (i <= j) ? si * Rr[i + j * ldr] : sL[i][j];
    // X Y1^H = Tw with Tw(i, j) = U'(i, j) conj(s_j) (i <= j): forward
    // substitution along row i in axpy form (x_l final at step l, then one
    // independent FMA per later entry; no serial dot-product chain)
    T acc[TW];
    #pragma unroll
    for (int j = 0; j < TW; ++j) acc[j] = (i <= j && j < nn) ? sL[i][j] * conj(sS[j]) : zero<T>();
    #pragma unroll
    for (int l = 0; l < TW; ++l) {
        if (l < nn) {
            const T xl = acc[l];
            Tm[i + l * ldt] = xl;
            if (l == i) tau[i] = xl;
            #pragma unroll
            for (int j = l + 1; j < TW; ++j) acc[j] -= xl * conj(sL[j][l]);
        }
    }
}

//------------------------------------------------------------------------------
// Sign-modified LU leaf: the 64-column block at column c0 of the n x n matrix
// A in ONE launch of single-wave workgroups (lu_dist.cc lu_sign; replaces the
// 32-column narrow kernels and the recursion's trsm / gemm levels between
// them).  Every workgroup factors the b x b diagonal block in registers
// (lane = row, right-looking, row k of U broadcast from lane k by v_readlane;
// identity padding past b); then by role:
//   0            LU11 -> W (or A when no other workgroup reads A11) and the
//                signs; copies the previous leaf's staged block into place
//   1 .. nr      a 64-row block of L21 = A21 U11^{-1} (rows of U in LDS)
//   nr+1 ..      a 64-column block of U12 = L11^{-1} A12 (columns of L in
//                LDS; the block is transposed through LDS so that global
//                loads and stores stay coalesced)
// The trailing A22 -= L21 U12 is one GEMM launch after it.
template <typename T>
__global__ __launch_bounds__(64)
void lu_sign_leaf_kernel(int64_t n, int64_t c0, int b, T* A, int64_t lda, T* sgn, T* W, const T* Wprev, T* Aprev,
                         int bprev, int nr) {
    SLATE_PANEL_WAVE_PRIO();
    constexpr int LS = kLeafLS, XS = 65;
    __shared__ __attribute__((aligned(16))) T S[64 * LS];
    __shared__ T X[64 * XS];
    const int i = threadIdx.x;
    const int wg = blockIdx.x;
    const int64_t r = n - c0 - b;          // rows below = columns to the right
    T* A11 = A + c0 + c0 * lda;
    T a[64];
    {
        const T* Ai = A11 + min(i, b - 1);
        int64_t off = 0;
        #pragma unroll
        for (int l = 0; l < 64; ++l) {
            const T v = Ai[off];
            a[l] = (i < b && l < b) ? v : ((i == l) ? one<T>() : zero<T>());
            if (l + 1 < b) off += lda;
        }
    }
    T s_mine = one<T>();
    auto fstep = [&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const T p = bcast_lane(a[j], j);
        const T sg = unit_phase(p);
        const T d = p + sg;                 // |d| >= 1
        const T rd = rcp_nr(d);
        const T lij = (i > j) ? a[j] * rd : zero<T>();
        if (i == j) {
            a[j] = d;
            s_mine = sg;
        } else if (i > j) {
            a[j] = lij;
        }
        // row j of U from lane j, 8 columns per scheduling group (the
        // readlanes land in SGPRs: hoisting a whole row spilled)
        #pragma unroll
        for (int l = j + 1; l < 64; ++l) {
            a[l] -= lij * bcast_lane(a[l], j);
            if ((l & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
#define LU_FSTEP(x) fstep(std::integral_constant<int, (x)>{});
    LEAF_REP64(LU_FSTEP)
#undef LU_FSTEP
    if (wg == 0) {
        const bool direct = (r == 0);
        T* Fi = direct ? A11 + i : W + i;
        const int64_t ld = direct ? lda : 64;
        if (i < b) {
            sgn[c0 + i] = s_mine;
            int64_t off = 0;
            #pragma unroll
            for (int l = 0; l < 64; ++l) {      // predicated, not `break`: an early
                if (l < b) Fi[off] = a[l];      // exit left the loop rolled and a[]
                off += ld;                      // in scratch
            }
        }
        if (Aprev && i < bprev) {
            // all loads, then all stores (see aux.hip tri_solve_cols)
            T* Ap = Aprev + i;
            const T* Wp = Wprev + i;
            T t[64];
            #pragma unroll
            for (int l = 0; l < 64; ++l) t[l] = Wp[l * 64];
            int64_t off = 0;
            #pragma unroll
            for (int l = 0; l < 64; ++l) {
                if (l < bprev) Ap[off] = t[l];
                off += lda;
            }
        }
        return;
    }
    if (wg <= nr) {
        // rows of U, reciprocal pivots on the diagonal
        #pragma unroll
        for (int l = 0; l < 64; ++l) S[i * LS + l] = (l == i) ? rcp_nr(a[l]) : a[l];
        __syncthreads();
        const int64_t row = c0 + b + (int64_t)(wg - 1) * 64 + i;
        const bool live = row < n;
        T* Ar = A + (live ? row : c0 + b) + c0 * lda;
        T y[64];
        {
            int64_t off = 0;
            #pragma unroll
            for (int c = 0; c < 64; ++c) {
                const T v = Ar[off];
                y[c] = (live && c < b) ? v : zero<T>();
                if (c + 1 < b) off += lda;
            }
        }
        leaf_solve<T, false, false>(y, S);
        if (live) {
            int64_t off = 0;
            #pragma unroll
            for (int c = 0; c < 64; ++c) {
                if (c < b) Ar[off] = y[c];
                off += lda;
            }
        }
        return;
    }
    // columns of L (unit diagonal): S(c, l) = L(l, c)
    #pragma unroll
    for (int l = 0; l < 64; ++l) S[l * LS + i] = a[l];
    // the 64-column block of A12, transposed through X (lane = row on the
    // global side, lane = column in the solve)
    const int64_t col0 = c0 + b + (int64_t)(wg - nr - 1) * 64;
    const int ncol = (int)min<int64_t>(64, n - col0);
    T* A12 = A + c0 + col0 * lda;
    {
        const T* Ai = A12 + min(i, b - 1);
        int64_t off = 0;
        T t[64];
        #pragma unroll
        for (int e = 0; e < 64; ++e) {
            t[e] = Ai[off];
            if (e + 1 < ncol) off += lda;
        }
        #pragma unroll
        for (int e = 0; e < 64; ++e) X[e * XS + i] = (i < b && e < ncol) ? t[e] : zero<T>();
    }
    __syncthreads();
    T x[64];
    #pragma unroll
    for (int c = 0; c < 64; ++c) x[c] = X[i * XS + c];
    leaf_solve<T, false, true>(x, S);
    #pragma unroll
    for (int c = 0; c < 64; ++c) X[i * XS + c] = x[c];
    __syncthreads();
    if (i < b) {
        T* Ai = A12 + i;
        int64_t off = 0;
        #pragma unroll
        for (int e = 0; e < 64; ++e) {
            if (e < ncol) Ai[off] = X[e * XS + i];
            off += lda;
        }
    }
}

}  // namespace

template <typename T>
void lu_sign_leaf(int64_t n, int64_t c0, int b, T* A, int64_t lda, T* sgn, T* W, const T* Wprev, T* Aprev, int bprev,
                  hipStream_t s) {
    if (b <= 0) return;
    const int64_t r = n - c0 - b;
    if (b > 64 || r < 0 || bprev > 64) throw std::invalid_argument("lu_sign_leaf: b, bprev <= 64, c0 + b <= n");
    if (r > 0 && !W) throw std::invalid_argument("lu_sign_leaf: r > 0 needs the 64 x 64 staging block W");
    if (Aprev && !Wprev) throw std::invalid_argument("lu_sign_leaf: Aprev needs Wprev");
    if constexpr (sizeof(T) > 8) {
        throw std::invalid_argument("lu_sign_leaf: complex<double> is not supported");
    } else {
        const int nr = (int)((r + 63) / 64);
        hipLaunchKernelGGL(lu_sign_leaf_kernel<T>, dim3(1 + 2 * nr), dim3(64), 0, s, n, c0, b, A, lda, sgn, W, Wprev,
                           Aprev, bprev, nr);
    }
}

template <typename T>
void lu_sign_narrow(int64_t m, int64_t r, int nn, T* A, int64_t lda, const T* Utop, T* sgn, hipStream_t s) {
    if (nn <= 0 || r >= m) return;
    const int grid = (int)std::max<int64_t>(1, (m - r - nn + 255) / 256);
    hipLaunchKernelGGL(lu_sign_narrow_kernel<T>, dim3(grid), dim3(256), 0, s, m, r, nn, (const T*)A, lda, A, lda,
                       Utop, (int64_t)TW, one<T>(), A + r + r * lda, lda, sgn);
}

int64_t qr_tsqr_levels(int64_t rows, int64_t* nblk) {
    int64_t n = (rows + 255) / 256, L = 0;
    if (nblk) nblk[0] = n;
    while (n > 1) { n = (n + 7) / 8; ++L; if (nblk) nblk[L] = n; }
    return L;
}

int64_t qr_tsqr_workspace(int64_t rows) {
    int64_t nblk[64];
    int64_t L = qr_tsqr_levels(rows, nblk);
    int64_t w = 0;
    for (int64_t l = 0; l <= L; ++l) {
        w += nblk[l] * TW * TW * 3;                 // R, T, E of level l
        if (l > 0) w += nblk[l - 1] * TW * TW;      // V of level l (its stacked input)
    }
    return w + rows * TW + 2 * TW * TW + TW;       // Q, LU top, sgn
}

template <typename T>
void qr_tsqr_narrow(int64_t rows, int nn, T* A, int64_t lda, T* Tm, int64_t ldt, T* tau, T* work, hipStream_t s) {
    if (rows <= 0 || nn <= 0) return;
    int64_t nblk[64];
    const int64_t L = qr_tsqr_levels(rows, nblk);
    // workspace layout
    T* p = work;
    T *Rl[64], *Tl[64], *El[64], *Vl[64];
    for (int64_t l = 0; l <= L; ++l) {
        Rl[l] = p; p += nblk[l] * TW * TW;
        Tl[l] = p; p += nblk[l] * TW * TW;
        El[l] = p; p += nblk[l] * TW * TW;
        Vl[l] = nullptr;
        if (l > 0) { Vl[l] = p; p += nblk[l - 1] * TW * TW; }
    }
    T* Qb = p; p += rows * TW;
    T* LUt = p; p += 2 * TW * TW;
    T* sg = p;
    // up the tree: leaves factor A's rows in place; nodes factor stacked R's
    hipLaunchKernelGGL(qr_node_kernel<T>, dim3((unsigned)nblk[0]), dim3(256), 0, s, rows, nn, (const T*)A, lda, A, lda,
                       Rl[0], nblk[0] * TW, Tl[0]);
    for (int64_t l = 1; l <= L; ++l) {
        const int64_t rl = nblk[l - 1] * TW;
        hipLaunchKernelGGL(qr_node_kernel<T>, dim3((unsigned)nblk[l]), dim3(256), 0, s, rl, nn, (const T*)Rl[l - 1], rl,
                           Vl[l], rl, Rl[l], nblk[l] * TW, Tl[l]);
    }
    // down the tree: E = [I; 0] at the root, Q_node [E; 0] split to the children
    for (int64_t l = L; l >= 1; --l) {
        const int64_t rl = nblk[l - 1] * TW;
        hipLaunchKernelGGL(qr_node_q_kernel<T>, dim3((unsigned)nblk[l]), dim3(256), 0, s, rl, nn, (const T*)Vl[l], rl,
                           (const T*)Tl[l], l == L ? (const T*)nullptr : (const T*)El[l], nblk[l] * TW, El[l - 1], rl);
    }
    hipLaunchKernelGGL(qr_node_q_kernel<T>, dim3((unsigned)nblk[0]), dim3(256), 0, s, rows, nn, (const T*)A, lda,
                       (const T*)Tl[0], L == 0 ? (const T*)nullptr : (const T*)El[0], nblk[0] * TW, Qb, rows);
    // Householder reconstruction: [S; 0] - Q = Y U'; V = Y below the top block
    hipLaunchKernelGGL(lu_sign_narrow_kernel<T>, dim3((unsigned)std::max<int64_t>(1, (rows - nn + 255) / 256)), dim3(256),
                       0, s, rows, (int64_t)0, nn, (const T*)Qb, rows, A, lda, (const T*)Qb, rows, make_val<T>(-1.0),
                       LUt, (int64_t)TW, sg);
    hipLaunchKernelGGL(qr_hr_finish_kernel<T>, dim3(1), dim3(64), 0, s, nn, (const T*)LUt, (int64_t)TW, (const T*)sg,
                       (const T*)Rl[L], nblk[L] * TW, A, lda, Tm, ldt, tau);
}

#define SLATE_INST_TSQR(T) \
    template void lu_sign_narrow<T>(int64_t, int64_t, int, T*, int64_t, const T*, T*, hipStream_t); \
    template void lu_sign_leaf<T>(int64_t, int64_t, int, T*, int64_t, T*, T*, const T*, T*, int, hipStream_t); \
    template void qr_tsqr_narrow<T>(int64_t, int, T*, int64_t, T*, int64_t, T*, T*, hipStream_t);

SLATE_INST_TSQR(float)
SLATE_INST_TSQR(double)
SLATE_INST_TSQR(cplx<float>)
SLATE_INST_TSQR(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
