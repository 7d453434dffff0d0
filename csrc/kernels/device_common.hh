// Shared device-side definitions for the gfx950 (CDNA4) kernels.
//
// Everything here is written for 64-wide wavefronts and the CDNA4 MFMA
// register layouts; there is no other target.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include "dev_types.hh"

// Panel (critical-path) kernels raise their waves' instruction-issue priority
// (s_setprio) so that trailing-update GEMM waves sharing the CU do not starve
// them: the hardware queue priority only orders dispatch, not issue inside a
// SIMD.  SLATE_PANEL_PRIO=0 at build time turns it off (A/B builds).
#ifndef SLATE_PANEL_PRIO
#define SLATE_PANEL_PRIO 1
#endif
#define SLATE_PANEL_WAVE_PRIO()                                   \
    do {                                                          \
        if (SLATE_PANEL_PRIO) __builtin_amdgcn_s_setprio(3);      \
    } while (0)

namespace slate_amd {
namespace dev {

__device__ inline float  absval(float x)  { return fabsf(x); }
__device__ inline double absval(double x) { return fabs(x); }
__device__ inline float  absval(cplx<float> x)  { return hypotf(x.re, x.im); }
__device__ inline double absval(cplx<double> x) { return hypot(x.re, x.im); }
// |re| + |im| (LAPACK cabs1), used for pivot search
__device__ inline float  abs1(float x)  { return fabsf(x); }
__device__ inline double abs1(double x) { return fabs(x); }
__device__ inline float  abs1(cplx<float> x)  { return fabsf(x.re) + fabsf(x.im); }
__device__ inline double abs1(cplx<double> x) { return fabs(x.re) + fabs(x.im); }



template <typename T> __host__ __device__ inline T make_val(double r) { return T(r); }
template <> __host__ __device__ inline cplx<float>  make_val<cplx<float>>(double r)  { return {float(r), 0.f}; }
template <> __host__ __device__ inline cplx<double> make_val<cplx<double>>(double r) { return {r, 0.0}; }

template <typename T> __host__ __device__ inline T zero() { return make_val<T>(0.0); }
template <typename T> __host__ __device__ inline T one()  { return make_val<T>(1.0); }

__device__ inline bool is_zero(float x) { return x == 0.f; }
__device__ inline bool is_zero(double x) { return x == 0.0; }
template <typename R> __device__ inline bool is_zero(cplx<R> x) { return x.re == R(0) && x.im == R(0); }

// Broadcast lane `src` of v to the whole wave (v_readlane; src is uniform).
__device__ inline float  bcast_lane(float v, int src)  { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src)); }
__device__ inline double bcast_lane(double v, int src) {
    int2 t = __builtin_bit_cast(int2, v);
    t.x = __builtin_amdgcn_readlane(t.x, src);
    t.y = __builtin_amdgcn_readlane(t.y, src);
    return __builtin_bit_cast(double, t);
}
template <typename R>
__device__ inline cplx<R> bcast_lane(cplx<R> v, int src) { return cplx<R>(bcast_lane(v.re, src), bcast_lane(v.im, src)); }


// NaN-propagating max, as in the reference's max_nan (device_util.cuh)
template <typename R>
__device__ inline R max_nan(R x, R y) { return (isnan(y) || y >= x) ? y : x; }

//------------------------------------------------------------------------------
// Wavefront helpers (64 lanes).
constexpr int kWave = 64;

// DPP lane moves (32-bit granules; 64-bit values move as two halves).
template <int CTRL>
__device__ inline int dpp_i(int x) { return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ inline float dpp_r(float x) { return __builtin_bit_cast(float, dpp_i<CTRL>(__builtin_bit_cast(int, x))); }
template <int CTRL>
__device__ inline double dpp_r(double x) {
    int2 t = __builtin_bit_cast(int2, x);
    t.x = dpp_i<CTRL>(t.x);
    t.y = dpp_i<CTRL>(t.y);
    return __builtin_bit_cast(double, t);
}

// Wave reductions: DPP butterflies inside each 16-lane row (quad_perm
// [1,0,3,2], [2,3,0,1], row_ror:4, row_ror:8), then v_readlane of the four
// row results.  No LDS traffic; the result is wave-uniform.
template <typename R, typename Op>
__device__ inline R wave_reduce(R v, Op op) {
    v = op(v, dpp_r<0xB1>(v));
    v = op(v, dpp_r<0x4E>(v));
    v = op(v, dpp_r<0x124>(v));
    v = op(v, dpp_r<0x128>(v));
    R r0 = bcast_lane(v, 0), r1 = bcast_lane(v, 16), r2 = bcast_lane(v, 32), r3 = bcast_lane(v, 48);
    return op(op(r0, r1), op(r2, r3));
}

template <typename R>
__device__ inline R wave_sum(R v) {
    return wave_reduce(v, [](R a, R b) { return a + b; });
}

template <typename R>
__device__ inline R wave_max_nan(R v) {
    return wave_reduce(v, [](R a, R b) { return max_nan(a, b); });
}

//------------------------------------------------------------------------------
// XCD-aware bijective remap of a 1-D grid: blocks b and b+8 share an XCD (L2)
// under round-robin dispatch, so hand each XCD a contiguous chunk of the
// logical tile order.  Speed only; any placement is correct.
__device__ inline int xcd_remap(int bid, int nblocks) {
    constexpr int NX = 8;
    if (nblocks < NX) return bid;
    int xcd = bid % NX;
    int q = nblocks / NX, r = nblocks % NX;
    int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + bid / NX;
}

}  // namespace dev
}  // namespace slate_amd
