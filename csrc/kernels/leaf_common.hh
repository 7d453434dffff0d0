// Shared machinery of the single-wave "leaf" kernels (aux.hip potrf_leaf,
// tsqr.hip lu_sign_leaf): 64-column blocks held one row per lane in
// registers, the finished factor in LDS, and row-streamed substitutions.
//
// Why it looks like this (all measured on gfx950 with the leaf probe,
// csrc/tools/leaf_probe.hip):
//  * One wave issues at most one instruction per 4-cycle slot, so every
//    instruction counts: the factor's pivot and row broadcasts, the 2016
//    FMAs of a 64 x 64 triangle and their LDS reads dominate.
//  * The 64 steps are expanded by the preprocessor (LEAF_REP64 over a generic
//    lambda taking the step as a type): a `#pragma unroll` loop of this size
//    exceeds LLVM's full-unroll threshold and falls back to a rolled loop
//    whose register arrays are indexed dynamically (scratch).
//  * LDS rows stream in kLeafG-element groups, the reads of a later group
//    issued before the current group's FMAs, each group ending in an empty
//    volatile asm on the registers it wrote plus a scheduling barrier: left
//    alone, the scheduler sank the FMAs below every read and spilled 15 KB
//    per lane.
#pragma once

#include "device_common.hh"

#include <type_traits>

namespace slate_amd {
namespace dev {

constexpr int kLeafG = 16;    // rows per LDS group
constexpr int kLeafLS = 64 + 2;   // LDS row stride (16-B aligned groups)
#ifdef LEAF_PROBE
__device__ long long g_leaf_probe[64 * 8];
#define LEAF_STAMP(k)                                                                      \
    do {                                                                                   \
        __builtin_amdgcn_s_waitcnt(0);                                                     \
        const long long t_ = clock64();                                                    \
        if (threadIdx.x == 0 && blockIdx.x < 64) g_leaf_probe[blockIdx.x * 8 + (k)] = t_;  \
    } while (0)
#else
#define LEAF_STAMP(k) do {} while (0)
#endif
template <typename T>
__device__ __forceinline__ void leaf_pin1(T& v) {
    if constexpr (is_cplx<T>::value) asm volatile("" : "+v"(v.re), "+v"(v.im));
    else asm volatile("" : "+v"(v));
}
template <typename R>
__device__ __forceinline__ R leaf_rsqrt(R d) {
    R r;
    if constexpr (sizeof(R) == 8) r = __builtin_amdgcn_rsq(d);
    else r = __builtin_amdgcn_rsqf(d);
    const R e = fma(-d * r, r, R(1));       // 1 - d r^2
    return fma(R(0.5) * r, e, r);
}
// first group of a stream column: the factor's delayed update of column k
// covers rows >= k + 2, the solve's column c rows >= c (diagonal first)
__device__ constexpr int leaf_g0(int first_row) { return first_row / kLeafG; }
// groups before the factor stream's column k (rows >= k + 2 of each column)
__device__ constexpr int leaf_fq0(int k) {
    int q = 0;
    for (int t = 0; t < k; ++t) q += 64 / kLeafG - leaf_g0(t + 2);
    return q;
}
// groups before the solve stream's column c (rows >= c) of an N-row solve
template <int N = 64>
__device__ constexpr int leaf_sq0(int c) {
    int q = 0;
    for (int t = 0; t < c; ++t) q += N / kLeafG - leaf_g0(t);
    return q;
}
// solve stream: next group after (col, grp)
struct LeafPos { int col, grp; };
template <int N = 64>
__device__ constexpr LeafPos leaf_snext(LeafPos p) {
    return p.grp + 1 < N / kLeafG ? LeafPos{p.col, p.grp + 1} : LeafPos{p.col + 1, leaf_g0(p.col + 1)};
}
// The 64 steps are expanded by the preprocessor, each a call of a generic
// lambda with its step number as a type: a `#pragma unroll` loop of this size
// exceeds LLVM's full-unroll threshold and falls back to a rolled loop whose
// register arrays are indexed dynamically (scratch).
#define LEAF_REP4(M, x) M((x)) M((x) + 1) M((x) + 2) M((x) + 3)
#define LEAF_REP16(M, x) LEAF_REP4(M, (x)) LEAF_REP4(M, (x) + 4) LEAF_REP4(M, (x) + 8) LEAF_REP4(M, (x) + 12)
#define LEAF_REP32(M) LEAF_REP16(M, 0) LEAF_REP16(M, 16)
#define LEAF_REP64(M) LEAF_REP16(M, 0) LEAF_REP16(M, 16) LEAF_REP16(M, 32) LEAF_REP16(M, 48)


// Row-streamed substitution of one N-element row per lane (N = 32 or 64)
// against the N x N matrix S in LDS (row stride kLeafLS): for c = 0..N-1,
//   y[c] *= S(c, c)                          (skipped when UNIT)
//   y[l] -= y[c] * op(S(c, l))  for l > c    (op = conj when CONJ)
// i.e. y := y op(U)^{-1} for the upper triangle U whose rows are S's rows
// (S's diagonal holds the reciprocal pivots).  The updates of a step are
// independent FMAs; S streams in groups with two groups in flight.
template <typename T, bool CONJ, bool UNIT, int N = 64>
__device__ __forceinline__ void leaf_solve(T (&y)[N], const T* S) {
    static_assert(N == 32 || N == 64, "leaf_solve: N = 32 or 64");
    constexpr int LS = kLeafLS;
    T buf[3][kLeafG];
    #pragma unroll
    for (int e = 0; e < kLeafG; ++e) {
        buf[0][e] = S[e];
        buf[1][e] = S[kLeafG + e];
    }
    auto step = [&](auto cc) __attribute__((always_inline)) {
        constexpr int c = decltype(cc)::value;
        constexpr int q0 = leaf_sq0<N>(c), g0 = leaf_g0(c);
        #pragma unroll
        for (int g = g0; g < N / kLeafG; ++g) {
            const int q = q0 + g - g0;
            const LeafPos n2 = leaf_snext<N>(leaf_snext<N>(LeafPos{c, g}));
            if (n2.col < N) {
                #pragma unroll
                for (int e = 0; e < kLeafG; ++e) buf[(q + 2) % 3][e] = S[n2.col * LS + n2.grp * kLeafG + e];
            }
            #pragma unroll
            for (int e = 0; e < kLeafG; ++e) {
                const int l = g * kLeafG + e;
                const T v = CONJ ? conj(buf[q % 3][e]) : buf[q % 3][e];
                if (l == c) {
                    if constexpr (!UNIT) y[c] = y[c] * v;
                } else if (l > c) {
                    y[l] -= y[c] * v;
                }
            }
            #pragma unroll
            for (int e = 0; e < kLeafG; ++e)
                if (g * kLeafG + e >= c) leaf_pin1(y[g * kLeafG + e]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
#define LEAF_SSTEP(x) step(std::integral_constant<int, (x)>{});
    if constexpr (N == 64) {
        LEAF_REP64(LEAF_SSTEP)
    } else {
        LEAF_REP32(LEAF_SSTEP)
    }
#undef LEAF_SSTEP
}

}  // namespace dev
}  // namespace slate_amd
