// Tournament pivoting (TSLU / CALU panel) for a narrow column block, on gfx950.
//
// Reference behaviour: getrf_tntpiv's panel (src/internal/internal_getrf_tntpiv.cc
// :180-330) runs a reduction tree over row tiles: every leaf factors its tile
// with partial pivoting (vendor getrf), the winning rows of pairs of leaves are
// stacked and factored again, and the rows that win the final round become the
// pivots of the whole panel, which is then factored WITHOUT further pivoting.
//
// MI355X design: the tournament is played on a 32-column narrow block inside
// the recursive device panel (local_blas.cc LuPanelDev), so a 32768-row panel
// costs four or five launches instead of two launches per column:
//   select  leaves: 256 rows per workgroup, one row per thread held in VGPRs;
//           tree nodes: 512-thread workgroups, fan-in 16 (16 x 32 candidates).
//           GEPP per step: a 32-bit key DPP max inside each wave, the wave's
//           best row published to LDS, ONE workgroup barrier, then every
//           thread picks the best slot (measured 46-59 us per launch for the
//           earlier two-barrier (value, index) form at small M, which made the
//           panel latency-bound).  The final round also emits the LU of the
//           winners, so the rows kernel does not refactor the top block.
//   permute each workgroup owns panel columns; it re-derives the interchanges
//           from the winners in one wave (ballot/readlane, all scalar), applies
//           the net row permutation to its columns and copies the permuted
//           top block of the narrow block to a scratch buffer.
//   rows    wave 0 factors the top 32x32 block (lane = row, v_readlane
//           broadcasts) and inverts U11; then L21 = A21 * U11^{-1} runs on
//           v_mfma_f64_16x16x4 for fp64, 16-row slabs per wave.
#include "device_common.hh"
#include "kernels.hh"
#include "slate_amd/device.hh"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace slate_amd {
namespace dev {

namespace {

constexpr int TW = 32;        // tournament / narrow-block width

// for (k = B; k < E; ++k) f(integral_constant<k>) -- compile-time indices
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}
constexpr int TR = 256;       // leaf rows per workgroup
constexpr int NODE_NT = 512;  // node workgroup size
constexpr int FANIN = NODE_NT / TW;

template <typename R>
__device__ inline void argmax_pick(R& v, int& idx, R ov, int oi) {
    // max |v|; ties -> smaller row index (deterministic, LAPACK-like)
    if (ov > v || (ov == v && oi < idx) || (isnan(ov) && !isnan(v))) { v = ov; idx = oi; }
}

template <int CTRL, typename R>
__device__ inline void argmax_dpp(R& v, int& id) {
    R ov = dpp_r<CTRL>(v);
    int oi = dpp_i<CTRL>(id);
    argmax_pick(v, id, ov, oi);
}

// Wave-uniform argmax: DPP within rows of 16 lanes, then v_readlane of the
// four row results (no LDS, no ds_bpermute).
template <typename R>
__device__ inline void wave_argmax(R& v, int& id) {
    argmax_dpp<0xB1>(v, id);    // quad_perm [1,0,3,2]
    argmax_dpp<0x4E>(v, id);    // quad_perm [2,3,0,1]
    argmax_dpp<0x124>(v, id);   // row_ror:4
    argmax_dpp<0x128>(v, id);   // row_ror:8
    R bv = bcast_lane(v, 0);
    int bi = __builtin_amdgcn_readlane(id, 0);
    #pragma unroll
    for (int q = 1; q < 4; ++q) argmax_pick(bv, bi, bcast_lane(v, 16 * q), __builtin_amdgcn_readlane(id, 16 * q));
    v = bv; id = bi;
}

// 32-bit pivot-search key of a candidate: 1 + the fp32 bit pattern of its
// magnitude (monotonic for non-negative floats; NaN sorts above +inf, so it
// wins as LAPACK's i*amax would report it), 0 for "no candidate".  A wave max
// of the key is one DPP v_max_u32 per stage instead of a (double, index) pair
// through compare / select chains; magnitudes within one fp32 ulp tie and the
// lowest lane wins, which is as good a tournament pivot.
template <typename T>
__device__ inline uint32_t pivot_key(T v) {
    return 1u + __float_as_uint(float(abs1(v)));
}

__device__ inline uint32_t wave_max_u32(uint32_t k) {
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x124, 0xF, 0xF, false));  // row_ror:4
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x128, 0xF, 0xF, false));  // row_ror:8
    uint32_t a = __builtin_amdgcn_readlane(k, 0), b = __builtin_amdgcn_readlane(k, 16);
    uint32_t c = __builtin_amdgcn_readlane(k, 32), d = __builtin_amdgcn_readlane(k, 48);
    return max(max(a, b), max(c, d));
}

// Reciprocal for the elimination multipliers: v_rcp + two Newton steps for
// fp64 (the correctly rounded division sequence is ~10 dependent fp64 ops on
// the critical path of every step).
__device__ inline double fast_rcp(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}
__device__ inline float fast_rcp(float d) { return 1.0f / d; }
template <typename R>
__device__ inline cplx<R> fast_rcp(cplx<R> d) { return one<cplx<R>>() / d; }

// One tournament round: each workgroup factors up to NT rows x nn columns with
// partial pivoting and emits its (up to nn) pivot rows, in pivot order.
// Leaves (cand_in == nullptr) take rows [r + NT*b, ...); nodes take the
// candidate lists of NT/TW children.  Rows are read from the unmodified panel
// (CALU plays every round on original rows).  One row per thread in VGPRs.
// Per step ONE workgroup barrier: every wave finds its best row (32-bit key,
// DPP max), and that row's lane publishes key, index and the whole row to the
// wave's LDS slot; after the barrier every thread picks the best slot and
// eliminates against its row.  Slots are double-buffered by step parity, so
// the next step's writes never meet this step's reads.  With lu_out (the
// final round, one workgroup) the winners' GEPP -- the LU of the permuted top
// block -- is written out as well (multipliers below the diagonal).
template <typename T, int NT>
__global__ __launch_bounds__(NT) void tslu_select_kernel(int64_t m, int64_t r, int nn, const T* A, int64_t lda,
                                                         const int* cand_in, const int* cnt_in, int nin,
                                                         int* cand_out, int* cnt_out, T* lu_out) {
    SLATE_PANEL_WAVE_PRIO();
    constexpr int NW = NT / 64;
    __shared__ uint32_t skey[2][NW];
    __shared__ int sidx[2][NW];
    __shared__ T srow[2][NW][TW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int idx = INT_MAX;
    bool act = false;
    if (cand_in == nullptr) {
        int64_t i = r + blockIdx.x * (int64_t)NT + tid;
        if (i < m) { idx = (int)i; act = true; }
    } else {
        int child = blockIdx.x * (NT / TW) + tid / TW, k = tid % TW;
        if (child < nin && k < cnt_in[child]) { idx = cand_in[child * TW + k]; act = true; }
    }
    T a[TW];
    #pragma unroll
    for (int j = 0; j < TW; ++j) a[j] = (act && j < nn) ? A[idx + j * lda] : zero<T>();

    int cnt = 0;
    bool done = false;
    static_for<0, TW>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int bf = k & 1;
        if (k < nn && !done) {
            const uint32_t key = act ? pivot_key(a[k]) : 0u;
            const uint32_t kw = wave_max_u32(key);
            const unsigned long long win = __ballot(key == kw && kw != 0u);
            const int wl = win ? __ffsll((long long)win) - 1 : 0;
            if (lane == wl) {
                skey[bf][w] = kw;
                sidx[bf][w] = idx;
                #pragma unroll
                for (int j = 0; j < TW; ++j) srow[bf][w][j] = a[j];
            }
            __syncthreads();
            uint32_t kb = skey[bf][0];
            int wb = 0;
            #pragma unroll
            for (int q = 1; q < NW; ++q) {
                const uint32_t kq = skey[bf][q];
                if (kq > kb) { kb = kq; wb = q; }
            }
            if (kb == 0u) {
                done = true;                       // uniform: no candidates left
            } else {
                const int id = sidx[bf][wb];
                if (act && idx == id) act = false;
                const T d = srow[bf][wb][k];
                const T rd = is_zero(d) ? zero<T>() : fast_rcp(d);
                if (act) {
                    const T l = a[k] * rd;
                    #pragma unroll
                    for (int j = k + 1; j < TW; ++j) a[j] -= l * srow[bf][wb][j];
                    a[k] = l;
                }
                if (tid == 0) cand_out[blockIdx.x * TW + k] = id;
                if (lu_out && tid < TW && tid < nn) lu_out[k + tid * TW] = srow[bf][wb][tid];
                cnt = k + 1;
            }
        }
    });
    if (tid == 0) cnt_out[blockIdx.x] = cnt;
}

// Winners -> LAPACK ipiv (sequential interchanges with row r+k) and the net
// row permutation as (pos <- orig).  One wave: lanes 0..31 track positions
// r..r+31, lanes 32..63 the winners that lie below; an interchange swaps the
// `orig` register of two lanes.  Every index is wave-uniform (v_readlane).
// Returns true in lanes whose position receives a different row.
__device__ inline bool tslu_interchanges(int r, const int* win, int cnt, int64_t* ipiv, int& pos, int& orig) {
    const int l = threadIdx.x & 63;
    int wl = (l & 31) < cnt ? win[l & 31] : -1;
    pos = -1;
    if (l < 32) { if (l < cnt) pos = r + l; }
    else if (l - 32 < cnt && wl >= r + cnt) pos = wl;
    orig = pos;
    for (int k = 0; k < cnt; ++k) {
        int wk = __builtin_amdgcn_readlane(wl, k);
        unsigned long long bal = __ballot(pos >= 0 && orig == wk);
        int ql = __ffsll(bal) - 1;
        int q = __builtin_amdgcn_readlane(pos, ql);
        if (ipiv && l == 0) ipiv[r + k] = q;
        int ok = __builtin_amdgcn_readlane(orig, k), oq = __builtin_amdgcn_readlane(orig, ql);
        if (l == ql) orig = ok;
        if (l == k) orig = oq;
    }
    return pos >= 0 && pos != orig;
}

// Apply the tournament's row permutation to panel columns [0, ncols) (a
// column per wave), record ipiv/perm (workgroup 0), and copy the permuted top
// block of the narrow block (columns [c0, c0+nn)) to Utop (column-major, ld TW).
template <typename T>
__global__ __launch_bounds__(256) void tslu_permute_kernel(int r, int nn, int64_t c0, T* A, int64_t lda,
                                                           int64_t ncols, const int* win, const int* wcnt,
                                                           int64_t* ipiv, int64_t* perm, T* Utop) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ int s_dst[64], s_src[64], s_top[TW];
    __shared__ int s_np;
    const int tid = threadIdx.x;
    const int cnt = *wcnt;
    if (tid < 64) {
        int pos, orig;
        bool mv = tslu_interchanges(r, win, cnt, blockIdx.x == 0 ? ipiv : nullptr, pos, orig);
        unsigned long long bal = __ballot(mv);
        int slot = __popcll(bal & ((1ull << tid) - 1));
        if (mv) { s_dst[slot] = pos; s_src[slot] = orig; }
        if (tid == 0) s_np = __popcll(bal);
        // source row of each top position r + p
        if (tid < 32 && tid < cnt) s_top[tid] = orig;
        if (blockIdx.x == 0 && perm) {
            int64_t pv = mv ? perm[orig] : 0;
            if (mv) perm[pos] = pv;
        }
    }
    __syncthreads();
    const int np = s_np;
    const int p = tid & 63;
    for (int64_t j = blockIdx.x * 4 + (tid >> 6); j < ncols; j += (int64_t)gridDim.x * 4) {
        T* col = A + j * lda;
        T v = zero<T>(), u = zero<T>();
        const bool top = (j >= c0 && j < c0 + nn && p < nn);
        if (p < np) v = col[s_src[p]];
        if (top) u = col[s_top[p]];
        __builtin_amdgcn_wave_barrier();
        if (p < np) col[s_dst[p]] = v;
        if (top) Utop[(j - c0) * TW + p] = u;
    }
}

__device__ inline void mfma16(double a, double b, double (&c)[4]) {
    typedef double v4d __attribute__((ext_vector_type(4)));
    v4d acc = {c[0], c[1], c[2], c[3]};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    c[0] = acc[0]; c[1] = acc[1]; c[2] = acc[2]; c[3] = acc[3];
}

// Top block LU without pivoting (one wave; lane i = row i, readlane
// broadcasts) -- or, with lu_in, the LU the final tournament round already
// produced -- and the inverse of U11 with lane j holding column j: per step k
// (backward) one scaling and k independent FMAs against U's column k read
// from LDS (axpy form: no serial dot-product chain and no divide per step).
// Writes Uinv[i*TW + j] (zero outside the nn x nn triangle); returns the first
// zero pivot (or -1).
template <typename T>
__device__ inline int tslu_top_factor(int nn, const T* Utop, const T* lu_in, T (&a)[TW], T* Uinv, T (*Us)[TW + 1],
                                      T* Rd) {
    const int tid = threadIdx.x & 63;
    const bool live = tid < nn;
    int bad = -1;
    if (lu_in) {
        #pragma unroll
        for (int j = 0; j < TW; ++j) a[j] = (live && j < nn) ? lu_in[tid + j * TW] : zero<T>();
        T dg = zero<T>();
        #pragma unroll
        for (int j = 0; j < TW; ++j) if (j == tid) dg = a[j];
        const unsigned long long z = __ballot(live && is_zero(dg));
        bad = z ? __ffsll((long long)z) - 1 : -1;
    } else {
        #pragma unroll
        for (int j = 0; j < TW; ++j) a[j] = (live && j < nn) ? Utop[j * TW + tid] : zero<T>();
        #pragma unroll
        for (int k = 0; k < TW; ++k) {
            if (k < nn) {
                T d = bcast_lane(a[k], k);
                if (is_zero(d) && bad < 0) bad = k;
                T rd = is_zero(d) ? zero<T>() : one<T>() / d;
                T lk = a[k] * rd;
                #pragma unroll
                for (int j = k + 1; j < TW; ++j) {
                    T ukj = bcast_lane(a[j], k);
                    if (tid > k) a[j] -= lk * ukj;
                }
                if (tid > k) a[k] = lk;
            }
        }
    }
    if (tid < TW) {
        T dg = zero<T>();
        #pragma unroll
        for (int j = 0; j < TW; ++j) {
            Us[tid][j] = a[j];
            if (j == tid) dg = a[j];
        }
        Rd[tid] = (live && !is_zero(dg)) ? fast_rcp(dg) : zero<T>();
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    T x[TW];
    #pragma unroll
    for (int i = 0; i < TW; ++i) x[i] = (i == tid && live) ? one<T>() : zero<T>();
    #pragma unroll
    for (int k = TW - 1; k >= 0; --k) {
        if (k < nn) {
            const T xk = x[k] * Rd[k];
            x[k] = xk;
            #pragma unroll
            for (int i = 0; i < k; ++i) x[i] -= Us[i][k] * xk;
        }
    }
    if (tid < TW) {
        #pragma unroll
        for (int i = 0; i < TW; ++i) Uinv[i * TW + tid] = x[i];
    }
    return bad;
}

// L21 = A21 U11^{-1} for rows [r+nn, m); workgroup 0 also stores the factored
// top block and the info flag.  256 threads = 4 waves x 4 slabs of 16 rows.
template <typename T>
__global__ __launch_bounds__(256) void tslu_rows_kernel(int64_t m, int64_t r, int nn, T* A, int64_t lda,
                                                        const T* Utop, const T* lu_in, int* info,
                                                        int64_t info_offset) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ T Uinv[TW * TW];
    __shared__ T Us[TW][TW + 1];
    __shared__ T Rd[TW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (w == 0) {
        T a[TW];
        int bad = tslu_top_factor<T>(nn, Utop, lu_in, a, Uinv, Us, Rd);
        if (blockIdx.x == 0) {
            if (lane < nn) {
                #pragma unroll
                for (int j = 0; j < TW; ++j) if (j < nn) A[r + lane + j * lda] = a[j];
            }
            if (lane == 0 && bad >= 0 && info && *info == 0) *info = (int)(info_offset + r + bad + 1);
        }
    }
    __syncthreads();
    const int64_t base = r + nn + blockIdx.x * (int64_t)256;
    if constexpr (std::is_same<T, double>::value) {
        // swapped operands: MFMA A-op = Uinv[k0 + (lane>>4)][n0 + (lane&15)],
        // B-op = A21[row0 + (lane&15)][k0 + (lane>>4)]; D[n][m] comes back with
        // lane&15 = row, (lane>>4) + 4*reg = column.
        double ub[TW / 4][2];
        #pragma unroll
        for (int ks = 0; ks < TW / 4; ++ks)
            #pragma unroll
            for (int nt = 0; nt < 2; ++nt) ub[ks][nt] = Uinv[(ks * 4 + (lane >> 4)) * TW + nt * 16 + (lane & 15)];
        #pragma unroll
        for (int sl = 0; sl < 4; ++sl) {
            const int64_t row = base + (w * 4 + sl) * 16 + (lane & 15);
            const bool ok = row < m;
            double av[TW / 4];
            #pragma unroll
            for (int ks = 0; ks < TW / 4; ++ks) {
                int col = ks * 4 + (lane >> 4);
                av[ks] = (ok && col < nn) ? A[row + col * lda] : 0.0;
            }
            double c0[4] = {0, 0, 0, 0}, c1[4] = {0, 0, 0, 0};
            #pragma unroll
            for (int ks = 0; ks < TW / 4; ++ks) {
                mfma16(ub[ks][0], av[ks], c0);
                mfma16(ub[ks][1], av[ks], c1);
            }
            if (ok) {
                #pragma unroll
                for (int q = 0; q < 4; ++q) {
                    int col0 = (lane >> 4) + 4 * q, col1 = 16 + col0;
                    if (col0 < nn) A[row + col0 * lda] = c0[q];
                    if (col1 < nn) A[row + col1 * lda] = c1[q];
                }
            }
        }
    } else {
        // float / complex: one row per thread, FMAs against Uinv in LDS
        const int64_t row = base + tid;
        if (row < m) {
            T av[TW];
            #pragma unroll
            for (int k = 0; k < TW; ++k) av[k] = k < nn ? A[row + k * lda] : zero<T>();
            #pragma unroll 1
            for (int j = 0; j < nn; ++j) {
                T s = zero<T>();
                #pragma unroll
                for (int k = 0; k < TW; ++k) s += av[k] * Uinv[k * TW + j];
                A[row + j * lda] = s;
            }
        }
    }
}


//==============================================================================
// Tournament v2: the whole reduction tree in ONE launch, and the permutation +
// L21 in one more (two launches per narrow block instead of five).
//
//   tree    every workgroup (256 threads = one GEMM workgroup's slot, so it can
//           start beside the trailing update; R rows per thread) plays one
//           leaf: NT*R consecutive rows.  It writes its <= 32 winners' row
//           indices and ORIGINAL rows (contiguous, column-major per level) with
//           agent-scope `sc1` stores, waits for them and adds to its group's
//           counter; the workgroup whose add comes last plays the group's node
//           on the F = NT*R/32 children's candidates (coalesced sc1 loads of the
//           level's slab instead of a strided gather from A), and so on up the
//           tree -- no relaunch per level.  The root writes the LU of the
//           winners into the top block, U11^{-1}, ipiv and the net row moves.
//           Leaf 0 keeps the top block's original rows (the rows the moves
//           displace below it) before anything overwrites them.
//   step    (GEPP on the rows held in VGPRs) every thread picks the best of its
//           R rows (32-bit fp32 key, as v1), ONE wave max, a ballot names the
//           winning lane, which publishes its row (columns >= k only) and
//           {key, thread-row, global row} to the wave's double-buffered LDS
//           slot; ONE barrier; every thread takes the max of the wave keys and
//           the lowest wave holding it (one ballot).  The next step's key comes
//           from an approximate update (v_rcp without Newton steps) and the
//           exact update is branch-free (l = 0 for inactive rows), so the
//           scheduler can overlap it with the next wave max.  No global memory
//           access inside the step loop (the v1 kernel stored its winner every
//           step and waited for the store before the next key).
//   finish  blocks [0, rgrid): L21 = A21 U11^{-1} on MFMA for rows below the
//           top block (displaced rows read from leaf 0's copy); the other
//           blocks apply the row moves to the panel columns outside the
//           narrow block; the last block also updates perm.
template <typename T> struct Tslu2Rows { static constexpr int R = 2; };
template <> struct Tslu2Rows<float> { static constexpr int R = 4; };
template <> struct Tslu2Rows<cplx<double>> { static constexpr int R = 1; };

constexpr int T2_NT = 256;
constexpr int T2_MOVES = 256;            // ints: [0] count, [2, 66) dst, [66, 130) src
constexpr int T2_CTR_MAX = 4096;         // counters (ints), zeroed per panel (tslu_init)

struct Tslu2Args {
    int64_t m, r, lda;
    int nn, nleaf;
    int* cand;      // per tree item: TW candidate rows (global index)
    int* ccnt;      // per tree item: candidate count
    int* ctr;       // group arrival counters (reset to 0 by the last arriver)
    void* slab;     // per level: the items' candidates' original rows, column-major, ld = items * TW
    void* topc;     // TW x TW: original top-block rows (row-major: topc[i*TW + j])
    int64_t* ipiv;
    int* info;
    int64_t info_offset;
    int* moves;
    void* uinv;     // TW x TW, Uinv[i*TW + j] = (U11^{-1})(i, j)
};

template <typename T> __device__ inline T rcp_approx(T d) { return fast_rcp(d); }
template <> __device__ inline double rcp_approx<double>(double d) { return __builtin_amdgcn_rcp(d); }
template <> __device__ inline float rcp_approx<float>(float d) { return __builtin_amdgcn_rcpf(d); }

__device__ inline float opaque(float v) { asm volatile("" :: "v"(v)); return v; }
__device__ inline double opaque(double v) { asm volatile("" :: "v"(v)); return v; }
__device__ inline int opaque(int v) { asm volatile("" :: "v"(v)); return v; }
template <typename R>
__device__ inline cplx<R> opaque(cplx<R> v) { return cplx<R>(opaque(v.re), opaque(v.im)); }

// agent-scope relaxed (sc1) loads / stores: the in-launch hand-off between workgroups
template <typename T> __device__ inline T ld_sc1(const T* q) {
    return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename R> __device__ inline cplx<R> ld_sc1(const cplx<R>* q) {
    const R* r = reinterpret_cast<const R*>(q);
    return cplx<R>(ld_sc1(r), ld_sc1(r + 1));
}
template <typename T> __device__ inline void st_sc1(T* q, T v) {
    __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename R> __device__ inline void st_sc1(cplx<R>* q, cplx<R> v) {
    R* r = reinterpret_cast<R*>(q);
    st_sc1(r, v.re);
    st_sc1(r + 1, v.im);
}

// wave max of a 32-bit key: DPP with bound_ctrl (0 is the identity), so each
// stage folds into one v_max_u32_dpp; the cross-row stages are DPP row
// broadcasts (gfx9 row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2
// and 3): lane 63 ends with the wave max, ONE readlane instead of four plus
// three scalar maxes
__device__ inline uint32_t wave_max_key(uint32_t k) {
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k, 0xB1, 0xF, 0xF, true));    // quad_perm [1,0,3,2]
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k, 0x4E, 0xF, 0xF, true));    // quad_perm [2,3,0,1]
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k, 0x124, 0xF, 0xF, true));   // row_ror:4
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k, 0x128, 0xF, 0xF, true));   // row_ror:8
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x142, 0xA, 0xF, false));   // row_bcast:15
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x143, 0xC, 0xF, false));   // row_bcast:31
    return __builtin_amdgcn_readlane(k, 63);
}

// one wave-row publish of columns [K, TW) with 16-byte LDS stores (the
// single-lane ds_write_b64 per element was the step's longest part,
// profiles/r5_tslu_v2.txt): all values first (opaque() pins them, and a
// store between two asm statements cannot be paired), then the stores
template <int K, typename T>
__device__ inline void publish_row(T* dst, const T (&v)[TW]) {
    if constexpr (!is_cplx<T>::value && (sizeof(T) == 8 || sizeof(T) == 4)) {
        constexpr int VEC = 16 / sizeof(T);
        using V = T __attribute__((ext_vector_type(VEC)));
        constexpr int J0 = (K + VEC - 1) / VEC * VEC;
        #pragma unroll
        for (int j = K; j < J0 && j < TW; ++j) dst[j] = v[j];
        #pragma unroll
        for (int j = J0; j + VEC <= TW; j += VEC) {
            V x;
            #pragma unroll
            for (int e = 0; e < VEC; ++e) x[e] = v[j + e];
            *reinterpret_cast<V*>(dst + j) = x;
        }
    } else {
        #pragma unroll
        for (int j = K; j < TW; ++j) dst[j] = v[j];
    }
}

#ifdef TSLU_PROBE
__device__ long long g_tslu_probe[128];
#define TSLU_T(slot)                                                                      \
    do {                                                                                  \
        if (tid == 0 && (level > 0 || blockIdx.x == 0))                                   \
            g_tslu_probe[level * 32 + (slot)] = (long long)__builtin_amdgcn_s_memtime();   \
    } while (0)
#define TSLU_S(k, sub)                                                                    \
    do {                                                                                  \
        if ((k) == 4 || (k) == 20) TSLU_T(((k) == 4 ? 16 : 24) + (sub));                  \
    } while (0)
#else
#define TSLU_T(slot) do {} while (0)
#define TSLU_S(k, sub) do {} while (0)
#endif

// WPE: waves per SIMD the kernel is compiled for (register budget 512 / WPE
// per lane); the fp32 R = 2 variant asks for 4 (<= 128 VGPRs), so its waves
// can start beside the trailing fp32 GEMM's
// NT: threads per workgroup (256: a GEMM workgroup's slot, so a leaf starts
// beside the trailing update; 512: twice the rows per leaf, fan-in 32, one
// tree level fewer for panels up to 32 K rows -- for CUs kept free of the
// update, SLATE_TSLU_NT)
template <typename T, int R, int WPE = 1, int NT = T2_NT>
__global__ __launch_bounds__(NT, WPE) void tslu2_tree_kernel(Tslu2Args p, T* A) {
    SLATE_PANEL_WAVE_PRIO();
    constexpr int NW = NT / 64, S = NT * R, F = S / TW;
    constexpr bool kReal = !is_cplx<T>::value;
    __shared__ int4 srec[2][NW];                 // {key, thread*R + row, global row, -}
    __shared__ alignas(16) T srow[2][NW][TW];    // each wave's best row: columns k ..
    __shared__ int swin[TW], swho[TW];
    __shared__ int s_flag;
    __shared__ T slu[TW][TW + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nn = p.nn;
    const int64_t lda = p.lda;
    T* slab = reinterpret_cast<T*>(p.slab);

    int level = 0, item = blockIdx.x, nl = p.nleaf, off = 0, offprev = 0, nprev = 0;
    while (true) {
        int idx[R];
        bool act[R];
        int chosen[R];
        T a[R][TW];
        const T* pin = slab + (int64_t)offprev * TW * TW;   // the previous level's slab
        const int64_t ldin = (int64_t)nprev * TW;
        #pragma unroll
        for (int i = 0; i < R; ++i) {
            const int s = tid + i * NT;
            idx[i] = 0;
            act[i] = false;
            chosen[i] = -1;
            if (level == 0) {
                const int64_t row = p.r + (int64_t)item * S + s;
                if (row < p.m) { idx[i] = (int)row; act[i] = true; }
                // branch-free loads (clamped addresses, then select)
                const int64_t rs = act[i] ? idx[i] : p.r;
                #pragma unroll
                for (int j = 0; j < TW; ++j) {
                    const T v = A[rs + (j < nn ? j : nn - 1) * lda];
                    a[i][j] = (act[i] && j < nn) ? v : zero<T>();
                }
                if (item == 0 && s < TW) {
                    // original top-block rows: the rows the interchanges displace
                    T* tc = reinterpret_cast<T*>(p.topc) + s * TW;
                    #pragma unroll
                    for (int j = 0; j < TW; ++j) tc[j] = a[i][j];
                }
            } else {
                const int child = item * F + s / TW, k = s % TW;
                if (child < nprev && k < ld_sc1(&p.ccnt[offprev + child])) {
                    idx[i] = ld_sc1(&p.cand[(int64_t)(offprev + child) * TW + k]);
                    act[i] = true;
                }
                const int64_t rs = act[i] ? (int64_t)item * S + s : (int64_t)item * S;
                #pragma unroll
                for (int j = 0; j < TW; ++j) {
                    const T v = ld_sc1(&pin[rs + j * ldin]);
                    a[i][j] = act[i] ? v : zero<T>();
                }
            }
        }

        TSLU_T(0);
        int cnt = 0;
        bool done = false;
        T tn[R];
        #pragma unroll
        for (int i = 0; i < R; ++i) tn[i] = a[i][0];
        const bool root = nl == 1;
        static_for<0, TW>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            constexpr int bf = k & 1;
            if (k < nn && !done) {
                // best of this thread's rows (full fp32 key; ties -> lowest row)
                uint32_t kt = 0u;
                int bi = 0;
                #pragma unroll
                for (int i = 0; i < R; ++i) {
                    const uint32_t key = act[i] ? pivot_key(kReal ? tn[i] : a[i][k]) : 0u;
                    if (key > kt) { kt = key; bi = i; }
                }
                TSLU_S(k, 0);
                const uint32_t kw = wave_max_key(kt);
                TSLU_S(k, 1);
                if (kw != 0u) {
                    const unsigned long long win = __ballot(kt == kw);
                    if (lane == __ffsll((long long)win) - 1) {
                        static_for<0, R>([&](auto ic) {
                            constexpr int i = decltype(ic)::value;
                            if (i == bi) {
                                // opaque() pins each branch's reads of row i: merged
                                // branches would read a dynamically indexed a[bi][j],
                                // which demotes a[][] to scratch memory
                                srec[bf][w] = make_int4((int)kw, tid * R + i, opaque(idx[i]), 0);
                                T v[TW];
                                #pragma unroll
                                for (int j = k; j < TW; ++j) v[j] = opaque(a[i][j]);
                                publish_row<k>(&srow[bf][w][0], v);
                            }
                        });
                    }
                } else if (lane == 0) {
                    srec[bf][w].x = 0;
                }
                TSLU_S(k, 2);
                __syncthreads();
                TSLU_S(k, 3);
                uint32_t kb = (uint32_t)srec[bf][0].x;
                #pragma unroll
                for (int q = 1; q < NW; ++q) kb = max(kb, (uint32_t)srec[bf][q].x);
                if (kb == 0u) {
                    done = true;                       // uniform: no candidates left
                } else {
                    const uint32_t myk = lane < NW ? (uint32_t)srec[bf][lane].x : 0u;
                    const int wb = __ffsll((long long)__ballot(myk == kb)) - 1;   // lowest wave
                    // the pivot row in registers at once (one batch of LDS reads and
                    // one wait, not a read / wait / FMA chain per column and row)
                    T u[TW];
                    #pragma unroll
                    for (int j = k; j < TW; ++j) u[j] = srow[bf][wb][j];
                    const int4 rec = srec[bf][wb];
                    const T d = u[k];
                    TSLU_S(k, 4);
                    if constexpr (kReal && k + 1 < TW) {
                        // approximate next-column values: only the next key uses them
                        const T u1 = u[k + 1];
                        const T r0 = is_zero(d) ? zero<T>() : rcp_approx<T>(d);
                        #pragma unroll
                        for (int i = 0; i < R; ++i) tn[i] = a[i][k + 1] - (a[i][k] * r0) * u1;
                    }
                    TSLU_S(k, 5);
                    #pragma unroll
                    for (int i = 0; i < R; ++i) {
                        const bool hit = tid * R + i == rec.y;
                        act[i] = act[i] && !hit;
                        chosen[i] = hit ? k : chosen[i];
                    }
                    // Branch-free update: inactive rows get l = 0.  A chosen row's
                    // columns >= its step are saved (root) before they change; its
                    // multipliers (columns < its step) are never written again.
                    const T rd = is_zero(d) ? zero<T>() : fast_rcp(d);
                    #pragma unroll
                    for (int i = 0; i < R; ++i) {
                        const T l = act[i] ? a[i][k] * rd : zero<T>();
                        #pragma unroll
                        for (int j = k + 1; j < TW; ++j) a[i][j] -= l * u[j];
                        a[i][k] = act[i] ? l : a[i][k];
                    }
                    TSLU_S(k, 6);
                    if (tid == 0) { swin[k] = rec.z; swho[k] = rec.y; }
                    if (root && tid >= k && tid < TW) slu[k][tid] = srow[bf][wb][tid];
                    cnt = k + 1;
                    if (k < 8 || k == 16 || k == 31) TSLU_T(1 + (k < 8 ? k : (k == 16 ? 8 : 9)));
                }
            }
        });

        TSLU_T(11);
        if (root) {
            // ---- root: outputs for the finish launch -------------------------
            // multipliers of the winners (their U parts were saved at selection)
            #pragma unroll
            for (int i = 0; i < R; ++i)
                if (chosen[i] >= 0) {
                    #pragma unroll
                    for (int j = 0; j < TW; ++j)
                        if (j < chosen[i]) slu[chosen[i]][j] = a[i][j];
                }
            __syncthreads();
            if (w == 0) {
                // LAPACK ipiv and the net row moves (pos <- orig)
                int pos, orig;
                const bool mv = tslu_interchanges((int)p.r, swin, cnt, p.ipiv, pos, orig);
                const unsigned long long bal = __ballot(mv);
                const int slot = __popcll(bal & ((1ull << lane) - 1));
                if (mv) { p.moves[2 + slot] = pos; p.moves[66 + slot] = orig; }
                if (lane == 0) p.moves[0] = __popcll(bal);
            } else if (w == 1) {
                // U11^{-1}, lane j = column j (axpy-form back substitution)
                T x[TW];
                #pragma unroll
                for (int i = 0; i < TW; ++i) x[i] = (i == lane && lane < nn) ? one<T>() : zero<T>();
                #pragma unroll
                for (int k = TW - 1; k >= 0; --k) {
                    if (k < nn) {
                        const T dk = slu[k][k];
                        const T xk = x[k] * (is_zero(dk) ? zero<T>() : fast_rcp(dk));
                        x[k] = xk;
                        #pragma unroll
                        for (int i = 0; i < k; ++i) x[i] -= slu[i][k] * xk;
                    }
                }
                T* U = reinterpret_cast<T*>(p.uinv);
                if (lane < TW) {
                    #pragma unroll
                    for (int i = 0; i < TW; ++i) U[i * TW + lane] = x[i];
                }
            } else {
                // the LU of the winners into the top block; the info flag
                for (int e = tid - 128; e < TW * TW; e += NT - 128) {
                    const int i = e % TW, j = e / TW;
                    if (i < cnt && j < nn) A[p.r + i + j * lda] = slu[i][j];
                }
                if (tid == 128 && p.info) {
                    int bad = -1;
                    for (int k = 0; k < nn; ++k)
                        if (is_zero(slu[k][k])) { bad = k; break; }
                    if (bad >= 0 && *p.info == 0) *p.info = (int)(p.info_offset + p.r + bad + 1);
                }
            }
            TSLU_T(12);
            return;
        }

        // ---- not the root: hand the winners to the group's node --------------
        __syncthreads();
        {
            T* pout = slab + (int64_t)off * TW * TW;
            const int64_t ldout = (int64_t)nl * TW;
            for (int e = tid; e < TW * TW; e += NT) {
                const int k = e % TW, j = e / TW;
                if (k >= cnt) continue;            // (cnt < TW: a narrow last block)
                const int who = swho[k];
                T v;
                if (level == 0) v = j < nn ? A[swin[k] + j * lda] : zero<T>();
                else v = ld_sc1(&pin[(int64_t)item * S + (who / R) + (who % R) * NT + j * ldin]);
                st_sc1(&pout[(int64_t)item * TW + k + j * ldout], v);
            }
        }
        if (tid < cnt) st_sc1(&p.cand[(int64_t)(off + item) * TW + tid], swin[tid]);
        if (tid == 0) st_sc1(&p.ccnt[off + item], cnt);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const int g = item / F, ng = min(F, nl - g * F);
            int* c = &p.ctr[off + nl + g];
            // acq_rel at agent scope: the release publishes this workgroup's
            // winners (stored above) before the count, the acquire makes the
            // other workgroups' winners visible to the last arriver -- the
            // HIP memory model's guarantee, not a gfx9 store-ordering detail
            const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == ng - 1;
            if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_flag = last;
        }
        __syncthreads();
        TSLU_T(13);
        if (!s_flag) return;
        offprev = off;
        nprev = nl;
        off += nl;
        nl = (nl + F - 1) / F;
        item /= F;
        ++level;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void tslu2_finish_kernel(int64_t m, int64_t r, int nn, int64_t c0, T* Ap,
                                                           int64_t lda, int64_t ncols, int rgrid, const int* moves,
                                                           const T* uinv, const T* topc, int64_t* perm) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ int s_dst[64], s_src[64];
    __shared__ T Uinv[TW * TW];
    __shared__ short smap[256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int np = moves[0];
    if (tid < np) { s_dst[tid] = moves[2 + tid]; s_src[tid] = moves[66 + tid]; }
    if (perm && blockIdx.x == gridDim.x - 1 && tid < 64) {
        // net permutation of the panel rows (all loads before any store)
        const int64_t pv = tid < np ? perm[moves[66 + tid]] : 0;
        if (tid < np) perm[moves[2 + tid]] = pv;
    }
    if ((int)blockIdx.x >= rgrid) {
        // row moves on the panel columns outside the narrow block, a column per wave
        __syncthreads();
        const int pb = blockIdx.x - rgrid, pg = gridDim.x - rgrid;
        for (int64_t jj = pb * 4 + w; jj < ncols - nn; jj += (int64_t)pg * 4) {
            const int64_t j = jj < c0 ? jj : jj + nn;
            T* col = Ap + j * lda;
            T v = zero<T>();
            if (lane < np) v = col[s_src[lane]];
            __builtin_amdgcn_wave_barrier();
            if (lane < np) col[s_dst[lane]] = v;
        }
        return;
    }
    T* A = Ap + c0 * lda;
    const int64_t base = r + nn + blockIdx.x * (int64_t)256;
    {
        // all loads, then the LDS stores (a load feeding the same iteration's
        // store waits alone)
        static_assert(TW * TW % 256 == 0, "finish: Uinv staging");
        T u[TW * TW / 256];
        #pragma unroll
        for (int k = 0; k < TW * TW / 256; ++k) u[k] = uinv[tid + 256 * k];
        #pragma unroll
        for (int k = 0; k < TW * TW / 256; ++k) Uinv[tid + 256 * k] = u[k];
    }
    smap[tid] = -1;
    __syncthreads();
    if (tid < np) {
        const int64_t d = s_dst[tid] - base;
        if (s_dst[tid] >= r + nn && d >= 0 && d < 256) smap[d] = (short)tid;
    }
    __syncthreads();
    if constexpr (std::is_same<T, double>::value) {
        double ub[TW / 4][2];
        #pragma unroll
        for (int ks = 0; ks < TW / 4; ++ks)
            #pragma unroll
            for (int nt = 0; nt < 2; ++nt) ub[ks][nt] = Uinv[(ks * 4 + (lane >> 4)) * TW + nt * 16 + (lane & 15)];
        #pragma unroll
        for (int sl = 0; sl < 4; ++sl) {
            const int loc = (w * 4 + sl) * 16 + (lane & 15);
            const int64_t row = base + loc;
            const bool ok = row < m;
            const int e = smap[loc];
            const double* src = e >= 0 ? topc + (s_src[e] - r) * TW : A + row;
            const int64_t sld = e >= 0 ? 1 : lda;
            double av[TW / 4];
            #pragma unroll
            for (int ks = 0; ks < TW / 4; ++ks) {
                const int col = ks * 4 + (lane >> 4);
                av[ks] = (ok && col < nn) ? src[col * sld] : 0.0;
            }
            double c0v[4] = {0, 0, 0, 0}, c1v[4] = {0, 0, 0, 0};
            #pragma unroll
            for (int ks = 0; ks < TW / 4; ++ks) {
                mfma16(ub[ks][0], av[ks], c0v);
                mfma16(ub[ks][1], av[ks], c1v);
            }
            if (ok) {
                #pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int col0 = (lane >> 4) + 4 * q, col1 = 16 + col0;
                    if (col0 < nn) A[row + col0 * lda] = c0v[q];
                    if (col1 < nn) A[row + col1 * lda] = c1v[q];
                }
            }
        }
    } else {
        const int64_t row = base + tid;
        if (row < m) {
            const int e = smap[tid];
            const T* src = e >= 0 ? topc + (s_src[e] - r) * TW : A + row;
            const int64_t sld = e >= 0 ? 1 : lda;
            T av[TW];
            #pragma unroll
            for (int k = 0; k < TW; ++k) av[k] = k < nn ? src[k * sld] : zero<T>();
            #pragma unroll 1
            for (int j = 0; j < nn; ++j) {
                T s = zero<T>();
                #pragma unroll
                for (int k = 0; k < TW; ++k) s += av[k] * Uinv[k * TW + j];
                A[row + j * lda] = s;
            }
        }
    }
}

}  // namespace

// Utop scratch (TW x TW, up to 16-byte scalars) first, then the candidate
// ping-pong buffers and counts (int); sizes in int64 units.
constexpr int64_t kUtopI64 = 2 * TW * TW;

// v2 layout (int64 units): [uinv | top-block copy | moves | counters | item
// counts | candidate rows | per-level slabs of candidate rows (16-byte scalars max)]
constexpr int64_t kT2Uinv = 0, kT2Top = 2 * TW * TW, kT2Moves = kT2Top + 2 * TW * TW;
constexpr int64_t kT2Ctr = kT2Moves + T2_MOVES / 2, kT2Cnt = kT2Ctr + T2_CTR_MAX / 2;

static int64_t tslu2_items_max(int64_t rows) {
    const int64_t nleaf = rows / T2_NT + 1;   // leaves hold >= T2_NT rows
    return 2 * nleaf + 16;                    // every tree level
}

int64_t tslu_workspace(int64_t rows) {
    int64_t nleaf = (rows + TR - 1) / TR;
    int64_t v1 = 2 * kUtopI64 + nleaf * TW + nleaf + 64;
    const int64_t items = tslu2_items_max(rows);
    int64_t v2 = kT2Cnt + (items + items * TW + 2) / 2 + 2 + items * TW * TW * 2 + 64;
    return std::max(v1, v2);
}

void tslu_init(int64_t* work, hipStream_t s) {
    (void)hipMemsetAsync(work + kT2Ctr, 0, T2_CTR_MAX * sizeof(int), s);
}

// Which tournament: v2 (one tree launch + one finish launch) for fp64, where
// it measured dgetrf n = 65536 56.4 -> 58.0 TFLOP/s and the isolated
// 32768 x 512 panel 3.71 -> 2.96 ms, and for fp32 with two rows per thread
// at <= 128 VGPRs (round 6: the dgesv_mixed fp32 factor 1876 ms (v1) ->
// 1849 ms; the round-5 four-row v2, whose 256-VGPR waves wait for a whole
// GEMM slot, 2039 ms, profiles/r6_cfg5_tslu_ab.txt); v1 (per-level
// launches) for complex, where v2 spills.  SLATE_TSLU=1|2 forces one.
template <typename T>
static bool tslu_use_v2() {
    static const int forced = [] {
        const char* e = std::getenv("SLATE_TSLU");
        if (!e) e = std::getenv("SLATE_TSLU_V1") ? "1" : nullptr;
        return e ? std::atoi(e) : 0;
    }();
    if (forced) return forced == 2;
    return std::is_same<T, double>::value || std::is_same<T, float>::value;
}

template <typename T, int R = Tslu2Rows<T>::R, int WPE = 1, int NT = T2_NT>
static void tslu2_narrow_launch(int64_t m, int64_t r, int nn, T* Ablk, T* Apanel, int64_t lda, int64_t ncols,
                         int64_t* ipiv, int64_t* perm, int* info, int64_t info_offset, int64_t* work, hipStream_t s) {
    constexpr int S = NT * R;
    const int64_t rows = m - r;
    Tslu2Args p;
    p.m = m; p.r = r; p.lda = lda; p.nn = nn;
    p.nleaf = (int)((rows + S - 1) / S);
    int64_t items = 0;
    for (int64_t n = p.nleaf; ; n = (n + S / TW - 1) / (S / TW)) { items += n; if (n == 1) break; }
    if (items + 1 > T2_CTR_MAX || items > tslu2_items_max(m))
        throw std::runtime_error("tslu: panel too tall for the tournament workspace");
    p.uinv = work + kT2Uinv;
    p.topc = work + kT2Top;
    p.moves = reinterpret_cast<int*>(work + kT2Moves);
    p.ctr = reinterpret_cast<int*>(work + kT2Ctr);
    p.ccnt = reinterpret_cast<int*>(work + kT2Cnt);
    p.cand = p.ccnt + items + 1;
    p.slab = work + kT2Cnt + (items + items * TW + 2) / 2 + 2;
    p.ipiv = ipiv; p.info = info; p.info_offset = info_offset;
    hipLaunchKernelGGL((tslu2_tree_kernel<T, R, WPE, NT>), dim3(p.nleaf), dim3(NT), 0, s, p, Ablk);
    if (hipError_t e = hipGetLastError(); e != hipSuccess)
        throw std::runtime_error(std::string("tslu tree kernel launch: ") + hipGetErrorString(e));
    const int64_t c0 = (Ablk - Apanel) / lda;
    const int rgrid = (int)std::max<int64_t>(0, (rows - nn + 255) / 256);
    const int pgrid = ncols > nn ? (int)std::min<int64_t>((ncols - nn + 3) / 4, 128) : 0;
    hipLaunchKernelGGL(tslu2_finish_kernel<T>, dim3(std::max(1, rgrid + pgrid)), dim3(256), 0, s, m, r, nn, c0,
                       Apanel, lda, ncols, rgrid, (const int*)p.moves, (const T*)p.uinv, (const T*)p.topc, perm);
    if (hipError_t e = hipGetLastError(); e != hipSuccess)
        throw std::runtime_error(std::string("tslu finish kernel launch: ") + hipGetErrorString(e));
}

template <typename T>
void tslu_narrow(int64_t m, int64_t r, int nn, T* Ablk, T* Apanel, int64_t lda, int64_t ncols,
                 int64_t* ipiv, int64_t* perm, int* info, int64_t info_offset, int64_t* work, hipStream_t s) {
    int64_t rows = m - r;
    if (rows <= 0 || nn <= 0) return;
    if (tslu_use_v2<T>()) {
        // fp32: two rows per thread at <= 128 VGPRs (default; SLATE_TSLU_F32_R=4:
        // four rows per thread, 256-VGPR waves that wait for a whole GEMM slot)
        static const bool f32_small = [] {
            const char* e = std::getenv("SLATE_TSLU_F32_R");
            return !e || std::atoi(e) == 2;
        }();
        // SLATE_TSLU_NT: tree workgroup size (fp64; fp32 at two rows per
        // thread).  512 by default when CUs are reserved for the panel
        // queues (the one-process-per-GPU default):
        // whole-CU leaves then find free CUs, and the tree is one level
        // shallower -- 2 x 4 / nb 256 LU model 175.8 -> 188.0 TFLOP/s; 256
        // otherwise, where a whole-CU leaf waits for the trailing GEMM to
        // drain a CU (1-GPU dgetrf 59.0 -> 55.0) (profiles/r6_tslu_nt.txt)
        static const int nt = [] {
            const char* e = std::getenv("SLATE_TSLU_NT");
            if (e) return std::atoi(e);
            return slate::device::reserved_cus() > 0 ? 512 : T2_NT;
        }();
        if constexpr (std::is_same<T, float>::value) {
            if (f32_small) {
                // SLATE_TSLU_F32_WPE: register budget of the 256-thread tree --
                // 2 (default): <= 256 VGPRs, 169 used, no spill; 4: <= 128
                // VGPRs, 180 bytes of scratch.  Config-5 fp32 factor 1852 ->
                // 1800 ms on one GPU (profiles/r6_f32_nt.txt)
                static const int f32_wpe = [] {
                    const char* e = std::getenv("SLATE_TSLU_F32_WPE");
                    return e ? std::atoi(e) : 2;
                }();
                if (nt == 512)
                    tslu2_narrow_launch<T, 2, 2, 512>(m, r, nn, Ablk, Apanel, lda, ncols, ipiv, perm, info, info_offset,
                                                      work, s);
                else if (f32_wpe == 2)
                    tslu2_narrow_launch<T, 2, 2>(m, r, nn, Ablk, Apanel, lda, ncols, ipiv, perm, info, info_offset, work,
                                                 s);
                else
                    tslu2_narrow_launch<T, 2, 4>(m, r, nn, Ablk, Apanel, lda, ncols, ipiv, perm, info, info_offset, work,
                                                 s);
                return;
            }
        }
        // SLATE_TSLU_NT512_ROWS: also 512 for panels of at most this many rows
        // (a short panel's trailing update no longer fills the GPU)
        static const int64_t nt512_rows = [] {
            const char* e = std::getenv("SLATE_TSLU_NT512_ROWS");
            return e ? std::atoll(e) : int64_t(0);
        }();
        if constexpr (std::is_same<T, double>::value) {
            if (nt == 512 || rows <= nt512_rows) {
                tslu2_narrow_launch<T, Tslu2Rows<T>::R, 1, 512>(m, r, nn, Ablk, Apanel, lda, ncols, ipiv, perm, info,
                                                                info_offset, work, s);
                return;
            }
        }
        tslu2_narrow_launch<T>(m, r, nn, Ablk, Apanel, lda, ncols, ipiv, perm, info, info_offset, work, s);
        return;
    }
    const int64_t nleaf_max = (rows + TR - 1) / TR;
    T* Utop = reinterpret_cast<T*>(work);
    T* LU11 = reinterpret_cast<T*>(work + kUtopI64);      // final round's LU of the winners
    int* candA = reinterpret_cast<int*>(work + 2 * kUtopI64);
    int* candB = candA + nleaf_max * TW;
    int* cntA = candB + nleaf_max * TW;
    int* cntB = cntA + nleaf_max + 1;
    const int nleaf = (int)nleaf_max;
    hipLaunchKernelGGL((tslu_select_kernel<T, TR>), dim3(nleaf), dim3(TR), 0, s, m, r, nn, Ablk, lda,
                       (const int*)nullptr, (const int*)nullptr, 0, candA, cntA, nleaf == 1 ? LU11 : nullptr);
    int n = nleaf;
    while (n > 1) {
        int n2 = (n + FANIN - 1) / FANIN;
        hipLaunchKernelGGL((tslu_select_kernel<T, NODE_NT>), dim3(n2), dim3(NODE_NT), 0, s, m, r, nn, Ablk, lda,
                           (const int*)candA, (const int*)cntA, n, candB, cntB, n2 == 1 ? LU11 : nullptr);
        std::swap(candA, candB);
        std::swap(cntA, cntB);
        n = n2;
    }
    const T* lu_final = LU11;
    const int64_t c0 = (Ablk - Apanel) / lda;
    const int pgrid = (int)std::min<int64_t>((ncols + 3) / 4, 1024);
    hipLaunchKernelGGL(tslu_permute_kernel<T>, dim3(pgrid), dim3(256), 0, s, (int)r, nn, c0, Apanel, lda, ncols,
                       (const int*)candA, (const int*)cntA, ipiv, perm, Utop);
    const int rgrid = (int)std::max<int64_t>(1, (rows - nn + 255) / 256);
    hipLaunchKernelGGL(tslu_rows_kernel<T>, dim3(rgrid), dim3(256), 0, s, m, r, nn, Ablk, lda, (const T*)Utop,
                       lu_final, info, info_offset);
}

#define SLATE_INST_TSLU(T) \
    template void tslu_narrow<T>(int64_t, int64_t, int, T*, T*, int64_t, int64_t, int64_t*, int64_t*, int*, int64_t, int64_t*, hipStream_t);

SLATE_INST_TSLU(double)
#ifndef TSLU_PROBE
SLATE_INST_TSLU(float)
SLATE_INST_TSLU(cplx<float>)
SLATE_INST_TSLU(cplx<double>)
#endif

}  // namespace dev
}  // namespace slate_amd
