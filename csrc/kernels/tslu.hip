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

#include <climits>
#include <cstdlib>
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

}  // namespace

// Utop scratch (TW x TW, up to 16-byte scalars) first, then the candidate
// ping-pong buffers and counts (int); sizes in int64 units.
constexpr int64_t kUtopI64 = 2 * TW * TW;

int64_t tslu_workspace(int64_t rows) {
    int64_t nleaf = (rows + TR - 1) / TR;
    return 2 * kUtopI64 + nleaf * TW + nleaf + 64;
}

template <typename T>
void tslu_narrow(int64_t m, int64_t r, int nn, T* Ablk, T* Apanel, int64_t lda, int64_t ncols,
                 int64_t* ipiv, int64_t* perm, int* info, int64_t info_offset, int64_t* work, hipStream_t s) {
    int64_t rows = m - r;
    if (rows <= 0 || nn <= 0) return;
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

SLATE_INST_TSLU(float)
SLATE_INST_TSLU(double)
SLATE_INST_TSLU(cplx<float>)
SLATE_INST_TSLU(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
