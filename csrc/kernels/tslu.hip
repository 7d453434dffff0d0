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
//   select  leaves: 256 rows per workgroup, one row per lane held in VGPRs;
//           GEPP with a DPP (quad_perm/row_ror) + v_readlane wave argmax and
//           an LDS broadcast of the pivot row.
//   select  tree nodes: 512-lane workgroups, fan-in 16 (16 x 32 candidates).
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
#include <type_traits>

namespace slate_amd {
namespace dev {

namespace {

constexpr int TW = 32;        // tournament / narrow-block width
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

// One tournament round: each workgroup factors up to NT rows x nn columns with
// partial pivoting and emits its (up to nn) pivot rows, in pivot order.
// Leaves (cand_in == nullptr) take rows [r + NT*b, ...); nodes take the
// candidate lists of NT/TW children.  Rows are read from the unmodified panel
// (CALU plays every round on original rows).
template <typename T, int NT>
__global__ __launch_bounds__(NT) void tslu_select_kernel(int64_t m, int64_t r, int nn, const T* A, int64_t lda,
                                                         const int* cand_in, const int* cnt_in, int nin,
                                                         int* cand_out, int* cnt_out) {
    SLATE_PANEL_WAVE_PRIO();
    using R = real_t<T>;
    constexpr int NW = NT / 64;
    __shared__ R sv[2][NW];
    __shared__ int si[2][NW];
    __shared__ T prow[2][TW];
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

    // (guarded, not `break`: the loop must fully unroll so a[] stays in VGPRs)
    int cnt = 0;
    bool done = false;
    #pragma unroll
    for (int k = 0; k < TW; ++k) {
        if (k < nn && !done) {
            R v = act ? abs1(a[k]) : R(-1);
            int id = act ? idx : INT_MAX;
            wave_argmax(v, id);
            if (lane == 0) { sv[k & 1][w] = v; si[k & 1][w] = id; }
            __syncthreads();
            v = sv[k & 1][0]; id = si[k & 1][0];
            #pragma unroll
            for (int q = 1; q < NW; ++q) argmax_pick(v, id, sv[k & 1][q], si[k & 1][q]);
            if (id == INT_MAX) {
                done = true;                       // uniform: no candidates left
            } else {
                if (act && idx == id) {
                    #pragma unroll
                    for (int j = k; j < TW; ++j) prow[k & 1][j] = a[j];
                    act = false;
                }
                __syncthreads();
                if (act) {
                    T d = prow[k & 1][k];
                    T l = a[k] * (is_zero(d) ? zero<T>() : one<T>() / d);
                    #pragma unroll
                    for (int j = k + 1; j < TW; ++j) a[j] -= l * prow[k & 1][j];
                }
                if (tid == 0) cand_out[blockIdx.x * TW + k] = id;
                cnt = k + 1;
            }
        }
    }
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
// broadcasts) and column-oriented inverse of U11 (lane j = column j of
// U11^{-1}, back substitution).  Writes Uinv[i*TW + j] (zero outside the nn x
// nn triangle); returns the first zero pivot (or -1).
template <typename T>
__device__ inline int tslu_top_factor(int nn, const T* Utop, T (&a)[TW], T* Uinv) {
    const int tid = threadIdx.x & 63;
    const bool live = tid < nn;
    #pragma unroll
    for (int j = 0; j < TW; ++j) a[j] = (live && j < nn) ? Utop[j * TW + tid] : zero<T>();
    int bad = -1;
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
    T x[TW];
    #pragma unroll
    for (int i = TW - 1; i >= 0; --i) {
        x[i] = zero<T>();
        if (i < nn) {
            T s = (i == tid) ? one<T>() : zero<T>();
            #pragma unroll
            for (int k = i + 1; k < TW; ++k)
                if (k < nn) s -= bcast_lane(a[k], i) * x[k];
            T d = bcast_lane(a[i], i);
            x[i] = is_zero(d) ? zero<T>() : s / d;
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
                                                        const T* Utop, int* info, int64_t info_offset) {
    SLATE_PANEL_WAVE_PRIO();
    __shared__ T Uinv[TW * TW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (w == 0) {
        T a[TW];
        int bad = tslu_top_factor<T>(nn, Utop, a, Uinv);
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
    return kUtopI64 + nleaf * TW + nleaf + 64;
}

template <typename T>
void tslu_narrow(int64_t m, int64_t r, int nn, T* Ablk, T* Apanel, int64_t lda, int64_t ncols,
                 int64_t* ipiv, int64_t* perm, int* info, int64_t info_offset, int64_t* work, hipStream_t s) {
    int64_t rows = m - r;
    if (rows <= 0 || nn <= 0) return;
    int nleaf = (int)((rows + TR - 1) / TR);
    T* Utop = reinterpret_cast<T*>(work);
    int* candA = reinterpret_cast<int*>(work + kUtopI64);
    int* candB = candA + (int64_t)nleaf * TW;
    int* cntA = candB + (int64_t)nleaf * TW;
    int* cntB = cntA + nleaf + 1;
    hipLaunchKernelGGL((tslu_select_kernel<T, TR>), dim3(nleaf), dim3(TR), 0, s, m, r, nn, Ablk, lda,
                       (const int*)nullptr, (const int*)nullptr, 0, candA, cntA);
    int n = nleaf;
    while (n > 1) {
        int n2 = (n + FANIN - 1) / FANIN;
        hipLaunchKernelGGL((tslu_select_kernel<T, NODE_NT>), dim3(n2), dim3(NODE_NT), 0, s, m, r, nn, Ablk, lda,
                           (const int*)candA, (const int*)cntA, n, candB, cntB);
        std::swap(candA, candB);
        std::swap(cntA, cntB);
        n = n2;
    }
    const int64_t c0 = (Ablk - Apanel) / lda;
    const int pgrid = (int)std::min<int64_t>((ncols + 3) / 4, 1024);
    hipLaunchKernelGGL(tslu_permute_kernel<T>, dim3(pgrid), dim3(256), 0, s, (int)r, nn, c0, Apanel, lda, ncols,
                       (const int*)candA, (const int*)cntA, ipiv, perm, Utop);
    const int rgrid = (int)std::max<int64_t>(1, (rows - nn + 255) / 256);
    hipLaunchKernelGGL(tslu_rows_kernel<T>, dim3(rgrid), dim3(256), 0, s, m, r, nn, Ablk, lda, (const T*)Utop, info,
                       info_offset);
}

#define SLATE_INST_TSLU(T) \
    template void tslu_narrow<T>(int64_t, int64_t, int, T*, T*, int64_t, int64_t, int64_t*, int64_t*, int*, int64_t, int64_t*, hipStream_t);

SLATE_INST_TSLU(float)
SLATE_INST_TSLU(double)
SLATE_INST_TSLU(cplx<float>)
SLATE_INST_TSLU(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
