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
// costs a handful of launches instead of two launches per column:
//   select (leaves: 256 rows per workgroup, one row per lane, rows held in
//          VGPRs; GEPP with wave argmax + LDS broadcast of the pivot row)
//   select (tree nodes: fan-in 8 -> 8*32 = 256 candidate rows per workgroup)
//   pivots (one wave: turn the winners into LAPACK ipiv + a (dst,src) row
//           permutation, wave-parallel with ballot/readlane)
//   permute_rows (aux.hip) over the whole panel width
//   top    (top 32x32 block LU without pivoting in one wave via readlane)
//   rows   (L21 = A21 U11^{-1}, one row per lane with U11 in LDS)
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

constexpr int TW = 32;    // tournament / narrow-block width
constexpr int TR = 256;   // rows per workgroup
constexpr int FANIN = TR / TW;

template <typename R>
__device__ inline void argmax_pick(R& v, int64_t& idx, R ov, int64_t oi) {
    // max |v|; ties -> smaller row index (deterministic, LAPACK-like)
    if (ov > v || (ov == v && oi < idx) || (isnan(ov) && !isnan(v))) { v = ov; idx = oi; }
}

// One tournament round: each workgroup factors up to 256 rows x nn columns with
// partial pivoting and emits its (up to nn) pivot rows, in pivot order.
// Leaves (cand_in == nullptr) take rows [r + 256*b, ...); nodes take the
// candidate lists of FANIN children.  Rows are read from the unmodified panel
// (CALU plays every round on original rows).
template <typename T>
__global__ __launch_bounds__(TR) void tslu_select_kernel(int64_t m, int64_t r, int nn, const T* A, int64_t lda,
                                                         const int64_t* cand_in, const int* cnt_in, int nin,
                                                         int64_t* cand_out, int* cnt_out) {
    using R = real_t<T>;
    __shared__ R sv[2][TR / 64];
    __shared__ int64_t si[2][TR / 64];
    __shared__ T prow[2][TW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int64_t idx = -1;
    bool act = false;
    if (cand_in == nullptr) {
        int64_t i = r + blockIdx.x * (int64_t)TR + tid;
        if (i < m) { idx = i; act = true; }
    } else {
        int child = blockIdx.x * FANIN + tid / TW, k = tid % TW;
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
            int64_t id = act ? idx : INT64_MAX;
            #pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                R ov = __shfl_xor(v, off, 64);
                int64_t oi = __shfl_xor(id, off, 64);
                argmax_pick(v, id, ov, oi);
            }
            if (lane == 0) { sv[k & 1][w] = v; si[k & 1][w] = id; }
            __syncthreads();
            v = sv[k & 1][0]; id = si[k & 1][0];
            #pragma unroll
            for (int q = 1; q < TR / 64; ++q) argmax_pick(v, id, sv[k & 1][q], si[k & 1][q]);
            if (id == INT64_MAX) {
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
// row permutation as (dst, src) pairs.  One wave: lanes 0..31 track positions
// r..r+31, lanes 32..63 the winners that lie below; interchanges are swaps of
// the `orig` register between two lanes.
template <typename T>
__global__ __launch_bounds__(64) void tslu_pivots_kernel(int64_t r, const int64_t* win, const int* wcnt,
                                                         int64_t* ipiv, int64_t* perm,
                                                         int64_t* pdst, int64_t* psrc, int* npairs) {
    const int l = threadIdx.x;
    const int cnt = *wcnt;
    int64_t wl = (l & 31) < cnt ? win[l & 31] : -1;
    int64_t pos = -1;
    if (l < 32) { if (l < cnt) pos = r + l; }
    else if (l - 32 < cnt && wl >= r + cnt) pos = wl;
    int64_t orig = pos;
    for (int k = 0; k < cnt; ++k) {
        int64_t wk = __shfl(wl, k, 64);
        unsigned long long bal = __ballot(pos >= 0 && orig == wk);
        int ql = __ffsll(bal) - 1;
        int64_t q = __shfl(pos, ql, 64);
        if (l == 0) ipiv[r + k] = q;
        int64_t ok = __shfl(orig, k, 64), oq = __shfl(orig, ql, 64);
        if (l == ql) orig = ok;
        if (l == k) orig = oq;
    }
    bool mv = pos >= 0 && pos != orig;
    unsigned long long bal = __ballot(mv);
    int slot = __popcll(bal & ((1ull << l) - 1));
    int64_t pv = (mv && perm) ? perm[orig] : 0;
    if (mv) {
        pdst[slot] = pos; psrc[slot] = orig;
        if (perm) perm[pos] = pv;
    }
    if (l == 0) *npairs = __popcll(bal);
}

// After the winners were permuted to rows r..r+nn-1: factor the top nn x nn
// block in place without pivoting (one wave, lane i = row r+i, pivot-row
// entries broadcast with v_readlane) and publish U11 + 1/diag to Uws.
template <typename T>
__global__ __launch_bounds__(64) void tslu_top_kernel(int64_t r, int nn, T* A, int64_t lda, T* Uws,
                                                      int* info, int64_t info_offset) {
    const int tid = threadIdx.x;
    T a[TW];
    bool live = tid < nn;
    #pragma unroll
    for (int j = 0; j < TW; ++j) a[j] = (live && j < nn) ? A[r + tid + j * lda] : zero<T>();
    int bad = -1;
    #pragma unroll
    for (int k = 0; k < TW; ++k) {
        if (k < nn) {
            T d = bcast_lane(a[k], k);
            if (is_zero(d) && bad < 0) bad = k;
            T rd = is_zero(d) ? zero<T>() : one<T>() / d;
            if (tid == 0) Uws[TW * TW + k] = rd;
            T lk = a[k] * rd;
            #pragma unroll
            for (int j = k + 1; j < TW; ++j) {
                T ukj = bcast_lane(a[j], k);
                if (tid > k) a[j] -= lk * ukj;
            }
            if (tid > k) a[k] = lk;
        }
    }
    if (live) {
        #pragma unroll
        for (int j = 0; j < TW; ++j) {
            Uws[tid * TW + j] = a[j];
            if (j < nn) A[r + tid + j * lda] = a[j];
        }
    }
    if (tid == 0 && bad >= 0 && info && *info == 0) *info = (int)(info_offset + r + bad + 1);
}

// L21 = A21 U11^{-1}: one row per lane, forward substitution against U11 in LDS.
template <typename T>
__global__ __launch_bounds__(TR) void tslu_rows_kernel(int64_t m, int64_t r, int nn, T* A, int64_t lda,
                                                       const T* Uws) {
    __shared__ T U[TW][TW];
    __shared__ T rdiag[TW];
    const int tid = threadIdx.x;
    for (int e = tid; e < TW * TW; e += TR) {
        int k = e / TW, j = e % TW;
        U[k][j] = (k < nn && j > k && j < nn) ? Uws[k * TW + j] : zero<T>();
    }
    if (tid < TW) rdiag[tid] = tid < nn ? Uws[TW * TW + tid] : zero<T>();
    __syncthreads();
    int64_t i = r + nn + blockIdx.x * (int64_t)TR + tid;
    if (i >= m) return;
    T a[TW];
    #pragma unroll
    for (int j = 0; j < TW; ++j) a[j] = j < nn ? A[i + j * lda] : zero<T>();
    // k is a runtime loop (a fully unrolled 32x32 triangle makes the compiler
    // hoist ~500 LDS loads and spill); a[k] is picked with a select chain.
    #pragma unroll 1
    for (int k = 0; k < nn; ++k) {
        T ak = a[0];
        #pragma unroll
        for (int j = 1; j < TW; ++j) ak = (j == k) ? a[j] : ak;
        T lk = ak * rdiag[k];
        #pragma unroll
        for (int j = 0; j < TW; ++j) {
            T u = U[k][j];                           // zero for j <= k
            a[j] = (j == k) ? lk : a[j] - lk * u;
        }
    }
    #pragma unroll
    for (int j = 0; j < TW; ++j) if (j < nn) A[i + j * lda] = a[j];
}

}  // namespace

// U11 + 1/diag (up to 16-byte scalars) first, then candidate ping-pong
// buffers, counts and the (dst, src) pairs; in int64 units.
constexpr int64_t kUwsI64 = 2 * TW * (TW + 1);

int64_t tslu_workspace(int64_t rows) {
    int64_t nleaf = (rows + TR - 1) / TR;
    return kUwsI64 + 2 * nleaf * TW + nleaf + 2 + 2 * 2 * TW + 1;
}

template <typename T>
void tslu_narrow(int64_t m, int64_t r, int nn, T* Ablk, T* Apanel, int64_t lda, int64_t ncols,
                 int64_t* ipiv, int64_t* perm, int* info, int64_t info_offset, int64_t* work, hipStream_t s) {
    int64_t rows = m - r;
    if (rows <= 0 || nn <= 0) return;
    int nleaf = (int)((rows + TR - 1) / TR);
    T* Uws = reinterpret_cast<T*>(work);
    int64_t* candA = work + kUwsI64;
    int64_t* candB = candA + (int64_t)nleaf * TW;
    int* cntA = reinterpret_cast<int*>(candB + (int64_t)nleaf * TW);
    int* cntB = cntA + nleaf;
    int64_t* pdst = candB + (int64_t)nleaf * TW + nleaf + 2;
    int64_t* psrc = pdst + 2 * TW;
    int* npairs = reinterpret_cast<int*>(psrc + 2 * TW);
    hipLaunchKernelGGL(tslu_select_kernel<T>, dim3(nleaf), dim3(TR), 0, s, m, r, nn, Ablk, lda,
                       (const int64_t*)nullptr, (const int*)nullptr, 0, candA, cntA);
    int n = nleaf;
    while (n > 1) {
        int nn2 = (n + FANIN - 1) / FANIN;
        hipLaunchKernelGGL(tslu_select_kernel<T>, dim3(nn2), dim3(TR), 0, s, m, r, nn, Ablk, lda,
                           (const int64_t*)candA, (const int*)cntA, n, candB, cntB);
        std::swap(candA, candB);
        std::swap(cntA, cntB);
        n = nn2;
    }
    hipLaunchKernelGGL(tslu_pivots_kernel<T>, dim3(1), dim3(64), 0, s, r, (const int64_t*)candA, (const int*)cntA,
                       ipiv, perm, pdst, psrc, npairs);
    permute_rows<T>(ncols, Apanel, lda, pdst, psrc, npairs, 2 * TW, s);
    hipLaunchKernelGGL(tslu_top_kernel<T>, dim3(1), dim3(64), 0, s, r, nn, Ablk, lda, Uws, info, info_offset);
    if (rows > nn)
        hipLaunchKernelGGL(tslu_rows_kernel<T>, dim3((unsigned)((rows - nn + TR - 1) / TR)), dim3(TR), 0, s, m, r, nn,
                           Ablk, lda, (const T*)Uws);
}

#define SLATE_INST_TSLU(T) \
    template void tslu_narrow<T>(int64_t, int64_t, int, T*, T*, int64_t, int64_t, int64_t*, int64_t*, int*, int64_t, int64_t*, hipStream_t);

SLATE_INST_TSLU(float)
SLATE_INST_TSLU(double)
SLATE_INST_TSLU(cplx<float>)
SLATE_INST_TSLU(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
