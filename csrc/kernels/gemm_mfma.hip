// MFMA GEMM for gfx950: C = alpha * op(A) * op(B) + beta * C  (real types).
//
// Replaces the reference's batched vendor gemm (src/internal/internal_gemm.cc:498,
// blas::batch::gemm over nb x nb tiles) with ONE large local GEMM per call:
// trailing updates in the drivers hand us the whole local sub-matrix.
//
// CDNA4 design:
//  * fp64: v_mfma_f64_16x16x4_f64 (64 cyc/SIMD, 2048 flop), fp32:
//    v_mfma_f32_16x16x4_f32 (32 cyc/SIMD).  One wave owns a 64x64 sub-tile =
//    4x4 MFMA tiles = 16 independent accumulator chains, so one wave per SIMD
//    already issues back-to-back.
//  * 256-thread workgroup (4 waves, 2x2) per 128x128 C tile, BK=16, LDS
//    double buffer with register prefetch (one barrier per K-tile).  fp64
//    products with a K-contiguous operand use 8 waves of 64x32 instead
//    (4 waves per SIMD at <= 128 VGPRs; see launch_gemm).
//  * Interior-only instantiation when every tile is full (no bounds-checked
//    path competing for registers); rotated K pipeline for fp64 (the last
//    k-step's MFMAs issue after the barrier, behind the next LDS reads).
//  * LDS image is [k][m] with row stride BM+16 elements: the MFMA operand
//    read (lanes 0-15 consecutive m, lanes 16-31 next k) then lands the two
//    16-lane halves on disjoint bank halves (ds_read_b64: bank=(a/4)%64).
//  * Operands are swapped in the MFMA (D = B^T A^T) so that the accumulator's
//    lane index runs along M: the column-major epilogue stores 16 consecutive
//    rows (128 B for fp64) per column instead of 4.
//  * XCD-aware grouped tile order (blocks b, b+8 share an L2).
#include "device_common.hh"
#include "kernels.hh"

#include <cstdlib>
#include <type_traits>

// lab switches (A/B builds of the standalone harness)
#ifndef GEMM_SPLIT
#define GEMM_SPLIT 1
#endif
#ifndef GEMM_JB
#define GEMM_JB 2
#endif
#ifndef GEMM_ROT
#define GEMM_ROT true
#endif

namespace slate_amd {
namespace dev {

template <typename T> struct Mfma;

template <> struct Mfma<double> {
    using acc_t = double __attribute__((ext_vector_type(4)));
    __device__ static inline acc_t run(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // C/D layout of v_mfma_f64_16x16x4_f64: col = lane&15, row = (lane>>4) + 4*reg
    __device__ static inline int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

template <> struct Mfma<float> {
    using acc_t = float __attribute__((ext_vector_type(4)));
    __device__ static inline acc_t run(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // C/D layout of v_mfma_f32_16x16x4_f32: col = lane&15, row = 4*(lane>>4) + reg
    __device__ static inline int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

// LDS row skew: row r of an operand image starts at r*LD + lds_skew(r).  A
// K-contiguous operand is transposed on its way into LDS; with a plain row
// stride (BM+16, a multiple of 32 dwords) the BK/VEC lanes that share a column
// write rows on the same bank (ds_write: bank = (addr/4)%32) - an 8-way (fp64)
// / 4-way (fp32) store conflict.  The skew spreads those rows over distinct
// banks while keeping the two rows an MFMA operand read touches per 32-lane
// group (r, r+1 with r even / r%4 < 2) on disjoint bank halves, and it is a
// per-row constant, so operand reads keep immediate address offsets.
template <typename T>
__device__ __forceinline__ constexpr int lds_skew(int r) {
    return sizeof(T) == 8 ? (r & ~1) : 8 * (r >> 2);
}

// Load a BX x BK operand tile into registers. Element (x, kk) of the operand
// lives at X[x*sx + kk*sk]; KCONTIG means sk == 1 (else sx == 1).
template <typename T, int BX, int BK, bool KCONTIG, int NTHR = 256>
struct TileLoader {
    static constexpr int VEC = 16 / sizeof(T);
    static constexpr int NV  = BX * BK / VEC;   // vectors per tile
    static constexpr int NVT = NV / NTHR;       // vectors per thread
    static_assert(NV % NTHR == 0, "tile must split evenly over the workgroup");
    T r[NVT][VEC];

    __device__ inline void coords(int v, int& x, int& kk) const {
        if constexpr (KCONTIG) {
            constexpr int KV = BK / VEC;
            kk = (v % KV) * VEC;
            x  = v / KV;
        } else {
            constexpr int XV = BX / VEC;
            x  = (v % XV) * VEC;
            kk = v / XV;
        }
    }

    __device__ inline void load(const T* __restrict__ X, int64_t ld, int64_t x0, int64_t k0,
                                int64_t xdim, int64_t kdim, bool fast) {
        const int tid = threadIdx.x;
        if (fast) {
            load_fast(X, ld, x0, k0);
        } else {
            #pragma unroll
            for (int i = 0; i < NVT; ++i) {
                int x, kk;
                coords(tid + NTHR * i, x, kk);
                #pragma unroll
                for (int e = 0; e < VEC; ++e) {
                    int64_t gx = x0 + x + (KCONTIG ? 0 : e);
                    int64_t gk = k0 + kk + (KCONTIG ? e : 0);
                    r[i][e] = (gx < xdim && gk < kdim)
                            ? (KCONTIG ? X[gk + gx * ld] : X[gx + gk * ld]) : T(0);
                }
            }
        }
    }

    /// Vector loads only (tile fully inside the operand, 16-B aligned).
    __device__ inline void load_fast(const T* __restrict__ X, int64_t ld, int64_t x0, int64_t k0) {
        const int tid = threadIdx.x;
        {
            #pragma unroll
            for (int i = 0; i < NVT; ++i) {
                int x, kk;
                coords(tid + NTHR * i, x, kk);
                const T* p = KCONTIG ? X + (k0 + kk) + (x0 + x) * ld
                                     : X + (x0 + x) + (k0 + kk) * ld;
                if constexpr (sizeof(T) == 8) {
                    using v2 = double __attribute__((ext_vector_type(2)));
                    v2 t = *reinterpret_cast<const v2*>(p);
                    r[i][0] = t[0]; r[i][1] = t[1];
                } else {
                    using v4 = float __attribute__((ext_vector_type(4)));
                    v4 t = *reinterpret_cast<const v4*>(p);
                    r[i][0] = t[0]; r[i][1] = t[1]; r[i][2] = t[2]; r[i][3] = t[3];
                }
            }
        }
    }

    static constexpr int elems(int LD) { return BK * LD + 32; }   // + max skew
    __device__ static inline int at(int LD, int x, int kr) { return kr * LD + lds_skew<T>(kr) + x; }

    // LDS image offsets of this thread's vectors (element units), computed
    // once: row kk at kk*LD + lds_skew(kk), column x.  A K-contiguous vector
    // spans VEC rows, all with the same skew (kk is a multiple of VEC), so
    // its elements sit at soff + e*LD.  Keeping one register per vector
    // (instead of re-deriving x, kk and the skew each K-tile) keeps the
    // 8-wave kernel within its 128-VGPR budget.
    int soff[NVT];
    template <int LD>
    __device__ inline void init_store() {
        const int tid = threadIdx.x;
        #pragma unroll
        for (int i = 0; i < NVT; ++i) {
            int x, kk;
            coords(tid + NTHR * i, x, kk);
            soff[i] = kk * LD + lds_skew<T>(kk) + x;
        }
    }

    template <int LD>
    __device__ inline void store(T* L) const {
        #pragma unroll
        for (int i = 0; i < NVT; ++i) {
            if constexpr (KCONTIG) {
                #pragma unroll
                for (int e = 0; e < VEC; ++e)
                    L[soff[i] + e * LD] = r[i][e];
            } else {
                // the skew is a multiple of VEC: the vector stays aligned
                #pragma unroll
                for (int e = 0; e < VEC; ++e)
                    L[soff[i] + e] = r[i][e];
            }
        }
    }
};

// Epilogue shared by the MFMA GEMM kernels: lane&15 runs along M (contiguous
// in column-major C).  For beta != 0 the C values of two accumulator columns
// are loaded together before any store so the loads overlap.
// First valid row (relative to C's row 0) of C's column gn under a StairMap.
__device__ inline int64_t stair_row0(StairMap const& sm, int64_t gn) {
    const int64_t lc = sm.c0 + gn;
    const int64_t lt = lc / sm.nb, o = lc - lt * sm.nb;
    const int64_t J = lt * sm.q + sm.pcol;                       // global tile of the column
    const int64_t li = J > sm.prow ? (J - sm.prow + sm.p - 1) / sm.p : 0;   // first local row tile >= J
    return li * sm.nb + (li * sm.p + sm.prow == J ? o : 0) - sm.r0;
}

template <typename T, int TM, int TN, char TRI>
__device__ inline void gemm_epilogue(typename Mfma<T>::acc_t (&acc)[TM][TN], int64_t m, int64_t n, T alpha,
                                     T beta, T* __restrict__ C, int64_t ldc, int64_t wm0, int64_t wn0, int lane,
                                     StairMap const& sm) {
    using M = Mfma<T>;
    const bool beta_zero = (beta == T(0));
    constexpr int JB = GEMM_JB;
    auto inside = [&](int64_t gm, int64_t gn) {
        bool in = gm < m && gn < n;
        if constexpr (TRI == 'L') in = in && gm >= gn;
        if constexpr (TRI == 'U') in = in && gm <= gn;
        if constexpr (TRI == 'S') in = in && gm >= stair_row0(sm, gn);
        return in;
    };
    #pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int64_t gm = wm0 + i * 16 + (lane & 15);
        #pragma unroll
        for (int j0 = 0; j0 < TN; j0 += JB) {
            T cv[JB][4];
            #pragma unroll
            for (int j = 0; j < JB; ++j)
                #pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t gn = wn0 + (j0 + j) * 16 + M::row(lane, r);
                    cv[j][r] = (!beta_zero && inside(gm, gn)) ? C[gm + gn * ldc] : T(0);
                }
            #pragma unroll
            for (int j = 0; j < JB; ++j)
                #pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t gn = wn0 + (j0 + j) * 16 + M::row(lane, r);
                    if (inside(gm, gn)) {
                        T v = alpha * acc[i][j0 + j][r];
                        if (!beta_zero) v += beta * cv[j][r];
                        C[gm + gn * ldc] = v;
                    }
                }
        }
    }
}

// Tile order: XCD-aware bijective remap, then GROUP tile-rows at a time.
__device__ inline void gemm_tile_coords(int64_t m, int64_t n, int BM, int BN, int& tm, int& tn) {
    const int mt = (int)((m + BM - 1) / BM), nt = (int)((n + BN - 1) / BN);
    const int nblk = mt * nt;
    int bid = xcd_remap(blockIdx.x, nblk);
    constexpr int GROUP = 8;
    int group = bid / (GROUP * nt);
    int first_m = group * GROUP;
    int gsize = min(mt - first_m, GROUP);
    int within = bid % (GROUP * nt);
    tm = first_m + within % gsize;
    tn = within / gsize;
}

// TRI: 0 = full C; 'L' / 'U' = only the lower / upper triangle of a square C
// is computed (tiles outside it are never launched; diagonal tiles are masked).
// NTHR = 64 * (BM/64) * (BN/64): one wave per 64 x 64 sub-tile.  128 x 128
// (4 waves, 2 workgroups per CU) or 256 x 128 (8 waves, 1 workgroup per CU:
// 25% less operand traffic per flop for large C).
template <typename T, int BM, int BN, int BK, bool A_KC, bool B_KC, char TRI, int WTN_ = 64, int WTM_ = 64,
          bool ROT = false, bool IONLY = false>
__global__ __launch_bounds__(64 * (BM / WTM_) * (BN / WTN_),
    (2 * BK * (BM + BN + 32) * sizeof(T) > 81920) ? 1
        : (BM == 128 && BN == 128 && 64 * (BM / WTM_) * (BN / WTN_) == 512) ? 4
        : 512 / (64 * (BM / WTM_) * (BN / WTN_)))
void gemm_mfma_kernel(int64_t m, int64_t n, int64_t k, T alpha,
                      const T* __restrict__ A, int64_t lda, int64_t sA,
                      const T* __restrict__ B, int64_t ldb, int64_t sB,
                      T beta, T* __restrict__ C, int64_t ldc, int64_t sC,
                      bool aligned, StairMap sm)
{
    using M = Mfma<T>;
    using acc_t = typename M::acc_t;
    constexpr int PAD = 16;
    constexpr int LDA_S = BM + PAD, LDB_S = BN + PAD;
    constexpr int WTM = WTM_, WTN = WTN_;           // per-wave tile
    constexpr int WN = BN / WTN;                     // waves along N
    constexpr int NTHR = 64 * (BM / WTM) * WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;     // MFMA tiles per wave
    using LA = TileLoader<T, BM, BK, A_KC, NTHR>;
    using LB = TileLoader<T, BN, BK, B_KC, NTHR>;
    constexpr int A_ELEMS = LA::elems(LDA_S), B_ELEMS = LB::elems(LDB_S);

    __shared__ __attribute__((aligned(16))) T smem[2 * (A_ELEMS + B_ELEMS)];

    // batch offset
    const int64_t bz = blockIdx.y;
    A += bz * sA; B += bz * sB; C += bz * sC;

    // tile coordinates: XCD remap, then grouped order (GROUP tile-rows)
    const int mt = (int)((m + BM - 1) / BM), nt = (int)((n + BN - 1) / BN);
    int tm, tn;
    if constexpr (TRI == 0 || TRI == 'S') {
        const int nblk = mt * nt;
        int bid = xcd_remap(blockIdx.x, nblk);
        constexpr int GROUP = 8;
        int group = bid / (GROUP * nt);
        int first_m = group * GROUP;
        int gsize = min(mt - first_m, GROUP);
        int within = bid % (GROUP * nt);
        tm = first_m + within % gsize;
        tn = within / gsize;
    } else {
        // triangular enumeration: row r holds r+1 tiles (BM == BN, mt == nt)
        const int nblk = mt * (mt + 1) / 2;
        int t = xcd_remap(blockIdx.x, nblk);
        int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while ((r + 1) * (r + 2) / 2 <= t) ++r;
        while (r * (r + 1) / 2 > t) --r;
        int c = t - r * (r + 1) / 2;
        if constexpr (TRI == 'L') { tm = r; tn = c; } else { tm = c; tn = r; }
    }
    const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
    if constexpr (TRI == 'S') {
        // tiles wholly above the staircase do nothing (the row start is
        // nondecreasing along the local columns, so column n0 has the lowest)
        if (stair_row0(sm, n0) >= m0 + BM) return;
        // this tile's B^T rows: its local column tile's slab in the operand
        const int64_t lc = sm.c0 + n0;
        B += sm.btab[lc / sm.nb - sm.c0 / sm.nb] + (lc % sm.nb) - n0;
    }

    const int lane = threadIdx.x & 63;
    const int wid  = threadIdx.x >> 6;
    const int wm = wid / WN, wn = wid % WN;

    acc_t acc[TM][TN];
    #pragma unroll
    for (int i = 0; i < TM; ++i)
        #pragma unroll
        for (int j = 0; j < TN; ++j)
            acc[i][j] = acc_t{0, 0, 0, 0};

    LA la;
    LB lb;
    la.template init_store<LDA_S>();
    lb.template init_store<LDB_S>();
    const bool mfull = (m0 + BM <= m), nfull = (n0 + BN <= n);

    const int KT = (int)((k + BK - 1) / BK);
    // Interior tiles (the common case) run a K loop with vector loads only;
    // edge tiles take the bounds-checked loop.  Keeping the two apart keeps
    // the checked path's 64-bit index math out of the hot loop's registers.
    auto kloop = [&](auto interior_tag) {
    constexpr bool INTERIOR = decltype(interior_tag)::value;
    auto load_a = [&](int64_t k0, bool kfull) {
        if constexpr (INTERIOR) la.load_fast(A, lda, m0, k0);
        else la.load(A, lda, m0, k0, m, k, aligned && mfull && kfull);
    };
    auto load_b = [&](int64_t k0, bool kfull) {
        if constexpr (INTERIOR) lb.load_fast(B, ldb, n0, k0);
        else lb.load(B, ldb, n0, k0, n, k, aligned && nfull && kfull);
    };
    if (KT > 0) {
        bool kfull = (BK <= k);
        load_a(0, kfull);
        load_b(0, kfull);
        la.template store<LDA_S>(smem);
        lb.template store<LDB_S>(smem + A_ELEMS);
        __syncthreads();
    }

    // MFMA operand fragments are double-buffered in registers: the LDS reads
    // of k-step s+1 are issued before the MFMAs of step s, so the LDS latency
    // hides behind 16 MFMAs instead of stalling every step.
    auto frag = [&](const T* As, const T* Bs, int s, T (&a)[TM], T (&b)[TN]) {
        const int kr = s * 4 + (lane >> 4);
        #pragma unroll
        for (int i = 0; i < TM; ++i)
            a[i] = As[LA::at(LDA_S, wm * WTM + i * 16 + (lane & 15), kr)];
        #pragma unroll
        for (int j = 0; j < TN; ++j)
            b[j] = Bs[LB::at(LDB_S, wn * WTN + j * 16 + (lane & 15), kr)];
    };
    auto mfma_step = [&](const T (&a)[TM], const T (&b)[TN]) {
        #pragma unroll
        for (int i = 0; i < TM; ++i)
            #pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[i][j] = M::run(b[j], a[i], acc[i][j]);
    };
    if constexpr (ROT) {
        // Rotated pipeline: the last k-step's MFMAs of tile kt are issued
        // AFTER the barrier, behind the LDS reads of tile kt+1's first step,
        // so the post-barrier LDS latency hides under 16 MFMAs instead of
        // idling the matrix pipe once per K-tile.
        T fa[2][TM], fb[2][TN];
        if (KT > 0) frag(smem, smem + A_ELEMS, 0, fa[0], fb[0]);
        for (int kt = 0; kt < KT; ++kt) {
            const int cur = kt & 1;
            const bool more = (kt + 1 < KT);
            if (more) {
                int64_t k0 = (int64_t)(kt + 1) * BK;
                bool kfull = (k0 + BK <= k);
                load_a(k0, kfull);
                load_b(k0, kfull);
            }
            const T* As = smem + cur * (A_ELEMS + B_ELEMS);
            const T* Bs = As + A_ELEMS;
            #pragma unroll
            for (int s = 0; s < BK / 4 - 1; ++s) {
                frag(As, Bs, s + 1, fa[(s + 1) & 1], fb[(s + 1) & 1]);
                mfma_step(fa[s & 1], fb[s & 1]);
            }
            constexpr int LAST = (BK / 4 - 1) & 1;
            if (more) {
                T* Asn = smem + (cur ^ 1) * (A_ELEMS + B_ELEMS);
                la.template store<LDA_S>(Asn);
                lb.template store<LDB_S>(Asn + A_ELEMS);
            }
            __syncthreads();
            if (more) {
                const T* An = smem + (cur ^ 1) * (A_ELEMS + B_ELEMS);
                frag(An, An + A_ELEMS, 0, fa[LAST ^ 1], fb[LAST ^ 1]);
            }
            mfma_step(fa[LAST], fb[LAST]);
        }
    } else {
    for (int kt = 0; kt < KT; ++kt) {
        const int cur = kt & 1;
        const bool more = (kt + 1 < KT);
        if (more) {
            int64_t k0 = (int64_t)(kt + 1) * BK;
            bool kfull = (k0 + BK <= k);
            load_a(k0, kfull);
            load_b(k0, kfull);
        }
        const T* As = smem + cur * (A_ELEMS + B_ELEMS);
        const T* Bs = As + A_ELEMS;
        #pragma unroll
        for (int s = 0; s < BK / 4; ++s) {
            T a[TM], b[TN];
            frag(As, Bs, s, a, b);
            mfma_step(a, b);
        }
        if (more) {
            T* Asn = smem + (cur ^ 1) * (A_ELEMS + B_ELEMS);
            la.template store<LDA_S>(Asn);
            lb.template store<LDB_S>(Asn + A_ELEMS);
        }
        __syncthreads();
    }
    }
    };
    if constexpr (IONLY) kloop(std::true_type{});
    else if (GEMM_SPLIT && aligned && mfull && nfull && k % BK == 0) kloop(std::true_type{});
    else kloop(std::false_type{});

    gemm_epilogue<T, TM, TN, TRI>(acc, m, n, alpha, beta, C, ldc, m0 + wm * WTM, n0 + wn * WTN, lane, sm);
}

template <typename T, bool A_KC, bool B_KC, char TRI, int BM, int BN, int BK = 16, int WTN = 64, int WTM = 64,
          bool ROT = (GEMM_ROT && sizeof(T) == 8)>
static void launch_tile(int64_t m, int64_t n, int64_t k, T alpha,
                        const T* A, int64_t lda, int64_t sA,
                        const T* B, int64_t ldb, int64_t sB,
                        T beta, T* C, int64_t ldc, int64_t sC,
                        int64_t batch, bool aligned, hipStream_t stream, StairMap const& sm = StairMap{})
{
    constexpr int NTHR = 64 * (BM / WTM) * (BN / WTN);
    int64_t mt = (m + BM - 1) / BM, nt = (n + BN - 1) / BN;
    int64_t nblk = (TRI == 'L' || TRI == 'U') ? mt * (mt + 1) / 2 : mt * nt;
    dim3 grid((unsigned)nblk, (unsigned)batch);
    // every tile interior (the common case for nb-multiple trailing updates):
    // a kernel without the bounds-checked path, whose registers then go to
    // the hot loop alone
    if (aligned && m % BM == 0 && n % BN == 0 && k % BK == 0 && k > 0)
        hipLaunchKernelGGL((gemm_mfma_kernel<T, BM, BN, BK, A_KC, B_KC, TRI, WTN, WTM, ROT, true>), grid, dim3(NTHR),
                           0, stream, m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, aligned, sm);
    else
        hipLaunchKernelGGL((gemm_mfma_kernel<T, BM, BN, BK, A_KC, B_KC, TRI, WTN, WTM, ROT, false>), grid, dim3(NTHR),
                           0, stream, m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, aligned, sm);
}

// fp32 only: 256 x 128 tiles (8 waves, 1 workgroup per CU) cut operand
// traffic per flop by 25%, worth +5% for large sgemm; measured neutral-to-worse
// for fp64, whose 64-cycle MFMA leaves the 128 x 128 tile compute-bound.
static bool big_tiles(int64_t m, int64_t n, int64_t batch) {
    static int env = [] { const char* e = std::getenv("SLATE_GEMM_BIG"); return e ? std::atoi(e) : 1; }();
    if (!env) return false;
    // only when they still give >= 2 waves of workgroups over 256 CUs
    return m >= 512 && ((m + 255) / 256) * ((n + 127) / 128) * batch >= 512;
}

// Latency-bound products (the panels' and the Cholesky leaves' GEMMs: a few
// hundred rows, K <= 512): fewer 128 x 128 tiles than half the CUs leave
// most of the chip idle while each workgroup walks K alone at one CU's fp64
// MFMA rate (~0.3 TFLOP/s: a 128 x 128 x 64 tile is >= 7 us).  64 x 64 tiles
// (4 waves of 32 x 32) give 4x the workgroups.  SLATE_GEMM_SMALL=0 disables.
static bool small_tiles(int64_t m, int64_t n, int64_t batch, bool tri) {
    static int env = [] { const char* e = std::getenv("SLATE_GEMM_SMALL"); return e ? std::atoi(e) : 1; }();
    if (!env) return false;
    const int64_t mt = (m + 127) / 128, nt = (n + 127) / 128;
    const int64_t tiles = (tri ? mt * (mt + 1) / 2 : mt * nt) * batch;
    return tiles < 128;
}

template <typename T, bool A_KC, bool B_KC, char TRI = 0>
static void launch_gemm(int64_t m, int64_t n, int64_t k, T alpha,
                        const T* A, int64_t lda, int64_t sA,
                        const T* B, int64_t ldb, int64_t sB,
                        T beta, T* C, int64_t ldc, int64_t sC,
                        int64_t batch, hipStream_t stream)
{
    constexpr int VEC = 16 / sizeof(T);
    auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) % 16) == 0; };
    bool aligned = al(A) && al(B) && (lda % VEC == 0) && (ldb % VEC == 0)
                && (batch == 1 || (sA % VEC == 0 && sB % VEC == 0));
    if constexpr (TRI != 'S') {
        if (small_tiles(m, n, batch, TRI != 0)) {
            launch_tile<T, A_KC, B_KC, TRI, 64, 64, 16, 32, 32>(m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc,
                                                                 sC, batch, aligned, stream);
            return;
        }
    }
    if constexpr (TRI == 0 && sizeof(T) == 4) {
        if (big_tiles(m, n, batch)) {
            launch_tile<T, A_KC, B_KC, TRI, 256, 128>(m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC,
                                                      batch, aligned, stream);
            return;
        }
    }
    if constexpr (TRI == 0 && sizeof(T) == 8 && (A_KC || B_KC)) {
        // fp64 with a K-contiguous operand: 8 waves of 64 x 32 per 128 x 128
        // tile (4 waves per SIMD at <= 128 VGPRs, so one wave's barrier or
        // LDS wait is covered by three others).  Measured on 16384^2 x 16384
        // against the 4-wave 64 x 64 tile: NN 68.5 vs 66.9, TN 69.5 vs 67.0
        // TFLOP/s (rotated pipeline on TN only: it spills NN); NT keeps the
        // 4-wave rotated tile (70.4).
        constexpr bool ROT8 = A_KC && B_KC;
        launch_tile<T, A_KC, B_KC, TRI, 128, 128, 16, 32, 64, ROT8>(m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C,
                                                                    ldc, sC, batch, aligned, stream);
    } else {
        launch_tile<T, A_KC, B_KC, TRI, 128, 128>(m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC,
                                                  batch, aligned, stream);
    }
}

template <typename T>
void gemm_real(char transA, char transB, int64_t m, int64_t n, int64_t k,
               T alpha, const T* A, int64_t lda, int64_t sA,
               const T* B, int64_t ldb, int64_t sB,
               T beta, T* C, int64_t ldc, int64_t sC, int64_t batch, hipStream_t stream)
{
    if (m <= 0 || n <= 0 || batch <= 0) return;
    // op(A) = A: contiguous along M; op(A) = A^T: contiguous along K.
    // op(B) = B: contiguous along K; op(B) = B^T: contiguous along N.
    bool a_kc = (transA != 'N'), b_kc = (transB == 'N');
    if (a_kc && b_kc)
        launch_gemm<T, true, true>(m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, stream);
    else if (a_kc)
        launch_gemm<T, true, false>(m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, stream);
    else if (b_kc)
        launch_gemm<T, false, true>(m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, stream);
    else
        launch_gemm<T, false, false>(m, n, k, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, stream);
}

// C(uplo triangle of n x n) = alpha op(A) op(B) + beta C   (herk/syrk/her2k core)
template <typename T>
void gemm_tri_real(char uplo, char transA, char transB, int64_t n, int64_t k,
                   T alpha, const T* A, int64_t lda, const T* B, int64_t ldb,
                   T beta, T* C, int64_t ldc, hipStream_t stream)
{
    if (n <= 0) return;
    bool a_kc = (transA != 'N'), b_kc = (transB == 'N');
#define SLATE_TRI_LAUNCH(U)                                                                   \
    if (a_kc && b_kc) launch_gemm<T, true, true, U>(n, n, k, alpha, A, lda, 0, B, ldb, 0, beta, C, ldc, 0, 1, stream); \
    else if (a_kc)    launch_gemm<T, true, false, U>(n, n, k, alpha, A, lda, 0, B, ldb, 0, beta, C, ldc, 0, 1, stream); \
    else if (b_kc)    launch_gemm<T, false, true, U>(n, n, k, alpha, A, lda, 0, B, ldb, 0, beta, C, ldc, 0, 1, stream); \
    else              launch_gemm<T, false, false, U>(n, n, k, alpha, A, lda, 0, B, ldb, 0, beta, C, ldc, 0, 1, stream);
    if (uplo == 'L') { SLATE_TRI_LAUNCH('L') }
    else { SLATE_TRI_LAUNCH('U') }
#undef SLATE_TRI_LAUNCH
}

// Staircase trailing update of a block-cyclic lower-triangular matrix (p x q
// potrf / herk): one launch over the whole local trailing block instead of one
// GEMM per local tile column; B^T tiles come from wherever the gathered panel
// keeps them (btab).  NT operand form on the 4-wave rotated 128 x 128 tile.
template <typename T>
void gemm_stair_real(int64_t m, int64_t n, int64_t k, T alpha, const T* A, int64_t lda, const T* B, int64_t ldb,
                     StairMap const& sm, T beta, T* C, int64_t ldc, hipStream_t stream)
{
    if (m <= 0 || n <= 0) return;
    constexpr int VEC = 16 / sizeof(T);
    auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) % 16) == 0; };
    bool aligned = al(A) && al(B) && (lda % VEC == 0) && (ldb % VEC == 0) && sm.nb % VEC == 0;
    launch_tile<T, false, false, 'S', 128, 128>(m, n, k, alpha, A, lda, 0, B, ldb, 0, beta, C, ldc, 0, 1,
                                                aligned, stream, sm);
}
template void gemm_stair_real<double>(int64_t, int64_t, int64_t, double, const double*, int64_t, const double*, int64_t,
                                      StairMap const&, double, double*, int64_t, hipStream_t);
template void gemm_stair_real<float>(int64_t, int64_t, int64_t, float, const float*, int64_t, const float*, int64_t,
                                     StairMap const&, float, float*, int64_t, hipStream_t);

// split-K reduction: C = alpha * sum_s P[s] + beta * C (P: splits x m x n, ld m)
template <typename T>
__global__ void splitk_reduce_kernel(int64_t m, int64_t n, int splits, const T* __restrict__ P, T alpha, T beta,
                                     T* __restrict__ C, int64_t ldc) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int64_t j = blockIdx.y;
    if (i >= m) return;
    // four independent partial sums keep several loads in flight
    T s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    const int64_t mn = m * n;
    const T* p = P + i + j * m;
    int b = 0;
    for (; b + 4 <= splits; b += 4) {
        s0 += p[(b + 0) * mn];
        s1 += p[(b + 1) * mn];
        s2 += p[(b + 2) * mn];
        s3 += p[(b + 3) * mn];
    }
    for (; b < splits; ++b) s0 += p[b * mn];
    T s = (s0 + s1) + (s2 + s3);
    T* c = C + i + j * ldc;
    *c = (beta == T(0)) ? alpha * s : alpha * s + beta * (*c);
}

template <typename T>
void splitk_reduce(int64_t m, int64_t n, int splits, const T* P, T alpha, T beta, T* C, int64_t ldc, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    dim3 grid((unsigned)((m + 255) / 256), (unsigned)n);
    hipLaunchKernelGGL(splitk_reduce_kernel<T>, grid, dim3(256), 0, s, m, n, splits, P, alpha, beta, C, ldc);
}
template void splitk_reduce<double>(int64_t, int64_t, int, const double*, double, double, double*, int64_t, hipStream_t);
template void splitk_reduce<float>(int64_t, int64_t, int, const float*, float, float, float*, int64_t, hipStream_t);

template void gemm_tri_real<double>(char, char, char, int64_t, int64_t, double, const double*, int64_t,
                                    const double*, int64_t, double, double*, int64_t, hipStream_t);
template void gemm_tri_real<float>(char, char, char, int64_t, int64_t, float, const float*, int64_t,
                                   const float*, int64_t, float, float*, int64_t, hipStream_t);

template void gemm_real<double>(char, char, int64_t, int64_t, int64_t, double, const double*, int64_t, int64_t,
                                const double*, int64_t, int64_t, double, double*, int64_t, int64_t, int64_t, hipStream_t);
template void gemm_real<float>(char, char, int64_t, int64_t, int64_t, float, const float*, int64_t, int64_t,
                               const float*, int64_t, int64_t, float, float*, int64_t, int64_t, int64_t, hipStream_t);

}  // namespace dev
}  // namespace slate_amd
