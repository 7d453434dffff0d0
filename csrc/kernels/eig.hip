// Device helpers of the two-stage eigensolver back-transform (unmtr_hb2st).
//
// The hb2st reflectors of kd consecutive sweeps at one bulge step form a block
// V (2 kd x kd) with H_1 ... H_kd = I - V T V^H.  T^{-1} = striu(V^H V) +
// diag(1 / tau) (the UT-transform identity behind LAPACK larft), so the
// application only needs the Gram matrix V^H V (one GEMM) turned into T^{-1}
// in place by this kernel, and a triangular solve.  A zero reflector (tau = 0,
// v = 0) gets a unit diagonal: its column of V is zero, so it contributes
// nothing.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

template <typename T>
__global__ __launch_bounds__(256) void tinv_from_gram_kernel(int64_t k, T* G, int64_t ldg, const T* tau) {
    for (int64_t idx = blockIdx.x * 256 + threadIdx.x; idx < k * k; idx += 256 * (int64_t)gridDim.x) {
        const int64_t i = idx % k, j = idx / k;
        if (i > j) G[i + j * ldg] = T();
        else if (i == j) {
            const T t = tau[i];
            G[i + j * ldg] = is_zero(t) ? make_val<T>(1.0) : make_val<T>(1.0) / t;
        }
    }
}

// ---- bdsqr / steqr rotations on the device.  Every row of M is
// independent; one thread owns one row and walks the columns once per batch
// of K QR sweeps with a register window of 2K columns: at step tau, sweep s
// applies its rotation at column pair (j, j + 1), j = tau - 2 s.  Sweep s at j
// only needs sweep s - 1 to be done with column j + 1, which happened at step
// tau - 1, so the K rotations of one step touch disjoint pairs and are
// independent (ILP instead of a K-long dependency chain).  Each column is read
// and written once per batch instead of once per sweep.  With only n rows
// (n / 64 waves for the whole chip) a step cannot hide an HBM round trip
// behind other waves, so the column a step needs is loaded PF steps ahead into
// a register ring.  D holds the rotations in step order: D[2 (tau - p0) K +
// 2 s + {0, 1}] = (c, s) of sweep s at step tau (identity where sweep s has no
// rotation); the step's 2K reals are wave-uniform loads.
// [x y] <- [c x - s y, s x + c y] on columns [p0, p1).
template <typename T, typename R>
struct RotJob {
    int64_t rows;
    T* M;
    int64_t ld, p0, p1;
    const R* D;
};

template <typename T, typename R, int K, int PF>
__device__ inline void rot_sweeps_row(RotJob<T, R> const& J, int64_t r, R* sD) {
    // sD: this wave's LDS ring, 2 x PF steps x 2K reals.  The step tables are
    // the same for every lane, so a block of PF steps is loaded once per wave
    // with coalesced vector loads (8 reals per lane) one block ahead, and each
    // step reads its 2K coefficients from LDS as broadcasts -- instead of 2K
    // wave-uniform global loads per step, whose latency a lone wave per CU
    // cannot hide.
    constexpr int BLK = PF * 2 * K, PER = BLK / 64;
    const int lane = threadIdx.x & 63;
    const bool live = r < J.rows;
    T* row = J.M + (live ? r : 0);
    const int64_t ld = J.ld, p0 = J.p0, p1 = J.p1;
    const R* D = J.D;
    const int64_t tend = p1 - 2 + 2 * (K - 1);
    const int64_t dtot = (tend - p0 + 1) * 2 * K;   // reals of the table in use
    R nxt[PER];
    auto fetch = [&](int64_t t0) {
        const int64_t base = (t0 - p0) * 2 * K;
        #pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int64_t idx = base + lane + 64 * i;
            nxt[i] = idx < dtot ? D[idx] : R(0);
        }
    };
    auto stash = [&](int buf) {
        #pragma unroll
        for (int i = 0; i < PER; ++i) sD[buf * BLK + lane + 64 * i] = nxt[i];
    };
    fetch(p0);
    stash(0);
    __syncthreads();
    T w[2 * K];
    #pragma unroll
    for (int i = 0; i < 2 * K; ++i) w[i] = T();
    if (live) {
        w[2 * K - 2] = row[p0 * ld];
        w[2 * K - 1] = (p0 + 1 < p1) ? row[(p0 + 1) * ld] : T();
    }
    T pf[PF];
    #pragma unroll
    for (int i = 0; i < PF; ++i) {
        const int64_t cpf = p0 + 2 + i;
        pf[i] = (live && cpf < p1) ? row[cpf * ld] : T();
    }
    int cur = 0;
    for (int64_t t0 = p0; t0 <= tend; t0 += PF) {
        if (t0 + PF <= tend) fetch(t0 + PF);
        const R* cb = sD + cur * BLK;
        #pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int64_t tau = t0 + u;
            if (tau > tend) break;
            const R* cs = cb + 2 * K * u;
            #pragma unroll
            for (int s = 0; s < K; ++s) {
                const R c = cs[2 * s], sn = cs[2 * s + 1];
                const T x = w[2 * K - 2 - 2 * s], y = w[2 * K - 1 - 2 * s];
                w[2 * K - 2 - 2 * s] = x * c - y * sn;
                w[2 * K - 1 - 2 * s] = x * sn + y * c;
            }
            const int64_t cr = tau - 2 * K + 2;
            if (live && cr >= p0) row[cr * ld] = w[0];
            #pragma unroll
            for (int i = 0; i < 2 * K - 1; ++i) w[i] = w[i + 1];
            w[2 * K - 1] = pf[u];                         // column tau + 2
            const int64_t cn = tau + 2 + PF;
            pf[u] = (live && cn < p1) ? row[cn * ld] : T();
        }
        if (t0 + PF <= tend) stash(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    if (live && p1 - 1 >= p0) row[(p1 - 1) * ld] = w[0];
}

constexpr int kRotPrefetch = 16;

// two independent jobs (U and Vt of bdsqr) in one launch: blocks [0, nblk_a)
// take job a, the rest job b
template <typename T, typename R, int K>
__global__ __launch_bounds__(64) void rot_sweeps_kernel(RotJob<T, R> a, RotJob<T, R> b, int64_t nblk_a) {
    __shared__ R sD[2 * kRotPrefetch * 2 * K];
    const bool first = int64_t(blockIdx.x) < nblk_a;
    const int64_t r = (first ? int64_t(blockIdx.x) : int64_t(blockIdx.x) - nblk_a) * 64 + threadIdx.x;
    // (every lane of the wave takes part in the table loads; rows past the
    // end only skip their matrix accesses)
    if (first) rot_sweeps_row<T, R, K, kRotPrefetch>(a, r, sD);
    else rot_sweeps_row<T, R, K, kRotPrefetch>(b, r, sD);
}

// one rotation on columns (a, b): [x y] <- [x c + y s, y c - x s]
template <typename T, typename R>
__global__ __launch_bounds__(256) void rot_cols_kernel(int64_t rows, T* M, int64_t ld, int64_t a, int64_t b, R c,
                                                       R s) {
    const int64_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const T x = M[r + a * ld], y = M[r + b * ld];
    M[r + a * ld] = x * c + y * s;
    M[r + b * ld] = y * c - x * s;
}

}  // namespace

template <typename T>
void rot_sweeps(int64_t rows, T* M, int64_t ld, int64_t p0, int64_t p1, const rt<T>* D, hipStream_t s) {
    rot_sweeps2(rows, M, ld, p0, p1, D, int64_t(0), static_cast<T*>(nullptr), int64_t(1), int64_t(0), int64_t(0),
                static_cast<const rt<T>*>(nullptr), s);
}

template <typename T>
void rot_sweeps2(int64_t rows_a, T* A, int64_t lda, int64_t pa0, int64_t pa1, const rt<T>* Da, int64_t rows_b, T* B,
                 int64_t ldb, int64_t pb0, int64_t pb1, const rt<T>* Db, hipStream_t s) {
    const bool ua = rows_a > 0 && A && pa1 - pa0 >= 2, ub = rows_b > 0 && B && pb1 - pb0 >= 2;
    if (!ua && !ub) return;
    RotJob<T, rt<T>> ja{ua ? rows_a : 0, A, lda, pa0, pa1, Da}, jb{ub ? rows_b : 0, B, ldb, pb0, pb1, Db};
    const int64_t na = (ja.rows + 63) / 64, nbk = (jb.rows + 63) / 64;
    // (neither a four-wave variant of this kernel -- the 16 sweeps split over
    // the SIMDs of a CU, columns handed between waves through LDS -- nor
    // multishift rounds in the host loop made bdsqr faster: svd n = 8192
    // bdsqr 1.44 s here against 2.17 s (four waves, even with an LDS-only
    // barrier and the handoff read ahead) and 1.80-1.97 s (two / three
    // shifts: cheaper host sweeps, but more of them for this kernel, which
    // already takes about as long as the host loop); profiles/r4_rot_pipe_ab.txt)
    hipLaunchKernelGGL((rot_sweeps_kernel<T, rt<T>, kRotBatch>), dim3((unsigned)(na + nbk)), dim3(64), 0, s, ja, jb,
                       na);
}

template <typename T>
void rot_cols(int64_t rows, T* M, int64_t ld, int64_t a, int64_t b, rt<T> c, rt<T> sn, hipStream_t s) {
    if (rows <= 0) return;
    hipLaunchKernelGGL((rot_cols_kernel<T, rt<T>>), dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, rows, M,
                       ld, a, b, c, sn);
}

template <typename T>
void tinv_from_gram(int64_t k, T* G, int64_t ldg, const T* tau, hipStream_t s) {
    if (k <= 0) return;
    const unsigned nb = (unsigned)std::min<int64_t>((k * k + 255) / 256, 256);
    hipLaunchKernelGGL(tinv_from_gram_kernel<T>, dim3(nb), dim3(256), 0, s, k, G, ldg, tau);
}

#define SLATE_INST_EIG(T)                                                                                          \
    template void tinv_from_gram<T>(int64_t, T*, int64_t, const T*, hipStream_t);                                 \
    template void rot_sweeps<T>(int64_t, T*, int64_t, int64_t, int64_t, const rt<T>*, hipStream_t);             \
    template void rot_sweeps2<T>(int64_t, T*, int64_t, int64_t, int64_t, const rt<T>*, int64_t, T*, int64_t,     \
                                 int64_t, int64_t, const rt<T>*, hipStream_t);                                  \
    template void rot_cols<T>(int64_t, T*, int64_t, int64_t, int64_t, rt<T>, rt<T>, hipStream_t);

SLATE_INST_EIG(float)
SLATE_INST_EIG(double)
SLATE_INST_EIG(cplx<float>)
SLATE_INST_EIG(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
