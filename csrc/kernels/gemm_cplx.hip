// Complex GEMM on the gfx950 matrix cores (c/z precisions):
//     C = alpha op(A) op(B) + beta C,   op in {N, T, C},
// with an optional triangular store mask (uplo 'L'/'U') for herk/her2k/syrk.
//
// Reference behaviour: batched vendor zgemm/cgemm over nb x nb tiles
// (src/internal/internal_gemm.cc:498, internal_herk.cc:491-515).
//
// CDNA4 design: a complex multiply-add is four real products,
//     Cr += Ar Br - Ai Bi,   Ci += Ar Bi + Ai Br,
// so each 16 x 16 complex output tile keeps TWO MFMA accumulators (re, im)
// and every k-step issues four v_mfma_f64_16x16x4 (zgemm) / f32_16x16x4
// (cgemm): (Ar,Br) and (Ai,-Bi) into re, (Ar,Bi) and (Ai,Br) into im.  No
// flop is wasted (a complex FMA is 8 real flops = 4 real FMAs).
//  * Global -> LDS: 16-B (z) / 8-B (c) complex loads; the tile is split into
//    separate real and imaginary planes [k][x] in LDS (conjugation = sign flip
//    of the imaginary plane on the way in), so MFMA operands are plain
//    ds_read of one real.
//  * 256-thread workgroup = 2 x 2 waves, 64 x 64 complex C tile (the byte
//    footprint of the real kernel's 128 x 128 fp64 tile), each wave 32 x 32 =
//    2 x 2 MFMA tiles x (re, im); BK = 16, LDS double buffer with register
//    prefetch of the next K-tile (one barrier per K-tile).
//  * Operands swapped in the MFMA (as in gemm_mfma.hip) so the accumulator's
//    lane index runs along M for column-major stores; XCD-aware tile order.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

template <typename R> struct CMfma;
template <> struct CMfma<double> {
    using acc_t = double __attribute__((ext_vector_type(4)));
    __device__ static inline acc_t run(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    __device__ static inline int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <> struct CMfma<float> {
    using acc_t = float __attribute__((ext_vector_type(4)));
    __device__ static inline acc_t run(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    __device__ static inline int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

constexpr int CBM = 64, CBN = 64, CBK = 8, CPAD = 16;
constexpr int CLD = CBM + CPAD;          // LDS row stride (reals) of a plane [k][x]
// row kk starts at kk * CLD + 2 * kk: the skew spreads the 16 rows a
// k-contiguous (transposed) tile store writes per column over distinct banks
__device__ __forceinline__ constexpr int cl_at(int kk, int x) { return kk * (CLD + 2) + x; }
constexpr int NTHR = 256;
constexpr int EPT = CBM * CBK / NTHR;    // complex elements per thread per operand tile (4)

// Operand tile loader: element (x, kk) of the op-applied BX(=64) x CBK tile.
// XC: x contiguous (X[x + kk*ld]) else k contiguous (X[kk + x*ld]); CONJ
// negates the imaginary part; CHECK bounds-checks (edge tiles only).  Each
// thread loads EPT complex values (one 16-B / 8-B load each).
template <typename R, bool XC, bool CONJ, bool CHECK>
struct CLoader {
    cplx<R> v[EPT];
    __device__ static inline void coords(int e, int& x, int& kk) {
        const int id = threadIdx.x + NTHR * e;
        if (XC) { x = id % CBM; kk = id / CBM; }
        else { kk = id % CBK; x = id / CBK; }
    }
    __device__ inline void load(const cplx<R>* __restrict__ X, int64_t ld, int64_t x0, int64_t k0, int64_t xdim,
                                int64_t kdim) {
        #pragma unroll
        for (int e = 0; e < EPT; ++e) {
            int x, kk;
            coords(e, x, kk);
            const int64_t gx = x0 + x, gk = k0 + kk;
            cplx<R> t(R(0), R(0));
            if (!CHECK || (gx < xdim && gk < kdim)) t = XC ? X[gx + gk * ld] : X[gk + gx * ld];
            if (CONJ) t.im = -t.im;
            v[e] = t;
        }
    }
    __device__ inline void store(R* Pr, R* Pi) const {
        #pragma unroll
        for (int e = 0; e < EPT; ++e) {
            int x, kk;
            coords(e, x, kk);
            Pr[cl_at(kk, x)] = v[e].re;
            Pi[cl_at(kk, x)] = v[e].im;
        }
    }
};

template <typename R, char TRI, char TA, char TB, bool CHECK>
__global__ __launch_bounds__(NTHR, 4) void gemm_cplx_mfma_kernel(int64_t m, int64_t n, int64_t k,
                                                                 cplx<R> alpha, const cplx<R>* __restrict__ A,
                                                                 int64_t lda, const cplx<R>* __restrict__ B,
                                                                 int64_t ldb, cplx<R> beta, cplx<R>* __restrict__ C,
                                                                 int64_t ldc) {
    using M = CMfma<R>;
    using acc_t = typename M::acc_t;
    constexpr int PLANE = CBK * (CLD + 2);
    // [buffer][A re, A im, B re, B im][plane]
    __shared__ __attribute__((aligned(16))) R smem[2][4][PLANE];

    const int mt = (int)((m + CBM - 1) / CBM), nt = (int)((n + CBN - 1) / CBN);
    int tm, tn;
    if constexpr (TRI == 0) {
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
        const int nblk = mt * (mt + 1) / 2;
        int t = xcd_remap(blockIdx.x, nblk);
        int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while ((r + 1) * (r + 2) / 2 <= t) ++r;
        while (r * (r + 1) / 2 > t) --r;
        int c = t - r * (r + 1) / 2;
        if constexpr (TRI == 'L') { tm = r; tn = c; } else { tm = c; tn = r; }
    }
    const int64_t m0 = (int64_t)tm * CBM, n0 = (int64_t)tn * CBN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = (w & 1) * 32, wn = (w >> 1) * 32;     // wave sub-tile origin in the C tile

    acc_t cr[2][2], ci[2][2];
    #pragma unroll
    for (int i = 0; i < 2; ++i)
        #pragma unroll
        for (int j = 0; j < 2; ++j) { cr[i][j] = acc_t{0, 0, 0, 0}; ci[i][j] = acc_t{0, 0, 0, 0}; }

    // op(A) (m x k) is loaded with x = row: A 'N' is x-contiguous; op(B) (k x n)
    // with x = column: B 'N' is k-contiguous, B 'T' / 'C' x-contiguous
    CLoader<R, TA == 'N', TA == 'C', CHECK> la;
    CLoader<R, TB != 'N', TB == 'C', CHECK> lb;
    auto gload = [&](int64_t k0) {
        la.load(A, lda, m0, k0, m, k);
        lb.load(B, ldb, n0, k0, n, k);
    };
    auto lstore = [&](int buf) {
        la.store(smem[buf][0], smem[buf][1]);
        lb.store(smem[buf][2], smem[buf][3]);
    };

    const int nk = (int)((k + CBK - 1) / CBK);
    gload(0);
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) gload((int64_t)(kt + 1) * CBK);
        const R* Ar = smem[buf][0];
        const R* Ai = smem[buf][1];
        const R* Br = smem[buf][2];
        const R* Bi = smem[buf][3];
        #pragma unroll
        for (int k4 = 0; k4 < CBK; k4 += 4) {
            const int kr = k4 + (lane >> 4);
            R ar[2], ai[2], br[2], bi[2], nbi[2];
            #pragma unroll
            for (int i = 0; i < 2; ++i) {
                ar[i] = Ar[cl_at(kr, wm + 16 * i + (lane & 15))];
                ai[i] = Ai[cl_at(kr, wm + 16 * i + (lane & 15))];
            }
            #pragma unroll
            for (int j = 0; j < 2; ++j) {
                br[j] = Br[cl_at(kr, wn + 16 * j + (lane & 15))];
                bi[j] = Bi[cl_at(kr, wn + 16 * j + (lane & 15))];
                nbi[j] = -bi[j];
            }
            // two passes over the 8 accumulators so consecutive MFMAs never
            // depend on each other (each chain's second product issues 8 later)
            #pragma unroll
            for (int i = 0; i < 2; ++i)
                #pragma unroll
                for (int j = 0; j < 2; ++j) {
                    cr[i][j] = M::run(br[j], ar[i], cr[i][j]);
                    ci[i][j] = M::run(bi[j], ar[i], ci[i][j]);
                }
            #pragma unroll
            for (int i = 0; i < 2; ++i)
                #pragma unroll
                for (int j = 0; j < 2; ++j) {
                    cr[i][j] = M::run(nbi[j], ai[i], cr[i][j]);
                    ci[i][j] = M::run(br[j], ai[i], ci[i][j]);
                }
        }
        if (kt + 1 < nk) lstore(buf ^ 1);
        __syncthreads();
    }

    // epilogue: lane & 15 runs along M, M::row along N
    const bool bzero = is_zero(beta);
    #pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int64_t gm = m0 + wm + 16 * i + (lane & 15);
        #pragma unroll
        for (int j = 0; j < 2; ++j)
            #pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t gn = n0 + wn + 16 * j + M::row(lane, r);
                bool in = gm < m && gn < n;
                if constexpr (TRI == 'L') in = in && gm >= gn;
                if constexpr (TRI == 'U') in = in && gm <= gn;
                if (in) {
                    cplx<R> v = alpha * cplx<R>(cr[i][j][r], ci[i][j][r]);
                    if (!bzero) v += beta * C[gm + gn * ldc];
                    C[gm + gn * ldc] = v;
                }
            }
    }
}

template <typename R, char TRI, char TA, char TB>
void launch_cplx(int64_t m, int64_t n, int64_t k, cplx<R> alpha, const cplx<R>* A, int64_t lda, const cplx<R>* B,
                 int64_t ldb, cplx<R> beta, cplx<R>* C, int64_t ldc, hipStream_t stream) {
    const int mt = (int)((m + CBM - 1) / CBM), nt = (int)((n + CBN - 1) / CBN);
    const unsigned nblk = TRI ? (unsigned)(mt * (mt + 1) / 2) : (unsigned)(mt * nt);
    // interior-only instantiation when every tile and K-tile is full
    const bool full = (m % CBM == 0) && (n % CBN == 0) && (k % CBK == 0);
    if (full && TRI == 0)
        hipLaunchKernelGGL((gemm_cplx_mfma_kernel<R, TRI, TA, TB, false>), dim3(nblk), dim3(NTHR), 0, stream, m, n, k,
                           alpha, A, lda, B, ldb, beta, C, ldc);
    else
        hipLaunchKernelGGL((gemm_cplx_mfma_kernel<R, TRI, TA, TB, true>), dim3(nblk), dim3(NTHR), 0, stream, m, n, k,
                           alpha, A, lda, B, ldb, beta, C, ldc);
}

template <typename R, char TRI, char TA>
void dispatch_b(char tb, int64_t m, int64_t n, int64_t k, cplx<R> alpha, const cplx<R>* A, int64_t lda,
                const cplx<R>* B, int64_t ldb, cplx<R> beta, cplx<R>* C, int64_t ldc, hipStream_t s) {
    if (tb == 'N') launch_cplx<R, TRI, TA, 'N'>(m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s);
    else if (tb == 'T') launch_cplx<R, TRI, TA, 'T'>(m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s);
    else launch_cplx<R, TRI, TA, 'C'>(m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s);
}

template <typename R, char TRI>
void dispatch_a(char ta, char tb, int64_t m, int64_t n, int64_t k, cplx<R> alpha, const cplx<R>* A, int64_t lda,
                const cplx<R>* B, int64_t ldb, cplx<R> beta, cplx<R>* C, int64_t ldc, hipStream_t s) {
    if (ta == 'N') dispatch_b<R, TRI, 'N'>(tb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s);
    else if (ta == 'T') dispatch_b<R, TRI, 'T'>(tb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s);
    else dispatch_b<R, TRI, 'C'>(tb, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, s);
}

}  // namespace

template <typename T>
void gemm_cplx(char uplo, char transA, char transB, int64_t m, int64_t n, int64_t k,
               T alpha, const T* A, int64_t lda, const T* B, int64_t ldb,
               T beta, T* C, int64_t ldc, hipStream_t stream) {
    using R = real_t<T>;
    if (m <= 0 || n <= 0) return;
    // triangular output ('L' / 'U', m == n): only the tiles that intersect the triangle
    if (uplo == 'L') dispatch_a<R, 'L'>(transA, transB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, stream);
    else if (uplo == 'U') dispatch_a<R, 'U'>(transA, transB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, stream);
    else dispatch_a<R, 0>(transA, transB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, stream);
}

template void gemm_cplx<cplx<float>>(char, char, char, int64_t, int64_t, int64_t, cplx<float>, const cplx<float>*,
                                     int64_t, const cplx<float>*, int64_t, cplx<float>, cplx<float>*, int64_t, hipStream_t);
template void gemm_cplx<cplx<double>>(char, char, char, int64_t, int64_t, int64_t, cplx<double>, const cplx<double>*,
                                      int64_t, const cplx<double>*, int64_t, cplx<double>, cplx<double>*, int64_t, hipStream_t);

}  // namespace dev
}  // namespace slate_amd
