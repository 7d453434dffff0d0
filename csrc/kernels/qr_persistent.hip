// Persistent narrow-block Householder QR for gfx950 (one launch per <= 32
// column block of a tall panel).
//
// Reference: the per-column Householder panel (src/internal/Tile_geqrf.hh:
// 67-490, threads + ThreadBarrier per column; vendor geqrf in
// internal_geqrf.cc:255).  The stream-ordered path in panel.hip needs two
// launches per column that each re-read the whole 32-column block from
// HBM/L2.  Here the block lives in LDS for the whole factorization: G
// workgroups own RB rows each (RB x 32 elements = 128 KB of LDS for fp64),
// and each column costs one grid-wide hand-off of per-workgroup partials:
//
//   per column j:  local partials  (|x|^2 below the diagonal, x^H A(:, k))
//                  publish         (sc1 atomic stores + drain + counter add)
//                  wait            (one lane polls the counter, bounded spin,
//                                   agent-scope acquire)
//                  reduce          (every workgroup sums all G partials in
//                                   block order: deterministic)
//                  reflector + rank-1 update of the local rows in LDS
//
// Hand-off protocol per cdna_hip_programming.md Guideline 16 (gfx950 has 8
// private L2s): payload words are 64-bit agent-scope atomic stores (sc1,
// write-through), every storing wave drains (s_waitcnt vmcnt(0)) before the
// block barrier, one lane then adds to the per-column counter; the consumer
// polls that counter relaxed, issues one agent acquire, and reads the payload
// with agent-scope atomic loads.  Counters are zeroed by a memset before each
// launch; partial slots are double-buffered by column parity (a workgroup can
// only write column j+2's slot after every workgroup has passed column j+1,
// i.e. finished reading column j's).  Spins are bounded: on timeout the
// workgroup sets the error word and skips every later wait and the write-back
// so the grid always drains; the driver reports the error.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

constexpr int QT = 256;       // threads per workgroup
constexpr int QNC = 32;       // max columns per narrow block
constexpr int QSLOT = 2 * QNC + 2;  // partial slot: [nrm, dots(32), alpha, row r (32)]
constexpr unsigned kSpinLimit = 1u << 21;

template <typename T>
__device__ inline void qr_reflector(T alpha, real_t<T> xnorm2, T& beta_o, T& tau, T& scal) {
    using R = real_t<T>;
    R ar = real(alpha), ai = imag(alpha);
    if (xnorm2 == R(0) && ai == R(0)) { beta_o = alpha; tau = zero<T>(); scal = one<T>(); return; }
    R nrm = sqrt((double)ar * ar + (double)ai * ai + (double)xnorm2);
    R beta = ar >= 0 ? -nrm : nrm;
    if constexpr (is_cplx<T>::value) {
        tau = T((beta - ar) / beta, -ai / beta);
        scal = one<T>() / (alpha - T(beta, 0));
        beta_o = T(beta, 0);
    } else {
        tau = (beta - ar) / beta;
        scal = one<T>() / (alpha - beta);
        beta_o = beta;
    }
}

// 64-bit payload words: a real value, or one half (re / im) of a complex one
using u64 = unsigned long long;
__device__ inline void put(u64* p, double v) {
    __hip_atomic_store(p, __builtin_bit_cast(u64, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double get(const u64* p) {
    return __builtin_bit_cast(double, __hip_atomic_load(const_cast<u64*>(p), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT));
}

template <typename T> constexpr int kWords = is_cplx<T>::value ? 2 : 1;

template <typename T>
__device__ inline void put_val(u64* p, T v) {
    if constexpr (is_cplx<T>::value) { put(p, double(v.re)); put(p + 1, double(v.im)); }
    else put(p, double(v));
}
template <typename T>
__device__ inline T get_val(const u64* p) {
    if constexpr (is_cplx<T>::value) return T(real_t<T>(get(p)), real_t<T>(get(p + 1)));
    else return T(get(p));
}

// Block-wide sums of the QNC + 1 values {v0, d[0..QNC)} in one LDS round:
// DPP wave reductions, lane 0 of each wave stores, one barrier, then every
// thread adds the wave results in wave order (deterministic).  Only entries
// k in (j, nn) of d are meaningful; the others are reduced but unused.
template <typename T>
__device__ inline void block_sum_vec(real_t<T>& v0, T (&d)[QNC], int j, int nn,
                                     real_t<T> (*red)[2 * QNC + 1]) {
    using R = real_t<T>;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    R s0 = wave_sum(v0);
    if (lane == 0) red[w][0] = s0;
    #pragma unroll
    for (int k = 0; k < QNC; ++k)
        if (k > j && k < nn) {
            R sr = wave_sum(real(d[k]));
            if (lane == 0) red[w][1 + k] = sr;
            if constexpr (is_cplx<T>::value) {
                R si = wave_sum(imag(d[k]));
                if (lane == 0) red[w][1 + QNC + k] = si;
            }
        }
    __syncthreads();
    R t0 = R(0);
    #pragma unroll
    for (int q = 0; q < QT / 64; ++q) t0 += red[q][0];
    v0 = t0;
    #pragma unroll
    for (int k = 0; k < QNC; ++k)
        if (k > j && k < nn) {
            R tr = R(0), ti = R(0);
            #pragma unroll
            for (int q = 0; q < QT / 64; ++q) {
                tr += red[q][1 + k];
                if constexpr (is_cplx<T>::value) ti += red[q][1 + QNC + k];
            }
            if constexpr (is_cplx<T>::value) d[k] = T(tr, ti); else d[k] = T(tr);
        }
    __syncthreads();   // red is reused by the next call
}

template <typename T, int RB>
__global__ __launch_bounds__(QT) void qr_narrow_kernel(int64_t m, int64_t c0, int nn, T* __restrict__ A, int64_t lda,
                                                       T* __restrict__ tau_out, u64* __restrict__ part,
                                                       unsigned* __restrict__ cnt, unsigned* __restrict__ err, int G) {
    using R = real_t<T>;
    constexpr int RPT = RB / QT;       // rows per thread
    __shared__ T tile[QNC * RB];
    __shared__ R red[QT / 64][2 * QNC + 1];
    __shared__ T tot[QNC + 2];         // reduced dots (by column) + alpha / beta scratch
    __shared__ T rowr[QNC];            // row r of the block (owner's copy)
    __shared__ R nrm_sh;
    __shared__ int fail_sh;

    const int b = blockIdx.x;
    const int64_t row0 = c0 + (int64_t)b * RB;
    const int rows = (int)min<int64_t>((int64_t)RB, m - row0);
    const int kmax = (int)min<int64_t>((int64_t)nn, m - c0);
    if (threadIdx.x == 0) fail_sh = 0;

    // ---- load the block's rows of the narrow panel into LDS
    for (int k = 0; k < nn; ++k)
        #pragma unroll
        for (int t = 0; t < RPT; ++t) {
            int i = threadIdx.x + t * QT;
            if (i < rows) tile[k * RB + i] = A[row0 + i + (c0 + k) * lda];
        }
    __syncthreads();

    for (int j = 0; j < kmax; ++j) {
        const int64_t r = c0 + j;
        const int lr = (int)(r - row0);     // local index of the diagonal row (may be outside)
        const bool owner = lr >= 0 && lr < rows;
        u64* slot = part + ((int64_t)(j & 1) * G + b) * (QSLOT * kWords<T>);

        // ---- local partials over rows below the diagonal
        R xn = R(0);
        T d[QNC];
        #pragma unroll
        for (int k = 0; k < QNC; ++k) d[k] = zero<T>();
        #pragma unroll
        for (int t = 0; t < RPT; ++t) {
            int i = threadIdx.x + t * QT;
            if (i < rows && row0 + i > r) {
                T x = tile[j * RB + i];
                xn += real(x) * real(x) + imag(x) * imag(x);
                #pragma unroll
                for (int k = 0; k < QNC; ++k)
                    if (k > j && k < nn) d[k] += conj(x) * tile[k * RB + i];
            }
        }
        // block reduction; thread 0 publishes
        block_sum_vec<T>(xn, d, j, nn, red);
        if (threadIdx.x == 0) {
            put(slot, double(xn));
            #pragma unroll
            for (int k = 0; k < QNC; ++k)
                if (k > j && k < nn) put_val(slot + (1 + k) * kWords<T>, d[k]);
        }
        if (owner && threadIdx.x < 64) {
            // alpha (column j) and row r of the columns to the right
            for (int k = threadIdx.x; k < nn; k += 64)
                if (k >= j) put_val(slot + (1 + QNC + k) * kWords<T>, tile[k * RB + lr]);
        }
        // every storing wave drains its sc1 stores, then one lane signals
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(&cnt[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // ---- wait for all G workgroups (bounded)
            unsigned spins = 0;
            int f = fail_sh;
            while (!f && __hip_atomic_load(&cnt[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)G) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins >= kSpinLimit ||
                    __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
                    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    f = 1;
                }
            }
            fail_sh = f;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (fail_sh) break;   // uniform across the workgroup

        // ---- reduce all G partials in block order (deterministic)
        const int nv = nn - j;   // nrm + dots for k in (j, nn)
        {
            // thread t handles blocks t, t + QT, ... for every value
            R accn = R(0);
            T accd[QNC];
            #pragma unroll
            for (int k = 0; k < QNC; ++k) accd[k] = zero<T>();
            for (int bb = threadIdx.x; bb < G; bb += QT) {
                const u64* sl = part + ((int64_t)(j & 1) * G + bb) * (QSLOT * kWords<T>);
                accn += R(get(sl));
                #pragma unroll
                for (int k = 0; k < QNC; ++k)
                    if (k > j && k < nn) accd[k] += get_val<T>(sl + (1 + k) * kWords<T>);
            }
            block_sum_vec<T>(accn, accd, j, nn, red);
            if (threadIdx.x == 0) {
                nrm_sh = accn;
                #pragma unroll
                for (int k = 0; k < QNC; ++k)
                    if (k > j && k < nn) tot[k] = accd[k];
            }
                // owner's alpha and row r
            const int ob = (int)((r - c0) / RB);
            const u64* os = part + ((int64_t)(j & 1) * G + ob) * (QSLOT * kWords<T>);
            for (int k = threadIdx.x; k < nn; k += QT)
                if (k >= j) rowr[k] = get_val<T>(os + (1 + QNC + k) * kWords<T>);
            (void)nv;
        }
        __syncthreads();

        // ---- reflector (every thread computes the same values)
        T beta, tau, scal;
        qr_reflector(rowr[j], nrm_sh, beta, tau, scal);
        if (b == 0 && threadIdx.x == 0) tau_out[c0 + j] = tau;
        const T ctau = conj(tau), cscal = conj(scal);

        // ---- update the local rows: v_i = x_i * scal (i > r), v_r = 1
        #pragma unroll
        for (int t = 0; t < RPT; ++t) {
            int i = threadIdx.x + t * QT;
            if (i >= rows || row0 + i < r) continue;
            const bool diag = (row0 + i == r);
            T v = diag ? one<T>() : tile[j * RB + i] * scal;
            tile[j * RB + i] = diag ? beta : v;
            for (int k = j + 1; k < nn; ++k) {
                // z_k = conj(tau) * (a_rk + conj(scal) * sum_{i>r} conj(x_i) a_ik)
                T z = ctau * (rowr[k] + cscal * tot[k]);
                tile[k * RB + i] -= v * z;
            }
        }
        __syncthreads();
    }

    // ---- write back (skipped after a failed hand-off: A keeps its input)
    if (fail_sh) return;
    for (int k = 0; k < nn; ++k)
        #pragma unroll
        for (int t = 0; t < RPT; ++t) {
            int i = threadIdx.x + t * QT;
            if (i < rows) A[row0 + i + (c0 + k) * lda] = tile[k * RB + i];
        }
}

template <typename T> constexpr int qr_rb() {
    return sizeof(T) == 4 ? 1024 : sizeof(T) == 8 ? 512 : 256;
}

}  // namespace

template <typename T>
int qr_narrow_groups(int64_t rows) {
    return (int)((rows + qr_rb<T>() - 1) / qr_rb<T>());
}

size_t qr_narrow_workspace_words(int groups) { return size_t(2) * groups * QSLOT * 2; }

template <typename T>
void qr_narrow(int64_t m, int64_t c0, int nn, T* A, int64_t lda, T* tau, unsigned long long* part,
               unsigned* cnt, unsigned* err, hipStream_t s) {
    if (m - c0 <= 0 || nn <= 0) return;
    constexpr int RB = qr_rb<T>();
    const int G = qr_narrow_groups<T>(m - c0);
    // per-column arrival counters start at 0 for every launch
    (void)hipMemsetAsync(cnt, 0, 128, s);
    hipLaunchKernelGGL((qr_narrow_kernel<T, RB>), dim3(G), dim3(QT), 0, s, m, c0, nn, A, lda, tau,
                       (u64*)part, cnt, err, G);
}

#define SLATE_QRN_INST(T)                                                                              \
    template int qr_narrow_groups<T>(int64_t);                                                         \
    template void qr_narrow<T>(int64_t, int64_t, int, T*, int64_t, T*, unsigned long long*, unsigned*, \
                               unsigned*, hipStream_t);
SLATE_QRN_INST(float)
SLATE_QRN_INST(double)
SLATE_QRN_INST(cplx<float>)
SLATE_QRN_INST(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
