// Stage-2 back-transform of the two-stage eigensolver / SVD on gfx950:
// Z := Q2 Z for the bulge-chasing reflectors (reference src/unmtr_hb2st.cc,
// which applies them as a wavefront of small vendor GEMMs per block).
//
// The reflectors come in groups of up to 64: the reflectors of 64 consecutive
// sweeps at one bulge step, reflector i of a group acting on rows
// r0 + i .. r0 + i + kd - 1 (kd <= 64).  A group is one block reflector
// I - V T V^H with V a 128 x 64 parallelogram (column i nonzero in rows
// i .. i + 63) and T upper triangular.  Columns of Z are independent under Q2,
// so:
//   hb2st_tfac   one wave per group: G = V^H V on the parallelogram, then the
//                forward larft recurrence T(0:j, j) = -tau_j T(0:j, 0:j) G(0:j, j)
//                (tau = 0 leaves a zero column: H_j = I).
//   hb2st_apply  one workgroup per NC-column slice of Z walks every group of a
//                chunk in order -- no inter-workgroup synchronisation at all:
//                Zr = Z(r0 : r0 + 127, slice) into LDS, W = V^H Zr, W2 = T W,
//                Z(r0 : r0 + 127, slice) -= V W2, each on v_mfma_f64_16x16x4
//                with the zero triangles of the parallelogram skipped at 16 x 4
//                granularity (about 1.25x the useful flops instead of the
//                2.5x of dense (GS + kd) x GS blocks).  V stays compact in LDS
//                (V(rho, i) = Vc(i, rho - i)), so one group moves 32 KB of V,
//                32 KB of T and a 128 x NC window of Z.
// Group order is the caller's: groups that share rows of Z must be applied in
// the order of Q2's factors (eig.cc unmtr_hb2st_blocked), which a sequential
// walk per slice preserves.
#include "device_common.hh"
#include "kernels.hh"

#include <cstdlib>

namespace slate_amd {
namespace dev {

namespace {

constexpr int HB = 64;          // reflectors per group (columns of V)
constexpr int HR = 128;         // rows of a group's window
constexpr int LDV = HB + 2;     // compact V in LDS: Vs[i * LDV + l]
constexpr int LDT = HB;         // T in LDS, column-major: Ts[k * LDT + i]

__device__ inline void mfma16(double a, double b, double (&c)[4]) {
    typedef double v4d __attribute__((ext_vector_type(4)));
    v4d acc = {c[0], c[1], c[2], c[3]};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    c[0] = acc[0]; c[1] = acc[1]; c[2] = acc[2]; c[3] = acc[3];
}

// one wave per group
__global__ __launch_bounds__(64) void hb2st_tfac_kernel(const double* __restrict__ Vc, const double* __restrict__ tau,
                                                        double* __restrict__ Tf) {
    __shared__ double Vs[HB * LDV];
    __shared__ double Gs[HB * (HB + 1)];   // G(a, j) at Gs[j * (HB + 1) + a]
    __shared__ double Ts[HB * (HB + 1)];   // T(i, j) at Ts[j * (HB + 1) + i]
    const int t = threadIdx.x;
    const size_t g = blockIdx.x;
    const double* V = Vc + g * HB * HB;
    for (int i = 0; i < HB; ++i) Vs[i * LDV + t] = V[i * HB + t];
    __syncthreads();
    // thread j: G(a, j) = sum_l v_a[l + (j - a)] v_j[l] for a < j
    const int j = t;
    for (int a = 0; a < j; ++a) {
        const int d = j - a;
        double s = 0.0;
        for (int l = 0; l + d < HB; ++l) s += Vs[a * LDV + l + d] * Vs[j * LDV + l];
        Gs[j * (HB + 1) + a] = s;
    }
    for (int i = 0; i < HB; ++i) Ts[j * (HB + 1) + i] = 0.0;
    __syncthreads();
    // column k of T needs columns 0 .. k-1: one step per column, thread i < k
    for (int k = 0; k < HB; ++k) {
        const double tk = tau[g * HB + k];
        if (t < k) {
            double s = 0.0;
            for (int m = t; m < k; ++m) s += Ts[m * (HB + 1) + t] * Gs[k * (HB + 1) + m];
            Ts[k * (HB + 1) + t] = -tk * s;
        } else if (t == k) {
            Ts[k * (HB + 1) + k] = tk;
        }
        __syncthreads();
    }
    double* Tg = Tf + g * HB * HB;
    for (int c = 0; c < HB; ++c) Tg[c * HB + t] = Ts[c * (HB + 1) + t];
}

template <int NC>
__global__ __launch_bounds__(256) void hb2st_apply_kernel(int64_t ng, const int64_t* __restrict__ R0,
                                                          const double* __restrict__ Vc,
                                                          const double* __restrict__ Tf, double* Z, int64_t ldz,
                                                          int64_t n, int64_t ncols, bool slide) {
    constexpr int LDZ = HR + 1;   // Zs[c * LDZ + rho]
    constexpr int LDW = HB + 1;   // Ws[c * LDW + i]
    constexpr int NCB = NC / 16;
    __shared__ double Vs[HB * LDV];
    __shared__ double Ts[HB * LDT];
    __shared__ double Zs[NC * LDZ];
    __shared__ double Ws[NC * LDW];
    __shared__ double W2s[NC * LDW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int lo = lane & 15, hi = lane >> 4;
    const int64_t c0 = int64_t(blockIdx.x) * NC;
    // rho blocks of the update, paired so every wave gets 20 k-steps
    const int rbA = (w == 0) ? 0 : (w == 1) ? 1 : (w == 2) ? 4 : 5;
    const int rbB = (w == 0) ? 3 : (w == 1) ? 2 : (w == 2) ? 7 : 6;
    // V and T of the next group are prefetched into registers while the
    // current one computes (all loads of a group in flight together: a load /
    // LDS-store loop would pay one memory latency per iteration)
    constexpr int NV = HB * HB / 256, NZ = HR * NC / 256;
    double rv[NV], rt[NV];
    auto fetch_vt = [&](int64_t g) {
        const double* V = Vc + g * HB * HB;
        const double* Tg = Tf + g * HB * HB;
        #pragma unroll
        for (int it = 0; it < NV; ++it) { rv[it] = V[tid + 256 * it]; rt[it] = Tg[tid + 256 * it]; }
    };
    if (ng > 0) fetch_vt(0);
    // Sliding window: consecutive groups of one sweep block J sit 64 rows
    // apart when kd = 64, so the lower half of the window stays in LDS (the
    // halves swap roles: physical row = logical row ^ (flip << 6)), the upper
    // half of the next window is prefetched into registers while this group
    // computes, and only the departing 64 rows are stored.
    constexpr int NZH = NZ / 2;
    double rz2[NZH];
    int flip = 0;
    bool slid = false;
    int64_t r0 = ng > 0 ? R0[0] : 0;
    int64_t r0n = ng > 1 ? R0[1] : 0;
    for (int64_t g = 0; g < ng; ++g) {
        const bool slide_next = slide && g + 1 < ng && r0n == r0 + 64;
        const int64_t r0nn = g + 2 < ng ? R0[g + 2] : 0;
        if (!slid) {
            double rz[NZ];
            #pragma unroll
            for (int it = 0; it < NZ; ++it) {
                const int e = tid + 256 * it, rho = e % HR, c = e / HR;
                const int64_t row = r0 + rho, col = c0 + c;
                rz[it] = (row < n && col < ncols) ? Z[row + col * ldz] : 0.0;
            }
            #pragma unroll
            for (int it = 0; it < NZ; ++it) {
                const int e = tid + 256 * it, rho = e % HR, c = e / HR;
                Zs[c * LDZ + (rho ^ (flip << 6))] = rz[it];
            }
        } else {
            #pragma unroll
            for (int it = 0; it < NZH; ++it) {
                const int e = tid + 256 * it, rho = 64 + e % 64, c = e / 64;
                Zs[c * LDZ + (rho ^ (flip << 6))] = rz2[it];
            }
        }
        #pragma unroll
        for (int it = 0; it < NV; ++it) {
            const int e = tid + 256 * it, i = e / HB, l = e % HB;
            Vs[i * LDV + l] = rv[it];
            Ts[e] = rt[it];         // column-major, LDT = HB
        }
        if (g + 1 < ng) fetch_vt(g + 1);
        if (slide_next) {
            // rows r0 + 128 .. r0 + 191: untouched by this group
            #pragma unroll
            for (int it = 0; it < NZH; ++it) {
                const int e = tid + 256 * it, rr = e % 64, c = e / 64;
                const int64_t row = r0 + 128 + rr, col = c0 + c;
                rz2[it] = (row < n && col < ncols) ? Z[row + col * ldz] : 0.0;
            }
        }
        __syncthreads();
        // W = V^H Zr: wave w owns rows i in [16 w, 16 w + 16); V(rho, i) is
        // nonzero for rho in [i, i + 63] -> rho in [16 w, 16 w + 79)
        {
            double acc[NCB][4];
            #pragma unroll
            for (int cb = 0; cb < NCB; ++cb) acc[cb][0] = acc[cb][1] = acc[cb][2] = acc[cb][3] = 0.0;
            const int i = 16 * w + lo;
            #pragma unroll 4
            for (int s = 0; s < 20; ++s) {
                const int rho = 16 * w + 4 * s + hi;
                const int l = rho - i;
                const double a = (l >= 0 && l < HB) ? Vs[i * LDV + l] : 0.0;
                #pragma unroll
                for (int cb = 0; cb < NCB; ++cb) mfma16(a, Zs[(16 * cb + lo) * LDZ + (rho ^ (flip << 6))], acc[cb]);
            }
            #pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
                #pragma unroll
                for (int q = 0; q < 4; ++q) Ws[(16 * cb + lo) * LDW + 16 * w + hi + 4 * q] = acc[cb][q];
        }
        __syncthreads();
        // W2 = T W (T upper triangular): rows i of block w need k >= 16 w
        {
            double acc[NCB][4];
            #pragma unroll
            for (int cb = 0; cb < NCB; ++cb) acc[cb][0] = acc[cb][1] = acc[cb][2] = acc[cb][3] = 0.0;
            const int i = 16 * w + lo;
            for (int k0 = 16 * w; k0 < HB; k0 += 4) {
                const int k = k0 + hi;
                const double a = Ts[k * LDT + i];
                #pragma unroll
                for (int cb = 0; cb < NCB; ++cb) mfma16(a, Ws[(16 * cb + lo) * LDW + k], acc[cb]);
            }
            #pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
                #pragma unroll
                for (int q = 0; q < 4; ++q) W2s[(16 * cb + lo) * LDW + 16 * w + hi + 4 * q] = acc[cb][q];
        }
        __syncthreads();
        // Zr -= V W2: rho block rb needs i in [16 rb - 63, 16 rb + 15]
        #pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            const int rb = pass ? rbB : rbA;
            const int ilo = max(0, 16 * rb - 64), ihi = min(HB, 16 * rb + 16);
            double acc[NCB][4];
            #pragma unroll
            for (int cb = 0; cb < NCB; ++cb) acc[cb][0] = acc[cb][1] = acc[cb][2] = acc[cb][3] = 0.0;
            const int rho = 16 * rb + lo;
            for (int i0 = ilo; i0 < ihi; i0 += 4) {
                const int i = i0 + hi, l = rho - i;
                const double a = (l >= 0 && l < HB) ? Vs[i * LDV + l] : 0.0;
                #pragma unroll
                for (int cb = 0; cb < NCB; ++cb) mfma16(a, W2s[(16 * cb + lo) * LDW + i], acc[cb]);
            }
            // (each wave owns its rho blocks of Zs: update in place)
            #pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                const int c = 16 * cb + lo;
                #pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int rr = 16 * rb + hi + 4 * q;
                    Zs[c * LDZ + (rr ^ (flip << 6))] -= acc[cb][q];
                }
            }
        }
        __syncthreads();
        // coalesced store (down the columns): the whole window, or only its
        // departing lower half when the next group slides
        if (slide_next) {
            #pragma unroll
            for (int it = 0; it < NZH; ++it) {
                const int e = tid + 256 * it, rho = e % 64, c = e / 64;
                const int64_t row = r0 + rho, col = c0 + c;
                if (row < n && col < ncols) Z[row + col * ldz] = Zs[c * LDZ + (rho ^ (flip << 6))];
            }
        } else {
            #pragma unroll
            for (int it = 0; it < NZ; ++it) {
                const int e = tid + 256 * it, rho = e % HR, c = e / HR;
                const int64_t row = r0 + rho, col = c0 + c;
                if (row < n && col < ncols) Z[row + col * ldz] = Zs[c * LDZ + (rho ^ (flip << 6))];
            }
        }
        // the next group may reload rows this one stored (workgroup-scope
        // visibility: same CU) and overwrites the LDS images
        __syncthreads();
        if (slide_next) flip ^= 1;
        slid = slide_next;
        r0 = r0n;
        r0n = r0nn;
    }
}

}  // namespace

void hb2st_tfac(int64_t ng, const double* Vc, const double* tau, double* Tf, hipStream_t s) {
    if (ng <= 0) return;
    hipLaunchKernelGGL(hb2st_tfac_kernel, dim3(unsigned(ng)), dim3(64), 0, s, Vc, tau, Tf);
}

void hb2st_apply(int64_t ng, const int64_t* R0, const double* Vc, const double* Tf, double* Z, int64_t ldz,
                 int64_t n, int64_t ncols, hipStream_t s) {
    if (ng <= 0 || ncols <= 0) return;
    static const bool slide = [] { const char* e = std::getenv("SLATE_HB2ST_SLIDE"); return !e || std::atoi(e) != 0; }();
    // 32-column slices while that still gives a workgroup per CU, else 16
    if ((ncols + 31) / 32 >= 256) {
        const unsigned nb = unsigned((ncols + 31) / 32);
        hipLaunchKernelGGL(hb2st_apply_kernel<32>, dim3(nb), dim3(256), 0, s, ng, R0, Vc, Tf, Z, ldz, n, ncols, slide);
    } else {
        const unsigned nb = unsigned((ncols + 15) / 16);
        hipLaunchKernelGGL(hb2st_apply_kernel<16>, dim3(nb), dim3(256), 0, s, ng, R0, Vc, Tf, Z, ldz, n, ncols, slide);
    }
}

}  // namespace dev
}  // namespace slate_amd
