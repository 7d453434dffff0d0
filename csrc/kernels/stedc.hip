// Device side of the distributed divide-and-conquer tridiagonal eigensolver
// (eig_dist.cc; reference src/stedc_secular.cc, stedc_merge.cc, and LAPACK
// laed3 / laed4 semantics).
//
// One merge of two halves (n2 = n1 + (n2 - n1) columns of Q) on the rank-one
// modified system D + rho z z^T after sorting and deflation (host, O(n2)):
//   * secular_roots: one thread per non-deflated root j, the rational
//     iteration of slate_amd/secular.hh to full relative precision of
//     tau_j = lambda_j - dd[org_j] (distance to the nearest pole), which the
//     Gu-Eisenstat vectors need;
//   * gu_eisenstat_z: z recomputed from the computed roots, one thread per i;
//   * merge_matrix: every rank builds ONLY its local entries of the n2 x n2
//     merge matrix M (Q_new = Q_old M): per output column one workgroup forms
//     the column in the sorted basis (normalized Gu-Eisenstat eigenvector of
//     the secular system, or a unit vector for a deflated column), applies the
//     deflation Givens rotations in reverse order, and scatters its local rows
//     through the sort permutation.  The product itself is the distributed
//     MFMA GEMM; no n x n matrix exists on any host.
#include "device_common.hh"
#include "kernels.hh"
#include "slate_amd/secular.hh"

#include <cstdlib>

namespace slate_amd {
namespace dev {

namespace {

__global__ __launch_bounds__(64) void secular_roots_kernel(int64_t k, double rho, const double* dd, const double* zz,
                                                           double znorm2, int64_t* org, double* tau) {
    const int64_t j = blockIdx.x * 64 + threadIdx.x;
    if (j >= k) return;
    int64_t o2 = j;
    const double t = slate::secular::root<double>(k, j, rho, dd, zz, znorm2, &o2);
    org[j] = o2;
    tau[j] = t;
}

// One WAVE per root: the O(k) sums of every iteration are split over the
// 64 lanes and reduced by an xor butterfly, then lane 0's totals are
// broadcast so every lane runs the identical (uniform) iteration.  The
// thread-per-root form left k / 64 waves for the whole chip with each lane
// walking all k poles per iteration (~1.9 ms a launch, ~60 ms of heev at
// n = 8192, profiles/r4_eig_kernel_stats_final.txt).
__global__ __launch_bounds__(256) void secular_roots_wave_kernel(int64_t k, double rho, const double* dd,
                                                                const double* zz, double znorm2, int64_t* org,
                                                                double* tau) {
    const int lane = threadIdx.x & 63;
    const int64_t j = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (j >= k) return;   // wave-uniform
    auto wsum = [&](int64_t o, double t) {
        slate::secular::Sums<double> s;
        const double d0 = dd[o];
        for (int64_t i = lane; i < k; i += 64) {
            const double r = zz[i] / ((dd[i] - d0) - t);
            if (i <= j) { s.psi += zz[i] * r; s.dpsi += r * r; }
            else { s.phi += zz[i] * r; s.dphi += r * r; }
        }
        #pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            s.psi += __shfl_xor(s.psi, off);
            s.phi += __shfl_xor(s.phi, off);
            s.dpsi += __shfl_xor(s.dpsi, off);
            s.dphi += __shfl_xor(s.dphi, off);
        }
        s.psi = __shfl(s.psi, 0);
        s.phi = __shfl(s.phi, 0);
        s.dpsi = __shfl(s.dpsi, 0);
        s.dphi = __shfl(s.dphi, 0);
        return s;
    };
    int64_t o2 = j;
    const double t = slate::secular::root_with<double>(k, j, rho, dd, znorm2, &o2, wsum);
    if (lane == 0) {
        org[j] = o2;
        tau[j] = t;
    }
}

__global__ __launch_bounds__(64) void gu_eisenstat_kernel(int64_t k, double rho, const double* dd, const double* zz,
                                                          const int64_t* org, const double* tau, double* zh) {
    const int64_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= k) return;
    auto lmd = [&](int64_t j) { return (dd[org[j]] - dd[i]) + tau[j]; };
    double pr = lmd(k - 1) / rho;
    for (int64_t j = 0; j < k - 1; ++j) {
        const double den = (j < i) ? (dd[j] - dd[i]) : (dd[j + 1] - dd[i]);
        pr *= lmd(j) / den;
    }
    zh[i] = copysign(sqrt(fabs(pr)), zz[i]);
}

// Merge matrix, local part.  Block-cyclic local rows / columns of the n2 x n2
// block (view-relative global index = l2g(local) - off).  Output column jo
// holds result column r = ord[jo]: r < k the secular eigenvector, else the
// deflated sorted column defl[r - k].  Sorted basis -> rows: row src takes
// vec[inv_perm[src]].  vec is per-workgroup global scratch (n2 reals).
struct MergeArgs {
    int64_t n2, k, nrot;
    const double *dd, *zh, *tau;
    const int64_t *org, *act, *defl, *ord, *inv_perm;
    const int64_t* rot_ab;          // nrot pairs (a, b) in application order
    const double* rot_cs;           // nrot pairs (c, s)
    // local layout of the block
    int64_t lrows, mb, p, rrel, row_off;     // row: global = ((l / mb) * p + rrel) * mb + l % mb - row_off
    int64_t nb, q, crel, col_off;             // col: same for local column index lc0 + blockIdx
    int64_t lr0, lc0;                         // first local row / col of the block
};

__device__ inline int64_t bc_l2g(int64_t l, int64_t b, int64_t procs, int64_t rel) {
    return ((l / b) * procs + rel) * b + l % b;
}

template <typename T>
__global__ __launch_bounds__(256) void merge_matrix_kernel(MergeArgs a, int64_t c_first, T* M, int64_t ldm,
                                                           double* scratch) {
    const int64_t lcb = c_first + blockIdx.x;                     // local column within the block
    const int64_t jo = bc_l2g(a.lc0 + lcb, a.nb, a.q, a.crel) - a.col_off;
    double* vec = scratch + blockIdx.x * a.n2;
    __shared__ double red[256];
    for (int64_t s = threadIdx.x; s < a.n2; s += 256) vec[s] = 0.0;
    __syncthreads();
    const int64_t r = a.ord[jo];
    if (r < a.k) {
        const double dr = a.dd[a.org[r]], tr = a.tau[r];
        double part = 0;
        for (int64_t i = threadIdx.x; i < a.k; i += 256) {
            const double u = a.zh[i] / ((a.dd[i] - dr) - tr);
            vec[a.act[i]] = u;
            part += u * u;
        }
        red[threadIdx.x] = part;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
            __syncthreads();
        }
        const double inv = 1.0 / sqrt(red[0]);
        for (int64_t i = threadIdx.x; i < a.k; i += 256) vec[a.act[i]] *= inv;
    } else if (threadIdx.x == 0) {
        vec[a.defl[r - a.k]] = 1.0;
    }
    __syncthreads();
    // G w with G = G_1 ... G_t: the last rotation acts first
    if (threadIdx.x == 0) {
        for (int64_t t = a.nrot - 1; t >= 0; --t) {
            const int64_t x = a.rot_ab[2 * t], y = a.rot_ab[2 * t + 1];
            const double c = a.rot_cs[2 * t], sn = a.rot_cs[2 * t + 1];
            const double vx = vec[x], vy = vec[y];
            vec[x] = c * vx - sn * vy;
            vec[y] = sn * vx + c * vy;
        }
    }
    __syncthreads();
    for (int64_t lr = threadIdx.x; lr < a.lrows; lr += 256) {
        const int64_t src = bc_l2g(a.lr0 + lr, a.mb, a.p, a.rrel) - a.row_off;
        M[lr + lcb * ldm] = T(vec[a.inv_perm[src]]);
    }
}

}  // namespace

void secular_roots(int64_t k, double rho, const double* dd, const double* zz, double znorm2, int64_t* org, double* tau,
                   hipStream_t s) {
    if (k <= 0) return;
    // SLATE_SECULAR_WAVE=0: one thread per root (A/B)
    static const bool wave = [] {
        const char* e = std::getenv("SLATE_SECULAR_WAVE");
        return !e || std::atoi(e) != 0;
    }();
    if (wave) {
        hipLaunchKernelGGL(secular_roots_wave_kernel, dim3((unsigned)((k + 3) / 4)), dim3(256), 0, s, k, rho, dd, zz,
                           znorm2, org, tau);
        return;
    }
    hipLaunchKernelGGL(secular_roots_kernel, dim3((unsigned)((k + 63) / 64)), dim3(64), 0, s, k, rho, dd, zz, znorm2,
                       org, tau);
}

void gu_eisenstat(int64_t k, double rho, const double* dd, const double* zz, const int64_t* org, const double* tau,
                  double* zh, hipStream_t s) {
    if (k <= 0) return;
    hipLaunchKernelGGL(gu_eisenstat_kernel, dim3((unsigned)((k + 63) / 64)), dim3(64), 0, s, k, rho, dd, zz, org,
                       tau, zh);
}

template <typename T>
void merge_matrix(StedcMerge const& m, int64_t c_first, int64_t ncols, T* M, int64_t ldm, double* scratch,
                  hipStream_t s) {
    if (ncols <= 0) return;
    MergeArgs a;
    a.n2 = m.n2; a.k = m.k; a.nrot = m.nrot;
    a.dd = m.dd; a.zh = m.zh; a.tau = m.tau;
    a.org = m.org; a.act = m.act; a.defl = m.defl; a.ord = m.ord; a.inv_perm = m.inv_perm;
    a.rot_ab = m.rot_ab; a.rot_cs = m.rot_cs;
    a.lrows = m.lrows; a.mb = m.mb; a.p = m.p; a.rrel = m.rrel; a.row_off = m.row_off;
    a.nb = m.nb; a.q = m.q; a.crel = m.crel; a.col_off = m.col_off;
    a.lr0 = m.lr0; a.lc0 = m.lc0;
    hipLaunchKernelGGL(merge_matrix_kernel<T>, dim3((unsigned)ncols), dim3(256), 0, s, a, c_first, M, ldm, scratch);
}
template void merge_matrix<double>(StedcMerge const&, int64_t, int64_t, double*, int64_t, double*, hipStream_t);
template void merge_matrix<float>(StedcMerge const&, int64_t, int64_t, float*, int64_t, double*, hipStream_t);

}  // namespace dev
}  // namespace slate_amd
