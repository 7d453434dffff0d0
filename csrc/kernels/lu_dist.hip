// Device side of the distributed LU row permutations (getrf / getrf_tntpiv on
// a p x q grid with p > 1).
//
// Reference behaviour: the panel's pivots are broadcast to every rank
// (src/getrf.cc:116, src/getrf_tntpiv.cc:185) and permuteRows<Devices>
// (src/internal/internal_swap.cc:511-805) moves the pivot rows between the
// ranks of each block column with MPI_Isend/Irecv sized from host-side pivot
// counts, plus one blas::swap per pivot on the device.
//
// MI355X design: the host never learns the pivots inside the k-loop.  The
// permutation of one panel touches at most 2*kd rows: the kd rows of the
// diagonal block T and the winner rows outside T (which receive the displaced
// rows of T).  Every row movement becomes a "slot" (src row -> dst row)
// computed on the device (perm_slots); each process packs the source rows it
// owns into a fixed 2*kd x ncols slot buffer (zeros elsewhere), one RCCL
// all-reduce over the column communicator assembles every slot on every
// process, and each process unpacks the rows it owns.  Message sizes are
// therefore known on the host without a device->host copy, and the winner
// slots (the new block row of U, before the triangular solve) arrive on
// EVERY process of the column, which removes the separate U broadcast.
#include "device_common.hh"
#include "kernels.hh"

namespace slate_amd {
namespace dev {

namespace {

constexpr int kMaxSlots = 1024;   // kd <= 1024 (tile size)

template <typename T>
__global__ __launch_bounds__(64) void gather_rows_ids_kernel(int64_t cnt, int64_t ncols, const int64_t* sel,
                                                             const T* A, int64_t lda, T* out, int64_t ldo,
                                                             const int64_t* id_in, int64_t* id_out, RowDist d,
                                                             int64_t li_base) {
    const int64_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= cnt) return;
    const int64_t r = sel[i];
    if (blockIdx.y == 0 && id_out) id_out[i] = id_in ? id_in[r] : rd_l2g(d, li_base + r);
    for (int64_t j = blockIdx.y; j < ncols; j += gridDim.y) out[i + j * ldo] = A[r + j * lda];
}

// One workgroup replays the cnt interchanges on a slot table in LDS:
// pos[s] = row of slot s (slots 0..cnt-1 are base..base+cnt-1, the rest are
// rows outside the block, registered on first touch), content[s] = slot whose
// ORIGINAL row currently sits at pos[s].  Lookups are parallel over the
// table; the swap itself is one thread (wave-uniform, a few LDS ops).
__global__ __launch_bounds__(256) void perm_slots_kernel(int mode, int64_t base, int cnt, const int64_t* in,
                                                         int64_t in_off, int64_t* ipiv_out, int64_t* slot_src,
                                                         int64_t* slot_dst) {
    __shared__ int64_t pos[2 * kMaxSlots];
    __shared__ int content[2 * kMaxSlots];
    __shared__ int s_found, s_n;
    const int tid = threadIdx.x;
    for (int s = tid; s < cnt; s += 256) { pos[s] = base + s; content[s] = s; }
    if (tid == 0) s_n = cnt;
    __syncthreads();
    for (int t = 0; t < cnt; ++t) {
        const int64_t key = in[t] + in_off;
        if (tid == 0) s_found = -1;
        __syncthreads();
        const int n = s_n;
        for (int s = tid; s < n; s += 256) {
            bool hit = mode == 0 ? (pos[content[s]] == key) : (pos[s] == key);
            if (hit) s_found = s;
        }
        __syncthreads();
        if (tid == 0) {
            int f = s_found;
            if (f < 0) { f = s_n++; pos[f] = key; content[f] = f; }
            ipiv_out[t] = pos[f];
            int a = content[t];
            content[t] = content[f];
            content[f] = a;
        }
        __syncthreads();
    }
    const int n = s_n;
    for (int s = tid; s < 2 * cnt; s += 256) {
        if (s < n) { slot_src[s] = pos[content[s]]; slot_dst[s] = pos[s]; }
        else { slot_src[s] = -1; slot_dst[s] = -1; }
    }
}

template <typename T>
__global__ __launch_bounds__(64) void slots_pack_kernel(int s0, int s1, int64_t ncols, const int64_t* slot_src,
                                                        const T* A, int64_t lda, RowDist d, T* buf, int64_t ldb) {
    const int s = s0 + blockIdx.x * 64 + threadIdx.x;
    if (s >= s1) return;
    const int64_t src = slot_src[s];
    const bool mine = src >= 0 && rd_owner(d, src) == d.myrow;
    const int64_t lr = mine ? rd_lrow(d, src) : 0;
    for (int64_t j = blockIdx.y; j < ncols; j += gridDim.y)
        buf[(s - s0) + j * ldb] = mine ? A[lr + j * lda] : zero<T>();
}

template <typename T>
__global__ __launch_bounds__(64) void slots_unpack_kernel(int s0, int s1, int64_t ncols, const int64_t* slot_dst,
                                                          const T* buf, int64_t ldb, T* A, int64_t lda, RowDist d) {
    const int s = s0 + blockIdx.x * 64 + threadIdx.x;
    if (s >= s1) return;
    const int64_t dst = slot_dst[s];
    if (dst < 0 || rd_owner(d, dst) != d.myrow) return;
    const int64_t lr = rd_lrow(d, dst);
    for (int64_t j = blockIdx.y; j < ncols; j += gridDim.y) A[lr + j * lda] = buf[(s - s0) + j * ldb];
}

inline unsigned col_blocks(int64_t ncols) { return (unsigned)std::min<int64_t>(std::max<int64_t>(ncols, 1), 8192); }

// ---- distributed partial pivoting (PPLU on a p > 1 grid), one column j of
// the panel at a time.  Every process of the panel column contributes an entry
// [ header(16 B: max |a|, global row) | its candidate row (kb) | row kk+j (kb,
// from the diagonal process) ] to one all-gather; every process then picks the
// same winner and applies the swap + rank-1 update to the rows it owns.
template <typename T>
__device__ inline rt<T>& pp_val(T* e) { return *reinterpret_cast<rt<T>*>(e); }
template <typename T>
__device__ inline int64_t& pp_gid(T* e) { return *reinterpret_cast<int64_t*>(reinterpret_cast<char*>(e) + 8); }
template <typename T>
__device__ inline rt<T> pp_val(const T* e) { return *reinterpret_cast<const rt<T>*>(e); }
template <typename T>
__device__ inline int64_t pp_gid(const T* e) { return *reinterpret_cast<const int64_t*>(reinterpret_cast<const char*>(e) + 8); }

template <typename T>
__global__ __launch_bounds__(256) void pplu_cand_kernel(int64_t mr, int64_t j, int64_t r0, const T* ap, int64_t lda,
                                                        int64_t kb, RowDist d, int64_t lr_k, int is_pk, T* buf,
                                                        int hdr) {
    SLATE_PANEL_WAVE_PRIO();
    using R = rt<T>;
    __shared__ R sv[256];
    __shared__ int64_t si[256];
    R best = R(-1);
    int64_t bi = INT64_MAX;
    for (int64_t r = r0 + threadIdx.x; r < mr; r += 256) {
        const R v = abs1(ap[r + j * lda]);
        if (v > best) { best = v; bi = r; }          // rows ascending per thread: first max kept
    }
    sv[threadIdx.x] = best;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const R ov = sv[threadIdx.x + w];
            const int64_t oi = si[threadIdx.x + w];
            if (ov > sv[threadIdx.x] || (ov == sv[threadIdx.x] && oi < si[threadIdx.x])) {
                sv[threadIdx.x] = ov;
                si[threadIdx.x] = oi;
            }
        }
        __syncthreads();
    }
    const int64_t r = si[0];
    const bool have = (r != INT64_MAX);
    if (threadIdx.x == 0) {
        pp_val(buf) = have ? sv[0] : R(-1);
        pp_gid(buf) = have ? rd_l2g(d, lr_k + r) : int64_t(-1);
    }
    T* cand = buf + hdr;
    T* cur = buf + hdr + kb;
    for (int64_t c = threadIdx.x; c < kb; c += 256) {
        cand[c] = have ? ap[r + c * lda] : T();
        cur[c] = is_pk ? ap[j + c * lda] : T();
    }
}

template <typename T>
__global__ __launch_bounds__(256) void pplu_apply_kernel(int np, const T* gbuf, int64_t E, int hdr, int64_t kb,
                                                         int64_t j, int64_t cend, int64_t mr, int64_t r_upd0, T* ap,
                                                         int64_t lda, RowDist d, int64_t lr_k, int64_t kk, int pk,
                                                         rt<T> thresh, int is_pk, int64_t* pip, int* info,
                                                         int64_t info_off) {
    SLATE_PANEL_WAVE_PRIO();
    using R = rt<T>;
    __shared__ int64_t s_piv;
    __shared__ int s_w;
    __shared__ T u[64];
    const T* crow = gbuf + pk * E + hdr + kb;
    if (threadIdx.x == 0) {
        R best = R(-1);
        int64_t bg = INT64_MAX;
        int w = -1;
        for (int e = 0; e < np; ++e) {
            const T* en = gbuf + e * E;
            const R v = pp_val(en);
            const int64_t gi = pp_gid(en);
            if (gi < 0) continue;
            if (v > best || (v == best && gi < bg)) { best = v; bg = gi; w = e; }
        }
        int64_t piv = (w < 0) ? kk + j : bg;
        // threshold pivoting: keep row kk+j while |a| >= thresh * max
        if (w >= 0 && thresh < R(1) && piv != kk + j && abs1(crow[j]) >= thresh * best) { piv = kk + j; w = -1; }
        s_piv = piv;
        s_w = w;
        if (blockIdx.x == 0) {
            pip[j] = piv - kk;
            if (info && best == R(0) && *info == 0) *info = (int)(info_off + j + 1);
        }
    }
    __syncthreads();
    const int64_t piv = s_piv;
    const T* prow = (s_w >= 0) ? gbuf + s_w * E + hdr : crow;
    const int64_t nc = cend - j;                 // narrow-block columns j .. cend-1 (<= 64)
    if (threadIdx.x < nc) u[threadIdx.x] = prow[j + threadIdx.x];
    __syncthreads();
    const bool swap = (piv != kk + j);
    const int64_t lp = (swap && rd_owner(d, piv) == d.myrow) ? rd_lrow(d, piv) - lr_k : int64_t(-1);
    if (blockIdx.x == 0) {
        // row kk+j (local row j on the diagonal process) becomes the pivot row,
        // full panel width; the vacated pivot row gets the old row outside [j, cend)
        for (int64_t c = threadIdx.x; c < kb; c += 256) {
            if (is_pk) ap[j + c * lda] = prow[c];
            if (lp >= 0 && (c < j || c >= cend)) ap[lp + c * lda] = crow[c];
        }
    }
    const T ujj = u[0];
    const bool nz = !is_zero(ujj);
    for (int64_t r = r_upd0 + blockIdx.x * 256 + threadIdx.x; r < mr; r += 256 * (int64_t)gridDim.x) {
        const bool isp = (r == lp);
        const T s0 = isp ? crow[j] : ap[r + j * lda];
        const T l = nz ? s0 / ujj : s0;
        ap[r + j * lda] = l;
        for (int64_t c = 1; c < nc; ++c) {
            const T x = isp ? crow[j + c] : ap[r + (j + c) * lda];
            ap[r + (j + c) * lda] = x - l * u[c];
        }
    }
}


// ---- exact partial pivoting on p > 1 with one collective per panel: every
// process of the panel column packs its panel rows (local order, ld maxr) into
// its block of an all-gather buffer G; the same M x kb panel (rows kk..m-1 in
// global order) is then assembled on every process (mode 0), factored
// redundantly by the device panel, and each process copies its own rows back
// (mode 1).  base[r] = storage-local index of process r's first panel row.
template <typename T>
__global__ __launch_bounds__(64) void panel_xfer_kernel(int64_t M, int64_t kb, int64_t kk, RowDist d, PanelBases pb,
                                                        int64_t maxr, T* G, T* P, int64_t ldp, T* ap, int64_t lda,
                                                        int mode) {
    const int64_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= M) return;
    const int64_t R = d.row0 + kk + i;
    const int r = int((R / d.mb + d.rsrc) % d.p);
    const int64_t t = (R / d.mb / d.p) * d.mb + R % d.mb - pb.base[r];
    if (mode == 0) {
        const T* g = G + (int64_t)r * maxr * kb + t;
        for (int64_t j = blockIdx.y; j < kb; j += gridDim.y) P[i + j * ldp] = g[j * maxr];
    } else if (r == d.myrow) {
        for (int64_t j = blockIdx.y; j < kb; j += gridDim.y) ap[t + j * lda] = P[i + j * ldp];
    }
}

}  // namespace

template <typename T>
void gather_rows_ids(int64_t cnt, int64_t ncols, const int64_t* sel, const T* A, int64_t lda, T* out, int64_t ldo,
                     const int64_t* id_in, int64_t* id_out, RowDist d, int64_t li_base, hipStream_t s) {
    if (cnt <= 0) return;
    dim3 g((unsigned)((cnt + 63) / 64), col_blocks(ncols));
    hipLaunchKernelGGL(gather_rows_ids_kernel<T>, g, dim3(64), 0, s, cnt, ncols, sel, A, lda, out, ldo, id_in, id_out,
                       d, li_base);
}

void perm_slots(int mode, int64_t base, int cnt, const int64_t* in, int64_t in_off, int64_t* ipiv_out,
                int64_t* slot_src, int64_t* slot_dst, hipStream_t s) {
    if (cnt <= 0) return;
    hipLaunchKernelGGL(perm_slots_kernel, dim3(1), dim3(256), 0, s, mode, base, cnt, in, in_off, ipiv_out, slot_src,
                       slot_dst);
}

template <typename T>
void slots_pack(int s0, int s1, int64_t ncols, const int64_t* slot_src, const T* A, int64_t lda, RowDist d, T* buf,
                int64_t ldb, hipStream_t s) {
    if (s1 <= s0 || ncols <= 0) return;
    dim3 g((unsigned)((s1 - s0 + 63) / 64), col_blocks(ncols));
    hipLaunchKernelGGL(slots_pack_kernel<T>, g, dim3(64), 0, s, s0, s1, ncols, slot_src, A, lda, d, buf, ldb);
}

template <typename T>
void slots_unpack(int s0, int s1, int64_t ncols, const int64_t* slot_dst, const T* buf, int64_t ldb, T* A,
                  int64_t lda, RowDist d, hipStream_t s) {
    if (s1 <= s0 || ncols <= 0) return;
    dim3 g((unsigned)((s1 - s0 + 63) / 64), col_blocks(ncols));
    hipLaunchKernelGGL(slots_unpack_kernel<T>, g, dim3(64), 0, s, s0, s1, ncols, slot_dst, buf, ldb, A, lda, d);
}

// ---- band LU (gbtrf): the blocked panel applies its row interchanges over
// the whole panel width (getrf convention); LAPACK's band solve (gbtrs) wants
// each column's multipliers as computed, i.e. without the later swaps.  Undo
// them column by column (one thread per column, later pivots first), as
// LAPACK dgbtrf does after each panel.
template <typename T>
__global__ __launch_bounds__(64) void undo_left_swaps_kernel(int64_t w, T* A, int64_t lda, const int64_t* ipiv) {
    const int64_t c = blockIdx.x * 64 + threadIdx.x;
    if (c >= w) return;
    for (int64_t jj = w - 1; jj > c; --jj) {
        const int64_t p = ipiv[jj];
        if (p != jj) {
            const T t = A[jj + c * lda];
            A[jj + c * lda] = A[p + c * lda];
            A[p + c * lda] = t;
        }
    }
}

template <typename T>
void undo_left_swaps(int64_t w, T* A, int64_t lda, const int64_t* ipiv, hipStream_t s) {
    if (w <= 1) return;
    hipLaunchKernelGGL(undo_left_swaps_kernel<T>, dim3((unsigned)((w + 63) / 64)), dim3(64), 0, s, w, A, lda, ipiv);
}

template <typename T>
constexpr int pp_hdr() { return int((16 + sizeof(T) - 1) / sizeof(T)); }

template <typename T>
int64_t pplu_entry(int64_t kb) { return pp_hdr<T>() + 2 * kb; }

template <typename T>
void pplu_cand(int64_t mr, int64_t j, int64_t r0, const T* ap, int64_t lda, int64_t kb, RowDist d, int64_t lr_k,
               bool is_pk, T* buf, hipStream_t s) {
    hipLaunchKernelGGL(pplu_cand_kernel<T>, dim3(1), dim3(256), 0, s, mr, j, r0, ap, lda, kb, d, lr_k, int(is_pk), buf,
                       pp_hdr<T>());
}

template <typename T>
void pplu_apply(int np, const T* gbuf, int64_t kb, int64_t j, int64_t cend, int64_t mr, int64_t r_upd0, T* ap,
                int64_t lda, RowDist d, int64_t lr_k, int64_t kk, int pk, double thresh, bool is_pk, int64_t* pip,
                int* info, int64_t info_off, hipStream_t s) {
    const int64_t rows = std::max<int64_t>(mr - r_upd0, 1);
    const unsigned nblk = (unsigned)std::min<int64_t>((rows + 255) / 256, 1024);
    hipLaunchKernelGGL(pplu_apply_kernel<T>, dim3(nblk), dim3(256), 0, s, np, gbuf, pplu_entry<T>(kb), pp_hdr<T>(),
                       kb, j, cend, mr, r_upd0, ap, lda, d, lr_k, kk, pk, rt<T>(thresh), int(is_pk), pip, info,
                       info_off);
}

template <typename T>
void panel_xfer(int64_t M, int64_t kb, int64_t kk, RowDist d, PanelBases pb, int64_t maxr, T* G, T* P, int64_t ldp,
                T* ap, int64_t lda, int mode, hipStream_t s) {
    if (M <= 0 || kb <= 0) return;
    dim3 g((unsigned)((M + 63) / 64), (unsigned)std::min<int64_t>(kb, 64));
    hipLaunchKernelGGL(panel_xfer_kernel<T>, g, dim3(64), 0, s, M, kb, kk, d, pb, maxr, G, P, ldp, ap, lda, mode);
}

#define SLATE_INST_LUDIST(T)                                                                                       \
    template void gather_rows_ids<T>(int64_t, int64_t, const int64_t*, const T*, int64_t, T*, int64_t,            \
                                     const int64_t*, int64_t*, RowDist, int64_t, hipStream_t);                    \
    template void slots_pack<T>(int, int, int64_t, const int64_t*, const T*, int64_t, RowDist, T*, int64_t,       \
                                hipStream_t);                                                                      \
    template void slots_unpack<T>(int, int, int64_t, const int64_t*, const T*, int64_t, T*, int64_t, RowDist,     \
                                  hipStream_t);                                                                    \
    template int64_t pplu_entry<T>(int64_t);                                                                       \
    template void undo_left_swaps<T>(int64_t, T*, int64_t, const int64_t*, hipStream_t);                           \
    template void pplu_cand<T>(int64_t, int64_t, int64_t, const T*, int64_t, int64_t, RowDist, int64_t, bool, T*,  \
                               hipStream_t);                                                                       \
    template void pplu_apply<T>(int, const T*, int64_t, int64_t, int64_t, int64_t, int64_t, T*, int64_t, RowDist, \
                                int64_t, int64_t, int, double, bool, int64_t*, int*, int64_t, hipStream_t);       \
    template void panel_xfer<T>(int64_t, int64_t, int64_t, RowDist, PanelBases, int64_t, T*, T*, int64_t, T*,     \
                                int64_t, int, hipStream_t);

SLATE_INST_LUDIST(float)
SLATE_INST_LUDIST(double)
SLATE_INST_LUDIST(cplx<float>)
SLATE_INST_LUDIST(cplx<double>)

}  // namespace dev
}  // namespace slate_amd
