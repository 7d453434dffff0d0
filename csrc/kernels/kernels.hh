// Device kernel API (host-callable launchers) for the gfx950 kernels.
// Counterpart of the reference's include/slate/internal/device.hh plus the
// vendor BLAS/LAPACK calls it makes (internal_gemm.cc:498, internal_potrf.cc:72,
// internal_getrf_tntpiv.cc:325, internal_geqrf.cc:255), all hand-written here.
//
// All launchers are asynchronous on `stream`.  Matrices are column-major with
// leading dimension ld.  Op chars: 'N', 'T', 'C'.  Uplo chars: 'L', 'U', 'G'.
// Scalar types are the device types of dev_types.hh (cplx<R> for complex).
#pragma once

#include <hip/hip_runtime_api.h>
#include <cstdint>
#include "dev_types.hh"
#include "matgen_entry.hh"

namespace slate_amd {
namespace dev {

template <typename T> using rt = typename real_type_t<T>::type;

// ---- 2-D block-cyclic row distribution of a view, as seen by one process
// (ScaLAPACK RSRC semantics: tile row ti lives on process row (ti + rsrc) % p).
// gr = view-relative global row; li = row index in the view's local block.
struct RowDist {
    int64_t row0;        // storage row of view row 0
    int64_t mb;          // tile rows
    int64_t lrow_begin;  // first local row of the view in the local array
    int p, rsrc, myrow, rrel;
};
SLATE_HD inline int rd_owner(RowDist const& d, int64_t gr) { return int(((d.row0 + gr) / d.mb + d.rsrc) % d.p); }
SLATE_HD inline int64_t rd_lrow(RowDist const& d, int64_t gr) {
    int64_t R = d.row0 + gr;
    return (R / d.mb / d.p) * d.mb + R % d.mb - d.lrow_begin;
}
SLATE_HD inline int64_t rd_l2g(RowDist const& d, int64_t li) {
    int64_t L = li + d.lrow_begin;
    return ((L / d.mb) * d.p + d.rrel) * d.mb + L % d.mb - d.row0;
}

/// storage-local index of every process row's first panel row (p <= 16)
struct PanelBases { int64_t base[16]; };
/// mode 0: P(i, :) = row kk+i gathered from G (process r's panel rows at
/// G + r maxr kb, ld maxr); mode 1: my rows of P back into ap (ld lda)
template <typename T>
void panel_xfer(int64_t M, int64_t kb, int64_t kk, RowDist d, PanelBases pb, int64_t maxr, T* G, T* P, int64_t ldp,
                T* ap, int64_t lda, int mode, hipStream_t s);

// ---- CholeskyQR panel helpers (cholqr.hip)
/// G(i,i) += c * trace(G) (the shifted first pass); flag = 1 unless the
/// ||G - I||_F <= tol (and finite); ssq: one double of scratch.
template <typename T>
void cholqr_shift(T* G, int64_t ldg, int n, double c, hipStream_t s);
template <typename T>
void cholqr_check(const T* G, int64_t ldg, int n, double tol, int* flag, double* ssq, hipStream_t s);

// ---- in-process communicator (comm.hip)
/// out[i] = op_b in[i + b stride], b < nbuf; type 'f' 'd' 'i' (int32) 'l'
/// (int64) 'b' (int8); op 0 sum, 1 max, 2 min.
void reduce_slabs(char type, int op, void* out, const void* in, int nbuf, int64_t count, int64_t stride,
                  hipStream_t s);

// ---- distributed LU row permutations (lu_dist.hip)
/// out(i, :) = A(sel[i], :) for i < cnt (ncols columns); id_out[i] = id_in[sel[i]]
/// when id_in is given, else the global row of local row li_base + sel[i].
template <typename T>
void gather_rows_ids(int64_t cnt, int64_t ncols, const int64_t* sel, const T* A, int64_t lda, T* out, int64_t ldo,
                     const int64_t* id_in, int64_t* id_out, RowDist d, int64_t li_base, hipStream_t s);
/// Row movements of `cnt` sequential interchanges at positions base..base+cnt-1.
/// mode 0: in[t] + in_off = ORIGINAL row that ends at base+t (tournament winners);
/// mode 1: in[t] + in_off = LAPACK ipiv (current position swapped with base+t).
/// Emits ipiv_out[t] (LAPACK ipiv, global rows) and 2*cnt slots:
/// slot t < cnt: dst base+t <- src (always filled); slot cnt+j: a row outside
/// [base, base+cnt) that receives a displaced row (-1 if unused).  cnt <= 1024.
void perm_slots(int mode, int64_t base, int cnt, const int64_t* in, int64_t in_off, int64_t* ipiv_out,
                int64_t* slot_src, int64_t* slot_dst, hipStream_t s);
/// buf(s - s0, j) = A(row slot_src[s], j) if this process owns that row, else
/// 0, for slots [s0, s1) and ncols local columns (buf ld = ldb).
template <typename T>
void slots_pack(int s0, int s1, int64_t ncols, const int64_t* slot_src, const T* A, int64_t lda, RowDist d, T* buf,
                int64_t ldb, hipStream_t s);
/// A(row slot_dst[s], j) = buf(s - s0, j) for owned destination rows, slots [s0, s1).
template <typename T>
void slots_unpack(int s0, int s1, int64_t ncols, const int64_t* slot_dst, const T* buf, int64_t ldb, T* A,
                  int64_t lda, RowDist d, hipStream_t s);

// ---- distributed partial-pivoting panel, one column per call (lu_dist.hip)
/// elements of T per process in the per-column all-gather: header + 2 rows
template <typename T>
int64_t pplu_entry(int64_t kb);
/// my candidate (max |ap(r, j)|, r in [r0, mr)) and, on the diagonal process,
/// row j -> buf (one all-gather entry)
template <typename T>
void pplu_cand(int64_t mr, int64_t j, int64_t r0, const T* ap, int64_t lda, int64_t kb, RowDist d, int64_t lr_k,
               bool is_pk, T* buf, hipStream_t s);
/// winner from the gathered entries (np of them, diagonal process pk), swap of
/// row kk+j with the pivot row over the panel width kb, scaling of column j and
/// rank-1 update of columns (j, cend) on local rows [r_upd0, mr); pip[j] = piv - kk
template <typename T>
void pplu_apply(int np, const T* gbuf, int64_t kb, int64_t j, int64_t cend, int64_t mr, int64_t r_upd0, T* ap,
                int64_t lda, RowDist d, int64_t lr_k, int64_t kk, int pk, double thresh, bool is_pk, int64_t* pip,
                int* info, int64_t info_off, hipStream_t s);

// ---- distributed divide and conquer (stedc.hip)
/// secular roots of D + rho z z^T (dd ascending, k of them): lambda_j = dd[org[j]] + tau[j]
void secular_roots(int64_t k, double rho, const double* dd, const double* zz, double znorm2, int64_t* org,
                   double* tau, hipStream_t s);
/// Gu-Eisenstat z from the computed roots
void gu_eisenstat(int64_t k, double rho, const double* dd, const double* zz, const int64_t* org, const double* tau,
                  double* zh, hipStream_t s);
/// one merge's device vectors and the local layout of the n2 x n2 block (see stedc.hip)
struct StedcMerge {
    int64_t n2 = 0, k = 0, nrot = 0;
    const double *dd = nullptr, *zh = nullptr, *tau = nullptr;
    const int64_t *org = nullptr, *act = nullptr, *defl = nullptr, *ord = nullptr, *inv_perm = nullptr;
    const int64_t* rot_ab = nullptr;
    const double* rot_cs = nullptr;
    int64_t lrows = 0, mb = 1, p = 1, rrel = 0, row_off = 0;
    int64_t nb = 1, q = 1, crel = 0, col_off = 0;
    int64_t lr0 = 0, lc0 = 0;
};
/// local columns [c_first, c_first + ncols) of the merge matrix into M (ld ldm); scratch: ncols * n2 reals
template <typename T>
void merge_matrix(StedcMerge const& m, int64_t c_first, int64_t ncols, T* M, int64_t ldm, double* scratch,
                  hipStream_t s);

// ---- eigensolver back-transform (eig.hip)
/// G (k x k Gram V^H V) -> T^{-1} = striu(G) + diag(1 / tau) in place.
/// Stage-2 back-transform (hb2st_apply.hip), fp64.  ng groups of 64
/// reflectors: Vc[g] = 64 x 64 compact reflectors (column i: the entries of
/// reflector i, rows R0[g] + i + l), tau[g] = 64 scalars.  hb2st_tfac writes
/// each group's 64 x 64 upper triangular T (forward larft); hb2st_apply
/// applies Z := (I - V T V^H) Z for g = 0 .. ng-1 in order to the n x ncols Z.
void hb2st_tfac(int64_t ng, const double* Vc, const double* tau, double* Tf, hipStream_t s);
void hb2st_apply(int64_t ng, const int64_t* R0, const double* Vc, const double* Tf, double* Z, int64_t ldz,
                 int64_t n, int64_t ncols, hipStream_t s);

template <typename T>
void tinv_from_gram(int64_t k, T* G, int64_t ldg, const T* tau, hipStream_t s);
/// sweeps per rot_sweeps call
constexpr int kRotBatch = 16;
/// Apply kRotBatch QR sweeps of plane rotations to the columns [p0, p1) of
/// every row of M: sweep s rotates columns (j, j+1), j ascending, [x y] <-
/// [c x - s y, s x + c y], with (c, s) at D[2 (j + 2 s - p0) kRotBatch + 2 s]
/// (step-ordered table, identity where a sweep has no rotation; steps
/// p0 .. p1 - 2 + 2 (kRotBatch - 1)).
template <typename T>
void rot_sweeps(int64_t rows, T* M, int64_t ld, int64_t p0, int64_t p1, const rt<T>* D, hipStream_t s);
/// Two independent rot_sweeps jobs (bdsqr's U and Vt) in one launch.
template <typename T>
void rot_sweeps2(int64_t rows_a, T* A, int64_t lda, int64_t pa0, int64_t pa1, const rt<T>* Da, int64_t rows_b, T* B,
                 int64_t ldb, int64_t pb0, int64_t pb1, const rt<T>* Db, hipStream_t s);
/// One rotation on columns (a, b): [x y] <- [x c + y s, y c - x s].
template <typename T>
void rot_cols(int64_t rows, T* M, int64_t ld, int64_t a, int64_t b, rt<T> c, rt<T> sn, hipStream_t s);

/// Band LU: undo the panel's interchanges to the left of each pivot (columns
/// c < jj of the w-column panel, jj = w-1 .. c+1), LAPACK gbtrs convention.
template <typename T>
void undo_left_swaps(int64_t w, T* A, int64_t lda, const int64_t* ipiv, hipStream_t s);

// ---- butterfly transforms (rbt.hip)
/// by_rows: buf(t, j) = A(idx[t], j) for t < cnt, j < len (scatter: the reverse);
/// by columns: buf(i, t) = A(i, idx[t]) for i < len.
template <typename T>
void rbt_gather(bool by_rows, bool scatter, int64_t cnt, int64_t len, const int64_t* idx, T* A, int64_t lda, T* buf,
                int64_t ldb, hipStream_t s);
/// Indexed 2-D gather: dst[rdst[a] + cdst[b] ldd] = src[ridx[a] + cidx[b] lds].
template <typename T>
void gather2d(int64_t nr, int64_t nc, const T* src, int64_t lds, const int64_t* ridx, const int64_t* cidx, T* dst,
              int64_t ldd, const int64_t* rdst, const int64_t* cdst, hipStream_t s);
/// A(i, j) = ca[r] A(i, j) + cp[r] P(i, j) with r = i (by_rows) or j.
template <typename T>
void rbt_combine(bool by_rows, int64_t m, int64_t n, T* A, int64_t lda, const T* P, int64_t ldp, const rt<T>* ca,
                 const rt<T>* cp, hipStream_t s);

// ---- TSQR Householder reconstruction (tsqr.hip): narrow block (nn <= 32) of
// the sign-modified LU without pivoting, rows [r, m), columns [r, r+nn) of A;
// Utop = copy of the nn x nn top block (ld 32); sgn[r+j] receives s_j.
template <typename T>
void lu_sign_narrow(int64_t m, int64_t r, int nn, T* A, int64_t lda, const T* Utop, T* sgn, hipStream_t s);
/// Sign-modified LU of the 64-column leaf at column c0 (width b) of the n x n
/// matrix A: LU11 (staged in W when r = n - c0 - b > 0, copied into place by
/// the next call via Wprev -> Aprev), L21 = A21 U11^{-1}, U12 = L11^{-1} A12,
/// signs into sgn[c0 ..]; the caller applies A22 -= L21 U12.  sizeof(T) <= 8.
template <typename T>
void lu_sign_leaf(int64_t n, int64_t c0, int b, T* A, int64_t lda, T* sgn, T* W, const T* Wprev, T* Aprev, int bprev,
                  hipStream_t s);
/// On-chip TSQR + Householder reconstruction of a narrow panel block: rows x nn
/// (nn <= 32) at A -> V below the diagonal, R on/above, the nn x nn T at Tm,
/// tau[0..nn).  work: qr_tsqr_workspace(rows) scalars.
int64_t qr_tsqr_workspace(int64_t rows);
template <typename T>
void qr_tsqr_narrow(int64_t rows, int nn, T* A, int64_t lda, T* Tm, int64_t ldt, T* tau, T* work, hipStream_t s);

// ---- GEMM (gemm_mfma.hip: real MFMA; gemm_cplx.hip: complex)
template <typename T>
void gemm_real(char transA, char transB, int64_t m, int64_t n, int64_t k,
               T alpha, const T* A, int64_t lda, int64_t sA,
               const T* B, int64_t ldb, int64_t sB,
               T beta, T* C, int64_t ldc, int64_t sC, int64_t batch, hipStream_t stream);
template <typename T>
void gemm_tri_real(char uplo, char transA, char transB, int64_t n, int64_t k,
                   T alpha, const T* A, int64_t lda, const T* B, int64_t ldb,
                   T beta, T* C, int64_t ldc, hipStream_t stream);
template <typename T>
void splitk_reduce(int64_t m, int64_t n, int splits, const T* P, T alpha, T beta, T* C, int64_t ldc, hipStream_t s);
/// Staircase (block-cyclic lower-triangular) output map for one launch of a
/// p x q trailing update: local column c0 + j of C belongs to global tile
/// (c0 + j) / nb * q + pcol; its valid local rows are those whose global index
/// is >= the column's (lower triangle of the global matrix), and its rows of
/// the B^T operand (n x k) start at btab[(c0 + j) / nb - c0 / nb] + (c0 + j) % nb.
struct StairMap {
    const int64_t* btab = nullptr;  // device: element offset of each local column tile's B rows
    int64_t c0 = 0, r0 = 0;         // local column / row index of C(0, 0)
    int nb = 0, p = 1, q = 1, prow = 0, pcol = 0;   // tile size, grid, my row / column (relative to the source)
};
/// C(staircase) = alpha A B^T + beta C over the StairMap's lower staircase;
/// tiles entirely above it are never computed.  Requires nb % 128 == 0.
template <typename T>
void gemm_stair_real(int64_t m, int64_t n, int64_t k, T alpha, const T* A, int64_t lda, const T* B, int64_t ldb,
                     StairMap const& sm, T beta, T* C, int64_t ldc, hipStream_t stream);
template <typename T>
void gemm_cplx(char uplo, char transA, char transB, int64_t m, int64_t n, int64_t k,
               T alpha, const T* A, int64_t lda, const T* B, int64_t ldb,
               T beta, T* C, int64_t ldc, hipStream_t stream);

// ---- skinny products and batched diagonal-block inverse (skinny.hip)
/// y(m x nr) = alpha op(A) x + beta y; trans 'N' (A m x k) or 'T' / 'C' (A k x m).
/// P: partial buffer of chunks * m * min(nr, 16) scalars when chunks > 1.
int gemv_chunks(char trans, int64_t m, int64_t k);
template <typename T>
void gemv(char trans, int64_t m, int64_t k, int nr, T alpha, const T* A, int64_t lda, const T* X, int64_t ldx,
          T beta, T* Y, int64_t ldy, T* P, int chunks, hipStream_t s);
/// inverses of the nblk full BS x BS diagonal blocks of A's uplo triangle
/// into W (block t at W + t BS^2, ld BS); work: nblk * BS^2 / 2 scalars
template <typename T>
void trtri_blocks(char uplo, char diag, int64_t BS, int64_t nblk, const T* A, int64_t lda, T* W, T* work,
                  hipStream_t s);

// ---- aux (aux.hip)
template <typename T>
void geset(char uplo, int64_t m, int64_t n, T offdiag, T diag, T* A, int64_t lda, hipStream_t s);
/// Explicit unit-lower reflector block: V(i, j) = 0 (i < j + off), 1 (i == j + off), A(i, j) below; m x k.
template <typename T>
void form_v(int64_t m, int64_t k, int64_t off, const T* A, int64_t lda, T* V, int64_t ldv, hipStream_t s);
template <typename Ts, typename Td>
void gecopy(char uplo, char trans, int64_t m, int64_t n, const Ts* A, int64_t lda, Td* B, int64_t ldb, hipStream_t s);
template <typename T>
void geadd(char uplo, int64_t m, int64_t n, T alpha, const T* A, int64_t lda, T beta, T* B, int64_t ldb, hipStream_t s);
template <typename T>
void gescale(char uplo, int64_t m, int64_t n, rt<T> mul, T* A, int64_t lda, hipStream_t s);
template <typename T>
void gescale_row_col(int64_t m, int64_t n, const rt<T>* R, const rt<T>* C, T* A, int64_t lda, hipStream_t s);
/// B(i, j) = sc[i] * A(i, j), A real (sc null: 1)
template <typename T>
void real_rowscale(int64_t m, int64_t n, const rt<T>* A, int64_t lda, const T* sc, T* B, int64_t ldb, hipStream_t s);
template <typename T>
void trtri_diag(char uplo, char diag, int64_t n, int nbs, const T* A, int64_t lda, T* W, int64_t ldw, hipStream_t s);
/// trtri_diag into a stack of bs x bs blocks (block t at W + t bs^2, ld bs); bs % nbs == 0
template <typename T>
void trtri_diag_stack(char uplo, char diag, int64_t n, int nbs, const T* A, int64_t lda, T* W, int64_t bs, hipStream_t s);
template <typename T>
void potrf_small(char uplo, int n, T* A, int64_t lda, int* info, int info_offset, hipStream_t s);
/// Lower Cholesky of an n <= 64 block (in place) plus the 64 x 64 inverse of its factor in W
template <typename T>
void potrf_inv_small(int n, T* A, int64_t lda, T* W, int64_t ldw, int* info, int info_offset, hipStream_t s);
/// Lower Cholesky of a b <= 64 diagonal block and A21 := A21 L11^{-H} for the
/// r rows below it, one launch.  With r > 0, L11 goes to the 64 x 64 block W
/// (ld 64), to be copied into A by the next call (Wprev -> Aprev, bprev
/// columns), when no workgroup of this call can still be reading A11.
template <typename T>
void potrf_leaf(int b, int64_t r, T* A, int64_t lda, int* info, int info_offset, T* W, const T* Wprev, T* Aprev,
                int bprev, hipStream_t s);
/// Left NoTrans triangular solve A X = B with m <= 64 (alpha = 1), one launch
template <typename T>
void trsm_small(char uplo, char diag, int m, int64_t n, const T* A, int64_t lda, T* B, int64_t ldb, hipStream_t s);
template <typename T>
void permute_rows(int64_t n, T* A, int64_t lda, const int64_t* dst, const int64_t* src,
                  const int* npairs, int max_pairs, hipStream_t s);
/// buf(t, :) = A(idx[t], :) (gather) or A(idx[t], :) = buf(t, :) (scatter);
/// buf is count x n column-major; idx device array.
template <typename T>
void rows_pack(int64_t n, T* A, int64_t lda, const int64_t* idx, int count, T* buf, bool scatter, hipStream_t s);
template <typename T>
void laswp(int64_t n, T* A, int64_t lda, int64_t k1, int64_t k2, const int64_t* ipiv, int64_t ipiv_offset, hipStream_t s);

// ---- norms (norm.hip): per-column / per-row / per-block partial results
// kind: 'M' max, '1' column sums, 'I' row sums, 'F' column (scale, sumsq)
template <typename T>
void genorm_partial(char kind, char uplo, char diag, int64_t m, int64_t n, const T* A, int64_t lda,
                    int64_t goff_row, int64_t goff_col, rt<T>* out, hipStream_t s, rt<T>* work = nullptr);
// elements of `work` genorm_partial uses for kind 'I' (column-chunk partial row sums)
int64_t genorm_work_size(char kind, int64_t m, int64_t n);

// ---- matgen (matgen.hip): fill a block-cyclic local array (view block at
// absolute local (rb, cb), global offset (row0, col0)) from matgen_entry.hh
template <typename T>
void generate(gen::Spec const& spec, int64_t mloc, int64_t nloc, T* A, int64_t lda, int64_t mb, int p, int rrel,
              int64_t rb, int64_t row0, int64_t nb, int q, int crel, int64_t cb, int64_t col0, hipStream_t s);
/// diagonal post-op on a block-cyclic local array: 'R' zero imaginary parts, 'S' add shift
template <typename T>
void gen_diag(char op, double shift, int64_t mloc, int64_t nloc, T* A, int64_t lda, int64_t mb, int p, int rrel,
              int64_t rb, int64_t row0, int64_t nb, int q, int crel, int64_t cb, int64_t col0, hipStream_t s);

// ---- panels (panel.hip)
template <typename T>
void lu_colmax(int64_t m, int64_t r, const T* A, int64_t lda, int64_t c, rt<T>* pval, int64_t* pidx,
               int nparts, hipStream_t s);
template <typename T>
void lu_pivot(int nparts, const rt<T>* pval, const int64_t* pidx, int64_t r, int64_t c, T* A, int64_t lda,
              int64_t ncols, int64_t* ipiv, int64_t ipiv_base, int64_t* perm, int* info, int64_t info_offset,
              int64_t* piv_out, hipStream_t s, double thresh = 1.0);
template <typename T>
void lu_update(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, rt<T>* pval, int64_t* pidx,
               hipStream_t s);
template <typename T>
void lu_update2d(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, rt<T>* pval, int64_t* pidx,
                 int scale_prev, hipStream_t s);
template <typename T>
void lu_scale_col(int64_t m, int64_t c, T* A, int64_t lda, hipStream_t s);
template <typename T>
void qr_dots2d(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, int nparts_norm, const rt<T>* psum,
               const T* alpha_in, T* tau_out, T* scal_buf, T* pdots, int scale_prev, hipStream_t s);
template <typename T>
void qr_update2d(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, int nparts, const T* pdots,
                 const T* tau_buf, const T* scal_buf, rt<T>* psum_next, T* alpha_next, hipStream_t s);
template <typename T>
void qr_scale_col(int64_t m, int64_t c, T* A, int64_t lda, const T* scal_buf, hipStream_t s);
void iota(int64_t n, int64_t* p, hipStream_t s);
/// Tournament-pivoted LU of the narrow block (columns at Ablk, nn <= 32) of a
/// device panel: rows [r, m), row interchanges applied over ncols columns of
/// Apanel; work holds tslu_workspace(m - r) int64 entries.
int64_t tslu_workspace(int64_t rows);
/// Zero the tournament's arrival counters (once per panel workspace).
void tslu_init(int64_t* work, hipStream_t s);
template <typename T>
void tslu_narrow(int64_t m, int64_t r, int nn, T* Ablk, T* Apanel, int64_t lda, int64_t ncols,
                 int64_t* ipiv, int64_t* perm, int* info, int64_t info_offset, int64_t* work, hipStream_t s);
void perm_pairs(int64_t k, const int64_t* perm, const int64_t* ipiv_local, int64_t* dst, int64_t* src, hipStream_t s);

template <typename T>
void qr_colnorm(int64_t m, int64_t r, const T* A, int64_t lda, int64_t c, rt<T>* psum, T* alpha_out,
                int nparts, hipStream_t s);
template <typename T>
void qr_reflect_dots(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, int nparts_norm,
                     const rt<T>* psum, const T* alpha_in, T* tau_out, T* pdots, int nblocks, hipStream_t s);
template <typename T>
void qr_update(int64_t m, int64_t r, int64_t c, int64_t cend, T* A, int64_t lda, int nparts, const T* pdots,
               const T* tau_in, rt<T>* psum_next, T* alpha_next, int nblocks, hipStream_t s);
template <typename T>
void tsip(int64_t K, int m, int n, T alpha, const T* A, int64_t lda, const T* B, int64_t ldb, T beta,
          T* C, int64_t ldc, T* work, int64_t work_elems, hipStream_t s);
template <typename T>
void larft_small(int k, const T* tau, T* Tm, int64_t ldt, hipStream_t s);

/// Persistent narrow-block QR (qr_persistent.hip): Householder QR of columns
/// [c0, c0+nn) (nn <= 32) of a panel over rows [c0, m) in ONE launch; tau[c0..]
/// receives the scalars, A the reflectors (unit diagonal implicit) and R.
/// part: qr_narrow_workspace_words(groups) 64-bit words; cnt: 32 counters
/// (zeroed by the launcher); err: set non-zero if a grid hand-off timed out.
template <typename T>
int qr_narrow_groups(int64_t rows);
size_t qr_narrow_workspace_words(int groups);
template <typename T>
void qr_narrow(int64_t m, int64_t c0, int nn, T* A, int64_t lda, T* tau, unsigned long long* part,
               unsigned* cnt, unsigned* err, hipStream_t s);

}  // namespace dev
}  // namespace slate_amd
