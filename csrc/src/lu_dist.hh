// Distributed LU row-permutation helpers (host loops or gfx950 kernels of
// kernels/lu_dist.hip), used by getrf.cc on p > 1 process grids.
#pragma once

#include "internal.hh"
#include "../kernels/kernels.hh"

namespace slate {
namespace internal {
namespace ludist {

using RowDist = slate_amd::dev::RowDist;
using PanelBases = slate_amd::dev::PanelBases;

/// Panel rows kk.. of the view: assemble the all-gathered per-process blocks
/// into one M x kb panel in global row order (mode 0), or copy my rows of the
/// assembled panel back to my local panel rows ap (mode 1).
template <typename T>
void panel_xfer(lb::Ctx const& c, int64_t M, int64_t kb, int64_t kk, RowDist const& d, PanelBases const& pb,
                int64_t maxr, T* G, T* P, int64_t ldp, T* ap, int64_t lda, int mode);

/// Row distribution of view A as seen by this process.
template <typename T>
RowDist row_dist(BaseMatrix<T> const& A) {
    auto& s = *A.storage();
    RowDist d;
    d.row0 = A.row0();
    d.mb = s.mb;
    d.lrow_begin = A.lrow_begin();
    d.p = s.grid->p();
    d.rsrc = s.rsrc;
    d.myrow = s.grid->myrow();
    d.rrel = s.rrel();
    return d;
}

template <typename T>
void gather_rows_ids(lb::Ctx const& c, int64_t cnt, int64_t ncols, int64_t const* sel, T const* A, int64_t lda,
                     T* out, int64_t ldo, int64_t const* id_in, int64_t* id_out, RowDist const& d, int64_t li_base);

void perm_slots(lb::Ctx const& c, int mode, int64_t base, int cnt, int64_t const* in, int64_t in_off,
                int64_t* ipiv_out, int64_t* slot_src, int64_t* slot_dst);

template <typename T>
void slots_pack(lb::Ctx const& c, int s0, int s1, int64_t ncols, int64_t const* slot_src, T const* A, int64_t lda,
                RowDist const& d, T* buf, int64_t ldb);

template <typename T>
void slots_unpack(lb::Ctx const& c, int s0, int s1, int64_t ncols, int64_t const* slot_dst, T const* buf,
                  int64_t ldb, T* A, int64_t lda, RowDist const& d);

/// Distributed partial pivoting, one panel column per call (reference
/// Tile_getrf.hh:270 MAXLOC + row exchange): elements of T per process in the
/// per-column all-gather, the local candidate entry, and the replicated
/// winner selection + swap + rank-1 update (see kernels/lu_dist.hip).
template <typename T>
int64_t pplu_entry(int64_t kb);
template <typename T>
void pplu_cand(lb::Ctx const& c, int64_t mr, int64_t j, int64_t r0, T const* ap, int64_t lda, int64_t kb,
               RowDist const& d, int64_t lr_k, bool is_pk, T* buf);
template <typename T>
void pplu_apply(lb::Ctx const& c, int np, T const* gbuf, int64_t kb, int64_t j, int64_t cend, int64_t mr,
                int64_t r_upd0, T* ap, int64_t lda, RowDist const& d, int64_t lr_k, int64_t kk, int pk, double thresh,
                bool is_pk, int64_t* pip, int* info, int64_t info_off);

/// Sign-modified LU without pivoting of the n x n block A (TSQR Householder
/// reconstruction): for each column j the diagonal b gets s_j = b/|b| added
/// (|pivot| = 1 + |b|); Y (unit lower) and U' overwrite A, sgn[j] = s_j.
template <typename T>
void lu_sign(lb::Ctx const& c, int64_t n, T* A, int64_t lda, T* sgn);

}  // namespace ludist
}  // namespace internal
}  // namespace slate
