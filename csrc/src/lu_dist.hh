// Distributed LU row-permutation helpers (host loops or gfx950 kernels of
// kernels/lu_dist.hip), used by getrf.cc on p > 1 process grids.
#pragma once

#include "internal.hh"
#include "../kernels/kernels.hh"

namespace slate {
namespace internal {
namespace ludist {

using RowDist = slate_amd::dev::RowDist;

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

/// Sign-modified LU without pivoting of the n x n block A (TSQR Householder
/// reconstruction): for each column j the diagonal b gets s_j = b/|b| added
/// (|pivot| = 1 + |b|); Y (unit lower) and U' overwrite A, sgn[j] = s_j.
template <typename T>
void lu_sign(lb::Ctx const& c, int64_t n, T* A, int64_t lda, T* sgn);

}  // namespace ludist
}  // namespace internal
}  // namespace slate
