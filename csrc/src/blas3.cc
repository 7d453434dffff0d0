// Distributed level-3 BLAS drivers.
//
// gemmC: SUMMA with lookahead (reference src/gemmC.cc:65-188).  Per step k,
//   A(:,k) is broadcast along process rows and B(k,:) down process columns
//   as ONE contiguous buffer each (RCCL broadcast on the comm queue), and
//   each process runs ONE local MFMA GEMM C_loc += A_k * B_k on queue 0
//   while the broadcasts for k+1.. proceed (ring of la+2 buffers).
//   A 1x1 grid is a single local GEMM over the whole k range.
// gemmA: stationary A (reference src/gemmA.cc:67-190): local partial
//   products reduced across the process row (allreduce replaces listReduce).
// trsm: block-row sweeps (reference src/work/work_trsm.cc:101-185).
// herk/syrk/her2k/syr2k: a single local call on 1x1 grids; on larger grids a
//   triangle-only SUMMA (tri_summa: diagonal tiles through the triangular MFMA
//   GEMM, never the other triangle).  trmm (Left, NoTrans A): SUMMA that skips
//   the zero part of each A panel.  hemm/symm: gemmC on the expanded operand.
#include "internal.hh"

#include <numeric>

namespace slate {

using namespace internal;

namespace {

inline int64_t option_la(Options const& opts) { return get_option<int64_t>(opts, Option::Lookahead, 1); }

/// New matrix on `g` with tile sizes mb x nb whose first tile sits on
/// process (rsrc, csrc), holding op(X) (any source distribution).
template <typename T>
Matrix<T> materialize(BaseMatrix<T> const& X, Target target, GridPtr g, int64_t mb, int64_t nb,
                      int rsrc, int csrc) {
    Matrix<T> M(X.m(), X.n(), mb, nb, g, rsrc, csrc);
    M.insertLocalTiles(target);
    Options o = {{Option::Target, target}};
    slate::copy<T, T>(X, M, o);
    return M;
}

/// first-tile owner of view C (process row/col)
template <typename T>
inline int row0_owner(BaseMatrix<T> const& C) { return C.mt() ? C.srow_owner(0) : 0; }
template <typename T>
inline int col0_owner(BaseMatrix<T> const& C) { return C.nt() ? C.scol_owner(0) : 0; }

/// do A's row tiles line up with C's (sizes and owners)?
template <typename T>
bool rows_conform(BaseMatrix<T> const& A, BaseMatrix<T> const& C) {
    if (A.op() != Op::NoTrans || !A.aligned() || !A.grid()->same_processes(*C.grid())) return false;
    if (A.grid()->p() != C.grid()->p() || A.grid()->q() != C.grid()->q() || A.grid()->order() != C.grid()->order()) return false;
    if (A.mt() != C.mt()) return false;
    for (int64_t i = 0; i < A.mt(); ++i)
        if (A.tileMb(i) != C.tileMb(i) || A.srow_owner(i) != C.srow_owner(i)) return false;
    return true;
}
template <typename T>
bool cols_conform(BaseMatrix<T> const& B, BaseMatrix<T> const& C) {
    if (B.op() != Op::NoTrans || !B.aligned() || !B.grid()->same_processes(*C.grid())) return false;
    if (B.grid()->p() != C.grid()->p() || B.grid()->q() != C.grid()->q() || B.grid()->order() != C.grid()->order()) return false;
    if (B.nt() != C.nt()) return false;
    for (int64_t j = 0; j < B.nt(); ++j)
        if (B.tileNb(j) != C.tileNb(j) || B.scol_owner(j) != C.scol_owner(j)) return false;
    return true;
}

}  // namespace

//------------------------------------------------------------------------------
template <typename T>
void gemmC(T alpha, Matrix<T> const& A_in, Matrix<T> const& B_in, T beta, Matrix<T>& C, Options const& opts) {
    trace::Block tb("gemmC");
    Target target = resolve_target(opts);
    const int64_t la = option_la(opts);
    slate_error_if_msg(A_in.m() != C.m() || B_in.n() != C.n() || A_in.n() != B_in.m(), "gemm: dimension mismatch");
    slate_error_if_msg(C.op() != Op::NoTrans, "gemm: C must not be a transposed view");
    slate_error_if_msg(!C.aligned(), "gemm: C must be tile aligned");
    auto gC = C.grid();
    // bring A and B into C-conforming layouts if needed (transposed views,
    // different grids or tilings)
    BaseMatrix<T> A = A_in, B = B_in;
    Matrix<T> Ac, Bc;
    if (!rows_conform(A, C)) {
        int64_t kb = A_in.nt() ? A_in.tileNb(0) : C.nb();
        Ac = materialize<T>(A_in, target, gC, C.mb(), kb, row0_owner(C), 0);
        A = Ac;
    }
    if (!cols_conform(B, C)) {
        int64_t kb = (B_in.mt() ? B_in.tileMb(0) : C.mb());
        if (A.nt()) kb = A.tileNb(0);
        Bc = materialize<T>(B_in, target, gC, kb, C.nb(), 0, col0_owner(C));
        B = Bc;
    }
    slate_error_if_msg(A.nt() != B.mt(), "gemm: inner tilings differ");
    for (int64_t k = 0; k < A.nt(); ++k)
        slate_error_if_msg(A.tileNb(k) != B.tileMb(k), "gemm: inner tile sizes differ");

    const Loc loc = loc_of(target);
    auto& g = *gC;
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    LocalBlock<T> lc = C.local(loc, true);
    LocalBlock<T> la_ = A.local(loc, false);
    LocalBlock<T> lb_ = B.local(loc, false);
    const int64_t kt = A.nt();
    Sched S(target);

    if (p == 1 && q == 1) {
        S.task(0, {}, {}, [&](lb::Ctx const& c) {
            trace::Block t2("gemm_local");
            lb::gemm(c, Op::NoTrans, Op::NoTrans, lc.m, lc.n, la_.n, alpha, la_.ptr, la_.ld, lb_.ptr, lb_.ld,
                     beta, lc.ptr, lc.ld);
        });
        S.wait_all();
        C.storage()->update_origin();
        return;
    }
    if (kt == 0) {
        S.wait_all();
        if (beta != T(1)) {
            lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
            lb::add(c, Uplo::General, lc.m, lc.n, T(0), lc.ptr, lc.ld, beta, lc.ptr, lc.ld);
            if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        }
        C.storage()->update_origin();
        return;
    }
    const int R = int(std::max<int64_t>(2, la + 2));
    int64_t kbmax = 0;
    for (int64_t k = 0; k < kt; ++k) kbmax = std::max(kbmax, A.tileNb(k));
    std::vector<Work<T>> WA(R), WB(R);
    for (int r = 0; r < R; ++r) {
        if (q > 1) WA[r].resize(target, size_t(std::max<int64_t>(lc.m, 1)) * kbmax);
        if (p > 1) WB[r].resize(target, size_t(kbmax) * std::max<int64_t>(lc.n, 1));
    }
    for (int64_t k = 0; k < kt; ++k) {
        const int slot = int(k % R);
        const int64_t kb = A.tileNb(k);
        const int qa = A.scol_owner(k), pb = B.srow_owner(k);
        T* pa = (q > 1) ? WA[slot].data() : nullptr;
        T* pbuf = (p > 1) ? WB[slot].data() : nullptr;
        int64_t ldwa = std::max<int64_t>(lc.m, 1), ldwb = kb;
        T const* Ak = nullptr; int64_t ldak = 0;
        T const* Bk = nullptr; int64_t ldbk = 0;
        if (q == 1) { Ak = la_.ptr + lcol_of(A, k) * la_.ld; ldak = la_.ld; }
        else { Ak = pa; ldak = ldwa; }
        if (p == 1) { Bk = lb_.ptr + lrow_of(B, k); ldbk = lb_.ld; }
        else { Bk = pbuf; ldbk = ldwb; }
        const int64_t tBc = Sched::bcast(slot);
        S.task(device::kCommQueue, {}, {tBc}, [&, k, kb, qa, pb, pa, pbuf, ldwa, ldwb](lb::Ctx const& c) {
            trace::Block t2("gemm_bcast");
            if (q > 1) {
                if (mycol == qa) pack(c, lc.m, kb, la_.ptr + lcol_of(A, k) * la_.ld, la_.ld, pa);
                bcast(g.row(), pa, size_t(lc.m * kb), qa, c);
            }
            if (p > 1) {
                if (myrow == pb) lb::copy2d(c, kb, lc.n, lb_.ptr + lrow_of(B, k), lb_.ld, pbuf, ldwb);
                bcast(g.col(), pbuf, size_t(kb * lc.n), pb, c);
            }
        });
        T bk = (k == 0) ? beta : T(1);
        S.task(0, {tBc}, {Sched::tok(9, 0)}, [&, Ak, ldak, Bk, ldbk, kb, bk](lb::Ctx const& c) {
            trace::Block t2("gemm_update");
            lb::gemm(c, Op::NoTrans, Op::NoTrans, lc.m, lc.n, kb, alpha, Ak, ldak, Bk, ldbk, bk, lc.ptr, lc.ld);
        });
    }
    S.wait_all();
    C.storage()->update_origin();
}

template <typename T>
void gemmA(T alpha, Matrix<T> const& A_in, Matrix<T> const& B_in, T beta, Matrix<T>& C, Options const& opts) {
    trace::Block tb("gemmA");
    Target target = resolve_target(opts);
    auto gC = C.grid();
    if (gC->size() == 1) { gemmC(alpha, A_in, B_in, beta, C, opts); return; }
    // stationary A: A conforms to C's rows; every process multiplies its
    // local A block by the matching rows of B (B gathered, it is narrow),
    // partial sums are reduced across the process row.
    BaseMatrix<T> A = A_in;
    Matrix<T> Ac;
    if (!rows_conform(A, C)) {
        int64_t kb = A_in.nt() ? A_in.tileNb(0) : C.nb();
        Ac = materialize<T>(A_in, target, gC, C.mb(), kb, row0_owner(C), 0);
        A = Ac;
    }
    std::vector<T> Bfull;
    gather(B_in, Bfull, opts);
    const int64_t k = A.n(), n = C.n();
    auto& g = *gC;
    const Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    LocalBlock<T> la_ = A.local(loc, false);
    auto& sa = *A.storage();
    // rows of B matching my local columns of A
    std::vector<T> Bl(size_t(std::max<int64_t>(la_.n, 1)) * n);
    for (int64_t jl = 0; jl < la_.n; ++jl) {
        int64_t kg = l2g(A.lcol_begin() + jl, sa.nb, sa.crel(), g.q()) - A.col0();
        for (int64_t j = 0; j < n; ++j) Bl[jl + j * la_.n] = Bfull[kg + j * k];
    }
    // partial P (my local rows x n) in host or device memory
    Work<T> P(target, size_t(std::max<int64_t>(la_.m, 1)) * n), Bd(target, Bl.size());
    if (c.dev()) device::memcpy_async(Bd.data(), Bl.data(), Bl.size() * sizeof(T), c.stream);
    else std::copy(Bl.begin(), Bl.end(), Bd.data());
    lb::gemm(c, Op::NoTrans, Op::NoTrans, la_.m, n, la_.n, T(1), la_.ptr, la_.ld,
             Bd.data(), std::max<int64_t>(la_.n, 1), T(0), P.data(), std::max<int64_t>(la_.m, 1));
    if (la_.n == 0) lb::set(c, Uplo::General, la_.m, n, T(0), T(0), P.data(), std::max<int64_t>(la_.m, 1));
    g.row().allreduce(P.data(), P.data(), size_t(la_.m) * n, scalar_type<T>(), ReduceOp::Sum, loc, c.stream);
    // owners of C's columns add alpha * P(:, their cols) + beta C
    LocalBlock<T> lc = C.local(loc, true);
    auto& sc = *C.storage();
    for (int64_t jl = 0; jl < lc.n; ++jl) {
        int64_t jg = l2g(C.lcol_begin() + jl, sc.nb, sc.crel(), g.q()) - C.col0();
        lb::add(c, Uplo::General, lc.m, 1, alpha, P.data() + jg * std::max<int64_t>(la_.m, 1),
                std::max<int64_t>(la_.m, 1), beta, lc.ptr + jl * lc.ld, lc.ld);
    }
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    C.storage()->update_origin();
}

template <typename T>
void gemm(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts) {
    Method m = get_option<int64_t>(opts, Option::MethodGemm, MethodGemm::Auto);
    if (m == MethodGemm::Auto) m = MethodGemm::select_algo(A, B, opts);
    if (m == MethodGemm::GemmA) gemmA(alpha, A, B, beta, C, opts);
    else gemmC(alpha, A, B, beta, C, opts);
}

//------------------------------------------------------------------------------
// trsm: block sweeps over B's block rows (Left).  Right-side and transposed
// solves are reduced to Left / NoTrans by explicit distributed transposes on
// grids larger than 1x1.
namespace {

template <typename T>
void trsm_left_notrans(Uplo uplo, Diag diag, T alpha, BaseMatrix<T> const& A, Matrix<T>& B, Target target,
                       int64_t la) {
    auto& g = *B.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    LocalBlock<T> lbk = B.local(loc, true);
    LocalBlock<T> lA = A.local(loc, false);
    const int64_t mt = B.mt();
    Sched S(target);
    // scale B by alpha once
    if (alpha != T(1))
        S.task(0, {}, {Sched::tok(9, 0)}, [&](lb::Ctx const& c) {
            lb::add(c, Uplo::General, lbk.m, lbk.n, T(0), lbk.ptr, lbk.ld, alpha, lbk.ptr, lbk.ld);
        });
    const int R = int(std::max<int64_t>(2, la + 2));
    int64_t nbmax = B.mb();
    std::vector<Work<T>> WA(R), WB(R), WD(R);
    for (int r = 0; r < R; ++r) {
        WA[r].resize(target, size_t(std::max<int64_t>(lbk.m, 1)) * nbmax);
        WB[r].resize(target, size_t(nbmax) * std::max<int64_t>(lbk.n, 1));
        WD[r].resize(target, size_t(nbmax) * nbmax);
    }
    const bool lower = (uplo == Uplo::Lower);
    for (int64_t t = 0; t < mt; ++t) {
        const int64_t k = lower ? t : mt - 1 - t;
        const int slot = int(t % R);
        const int64_t kb = B.tileMb(k);
        const int pk = B.srow_owner(k), qk = A.scol_owner(k);
        const int64_t lrk = lrow_of(B, k);
        T* D = WD[slot].data();
        T* WAk = WA[slot].data();
        T* WBk = WB[slot].data();
        // A(k,k) to every process of row pk; A(:,k) local rows along rows
        S.task(device::kCommQueue, {}, {Sched::bcast(slot)}, [&, k, kb, pk, qk, D, WAk](lb::Ctx const& c) {
            // diagonal tile: owner (pk, qk) -> process row pk
            if (myrow == pk) {
                if (mycol == qk) pack(c, kb, kb, lA.ptr + lrow_of(A, k) + lcol_of(A, k) * lA.ld, lA.ld, D);
                bcast(g.row(), D, size_t(kb * kb), qk, c);
            }
            // column panel A(:, k) rows local to me (all my rows) along process rows
            if (mycol == qk) pack(c, lbk.m, kb, lA.ptr + lcol_of(A, k) * lA.ld, lA.ld, WAk);
            bcast(g.row(), WAk, size_t(lbk.m * kb), qk, c);
        });
        // solve the block row on process row pk, then broadcast it down columns
        S.task(0, {Sched::bcast(slot)}, {Sched::tok(9, 0)}, [&, k, kb, pk, D, WBk, lrk](lb::Ctx const& c) {
            if (myrow == pk) {
                lb::trsm(c, Side::Left, uplo, Op::NoTrans, diag, kb, lbk.n, T(1), D, kb, lbk.ptr + lrk, lbk.ld);
                lb::copy2d(c, kb, lbk.n, lbk.ptr + lrk, lbk.ld, WBk, kb);
            }
        });
        S.task(device::kCommQueue, {Sched::tok(9, 0)}, {Sched::tok(8, slot)}, [&, kb, pk, WBk](lb::Ctx const& c) {
            bcast(g.col(), WBk, size_t(kb * lbk.n), pk, c);
        });
        // update the remaining block rows: B(i) -= A(i,k) X(k)
        S.task(0, {Sched::tok(8, slot), Sched::bcast(slot)}, {Sched::tok(9, 0)}, [&, k, kb, WAk, WBk](lb::Ctx const& c) {
            int64_t r0 = lower ? lrow_of(B, k + 1) : 0;
            int64_t r1 = lower ? lbk.m : lrow_of(B, k);
            if (r1 > r0)
                lb::gemm(c, Op::NoTrans, Op::NoTrans, r1 - r0, lbk.n, kb, T(-1), WAk + r0, std::max<int64_t>(lbk.m, 1),
                         WBk, kb, T(1), lbk.ptr + r0, lbk.ld);
        });
    }
    S.wait_all();
}

}  // namespace

template <typename T>
void trsm(Side side, T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("trsm");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    auto gB = B.grid();
    if (gB->size() == 1 && A.grid()->size() == 1 && B.op() == Op::NoTrans) {
        LocalBlock<T> lA = A.local(loc, false);
        LocalBlock<T> lbk = B.local(loc, true);
        lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
        // A's logical op applied to its physical triangle
        lb::trsm(c, side, A.uplo_physical(), A.op(), A.diag(), lbk.m, lbk.n, alpha, lA.ptr, lA.ld, lbk.ptr, lbk.ld);
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        B.storage()->update_origin();
        return;
    }
    // distributed: reduce to Left, NoTrans, A conforming to B's rows
    if (side == Side::Right) {
        // X op(A) = alpha B  <=>  op(A)^T X^T = alpha B^T (use conj for ConjTrans pairs)
        bool conj = is_complex_v<T>;
        Matrix<T> Bt = materialize<T>(conj ? conj_transpose(B) : transpose(B), target, gB, B.nb(), B.mb(),
                                      0, 0);
        TriangularMatrix<T> Ah = conj ? conj_transpose(A) : transpose(A);
        TriangularMatrix<T> At(Ah.uplo(), A.diag(), Ah);
        trsm(Side::Left, conj ? slate::conj(alpha) : alpha, At, Bt, opts);
        slate::copy<T, T>(conj ? conj_transpose(Bt) : transpose(Bt), B, opts);
        return;
    }
    // materialize op(A) as a NoTrans triangle conforming to B (rows and cols)
    Uplo u = A.uplo();
    BaseMatrix<T> Ause = A;
    Matrix<T> Ac;
    bool conform = A.op() == Op::NoTrans && rows_conform(BaseMatrix<T>(A), BaseMatrix<T>(B)) &&
                   A.grid()->same_processes(*gB);
    if (conform) {
        for (int64_t j = 0; j < A.nt(); ++j) if (A.tileNb(j) != B.tileMb(j)) conform = false;
    }
    if (!conform) {
        Ac = materialize<T>(A, target, gB, B.mb(), B.mb(), row0_owner(B), 0);
        Ause = Ac;
    }
    trsm_left_notrans(u, A.diag(), alpha, Ause, B, target, option_la(opts));
    B.storage()->update_origin();
}

//------------------------------------------------------------------------------
// herk / syrk / her2k / syr2k / hemm / symm / trmm
namespace {

template <typename T>
bool local_only(BaseMatrix<T> const& A) { return A.grid()->size() == 1; }

inline lb::Ctx ctx_for(Target t) { return t == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host(); }
inline void sync_ctx(lb::Ctx const& c) { if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream)); }

/// C(uplo) = alpha * G + beta * C(uplo) with G general (same layout as C)
template <typename T>
void tri_axpby(T alpha, Matrix<T> const& G, T beta, BaseTrapezoidMatrix<T>& C, Target target) {
    Options o = {{Option::Target, target}};
    BaseTrapezoidMatrix<T> Gt(C.uplo(), G, MatrixKind::Trapezoid);
    add(alpha, Gt, beta, C, o);
}

}  // namespace

namespace {

/// C(uplo) = alpha * A * B + beta * C(uplo) on a p x q grid, touching only the
/// stored triangle of C: the reference's herk/syrk/her2k updates do a
/// triangular product on the diagonal tiles and a gemm on the off-diagonal
/// ones and never form the other triangle (internal_herk.cc:491-515).  Here:
/// SUMMA over k with gemmC's whole-panel broadcasts (A(:, k) along process
/// rows, B(k, :) down process columns), and per local tile column J one
/// triangular-output MFMA GEMM on the diagonal tile (when local) plus one
/// GEMM over the local tiles strictly inside the triangle.
template <typename T>
void tri_summa(Uplo uplo, T alpha, BaseMatrix<T> const& A_in, BaseMatrix<T> const& B_in, T beta,
               BaseMatrix<T> const& C, Options const& opts) {
    Target target = resolve_target(opts);
    const int64_t la = option_la(opts);
    auto gC = C.grid();
    BaseMatrix<T> A = A_in, B = B_in;
    Matrix<T> Ac, Bc;
    if (!rows_conform(A, C)) {
        int64_t kb = A_in.nt() ? A_in.tileNb(0) : C.nb();
        Ac = materialize<T>(A_in, target, gC, C.mb(), kb, row0_owner(C), 0);
        A = Ac;
    }
    if (!cols_conform(B, C)) {
        int64_t kb = A.nt() ? A.tileNb(0) : C.mb();
        Bc = materialize<T>(B_in, target, gC, kb, C.nb(), 0, col0_owner(C));
        B = Bc;
    }
    slate_error_if_msg(A.nt() != B.mt(), "tri_summa: inner tilings differ");
    // scale the stored triangle by beta once
    if (beta != T(1)) {
        Options o = {{Option::Target, target}};
        BaseTrapezoidMatrix<T> Ct(uplo, C, MatrixKind::Trapezoid);
        add(T(0), Ct, beta, Ct, o);
    }
    const Loc loc = loc_of(target);
    auto& g = *gC;
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    LocalBlock<T> lc = C.local(loc, true);
    LocalBlock<T> la_ = A.local(loc, false);
    LocalBlock<T> lb_ = B.local(loc, false);
    const int64_t kt = A.nt(), nt = C.nt();
    Sched S(target);
    const int R = int(std::max<int64_t>(2, la + 2));
    int64_t kbmax = 0;
    for (int64_t k = 0; k < kt; ++k) kbmax = std::max(kbmax, A.tileNb(k));
    std::vector<Work<T>> WA(R), WB(R);
    for (int r = 0; r < R; ++r) {
        if (q > 1) WA[r].resize(target, size_t(std::max<int64_t>(lc.m, 1)) * std::max<int64_t>(kbmax, 1));
        if (p > 1) WB[r].resize(target, size_t(std::max<int64_t>(kbmax, 1)) * std::max<int64_t>(lc.n, 1));
    }
    // my local tile columns of C
    std::vector<int64_t> myJ;
    for (int64_t J = 0; J < nt; ++J) if (C.scol_owner(J) == mycol) myJ.push_back(J);
    for (int64_t k = 0; k < kt; ++k) {
        const int slot = int(k % R);
        const int64_t kb = A.tileNb(k);
        const int qa = A.scol_owner(k), pb = B.srow_owner(k);
        T* pa = (q > 1) ? WA[slot].data() : nullptr;
        T* pbuf = (p > 1) ? WB[slot].data() : nullptr;
        T const* Ak = (q == 1) ? la_.ptr + lcol_of(A, k) * la_.ld : pa;
        const int64_t ldak = (q == 1) ? la_.ld : std::max<int64_t>(lc.m, 1);
        T const* Bk = (p == 1) ? lb_.ptr + lrow_of(B, k) : pbuf;
        const int64_t ldbk = (p == 1) ? lb_.ld : kb;
        const int64_t tBc = Sched::bcast(slot);
        S.task(device::kCommQueue, {}, {tBc}, [&, k, kb, qa, pb, pa, pbuf](lb::Ctx const& c) {
            trace::Block t2("trisumma_bcast");
            if (q > 1) {
                if (mycol == qa) pack(c, lc.m, kb, la_.ptr + lcol_of(A, k) * la_.ld, la_.ld, pa);
                bcast(g.row(), pa, size_t(lc.m * kb), qa, c);
            }
            if (p > 1) {
                if (myrow == pb) lb::copy2d(c, kb, lc.n, lb_.ptr + lrow_of(B, k), lb_.ld, pbuf, kb);
                bcast(g.col(), pbuf, size_t(kb * lc.n), pb, c);
            }
        });
        S.task(0, {tBc}, {Sched::tok(9, 0)}, [&, Ak, ldak, Bk, ldbk, kb](lb::Ctx const& c) {
            trace::Block t2("trisumma_update");
            for (int64_t J : myJ) {
                const int64_t c0 = lcol_of(C, J), nc = lcol_of(C, J + 1) - c0;
                const int64_t r0 = lrow_of(C, J), r1 = lrow_of(C, J + 1);   // my rows of tile row J
                const bool diag_local = (C.srow_owner(J) == myrow) && r1 > r0;
                if (uplo == Uplo::Lower) {
                    if (diag_local)
                        lb::gemm_tri(c, Uplo::Lower, Op::NoTrans, Op::NoTrans, nc, kb, alpha, Ak + r0, ldak,
                                     Bk + c0 * ldbk, ldbk, T(1), lc.ptr + r0 + c0 * lc.ld, lc.ld);
                    const int64_t rs = diag_local ? r1 : r0;          // rows strictly below tile row J
                    if (lc.m > rs)
                        lb::gemm(c, Op::NoTrans, Op::NoTrans, lc.m - rs, nc, kb, alpha, Ak + rs, ldak,
                                 Bk + c0 * ldbk, ldbk, T(1), lc.ptr + rs + c0 * lc.ld, lc.ld);
                } else {
                    if (diag_local)
                        lb::gemm_tri(c, Uplo::Upper, Op::NoTrans, Op::NoTrans, nc, kb, alpha, Ak + r0, ldak,
                                     Bk + c0 * ldbk, ldbk, T(1), lc.ptr + r0 + c0 * lc.ld, lc.ld);
                    if (r0 > 0)                                        // rows strictly above tile row J
                        lb::gemm(c, Op::NoTrans, Op::NoTrans, r0, nc, kb, alpha, Ak, ldak, Bk + c0 * ldbk, ldbk,
                                 T(1), lc.ptr + c0 * lc.ld, lc.ld);
                }
            }
        });
    }
    S.wait_all();
    C.storage()->update_origin();
}

}  // namespace

template <typename T>
void herk(real_type<T> alpha, Matrix<T> const& A, real_type<T> beta, HermitianMatrix<T>& C, Options const& opts) {
    trace::Block tb("herk");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && C.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lc = C.local(loc, true);
        Op op = A.op() == Op::NoTrans ? Op::NoTrans : Op::ConjTrans;
        lb::herk(c, C.uplo(), op, lc.m, A.n(), alpha, la_.ptr, la_.ld, beta, lc.ptr, lc.ld);
        sync_ctx(c);
        C.storage()->update_origin();
        return;
    }
    if (C.op() == Op::NoTrans && C.aligned() && C.mb() == C.nb()) {
        tri_summa<T>(C.uplo(), T(alpha), A, conj_transpose(A), T(beta), C, opts);
        return;
    }
    Matrix<T> G = Matrix<T>(C).emptyLike();
    G.insertLocalTiles(target);
    gemmC(T(1), A, conj_transpose(A), T(0), G, opts);
    tri_axpby(T(alpha), G, T(beta), C, target);
}

template <typename T>
void syrk(T alpha, Matrix<T> const& A, T beta, SymmetricMatrix<T>& C, Options const& opts) {
    trace::Block tb("syrk");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && C.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lc = C.local(loc, true);
        Op op = A.op() == Op::NoTrans ? Op::NoTrans : Op::Trans;
        lb::syrk(c, C.uplo(), op, lc.m, A.n(), alpha, la_.ptr, la_.ld, beta, lc.ptr, lc.ld);
        sync_ctx(c);
        C.storage()->update_origin();
        return;
    }
    if (C.op() == Op::NoTrans && C.aligned() && C.mb() == C.nb()) {
        tri_summa<T>(C.uplo(), alpha, A, transpose(A), beta, C, opts);
        return;
    }
    Matrix<T> G = Matrix<T>(C).emptyLike();
    G.insertLocalTiles(target);
    gemmC(T(1), A, transpose(A), T(0), G, opts);
    tri_axpby(alpha, G, beta, C, target);
}

template <typename T>
void her2k(T alpha, Matrix<T> const& A, Matrix<T> const& B, real_type<T> beta, HermitianMatrix<T>& C,
           Options const& opts) {
    trace::Block tb("her2k");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && local_only(B) && C.op() == Op::NoTrans && A.op() == B.op()) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
        Op op = A.op() == Op::NoTrans ? Op::NoTrans : Op::ConjTrans;
        lb::her2k(c, C.uplo(), op, lc.m, A.n(), alpha, la_.ptr, la_.ld, lbk.ptr, lbk.ld, beta, lc.ptr, lc.ld);
        sync_ctx(c);
        C.storage()->update_origin();
        return;
    }
    if (C.op() == Op::NoTrans && C.aligned() && C.mb() == C.nb()) {
        tri_summa<T>(C.uplo(), alpha, A, conj_transpose(B), T(beta), C, opts);
        tri_summa<T>(C.uplo(), slate::conj(alpha), B, conj_transpose(A), T(1), C, opts);
        return;
    }
    Matrix<T> G = Matrix<T>(C).emptyLike();
    G.insertLocalTiles(target);
    gemmC(alpha, A, conj_transpose(B), T(0), G, opts);
    gemmC(slate::conj(alpha), B, conj_transpose(A), T(1), G, opts);
    tri_axpby(T(1), G, T(beta), C, target);
}

template <typename T>
void syr2k(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, SymmetricMatrix<T>& C, Options const& opts) {
    trace::Block tb("syr2k");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && local_only(B) && C.op() == Op::NoTrans && A.op() == B.op()) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
        Op op = A.op() == Op::NoTrans ? Op::NoTrans : Op::Trans;
        lb::syr2k(c, C.uplo(), op, lc.m, A.n(), alpha, la_.ptr, la_.ld, lbk.ptr, lbk.ld, beta, lc.ptr, lc.ld);
        sync_ctx(c);
        C.storage()->update_origin();
        return;
    }
    if (C.op() == Op::NoTrans && C.aligned() && C.mb() == C.nb()) {
        tri_summa<T>(C.uplo(), alpha, A, transpose(B), beta, C, opts);
        tri_summa<T>(C.uplo(), alpha, B, transpose(A), T(1), C, opts);
        return;
    }
    Matrix<T> G = Matrix<T>(C).emptyLike();
    G.insertLocalTiles(target);
    gemmC(alpha, A, transpose(B), T(0), G, opts);
    gemmC(alpha, B, transpose(A), T(1), G, opts);
    tri_axpby(T(1), G, beta, C, target);
}

namespace {

/// B := alpha A B, A triangular (NoTrans, conforming to B's rows and with
/// square tiles), on a p x q grid: SUMMA over k where step k only touches
/// the rows that A(:, k) reaches -- tile rows >= k (Lower) or <= k (Upper) --
/// instead of a dense product with explicit zeros (reference src/trmm.cc +
/// work::trmm).  B's old values are read from a copy; the diagonal tile of
/// each broadcast panel is masked to its triangle (unit diagonal if asked).
template <typename T>
void trmm_left_notrans(Uplo uplo, Diag diag, T alpha, BaseMatrix<T> const& A, Matrix<T>& B, Target target,
                       int64_t la) {
    Options o = {{Option::Target, target}};
    Matrix<T> B0 = B.emptyLike();
    B0.insertLocalTiles(target);
    slate::copy<T, T>(B, B0, o);
    auto& g = *B.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    LocalBlock<T> lbk = B.local(loc, true);
    LocalBlock<T> lb0 = B0.local(loc, false);
    LocalBlock<T> lA = A.local(loc, false);
    const int64_t kt = A.nt();
    Sched S(target);
    const int R = int(std::max<int64_t>(2, la + 2));
    const int64_t nb = B.mb();
    std::vector<Work<T>> WA(R), WB(R);
    for (int r = 0; r < R; ++r) {
        WA[r].resize(target, size_t(std::max<int64_t>(lbk.m, 1)) * nb);
        if (p > 1) WB[r].resize(target, size_t(nb) * std::max<int64_t>(lbk.n, 1));
    }
    const bool lower = (uplo == Uplo::Lower);
    // Lower: panel k reaches rows >= k, so k = 0 touches every row first;
    // Upper: rows <= k, so run k downwards
    for (int64_t kk = 0; kk < kt; ++kk) {
        const int64_t k = lower ? kk : kt - 1 - kk;
        const int slot = int(kk % R);
        const int64_t kb = A.tileNb(k);
        const int qk = A.scol_owner(k), pk = B.srow_owner(k);
        const int64_t r0 = lower ? lrow_of(B, k) : 0, r1 = lower ? lbk.m : lrow_of(B, k + 1);  // rows A(:, k) reaches
        const int64_t rk = lrow_of(B, k);
        T* WAk = WA[slot].data();
        T* WBk = (p > 1) ? WB[slot].data() : nullptr;
        const int64_t tBc = Sched::bcast(slot);
        S.task(device::kCommQueue, {}, {tBc}, [&, k, kb, qk, pk, r0, r1, rk, WAk, WBk](lb::Ctx const& c) {
            trace::Block t2("trmm_bcast");
            const int64_t nr = r1 - r0;
            if (nr > 0) {
                if (mycol == qk) pack(c, nr, kb, lA.ptr + r0 + lcol_of(A, k) * lA.ld, lA.ld, WAk);
                if (q > 1) bcast(g.row(), WAk, size_t(nr * kb), qk, c);
                if (myrow == pk) {
                    // diagonal tile sits at rows rk - r0 of the panel: keep its triangle only
                    T* D = WAk + (rk - r0);
                    if (kb > 1) {
                        if (lower) lb::set(c, Uplo::Upper, kb - 1, kb - 1, T(0), T(0), D + nr, nr);
                        else lb::set(c, Uplo::Lower, kb - 1, kb - 1, T(0), T(0), D + 1, nr);
                    }
                    if (diag == Diag::Unit) lb::set(c, Uplo::General, 1, kb, T(1), T(1), D, nr + 1);
                }
            }
            if (p > 1) {
                if (myrow == pk) lb::copy2d(c, kb, lb0.n, lb0.ptr + rk, lb0.ld, WBk, kb);
                bcast(g.col(), WBk, size_t(kb * lb0.n), pk, c);
            }
        });
        T const* Bk = (p > 1) ? WBk : lb0.ptr + rk;
        const int64_t ldbk = (p > 1) ? kb : lb0.ld;
        S.task(0, {tBc}, {Sched::tok(9, 0)}, [&, r0, r1, kb, WAk, Bk, ldbk, kk](lb::Ctx const& c) {
            trace::Block t2("trmm_update");
            const int64_t nr = r1 - r0;
            if (nr > 0)
                lb::gemm(c, Op::NoTrans, Op::NoTrans, nr, lbk.n, kb, alpha, WAk, nr, Bk, ldbk, kk == 0 ? T(0) : T(1),
                         lbk.ptr + r0, lbk.ld);
        });
    }
    S.wait_all();
}

/// full (dense) copy of a symmetric/Hermitian matrix on the same layout
template <typename T>
Matrix<T> expand_sym(BaseTrapezoidMatrix<T> const& A, bool herm, Target target) {
    Options o = {{Option::Target, target}};
    Matrix<T> F = Matrix<T>(BaseMatrix<T>(A)).emptyLike();
    F.insertLocalTiles(target);
    // mirror: F = op(A) fully, then overwrite the stored triangle
    Matrix<T> Ag{BaseMatrix<T>(A)};
    Ag.set_uplo(Uplo::General);
    slate::copy<T, T>(herm ? conj_transpose(Ag) : transpose(Ag), F, o);
    BaseTrapezoidMatrix<T> Ft(A.uplo(), F, MatrixKind::Trapezoid);
    BaseTrapezoidMatrix<T> At(A.uplo(), Ag, MatrixKind::Trapezoid);
    slate::copy<T, T>(At, Ft, o);
    return F;
}

}  // namespace

template <typename T>
void hemm(Side side, T alpha, HermitianMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts) {
    trace::Block tb("hemm");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && local_only(B) && C.op() == Op::NoTrans && B.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
        lb::hemm(c, side, A.uplo_physical(), lc.m, lc.n, alpha, la_.ptr, la_.ld, lbk.ptr, lbk.ld, beta,
                 lc.ptr, lc.ld, true);
        sync_ctx(c);
        C.storage()->update_origin();
        return;
    }
    Matrix<T> F = expand_sym<T>(A, true, target);
    if (side == Side::Left) gemmC(alpha, F, B, beta, C, opts);
    else gemmC(alpha, B, F, beta, C, opts);
}

template <typename T>
void symm(Side side, T alpha, SymmetricMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts) {
    trace::Block tb("symm");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && local_only(B) && C.op() == Op::NoTrans && B.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
        lb::hemm(c, side, A.uplo_physical(), lc.m, lc.n, alpha, la_.ptr, la_.ld, lbk.ptr, lbk.ld, beta,
                 lc.ptr, lc.ld, false);
        sync_ctx(c);
        C.storage()->update_origin();
        return;
    }
    Matrix<T> F = expand_sym<T>(A, false, target);
    if (side == Side::Left) gemmC(alpha, F, B, beta, C, opts);
    else gemmC(alpha, B, F, beta, C, opts);
}

template <typename T>
void trmm(Side side, T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("trmm");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(B) && local_only(A) && B.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, true);
        lb::trmm(c, side, A.uplo_physical(), A.op(), A.diag(), lbk.m, lbk.n, alpha, la_.ptr, la_.ld,
                 lbk.ptr, lbk.ld);
        sync_ctx(c);
        B.storage()->update_origin();
        return;
    }
    // distributed: reduce to Left with a NoTrans triangle conforming to B's
    // rows (as trsm does), then a SUMMA that skips the zero part of A
    auto gB = B.grid();
    if (side == Side::Right) {
        // B op(A) = (op(A)^H B^H)^H
        bool conj = is_complex_v<T>;
        Matrix<T> Bt = materialize<T>(conj ? conj_transpose(B) : transpose(B), target, gB, B.nb(), B.mb(), 0, 0);
        TriangularMatrix<T> Ah = conj ? conj_transpose(A) : transpose(A);
        TriangularMatrix<T> At(Ah.uplo(), A.diag(), Ah);
        trmm(Side::Left, conj ? slate::conj(alpha) : alpha, At, Bt, opts);
        slate::copy<T, T>(conj ? conj_transpose(Bt) : transpose(Bt), B, opts);
        return;
    }
    BaseMatrix<T> Ause = A;
    Matrix<T> Ac;
    bool conform = A.op() == Op::NoTrans && rows_conform(BaseMatrix<T>(A), BaseMatrix<T>(B)) &&
                   A.grid()->same_processes(*gB);
    if (conform)
        for (int64_t j = 0; j < A.nt(); ++j) if (A.tileNb(j) != B.tileMb(j)) conform = false;
    if (!conform) {
        Ac = materialize<T>(A, target, gB, B.mb(), B.mb(), row0_owner(B), 0);
        Ause = Ac;
    }
    trmm_left_notrans<T>(A.uplo(), A.diag(), alpha, Ause, B, target, option_la(opts));
    B.storage()->update_origin();
}

//------------------------------------------------------------------------------
#define SLATE_BLAS3_INST(T)                                                                              \
    template void gemm<T>(T, Matrix<T> const&, Matrix<T> const&, T, Matrix<T>&, Options const&);        \
    template void gemmA<T>(T, Matrix<T> const&, Matrix<T> const&, T, Matrix<T>&, Options const&);       \
    template void gemmC<T>(T, Matrix<T> const&, Matrix<T> const&, T, Matrix<T>&, Options const&);       \
    template void trsm<T>(Side, T, TriangularMatrix<T> const&, Matrix<T>&, Options const&);             \
    template void trmm<T>(Side, T, TriangularMatrix<T> const&, Matrix<T>&, Options const&);             \
    template void herk<T>(real_type<T>, Matrix<T> const&, real_type<T>, HermitianMatrix<T>&, Options const&); \
    template void syrk<T>(T, Matrix<T> const&, T, SymmetricMatrix<T>&, Options const&);                 \
    template void her2k<T>(T, Matrix<T> const&, Matrix<T> const&, real_type<T>, HermitianMatrix<T>&, Options const&); \
    template void syr2k<T>(T, Matrix<T> const&, Matrix<T> const&, T, SymmetricMatrix<T>&, Options const&); \
    template void hemm<T>(Side, T, HermitianMatrix<T> const&, Matrix<T> const&, T, Matrix<T>&, Options const&); \
    template void symm<T>(Side, T, SymmetricMatrix<T> const&, Matrix<T> const&, T, Matrix<T>&, Options const&);

SLATE_BLAS3_INST(float)
SLATE_BLAS3_INST(double)
SLATE_BLAS3_INST(std::complex<float>)
SLATE_BLAS3_INST(std::complex<double>)

}  // namespace slate
