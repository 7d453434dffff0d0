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
//   the zero part of each A panel.  hemm/symm: hemmC (SUMMA over the stored
//   triangle, partial A^H B products reduced down process columns) or hemmA
//   (stationary A, narrow B replicated, one world reduction); MethodHemm.
// gemmA / trsmA / hemmA replicate the narrow operand on the device instead of
//   moving A (reference method.hh select_algo: B.nt() < 2).
#include "internal.hh"
#include "spread.hh"

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
inline lb::Ctx ctx_for(Target t) { return t == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host(); }
inline void sync_ctx(lb::Ctx const& c) { if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream)); }

/// in-place sum over `comm` of a contiguous buffer (stream-ordered)
template <typename T>
inline void allreduce_sum(Comm& comm, T* buf, size_t count, lb::Ctx const& c) {
    if (comm.size() == 1 || count == 0) return;
    comm.allreduce(buf, buf, count, scalar_type<T>(), ReduceOp::Sum, c.loc(), c.stream);
}

/// Stationary-A building block: every process of the grid gets the whole
/// (narrow) NoTrans matrix X in G (X.m() x X.n(), ld X.m()) -- zero fill,
/// local tiles written at their global positions, one world allreduce --
/// O(m n) traffic on the device, no host gather.
template <typename T>
void replicate(lb::Ctx const& c, BaseMatrix<T> const& X, T* G) {
    const int64_t ldg = std::max<int64_t>(X.m(), 1);
    lb::set(c, Uplo::General, X.m(), X.n(), T(0), T(0), G, ldg);
    LocalBlock<T> lx = X.local(c.loc(), false);
    auto& g = *X.grid();
    for (int64_t i = 0; i < X.mt(); ++i) {
        if (X.srow_owner(i) != g.myrow()) continue;
        for (int64_t j = 0; j < X.nt(); ++j)
            if (X.scol_owner(j) == g.mycol())
                lb::copy2d(c, X.tileMb(i), X.tileNb(j), lx.ptr + lrow_of(X, i) + lcol_of(X, j) * lx.ld, lx.ld,
                           G + grow_of(X, i) + gcol_of(X, j) * ldg, ldg);
    }
    allreduce_sum(g.world(), G, size_t(ldg) * X.n(), c);
}

/// rows of a replicated global G (ld ldg, n columns) at A's local row tiles
/// (by_cols: at A's local column tiles) -> W (ld ldw); add = true adds W back
/// into G instead (W -> G, G += W).
template <typename T>
void gather_local(lb::Ctx const& c, BaseMatrix<T> const& A, bool by_cols, T* G, int64_t ldg, int64_t n, T* W,
                  int64_t ldw, bool add) {
    auto& g = *A.grid();
    const int64_t nt = by_cols ? A.nt() : A.mt();
    for (int64_t t = 0; t < nt; ++t) {
        if ((by_cols ? A.scol_owner(t) : A.srow_owner(t)) != (by_cols ? g.mycol() : g.myrow())) continue;
        const int64_t sz = by_cols ? A.tileNb(t) : A.tileMb(t);
        T* gp = G + (by_cols ? gcol_of(A, t) : grow_of(A, t));
        T* wp = W + (by_cols ? lcol_of(A, t) : lrow_of(A, t));
        if (add) lb::add(c, Uplo::General, sz, n, T(1), wp, ldw, T(1), gp, ldg);
        else lb::copy2d(c, sz, n, gp, ldg, wp, ldw);
    }
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
    internal::DriverScope ds_;
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
        internal::finish_origin(C, opts);
        return;
    }
    if (kt == 0) {
        S.wait_all();
        if (beta != T(1)) {
            lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
            lb::add(c, Uplo::General, lc.m, lc.n, T(0), lc.ptr, lc.ld, beta, lc.ptr, lc.ld);
            if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        }
        internal::finish_origin(C, opts);
        return;
    }
    // Wide SUMMA steps: w consecutive k tiles are broadcast into one
    // buffer per operand (one message per tile, each from its owner) and
    // multiplied by ONE local GEMM with K = w nb.  A K = 512 GEMM runs ~11 %
    // below the long-K rate (profiles/r5_critpath_2x4.txt: 63.2 vs 70.9
    // TFLOP/s); with 288 GB per GPU the wider panels cost nothing that
    // matters.  $SLATE_SUMMA_K = target K per step (default 2048; <= nb: one
    // tile per step, the classic SUMMA).
    const int64_t summa_k = [] {
        const char* e = std::getenv("SLATE_SUMMA_K");
        return e ? std::max<int64_t>(1, std::atoll(e)) : int64_t(2048);
    }();
    int64_t kbmax = 0;
    for (int64_t k = 0; k < kt; ++k) kbmax = std::max(kbmax, A.tileNb(k));
    const int64_t w = std::max<int64_t>(1, std::min<int64_t>(kt, summa_k / std::max<int64_t>(kbmax, 1)));
    const int R = int(std::max<int64_t>(2, la + 2));
    const int64_t kw = w * kbmax;                       // widest K of a step
    std::vector<Work<T>> WA(R), WB(R), WS(R);
    for (int r = 0; r < R; ++r) {
        if (q > 1) WA[r].resize(target, size_t(std::max<int64_t>(lc.m, 1)) * kw);
        if (p > 1) WB[r].resize(target, size_t(kw) * std::max<int64_t>(lc.n, 1));
        if (p > 1 && w > 1) WS[r].resize(target, size_t(kbmax) * std::max<int64_t>(lc.n, 1));
    }
    const int64_t nsteps = (kt + w - 1) / w;
    const int gq = target == Target::Devices ? device::full_queue() : 0;
    for (int64_t st = 0; st < nsteps; ++st) {
        const int slot = int(st % R);
        const int64_t k0 = st * w, k1 = std::min(kt, k0 + w);   // tiles [k0, k1)
        int64_t K = 0;
        for (int64_t k = k0; k < k1; ++k) K += A.tileNb(k);
        T* pa = (q > 1) ? WA[slot].data() : nullptr;
        T* pbuf = (p > 1) ? WB[slot].data() : nullptr;
        const int64_t ldwa = std::max<int64_t>(lc.m, 1), ldwb = std::max<int64_t>(K, 1);
        T const* Ak = nullptr; int64_t ldak = 0;
        T const* Bk = nullptr; int64_t ldbk = 0;
        // one process column (row): the step's tiles are adjacent local columns (rows)
        if (q == 1) { Ak = la_.ptr + lcol_of(A, k0) * la_.ld; ldak = la_.ld; }
        else { Ak = pa; ldak = ldwa; }
        if (p == 1) { Bk = lb_.ptr + lrow_of(B, k0); ldbk = lb_.ld; }
        else { Bk = pbuf; ldbk = ldwb; }
        const int64_t tBc = Sched::bcast(slot);
        S.task(device::kCommQueue, {}, {tBc}, [&, k0, k1, slot, pa, pbuf, ldwa, ldwb](lb::Ctx const& c) {
            trace::Block t2("gemm_bcast");
            int64_t off = 0;
            for (int64_t k = k0; k < k1; ++k) {
                const int64_t kb = A.tileNb(k);
                if (q > 1) {
                    const int qa = A.scol_owner(k);
                    T* dst = pa + off * ldwa;
                    if (mycol == qa) pack(c, lc.m, kb, la_.ptr + lcol_of(A, k) * la_.ld, la_.ld, dst);
                    bcast(g.row(), dst, size_t(lc.m * kb), qa, c);
                }
                if (p > 1) {
                    // B(k, :) travels packed (kb x n contiguous) and lands in
                    // rows [off, off + kb) of the step's K x n operand
                    const int pb = B.srow_owner(k);
                    T* msg = (w == 1) ? pbuf : WS[slot].data();
                    if (myrow == pb) lb::copy2d(c, kb, lc.n, lb_.ptr + lrow_of(B, k), lb_.ld, msg, kb);
                    bcast(g.col(), msg, size_t(kb * lc.n), pb, c);
                    if (w > 1) lb::copy2d(c, kb, lc.n, msg, kb, pbuf + off, ldwb);
                }
                off += kb;
            }
        });
        T bk = (st == 0) ? beta : T(1);
        // no panel chain to protect: the GEMMs take every CU (device::full_queue)
        S.task(gq, {tBc}, {Sched::tok(9, 0)}, [&, Ak, ldak, Bk, ldbk, K, bk](lb::Ctx const& c) {
            trace::Block t2("gemm_update");
            lb::PackAHint tn;   // K = summa_k steps: TN on a packed A beats NT on a copied B
            lb::gemm(c, Op::NoTrans, Op::NoTrans, lc.m, lc.n, K, alpha, Ak, ldak, Bk, ldbk, bk, lc.ptr, lc.ld);
        });
    }
    S.wait_all();
    internal::finish_origin(C, opts);
}

template <typename T>
void gemmA(T alpha, Matrix<T> const& A_in, Matrix<T> const& B_in, T beta, Matrix<T>& C, Options const& opts) {
    trace::Block tb("gemmA");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    auto gC = C.grid();
    if (gC->size() == 1) { gemmC(alpha, A_in, B_in, beta, C, opts); return; }
    // stationary A: A conforms to C's rows; B (narrow) is replicated on the
    // device with one world allreduce, every process multiplies its local A
    // block by the rows of B matching its local columns, and the partial
    // products are summed across the process row (reference src/gemmA.cc).
    BaseMatrix<T> A = A_in;
    Matrix<T> Ac, Bc;
    if (!rows_conform(A, C)) {
        int64_t kb = A_in.nt() ? A_in.tileNb(0) : C.nb();
        Ac = materialize<T>(A_in, target, gC, C.mb(), kb, row0_owner(C), 0);
        A = Ac;
    }
    BaseMatrix<T> B = B_in;
    if (B_in.op() != Op::NoTrans || !B_in.grid()->same_processes(*gC)) {
        Bc = materialize<T>(B_in, target, gC, B_in.m() ? std::min<int64_t>(B_in.m(), A.mb()) : 1,
                            std::max<int64_t>(B_in.n(), 1), 0, 0);
        B = Bc;
    }
    const int64_t k = A.n(), n = C.n();
    auto& g = *gC;
    const Loc loc = loc_of(target);
    lb::Ctx c = ctx_for(target);
    LocalBlock<T> la_ = A.local(loc, false);
    const int64_t ldbl = std::max<int64_t>(la_.n, 1), ldp = std::max<int64_t>(la_.m, 1);
    Work<T> G(target, size_t(std::max<int64_t>(k, 1)) * std::max<int64_t>(n, 1));
    Work<T> Bl(target, size_t(ldbl) * std::max<int64_t>(n, 1)), P(target, size_t(ldp) * std::max<int64_t>(n, 1));
    replicate(c, B, G.data());
    gather_local(c, A, true, G.data(), std::max<int64_t>(k, 1), n, Bl.data(), ldbl, false);
    if (la_.n > 0)
        lb::gemm(c, Op::NoTrans, Op::NoTrans, la_.m, n, la_.n, T(1), la_.ptr, la_.ld, Bl.data(), ldbl, T(0),
                 P.data(), ldp);
    else
        lb::set(c, Uplo::General, la_.m, n, T(0), T(0), P.data(), ldp);
    allreduce_sum(g.row(), P.data(), size_t(ldp) * n, c);
    // owners of C's column tiles: C = alpha P(:, their cols) + beta C
    LocalBlock<T> lc = C.local(loc, true);
    for (int64_t j = 0; j < C.nt(); ++j)
        if (C.scol_owner(j) == g.mycol())
            lb::add(c, Uplo::General, lc.m, C.tileNb(j), alpha, P.data() + gcol_of(C, j) * ldp, ldp, beta,
                    lc.ptr + lcol_of(C, j) * lc.ld, lc.ld);
    sync_ctx(c);
    internal::finish_origin(C, opts);
}

template <typename T>
void gemm(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts) {
    if (internal::spread<T>(opts, {{&C, true}, {&A, false}, {&B, false}}, [&](std::vector<Matrix<T>>& M, int) {
            gemm(alpha, M[1], M[2], beta, M[0], opts);
        }))
        return;
    if (A.arbitrary_layout() || B.arbitrary_layout() || C.arbitrary_layout()) {
        Matrix<T> Ab = bc_operand(A, opts), Bb = bc_operand(B, opts), Cb = block_cyclic(C, opts);
        gemm(alpha, Ab, Bb, beta, Cb, opts);
        slate::copy<T, T>(Cb, C, opts);
        return;
    }
    Method m = get_option<int64_t>(opts, Option::MethodGemm, MethodGemm::Auto);
    if (m == MethodGemm::Auto) m = MethodGemm::select_algo(A, B, opts);
    if (m == MethodGemm::GemmA) gemmA(alpha, A, B, beta, C, opts);
    else gemmC(alpha, A, B, beta, C, opts);
}

//------------------------------------------------------------------------------
// trsm: block sweeps over B's block rows (Left), reference
// src/work/work_trsm.cc:101-185 (forward) / :186+ (backward) and
// src/work/work_trsmA.cc.  op(A) = A^T / A^H is NOT materialized: the sweep
// runs on the transposed process grid, where A^T is A's own local array read
// with a transposed operand (zero copy) and B's rows follow A's COLUMN
// distribution; only B (m x nrhs) is redistributed when it does not conform.
// Right-side solves are reduced to Left by transposing B.
namespace {

/// Process column of B's grid holding op(A)'s panel k (and the diagonal
/// tile): A's column owner for NoTrans, its row owner for (conj-)transposes
/// (B's grid is then A's transposed grid).
template <typename T>
inline int panel_col(BaseMatrix<T> const& A, Op op, int64_t k) {
    return op == Op::NoTrans ? A.scol_owner(k) : A.srow_owner(k);
}
/// op(A)'s panel k for my local rows of B (mloc x kb, ld mloc): A(:, k) or
/// op(A(k, :)) packed from the local array
template <typename T>
inline void pack_op_panel(lb::Ctx const& c, BaseMatrix<T> const& A, LocalBlock<T> const& lA, Op op, int64_t k,
                          int64_t mloc, int64_t kb, T* W) {
    if (op == Op::NoTrans) pack(c, mloc, kb, lA.ptr + lcol_of(A, k) * lA.ld, lA.ld, W);
    else lb::copy<T, T>(c, Uplo::General, op, mloc, kb, lA.ptr + lrow_of(A, k), lA.ld, W, std::max<int64_t>(mloc, 1));
}

/// op(A) X = alpha B, A the PHYSICAL triangle (NoTrans storage view, uplo_phys),
/// B's rows conforming to op(A)'s rows (NoTrans: A's grid and row tiles;
/// otherwise A's transposed grid and column tiles).  trsmB sweep: per step
/// the diagonal tile along B's process row, op(A)'s panel along process rows,
/// the solved block row down process columns, one local GEMM per process.
template <typename T>
void trsm_left_sweep(Uplo uplo_phys, Op op, Diag diag, T alpha, BaseMatrix<T> const& A, Matrix<T>& B, Target target,
                     int64_t la) {
    auto& g = *B.grid();
    const int myrow = g.myrow(), mycol = g.mycol();
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
    // op(A) lower <=> forward sweep
    const bool lower = (op == Op::NoTrans) == (uplo_phys == Uplo::Lower);
    for (int64_t t = 0; t < mt; ++t) {
        const int64_t k = lower ? t : mt - 1 - t;
        const int slot = int(t % R);
        const int64_t kb = B.tileMb(k);
        const int pk = B.srow_owner(k), qk = panel_col(A, op, k);
        const int64_t lrk = lrow_of(B, k);
        T* D = WD[slot].data();
        T* WAk = WA[slot].data();
        T* WBk = WB[slot].data();
        // A(k,k) to every process of row pk; op(A)'s panel k (my rows) along rows
        S.task(device::kCommQueue, {}, {Sched::bcast(slot)}, [&, k, kb, pk, qk, D, WAk](lb::Ctx const& c) {
            trace::Block t2("trsm_bcast_panel");
            if (myrow == pk) {
                if (mycol == qk) pack(c, kb, kb, lA.ptr + lrow_of(A, k) + lcol_of(A, k) * lA.ld, lA.ld, D);
                bcast(g.row(), D, size_t(kb * kb), qk, c);
            }
            if (mycol == qk) pack_op_panel(c, A, lA, op, k, lbk.m, kb, WAk);
            bcast(g.row(), WAk, size_t(lbk.m * kb), qk, c);
        });
        // solve the block row on process row pk, then broadcast it down columns
        S.task(0, {Sched::bcast(slot)}, {Sched::tok(9, 0)}, [&, k, kb, pk, D, WBk, lrk](lb::Ctx const& c) {
            if (myrow == pk) {
                lb::trsm(c, Side::Left, uplo_phys, op, diag, kb, lbk.n, T(1), D, kb, lbk.ptr + lrk, lbk.ld);
                lb::copy2d(c, kb, lbk.n, lbk.ptr + lrk, lbk.ld, WBk, kb);
            }
        });
        S.task(device::kCommQueue, {Sched::tok(9, 0)}, {Sched::tok(8, slot)}, [&, kb, pk, WBk](lb::Ctx const& c) {
            trace::Block t2("trsm_bcast_x");
            bcast(g.col(), WBk, size_t(kb * lbk.n), pk, c);
        });
        // update the remaining block rows: B(i) -= op(A)(i,k) X(k)
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

/// X op(A) = alpha B (Side::Right), the column sweep mirroring
/// trsm_left_sweep, so a right-side solve never transposes B (the reference
/// turns Right into Left with shallow transpose views, work_trsm.cc:74-82;
/// here B's local array is used in place).  A is the PHYSICAL triangle whose
/// op(A) columns conform to B's columns: NoTrans -- A on B's grid, A's column
/// tiles = B's; otherwise A on B's transposed grid, A's ROW tiles = B's
/// column tiles (op(A)(k, j) = op(A(j, k)) then lives in A's local column k).
/// Per step: the diagonal tile down B's process column qk, the solve of B's
/// block column k there, X(:, k) along the process rows, op(A)'s block row k
/// (my local columns) down the process columns, one local GEMM.
///
/// same_grid (op(A) = A^T / A^H with A on B's OWN grid, A's row tiles = B's
/// column tiles): op(A)(k, j) = op(A(j, k)) for my columns j sits in other
/// process rows, so A's block column k (a panel, n x kb) goes along the
/// process rows from its owner and is all-gathered over the process column;
/// every process then packs op() of the tiles of its own columns.
///
/// solve = false runs trmm's B := alpha B op(A) with the same panels, in
/// place: op(A) upper -> block columns in descending order (B(:, k) is still
/// the original when its turn comes), lower -> ascending; per step the old
/// B(:, k) goes along the rows, the other columns accumulate B(:, k) op(A)(k, j)
/// and B(:, k) is multiplied by the diagonal triangle last.
template <typename T>
void tr_right_sweep(bool solve, Uplo uplo_phys, Op op, Diag diag, T alpha, BaseMatrix<T> const& A, Matrix<T>& B,
                    Target target, int64_t la, bool same_grid = false) {
    auto& g = *B.grid();
    const int myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    LocalBlock<T> lbk = B.local(loc, true);
    LocalBlock<T> lA = A.local(loc, false);
    const int64_t nt = B.nt(), mloc = lbk.m, nloc = lbk.n, ldx = std::max<int64_t>(mloc, 1);
    const int p = g.p();
    // same_grid: offset of tile i within its owner's local rows, and the
    // largest local row count (all-gather slab)
    std::vector<int64_t> rowoff(size_t(A.mt()), 0);
    int64_t maxr = 1;
    if (same_grid) {
        std::vector<int64_t> cnt(p, 0);
        for (int64_t i = 0; i < A.mt(); ++i) {
            rowoff[i] = cnt[A.srow_owner(i)];
            cnt[A.srow_owner(i)] += A.tileMb(i);
        }
        maxr = std::max<int64_t>(1, *std::max_element(cnt.begin(), cnt.end()));
    }
    Sched S(target);
    if (solve && alpha != T(1))
        S.task(0, {}, {Sched::tok(9, 0)}, [&](lb::Ctx const& c) {
            lb::add(c, Uplo::General, mloc, nloc, T(0), lbk.ptr, lbk.ld, alpha, lbk.ptr, lbk.ld);
        });
    const int R = int(std::max<int64_t>(2, la + 2));
    const int64_t nbmax = B.nb();
    std::vector<Work<T>> WA(R), WX(R), WD(R), WG(R);
    Work<T> Gs;
    for (int r = 0; r < R; ++r) {
        WA[r].resize(target, size_t(nbmax) * std::max<int64_t>(nloc, 1));
        WX[r].resize(target, size_t(ldx) * nbmax);
        WD[r].resize(target, size_t(nbmax) * nbmax);
        if (same_grid) WG[r].resize(target, size_t(p) * maxr * nbmax);
    }
    if (same_grid) Gs.resize(target, size_t(maxr) * nbmax);
    // op(A) upper <=> forward over B's block columns (solve), backward (multiply)
    const bool upper = (op == Op::NoTrans) == (uplo_phys == Uplo::Upper);
    const bool forward = solve ? upper : !upper;
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t k = forward ? t : nt - 1 - t;
        const int slot = int(t % R);
        const int64_t kb = B.tileNb(k);
        const int qk = B.scol_owner(k);
        const int pr = op == Op::NoTrans ? A.srow_owner(k) : A.scol_owner(k);   // B's process row holding op(A)(k, :)
        const int64_t lck = lcol_of(B, k);
        T* D = WD[slot].data();
        T* WAk = WA[slot].data();
        T* WXk = WX[slot].data();
        // op(A)(k, k) down process column qk; op(A)'s block row k (my local
        // columns, kb x nloc) down every process column from row pr
        if (same_grid) {
            T* G = WG[slot].data();
            const int qa = A.scol_owner(k);
            S.task(device::kCommQueue, {}, {Sched::bcast(slot)}, [&, k, kb, qa, D, WAk, G](lb::Ctx const& c) {
                trace::Block t2("trsm_bcast_panel");
                if (mycol == qa) lb::copy2d(c, lA.m, kb, lA.ptr + lcol_of(A, k) * lA.ld, lA.ld, Gs.data(), maxr);
                bcast(g.row(), Gs.data(), size_t(maxr * kb), qa, c);
                g.col().allgather(Gs.data(), G, size_t(maxr * kb), scalar_type<T>(), c.loc(), c.stream);
                // op() of the tiles of my columns -> W (kb x nloc), and op(A)(k, k)
                for (int64_t j = 0; j < nt; ++j) {
                    if (B.scol_owner(j) != mycol) continue;
                    const T* src = G + size_t(A.srow_owner(j)) * maxr * kb + rowoff[j];
                    lb::copy<T, T>(c, Uplo::General, op, kb, B.tileNb(j), src, maxr, WAk + lcol_of(B, j) * kb, kb);
                }
                lb::copy<T, T>(c, Uplo::General, op, kb, kb, G + size_t(A.srow_owner(k)) * maxr * kb + rowoff[k], maxr,
                               D, kb);
            });
        } else
        S.task(device::kCommQueue, {}, {Sched::bcast(slot)}, [&, k, kb, qk, pr, D, WAk](lb::Ctx const& c) {
            trace::Block t2("trsm_bcast_panel");
            const int64_t lrA = op == Op::NoTrans ? lrow_of(A, k) : 0, lcA = op == Op::NoTrans ? 0 : lcol_of(A, k);
            if (myrow == pr) {
                if (op == Op::NoTrans) lb::copy2d(c, kb, nloc, lA.ptr + lrA, lA.ld, WAk, kb);
                else lb::copy<T, T>(c, Uplo::General, op, kb, nloc, lA.ptr + lcA * lA.ld, lA.ld, WAk, kb);
                if (mycol == qk) lb::copy2d(c, kb, kb, WAk + lck * kb, kb, D, kb);   // op(A)(k, k)
            }
            bcast(g.col(), WAk, size_t(kb * nloc), pr, c);
            if (mycol == qk) bcast(g.col(), D, size_t(kb * kb), pr, c);
        });
        if (!solve) {
            // multiply: the ORIGINAL B(:, k) along the rows, the other columns
            // accumulate it, B(:, k) times the diagonal triangle last
            S.task(device::kCommQueue, {Sched::tok(9, 0)}, {Sched::tok(8, slot)}, [&, kb, qk, WXk, lck](lb::Ctx const& c) {
                trace::Block t2("trmm_bcast_b");
                if (mycol == qk) lb::copy2d(c, mloc, kb, lbk.ptr + lck * lbk.ld, lbk.ld, WXk, ldx);
                bcast(g.row(), WXk, size_t(ldx * kb), qk, c);
            });
            S.task(0, {Sched::tok(8, slot), Sched::bcast(slot)}, {Sched::tok(9, 0)},
                   [&, k, kb, qk, D, WAk, WXk, lck](lb::Ctx const& c) {
                trace::Block t2("trmm_update");
                const int64_t c0 = upper ? lcol_of(B, k + 1) : 0;
                const int64_t c1 = upper ? nloc : lcol_of(B, k);
                if (c1 > c0 && mloc > 0)
                    lb::gemm(c, Op::NoTrans, Op::NoTrans, mloc, c1 - c0, kb, T(1), WXk, ldx, WAk + c0 * kb, kb, T(1),
                             lbk.ptr + c0 * lbk.ld, lbk.ld);
                if (mycol == qk && mloc > 0)
                    lb::trmm(c, Side::Right, upper ? Uplo::Upper : Uplo::Lower, Op::NoTrans, diag, mloc, kb, T(1), D, kb,
                             lbk.ptr + lck * lbk.ld, lbk.ld);
            });
            continue;
        }
        // solve B(:, k) on process column qk, then X(:, k) along the rows
        S.task(0, {Sched::bcast(slot)}, {Sched::tok(9, 0)}, [&, kb, qk, D, WXk, lck](lb::Ctx const& c) {
            if (mycol == qk && mloc > 0) {
                // D holds op(A)(k, k) explicitly: solve against it as NoTrans
                // with op(A)'s triangle (upper iff forward)
                lb::trsm(c, Side::Right, upper ? Uplo::Upper : Uplo::Lower, Op::NoTrans, diag, mloc, kb, T(1), D, kb,
                         lbk.ptr + lck * lbk.ld, lbk.ld);
                lb::copy2d(c, mloc, kb, lbk.ptr + lck * lbk.ld, lbk.ld, WXk, ldx);
            }
        });
        S.task(device::kCommQueue, {Sched::tok(9, 0)}, {Sched::tok(8, slot)}, [&, kb, qk, WXk](lb::Ctx const& c) {
            trace::Block t2("trsm_bcast_x");
            bcast(g.row(), WXk, size_t(ldx * kb), qk, c);
        });
        // B(:, j) -= X(:, k) op(A)(k, j) for the block columns still to solve
        S.task(0, {Sched::tok(8, slot), Sched::bcast(slot)}, {Sched::tok(9, 0)}, [&, k, kb, WAk, WXk](lb::Ctx const& c) {
            const int64_t c0 = upper ? lcol_of(B, k + 1) : 0;
            const int64_t c1 = upper ? nloc : lcol_of(B, k);
            if (c1 > c0 && mloc > 0)
                lb::gemm(c, Op::NoTrans, Op::NoTrans, mloc, c1 - c0, kb, T(-1), WXk, ldx, WAk + c0 * kb, kb, T(1),
                         lbk.ptr + c0 * lbk.ld, lbk.ld);
        });
    }
    if (!solve && alpha != T(1))
        S.task(0, {}, {Sched::tok(9, 0)}, [&](lb::Ctx const& c) {
            lb::add(c, Uplo::General, mloc, nloc, T(0), lbk.ptr, lbk.ld, alpha, lbk.ptr, lbk.ld);
        });
    S.wait_all();
}

/// Do op(A)'s columns line up with B's columns (tr_right_sweep's layout)?
template <typename T>
bool b_conforms_right(BaseMatrix<T> const& Ap, Op op, BaseMatrix<T> const& B) {
    if (B.op() != Op::NoTrans || !B.aligned()) return false;
    auto& ga = *Ap.grid();
    auto& gb = *B.grid();
    if (!ga.same_processes(gb) || Ap.mb() != Ap.nb()) return false;
    if (op == Op::NoTrans) {
        if (!cols_conform(Ap, B)) return false;
        for (int64_t j = 0; j < Ap.nt(); ++j) if (Ap.tileMb(j) != B.tileNb(j)) return false;
        return true;
    }
    // A on B's transposed grid: A's process (r, c) is B's process (c, r)
    if (gb.p() != ga.q() || gb.q() != ga.p() || (gb.size() > 1 && gb.order() == ga.order())) return false;
    if (B.nt() != Ap.mt()) return false;
    for (int64_t j = 0; j < Ap.mt(); ++j)
        if (Ap.tileMb(j) != B.tileNb(j) || Ap.srow_owner(j) != B.scol_owner(j) || Ap.tileMb(j) != Ap.tileNb(j))
            return false;
    return true;
}

/// Stationary-A triangular solve for narrow B (reference src/work/work_trsmA.cc):
/// A never moves.  Each process keeps a partial-sum block W (its local rows x
/// all columns of B); step k sums block row k of W across process row pk,
/// the owner of A(k,k) solves it, broadcasts X(k) down its process column, and
/// that column updates W(i) -= op(A)(i,k) X(k) for its local rows.  Traffic per
/// step is kb x n, instead of trsmB's A panel of (local rows) x kb.  For
/// op(A) = A^T / A^H the same algorithm runs on the transposed grid (B's
/// rows follow A's columns) and the update reads op(A(k, i)) straight from
/// the local array.
///
/// Lookahead 1: step k's update is split into the NEXT block row (k +- 1,
/// panel queue, right after the broadcast) and the REST (trailing queue), so
/// the reduce / solve / broadcast of step k+1 -- the latency chain -- runs
/// while the rest of step k's update is still computing; the REST of step k
/// only has to finish before step k+2's reduce.
template <typename T>
void trsmA_left(Uplo uplo_phys, Op op, Diag diag, T alpha, BaseMatrix<T> const& A, Matrix<T>& B, Target target) {
    auto& g = *B.grid();
    const int myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    LocalBlock<T> lbk = B.local(loc, true);
    LocalBlock<T> lA = A.local(loc, false);
    const int64_t mt = B.mt(), n = B.n(), mloc = lbk.m, ldw = std::max<int64_t>(mloc, 1);
    Sched S(target);
    Work<T> W(target, size_t(ldw) * std::max<int64_t>(n, 1)), X(target, size_t(ldw) * std::max<int64_t>(n, 1));
    Work<T> WX[2];
    for (auto& w : WX) w.resize(target, size_t(B.mb()) * std::max<int64_t>(n, 1));
    constexpr int qP = 1, qT = 0;
    // tokens: tI init; tS(k%2) step k's solved X(k) in WX; tN next-row update
    // done; tR(k%2) step k's rest update done
    const int64_t tI = Sched::tok(9, 0), tN = Sched::tok(9, 1);
    auto tS = [](int64_t k) { return Sched::tok(8, k & 1); };
    auto tR = [](int64_t k) { return Sched::tok(7, k & 1); };
    // W = alpha B at B's global columns (zero elsewhere), X = 0
    S.task(qT, {}, {tI, tN, tR(-1), tR(-2)}, [&](lb::Ctx const& c) {
        lb::set(c, Uplo::General, mloc, n, T(0), T(0), W.data(), ldw);
        lb::set(c, Uplo::General, mloc, n, T(0), T(0), X.data(), ldw);
        for (int64_t j = 0; j < B.nt(); ++j)
            if (B.scol_owner(j) == mycol)
                lb::add(c, Uplo::General, mloc, B.tileNb(j), alpha, lbk.ptr + lcol_of(B, j) * lbk.ld, lbk.ld, T(1),
                        W.data() + gcol_of(B, j) * ldw, ldw);
    });
    const bool lower = (op == Op::NoTrans) == (uplo_phys == Uplo::Lower);
    // W(rows [r0, r1)) -= op(A)(rows, k) X(k)
    auto update = [&, op, lower](lb::Ctx const& c, int64_t k, int64_t kb, T const* Xk, int64_t r0, int64_t r1) {
        if (r1 <= r0) return;
        if (op == Op::NoTrans)
            lb::gemm(c, Op::NoTrans, Op::NoTrans, r1 - r0, n, kb, T(-1), lA.ptr + r0 + lcol_of(A, k) * lA.ld, lA.ld,
                     Xk, kb, T(1), W.data() + r0, ldw);
        else   // op(A(k, cols r0..r1)): my local columns of A = my local rows of B
            lb::gemm(c, op, Op::NoTrans, r1 - r0, n, kb, T(-1), lA.ptr + lrow_of(A, k) + r0 * lA.ld, lA.ld, Xk, kb,
                     T(1), W.data() + r0, ldw);
    };
    for (int64_t t = 0; t < mt; ++t) {
        const int64_t k = lower ? t : mt - 1 - t;
        const int64_t kb = B.tileMb(k);
        const int pk = B.srow_owner(k), qk = panel_col(A, op, k);
        const int64_t lrk = lrow_of(B, k);
        T* WXk = WX[t & 1].data();
        // reduce: block row k of W is final after step t-1's next-row update
        // and step t-2's rest (earlier rests are ordered before it)
        S.task(device::kCommQueue, {tI, tN, tR(t - 2)}, {tS(t)}, [&, kb, pk, lrk, WXk](lb::Ctx const& c) {
            trace::Block t2("trsmA_reduce");
            if (myrow != pk) return;
            pack(c, kb, n, W.data() + lrk, ldw, WXk);
            allreduce_sum(g.row(), WXk, size_t(kb) * n, c);
        });
        S.task(qP, {tS(t)}, {tS(t)}, [&, k, kb, pk, qk, lrk, WXk](lb::Ctx const& c) {
            if (myrow != pk || mycol != qk) return;
            lb::trsm(c, Side::Left, uplo_phys, op, diag, kb, n, T(1),
                     lA.ptr + lrow_of(A, k) + lcol_of(A, k) * lA.ld, lA.ld, WXk, kb);
            lb::copy2d(c, kb, n, WXk, kb, X.data() + lrk, ldw);
        });
        S.task(device::kCommQueue, {tS(t)}, {tS(t)}, [&, kb, pk, qk, WXk](lb::Ctx const& c) {
            trace::Block t2("trsmA_bcast");
            if (mycol == qk) bcast(g.col(), WXk, size_t(kb) * n, pk, c);
        });
        // my local rows of the next block row to solve, and the rest
        int64_t n0 = 0, n1 = 0;
        if (t + 1 < mt) {
            const int64_t kn = lower ? k + 1 : k - 1;
            if (B.srow_owner(kn) == myrow) { n0 = lrow_of(B, kn); n1 = n0 + B.tileMb(kn); }
        }
        const int64_t r0 = lower ? lrow_of(B, k + 1) : 0, r1 = lower ? mloc : lrk;
        // next row: needs X(k) and step t-1's rest (it also writes these rows)
        S.task(qP, {tS(t), tR(t - 1)}, {tN}, [&, k, kb, qk, WXk, n0, n1](lb::Ctx const& c) {
            if (mycol != qk) return;
            update(c, k, kb, WXk, n0, n1);
        });
        S.task(qT, {tS(t), tR(t - 1)}, {tR(t)}, [&, k, kb, qk, WXk, n0, n1, r0, r1](lb::Ctx const& c) {
            if (mycol != qk) return;
            if (n1 > n0) {
                update(c, k, kb, WXk, r0, std::min(r1, n0));
                update(c, k, kb, WXk, std::max(r0, n1), r1);
            } else {
                update(c, k, kb, WXk, r0, r1);
            }
        });
    }
    // X(k) sits on process column qk of block row k: sum across the process
    // row, then each process keeps its own columns of B
    S.task(device::kCommQueue, {tN, tR(mt - 1), tR(mt - 2), tS(mt - 1)}, {tI}, [&](lb::Ctx const& c) {
        allreduce_sum(g.row(), X.data(), size_t(ldw) * n, c);
    });
    S.task(qT, {tI}, {tI}, [&](lb::Ctx const& c) {
        for (int64_t j = 0; j < B.nt(); ++j)
            if (B.scol_owner(j) == mycol)
                lb::copy2d(c, mloc, B.tileNb(j), X.data() + gcol_of(B, j) * ldw, ldw,
                           lbk.ptr + lcol_of(B, j) * lbk.ld, lbk.ld);
    });
    S.wait_all();
}

/// Do B's row tiles follow op(A)'s rows (NoTrans: A's rows on A's grid;
/// otherwise A's columns on A's transposed grid)?
template <typename T>
bool b_conforms(BaseMatrix<T> const& Ap, Op op, BaseMatrix<T> const& B) {
    if (B.op() != Op::NoTrans || !B.aligned()) return false;
    auto& ga = *Ap.grid();
    auto& gb = *B.grid();
    if (!ga.same_processes(gb)) return false;
    if (op == Op::NoTrans) {
        if (!rows_conform(Ap, B)) return false;
        for (int64_t j = 0; j < Ap.nt(); ++j) if (Ap.tileNb(j) != B.tileMb(j)) return false;
        return true;
    }
    // B on the transposed grid: B's process (r, c) is A's process (c, r)
    // (swapped dimensions + opposite order: rank_of_B(r, c) == rank_of_A(c, r))
    if (gb.p() != ga.q() || gb.q() != ga.p() || (gb.size() > 1 && gb.order() == ga.order())) return false;
    if (B.mt() != Ap.nt()) return false;
    for (int64_t i = 0; i < Ap.nt(); ++i)
        if (Ap.tileNb(i) != B.tileMb(i) || Ap.scol_owner(i) != B.srow_owner(i) || Ap.tileMb(i) != Ap.tileNb(i))
            return false;
    return true;
}

}  // namespace

template <typename T>
void trsm(Side side, T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    if (internal::spread<T>(opts, {{&A, false}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int) {
            auto Ar = internal::rewrap(A, M[0]);
            trsm(side, alpha, Ar, M[1], opts);
        }, false))
        return;
    if (A.arbitrary_layout() || B.arbitrary_layout()) {
        TriangularMatrix<T> Ab(A.uplo(), A.diag(), bc_operand(A, opts));
        Matrix<T> Bb = block_cyclic(B, opts);
        trsm(side, alpha, Ab, Bb, opts);
        slate::copy<T, T>(Bb, B, opts);
        return;
    }
    trace::Block tb("trsm");
    internal::DriverScope ds_;
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
        internal::finish_origin(B, opts);
        return;
    }
    // MethodTrsm (reference include/slate/method.hh:35-45): stationary A for a
    // single block column of right-hand sides, else the trsmB sweep
    Method method = get_option<int64_t>(opts, Option::MethodTrsm, MethodTrsm::Auto);
    // (narrow = one block column of right-hand sides: B's columns for Left,
    // its rows for Right)
    if (method == MethodTrsm::Auto)
        method = (side == Side::Left ? B.nt() : B.mt()) < 2 ? MethodTrsm::TrsmA : MethodTrsm::TrsmB;
    slate_error_if_msg(method != MethodTrsm::TrsmA && method != MethodTrsm::TrsmB, "trsm: unknown MethodTrsm");
    // Right side: the column sweep on B in place when op(A)'s columns conform
    // to B's (the usual case: same tiles, A on B's grid or, for op(A) =
    // A^T / A^H, on its transposed grid); else reduced to Left below
    if (side == Side::Right && method == MethodTrsm::TrsmB) {
        const Op op = A.op();
        BaseMatrix<T> Ap = op == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(op == Op::ConjTrans);
        if (Ap.aligned() && b_conforms_right(Ap, op, B)) {
            tr_right_sweep(true, A.uplo_physical(), op, A.diag(), alpha, Ap, B, target, option_la(opts));
            internal::finish_origin(B, opts);
            return;
        }
        if (op != Op::NoTrans && Ap.aligned() && b_conforms_right(Ap, Op::NoTrans, B)) {
            // op(A) = A^T / A^H with A on B's own grid: column panels gathered
            tr_right_sweep(true, A.uplo_physical(), op, A.diag(), alpha, Ap, B, target, option_la(opts), true);
            internal::finish_origin(B, opts);
            return;
        }
    }
    // distributed: reduce to Left
    if (side == Side::Right) {
        // X op(A) = alpha B  <=>  op(A)^T X^T = alpha B^T (use conj for ConjTrans pairs)
        bool conj = is_complex_v<T>;
        Matrix<T> Bt = materialize<T>(conj ? conj_transpose(B) : transpose(B), target, gB, B.nb(), B.mb(),
                                      0, 0);
        TriangularMatrix<T> Ah = conj ? conj_transpose(A) : transpose(A);
        TriangularMatrix<T> At(Ah.uplo(), A.diag(), Ah);
        Options o2 = opts;
        o2[Option::MethodTrsm] = method;
        trsm(Side::Left, conj ? slate::conj(alpha) : alpha, At, Bt, o2);
        slate::copy<T, T>(conj ? conj_transpose(Bt) : transpose(Bt), B, opts);
        return;
    }
    // A's physical triangle (no copy); op(A) is handled by the sweeps
    const Op op = A.op();
    BaseMatrix<T> Ap = op == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(op == Op::ConjTrans);
    const Uplo up = A.uplo_physical();
    Matrix<T> Ac;
    if (!Ap.aligned() || Ap.mb() != Ap.nb()) {
        // unaligned sub-view of A: square-tile aligned copy (the only case
        // that still copies A)
        Ac = materialize<T>(Ap, target, Ap.grid(), B.mb(), B.mb(), 0, 0);
        Ap = Ac;
    }
    auto run = [&](Matrix<T>& Bx) {
        if (method == MethodTrsm::TrsmA) trsmA_left(up, op, A.diag(), alpha, Ap, Bx, target);
        else trsm_left_sweep(up, op, A.diag(), alpha, Ap, Bx, target, option_la(opts));
    };
    if (b_conforms(Ap, op, B)) {
        run(B);
        internal::finish_origin(B, opts);
        return;
    }
    // redistribute B (m x nrhs) to follow op(A)'s rows, never A
    GridPtr gx = op == Op::NoTrans ? Ap.grid() : Ap.grid()->transposed();
    const int rsrc = op == Op::NoTrans ? row0_owner(Ap) : col0_owner(Ap);
    Matrix<T> Bx = materialize<T>(B, target, gx, Ap.nb(), B.nb(), rsrc, 0);
    run(Bx);
    slate::copy<T, T>(Bx, B, opts);
}

//------------------------------------------------------------------------------
// herk / syrk / her2k / syr2k / hemm / symm / trmm
namespace {

template <typename T>
bool local_only(BaseMatrix<T> const& A) { return A.grid()->size() == 1; }


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
    internal::finish_origin(C, opts);
}

}  // namespace

template <typename T>
void herk(real_type<T> alpha, Matrix<T> const& A, real_type<T> beta, HermitianMatrix<T>& C, Options const& opts) {
    if (internal::spread<T>(opts, {{&A, false}, {&C, true}}, [&](std::vector<Matrix<T>>& M, int) {
            auto Cr = internal::rewrap(C, M[1]);
            herk(alpha, M[0], beta, Cr, opts);
        }, false))
        return;
    trace::Block tb("herk");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && C.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lc = C.local(loc, true);
        Op op = A.op() == Op::NoTrans ? Op::NoTrans : Op::ConjTrans;
        lb::herk(c, C.uplo(), op, lc.m, A.n(), alpha, la_.ptr, la_.ld, beta, lc.ptr, lc.ld);
        sync_ctx(c);
        internal::finish_origin(C, opts);
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
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && C.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lc = C.local(loc, true);
        Op op = A.op() == Op::NoTrans ? Op::NoTrans : Op::Trans;
        lb::syrk(c, C.uplo(), op, lc.m, A.n(), alpha, la_.ptr, la_.ld, beta, lc.ptr, lc.ld);
        sync_ctx(c);
        internal::finish_origin(C, opts);
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
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && local_only(B) && C.op() == Op::NoTrans && A.op() == B.op()) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
        Op op = A.op() == Op::NoTrans ? Op::NoTrans : Op::ConjTrans;
        lb::her2k(c, C.uplo(), op, lc.m, A.n(), alpha, la_.ptr, la_.ld, lbk.ptr, lbk.ld, beta, lc.ptr, lc.ld);
        sync_ctx(c);
        internal::finish_origin(C, opts);
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
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && local_only(B) && C.op() == Op::NoTrans && A.op() == B.op()) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
        Op op = A.op() == Op::NoTrans ? Op::NoTrans : Op::Trans;
        lb::syr2k(c, C.uplo(), op, lc.m, A.n(), alpha, la_.ptr, la_.ld, lbk.ptr, lbk.ld, beta, lc.ptr, lc.ld);
        sync_ctx(c);
        internal::finish_origin(C, opts);
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

/// C = beta C, with beta = 0 overwriting (NaN-safe)
template <typename T>
inline void scale_c(lb::Ctx const& c, T beta, int64_t m, int64_t n, T* C, int64_t ldc) {
    if (beta == T(0)) lb::set(c, Uplo::General, m, n, T(0), T(0), C, ldc);
    else if (beta != T(1)) lb::add(c, Uplo::General, m, n, T(0), C, ldc, beta, C, ldc);
}

/// hemmC / symmC, Left (reference src/hemmC.cc): SUMMA over the STORED
/// triangle only.  With A = L + L_s^H (Lower; Upper mirrors it), step k
/// broadcasts the stored part of column k along process rows and B(k,:) down
/// process columns, then
///   C(i,:) += A(i,k) B(k,:)           rows strictly inside the triangle,
///   C(k,:) += hemm(A(k,k)) B(k,:)     diagonal tile,
///   C(k,:) += sum_j A(j,k)^H B(j,:)   partial products on every process,
///                                     summed over the process column.
/// No n x n temporary and no transposed copy of A.  A: rows conform to C,
/// column tiles = C's row tiles; B conforms to C.
template <typename T>
void hemmC_left(Uplo uplo, bool herm, T alpha, BaseMatrix<T> const& A, BaseMatrix<T> const& B, T beta,
                Matrix<T>& C, Target target, int64_t la) {
    auto& g = *C.grid();
    const int myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    LocalBlock<T> lc = C.local(loc, true), lB = B.local(loc, false), lA = A.local(loc, false);
    const int64_t kt = A.nt(), nloc = lc.n, mloc = lc.m, nb = C.mb();
    const bool lower = (uplo == Uplo::Lower);
    const Op opH = herm ? Op::ConjTrans : Op::Trans;
    Sched S(target);
    const int64_t tC = Sched::tok(9, 0);
    S.task(0, {}, {tC}, [&](lb::Ctx const& c) { scale_c(c, beta, mloc, nloc, lc.ptr, lc.ld); });
    const int R = int(std::max<int64_t>(2, la + 2));
    std::vector<Work<T>> WA(R), WB(R), WP(R);
    for (int r = 0; r < R; ++r) {
        WA[r].resize(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
        WB[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
        WP[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
    }
    for (int64_t k = 0; k < kt; ++k) {
        const int slot = int(k % R);
        const int64_t kb = A.tileNb(k);
        const int qk = A.scol_owner(k), pk = C.srow_owner(k);
        const int64_t rk = lrow_of(C, k), rk1 = lrow_of(C, k + 1);
        const int64_t lo = lower ? rk : 0, hi = lower ? mloc : rk1;   // stored rows of column k
        const int64_t rs = lower ? rk1 : 0, re = lower ? mloc : rk;   // strictly off-diagonal rows
        const int64_t nr = hi - lo, ldw = std::max<int64_t>(nr, 1);
        T* WAk = WA[slot].data();
        T* WBk = WB[slot].data();
        T* WPk = WP[slot].data();
        const int64_t tBc = Sched::bcast(slot), tP = Sched::tok(7, slot);
        S.task(device::kCommQueue, {}, {tBc}, [&, k, kb, qk, pk, rk, lo, nr, WAk, WBk](lb::Ctx const& c) {
            trace::Block t2("hemm_bcast");
            if (nr > 0) {
                if (mycol == qk) pack(c, nr, kb, lA.ptr + lo + lcol_of(A, k) * lA.ld, lA.ld, WAk);
                bcast(g.row(), WAk, size_t(nr * kb), qk, c);
            }
            if (nloc > 0) {
                if (myrow == pk) lb::copy2d(c, kb, nloc, lB.ptr + rk, lB.ld, WBk, kb);
                bcast(g.col(), WBk, size_t(kb * nloc), pk, c);
            }
        });
        S.task(0, {tBc}, {tC, tP}, [&, kb, pk, rk, lo, rs, re, ldw, WAk, WBk, WPk](lb::Ctx const& c) {
            trace::Block t2("hemm_update");
            if (nloc == 0) return;
            if (myrow == pk)
                lb::hemm(c, Side::Left, uplo, kb, nloc, alpha, WAk + (rk - lo), ldw, WBk, kb, T(1), lc.ptr + rk, lc.ld,
                         herm);
            if (re > rs) {
                lb::gemm(c, Op::NoTrans, Op::NoTrans, re - rs, nloc, kb, alpha, WAk + (rs - lo), ldw, WBk, kb, T(1),
                         lc.ptr + rs, lc.ld);
                lb::gemm(c, opH, Op::NoTrans, kb, nloc, re - rs, T(1), WAk + (rs - lo), ldw, lB.ptr + rs, lB.ld, T(0),
                         WPk, kb);
            } else {
                lb::set(c, Uplo::General, kb, nloc, T(0), T(0), WPk, kb);
            }
        });
        S.task(device::kCommQueue, {tP}, {tP}, [&, kb, WPk](lb::Ctx const& c) {
            trace::Block t2("hemm_reduce");
            allreduce_sum(g.col(), WPk, size_t(kb * nloc), c);
        });
        S.task(0, {tP}, {tC}, [&, kb, pk, rk, WPk](lb::Ctx const& c) {
            if (myrow == pk && nloc > 0) lb::add(c, Uplo::General, kb, nloc, alpha, WPk, kb, T(1), lc.ptr + rk, lc.ld);
        });
    }
    S.wait_all();
}

/// hemm / symm, Right, in place on C (no transposed copies of B and C):
/// C = alpha B A + beta C as a SUMMA over A's block rows.  Row k of the
/// Hermitian A is assembled from what is stored: the stored part of block row
/// k (process row pk, down the process columns) and, mirrored, the stored
/// part of block column k (gathered: along the rows from its owner, then
/// all-gathered over the column), op = ^H (herm) or ^T (symm); the diagonal
/// tile is expanded from its stored triangle.  B(:, k) goes along the rows and
/// every process adds B(:, k) A(k, my columns) to its C in one GEMM.
/// Needs A on C's grid with A's tiles = C's column tiles, B's rows = C's rows
/// and B's column tiles = A's tiles.
template <typename T>
void hemmC_right(Uplo uplo, bool herm, T alpha, BaseMatrix<T> const& A, BaseMatrix<T> const& B, T beta,
                 Matrix<T>& C, Target target, int64_t la) {
    auto& g = *C.grid();
    const int p = g.p(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    LocalBlock<T> lc = C.local(loc, true), lB = B.local(loc, false), lA = A.local(loc, false);
    const int64_t kt = A.nt(), nloc = lc.n, mloc = lc.m, nb = A.nb(), ldx = std::max<int64_t>(mloc, 1);
    const bool lower = (uplo == Uplo::Lower);
    const Op opH = herm ? Op::ConjTrans : Op::Trans;
    std::vector<int64_t> rowoff(size_t(A.mt()), 0);
    std::vector<int64_t> cnt(p, 0);
    for (int64_t i = 0; i < A.mt(); ++i) {
        rowoff[i] = cnt[A.srow_owner(i)];
        cnt[A.srow_owner(i)] += A.tileMb(i);
    }
    const int64_t maxr = std::max<int64_t>(1, *std::max_element(cnt.begin(), cnt.end()));
    Sched S(target);
    const int64_t tC = Sched::tok(9, 0);
    S.task(0, {}, {tC}, [&](lb::Ctx const& c) { scale_c(c, beta, mloc, nloc, lc.ptr, lc.ld); });
    const int R = int(std::max<int64_t>(2, la + 2));
    std::vector<Work<T>> WA(R), WX(R), WR(R), WG(R);
    Work<T> Gs(target, size_t(maxr) * nb);
    for (int r = 0; r < R; ++r) {
        WA[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
        WR[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
        WX[r].resize(target, size_t(ldx) * nb);
        WG[r].resize(target, size_t(p) * maxr * nb);
    }
    for (int64_t k = 0; k < kt; ++k) {
        const int slot = int(k % R);
        const int64_t kb = A.tileNb(k);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k), qb = B.scol_owner(k);
        T* WAk = WA[slot].data();
        T* WXk = WX[slot].data();
        T* WRk = WR[slot].data();
        T* G = WG[slot].data();
        S.task(device::kCommQueue, {}, {Sched::bcast(slot)}, [&, k, kb, pk, qk, qb, WAk, WXk, WRk, G](lb::Ctx const& c) {
            trace::Block t2("hemm_bcast");
            // block column k (all rows) everywhere, block row k down the columns
            if (mycol == qk) lb::copy2d(c, lA.m, kb, lA.ptr + lcol_of(A, k) * lA.ld, lA.ld, Gs.data(), maxr);
            bcast(g.row(), Gs.data(), size_t(maxr * kb), qk, c);
            g.col().allgather(Gs.data(), G, size_t(maxr * kb), scalar_type<T>(), c.loc(), c.stream);
            if (nloc > 0) {
                if (myrow == pk) lb::copy2d(c, kb, nloc, lA.ptr + lrow_of(A, k), lA.ld, WRk, kb);
                bcast(g.col(), WRk, size_t(kb * nloc), pk, c);
            }
            if (mloc > 0) {
                if (mycol == qb) lb::copy2d(c, mloc, kb, lB.ptr + lcol_of(B, k) * lB.ld, lB.ld, WXk, ldx);
                bcast(g.row(), WXk, size_t(ldx * kb), qb, c);
            }
            // A(k, j) for my column tiles j: stored in row k (j on the stored
            // side), mirrored from column k (other side), expanded diagonal
            for (int64_t j = 0; j < C.nt(); ++j) {
                if (C.scol_owner(j) != mycol) continue;
                const int64_t nbj = C.tileNb(j), cj = lcol_of(C, j);
                T const* Gj = G + size_t(A.srow_owner(j)) * maxr * kb + rowoff[j];
                T* Wj = WAk + cj * kb;
                if (j == k) {
                    lb::copy<T, T>(c, uplo, Op::NoTrans, kb, kb, Gj, maxr, Wj, kb);
                    lb::copy<T, T>(c, lower ? Uplo::Upper : Uplo::Lower, opH, kb, kb, Gj, maxr, Wj, kb);
                } else if (lower ? j < k : j > k) {
                    lb::copy2d(c, kb, nbj, WRk + cj * kb, kb, Wj, kb);
                } else {
                    lb::copy<T, T>(c, Uplo::General, opH, kb, nbj, Gj, maxr, Wj, kb);
                }
            }
        });
        S.task(0, {Sched::bcast(slot)}, {tC}, [&, kb, WAk, WXk](lb::Ctx const& c) {
            trace::Block t2("hemm_update");
            if (mloc > 0 && nloc > 0)
                lb::gemm(c, Op::NoTrans, Op::NoTrans, mloc, nloc, kb, alpha, WXk, ldx, WAk, kb, T(1), lc.ptr, lc.ld);
        });
    }
    S.wait_all();
}

/// hemmA / symmA, Left (reference src/hemmA.cc): A stays where it is.  B
/// (narrow) is replicated on the device; every process multiplies its stored
/// tiles by the matching rows of B, both as A(i,j) B(j,:) into row i and as
/// A(i,j)^H B(i,:) into row j, and one world allreduce sums the partial rows.
/// C, B: any distribution (NoTrans); A: aligned, square diagonal tiles.
template <typename T>
void hemmA_left(Uplo uplo, bool herm, T alpha, BaseMatrix<T> const& A, BaseMatrix<T> const& B, T beta,
                Matrix<T>& C, Target target) {
    auto& g = *C.grid();
    const int myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    lb::Ctx c = ctx_for(target);
    LocalBlock<T> lA = A.local(loc, false), lc = C.local(loc, true);
    const int64_t n = C.m(), nrhs = C.n(), mloc = lA.m, nloc = lA.n;
    const int64_t ldg = std::max<int64_t>(n, 1), ldr = std::max<int64_t>(mloc, 1), ldq = std::max<int64_t>(nloc, 1);
    const size_t w = size_t(std::max<int64_t>(nrhs, 1));
    const bool lower = (uplo == Uplo::Lower);
    const Op opH = herm ? Op::ConjTrans : Op::Trans;
    Work<T> G(target, ldg * w), Br(target, ldr * w), Wr(target, ldr * w), Bq(target, ldq * w), Wq(target, ldq * w);
    replicate(c, B, G.data());
    gather_local(c, A, false, G.data(), ldg, nrhs, Br.data(), ldr, false);
    gather_local(c, A, true, G.data(), ldg, nrhs, Bq.data(), ldq, false);
    lb::set(c, Uplo::General, mloc, nrhs, T(0), T(0), Wr.data(), ldr);
    lb::set(c, Uplo::General, nloc, nrhs, T(0), T(0), Wq.data(), ldq);
    for (int64_t j = 0; j < A.nt(); ++j) {
        if (A.scol_owner(j) != mycol) continue;
        const int64_t cj = lcol_of(A, j), nbj = A.tileNb(j), rj = lrow_of(A, j), rj1 = lrow_of(A, j + 1);
        T const* Aj = lA.ptr + cj * lA.ld;
        if (A.srow_owner(j) == myrow)
            lb::hemm(c, Side::Left, uplo, nbj, nrhs, T(1), Aj + rj, lA.ld, Bq.data() + cj, ldq, T(1),
                     Wr.data() + rj, ldr, herm);
        const int64_t rs = lower ? rj1 : 0, re = lower ? mloc : rj;
        if (re > rs) {
            lb::gemm(c, Op::NoTrans, Op::NoTrans, re - rs, nrhs, nbj, T(1), Aj + rs, lA.ld, Bq.data() + cj, ldq, T(1),
                     Wr.data() + rs, ldr);
            lb::gemm(c, opH, Op::NoTrans, nbj, nrhs, re - rs, T(1), Aj + rs, lA.ld, Br.data() + rs, ldr, T(1),
                     Wq.data() + cj, ldq);
        }
    }
    lb::set(c, Uplo::General, n, nrhs, T(0), T(0), G.data(), ldg);
    gather_local(c, A, false, G.data(), ldg, nrhs, Wr.data(), ldr, true);
    gather_local(c, A, true, G.data(), ldg, nrhs, Wq.data(), ldq, true);
    allreduce_sum(g.world(), G.data(), ldg * size_t(nrhs), c);
    for (int64_t i = 0; i < C.mt(); ++i) {
        if (C.srow_owner(i) != myrow) continue;
        for (int64_t j = 0; j < C.nt(); ++j) {
            if (C.scol_owner(j) != mycol) continue;
            T* cp = lc.ptr + lrow_of(C, i) + lcol_of(C, j) * lc.ld;
            scale_c(c, beta, C.tileMb(i), C.tileNb(j), cp, lc.ld);
            lb::add(c, Uplo::General, C.tileMb(i), C.tileNb(j), alpha, G.data() + grow_of(C, i) + gcol_of(C, j) * ldg,
                    ldg, T(1), cp, lc.ld);
        }
    }
    sync_ctx(c);
}

/// distributed hemm / symm: MethodHemm picks hemmA (narrow B) or hemmC;
/// Right is reduced to Left on (conj-)transposed copies of B and C.
template <typename T>
void hemm_dist(Side side, bool herm, T alpha, BaseTrapezoidMatrix<T> const& A, Matrix<T> const& B, T beta,
               Matrix<T>& C, Options const& opts) {
    Target target = resolve_target(opts);
    Method method = get_option<int64_t>(opts, Option::MethodHemm, MethodHemm::Auto);
    if (method == MethodHemm::Auto)   // narrow B: one block of right-hand sides (columns Left, rows Right)
        method = (side == Side::Left ? B.nt() : B.mt()) < 2 ? MethodHemm::HemmA : MethodHemm::HemmC;
    slate_error_if_msg(method != MethodHemm::HemmA && method != MethodHemm::HemmC, "hemm: unknown MethodHemm");
    auto gC = C.grid();
    if (side == Side::Right && method == MethodHemm::HemmC && C.op() == Op::NoTrans && C.aligned() &&
        A.op() == Op::NoTrans && A.aligned() && A.mb() == A.nb() && B.op() == Op::NoTrans && B.aligned() &&
        cols_conform(BaseMatrix<T>(A), BaseMatrix<T>(C)) && rows_conform(BaseMatrix<T>(B), BaseMatrix<T>(C)) &&
        B.nt() == A.nt()) {
        bool ok = true;
        for (int64_t j = 0; j < A.nt(); ++j) ok = ok && B.tileNb(j) == A.tileNb(j) && A.tileMb(j) == A.tileNb(j);
        if (ok) {
            hemmC_right(A.uplo(), herm, alpha, A, B, beta, C, target, option_la(opts));
            return;
        }
    }
    if (side == Side::Right) {
        // C = a B A + b C  <=>  C^H = conj(a) A B^H + conj(b) C^H (A = A^H), C^T = a A B^T + b C^T (A = A^T)
        Matrix<T> Ct = materialize<T>(herm ? conj_transpose(C) : transpose(C), target, gC, C.nb(), C.mb(), 0, 0);
        Matrix<T> Bt = materialize<T>(herm ? conj_transpose(B) : transpose(B), target, gC, C.nb(), C.mb(), 0, 0);
        Options o2 = opts;
        o2[Option::MethodHemm] = method;
        hemm_dist(Side::Left, herm, herm ? slate::conj(alpha) : alpha, A, Bt, herm ? slate::conj(beta) : beta, Ct, o2);
        slate::copy<T, T>(herm ? conj_transpose(Ct) : transpose(Ct), C, opts);
        return;
    }
    // C must be a NoTrans aligned view; B and A conform to it (else copies)
    Matrix<T> Cx, Bx, Ax;
    Matrix<T>* Cu = &C;
    const bool cdirect = C.op() == Op::NoTrans && C.aligned();
    if (!cdirect) {
        Cx = materialize<T>(C, target, gC, C.mb(), C.nb(), 0, 0);
        Cu = &Cx;
    }
    BaseMatrix<T> Bu = B;
    if (!(rows_conform(BaseMatrix<T>(B), BaseMatrix<T>(*Cu)) && cols_conform(BaseMatrix<T>(B), BaseMatrix<T>(*Cu)))) {
        Bx = materialize<T>(B, target, gC, Cu->mb(), Cu->nb(), row0_owner(*Cu), col0_owner(*Cu));
        Bu = Bx;
    }
    BaseMatrix<T> Au = A;
    bool aconf = A.op() == Op::NoTrans && rows_conform(BaseMatrix<T>(A), BaseMatrix<T>(*Cu)) && A.nt() == Cu->mt();
    if (aconf)
        for (int64_t j = 0; j < A.nt(); ++j) if (A.tileNb(j) != Cu->tileMb(j)) aconf = false;
    if (!aconf) {
        Ax = materialize<T>(A, target, gC, Cu->mb(), Cu->mb(), row0_owner(*Cu), 0);
        Au = Ax;
    }
    if (method == MethodHemm::HemmA) hemmA_left(A.uplo(), herm, alpha, Au, Bu, beta, *Cu, target);
    else hemmC_left(A.uplo(), herm, alpha, Au, Bu, beta, *Cu, target, option_la(opts));
    if (!cdirect) slate::copy<T, T>(Cx, C, opts);
}

}  // namespace

template <typename T>
void hemm(Side side, T alpha, HermitianMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts) {
    if (internal::spread<T>(opts, {{&A, false}, {&B, false}, {&C, true}}, [&](std::vector<Matrix<T>>& M, int) {
            auto Ar = internal::rewrap(A, M[0]);
            hemm(side, alpha, Ar, M[1], beta, M[2], opts);
        }, false))
        return;
    trace::Block tb("hemm");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && local_only(B) && C.op() == Op::NoTrans && B.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
        lb::hemm(c, side, A.uplo_physical(), lc.m, lc.n, alpha, la_.ptr, la_.ld, lbk.ptr, lbk.ld, beta,
                 lc.ptr, lc.ld, true);
        sync_ctx(c);
        internal::finish_origin(C, opts);
        return;
    }
    hemm_dist<T>(side, true, alpha, A, B, beta, C, opts);
    internal::finish_origin(C, opts);
}

template <typename T>
void symm(Side side, T alpha, SymmetricMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts) {
    trace::Block tb("symm");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(C) && local_only(A) && local_only(B) && C.op() == Op::NoTrans && B.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
        lb::hemm(c, side, A.uplo_physical(), lc.m, lc.n, alpha, la_.ptr, la_.ld, lbk.ptr, lbk.ld, beta,
                 lc.ptr, lc.ld, false);
        sync_ctx(c);
        internal::finish_origin(C, opts);
        return;
    }
    hemm_dist<T>(side, false, alpha, A, B, beta, C, opts);
    internal::finish_origin(C, opts);
}

template <typename T>
void trmm(Side side, T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    if (internal::spread<T>(opts, {{&A, false}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int) {
            auto Ar = internal::rewrap(A, M[0]);
            trmm(side, alpha, Ar, M[1], opts);
        }, false))
        return;
    trace::Block tb("trmm");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    if (local_only(B) && local_only(A) && B.op() == Op::NoTrans) {
        lb::Ctx c = ctx_for(target);
        LocalBlock<T> la_ = A.local(loc, false), lbk = B.local(loc, true);
        lb::trmm(c, side, A.uplo_physical(), A.op(), A.diag(), lbk.m, lbk.n, alpha, la_.ptr, la_.ld,
                 lbk.ptr, lbk.ld);
        sync_ctx(c);
        internal::finish_origin(B, opts);
        return;
    }
    // distributed: reduce to Left with a NoTrans triangle conforming to B's
    // rows (as trsm does), then a SUMMA that skips the zero part of A
    auto gB = B.grid();
    if (side == Side::Right) {
        // in place on B when op(A)'s columns conform to B's (see tr_right_sweep)
        const Op op = A.op();
        BaseMatrix<T> Ap = op == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(op == Op::ConjTrans);
        if (Ap.aligned() && (b_conforms_right(Ap, op, B) || (op != Op::NoTrans && b_conforms_right(Ap, Op::NoTrans, B)))) {
            tr_right_sweep(false, A.uplo_physical(), op, A.diag(), alpha, Ap, B, target, option_la(opts),
                           !b_conforms_right(Ap, op, B));
            internal::finish_origin(B, opts);
            return;
        }
    }
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
    internal::finish_origin(B, opts);
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
