// Distributed Householder QR / LQ and least squares (reference src/geqrf.cc,
// unmqr.cc, gelqf.cc, unmlq.cc, gels.cc, gels_qr.cc, gels_cholqr.cc, cholqr.cc).
//
// geqrf per block column k:
//   panel: the m x nb panel is factored on the device by the recursive
//     Householder kernel (column norms, reflector, rank-1 updates and the
//     T factor all on the GPU; T from V^H V + the larft recurrence, as the
//     reference's larft-by-gemm trick internal_geqrf.cc:286-330).  p > 1:
//     gathered to the diagonal process, factored, scattered back.
//   update: the explicit V (unit lower) and T_k are broadcast along process
//     rows; every process computes W = V_loc^H C_loc for its trailing
//     columns, the partial W is all-reduced over the column communicator
//     (p > 1), then W = T^H W and C_loc -= V_loc W -- two MFMA GEMMs and a
//     small one per process (ScaLAPACK-style 2D larfb).  The reference uses
//     a TSQR tree (ttqrt/ttmqr) for the p > 1 panel instead.
// T factors: T[0] is an nb x n matrix replicated on every rank (tile k holds
// the panel's nb x nb upper-triangular T).
#include "internal.hh"

#include <cstdlib>

namespace slate {

using namespace internal;

namespace {

/// K-chunk (rows) of the trailing update's W = V^H C; SLATE_QR_KCHUNK, 0 = off
inline int64_t qr_kchunk() {
    static int64_t v = [] {
        const char* e = std::getenv("SLATE_QR_KCHUNK");
        return e ? std::atoll(e) : int64_t(8192);
    }();
    return v;
}

template <typename T>
void geqrf_impl(BaseMatrix<T> A, Matrix<T>& Tf, Target target, int64_t la) {
    auto& g = *A.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t mt = A.mt(), nt = A.nt(), m = A.m(), n = A.n();
    const int64_t kt = std::min(mt, nt);
    const int64_t nb = A.nb();
    LocalBlock<T> L = A.local(loc, true);
    T* a = L.ptr;
    const int64_t lda = L.ld, mloc = L.m, nloc = L.n;
    LocalBlock<T> LT = Tf.local(loc, true);   // replicated nb x n
    T* tm = LT.ptr;
    const int64_t ldt = LT.ld;

    Sched S(target);
    const int R = int(std::max<int64_t>(2, la + 2));
    std::vector<Work<T>> WV(R), WT(R), WW(R), WW2(R), Wtau(R);
    for (int r = 0; r < R; ++r) {
        WV[r].resize(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
        WT[r].resize(target, size_t(nb) * nb);
        WW[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
        WW2[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
        Wtau[r].resize(target, size_t(nb));
    }
    Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;

    for (int64_t k = 0; k < kt; ++k) {
        const int64_t kb = A.tileNb(k);
        const int64_t kk = grow_of(A, k);
        const int64_t M = m - kk;
        const int64_t kd = std::min(kb, M);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const bool in_col = (mycol == qk);
        const int64_t lr_k = lrow_of(A, k);
        const int64_t lc_k = in_col ? lcol_of(A, k) : 0;
        const int64_t mr = mloc - lr_k;          // my rows >= kk
        const int slot = int(k % R);
        T* Tk = WT[slot].data();
        T* tau = Wtau[slot].data();
        const int64_t tP = Sched::tok(6, slot), tB = Sched::bcast(slot);

        // ---------------------------------------------------------- panel
        if (in_col) {
            int qq = (p == 1) ? 1 : device::kCommQueue;
            S.task(qq, {}, {Sched::col(k), tP}, [&, k, kb, kk, M, kd, lr_k, lc_k, mr, pk, Tk, tau](lb::Ctx const& c) {
                trace::Block t2("geqrf_panel");
                T* ap = a + lr_k + lc_k * lda;
                if (p == 1) {
                    lb::geqrf_panel(c, M, kb, ap, lda, tau, Tk, kb);
                    return;
                }
                // gather rows >= kk of the panel to pk, factor, scatter back
                std::vector<int64_t> cnt(p, 0);
                for (int64_t i = k; i < mt; ++i) cnt[A.srow_owner(i)] += A.tileMb(i);
                Work<T> full(target, size_t(std::max<int64_t>(M, 1)) * kb);
                Work<T> mine(target, size_t(std::max<int64_t>(mr, 1)) * kb);
                pack(c, mr, kb, ap, lda, mine.data());
                std::vector<Work<T>> rb(p);
                std::vector<Comm::P2P> ops;
                if (myrow == pk) {
                    for (int r = 0; r < p; ++r) if (r != pk && cnt[r]) {
                        rb[r].resize(target, size_t(cnt[r]) * kb);
                        ops.push_back({rb[r].data(), size_t(cnt[r] * kb), r, false});
                    }
                } else if (mr > 0) ops.push_back({mine.data(), size_t(mr * kb), pk, true});
                g.col().exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                if (myrow == pk) {
                    std::vector<int64_t> off(p, 0);
                    for (int64_t i = k; i < mt; ++i) {
                        int r = A.srow_owner(i); int64_t ib = A.tileMb(i);
                        T* src = (r == pk) ? mine.data() + off[r] : rb[r].data() + off[r];
                        int64_t lds = (r == pk) ? std::max<int64_t>(mr, 1) : cnt[r];
                        lb::copy2d(c, ib, kb, src, lds, full.data() + (grow_of(A, i) - kk), std::max<int64_t>(M, 1));
                        off[r] += ib;
                    }
                    lb::geqrf_panel(c, M, kb, full.data(), std::max<int64_t>(M, 1), tau, Tk, kb);
                    std::fill(off.begin(), off.end(), 0);
                    for (int64_t i = k; i < mt; ++i) {
                        int r = A.srow_owner(i); int64_t ib = A.tileMb(i);
                        T* dst = (r == pk) ? mine.data() + off[r] : rb[r].data() + off[r];
                        int64_t ldd = (r == pk) ? std::max<int64_t>(mr, 1) : cnt[r];
                        lb::copy2d(c, ib, kb, full.data() + (grow_of(A, i) - kk), std::max<int64_t>(M, 1), dst, ldd);
                        off[r] += ib;
                    }
                }
                ops.clear();
                if (myrow == pk) {
                    for (int r = 0; r < p; ++r) if (r != pk && cnt[r]) ops.push_back({rb[r].data(), size_t(cnt[r] * kb), r, true});
                } else if (mr > 0) ops.push_back({mine.data(), size_t(mr * kb), pk, false});
                g.col().exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                lb::copy2d(c, mr, kb, mine.data(), std::max<int64_t>(mr, 1), ap, lda);
                if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
            });
        }
        // -------------------- broadcast T_k (world, from the diagonal owner) and V
        T* Vk = WV[slot].data();
        const int64_t ldv = std::max<int64_t>(mr, 1);
        S.task(device::kCommQueue, {tP, Sched::col(k)}, {tB}, [&, k, kb, kk, kd, lr_k, lc_k, mr, pk, qk, Tk, Vk, ldv](lb::Ctx const& c) {
            trace::Block t2("geqrf_bcast");
            int root = g.rank_of(pk, qk);
            g.world().bcast(Tk, size_t(kb * kb), scalar_type<T>(), root, c.loc(), c.stream);
            if (mycol == qk) {
                // explicit V: my rows >= kk; the diagonal process row has the unit upper part
                pack(c, mr, kb, a + lr_k + lc_k * lda, lda, Vk);
                if (myrow == pk) lb::set(c, Uplo::Upper, std::min<int64_t>(kb, mr), kb, T(0), T(1), Vk, ldv);
            }
            if (q > 1) bcast(g.row(), Vk, size_t(mr * kb), qk, c);
            // keep T_k in the replicated factor matrix
            lb::copy2d(c, kb, kb, Tk, kb, tm + kk * ldt, ldt);
        });

        // ---------------------------------------------------------- update
        T* Wk = WW[slot].data();
        T* W2k = WW2[slot].data();
        auto update = [&, k, kb, lr_k, mr, Tk, Vk, ldv, Wk, W2k, cT](lb::Ctx const& c, int64_t j0, int64_t j1) {
            int64_t c0 = lcol_of(A, j0), c1 = lcol_of(A, j1), nc = c1 - c0;
            if (nc <= 0) return;
            trace::Block t2("geqrf_update");
            T* Cc = a + lr_k + c0 * lda;
            T* W = Wk + c0 * kb;
            T* W2 = W2k + c0 * kb;
            // W = V^H C  (kb x nc), all-reduced over the process column
            // On a wide trailing block this GEMM's K (= mr rows) is long, so
            // without chunking each workgroup lives for milliseconds and the
            // next panel's short kernels (high-priority stream) find no free
            // CU until it drains.  K chunks of kch rows, accumulated in W,
            // bound the workgroup lifetime.
            const int64_t kch = qr_kchunk();
            if (mr > 0 && kch > 0 && mr > kch && nc >= 4 * kb) {
                for (int64_t r0 = 0; r0 < mr; r0 += kch)
                    lb::gemm(c, cT, Op::NoTrans, kb, nc, std::min(kch, mr - r0), T(1), Vk + r0, ldv, Cc + r0, lda,
                             r0 ? T(1) : T(0), W, kb);
            } else if (mr > 0) lb::gemm(c, cT, Op::NoTrans, kb, nc, mr, T(1), Vk, ldv, Cc, lda, T(0), W, kb);
            else lb::set(c, Uplo::General, kb, nc, T(0), T(0), W, kb);
            if (p > 1) g.col().allreduce(W, W, size_t(kb * nc), scalar_type<T>(), ReduceOp::Sum, c.loc(), c.stream);
            lb::gemm(c, cT, Op::NoTrans, kb, nc, kb, T(1), Tk, kb, W, kb, T(0), W2, kb);
            if (mr > 0) lb::gemm(c, Op::NoTrans, Op::NoTrans, mr, nc, kb, T(-1), Vk, ldv, W2, kb, T(1), Cc, lda);
        };
        auto range = [&](int queue, int64_t j0, int64_t j1) {
            std::vector<int64_t> cols;
            for (int64_t j = j0; j < j1; ++j) cols.push_back(Sched::col(j));
            // with p > 1 the update contains an all-reduce: keep it on the comm queue
            int qq = (p == 1) ? queue : device::kCommQueue;
            S.task(qq, {tB}, cols, [&, update, j0, j1](lb::Ctx const& c) { update(c, j0, j1); });
        };
        int64_t jla_end = std::min(nt, k + 1 + la);
        for (int64_t j = k + 1; j < jla_end; ++j) range(device::kLookaheadQueue, j, j + 1);
        if (jla_end < nt) range(device::kTrailQueue, jla_end, nt);
        (void)kd;
    }
    S.wait_all();
    A.storage()->update_origin();
    Tf.storage()->update_origin();
}

/// Apply Q (or Q^H) from geqrf to C from the left: C = op(Q) C.
template <typename T>
void unmqr_left(Op op, BaseMatrix<T> A, Matrix<T> const& Tf, Matrix<T>& C, Target target) {
    auto& g = *A.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    (void)myrow;
    const Loc loc = loc_of(target);
    const int64_t kt = std::min(A.mt(), A.nt());
    const int64_t m = A.m();
    LocalBlock<T> L = A.local(loc, false);
    LocalBlock<T> LC = C.local(loc, true);
    LocalBlock<T> LT = Tf.local(loc, false);
    const int64_t nb = A.nb();
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    Work<T> Vk(target, size_t(std::max<int64_t>(L.m, 1)) * nb), W(target, size_t(nb) * std::max<int64_t>(LC.n, 1)),
        W2(target, size_t(nb) * std::max<int64_t>(LC.n, 1));
    Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
    // Q^H C: k ascending with T^H; Q C: k descending with T
    for (int64_t t = 0; t < kt; ++t) {
        int64_t k = (op == Op::NoTrans) ? kt - 1 - t : t;
        int64_t kb = A.tileNb(k), kk = grow_of(A, k);
        int pk = A.srow_owner(k), qk = A.scol_owner(k);
        int64_t lr_k = lrow_of(A, k), mr = L.m - lr_k, ldv = std::max<int64_t>(mr, 1);
        int64_t lcr = lrow_of(C, k);    // C's local rows >= kk (C conforms to A's rows)
        if (mycol == qk) {
            pack(c, mr, kb, L.ptr + lr_k + lcol_of(A, k) * L.ld, L.ld, Vk.data());
            if (g.myrow() == pk) lb::set(c, Uplo::Upper, std::min<int64_t>(kb, mr), kb, T(0), T(1), Vk.data(), ldv);
        }
        if (q > 1) bcast(g.row(), Vk.data(), size_t(mr * kb), qk, c);
        int64_t nc = LC.n;
        T* Cc = LC.ptr + lcr;
        if (mr > 0) lb::gemm(c, cT, Op::NoTrans, kb, nc, mr, T(1), Vk.data(), ldv, Cc, LC.ld, T(0), W.data(), kb);
        else lb::set(c, Uplo::General, kb, nc, T(0), T(0), W.data(), kb);
        if (p > 1) g.col().allreduce(W.data(), W.data(), size_t(kb * nc), scalar_type<T>(), ReduceOp::Sum, c.loc(), c.stream);
        lb::gemm(c, op == Op::NoTrans ? Op::NoTrans : cT, Op::NoTrans, kb, nc, kb, T(1), LT.ptr + kk * LT.ld, LT.ld,
                 W.data(), kb, T(0), W2.data(), kb);
        if (mr > 0) lb::gemm(c, Op::NoTrans, Op::NoTrans, mr, nc, kb, T(-1), Vk.data(), ldv, W2.data(), kb, T(1), Cc, LC.ld);
        (void)m;
    }
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    C.storage()->update_origin();
}

}  // namespace

template <typename T>
void geqrf(Matrix<T>& A, TriangularFactors<T>& T_, Options const& opts) {
    trace::Block tb("geqrf");
    Target target = resolve_target(opts);
    int64_t la = get_option<int64_t>(opts, Option::Lookahead, 1);
    slate_error_if_msg(A.op() != Op::NoTrans || !A.aligned() || A.mb() != A.nb(),
                       "geqrf: NoTrans, tile-aligned, square-tile matrix required");
    Matrix<T> Tf(A.nb(), std::max<int64_t>(A.n(), 1), A.nb(), A.nb(), Grid::self());
    Tf.insertLocalTiles(target);
    set(T(0), T(0), Tf, opts);
    geqrf_impl<T>(A, Tf, target, la);
    if (target == Target::Devices) lb::check_panel_errors();
    T_.clear();
    T_.push_back(Tf);
}

template <typename T>
void unmqr(Side side, Op op, Matrix<T> const& A, TriangularFactors<T> const& T_, Matrix<T>& C, Options const& opts) {
    trace::Block tb("unmqr");
    Target target = resolve_target(opts);
    slate_error_if_msg(T_.empty(), "unmqr: missing T factors");
    if (is_complex_v<T> == false && op == Op::ConjTrans) op = Op::Trans;
    if (side == Side::Left) {
        // same processes in the same p x q arrangement (a transposed grid has
        // the same processes and sizes but a different rank mapping)
        bool conform = C.op() == Op::NoTrans && C.aligned() && C.grid()->same_processes(*A.grid())
                    && C.grid()->p() == A.grid()->p() && C.grid()->q() == A.grid()->q()
                    && C.grid()->order() == A.grid()->order() && C.mt() == A.mt();
        if (conform)
            for (int64_t i = 0; i < A.mt(); ++i)
                if (A.tileMb(i) != C.tileMb(i) || A.srow_owner(i) != C.srow_owner(i)) { conform = false; break; }
        if (conform) {
            unmqr_left<T>(op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans, A, T_[0], C, target);
        } else {
            Matrix<T> Cx(C.m(), C.n(), A.mb(), C.nb(), A.grid(), A.mt() ? A.srow_owner(0) : 0, 0);
            Cx.insertLocalTiles(target);
            slate::copy<T, T>(C, Cx, opts);
            unmqr_left<T>(op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans, A, T_[0], Cx, target);
            slate::copy<T, T>(Cx, C, opts);
        }
        return;
    }
    // C op(Q) = (op(Q)^H C^H)^H
    Matrix<T> Ch = C.emptyLike(0, 0, Op::ConjTrans);
    Ch.insertLocalTiles(target);
    slate::copy<T, T>(conj_transpose(C), Ch, opts);
    // Ch must conform to A's rows: materialize on A's grid
    Matrix<T> Cx(Ch.m(), Ch.n(), A.mb(), C.mb(), A.grid(), A.mt() ? A.srow_owner(0) : 0, 0);
    Cx.insertLocalTiles(target);
    slate::copy<T, T>(Ch, Cx, opts);
    unmqr_left<T>(op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans, A, T_[0], Cx, target);
    slate::copy<T, T>(conj_transpose(Cx), C, opts);
}

// LQ via the QR of A^H: A^H = Q' R'  =>  A = R'^H Q'^H = L Q.
template <typename T>
void gelqf(Matrix<T>& A, TriangularFactors<T>& T_, Options const& opts) {
    trace::Block tb("gelqf");
    Target target = resolve_target(opts);
    Matrix<T> Ah = A.emptyLike(0, 0, Op::ConjTrans);
    Ah.insertLocalTiles(target);
    slate::copy<T, T>(conj_transpose(A), Ah, opts);
    geqrf(Ah, T_, opts);
    slate::copy<T, T>(conj_transpose(Ah), A, opts);
}

template <typename T>
void unmlq(Side side, Op op, Matrix<T> const& A, TriangularFactors<T> const& T_, Matrix<T>& C, Options const& opts) {
    trace::Block tb("unmlq");
    Target target = resolve_target(opts);
    // Q = Q'^H where Q' is the QR factor of A^H
    Matrix<T> Ah = A.emptyLike(0, 0, Op::ConjTrans);
    Ah.insertLocalTiles(target);
    slate::copy<T, T>(conj_transpose(A), Ah, opts);
    Op o2 = (op == Op::NoTrans) ? Op::ConjTrans : Op::NoTrans;
    unmqr(side, o2, Ah, T_, C, opts);
}

template <typename T>
void gels(Matrix<T>& A, TriangularFactors<T>& T_, Matrix<T>& BX, Options const& opts) {
    trace::Block tb("gels");
    const int64_t m = A.m(), n = A.n(), nrhs = BX.n();
    Method method = get_option<int64_t>(opts, Option::MethodGels, MethodGels::Geqrf);
    if (m >= n) {
        if (method == MethodGels::Cholqr) {
            Matrix<T> R(n, n, A.nb(), A.nb(), A.grid());
            R.insertLocalTiles(resolve_target(opts));
            cholqr(A, R, opts);
            // X = R^{-1} Q^H B
            Matrix<T> Y(n, nrhs, A.nb(), BX.nb(), A.grid());
            Y.insertLocalTiles(resolve_target(opts));
            gemm(T(1), conj_transpose(A), Matrix<T>(BX.sub(0, BX.mt() - 1, 0, BX.nt() - 1)), T(0), Y, opts);
            Matrix<T> Rg(R); Rg.set_uplo(Uplo::General);
            trsm(Side::Left, T(1), TriangularMatrix<T>(Uplo::Upper, Diag::NonUnit, Rg), Y, opts);
            Matrix<T> X = BX.slice(0, n - 1, 0, nrhs - 1);
            slate::copy<T, T>(Y, X, opts);
            return;
        }
        geqrf(A, T_, opts);
        unmqr(Side::Left, Op::ConjTrans, A, T_, BX, opts);
        Matrix<T> R = A.slice(0, n - 1, 0, n - 1);
        R.set_uplo(Uplo::General);
        Matrix<T> X = BX.slice(0, n - 1, 0, nrhs - 1);
        trsm(Side::Left, T(1), TriangularMatrix<T>(Uplo::Upper, Diag::NonUnit, R), X, opts);
    } else {
        // minimum-norm solution: A = L Q, X = Q^H L^{-1} B
        gelqf(A, T_, opts);
        Matrix<T> Lm = A.slice(0, m - 1, 0, m - 1);
        Lm.set_uplo(Uplo::General);
        Matrix<T> Bt = BX.slice(0, m - 1, 0, nrhs - 1);
        trsm(Side::Left, T(1), TriangularMatrix<T>(Uplo::Lower, Diag::NonUnit, Lm), Bt, opts);
        // zero rows m..n-1 of BX, then apply Q^H
        if (n > m) {
            Matrix<T> Z = BX.slice(m, n - 1, 0, nrhs - 1);
            set(T(0), T(0), Z, opts);
        }
        unmlq(Side::Left, Op::ConjTrans, A, T_, BX, opts);
    }
}

template <typename T>
int64_t cholqr(Matrix<T>& A, Matrix<T>& R, Options const& opts) {
    trace::Block tb("cholqr");
    // R^H R = A^H A ; Q = A R^{-1} (reference src/cholqr.cc)
    Target target = resolve_target(opts);
    (void)target;
    HermitianMatrix<T> H(Uplo::Upper, R);
    herk(real_type<T>(1), conj_transpose(A), real_type<T>(0), H, opts);
    int64_t info = potrf(H, opts);
    if (info) return info;
    Matrix<T> Rg(R); Rg.set_uplo(Uplo::General);
    trsm(Side::Right, T(1), TriangularMatrix<T>(Uplo::Upper, Diag::NonUnit, Rg), A, opts);
    return 0;
}

#define SLATE_QR_INST(T)                                                                                 \
    template void geqrf<T>(Matrix<T>&, TriangularFactors<T>&, Options const&);                          \
    template void unmqr<T>(Side, Op, Matrix<T> const&, TriangularFactors<T> const&, Matrix<T>&, Options const&); \
    template void gelqf<T>(Matrix<T>&, TriangularFactors<T>&, Options const&);                          \
    template void unmlq<T>(Side, Op, Matrix<T> const&, TriangularFactors<T> const&, Matrix<T>&, Options const&); \
    template void gels<T>(Matrix<T>&, TriangularFactors<T>&, Matrix<T>&, Options const&);               \
    template int64_t cholqr<T>(Matrix<T>&, Matrix<T>&, Options const&);

SLATE_QR_INST(float)
SLATE_QR_INST(double)
SLATE_QR_INST(std::complex<float>)
SLATE_QR_INST(std::complex<double>)

}  // namespace slate
