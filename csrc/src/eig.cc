// Two-stage Hermitian eigensolver and SVD drivers (reference src/heev.cc,
// he2hb.cc, hb2st.cc, unmtr_he2hb.cc, unmtr_hb2st.cc, hegst.cc, hegv.cc,
// svd.cc, ge2tb.cc, tb2bd.cc, bdsqr.cc, unmbr_ge2tb.cc).
//
// Stage 1 (distributed, target = Devices runs on the MFMA kernels): he2hb /
// ge2tb reduce to band form with one geqrf (and gelqf) per block column and
// two-sided block updates through unmqr / unmlq, so every flop-heavy piece is
// the same device-resident QR machinery as the geqrf headline.
// Stage 2: the band (O(n nb) data) is gathered to every rank and chased to
// tridiagonal / bidiagonal on the host (eig_host.cc, deterministic); the
// tridiagonal eigenvectors come from the distributed divide and conquer (Q on
// the 2-D grid, merges as MFMA GEMMs) or the QL iteration with the rotations
// applied to each rank's rows (eig_dist.cc); bdsqr's rotations likewise act on
// each rank's rows of U / Vt (eig_sinks.hh).  The stage-2 reflectors are
// applied blocked to each rank's columns (unmtr_hb2st_blocked), then the
// stage-1 back-transform runs distributed (unmqr / unmlq on Z, U, VT).  No
// rank holds an n x n array on the host.
#include "internal.hh"
#include "spread.hh"
#include "eig_sinks.hh"
#include "slate_amd/eig_host.hh"
#include "../kernels/kernels.hh"

#include <algorithm>
#include <exception>
#include <thread>
#include <omp.h>
#include <cmath>
#include <map>

namespace slate {

using namespace internal;

namespace {

/// Dense Hermitian copy (both triangles) of A in a general matrix.
template <typename T>
Matrix<T> hermitian_full(HermitianMatrix<T> const& A, Options const& opts) {
    Target target = resolve_target(opts);
    Matrix<T> Ag(A);
    Ag.set_uplo(Uplo::General);
    Matrix<T> F = Ag.emptyLike();
    F.insertLocalTiles(target);
    slate::copy<T, T>(conj_transpose(Ag), F, opts);
    BaseTrapezoidMatrix<T> At(A.uplo(), Ag, MatrixKind::Trapezoid), Ft(A.uplo(), F, MatrixKind::Trapezoid);
    slate::copy<T, T>(At, Ft, opts);
    return F;
}

/// Fill a distributed matrix from a replicated host array (column-major).
template <typename T>
void fill_from_host(Matrix<T>& M, std::vector<T> const& h, int64_t ldh) {
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) { return h[i + j * ldh]; }), M, oh);
}

template <typename T>
bool wanted(Matrix<T> const& M) { return M.m() > 0 && M.n() > 0; }

/// Band of a distributed matrix (reference heev.cc he2hbGather, but onto every
/// process): only the tiles (k, k) and (k+1, k) (lower) or (k, k+1) (upper)
/// move, and only their entries with 0 <= i - j <= kd (lower) or 0 <= j - i
/// <= kd (upper), into general band storage with kl = ku = M (room for the
/// bulge chase: M = 2 kd for hb2st, 3 kd + 2 for tb2bd): (i, j) at
/// ab[M + i - j + j ldab], ldab = 2 M + 1.  One world all-reduce of O(n kd)
/// data; no n x n array anywhere.  Hermitian (mirror = true): the other half is filled with the conjugate.
template <typename T>
std::vector<T> gather_band(Matrix<T> const& A, int64_t kd, int64_t M, bool lower, bool mirror, Options const& opts) {
    trace::Block tb("gather_band");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    auto& g = *A.grid();
    const int64_t n = std::min(A.m(), A.n()), ldab = 2 * M + 1;
    std::vector<T> ab(size_t(ldab) * std::max<int64_t>(n, 1), T(0));
    LocalBlock<T> la = A.local(loc, false);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    const int64_t mb = A.mb(), nbt = A.nb();
    Work<T> dt(target, size_t(mb) * nbt);
    std::vector<T> ht(size_t(mb) * nbt);
    auto take = [&](int64_t i, int64_t j) {
        if (i < 0 || j < 0 || i >= A.mt() || j >= A.nt()) return;
        if (A.srow_owner(i) != g.myrow() || A.scol_owner(j) != g.mycol()) return;
        const int64_t tm = A.tileMb(i), tn = A.tileNb(j), gi0 = grow_of(A, i), gj0 = gcol_of(A, j);
        T const* src = la.ptr + lrow_of(A, i) + lcol_of(A, j) * la.ld;
        if (c.dev()) {
            lb::copy2d(c, tm, tn, src, la.ld, dt.data(), tm);
            device::memcpy_async(ht.data(), dt.data(), size_t(tm) * tn * sizeof(T), c.stream);
            slate_hip_call(hipStreamSynchronize(c.stream));
        } else {
            for (int64_t jj = 0; jj < tn; ++jj)
                for (int64_t ii = 0; ii < tm; ++ii) ht[ii + jj * tm] = src[ii + jj * la.ld];
        }
        for (int64_t jj = 0; jj < tn; ++jj)
            for (int64_t ii = 0; ii < tm; ++ii) {
                const int64_t gi = gi0 + ii, gj = gj0 + jj, off = lower ? gi - gj : gj - gi;
                if (off < 0 || off > kd || gi >= n || gj >= n) continue;
                ab[size_t(M + gi - gj + gj * ldab)] = ht[ii + jj * tm];
            }
    };
    for (int64_t k = 0; k < std::min(A.mt(), A.nt()); ++k) {
        take(k, k);
        if (lower) take(k + 1, k);
        else take(k, k + 1);
    }
    internal::allreduce_host(g.world(), ab.data(), ab.size(), ReduceOp::Sum);
    if (mirror) {
        for (int64_t j = 0; j < n; ++j) {
            for (int64_t i = j + 1; i <= std::min(n - 1, j + kd); ++i) {
                T& lo = ab[size_t(M + i - j + j * ldab)];
                T& up = ab[size_t(M + j - i + i * ldab)];
                if (lower) up = slate::conj(lo); else lo = slate::conj(up);
            }
            T& dd = ab[size_t(M + j * ldab)];
            dd = T(std::real(dd));
        }
    }
    return ab;
}

/// The T factors of the two-stage reductions' panels (he2hb / ge2tb: panel k
/// factored on its own, T_k tile-column 0 of Ts[k][0]) side by side, as the T
/// of the geqrf- / gelqf-shaped view the panels form together: the stage-1
/// back-transforms are then ONE unmqr / unmlq call over all panels, one DAG
/// with no host wait between panels, where the panel-by-panel loop built a
/// scheduler and waited nt - 1 times.  Width: the view's
/// columns plus one tile (gelqf's convention, room for a full last tile).
template <typename T>
TriangularFactors<T> stacked_T(std::vector<TriangularFactors<T>> const& Ts, int64_t nk, int64_t nb, int64_t ncols,
                               Options const& opts) {
    Target target = resolve_target(opts);
    Matrix<T> Tf(nb, ncols + nb, nb, nb, Grid::self());
    Tf.insertLocalTiles(target);
    set(T(0), T(0), Tf, opts);
    for (int64_t k = 0; k < nk && k < int64_t(Ts.size()); ++k) {
        if (Ts[k].empty()) continue;
        Matrix<T> const& Tk = Ts[k][0];
        const int64_t w = std::min<int64_t>({Tk.n(), nb, ncols + nb - k * nb});
        if (w <= 0) continue;
        Matrix<T> src = Tk.slice(0, nb - 1, 0, w - 1);
        Matrix<T> dst = Tf.slice(0, nb - 1, k * nb, k * nb + w - 1);
        slate::copy<T, T>(src, dst, opts);
    }
    return TriangularFactors<T>{Tf};
}

/// Stage 2 and the stage-1 back-transform overlapped: the host bulge chase
/// (hb2st / tb2bd, rank 0, OpenMP) runs in a side thread while this thread
/// forms the explicit stage-1 orthogonal factor on the device (unmqr / unmlq
/// of the panels on an identity); the back-transform at the end is then one
/// GEMM instead of the reflector application, which used to run after the
/// chase with the GPU idle meanwhile.  GPU work stays on the calling thread.
/// SLATE_EIG_OVERLAP=0: sequential (the reflectors applied at the end);
/// 1: on for the device target; 2: on for the host target as well (the CPU
/// tests cover the path with it).  Unset: on for svd, off for heev -- the
/// side thread slows hb2st's spin-waiting pipeline by 15-70 ms, about what
/// hiding the 105 ms stage-1 application gains (same-box A/B 1.089 vs 1.135
/// and 1.172 vs 1.157 s), while svd gains ~100 ms
/// (profiles/r4_eig_overlap_ab.txt).
inline bool eig_overlap(Target target, bool by_default) {
    const char* e = std::getenv("SLATE_EIG_OVERLAP");
    const int v = e ? std::atoi(e) : (by_default ? 1 : 0);
    return v == 2 || (v != 0 && target == Target::Devices);
}

/// C = op(A) B for the overlapped back-transforms on one process: one local
/// GEMM straight from the operands' arrays into C's (no work copies of the
/// n x n operands or the result).  Returns false (nothing done) otherwise.
template <typename T>
bool local_product(Op opA, Matrix<T>& A, Matrix<T>& B, Matrix<T>& C, Options const& opts) {
    if (A.grid()->size() != 1 || B.grid()->size() != 1 || C.grid()->size() != 1 || A.op() != Op::NoTrans ||
        B.op() != Op::NoTrans || C.op() != Op::NoTrans || A.arbitrary_layout() || B.arbitrary_layout() ||
        C.arbitrary_layout())
        return false;
    trace::Block tb("eig_product");
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    LocalBlock<T> la = A.local(loc, false), lbk = B.local(loc, false), lc = C.local(loc, true);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    const int64_t k = opA == Op::NoTrans ? A.n() : A.m();
    lb::gemm(c, opA, Op::NoTrans, C.m(), C.n(), k, T(1), la.ptr, la.ld, lbk.ptr, lbk.ld, T(0), lc.ptr, lc.ld);
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    internal::finish_origin(C, opts);
    return true;
}

template <typename Host, typename Dev>
void overlapped(bool on, Host&& host_work, Dev&& dev_work) {
    if (!on) { host_work(); return; }
    std::exception_ptr err;
    // one core less for the chase's OpenMP team: this thread keeps issuing
    // and waiting on device work, and an oversubscribed team of spin-waiting
    // pipeline threads slowed hb2st 473 -> 580 ms
    const int nth = std::max(1, omp_get_max_threads() - 1);
    std::thread th([&] {
        try {
            omp_set_num_threads(nth);
            host_work();
        } catch (...) { err = std::current_exception(); }
    });
    try {
        dev_work();
    } catch (...) {
        th.join();
        throw;
    }
    th.join();
    if (err) std::rethrow_exception(err);
}

/// Broadcast a host vector from `root` (size first: the other ranks may not
/// know it).
template <typename X>
void bcast_vec(Comm& w, std::vector<X>& v, int root) {
    int64_t sz = int64_t(v.size());
    w.bcast(&sz, 1, root, Loc::Host, nullptr);
    v.resize(size_t(sz));
    if (sz > 0) w.bcast(v.data(), size_t(sz), root, Loc::Host, nullptr);
}

/// Stage-2 results of one rank to all (reference heev.cc:128-140 / svd.cc run
/// hb2st / tb2bd on one rank and broadcast): the bulge chase is a host
/// pipeline that uses every core of the node, so running it once instead of
/// on every rank of the node at the same time (each with its own thread
/// team) stops the ranks from competing for the cores.
template <typename T>
void bcast_reflectors(Comm& w, host::Reflectors<T>& Q, int root) {
    bcast_vec(w, Q.off, root);
    bcast_vec(w, Q.len, root);
    bcast_vec(w, Q.voff, root);
    bcast_vec(w, Q.tag, root);
    bcast_vec(w, Q.tau, root);
    bcast_vec(w, Q.v, root);
}

/// he2hb on one process: the same per-panel steps as the distributed loop
/// below (panel QR, W = A22 V, the WY correction, her2k), but as local
/// lb:: calls on one stream into preallocated buffers, with no driver, no
/// scheduler and no host wait per panel.  The driver form paid a geqrf call
/// (scheduler, T-matrix allocation, panel-error check) plus a V / W matrix
/// allocation per panel: geqrf 168 of he2hb's 266 ms at n = 8192, nb = 256,
/// for panel kernels worth 8 ms.  SLATE_HE2HB_LOCAL=0 keeps the driver form.
template <typename T>
bool he2hb_local(Matrix<T>& A, std::vector<TriangularFactors<T>>& Ts, Options const& opts) {
    static const bool env = [] {
        const char* e = std::getenv("SLATE_HE2HB_LOCAL");
        return e ? std::atoi(e) != 0 : true;
    }();
    auto gA = A.grid();
    if (!env || gA->size() != 1 || A.mb() != A.nb() || A.arbitrary_layout() || A.op() != Op::NoTrans) return false;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    const int64_t nt = A.nt(), n = A.n(), nb = A.nb();
    Ts.assign(std::max<int64_t>(nt - 1, 0), {});
    if (nt < 2) return true;
    LocalBlock<T> la = A.local(loc, true);
    T* a = la.ptr;
    const int64_t lda = la.ld;
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    const int64_t mmax = std::max<int64_t>(n - A.tileNb(0), 1);
    Work<T> V(target, size_t(mmax) * nb), W(target, size_t(mmax) * nb), X(target, size_t(nb) * nb), tau(target, size_t(nb));
    int64_t r0 = 0;
    for (int64_t k = 0; k + 1 < nt; ++k) {
        const int64_t kb = A.tileNb(k);
        const int64_t c0 = r0;
        r0 += kb;
        const int64_t m = n - r0;
        Matrix<T> Tf(nb, std::max<int64_t>(kb, 1), nb, nb, Grid::self());
        Tf.insertLocalTiles(target);
        LocalBlock<T> lt = Tf.local(loc, true);
        T* P = a + r0 + c0 * lda;
        T* A22 = a + r0 + r0 * lda;
        // all of T zero first: the host panel writes only its min(m, kb)
        // square, and a ragged last panel (m < kb) multiplies the rest
        lb::set(c, Uplo::General, nb, std::max<int64_t>(kb, 1), T(0), T(0), lt.ptr, lt.ld);
        lb::geqrf_panel(c, m, kb, P, lda, tau.data(), lt.ptr, lt.ld);
        // explicit unit-lower V
        lb::copy2d(c, m, kb, P, lda, V.data(), m);
        lb::set(c, Uplo::Upper, std::min(m, kb), kb, T(0), T(1), V.data(), m);
        // W = A22 V T,  W -= V (T^H V^H W) / 2,  A22 -= V W^H + W V^H
        lb::hemm(c, Side::Left, Uplo::Lower, m, kb, T(1), A22, lda, V.data(), m, T(0), W.data(), m);
        lb::trmm(c, Side::Right, Uplo::Upper, Op::NoTrans, Diag::NonUnit, m, kb, T(1), lt.ptr, lt.ld, W.data(), m);
        lb::gemm(c, Op::ConjTrans, Op::NoTrans, kb, kb, m, T(1), V.data(), m, W.data(), m, T(0), X.data(), kb);
        lb::trmm(c, Side::Left, Uplo::Upper, Op::ConjTrans, Diag::NonUnit, kb, kb, T(1), lt.ptr, lt.ld, X.data(), kb);
        lb::gemm(c, Op::NoTrans, Op::NoTrans, m, kb, kb, T(-0.5), V.data(), m, X.data(), kb, T(1), W.data(), m);
        lb::her2k(c, Uplo::Lower, Op::NoTrans, m, kb, T(-1), V.data(), m, W.data(), m, real_type<T>(1), A22, lda);
        Ts[k].push_back(Tf);
    }
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    return true;
}

/// ge2tb on one process, as he2hb_local: per block column the QR panel
/// (geqrf_panel), Q^H on the columns to its right (larfb), the LQ panel of the
/// block row as QR of its conjugate transpose (gelqf's own convention: row =
/// Y^H, T_k at column 0 of an nb x (n1 + nb) T matrix), and H on the rows
/// below (larfb from the right) -- local calls on one stream instead of a
/// geqrf / unmqr / gelqf / unmlq driver call per panel (ge2tb ~470 of the
/// n = 8192 svd's 3.4 s, for ~1.5 TFLOP).  SLATE_GE2TB_LOCAL=0: driver form.
template <typename T>
bool ge2tb_local(Matrix<T>& A, std::vector<TriangularFactors<T>>& TU, std::vector<TriangularFactors<T>>& TV,
                 Options const& opts) {
    static const bool env = [] {
        const char* e = std::getenv("SLATE_GE2TB_LOCAL");
        return e ? std::atoi(e) != 0 : true;
    }();
    auto gA = A.grid();
    if (!env || gA->size() != 1 || A.mb() != A.nb() || A.arbitrary_layout() || A.op() != Op::NoTrans) return false;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    const int64_t nt = A.nt(), M = A.m(), N = A.n(), nb = A.nb();
    TU.assign(nt, {});
    TV.assign(std::max<int64_t>(nt - 1, 0), {});
    LocalBlock<T> la = A.local(loc, true);
    T* a = la.ptr;
    const int64_t lda = la.ld;
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    Work<T> Y(target, size_t(std::max<int64_t>(N, 1)) * nb), tau(target, size_t(nb));
    int64_t r0 = 0;
    for (int64_t k = 0; k < nt; ++k) {
        const int64_t kb = A.tileNb(k), m = M - r0;
        Matrix<T> Tq(nb, std::max<int64_t>(kb, 1), nb, nb, Grid::self());
        Tq.insertLocalTiles(target);
        LocalBlock<T> lq = Tq.local(loc, true);
        T* P = a + r0 + r0 * lda;
        lb::set(c, Uplo::General, nb, std::max<int64_t>(kb, 1), T(0), T(0), lq.ptr, lq.ld);
        if (m > 0) lb::geqrf_panel(c, m, kb, P, lda, tau.data(), lq.ptr, lq.ld);
        TU[k].push_back(Tq);
        const int64_t c1 = r0 + kb, n1 = N - c1;
        if (k + 1 < nt && n1 > 0) {
            if (m > 0)
                lb::larfb(c, Side::Left, Op::ConjTrans, m, n1, kb, P, lda, lq.ptr, lq.ld, a + r0 + c1 * lda, lda);
            Matrix<T> Tl(nb, n1 + nb, nb, nb, Grid::self());
            Tl.insertLocalTiles(target);
            LocalBlock<T> ll = Tl.local(loc, true);
            lb::set(c, Uplo::General, nb, n1 + nb, T(0), T(0), ll.ptr, ll.ld);
            T* rp = a + r0 + c1 * lda;
            const int64_t kr = std::min<int64_t>(kb, m);   // rows of the row panel
            if (kr > 0) {
                lb::copy<T, T>(c, Uplo::General, Op::ConjTrans, n1, kr, rp, lda, Y.data(), n1);
                lb::geqrf_panel(c, n1, kr, Y.data(), n1, tau.data(), ll.ptr, ll.ld);
                lb::copy<T, T>(c, Uplo::General, Op::ConjTrans, kr, n1, Y.data(), n1, rp, lda);
                const int64_t mr = M - c1;   // rows below the row panel
                if (mr > 0)
                    lb::larfb(c, Side::Right, Op::NoTrans, mr, n1, kr, Y.data(), n1, ll.ptr, ll.ld, a + c1 + c1 * lda,
                              lda);
            }
            TV[k].push_back(Tl);
        }
        r0 = c1;
    }
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    return true;
}

}  // namespace

//------------------------------------------------------------------------------
/// he2hb: A (Hermitian, lower triangle referenced) -> band of width nb; the
/// reflectors stay below the band, their T factors in Ts.  Per block column
/// (reference src/he2hb.cc:401-572): geqrf of the panel, then the two-sided
/// update A22 := Q^H A22 Q as  W = A22 V T  (hemm),  Y = W - V (T^H V^H W)/2
/// (local, one column all-reduce of the nb x nb V^H W),  A22 -= V Y^H + Y V^H
/// (her2k on the lower triangle only) -- half the flops of applying Q from
/// both sides to the full square.
template <typename T>
void he2hb(Matrix<T>& A, std::vector<TriangularFactors<T>>& Ts, Options const& opts) {
    trace::Block tb("he2hb");
    internal::DriverScope ds_;
    if (he2hb_local(A, Ts, opts)) return;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    const int64_t nt = A.nt();
    auto gA = A.grid();
    Ts.assign(std::max<int64_t>(nt - 1, 0), {});
    for (int64_t k = 0; k + 1 < nt; ++k) {
        Matrix<T> panel = A.sub(k + 1, nt - 1, k, k);
        geqrf(panel, Ts[k], opts);
        const int64_t m = panel.m(), kb = panel.n();
        // explicit unit-lower V on the panel's layout
        Matrix<T> V(m, kb, A.mb(), kb, gA, panel.srow_owner(0), panel.scol_owner(0));
        V.insertLocalTiles(target);
        slate::copy<T, T>(panel, V, opts);
        {
            TrapezoidMatrix<T> V0(Uplo::Upper, Diag::NonUnit, V.sub(0, 0, 0, 0));
            set(T(0), T(1), V0, opts);
        }
        HermitianMatrix<T> A22(Uplo::Lower, A.sub(k + 1, nt - 1, k + 1, nt - 1));
        Matrix<T> W = V.emptyLike();
        W.insertLocalTiles(target);
        hemm(Side::Left, T(1), A22, V, T(0), W, opts);
        {
            trace::Block t2("he2hb_wy");
            LocalBlock<T> lv = V.local(loc, false), lw = W.local(loc, true);
            LocalBlock<T> lt = Ts[k][0].local(loc, false);
            if (lw.n > 0) {
                lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
                Work<T> X(target, size_t(kb) * kb);
                lb::trmm(c, Side::Right, Uplo::Upper, Op::NoTrans, Diag::NonUnit, lw.m, kb, T(1), lt.ptr, lt.ld,
                         lw.ptr, lw.ld);
                if (lw.m > 0)
                    lb::gemm(c, Op::ConjTrans, Op::NoTrans, kb, kb, lw.m, T(1), lv.ptr, lv.ld, lw.ptr, lw.ld, T(0),
                             X.data(), kb);
                else
                    lb::set(c, Uplo::General, kb, kb, T(0), T(0), X.data(), kb);
                if (gA->col().size() > 1)
                    gA->col().allreduce(X.data(), size_t(kb) * kb, ReduceOp::Sum, loc, c.stream);
                lb::trmm(c, Side::Left, Uplo::Upper, Op::ConjTrans, Diag::NonUnit, kb, kb, T(1), lt.ptr, lt.ld,
                         X.data(), kb);
                if (lw.m > 0)
                    lb::gemm(c, Op::NoTrans, Op::NoTrans, lw.m, kb, kb, T(-0.5), lv.ptr, lv.ld, X.data(), kb, T(1),
                             lw.ptr, lw.ld);
                if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
            }
            W.storage()->modified(loc);
        }
        her2k(T(-1), V, W, real_type<T>(1), A22, opts);
    }
}

/// Z := Q2 Z on the device for the hb2st reflectors (reference
/// unmtr_hb2st.cc).  The reflectors of GS consecutive sweeps J GS .. J GS +
/// GS - 1 at the same bulge step t act on rows r0 + i .. r0 + i + kd - 1
/// (r0 = J GS + t kd + 1, i = sweep - J GS): one (GS + kd) x GS block V with
/// H_{J GS} ... H_{J GS + GS - 1} = I - V T V^H.  Reflector (j, t) only has to
/// precede the overlapping (j + d, t) and (j + d, t - 1), (j + d, t - 2) of
/// later sweeps, and two reflectors of one sweep touch disjoint rows, so Q2 is
/// the product over J ascending, t DEScending of the blocks, and Z is updated
/// for J descending, t ascending:  W = V^H Z_r,  W := T W (triangular solve
/// with T^{-1} = striu(V^H V) + diag(1/tau)),  Z_r -= V W.  GS = 4 kd keeps
/// the GEMMs large (about 2 n^2 / (GS kd) blocks).  Z holds all n rows of its
/// columns (1-D column layout).  Host and device run the same blocked
/// sequence (lb:: dispatch), so the CPU tests check the ordering.
/// fp64 on the device: the same product through the fused kernels of
/// hb2st_apply.hip -- groups of 64 reflectors (64 consecutive sweeps at one
/// bulge step, so V is a 128 x 64 parallelogram kept compact), T per group by
/// one wave, and one workgroup per column slice of Z walking the groups in
/// order (no per-group launches, no dense zero blocks).  Groups are packed on
/// the host into pinned chunks that upload while the previous chunk applies.
/// SLATE_HB2ST_FUSED=0 keeps the blocked GEMM sequence.
/// bc != nullptr: only rank 0 of bc holds Q (Qp); it packs each chunk and
/// the chunk travels to the other ranks' device buffers by one broadcast, so
/// no other rank keeps the O(n^2) reflectors on its host.  Every rank of bc
/// calls this (ncols may be 0).
void unmtr_hb2st_fused(host::Reflectors<double> const* Qp, int64_t n, int64_t kd, double* Z, int64_t ldz,
                       int64_t ncols, lb::Ctx const& c, Comm* bc = nullptr) {
    trace::Block tb("unmtr_hb2st_fused");
    constexpr int64_t HB = 64;
    const bool root = !bc || bc->rank() == 0;
    std::map<std::pair<int64_t, int64_t>, std::vector<size_t>> groups;
    std::vector<std::pair<int64_t, int64_t>> keys;
    if (root) {
        host::Reflectors<double> const& Q = *Qp;
        for (size_t r = 0; r < Q.size(); ++r) {
            const int64_t j = Q.tag[r];
            slate_assert(j >= 0);
            groups[{j / HB, (Q.off[r] - j - 1) / kd}].push_back(r);
        }
        for (auto& kv : groups) keys.push_back(kv.first);
        std::sort(keys.begin(), keys.end(), [](auto const& a, auto const& b) {
            return a.first != b.first ? a.first > b.first : a.second < b.second;
        });
    }
    int64_t ng = int64_t(keys.size());
    const int64_t CG = 512;
    if (bc && bc->size() > 1) bc->bcast(&ng, 1, 0, Loc::Host, nullptr);
    const size_t vsz = size_t(CG) * HB * HB, tsz = size_t(CG) * HB;
    // one pinned staging block per buffer: V | tau | R0
    const size_t bytes = (vsz + tsz) * sizeof(double) + size_t(CG) * sizeof(int64_t);
    void* hbuf[2] = {device::malloc_host(bytes), device::malloc_host(bytes)};
    void* dbuf[2] = {device::malloc(bytes), device::malloc(bytes)};
    double* dT[2] = {static_cast<double*>(device::malloc(vsz * sizeof(double))),
                     static_cast<double*>(device::malloc(vsz * sizeof(double)))};
    hipEvent_t ev[2] = {device::event_get(), device::event_get()};
    for (int b = 0; b < 2; ++b) slate_hip_call(hipEventRecord(ev[b], c.stream));
    int cur = 0;
    for (int64_t g0 = 0; g0 < ng; g0 += CG) {
        const int64_t nc = std::min(CG, ng - g0);
        slate_hip_call(hipEventSynchronize(ev[cur]));   // buffers of two chunks ago are free
        double* hV = static_cast<double*>(hbuf[cur]);
        double* htau = hV + vsz;
        int64_t* hR0 = reinterpret_cast<int64_t*>(htau + tsz);
        double* dV = static_cast<double*>(dbuf[cur]);
        double* dtau = dV + vsz;
        int64_t* dR0 = reinterpret_cast<int64_t*>(dtau + tsz);
        if (root) {
        host::Reflectors<double> const& Q = *Qp;
        #pragma omp parallel for schedule(dynamic, 8)
        for (int64_t bi = 0; bi < nc; ++bi) {
            const auto key = keys[size_t(g0 + bi)];
            const int64_t J = key.first, t = key.second, r0 = J * HB + t * kd + 1;
            double* Vg = hV + size_t(bi) * HB * HB;
            std::fill(Vg, Vg + HB * HB, 0.0);
            std::fill(htau + bi * HB, htau + (bi + 1) * HB, 0.0);
            hR0[bi] = r0;
            for (size_t r : groups.at(key)) {
                const int64_t i = Q.tag[r] - J * HB;
                slate_assert(Q.off[r] - r0 == i && Q.len[r] <= HB);
                std::copy(Q.v.data() + Q.voff[r], Q.v.data() + Q.voff[r] + Q.len[r], Vg + i * HB);
                htau[bi * HB + i] = Q.tau[r];
            }
        }
        device::memcpy_async(dV, hV, size_t(nc) * HB * HB * sizeof(double), c.stream);
        device::memcpy_async(dtau, htau, size_t(nc) * HB * sizeof(double), c.stream);
        device::memcpy_async(dR0, hR0, size_t(nc) * sizeof(int64_t), c.stream);
        }
        if (bc && bc->size() > 1) {
            // the packed chunk (V | tau | R0, contiguous) to every rank
            bc->bcast(dbuf[cur], bytes, ScalarType::Byte, 0, Loc::Device, c.stream);
        }
        if (ncols > 0) slate_amd::dev::hb2st_tfac(nc, dV, dtau, dT[cur], c.stream);
        slate_amd::dev::hb2st_apply(nc, dR0, dV, dT[cur], Z, ldz, n, ncols, c.stream);
        slate_hip_call(hipEventRecord(ev[cur], c.stream));
        cur ^= 1;
    }
    slate_hip_call(hipStreamSynchronize(c.stream));
    for (int b = 0; b < 2; ++b) {
        device::event_put(ev[b]);
        device::free_host(hbuf[b]);
        device::free(dbuf[b]);
        device::free(dT[b]);
    }
}

/// Band width of the two-stage reductions: at most 64 (SLATE_EIG_KD lowers
/// it: the host bulge chase costs O(n^2 kd) with a pipeline chain of
/// O(n kd^2), the first stage prefers wide panels).
int64_t eig_band_width() {
    static const int64_t kd = [] {
        const char* e = std::getenv("SLATE_EIG_KD");
        const int64_t v = e ? std::atoll(e) : 64;
        return std::max<int64_t>(8, std::min<int64_t>(v, 64));
    }();
    return kd;
}

bool hb2st_fused_enabled() {
    static const bool fused = [] {
        const char* e = std::getenv("SLATE_HB2ST_FUSED");
        return !e || std::atoi(e) != 0;
    }();
    return fused;
}

/// Do the stage-2 reflectors stay on rank 0 and stream to the others in
/// packed device chunks (fp64, device, fused kernels, more than one rank)?
template <typename T>
bool stage2_streamed(Target target, int64_t kd, Comm& w) {
    return std::is_same<T, double>::value && target == Target::Devices && hb2st_fused_enabled() && kd <= 64 &&
           w.size() > 1;
}

template <typename T>
void unmtr_hb2st_blocked(host::Reflectors<T> const& Q, int64_t n, int64_t kd, T* Z, int64_t ldz, int64_t ncols,
                        lb::Ctx const& c);

/// Stage-2 back-transform of this rank's columns; every rank calls it.
/// streamed: Q is on rank 0 of w only (stage2_streamed).
template <typename T>
void stage2_apply(host::Reflectors<T> const& Q, bool streamed, int64_t n, int64_t kd, T* Z, int64_t ldz,
                  int64_t ncols, lb::Ctx const& c, Comm& w) {
    if constexpr (std::is_same<T, double>::value) {
        if (streamed) {
            unmtr_hb2st_fused(w.rank() == 0 ? &Q : nullptr, n, kd, Z, ldz, ncols, c, &w);
            return;
        }
    }
    if (ncols > 0) unmtr_hb2st_blocked(Q, n, kd, Z, ldz, ncols, c);
}

template <typename T>
void unmtr_hb2st_blocked(host::Reflectors<T> const& Q, int64_t n, int64_t kd, T* Z, int64_t ldz, int64_t ncols,
                        lb::Ctx const& c) {
    namespace kd_ = slate_amd::dev;
    if (Q.size() == 0 || ncols <= 0) return;
    if constexpr (std::is_same<T, double>::value) {
        if (c.dev() && hb2st_fused_enabled() && kd <= 64) {
            unmtr_hb2st_fused(&Q, n, kd, Z, ldz, ncols, c);
            return;
        }
    }
    trace::Block tb("unmtr_hb2st_blocked");
    const int64_t GS = 4 * kd;
    std::map<std::pair<int64_t, int64_t>, std::vector<size_t>> groups;
    for (size_t r = 0; r < Q.size(); ++r) {
        const int64_t j = Q.tag[r];
        slate_assert(j >= 0);
        groups[{j / GS, (Q.off[r] - j - 1) / kd}].push_back(r);
    }
    std::vector<std::pair<int64_t, int64_t>> keys;
    for (auto& kv : groups) keys.push_back(kv.first);
    std::sort(keys.begin(), keys.end(), [](auto const& a, auto const& b) {
        return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    const int64_t vr = GS + kd, VB = vr * GS;
    const size_t ng = keys.size();
    // blocks are staged in batches of at most kBatch groups (pinned host,
    // double-buffered device copies): bounded host memory instead of the
    // whole blocked Q2
    const size_t kBatch = 64;
    const Target tg = c.dev() ? Target::Devices : Target::HostTask;
    Work<T> G(tg, size_t(GS) * GS), W(tg, size_t(GS) * ncols);
    auto tinv = [&](int64_t w, T* Gm, T const* tau) {
        if (c.dev()) { kd_::tinv_from_gram(w, kd_::dptr(Gm), GS, kd_::dptr(tau), c.stream); return; }
        for (int64_t j = 0; j < w; ++j)
            for (int64_t i = 0; i < w; ++i) {
                T& x = Gm[i + j * GS];
                if (i > j) x = T(0);
                else if (i == j) x = tau[i] == T(0) ? T(1) : T(1) / tau[i];
            }
    };
    std::vector<T> hVb(kBatch * VB), htb(kBatch * GS);
    Work<T> dV[2], dtv[2];
    hipEvent_t ev[2] = {nullptr, nullptr};
    if (c.dev())
        for (int b = 0; b < 2; ++b) {
            dV[b].resize(tg, hVb.size());
            dtv[b].resize(tg, htb.size());
            ev[b] = device::event_get();
            slate_hip_call(hipEventRecord(ev[b], c.stream));
        }
    std::vector<int64_t> r0s(kBatch), ws(kBatch);
    int cur = 0;
    for (size_t g0 = 0; g0 < ng; g0 += kBatch) {
        const size_t nbat = std::min(kBatch, ng - g0);
        // the device buffer about to be refilled must be free (its last use
        // was two batches ago)
        if (c.dev()) slate_hip_call(hipEventSynchronize(ev[cur]));
        std::fill(hVb.begin(), hVb.end(), T(0));
        std::fill(htb.begin(), htb.end(), T(0));
        #pragma omp parallel for schedule(dynamic)
        for (size_t bi = 0; bi < nbat; ++bi) {
            const size_t gi = g0 + bi;
            const int64_t J = keys[gi].first, t = keys[gi].second, r0 = J * GS + t * kd + 1;
            r0s[bi] = r0;
            int64_t w = 0;
            for (size_t r : groups.at(keys[gi])) {
                const int64_t i = Q.tag[r] - J * GS;
                slate_assert(Q.off[r] - r0 == i && i + Q.len[r] <= vr);
                T const* v = Q.v.data() + Q.voff[r];
                for (int64_t ii = 0; ii < Q.len[r]; ++ii) hVb[bi * VB + (i + ii) + i * vr] = v[ii];
                htb[bi * GS + i] = Q.tau[r];
                w = std::max(w, i + 1);
            }
            ws[bi] = w;
        }
        T const* Vall = hVb.data();
        T const* tall = htb.data();
        if (c.dev()) {
            device::memcpy_async(dV[cur].data(), hVb.data(), nbat * VB * sizeof(T), c.stream);
            device::memcpy_async(dtv[cur].data(), htb.data(), nbat * GS * sizeof(T), c.stream);
            Vall = dV[cur].data();
            tall = dtv[cur].data();
        }
        for (size_t bi = 0; bi < nbat; ++bi) {
            const int64_t r0 = r0s[bi], w = ws[bi];                 // w: columns in use
            const int64_t rows = std::min(w - 1 + kd, n - r0);
            if (rows <= 0 || w <= 0) continue;
            T const* V = Vall + bi * VB;
            T* Zr = Z + r0;
            lb::gemm(c, Op::ConjTrans, Op::NoTrans, w, w, rows, T(1), V, vr, V, vr, T(0), G.data(), GS);
            tinv(w, G.data(), tall + bi * GS);
            lb::gemm(c, Op::ConjTrans, Op::NoTrans, w, ncols, rows, T(1), V, vr, Zr, ldz, T(0), W.data(), GS);
            lb::trsm(c, Side::Left, Uplo::Upper, Op::NoTrans, Diag::NonUnit, w, ncols, T(1), G.data(), GS, W.data(), GS);
            lb::gemm(c, Op::NoTrans, Op::NoTrans, rows, ncols, w, T(-1), V, vr, W.data(), GS, T(1), Zr, ldz);
        }
        if (c.dev()) {
            // the host staging buffer is reused next batch: wait for the upload
            slate_hip_call(hipEventRecord(ev[cur], c.stream));
            slate_hip_call(hipStreamSynchronize(c.stream));
            cur ^= 1;
        }
    }
    if (c.dev()) {
        slate_hip_call(hipStreamSynchronize(c.stream));
        for (int b = 0; b < 2; ++b) device::event_put(ev[b]);
    }
}

/// Local rows of a P x 1 row-layout n x n matrix set to diag(dg): zero fill,
/// then each local tile's diagonal run written with one strided copy
/// (O(n) host memory).
template <typename T>
void set_diag_rows(Matrix<T>& M, std::vector<T> const& dg, Target target) {
    Options o = {{Option::Target, target}};
    set(T(0), T(0), M, o);
    const Loc loc = loc_of(target);
    LocalBlock<T> lm = M.local(loc, true);
    if (lm.m == 0) return;
    hipStream_t st = target == Target::Devices ? device::queue(0) : nullptr;
    for (int64_t i = 0; i < M.mt(); ++i) {
        if (M.srow_owner(i) != M.grid()->myrow()) continue;
        const int64_t lr = lrow_of(M, i), gr = grow_of(M, i), mb = M.tileMb(i);
        T* dst = lm.ptr + lr + gr * lm.ld;
        if (target == Target::Devices)
            device::memcpy2d_async(dst, (lm.ld + 1) * sizeof(T), dg.data() + gr, sizeof(T), sizeof(T), mb, st);
        else
            for (int64_t ii = 0; ii < mb; ++ii) dst[ii * (lm.ld + 1)] = dg[gr + ii];
    }
    if (st) slate_hip_call(hipStreamSynchronize(st));
}

namespace {

/// Range guard shared by heev and svd (reference heev.cc:73-102, svd.cc:85-125):
/// returns the factor alpha the matrix was scaled to (1 if untouched) and sets
/// `bad` when ||A||_max is NaN or Inf.  A matrix with ||A||_max below
/// sqrt(safe_min / eps) or above its reciprocal is scaled by alpha / ||A||_max,
/// so the reductions neither underflow nor overflow; the caller rescales the
/// eigen / singular values by ||A||_max / alpha afterwards.
template <typename R>
R range_alpha(R anorm, bool& bad) {
    const R sml = std::numeric_limits<R>::min() / std::numeric_limits<R>::epsilon();
    const R sqrt_sml = std::sqrt(sml), sqrt_big = R(1) / sqrt_sml;
    bad = std::isnan(anorm) || std::isinf(anorm);
    if (bad) return R(1);
    if (anorm > R(0) && anorm < sqrt_sml) return sqrt_sml;
    if (anorm > sqrt_big) return sqrt_big;
    return R(1);
}

template <typename R>
void rescale_values(std::vector<R>& v, R anorm, R alpha) {
    if (alpha == R(1)) return;
    for (auto& x : v) x = x / alpha * anorm;   // divide first: x / alpha stays in range
}

}  // namespace

template <typename T>
void heev(HermitianMatrix<T>& A, std::vector<real_type<T>>& Lambda, Matrix<T>& Z, Options const& opts) {
    {   // multi-device A (and Z): on its devices
        bool ran = internal::spread<T>(opts, {{&A, true}, {&Z, true}}, [&](std::vector<Matrix<T>>& M, int r) {
            auto H = internal::rewrap(A, M[0]);
            std::vector<real_type<T>> L;
            heev(H, L, M[1], opts);
            if (r == 0) Lambda.swap(L);
        }, false);
        if (ran) return;
    }
    if (A.arbitrary_layout() || Z.arbitrary_layout()) {
        HermitianMatrix<T> Ab(A.uplo(), bc_operand(A, opts));
        Matrix<T> Zb = wanted(Z) ? block_cyclic(Z, opts) : Z;
        heev(Ab, Lambda, Zb, opts);
        if (wanted(Z)) slate::copy<T, T>(Zb, Z, opts);
        return;
    }
    trace::Block tb("heev");
    internal::DriverScope ds_;
    using R = real_type<T>;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    const int64_t n = A.n();
    Lambda.assign(n, R(0));
    if (n == 0) return;
    // range guard (reference heev.cc:73-102): the scaled copy F is reduced,
    // Lambda is rescaled at the end; eigenvectors are scale-invariant
    const R anorm = slate::norm(Norm::Max, A, opts);
    bool bad = false;
    const R alpha = range_alpha(anorm, bad);
    if (bad) { Lambda.assign(n, anorm); return; }
    // band width of the two-stage reduction: the bulge chase costs O(n^2 kd)
    // on the host, the first stage is memory-bound either way, so large tiles
    // are re-tiled to kd <= 64 (reference uses the tile size)
    const int64_t kd = std::min<int64_t>(A.nb(), eig_band_width());
    auto gA = A.grid();
    Matrix<T> F(n, n, kd, kd, gA);
    F.insertLocalTiles(target);
    {
        Matrix<T> Ag(A);
        Ag.set_uplo(Uplo::General);
        BaseTrapezoidMatrix<T> At(A.uplo(), Ag, MatrixKind::Trapezoid);
        BaseTrapezoidMatrix<T> Fl(Uplo::Lower, F, MatrixKind::Trapezoid);
        if (A.uplo() == Uplo::Lower) slate::copy<T, T>(At, Fl, opts);
        else slate::copy<T, T>(conj_transpose(Ag), F, opts);   // upper: mirror into the lower triangle
    }
    if (alpha != R(1)) scale(alpha, anorm, F, opts);
    const int64_t nt = F.nt();
    std::vector<TriangularFactors<T>> Ts;
    he2hb(F, Ts, opts);
    // stage 2 on the host: band (lower, width kd) -> tridiagonal, in band
    // storage (the bulge chase stays within 2 kd of the diagonal)
    std::vector<T> B = gather_band(F, kd, 2 * kd, true, true, opts);
    std::vector<R> d, e;
    host::Reflectors<T> Q2;
    std::vector<T> phase;
    const bool ovl = wanted(Z) && eig_overlap(target, false) && nt >= 2;
    Matrix<T> Q1x;   // explicit stage-1 Q (ovl)
    {
        trace::Block t2("hb2st");
        Comm& w = gA->world();
        overlapped(ovl, [&] { if (w.rank() == 0) host::hb2st<T>(n, kd, B.data() + 2 * kd, 4 * kd, d, e, Q2, phase); },
                   [&] {
                       trace::Block t3("unmtr_he2hb_form");
                       Q1x = Matrix<T>(n, n, kd, kd, gA);
                       Q1x.insertLocalTiles(target);
                       set(T(0), T(1), Q1x, opts);
                       Matrix<T> P = F.sub(1, nt - 1, 0, nt - 2);
                       Matrix<T> Qs = Q1x.sub(1, nt - 1, 0, nt - 1);
                       unmqr(Side::Left, Op::NoTrans, P, stacked_T(Ts, nt - 1, F.nb(), P.n(), opts), Qs, opts);
                   });
        if (w.size() > 1) {
            bcast_vec(w, d, 0);
            bcast_vec(w, e, 0);
            bcast_vec(w, phase, 0);
            if (wanted(Z) && !stage2_streamed<T>(target, kd, w)) bcast_reflectors(w, Q2, 0);
        }
    }
    B.clear(); B.shrink_to_fit();
    if (!wanted(Z)) {
        trace::Block t2("sterf");
        host::sterf<R>(n, d.data(), e.data());
        Lambda = d;
        rescale_values(Lambda, anorm, alpha);
        return;
    }
    const int64_t me = get_option<int64_t>(opts, Option::MethodEig, int64_t(MethodEig::DC));
    const bool use_qr = (me == int64_t(MethodEig::QR) || me == 'q');
    // tridiagonal eigenvectors, distributed on A's grid (no n x n host array):
    // divide and conquer with the merges as distributed GEMMs, or QL with the
    // rotations applied to each rank's rows (eig_dist.cc)
    const int64_t nbq = std::max<int64_t>(kd, std::min<int64_t>(A.nb(), 512));
    Matrix<R> Qt(n, n, nbq, nbq, gA);
    Qt.insertLocalTiles(target);
    {
        trace::Block t2("tridiag_eig");
        if (use_qr) {
            set(R(0), R(1), Qt, opts);
            steqr2_dist<R>(d, e, Qt, opts);
        } else {
            stedc_dist<R>(d, e, Qt, opts);
        }
    }
    Lambda = d;
    rescale_values(Lambda, anorm, alpha);
    // Z1 (1-D column layout, kd-wide column tiles): diag(phase) Qt, then Q2
    // applied to all rows of my columns
    Matrix<T> Z1(n, n, n, kd, row_grid(gA));
    Z1.insertLocalTiles(target);
    {
        trace::Block t2("unmtr_hb2st");
        Matrix<R> Q1(n, n, n, kd, row_grid(gA));
        Q1.insertLocalTiles(target);
        slate::copy<R, R>(Qt, Q1, opts);
        Qt = Matrix<R>();
        LocalBlock<R> lq = Q1.local(loc, false);
        LocalBlock<T> lz = Z1.local(loc, true);
        lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
        if (lz.n > 0) {
            if (c.dev()) {
                Work<T> dph(Target::Devices, size_t(n));
                device::memcpy_async(dph.data(), phase.data(), n * sizeof(T), c.stream);
                slate_amd::dev::real_rowscale(n, lz.n, lq.ptr, lq.ld, slate_amd::dev::dptr(dph.data()),
                                              slate_amd::dev::dptr(lz.ptr), lz.ld, c.stream);
                slate_hip_call(hipStreamSynchronize(c.stream));
            } else {
                for (int64_t j = 0; j < lz.n; ++j)
                    for (int64_t i = 0; i < n; ++i) lz.ptr[i + j * lz.ld] = phase[i] * T(lq.ptr[i + j * lq.ld]);
            }
        }
        Comm& w = gA->world();
        stage2_apply(Q2, stage2_streamed<T>(target, kd, w), n, kd, lz.ptr, lz.ld, lz.n, c, w);
    }
    // stage-1 back-transform (unmtr_he2hb) on F's layout, then into Z
    if (ovl) {
        trace::Block t3("unmtr_he2hb_gemm");
        if (local_product(Op::NoTrans, Q1x, Z1, Z, opts)) return;
        Matrix<T> Zw(n, n, kd, kd, gA), Zo(n, n, kd, kd, gA);
        Zw.insertLocalTiles(target);
        Zo.insertLocalTiles(target);
        slate::copy<T, T>(Z1, Zw, opts);
        gemm(T(1), Q1x, Zw, T(0), Zo, opts);
        slate::copy<T, T>(Zo, Z, opts);
        return;
    }
    Matrix<T> Zw(n, n, kd, kd, gA);
    Zw.insertLocalTiles(target);
    slate::copy<T, T>(Z1, Zw, opts);
    {
        trace::Block t3("unmtr_he2hb");
        // panels F(k+1:, k), k = 0 .. nt-2, together: the QR-shaped view
        // F(1:, 0:nt-2) applied to Z(1:, :) in one call
        const int64_t znt = Zw.nt();
        if (nt >= 2) {
            Matrix<T> P = F.sub(1, nt - 1, 0, nt - 2);
            Matrix<T> Zs = Zw.sub(1, nt - 1, 0, znt - 1);
            unmqr(Side::Left, Op::NoTrans, P, stacked_T(Ts, nt - 1, F.nb(), P.n(), opts), Zs, opts);
        }
    }
    slate::copy<T, T>(Zw, Z, opts);
    (void)loc;
}

//------------------------------------------------------------------------------
/// Reduce the generalized problem to standard form with the Cholesky factor
/// in B (potrf output).  itype 1: A = L^{-1} A L^{-H} (or U^{-H} A U^{-1});
/// itype 2/3: A = L^H A L (or U A U^H).  Reference src/hegst.cc.
template <typename T>
void hegst(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T> const& B, Options const& opts) {
    trace::Block tb("hegst");
    internal::DriverScope ds_;
    slate_error_if_msg(itype < 1 || itype > 3, "hegst: itype must be 1, 2 or 3");
    Target target = resolve_target(opts);
    Matrix<T> F = hermitian_full(A, opts);
    Matrix<T> Bg(B);
    Bg.set_uplo(Uplo::General);
    const bool lower = (B.uplo() == Uplo::Lower);
    TriangularMatrix<T> L(B.uplo(), Diag::NonUnit, Bg);
    // work with the lower factor L: if B stores U (= L^H), use its conj-transpose
    TriangularMatrix<T> Lw = lower ? L : TriangularMatrix<T>(conj_transpose(L));
    if (itype == 1) {
        trsm(Side::Left, T(1), Lw, F, opts);                   // L^{-1} A
        trsm(Side::Right, T(1), conj_transpose(Lw), F, opts);  // ... L^{-H}
    } else {
        trmm(Side::Left, T(1), conj_transpose(Lw), F, opts);   // L^H A
        trmm(Side::Right, T(1), Lw, F, opts);                  // ... L
    }
    // write back A's triangle
    Matrix<T> Ag(A);
    Ag.set_uplo(Uplo::General);
    BaseTrapezoidMatrix<T> Ft(A.uplo(), F, MatrixKind::Trapezoid), At(A.uplo(), Ag, MatrixKind::Trapezoid);
    slate::copy<T, T>(Ft, At, opts);
    (void)target;
}

/// Generalized Hermitian-definite eigenproblem.  Reference src/hegv.cc.
template <typename T>
void hegv(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_type<T>>& Lambda,
          Matrix<T>& Z, Options const& opts) {
    trace::Block tb("hegv");
    internal::DriverScope ds_;
    int64_t info = potrf(B, opts);
    slate_error_if_msg(info != 0, "hegv: B is not positive definite");
    hegst(itype, A, B, opts);
    heev(A, Lambda, Z, opts);
    if (!wanted(Z)) return;
    Matrix<T> Bg(B);
    Bg.set_uplo(Uplo::General);
    TriangularMatrix<T> L(B.uplo(), Diag::NonUnit, Bg);
    TriangularMatrix<T> Lw = B.uplo() == Uplo::Lower ? L : TriangularMatrix<T>(conj_transpose(L));
    if (itype == 1 || itype == 2) trsm(Side::Left, T(1), conj_transpose(Lw), Z, opts);   // x = L^{-H} y
    else trmm(Side::Left, T(1), Lw, Z, opts);                                             // x = L y
}

//------------------------------------------------------------------------------
/// ge2tb: A (m >= n) -> upper band of width nb; Householder QR of each block
/// column, LQ of each block row.  Reference src/ge2tb.cc.
template <typename T>
void ge2tb(Matrix<T>& A, std::vector<TriangularFactors<T>>& TU, std::vector<TriangularFactors<T>>& TV,
           Options const& opts) {
    trace::Block tb("ge2tb");
    internal::DriverScope ds_;
    if (ge2tb_local(A, TU, TV, opts)) return;
    const int64_t mt = A.mt(), nt = A.nt();
    TU.assign(nt, {});
    TV.assign(std::max<int64_t>(nt - 1, 0), {});
    for (int64_t k = 0; k < nt; ++k) {
        Matrix<T> cp = A.sub(k, mt - 1, k, k);
        geqrf(cp, TU[k], opts);
        if (k + 1 < nt) {
            Matrix<T> A2 = A.sub(k, mt - 1, k + 1, nt - 1);
            unmqr(Side::Left, Op::ConjTrans, cp, TU[k], A2, opts);
            Matrix<T> rp = A.sub(k, k, k + 1, nt - 1);
            gelqf(rp, TV[k], opts);
            if (k + 1 < mt) {
                Matrix<T> A3 = A.sub(k + 1, mt - 1, k + 1, nt - 1);
                unmlq(Side::Right, Op::ConjTrans, rp, TV[k], A3, opts);
            }
        }
    }
}


template <typename T>
void svd_square(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Matrix<T>& U, Matrix<T>& VT, Options const& opts);

/// SVD A = U diag(Sigma) VT (thin: U m x k, VT k x n, k = min(m, n)).
/// Reference src/svd.cc: range scaling with a NaN / Inf guard, then
///   m > 5/3 n: QR pre-reduction, A = Q R, SVD of the n x n R, U = Q [U_R; 0];
///   n > m:     LQ pre-reduction, A = L Q, SVD of the m x m L, VT = [VT_L 0] Q;
///   otherwise  the three-stage ge2tb -> tb2bd -> bdsqr path on A itself.
/// The pre-reductions factor A in place (A is destroyed, as in the reference)
/// and never form a transposed copy of A.
template <typename T>
void svd(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Matrix<T>& U, Matrix<T>& VT, Options const& opts) {
    {
        bool ran = internal::spread<T>(opts, {{&A, true}, {&U, true}, {&VT, true}}, [&](std::vector<Matrix<T>>& M,
                                                                                          int r) {
            std::vector<real_type<T>> S;
            svd(M[0], S, M[1], M[2], opts);
            if (r == 0) Sigma.swap(S);
        }, false);
        if (ran) return;
    }
    if (A.arbitrary_layout() || U.arbitrary_layout() || VT.arbitrary_layout()) {
        Matrix<T> Ab = bc_operand(A, opts);
        Matrix<T> Ub = wanted(U) ? block_cyclic(U, opts) : U, Vb = wanted(VT) ? block_cyclic(VT, opts) : VT;
        svd(Ab, Sigma, Ub, Vb, opts);
        if (wanted(U)) slate::copy<T, T>(Ub, U, opts);
        if (wanted(VT)) slate::copy<T, T>(Vb, VT, opts);
        return;
    }
    trace::Block tb("svd");
    internal::DriverScope ds_;
    using R = real_type<T>;
    Target target = resolve_target(opts);
    const int64_t m = A.m(), n = A.n(), k = std::min(m, n);
    if (k == 0) { Sigma.clear(); return; }
    const R anorm = slate::norm(Norm::Max, A, opts);
    bool bad = false;
    const R alpha = range_alpha(anorm, bad);
    if (bad) { Sigma.assign(k, anorm); return; }
    if (alpha != R(1)) scale(alpha, anorm, A, opts);
    const bool wu = wanted(U), wv = wanted(VT);
    auto gA = A.grid();
    if (3 * m > 5 * n || n > m) {
        const bool qr = (3 * m > 5 * n);
        TriangularFactors<T> TQ;
        if (qr) geqrf(A, TQ, opts);
        else gelqf(A, TQ, opts);
        // the k x k triangle (R upper / L lower), zero elsewhere
        Matrix<T> Ak = A.slice(0, k - 1, 0, k - 1);
        Matrix<T> Ah(k, k, A.mb(), A.nb(), gA);
        Ah.insertLocalTiles(target);
        set(T(0), T(0), Ah, opts);
        {
            const Uplo ul = qr ? Uplo::Upper : Uplo::Lower;
            BaseTrapezoidMatrix<T> St(ul, Ak, MatrixKind::Trapezoid), Dt(ul, Ah, MatrixKind::Trapezoid);
            slate::copy<T, T>(St, Dt, opts);
        }
        // the side that the pre-reduction's Q multiplies gets a k x k
        // factor first; the other side is the caller's matrix directly
        Matrix<T> Uk, Vk;
        if (wu) { if (qr) { Uk = Matrix<T>(k, k, A.nb(), A.nb(), gA); Uk.insertLocalTiles(target); } else Uk = U; }
        if (wv) { if (!qr) { Vk = Matrix<T>(k, k, A.mb(), A.mb(), gA); Vk.insertLocalTiles(target); } else Vk = VT; }
        svd_square(Ah, Sigma, Uk, Vk, opts);
        // the caller's U / VT is used in place when it shares A's tiling of
        // the dimension Q acts on (the usual case), else a work copy
        auto fits = [&](Matrix<T> const& X, bool rows) {
            return X.grid().get() == gA.get() && X.aligned() && X.op() == Op::NoTrans &&
                   (rows ? X.mb() == A.mb() : X.nb() == A.nb());
        };
        if (qr && wu) {
            // U = Q [U_R; 0]
            const bool direct = fits(U, true);
            Matrix<T> Uw = U;
            if (!direct) { Uw = Matrix<T>(m, k, A.mb(), A.nb(), gA); Uw.insertLocalTiles(target); }
            set(T(0), T(0), Uw, opts);
            Matrix<T> Ut = Uw.slice(0, k - 1, 0, k - 1);
            slate::copy<T, T>(Uk, Ut, opts);
            unmqr(Side::Left, Op::NoTrans, A, TQ, Uw, opts);
            if (!direct) slate::copy<T, T>(Uw, U, opts);
        }
        if (!qr && wv) {
            // VT = [VT_L 0] Q
            const bool direct = fits(VT, false);
            Matrix<T> Vw = VT;
            if (!direct) { Vw = Matrix<T>(k, n, A.mb(), A.nb(), gA); Vw.insertLocalTiles(target); }
            set(T(0), T(0), Vw, opts);
            Matrix<T> Vt = Vw.slice(0, k - 1, 0, k - 1);
            slate::copy<T, T>(Vk, Vt, opts);
            unmlq(Side::Right, Op::NoTrans, A, TQ, Vw, opts);
            if (!direct) slate::copy<T, T>(Vw, VT, opts);
        }
    } else {
        svd_square(A, Sigma, U, VT, opts);
    }
    rescale_values(Sigma, anorm, alpha);
}

/// Three-stage SVD of an m x n matrix with n <= m <= 5/3 n (no pre-reduction).
template <typename T>
void svd_square(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Matrix<T>& U, Matrix<T>& VT, Options const& opts) {
    using R = real_type<T>;
    Target target = resolve_target(opts);
    const int64_t m = A.m(), n = A.n();
    slate_assert(m >= n);
    // stage 1 on kd-wide tiles (see heev)
    const int64_t kd = std::min<int64_t>(A.nb(), eig_band_width());
    auto gA = A.grid();
    Matrix<T> W(m, n, kd, kd, gA);
    W.insertLocalTiles(target);
    slate::copy<T, T>(A, W, opts);
    std::vector<TriangularFactors<T>> TU, TV;
    ge2tb(W, TU, TV, opts);
    // stage 2 on the host, band storage: tb2bd's windows reach 3 kd + 1 off the diagonal
    const int64_t Mg = 3 * kd + 2;
    std::vector<R> d, e;
    host::Reflectors<T> QU2, QV2;
    std::vector<T> pu, pv;
    const bool ovl = (wanted(U) || wanted(VT)) && eig_overlap(target, true);
    const int64_t wnt = W.nt();
    Matrix<T> QUx, QVx;   // explicit stage-1 factors (ovl)
    {
        std::vector<T> Bb = gather_band(W, kd, Mg, false, false, opts);
        trace::Block t2("tb2bd");
        Comm& w = gA->world();
        overlapped(ovl, [&] { if (w.rank() == 0) host::tb2bd<T>(n, n, kd, Bb.data() + Mg, 2 * Mg, d, e, QU2, QV2, pu, pv); },
                   [&] {
                       trace::Block t3("unmbr_ge2tb_form");
                       if (wanted(U)) {
                           // Q_U [I_n; 0]
                           QUx = Matrix<T>(m, n, kd, kd, gA);
                           QUx.insertLocalTiles(target);
                           set(T(0), T(1), QUx, opts);
                           unmqr(Side::Left, Op::NoTrans, W, stacked_T(TU, wnt, W.nb(), W.n(), opts), QUx, opts);
                       }
                       if (wanted(VT) && wnt >= 2) {
                           QVx = Matrix<T>(n, n, kd, kd, gA);
                           QVx.insertLocalTiles(target);
                           set(T(0), T(1), QVx, opts);
                           Matrix<T> P = W.sub(0, wnt - 2, 1, wnt - 1);
                           Matrix<T> Vs = QVx.sub(0, QVx.mt() - 1, 1, QVx.nt() - 1);
                           unmlq(Side::Right, Op::NoTrans, P, stacked_T(TV, wnt - 1, W.nb(), P.n(), opts), Vs, opts);
                       }
                   });
        if (w.size() > 1) {
            bcast_vec(w, d, 0);
            bcast_vec(w, e, 0);
            bcast_vec(w, pu, 0);
            bcast_vec(w, pv, 0);
            if (!stage2_streamed<T>(target, kd, w)) {
                if (wanted(U)) bcast_reflectors(w, QU2, 0);
                if (wanted(VT)) bcast_reflectors(w, QV2, 0);
            }
        }
    }
    const bool wu = wanted(U), wv = wanted(VT);
    if (!wu && !wv) {
        trace::Block t2("bdsqr");
        host::bdsqr_core<R>(n, d.data(), e.data(), nullptr);
        Sigma = d;
        return;
    }
    // bdsqr: U2 and Vt = VT2^T in the row layout (rotations mix columns)
    GridPtr gr = col_grid(gA), gc = row_grid(gA);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    Matrix<T> U2(n, n, kd, n, gr), V2(n, n, kd, n, gr);
    U2.insertLocalTiles(target);
    V2.insertLocalTiles(target);
    {
        std::vector<T> cpv(n);
        for (int64_t i = 0; i < n; ++i) cpv[i] = slate::conj(pv[i]);
        set_diag_rows(U2, pu, target);
        set_diag_rows(V2, cpv, target);
    }
    {
        trace::Block t2("bdsqr");
        LocalBlock<T> lu = U2.local(loc_of(target), true), lv = V2.local(loc_of(target), true);
        RowRotSink<T> sink(c, n);
        sink.U = wu ? lu.ptr : nullptr; sink.ldu = lu.ld; sink.urows = lu.m;
        sink.V = wv ? lv.ptr : nullptr; sink.ldv = lv.ld; sink.vrows = lv.m;
        host::bdsqr_core<R>(n, d.data(), e.data(), &sink);
        sink.finish();
    }
    Sigma = d;
    if (wu) {
        // U = [QU2 U2; 0], then the stage-1 reflectors
        Matrix<T> U1(n, n, n, kd, gc);
        U1.insertLocalTiles(target);
        slate::copy<T, T>(U2, U1, opts);
        {
            LocalBlock<T> l1 = U1.local(loc_of(target), true);
            Comm& w = gA->world();
            stage2_apply(QU2, stage2_streamed<T>(target, kd, w), n, kd, l1.ptr, l1.ld, l1.n, c, w);
        }
        if (ovl) {
            trace::Block t3("unmbr_ge2tb_u_gemm");
            if (!local_product(Op::NoTrans, QUx, U1, U, opts)) {
                Matrix<T> Un(n, n, kd, kd, gA), Uo(m, n, kd, kd, gA);
                Un.insertLocalTiles(target);
                Uo.insertLocalTiles(target);
                slate::copy<T, T>(U1, Un, opts);
                gemm(T(1), QUx, Un, T(0), Uo, opts);
                slate::copy<T, T>(Uo, U, opts);
            }
        } else {
        Matrix<T> Uw(m, n, kd, kd, gA);
        Uw.insertLocalTiles(target);
        set(T(0), T(0), Uw, opts);
        {
            Matrix<T> Ut = Uw.slice(0, n - 1, 0, n - 1);
            slate::copy<T, T>(U1, Ut, opts);
        }
        trace::Block t3("unmbr_ge2tb_u");
        // the QR panels W(k:, k) together: W itself is their geqrf-shaped view
        unmqr(Side::Left, Op::NoTrans, W, stacked_T(TU, W.nt(), W.nb(), W.n(), opts), Uw, opts);
        slate::copy<T, T>(Uw, U, opts);
        }
    }
    if (wv) {
        // VT2 := VT2 QV2^H  <=>  Vt := conj(QV2) Vt  (Vt = VT2^T), then the stage-1 reflectors
        host::Reflectors<T> QV2c = QV2;
        for (auto& x : QV2c.v) x = slate::conj(x);
        for (auto& x : QV2c.tau) x = slate::conj(x);
        Matrix<T> V1(n, n, n, kd, gc);
        V1.insertLocalTiles(target);
        slate::copy<T, T>(V2, V1, opts);
        {
            LocalBlock<T> l1 = V1.local(loc_of(target), true);
            Comm& w = gA->world();
            stage2_apply(QV2c, stage2_streamed<T>(target, kd, w), n, kd, l1.ptr, l1.ld, l1.n, c, w);
        }
        if (ovl && wnt >= 2) {
            // VT = V1^T QVx
            trace::Block t3("unmbr_ge2tb_v_gemm");
            if (local_product(Op::Trans, V1, QVx, VT, opts)) return;
        }
        Matrix<T> VTw(n, n, kd, kd, gA);
        VTw.insertLocalTiles(target);
        slate::copy<T, T>(transpose(V1), VTw, opts);
        if (ovl && wnt >= 2) {
            Matrix<T> Vo(n, n, kd, kd, gA);
            Vo.insertLocalTiles(target);
            gemm(T(1), VTw, QVx, T(0), Vo, opts);
            slate::copy<T, T>(Vo, VT, opts);
            return;
        }
        trace::Block t3("unmbr_ge2tb_v");
        // the LQ panels W(k, k+1:), k = 0 .. nt-2, together: the gelqf-shaped
        // view W(0:nt-2, 1:) applied to VT(:, 1:)
        const int64_t nt = W.nt(), vmt = VTw.mt();
        if (nt >= 2) {
            Matrix<T> P = W.sub(0, nt - 2, 1, nt - 1);
            Matrix<T> Vs = VTw.sub(0, vmt - 1, 1, VTw.nt() - 1);
            unmlq(Side::Right, Op::NoTrans, P, stacked_T(TV, nt - 1, W.nb(), P.n(), opts), Vs, opts);
        }
        slate::copy<T, T>(VTw, VT, opts);
    }
}

#define SLATE_EIG_INST(T)                                                                                   \
    template void he2hb<T>(Matrix<T>&, std::vector<TriangularFactors<T>>&, Options const&);                 \
    template void heev<T>(HermitianMatrix<T>&, std::vector<real_type<T>>&, Matrix<T>&, Options const&);     \
    template void hegst<T>(int64_t, HermitianMatrix<T>&, HermitianMatrix<T> const&, Options const&);        \
    template void hegv<T>(int64_t, HermitianMatrix<T>&, HermitianMatrix<T>&, std::vector<real_type<T>>&,    \
                          Matrix<T>&, Options const&);                                                      \
    template void ge2tb<T>(Matrix<T>&, std::vector<TriangularFactors<T>>&, std::vector<TriangularFactors<T>>&, \
                           Options const&);                                                                 \
    template void svd<T>(Matrix<T>&, std::vector<real_type<T>>&, Matrix<T>&, Matrix<T>&, Options const&);

SLATE_EIG_INST(float)
SLATE_EIG_INST(double)
SLATE_EIG_INST(std::complex<float>)
SLATE_EIG_INST(std::complex<double>)

}  // namespace slate
