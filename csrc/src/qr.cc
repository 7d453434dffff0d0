// Distributed Householder QR / LQ and least squares (reference src/geqrf.cc,
// unmqr.cc, gelqf.cc, unmlq.cc, gels.cc, gels_qr.cc, gels_cholqr.cc, cholqr.cc).
//
// geqrf per block column k:
//   panel: the m x nb panel is factored on the device by the recursive
//     Householder kernel (column norms, reflector, rank-1 updates and the
//     T factor all on the GPU; T from V^H V + the larft recurrence, as the
//     reference's larft-by-gemm trick internal_geqrf.cc:286-330).  p > 1:
//     TSQR over the process column (local QR of every process's panel rows,
//     binary tree of stacked-R QRs rooted at the diagonal process, reference
//     ttqrt internal_ttqrt.cc:35-130), then Householder reconstruction of
//     the panel's (V, T) from the tree's explicit Q (sign-modified LU), so
//     the trailing update below stays one 2-D larfb.
//   update: the explicit V (unit lower) and T_k are broadcast along process
//     rows; every process computes W = V_loc^H C_loc for its trailing
//     columns, the partial W is all-reduced over the column communicator
//     (p > 1), then W = T^H W and C_loc -= V_loc W -- two MFMA GEMMs and a
//     small one per process (ScaLAPACK-style 2D larfb) -- instead of the
//     reference's tree application ttmqr (internal_ttmqr.cc:99-290).
//   lanes: TSQR / (V, T) / lookahead-W messages on the panel queue over the
//     duplicate comms (Grid::col_fast / row_fast), trailing W all-reduces on
//     the comm queue, so step k+1's tree never queues behind step k's bulk
//     all-reduces.
// T factors: T[0] is an nb x n matrix replicated on every rank (tile k holds
// the panel's nb x nb upper-triangular T).
#include "internal.hh"
#include "spread.hh"
#include "lu_dist.hh"

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

/// TSQR of one distributed panel over a communicator (tree rooted at `root`)
/// followed by Householder reconstruction of the panel's (V, T): every
/// participant's local panel rows (ap, mr x kb) are overwritten with V (and,
/// at the root, R + Y1 in the top kd rows); the root gets T in Tk.  The tree
/// (reference ttqrt, internal_ttqrt.cc:35-130) runs on the panel queue over
/// the given (fast-lane) communicator; the reconstruction makes the trailing
/// update one 2-D larfb instead of the reference's tree application (ttmqr).
/// Used by geqrf (process-column tree) and gelqf (process-row tree on the
/// conjugate-transposed row panel).
///
/// CholeskyQR panel (default on the device; SLATE_QR_CHOLQR=0 turns it off):
/// the tree (a)-(d) costs ~27 ms per 32768 x 512 panel on a 2 x 4 grid,
/// several times the per-step trailing update (profiles/r4_critpath_*).  The
/// explicit Q and R come instead from shifted CholeskyQR3 (Fukaya, Kannan,
/// Nakatsukasa, Yamamoto, Yanagisawa 2020: stable for cond(panel) up to
/// ~1/u), tried after plain CholeskyQR2 (two passes, stable for cond <~
/// u^{-1/2}): passes of  G = Q^H Q (local herk + ONE kb x kb all-reduce),
/// G = L L^H (the shifted variant's first pass adds 11 (M kb + kb(kb+1)) u
/// tr(G) to the diagonal), Q := Q L^{-H}; R = product of the L^H.  The
/// Householder reconstruction (e)-(g) then turns Q into the same (V, T, R)
/// the tree would give.  The Gram matrix before the last pass measures Q's
/// orthogonality: it must satisfy ||G - I||_F <= 0.5 (then every singular
/// value of Q lies in [0.7, 1.23] and the last pass leaves Q orthogonal to
/// working precision), and no pass's Cholesky factorization may report a
/// non-positive pivot.  Otherwise the column's processes -- which all hold the
/// same all-reduced G -- retry with the shifted variant, then fall back to
/// the TSQR tree on the untouched panel (an ill-conditioned, rank-deficient
/// or NaN panel).  That decision is the one host wait per
/// panel step (the panel queue drains; the trailing queues keep running).
template <typename T>
struct TsqrPanel {
    static constexpr int maxr = 8;   // tree levels (comm size <= 256)
    int64_t nb;
    Work<T> Tloc, Rcur, Rrecv, Ecur, Etmp, Qloc, LUb, Ytmp, Dg, Tw, sgn, taul, Gq;
    Work<int> cq_flag;
    Work<double> cq_ssq;
    int* cq_host = nullptr;
    bool cholqr_on = false;
    std::vector<Work<T>> Sst, Ttt;
    const int64_t tSel = Sched::tok(30, 0);

    TsqrPanel(Target target, int np, int64_t nb_, int64_t max_rows, bool single_cholqr = false) : nb(nb_) {
        if (np <= 1 && !single_cholqr) return;
        const size_t nn = size_t(nb) * nb;
        Tloc.resize(target, nn); Rcur.resize(target, nn); Rrecv.resize(target, nn);
        Ecur.resize(target, 2 * nn); Etmp.resize(target, 2 * nn); LUb.resize(target, nn); Ytmp.resize(target, nn);
        Dg.resize(target, nn); Tw.resize(target, nn); sgn.resize(target, nb); taul.resize(target, 2 * nb);
        Qloc.resize(target, size_t(std::max<int64_t>(max_rows, 1)) * nb);
        Sst.resize(maxr); Ttt.resize(maxr);
        for (int r = 0; r < maxr; ++r) { Sst[r].resize(target, 2 * nn); Ttt[r].resize(target, nn); }
        static const bool env_on = [] {
            const char* e = std::getenv("SLATE_QR_CHOLQR");
            return e ? std::atoi(e) != 0 : true;
        }();
        cholqr_on = env_on;
        if (cholqr_on) {
            Gq.resize(target, nn);
            cq_flag.resize(target, 2);
            cq_ssq.resize(target, 1);
            cq_host = target == Target::Devices ? static_cast<int*>(device::malloc_host(sizeof(int) * 2)) : cq_flag.data();
            dev_ = target == Target::Devices;
        }
    }
    ~TsqrPanel() { if (cq_host && dev_) device::free_host(cq_host); }
    bool dev_ = false;
    TsqrPanel(TsqrPanel const&) = delete;
    TsqrPanel& operator=(TsqrPanel const&) = delete;

    /// CholeskyQR of the distributed panel into Qloc (mr x kb) and Rcur (kb x
    /// kb, upper); every process of the column calls it.  shifted = false:
    /// CholeskyQR2 (two passes, stable for cond <~ u^{-1/2}); true: shifted
    /// CholeskyQR3.  The Gram matrix before the last pass is tested against
    /// I; returns whether it passed (the same answer on every process).
    /// Passes use the lower Cholesky factor: G = L L^H, Q := Q L^{-H}, R_i = L^H.
    bool cholqr(Sched& S, int qP, Comm& cm, T* ap, int64_t lda, int64_t mr, int64_t kb, int64_t M, int64_t tPan,
                bool shifted) {
        using R = real_type<T>;
        const double u = double(std::numeric_limits<R>::epsilon()) / 2;
        const double shift = 11.0 * (double(M) * double(kb) + double(kb) * double(kb + 1)) * u;
        const Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
        S.task(qP, {tPan}, {tSel}, [&, ap, mr, kb, shift, shifted, cT](lb::Ctx const& c) {
            trace::Block t2("geqrf_cholqr");
            using DT = slate_amd::dev::dev_t<T>;
            const int64_t ldq = std::max<int64_t>(mr, 1);
            int* dflag = cq_flag.data();
            const int npass = shifted ? 3 : 2;
            lb::copy2d(c, mr, kb, ap, lda, Qloc.data(), ldq);
            // dflag[1]: first non-positive Cholesky pivot of any pass
            if (c.dev()) device::memset_async(dflag + 1, 0, sizeof(int), c.stream);
            else dflag[1] = 0;
            for (int pass = 0; pass < npass; ++pass) {
                T* G = Gq.data();
                lb::herk(c, Uplo::Lower, Op::ConjTrans, kb, mr, R(1), Qloc.data(), ldq, R(0), G, kb);
                cm.allreduce(G, size_t(kb * kb), ReduceOp::Sum, c.loc(), c.stream);
                const bool sh = shifted && pass == 0, chk = pass == npass - 1;
                if (c.dev()) {
                    if (sh) slate_amd::dev::cholqr_shift<DT>(slate_amd::dev::dptr(G), kb, int(kb), shift, c.stream);
                    if (chk)
                        slate_amd::dev::cholqr_check<DT>(slate_amd::dev::dptr(G), kb, int(kb), 0.5, dflag,
                                                         cq_ssq.data(), c.stream);
                } else if (sh) {
                    R tr = 0;
                    for (int64_t i = 0; i < kb; ++i) tr += std::real(G[i + i * kb]);
                    for (int64_t i = 0; i < kb; ++i) G[i + i * kb] += T(R(shift) * tr);
                } else if (chk) {
                    double ssq = 0;   // ||G - I||_F^2 from the lower triangle
                    for (int64_t j = 0; j < kb; ++j)
                        for (int64_t i = j; i < kb; ++i) {
                            const double d = double(std::abs(G[i + j * kb] - (i == j ? T(1) : T(0))));
                            ssq += (i == j ? 1.0 : 2.0) * d * d;
                        }
                    dflag[0] = (ssq <= 0.25) ? 0 : 1;
                }
                lb::potrf(c, Uplo::Lower, kb, G, kb, dflag + 1, 0);
                lb::trsm(c, Side::Right, Uplo::Lower, cT, Diag::NonUnit, mr, kb, T(1), G, kb, Qloc.data(), ldq);
                if (pass == 0) {
                    lb::set(c, Uplo::General, kb, kb, T(0), T(0), Rcur.data(), kb);
                    lb::copy<T, T>(c, Uplo::Upper, cT, kb, kb, G, kb, Rcur.data(), kb);     // L^H
                } else {
                    lb::trmm(c, Side::Left, Uplo::Lower, cT, Diag::NonUnit, kb, kb, T(1), G, kb, Rcur.data(), kb);
                }
            }
            if (c.dev()) device::memcpy_async(cq_host, dflag, 2 * sizeof(int), c.stream);
        });
        if (dev_) slate_hip_call(hipStreamSynchronize(S.ctx(qP).stream));
        return cq_host[0] == 0 && cq_host[1] == 0;
    }

    /// rows_r[r]: panel rows of comm rank r; me: my comm rank; tPan: the
    /// panel's data token; tP: output token of (V, T).
    void enqueue(Sched& S, int qP, Comm& cm, int root, int me, std::vector<int64_t> const& rows_r, T* ap,
                 int64_t lda, int64_t mr, int64_t kb, int64_t kd, T* Tk, int64_t tPan, int64_t tP) {
        int64_t Mtot = 0;
        for (auto r : rows_r) Mtot += r;
        // CholeskyQR2, else shifted CholeskyQR3 (from the untouched panel),
        // else the TSQR tree (see above)
        if (cholqr_on && kd == kb && Mtot >= 2 * kb &&
            (cholqr(S, qP, cm, ap, lda, mr, kb, Mtot, tPan, false) ||
             cholqr(S, qP, cm, ap, lda, mr, kb, Mtot, tPan, true))) {
            reconstruct(S, qP, cm, root, me, ap, lda, mr, kb, kd, Tk, tPan, tP);
            return;
        }
        tree(S, qP, cm, root, me, rows_r, ap, lda, mr, kb, kd, tPan);
        reconstruct(S, qP, cm, root, me, ap, lda, mr, kb, kd, Tk, tPan, tP);
    }

    /// (a)-(d): TSQR tree; leaves Qloc (explicit Q, my rows) and, at the
    /// root, Rcur.
    void tree(Sched& S, int qP, Comm& cm, int root, int me, std::vector<int64_t> const& rows_r, T* ap,
              int64_t lda, int64_t mr, int64_t kb, int64_t kd, int64_t tPan) {
        const int p = int(rows_r.size());
        const int pk = root;
        const bool diag = (me == root);
        const int myrow = me;
        Comm& colF = cm;
        std::vector<int> part;
        for (int d = 0; d < p; ++d) { int r = (pk + d) % p; if (rows_r[r] > 0) part.push_back(r); }
        const int np = int(part.size());
        std::vector<int64_t> cnt(np);
        for (int i = 0; i < np; ++i) cnt[i] = std::min(rows_r[part[i]], kb);
        int ix = -1;
        for (int i = 0; i < np; ++i) if (part[i] == myrow) ix = i;
        struct Round { bool recv; int peer; int64_t mine, theirs; int level; };
        std::vector<Round> rounds;
        int lev = 0;
        for (int l = 1; l < np; l *= 2, ++lev) {
            for (int i = 0; i + l < np; i += 2 * l) {
                if (i == ix) rounds.push_back({true, part[i + l], cnt[i], cnt[i + l], lev});
                if (i + l == ix) rounds.push_back({false, part[i], cnt[i + l], 0, lev});
                cnt[i] = std::min(cnt[i] + cnt[i + l], kb);
            }
        }
        slate_error_if_msg(lev > maxr, "TSQR: process grid too tall for the tree");
        const int64_t rr = std::min(mr, kb);     // rows of my local R
        if (ix >= 0) {
            // (a) local QR of my panel rows; R -> Rcur (rr x kb, ld rr, zeros below)
            S.task(qP, {tPan}, {tPan, tSel}, [&, ap, mr, kb, rr](lb::Ctx const& c) {
                trace::Block t2("geqrf_tsqr_local");
                lb::geqrf_panel(c, mr, kb, ap, lda, taul.data(), Tloc.data(), nb);
                lb::set(c, Uplo::General, rr, kb, T(0), T(0), Rcur.data(), rr);
                lb::copy<T, T>(c, Uplo::Upper, Op::NoTrans, rr, kb, ap, lda, Rcur.data(), rr);
            });
            // (b) reduction tree: QR of the stacked [R_a; R_b], factors kept per level
            int64_t cur = rr;
            int nrecv = 0;
            for (auto const& r_ : rounds) {
                if (!r_.recv) {
                    S.task(qP, {tSel}, {tSel}, [&, r_, kb](lb::Ctx const& c) {
                        trace::Block t2("geqrf_tsqr_sendR");
                        std::vector<Comm::P2P> ops{{Rcur.data(), size_t(r_.mine * kb), r_.peer, true}};
                        colF.exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                    });
                    break;
                }
                const int64_t ms = r_.mine + r_.theirs, c2 = std::min(ms, kb);
                S.task(qP, {}, {tSel}, [&, r_, kb](lb::Ctx const& c) {
                    trace::Block t2("geqrf_tsqr_recvR");
                    std::vector<Comm::P2P> ops{{Rrecv.data(), size_t(r_.theirs * kb), r_.peer, false}};
                    colF.exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                });
                T* Sb = Sst[r_.level].data();
                T* Tt = Ttt[r_.level].data();
                S.task(qP, {}, {tSel}, [&, r_, kb, ms, c2, Sb, Tt](lb::Ctx const& c) {
                    trace::Block t2("geqrf_tsqr_merge");
                    lb::copy2d(c, r_.mine, kb, Rcur.data(), r_.mine, Sb, ms);
                    lb::copy2d(c, r_.theirs, kb, Rrecv.data(), r_.theirs, Sb + r_.mine, ms);
                    lb::geqrf_panel(c, ms, kb, Sb, ms, taul.data(), Tt, nb);
                    lb::set(c, Uplo::General, c2, kb, T(0), T(0), Rcur.data(), c2);
                    lb::copy<T, T>(c, Uplo::Upper, Op::NoTrans, c2, kb, Sb, ms, Rcur.data(), c2);
                });
                cur = c2;
                ++nrecv;
            }
            // (c) explicit Q (first kd columns), top-down: E = [I; 0] at the root
            const bool sender = !rounds.empty() && !rounds.back().recv;
            int64_t ecnt = 0;                  // rows of my current E block (ld ecnt)
            if (diag) {
                S.task(qP, {}, {tSel}, [&, cur, kd](lb::Ctx const& c) {
                    lb::set(c, Uplo::General, cur, kd, T(0), T(1), Ecur.data(), cur);
                });
                ecnt = cur;
            } else if (sender) {
                auto const r_ = rounds.back();
                S.task(qP, {}, {tSel}, [&, r_, kd](lb::Ctx const& c) {
                    trace::Block t2("geqrf_tsqr_recvE");
                    std::vector<Comm::P2P> ops{{Ecur.data(), size_t(r_.mine * kd), r_.peer, false}};
                    colF.exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                });
                ecnt = r_.mine;
            }
            for (int t = nrecv - 1; t >= 0; --t) {
                auto const r_ = rounds[t];
                const int64_t ms = r_.mine + r_.theirs, c2 = std::min(ms, kb);
                T* Sb = Sst[r_.level].data();
                T* Tt = Ttt[r_.level].data();
                // E (c2 x kd) -> [E; 0] (ms x kd) -> Q_level [E; 0]
                S.task(qP, {}, {tSel}, [&, ms, c2, kd, Sb, Tt](lb::Ctx const& c) {
                    trace::Block t2("geqrf_tsqr_qtree");
                    lb::set(c, Uplo::General, ms, kd, T(0), T(0), Etmp.data(), ms);
                    lb::copy2d(c, c2, kd, Ecur.data(), c2, Etmp.data(), ms);
                    lb::larfb(c, Side::Left, Op::NoTrans, ms, kd, c2, Sb, ms, Tt, nb, Etmp.data(), ms);
                });
                // partner's rows go down the tree, mine stay (compacted to ld = mine)
                S.task(qP, {}, {tSel}, [&, r_, ms, kd](lb::Ctx const& c) {
                    trace::Block t2("geqrf_tsqr_sendE");
                    lb::copy2d(c, r_.theirs, kd, Etmp.data() + r_.mine, ms, Rrecv.data(), r_.theirs);
                    std::vector<Comm::P2P> ops{{Rrecv.data(), size_t(r_.theirs * kd), r_.peer, true}};
                    colF.exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                });
                S.task(qP, {}, {tSel}, [&, r_, ms, kd](lb::Ctx const& c) {
                    lb::copy2d(c, r_.mine, kd, Etmp.data(), ms, Ecur.data(), r_.mine);
                });
                ecnt = r_.mine;
            }
            // (d) local rows of Q: Qloc = Q_local [E; 0]  (mr x kd)
            S.task(qP, {tSel}, {tSel}, [&, ap, mr, rr, kd, ecnt](lb::Ctx const& c) {
                trace::Block t2("geqrf_tsqr_qlocal");
                lb::set(c, Uplo::General, mr, kd, T(0), T(0), Qloc.data(), mr);
                lb::copy2d(c, ecnt, kd, Ecur.data(), ecnt, Qloc.data(), mr);
                lb::larfb(c, Side::Left, Op::NoTrans, mr, kd, rr, ap, lda, Tloc.data(), nb, Qloc.data(), mr);
            });
        }
    }

    /// (e)-(g): Householder reconstruction of (V, T, R) from Qloc / Rcur.
    void reconstruct(Sched& S, int qP, Comm& cm, int root, int me, T* ap, int64_t lda, int64_t mr, int64_t kb,
                     int64_t kd, T* Tk, int64_t tPan, int64_t tP) {
        const int pk = root;
        const bool diag = (me == root);
        Comm& colF = cm;
        // (e) pk: sign-modified LU of [S - Q11]  ->  Y1, U', S
        if (diag) {
            S.task(qP, {tSel}, {tSel}, [&, mr, kd](lb::Ctx const& c) {
                trace::Block t2("geqrf_tsqr_hr_lu");
                lb::add(c, Uplo::General, kd, kd, T(-1), Qloc.data(), mr, T(0), LUb.data(), kd);
                internal::ludist::lu_sign(c, kd, LUb.data(), kd, sgn.data());
            });
        }
        S.task(qP, {}, {tSel}, [&, kd, pk](lb::Ctx const& c) {
            trace::Block t2("geqrf_tsqr_bcast_lu");
            bcast(colF, LUb.data(), size_t(kd * kd), pk, c);
            bcast(colF, sgn.data(), size_t(kd), pk, c);
        });
        // (f) V below T: Y2 = -Q21 U'^{-1}, written into the panel rows
        const int64_t off = diag ? kd : 0, nbelow = std::max<int64_t>(mr - off, 0);
        S.task(qP, {tSel}, {tPan, tSel}, [&, ap, mr, kd, off, nbelow](lb::Ctx const& c) {
            trace::Block t2("geqrf_tsqr_hr_v");
            lb::trsm(c, Side::Right, Uplo::Upper, Op::NoTrans, Diag::NonUnit, nbelow, kd, T(-1), LUb.data(), kd,
                     Qloc.data() + off, std::max<int64_t>(mr, 1));
            lb::copy2d(c, nbelow, kd, Qloc.data() + off, std::max<int64_t>(mr, 1), ap + off, lda);
        });
        // (g) pk: R = S R_tsqr and Y1 into the diagonal block; T = U' S^H Y1^{-H}
        if (diag) {
            S.task(qP, {tSel}, {tPan, tSel, tP}, [&, ap, kb, kd, Tk](lb::Ctx const& c) {
                trace::Block t2("geqrf_tsqr_hr_t");
                // Dg = diag(s)
                lb::set(c, Uplo::General, kd, kd, T(0), T(0), Dg.data(), kd);
                lb::copy2d(c, int64_t(1), kd, sgn.data(), int64_t(1), Dg.data(), kd + 1);
                // A(T rows) = S R_tsqr (upper trapezoid) + strictly-lower Y1
                lb::gemm(c, Op::NoTrans, Op::NoTrans, kd, kb, kd, T(1), Dg.data(), kd, Rcur.data(), kd, T(0), ap,
                         lda);
                lb::copy2d(c, kd, kd, LUb.data(), kd, Ytmp.data(), kd);
                lb::set(c, Uplo::Upper, kd, kd, T(0), T(0), Ytmp.data(), kd);
                lb::add(c, Uplo::Lower, kd, kd, T(1), Ytmp.data(), kd, T(1), ap, lda);
                // T = triu(U') S^H Y1^{-H}, padded to kb x kb
                lb::set(c, Uplo::General, kd, kd, T(0), T(0), Tw.data(), kd);
                lb::copy<T, T>(c, Uplo::Upper, Op::NoTrans, kd, kd, LUb.data(), kd, Tw.data(), kd);
                lb::set(c, Uplo::General, kb, kb, T(0), T(0), Tk, kb);
                lb::gemm(c, Op::NoTrans, Op::ConjTrans, kd, kd, kd, T(1), Tw.data(), kd, Dg.data(), kd, T(0), Tk, kb);
                lb::trsm(c, Side::Right, Uplo::Lower, Op::ConjTrans, Diag::Unit, kd, kd, T(1), LUb.data(), kd, Tk, kb);
            });
        }
    }
};

template <typename T>
void geqrf_impl(BaseMatrix<T> A, Matrix<T>& Tf, Target target, int64_t la) {
    auto& g = *A.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t mt = A.mt(), nt = A.nt(), m = A.m();
    const int64_t kt = std::min(mt, nt);
    const int64_t nb = A.nb();
    LocalBlock<T> L = A.local(loc, true);
    T* a = L.ptr;
    const int64_t lda = L.ld, mloc = L.m, nloc = L.n;
    LocalBlock<T> LT = Tf.local(loc, true);   // replicated nb x n
    T* tm = LT.ptr;
    const int64_t ldt = LT.ld;
    const int qC = device::kCommQueue, qP = 1;
    // critical-path lane: TSQR tree, (V, T) broadcasts and the lookahead
    // columns' W all-reduce on the panel queue over the duplicate comms;
    // the trailing chunks' W all-reduces stay on the comm queue (bulk lane)
    Comm& colF = g.col_fast();
    Comm& rowF = g.row_fast();

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
    // p == 1 on the device: the local panel by CholeskyQR2 (shifted CholQR3,
    // then the TSQR tree, as fallbacks) + reconstruction as well; measured
    // dgeqrf n = 65536: 6715 -> 6626 ms (profiles/r4_ab_tail.txt).
    // SLATE_QR_CHOLQR1=0 keeps the on-chip TSQR panel (lb::geqrf_panel).
    static const bool cq1_env = [] {
        const char* e = std::getenv("SLATE_QR_CHOLQR1");
        return !e || std::atoi(e) != 0;
    }();
    // (large factorizations only: for the narrow, short panels of he2hb /
    // ge2tb -- 64-wide tiles, m <= n of the eigenproblem -- the on-chip TSQR
    // panel is faster: he2hb at n = 8192 took 466 ms in geqrf with CholQR)
    const bool cq1 = p == 1 && cq1_env && target == Target::Devices && nb >= 256 && A.m() >= 16384;
    TsqrPanel<T> tsqr(target, p > 1 ? p : 1, nb, mloc, cq1);
    const Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;

    for (int64_t k = 0; k < kt; ++k) {
        const int64_t kb = A.tileNb(k);
        const int64_t kk = grow_of(A, k);
        const int64_t M = m - kk;
        const int64_t kd = std::min(kb, M);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const bool in_col = (mycol == qk), diag = (myrow == pk);
        const int64_t lr_k = lrow_of(A, k);
        const int64_t lc_k = in_col ? lcol_of(A, k) : 0;
        const int64_t mr = mloc - lr_k;          // my rows >= kk
        const int slot = int(k % R);
        T* Tk = WT[slot].data();
        T* tau = Wtau[slot].data();
        T* ap = a + lr_k + lc_k * lda;
        const int64_t tP = Sched::tok(6, slot), tB = Sched::bcast(slot);

        // ================================================================ panel
        if (in_col && p == 1 && cq1 && kd == kb && M >= 2 * kb) {
            std::vector<int64_t> rows_r{M};
            tsqr.enqueue(S, qP, g.col(), 0, 0, rows_r, ap, lda, mr, kb, kd, Tk, Sched::col(k), tP);
        } else if (in_col && p == 1) {
            S.task(qP, {}, {Sched::col(k), tP}, [&, kb, M, Tk, tau, ap](lb::Ctx const& c) {
                trace::Block t2("geqrf_panel");
                lb::geqrf_panel(c, M, kb, ap, lda, tau, Tk, kb);
            });
        } else if (in_col) {
            // ---- TSQR over the process column (tree rooted at pk) + Householder
            //      reconstruction of (V, T) (kernels/tsqr.hip)
            std::vector<int64_t> rows_r(p, 0);
            for (int64_t i = k; i < mt; ++i) rows_r[A.srow_owner(i)] += A.tileMb(i);
            tsqr.enqueue(S, qP, colF, pk, myrow, rows_r, ap, lda, mr, kb, kd, Tk, Sched::col(k), tP);
        }

        // ======================= T_k down the panel column, then (V, T_k) along rows
        T* Vk = WV[slot].data();
        const int64_t ldv = std::max<int64_t>(mr, 1);
        S.task(qP, {tP, Sched::col(k)}, {tB}, [&, kb, kk, lr_k, lc_k, mr, pk, qk, Tk, Vk, ldv, in_col, diag](lb::Ctx const& c) {
            trace::Block t2("geqrf_bcast");
            if (in_col) {
                if (p > 1) bcast(colF, Tk, size_t(kb * kb), pk, c);
                // explicit V: my rows >= kk; the diagonal process row has the unit upper part
                pack(c, mr, kb, a + lr_k + lc_k * lda, lda, Vk);
                if (diag) lb::set(c, Uplo::Upper, std::min<int64_t>(kb, mr), kb, T(0), T(1), Vk, ldv);
            }
            if (q > 1) {
                bcast(rowF, Tk, size_t(kb * kb), qk, c);
                bcast(rowF, Vk, size_t(mr * kb), qk, c);
            }
            // keep T_k in the replicated factor matrix
            lb::copy2d(c, kb, kb, Tk, kb, tm + kk * ldt, ldt);
        });

        // ============================================================ update
        T* Wk = WW[slot].data();
        T* W2k = WW2[slot].data();
        // W = V^H C  (kb x nc); on a wide trailing block the GEMM's K (= mr rows)
        // is long, so K chunks of kch rows bound each workgroup's lifetime and
        // the next panel's short kernels (high-priority stream) find free CUs.
        auto vhc = [&, kb, lr_k, mr, Vk, ldv, Wk](lb::Ctx const& c, int64_t c0, int64_t nc) {
            T* Cc = a + lr_k + c0 * lda;
            T* W = Wk + c0 * kb;
            const int64_t kch = qr_kchunk();
            if (mr > 0 && kch > 0 && mr > kch && nc >= 4 * kb) {
                // K slices of <= kch rows as one batched launch (partials +
                // in-order reduce): no wave-quantization tail per slice, as
                // sequential beta-accumulating launches had (isolated
                // 512 x 20000 x 44000: 53.4 -> 64-67 TFLOP/s)
                lb::gemm_splitk(c, cT, Op::NoTrans, kb, nc, mr, std::min<int64_t>(ceildiv(mr, kch), 8), T(1), Vk, ldv,
                                Cc, lda, T(0), W, kb);
            } else if (mr > 0) lb::gemm(c, cT, Op::NoTrans, kb, nc, mr, T(1), Vk, ldv, Cc, lda, T(0), W, kb);
            else lb::set(c, Uplo::General, kb, nc, T(0), T(0), W, kb);
        };
        // C -= V (T^H W)
        auto apply = [&, kb, lr_k, mr, Tk, Vk, ldv, Wk, W2k](lb::Ctx const& c, int64_t c0, int64_t nc) {
            T* Cc = a + lr_k + c0 * lda;
            if (!is_complex_v<T> && c.dev() && update_nt()) {
                // (T^H W)^H = W^H T (nc x kb, ld nc): C -= V (W^H T)^H runs as
                // an NT product
                T* W2h = W2k + c0 * kb;
                lb::gemm(c, cT, Op::NoTrans, nc, kb, kb, T(1), Wk + c0 * kb, kb, Tk, kb, T(0), W2h, nc);
                if (mr > 0) lb::gemm(c, Op::NoTrans, cT, mr, nc, kb, T(-1), Vk, ldv, W2h, nc, T(1), Cc, lda);
                return;
            }
            lb::gemm(c, cT, Op::NoTrans, kb, nc, kb, T(1), Tk, kb, Wk + c0 * kb, kb, T(0), W2k + c0 * kb, kb);
            if (mr > 0) lb::gemm(c, Op::NoTrans, Op::NoTrans, mr, nc, kb, T(-1), Vk, ldv, W2k + c0 * kb, kb, T(1), Cc, lda);
        };
        auto range = [&, kb, Wk](int queue, int64_t j0, int64_t j1) {
            const int64_t c0 = lcol_of(A, j0), nc = lcol_of(A, j1) - c0;
            if (nc <= 0) return;
            std::vector<int64_t> cols;
            for (int64_t j = j0; j < j1; ++j) cols.push_back(Sched::col(j));
            if (p == 1) {
                S.task(queue, {tB}, cols, [&, c0, nc](lb::Ctx const& c) {
                    trace::Block t2("geqrf_update");
                    vhc(c, c0, nc);
                    apply(c, c0, nc);
                });
                return;
            }
            // p > 1: the column all-reduce of W runs on the comm queue between
            // the two halves, which stay on the compute queue
            S.task(queue, {tB}, cols, [&, c0, nc](lb::Ctx const& c) { trace::Block t2("geqrf_update_w"); vhc(c, c0, nc); });
            const bool crit = (queue == device::kLookaheadQueue);
            Comm& cw = crit ? colF : g.col();
            S.task(crit ? qP : qC, {}, cols, [&, c0, nc, kb, Wk](lb::Ctx const& c) {
                trace::Block t2("geqrf_update_allreduce");
                cw.allreduce(Wk + c0 * kb, size_t(kb * nc), ReduceOp::Sum, c.loc(), c.stream);
            });
            S.task(queue, {tB}, cols, [&, c0, nc](lb::Ctx const& c) { trace::Block t2("geqrf_update_c"); apply(c, c0, nc); });
        };
        const int64_t jla_end = std::min(nt, k + 1 + la);
        for (int64_t j = k + 1; j < jla_end; ++j) range(device::kLookaheadQueue, j, j + 1);
        if (jla_end < nt) {
            const int64_t ntr = nt - jla_end, nch = (p == 1) ? 1 : std::min<int64_t>(4, ntr);
            for (int64_t ch = 0; ch < nch; ++ch)
                range(device::kTrailQueue, jla_end + ch * ntr / nch, jla_end + (ch + 1) * ntr / nch);
        }
    }
    S.wait_all();
    A.storage()->update_origin();
    Tf.storage()->update_origin();
}

/// Apply Q (or Q^H) from geqrf to C from the left: C = op(Q) C (reference
/// src/unmqr.cc, internal_unmqr.cc:161-234), as a stream DAG: per step the
/// explicit V_k (my panel rows) is packed and broadcast along the process
/// row on the panel queue (fast lane) one step ahead; C's local columns are
/// split in up to 4 chunks, each W = V^H C chunk is all-reduced down the
/// process column on the comm queue while the next chunk's GEMM runs, then
/// C -= V (op(T) W).  No host synchronization until the end.
template <typename T>
void unmqr_left(Op op, BaseMatrix<T> A, Matrix<T> const& Tf, Matrix<T>& C, Target target) {
    auto& g = *A.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t kt = std::min(A.mt(), A.nt());
    LocalBlock<T> L = A.local(loc, false);
    LocalBlock<T> LC = C.local(loc, true);
    LocalBlock<T> LT = Tf.local(loc, false);
    const int64_t nb = A.nb(), ncC = LC.n;
    const Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
    Sched S(target);
    const int R = 3;
    std::vector<Work<T>> WV(R), WW(R), WW2(R);
    for (int r = 0; r < R; ++r) {
        WV[r].resize(target, size_t(std::max<int64_t>(L.m, 1)) * nb);
        WW[r].resize(target, size_t(nb) * std::max<int64_t>(ncC, 1));
        WW2[r].resize(target, size_t(nb) * std::max<int64_t>(ncC, 1));
    }
    // column chunks of C (whole local tiles)
    std::vector<int64_t> cb{0};
    {
        const int64_t nch = std::min<int64_t>(4, std::max<int64_t>(C.nt(), 1));
        for (int64_t ch = 1; ch <= nch; ++ch) {
            int64_t j = ch * C.nt() / nch;
            int64_t lc = j >= C.nt() ? ncC : lcol_of(C, j);
            if (lc > cb.back()) cb.push_back(lc);
        }
        if (cb.back() < ncC) cb.push_back(ncC);
    }
    for (int64_t t = 0; t < kt; ++t) {
        const int64_t k = (op == Op::NoTrans) ? kt - 1 - t : t;   // Q C: k descending with T; Q^H C: ascending, T^H
        const int64_t kb = A.tileNb(k), kk = grow_of(A, k);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const int64_t lr_k = lrow_of(A, k), mr = L.m - lr_k, ldv = std::max<int64_t>(mr, 1);
        const int64_t lcr = lrow_of(C, k);    // C's local rows >= kk (C conforms to A's rows)
        const int slot = int(t % R);
        T* Vk = WV[slot].data();
        T* W = WW[slot].data();
        T* W2 = WW2[slot].data();
        const int64_t tV = Sched::bcast(slot);
        S.task(1, {}, {tV}, [&, k, kb, mr, ldv, lr_k, pk, qk, Vk](lb::Ctx const& c) {
            trace::Block t2("unmqr_bcast_v");
            if (mycol == qk) {
                pack(c, mr, kb, L.ptr + lr_k + lcol_of(A, k) * L.ld, L.ld, Vk);
                if (myrow == pk) lb::set(c, Uplo::Upper, std::min<int64_t>(kb, mr), kb, T(0), T(1), Vk, ldv);
            }
            if (q > 1) bcast(g.row_fast(), Vk, size_t(mr * kb), qk, c);
        });
        T const* Tk = LT.ptr + kk * LT.ld;
        for (size_t ch = 0; ch + 1 < cb.size(); ++ch) {
            const int64_t c0 = cb[ch], nc = cb[ch + 1] - c0;
            T* Cc = LC.ptr + lcr + c0 * LC.ld;
            const int64_t tc = Sched::col(int64_t(ch));
            S.task(0, {tV}, {tc}, [&, kb, mr, ldv, nc, Cc, Vk, W, c0](lb::Ctx const& c) {
                trace::Block t2("unmqr_w");
                if (mr > 0) lb::gemm(c, cT, Op::NoTrans, kb, nc, mr, T(1), Vk, ldv, Cc, LC.ld, T(0), W + c0 * kb, kb);
                else lb::set(c, Uplo::General, kb, nc, T(0), T(0), W + c0 * kb, kb);
            });
            if (p > 1)
                S.task(device::kCommQueue, {}, {tc}, [&, kb, nc, W, c0](lb::Ctx const& c) {
                    trace::Block t2("unmqr_allreduce");
                    g.col().allreduce(W + c0 * kb, W + c0 * kb, size_t(kb * nc), scalar_type<T>(), ReduceOp::Sum,
                                      c.loc(), c.stream);
                });
            S.task(0, {tV}, {tc}, [&, kb, mr, ldv, nc, Cc, Vk, W, W2, c0, Tk](lb::Ctx const& c) {
                trace::Block t2("unmqr_c");
                lb::gemm(c, op == Op::NoTrans ? Op::NoTrans : cT, Op::NoTrans, kb, nc, kb, T(1), Tk, LT.ld,
                         W + c0 * kb, kb, T(0), W2 + c0 * kb, kb);
                if (mr > 0) lb::gemm(c, Op::NoTrans, Op::NoTrans, mr, nc, kb, T(-1), Vk, ldv, W2 + c0 * kb, kb, T(1), Cc,
                                     LC.ld);
            });
        }
    }
    S.wait_all();
    C.storage()->update_origin();
}

/// C = C op(Q) (Side::Right) in place: C on A's grid with C's column tiles =
/// A's row tiles (C's columns are Q's rows).  Per block k (ascending for Q,
/// descending for Q^H): V_k -- A's block column k, unit upper on the
/// diagonal block, zero above -- is gathered whole (along the process rows
/// from its owner, then all-gathered over the process column), each process
/// takes the rows matching its local columns of C, W = C V_k is summed over
/// the process row, and C -= (W op(T_k)) V_k^H: no (conj-)transposed copy of
/// C (the reference applies ttmqr / unmqr tile by tile on C's columns).
template <typename T>
void unmqr_right(Op op, BaseMatrix<T> A, Matrix<T> const& Tf, Matrix<T>& C, Target target) {
    auto& g = *A.grid();
    const int p = g.p(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t kt = std::min(A.mt(), A.nt());
    LocalBlock<T> L = A.local(loc, false);
    LocalBlock<T> LC = C.local(loc, true);
    LocalBlock<T> LT = Tf.local(loc, false);
    const int64_t nb = A.nb(), mC = LC.m, ncC = LC.n, ldw = std::max<int64_t>(mC, 1), ldv = std::max<int64_t>(ncC, 1);
    const Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
    std::vector<int64_t> rowoff(size_t(A.mt()), 0), cnt(p, 0);
    for (int64_t i = 0; i < A.mt(); ++i) {
        rowoff[i] = cnt[A.srow_owner(i)];
        cnt[A.srow_owner(i)] += A.tileMb(i);
    }
    const int64_t maxr = std::max<int64_t>(1, *std::max_element(cnt.begin(), cnt.end()));
    Sched S(target);
    const int R = 3;
    std::vector<Work<T>> WG(R), WV(R), WW(R), WW2(R);
    Work<T> Gs(target, size_t(maxr) * nb);
    for (int r = 0; r < R; ++r) {
        WG[r].resize(target, size_t(p) * maxr * nb);
        WV[r].resize(target, size_t(ldv) * nb);
        WW[r].resize(target, size_t(ldw) * nb);
        WW2[r].resize(target, size_t(ldw) * nb);
    }
    const int64_t tC = Sched::tok(9, 0);
    for (int64_t t = 0; t < kt; ++t) {
        const int64_t k = (op == Op::NoTrans) ? t : kt - 1 - t;
        const int64_t kb = A.tileNb(k), kk = grow_of(A, k);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const int slot = int(t % R);
        T* G = WG[slot].data();
        T* Vc = WV[slot].data();
        T* W = WW[slot].data();
        T* W2 = WW2[slot].data();
        const int64_t tV = Sched::bcast(slot);
        S.task(1, {}, {tV}, [&, k, kb, kk, pk, qk, G, Vc](lb::Ctx const& c) {
            trace::Block t2("unmqr_bcast_v");
            if (mycol == qk) {
                // my rows of A(:, k): zero above row kk, unit upper diagonal block
                const int64_t lr_k = lrow_of(A, k);
                lb::set(c, Uplo::General, maxr, kb, T(0), T(0), Gs.data(), maxr);
                lb::copy2d(c, L.m - lr_k, kb, L.ptr + lr_k + lcol_of(A, k) * L.ld, L.ld, Gs.data() + lr_k, maxr);
                if (myrow == pk)
                    lb::set(c, Uplo::Upper, std::min<int64_t>(kb, L.m - lr_k), kb, T(0), T(1), Gs.data() + lr_k, maxr);
            }
            bcast(g.row_fast(), Gs.data(), size_t(maxr * kb), qk, c);
            g.col_fast().allgather(Gs.data(), G, size_t(maxr * kb), scalar_type<T>(), c.loc(), c.stream);
            // the rows of V matching my local columns of C (V is zero above kk)
            lb::set(c, Uplo::General, ncC, kb, T(0), T(0), Vc, ldv);
            for (int64_t J = k; J < C.nt(); ++J) {
                if (C.scol_owner(J) != mycol) continue;
                lb::copy2d(c, C.tileNb(J), kb, G + size_t(A.srow_owner(J)) * maxr * kb + rowoff[J], maxr,
                           Vc + lcol_of(C, J), ldv);
            }
            (void)kk;
        });
        T const* Tk = LT.ptr + kk * LT.ld;
        S.task(0, {tV}, {tC}, [&, kb, Vc, W](lb::Ctx const& c) {
            trace::Block t2("unmqr_w");
            if (mC > 0) lb::gemm(c, Op::NoTrans, Op::NoTrans, mC, kb, ncC, T(1), LC.ptr, LC.ld, Vc, ldv, T(0), W, ldw);
        });
        S.task(device::kCommQueue, {}, {tC}, [&, kb, W](lb::Ctx const& c) {
            trace::Block t2("unmqr_allreduce");
            if (mC > 0) g.row().allreduce(W, W, size_t(ldw * kb), scalar_type<T>(), ReduceOp::Sum, c.loc(), c.stream);
        });
        S.task(0, {tV}, {tC}, [&, kb, Vc, W, W2, Tk](lb::Ctx const& c) {
            trace::Block t2("unmqr_c");
            if (mC <= 0) return;
            lb::gemm(c, Op::NoTrans, op == Op::NoTrans ? Op::NoTrans : cT, mC, kb, kb, T(1), W, ldw, Tk, LT.ld, T(0), W2,
                     ldw);
            lb::gemm(c, Op::NoTrans, cT, mC, ncC, kb, T(-1), W2, ldw, Vc, ldv, T(1), LC.ptr, LC.ld);
        });
    }
    S.wait_all();
    C.storage()->update_origin();
}

}  // namespace

template <typename T>
void geqrf(Matrix<T>& A, TriangularFactors<T>& T_, Options const& opts) {
    if (auto grp = internal::multi_group<T>({&A})) {   // multi-device A: factor on its devices
        std::vector<TriangularFactors<T>> Tr(grp->size());
        internal::spread<T>(opts, {{&A, true}}, [&](std::vector<Matrix<T>>& M, int r) {
            geqrf(M[0], Tr[r], opts);
        }, false);
        T_ = internal::factors_from_parts(grp, Tr);
        return;
    }
    if (A.arbitrary_layout()) {
        Matrix<T> Ab = internal::block_cyclic(A, opts);
        geqrf(Ab, T_, opts);
        slate::copy<T, T>(Ab, A, opts);
        return;
    }
    trace::Block tb("geqrf");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    int64_t la = get_option<int64_t>(opts, Option::Lookahead, 1);
    slate_error_if_msg(A.op() != Op::NoTrans || !A.aligned() || A.mb() != A.nb(),
                       "geqrf: NoTrans, tile-aligned, square-tile matrix required");
    Matrix<T> Tf(A.nb(), std::max<int64_t>(A.n(), 1), A.nb(), A.nb(), Grid::self());
    Tf.insertLocalTiles(target);
    set(T(0), T(0), Tf, opts);
    geqrf_impl<T>(A, Tf, target, la);
    if (target == Target::Devices) lb::check_panel_errors();
    internal::finish_origin(A, opts);
    T_.clear();
    T_.push_back(Tf);
}

template <typename T>
void unmqr(Side side, Op op, Matrix<T> const& A, TriangularFactors<T> const& T_, Matrix<T>& C, Options const& opts) {
    if (internal::multi_group<T>({&A, &C})) {
        auto args = internal::with_factors<T>({{&A, false}, {&C, true}}, T_);
        internal::spread<T>(opts, args, [&](std::vector<Matrix<T>>& M, int) {
            TriangularFactors<T> Tr(M.begin() + 2, M.end());
            unmqr(side, op, M[0], Tr, M[1], opts);
        }, false);
        return;
    }
    if (A.arbitrary_layout()) {
        // T is expressed in the tiling of A's block-cyclic working copy
        Matrix<T> Ab = internal::block_cyclic(A, opts);
        unmqr(side, op, Ab, T_, C, opts);
        return;
    }
    trace::Block tb("unmqr");
    internal::DriverScope ds_;
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
            internal::finish_origin(C, opts);
        } else {
            Matrix<T> Cx(C.m(), C.n(), A.mb(), C.nb(), A.grid(), A.mt() ? A.srow_owner(0) : 0, 0);
            Cx.insertLocalTiles(target);
            slate::copy<T, T>(C, Cx, opts);
            unmqr_left<T>(op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans, A, T_[0], Cx, target);
            slate::copy<T, T>(Cx, C, opts);
        }
        return;
    }
    {
        // in place when C is on A's grid with C's column tiles = A's row tiles
        bool conform = C.op() == Op::NoTrans && C.aligned() && A.aligned() && C.grid()->same_processes(*A.grid())
                    && C.grid()->p() == A.grid()->p() && C.grid()->q() == A.grid()->q()
                    && C.grid()->order() == A.grid()->order() && C.nt() == A.mt();
        if (conform)
            for (int64_t j = 0; j < A.mt(); ++j)
                if (A.tileMb(j) != C.tileNb(j)) { conform = false; break; }
        if (conform) {
            unmqr_right<T>(op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans, A, T_[0], C, target);
            internal::finish_origin(C, opts);
            return;
        }
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

//------------------------------------------------------------------------------
// LQ (reference src/gelqf.cc:207-298 with ttlqt/ttmlq, src/unmlq.cc).
namespace {

/// A = L Q on row panels, in place, no transposed copy of A.  Per block row
/// k the row panel A(k, k:) (process row pk, spread over the process
/// columns) is conjugate-transposed into a column buffer P (my local columns
/// x kb), QR-factored there -- the device panel kernel when q == 1, else the
/// TSQR tree over the PROCESS ROW (fast-lane row comm) -- and written back:
/// L(k,k) on/below the diagonal, the reflectors Y^H stored row-wise to its
/// right (LAPACK gelqf layout).  With H_k = I - Y T Y^H, the rows below are
/// updated from the right, C := C H_k = C - (C Y) T Y^H: W = C Y per
/// process, all-reduced across the process row, then two GEMMs.  Y goes down
/// the process columns, T along the row; the block row k+1 is updated first
/// (lookahead queue, fast lane), the rest on the trailing queue.
template <typename T>
void gelqf_impl(BaseMatrix<T> A, Matrix<T>& Tf, Target target) {
    auto& g = *A.grid();
    const int q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t mt = A.mt(), nt = A.nt(), n = A.n();
    const int64_t kt = std::min(mt, nt);
    const int64_t nb = A.nb();
    LocalBlock<T> L = A.local(loc, true);
    T* a = L.ptr;
    const int64_t lda = L.ld, mloc = L.m, nloc = L.n;
    LocalBlock<T> LT = Tf.local(loc, true);
    T* tm = LT.ptr;
    const int64_t ldt = LT.ld;
    const int qC = device::kCommQueue, qP = 1;
    Comm& colF = g.col_fast();
    Comm& rowF = g.row_fast();
    Sched S(target);
    const int R = 3;
    std::vector<Work<T>> WY(R), WT(R), WW(R), WW2(R), Wtau(R);
    for (int r = 0; r < R; ++r) {
        WY[r].resize(target, size_t(std::max<int64_t>(nloc, 1)) * nb);
        WT[r].resize(target, size_t(nb) * nb);
        WW[r].resize(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
        WW2[r].resize(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
        Wtau[r].resize(target, size_t(nb));
    }
    TsqrPanel<T> tsqr(target, q, nb, nloc);
    for (int64_t k = 0; k < kt; ++k) {
        const int64_t kb = A.tileMb(k);               // panel rows
        const int64_t kk = gcol_of(A, k);             // first panel column
        const int64_t N = n - kk, kd = std::min(kb, N);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const bool in_row = (myrow == pk), diag = (mycol == qk);
        const int64_t lc_k = lcol_of(A, k), nc = nloc - lc_k, ldy = std::max<int64_t>(nc, 1);
        const int64_t lr_k = in_row ? lrow_of(A, k) : 0;
        T* rp = a + lr_k + lc_k * lda;
        const int slot = int(k % R);
        T* Yk = WY[slot].data();
        T* Tk = WT[slot].data();
        const int64_t tP = Sched::tok(6, slot), tB = Sched::bcast(slot), tPan = Sched::row(k);
        // ---- panel: P = rp^H, QR(P), rp = P^H, explicit Y
        if (in_row) {
            // (tB as an output: Y_k / T_k of this ring slot are free once the
            // previous step using the slot has finished its updates)
            S.task(qP, {Sched::row(k)}, {tPan, tB}, [&, kb, nc, rp, Yk, ldy](lb::Ctx const& c) {
                trace::Block t2("gelqf_panel_pack");
                lb::copy<T, T>(c, Uplo::General, Op::ConjTrans, nc, kb, rp, lda, Yk, ldy);
            });
            if (q == 1) {
                S.task(qP, {tPan}, {tPan, tP}, [&, nc, kb, Yk, ldy, Tk, slot](lb::Ctx const& c) {
                    trace::Block t2("gelqf_panel");
                    lb::geqrf_panel(c, nc, kb, Yk, ldy, Wtau[slot].data(), Tk, kb);
                });
            } else {
                std::vector<int64_t> cols_c(q, 0);
                for (int64_t j = k; j < nt; ++j) cols_c[A.scol_owner(j)] += A.tileNb(j);
                tsqr.enqueue(S, qP, rowF, qk, mycol, cols_c, Yk, ldy, nc, kb, kd, Tk, tPan, tP);
            }
            S.task(qP, {tPan}, {tPan, Sched::row(k)}, [&, kb, kd, nc, rp, Yk, ldy, diag](lb::Ctx const& c) {
                trace::Block t2("gelqf_panel_unpack");
                lb::copy<T, T>(c, Uplo::General, Op::ConjTrans, kb, nc, Yk, ldy, rp, lda);
                if (diag) lb::set(c, Uplo::Upper, std::min<int64_t>(kd, nc), kb, T(0), T(1), Yk, ldy);
            });
        }
        // ---- T_k along the panel's process row, then Y and T_k down the columns
        S.task(qP, {tP, tPan}, {tB}, [&, kb, kk, nc, pk, qk, Tk, Yk, in_row](lb::Ctx const& c) {
            trace::Block t2("gelqf_bcast");
            if (in_row && q > 1) bcast(rowF, Tk, size_t(kb * kb), qk, c);
            bcast(colF, Tk, size_t(kb * kb), pk, c);
            bcast(colF, Yk, size_t(nc * kb), pk, c);
            lb::copy2d(c, kb, kb, Tk, kb, tm + kk * ldt, ldt);
        });
        // ---- rows below: C := C - (C Y) T Y^H
        auto upd = [&, k, kb, nc, lc_k, Yk, Tk, ldy, slot](int queue, int64_t i0, int64_t i1, bool crit) {
            const int64_t r0 = lrow_of(A, i0), r1 = lrow_of(A, i1), mr = r1 - r0;
            std::vector<int64_t> rows;
            for (int64_t i = i0; i < i1; ++i) rows.push_back(Sched::row(i));
            // row chunk [r0, r1) of W / W2, contiguous (ld = mr) for the all-reduce
            T* W = WW[slot].data() + r0 * kb;
            T* W2 = WW2[slot].data() + r0 * kb;
            const int64_t ldw = std::max<int64_t>(mr, 1);
            T* C = a + r0 + lc_k * lda;
            S.task(queue, {tB}, rows, [&, mr, W, C](lb::Ctx const& c) {
                trace::Block t2("gelqf_update_w");
                if (mr <= 0) return;
                if (nc > 0) lb::gemm(c, Op::NoTrans, Op::NoTrans, mr, kb, nc, T(1), C, lda, Yk, ldy, T(0), W, ldw);
                else lb::set(c, Uplo::General, mr, kb, T(0), T(0), W, ldw);
            });
            if (q > 1) {
                Comm& cw = crit ? rowF : g.row();
                S.task(crit ? qP : qC, {}, rows, [&, mr, W](lb::Ctx const& c) {
                    trace::Block t2("gelqf_update_allreduce");
                    if (mr > 0) cw.allreduce(W, W, size_t(mr * kb), scalar_type<T>(), ReduceOp::Sum, c.loc(), c.stream);
                });
            }
            S.task(queue, {tB}, rows, [&, mr, W, W2, C](lb::Ctx const& c) {
                trace::Block t2("gelqf_update_c");
                if (mr <= 0) return;
                lb::gemm(c, Op::NoTrans, Op::NoTrans, mr, kb, kb, T(1), W, ldw, Tk, kb, T(0), W2, ldw);
                if (nc > 0) lb::gemm(c, Op::NoTrans, Op::ConjTrans, mr, nc, kb, T(-1), W2, ldw, Yk, ldy, T(1), C, lda);
            });
        };
        if (k + 1 < mt) {
            upd(device::kLookaheadQueue, k + 1, k + 2, true);
            if (k + 2 < mt) upd(device::kTrailQueue, k + 2, mt, false);
        }
    }
    S.wait_all();
    A.storage()->update_origin();
    Tf.storage()->update_origin();
}

/// C = op(Q) C with the gelqf factors, C's rows following A's COLUMNS (C on
/// A's transposed grid): Q = H_{kt-1}^H ... H_0^H, H_k = I - Y T Y^H.
/// NoTrans: k ascending with T^H; ConjTrans: k descending with T.  Per step
/// Y_k (the conj-transposed row panel, my local columns) goes down the
/// process columns of A, W = Y^H C is all-reduced across A's process row,
/// C -= Y (op(T) W).
template <typename T>
void unmlq_left(Op op, BaseMatrix<T> A, Matrix<T> const& Tf, Matrix<T>& C, Target target) {
    auto& g = *A.grid();
    const int mycol = g.mycol(), myrow = g.myrow();
    const Loc loc = loc_of(target);
    const int64_t kt = std::min(A.mt(), A.nt());
    LocalBlock<T> L = A.local(loc, false);
    LocalBlock<T> LC = C.local(loc, true);
    LocalBlock<T> LT = Tf.local(loc, false);
    const int64_t nb = A.nb(), nloc = L.n;
    Sched S(target);
    Work<T> Y(target, size_t(std::max<int64_t>(nloc, 1)) * nb), W(target, size_t(nb) * std::max<int64_t>(LC.n, 1)),
        W2(target, size_t(nb) * std::max<int64_t>(LC.n, 1));
    const int64_t tY = Sched::tok(40, 0), tC = Sched::tok(41, 0);
    for (int64_t t = 0; t < kt; ++t) {
        const int64_t k = (op == Op::NoTrans) ? t : kt - 1 - t;
        const int64_t kb = A.tileMb(k), kk = gcol_of(A, k), kd = std::min(kb, A.n() - kk);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const int64_t lc_k = lcol_of(A, k), nc = nloc - lc_k, ldy = std::max<int64_t>(nc, 1);
        const int64_t lcr = lrow_of(C, k);     // C's local rows >= kk (rows follow A's columns)
        S.task(1, {tC}, {tY}, [&, kb, kd, nc, lc_k, ldy, pk, qk](lb::Ctx const& c) {
            trace::Block t2("unmlq_bcast_y");
            if (myrow == pk) {
                lb::copy<T, T>(c, Uplo::General, Op::ConjTrans, nc, kb, L.ptr + lrow_of(A, k) + lc_k * L.ld, L.ld,
                               Y.data(), ldy);
                if (mycol == qk) lb::set(c, Uplo::Upper, std::min<int64_t>(kd, nc), kb, T(0), T(1), Y.data(), ldy);
            }
            bcast(g.col_fast(), Y.data(), size_t(nc * kb), pk, c);
        });
        S.task(0, {tY}, {tC}, [&, kb, kk, nc, ldy, lcr](lb::Ctx const& c) {
            trace::Block t2("unmlq_update");
            const int64_t ncC = LC.n;
            T* Cc = LC.ptr + lcr;
            if (nc > 0) lb::gemm(c, Op::ConjTrans, Op::NoTrans, kb, ncC, nc, T(1), Y.data(), ldy, Cc, LC.ld, T(0),
                                 W.data(), kb);
            else lb::set(c, Uplo::General, kb, ncC, T(0), T(0), W.data(), kb);
            if (g.q() > 1) g.row().allreduce(W.data(), W.data(), size_t(kb * ncC), scalar_type<T>(), ReduceOp::Sum,
                                             c.loc(), c.stream);
            lb::gemm(c, op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans, Op::NoTrans, kb, ncC, kb, T(1),
                     LT.ptr + kk * LT.ld, LT.ld, W.data(), kb, T(0), W2.data(), kb);
            if (nc > 0) lb::gemm(c, Op::NoTrans, Op::NoTrans, nc, ncC, kb, T(-1), Y.data(), ldy, W2.data(), kb, T(1),
                                 Cc, LC.ld);
        });
    }
    S.wait_all();
    C.storage()->update_origin();
}

/// C = C op(Q) with the gelqf factors when C's COLUMNS follow A's columns
/// (same grid, e.g. the trailing block of ge2tb): C H^(H) = C - (C Y) op(T)^.. Y^H
/// row-wise, with no transposed copy of C.  Q = H_{kt-1}^H ... H_0^H:
/// C Q applies k descending with T^H, C Q^H k ascending with T.  Per step:
/// Y_k down the process columns (fast lane), W = C Y all-reduced across the
/// process row, C -= (W op(T)) Y^H.
template <typename T>
void unmlq_right(Op op, BaseMatrix<T> A, Matrix<T> const& Tf, Matrix<T>& C, Target target) {
    auto& g = *A.grid();
    const int mycol = g.mycol(), myrow = g.myrow();
    const Loc loc = loc_of(target);
    const int64_t kt = std::min(A.mt(), A.nt());
    LocalBlock<T> L = A.local(loc, false);
    LocalBlock<T> LC = C.local(loc, true);
    LocalBlock<T> LT = Tf.local(loc, false);
    const int64_t nb = A.nb(), nloc = L.n, mrC = LC.m, ldw = std::max<int64_t>(mrC, 1);
    Sched S(target);
    Work<T> Y(target, size_t(std::max<int64_t>(nloc, 1)) * nb), W(target, size_t(ldw) * nb), W2(target, size_t(ldw) * nb);
    const int64_t tY = Sched::tok(40, 0), tC = Sched::tok(41, 0);
    for (int64_t t = 0; t < kt; ++t) {
        const int64_t k = (op == Op::NoTrans) ? kt - 1 - t : t;
        const int64_t kb = A.tileMb(k), kk = gcol_of(A, k), kd = std::min(kb, A.n() - kk);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const int64_t lc_k = lcol_of(A, k), nc = nloc - lc_k, ldy = std::max<int64_t>(nc, 1);
        const int64_t lcc = lcol_of(C, k);    // C's local columns >= kk
        S.task(1, {tC}, {tY}, [&, k, kb, kd, nc, lc_k, ldy, pk, qk](lb::Ctx const& c) {
            trace::Block t2("unmlq_bcast_y");
            if (myrow == pk) {
                lb::copy<T, T>(c, Uplo::General, Op::ConjTrans, nc, kb, L.ptr + lrow_of(A, k) + lc_k * L.ld, L.ld,
                               Y.data(), ldy);
                if (mycol == qk) lb::set(c, Uplo::Upper, std::min<int64_t>(kd, nc), kb, T(0), T(1), Y.data(), ldy);
            }
            bcast(g.col_fast(), Y.data(), size_t(nc * kb), pk, c);
        });
        S.task(0, {tY}, {tC}, [&, kb, kk, nc, ldy, lcc](lb::Ctx const& c) {
            trace::Block t2("unmlq_update_right");
            if (mrC <= 0) return;
            T* Cc = LC.ptr + lcc * LC.ld;
            if (nc > 0) lb::gemm(c, Op::NoTrans, Op::NoTrans, mrC, kb, nc, T(1), Cc, LC.ld, Y.data(), ldy, T(0),
                                 W.data(), ldw);
            else lb::set(c, Uplo::General, mrC, kb, T(0), T(0), W.data(), ldw);
            if (g.q() > 1) g.row().allreduce(W.data(), W.data(), size_t(ldw * kb), scalar_type<T>(), ReduceOp::Sum,
                                             c.loc(), c.stream);
            lb::gemm(c, Op::NoTrans, op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans, mrC, kb, kb, T(1), W.data(), ldw,
                     LT.ptr + kk * LT.ld, LT.ld, T(0), W2.data(), ldw);
            if (nc > 0) lb::gemm(c, Op::NoTrans, Op::ConjTrans, mrC, nc, kb, T(-1), W2.data(), ldw, Y.data(), ldy, T(1),
                                 Cc, LC.ld);
        });
    }
    S.wait_all();
    C.storage()->update_origin();
}

/// Do C's columns follow A's columns (same grid and column tiles)?
template <typename T>
bool cols_follow_cols(BaseMatrix<T> const& A, BaseMatrix<T> const& C) {
    auto& ga = *A.grid();
    auto& gc = *C.grid();
    if (C.op() != Op::NoTrans || !C.aligned() || !ga.same_processes(gc)) return false;
    if (gc.p() != ga.p() || gc.q() != ga.q() || gc.order() != ga.order()) return false;
    if (C.nt() != A.nt()) return false;
    for (int64_t j = 0; j < A.nt(); ++j)
        if (A.tileNb(j) != C.tileNb(j) || A.scol_owner(j) != C.scol_owner(j)) return false;
    return true;
}

/// Does C's row distribution follow A's columns (C on A's transposed grid)?
template <typename T>
bool rows_follow_cols(BaseMatrix<T> const& A, BaseMatrix<T> const& C) {
    auto& ga = *A.grid();
    auto& gc = *C.grid();
    if (C.op() != Op::NoTrans || !C.aligned() || !ga.same_processes(gc)) return false;
    if (gc.p() != ga.q() || gc.q() != ga.p() || (gc.size() > 1 && gc.order() == ga.order())) return false;
    if (C.mt() != A.nt()) return false;
    for (int64_t j = 0; j < A.nt(); ++j)
        if (A.tileNb(j) != C.tileMb(j) || A.scol_owner(j) != C.srow_owner(j)) return false;
    return true;
}

}  // namespace

template <typename T>
void gelqf(Matrix<T>& A, TriangularFactors<T>& T_, Options const& opts) {
    if (auto grp = internal::multi_group<T>({&A})) {
        std::vector<TriangularFactors<T>> Tr(grp->size());
        internal::spread<T>(opts, {{&A, true}}, [&](std::vector<Matrix<T>>& M, int r) {
            gelqf(M[0], Tr[r], opts);
        }, false);
        T_ = internal::factors_from_parts(grp, Tr);
        return;
    }
    if (A.arbitrary_layout()) {
        Matrix<T> Ab = internal::block_cyclic(A, opts);
        gelqf(Ab, T_, opts);
        slate::copy<T, T>(Ab, A, opts);
        return;
    }
    trace::Block tb("gelqf");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    slate_error_if_msg(A.op() != Op::NoTrans || !A.aligned() || A.mb() != A.nb(),
                       "gelqf: NoTrans, tile-aligned, square-tile matrix required");
    // T_k is tileMb(k) x tileMb(k) at column gcol(k): room for a full last tile
    Matrix<T> Tf(A.nb(), std::max<int64_t>(A.n(), 1) + A.nb(), A.nb(), A.nb(), Grid::self());
    Tf.insertLocalTiles(target);
    set(T(0), T(0), Tf, opts);
    gelqf_impl<T>(A, Tf, target);
    if (target == Target::Devices) lb::check_panel_errors();
    internal::finish_origin(A, opts);
    T_.clear();
    T_.push_back(Tf);
}

template <typename T>
void unmlq(Side side, Op op, Matrix<T> const& A, TriangularFactors<T> const& T_, Matrix<T>& C, Options const& opts) {
    if (internal::multi_group<T>({&A, &C})) {
        auto args = internal::with_factors<T>({{&A, false}, {&C, true}}, T_);
        internal::spread<T>(opts, args, [&](std::vector<Matrix<T>>& M, int) {
            TriangularFactors<T> Tr(M.begin() + 2, M.end());
            unmlq(side, op, M[0], Tr, M[1], opts);
        }, false);
        return;
    }
    if (A.arbitrary_layout()) {
        Matrix<T> Ab = internal::block_cyclic(A, opts);
        unmlq(side, op, Ab, T_, C, opts);
        return;
    }
    trace::Block tb("unmlq");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    slate_error_if_msg(T_.empty(), "unmlq: missing T factors");
    if (!is_complex_v<T> && op == Op::Trans) op = Op::ConjTrans;
    const Op opl = (op == Op::NoTrans) ? Op::NoTrans : Op::ConjTrans;
    GridPtr gt = A.grid()->transposed();
    const int rsrc = A.nt() ? A.scol_owner(0) : 0;
    if (side == Side::Left) {
        if (rows_follow_cols(A, C)) {
            unmlq_left<T>(opl, A, T_[0], C, target);
            internal::finish_origin(C, opts);
            return;
        }
        // C (n x nrhs) redistributed to follow A's columns -- never A
        Matrix<T> Cx(C.m(), C.n(), A.nb(), C.nb(), gt, rsrc, 0);
        Cx.insertLocalTiles(target);
        slate::copy<T, T>(C, Cx, opts);
        unmlq_left<T>(opl, A, T_[0], Cx, target);
        slate::copy<T, T>(Cx, C, opts);
        return;
    }
    if (cols_follow_cols(A, C)) {
        unmlq_right<T>(opl, A, T_[0], C, target);
        internal::finish_origin(C, opts);
        return;
    }
    // C op(Q) = (op(Q)^H C^H)^H
    Matrix<T> Cx(C.n(), C.m(), A.nb(), C.mb(), gt, rsrc, 0);
    Cx.insertLocalTiles(target);
    slate::copy<T, T>(conj_transpose(C), Cx, opts);
    unmlq_left<T>(opl == Op::NoTrans ? Op::ConjTrans : Op::NoTrans, A, T_[0], Cx, target);
    slate::copy<T, T>(conj_transpose(Cx), C, opts);
}

template <typename T>
void gels(Matrix<T>& A, TriangularFactors<T>& T_, Matrix<T>& BX, Options const& opts) {
    if (auto grp = internal::multi_group<T>({&A, &BX})) {
        std::vector<TriangularFactors<T>> Tr(grp->size());
        internal::spread<T>(opts, {{&A, true}, {&BX, true}}, [&](std::vector<Matrix<T>>& M, int r) {
            gels(M[0], Tr[r], M[1], opts);
        }, false);
        T_ = internal::factors_from_parts(grp, Tr);
        return;
    }
    trace::Block tb("gels");
    internal::DriverScope ds_;
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
    {
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}, {&R, true}}, [&](std::vector<Matrix<T>>& M, int r) {
                const int64_t i = cholqr(M[0], M[1], opts);
                if (r == 0) info = i;
            }, false))
            return info;
    }
    trace::Block tb("cholqr");
    internal::DriverScope ds_;
    // R^H R = A^H A ; Q = A R^{-1} (reference src/cholqr.cc:24-130).
    // Option::MethodCholQR picks how A^H A is formed: HerkC computes the upper
    // triangle only (half the flops; device default), GemmA / GemmC the full
    // product with the stationary-A or SUMMA gemm (host default GemmA).
    Target target = resolve_target(opts);
    Method method = get_option<int64_t>(opts, Option::MethodCholQR, MethodCholQR::Auto);
    if (method == MethodCholQR::Auto) method = MethodCholQR::select_algo(target);
    switch (method) {
        case MethodCholQR::HerkC: {
            HermitianMatrix<T> H(Uplo::Upper, R);
            herk(real_type<T>(1), conj_transpose(A), real_type<T>(0), H, opts);
            break;
        }
        case MethodCholQR::GemmA:
        case MethodCholQR::GemmC: {
            Options o2 = opts;
            o2[Option::MethodGemm] = int64_t(method == MethodCholQR::GemmA ? MethodGemm::GemmA : MethodGemm::GemmC);
            Matrix<T> Rg(R); Rg.set_uplo(Uplo::General);
            gemm(T(1), conj_transpose(A), A, T(0), Rg, o2);
            break;
        }
        default:
            slate_error("cholqr: unknown MethodCholQR");
    }
    HermitianMatrix<T> H(Uplo::Upper, R);
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
