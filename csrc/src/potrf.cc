// Distributed Cholesky factorization A = L L^H (reference src/potrf.cc:22-303).
//
// Per block column k (right-looking, lookahead `la`):
//   panel (queue 1):   potrf of A(k,k) on its owner; diag tile broadcast down
//                      the process column (comm queue); trsm of the local
//                      rows of A(k+1:,k) against L(k,k)^H.
//   bcast (comm queue): the local rows of L(k+1:,k) along the process row
//                      (one RCCL broadcast of a contiguous buffer), then the
//                      tiles each process column needs as the "transposed"
//                      operand, exchanged by one all-gather in the column
//                      communicator.
//   update:            lookahead columns k+1..k+la on their own queues,
//                      everything else as ONE trailing update on queue 0.
//                      On a 1x1 grid the trailing update is a single
//                      triangular-output MFMA GEMM (herk) over the whole
//                      trailing matrix.
//                      On a p x q grid (device, real types, nb % 128 == 0)
//                      every range is ONE staircase MFMA launch over the
//                      local lower-trapezoidal block (gemm_stair_real): the
//                      valid rows of each local column follow from the
//                      block-cyclic map, and each local tile column's B^T
//                      rows are read where the gathered panel keeps them.
// The reference instead issues one batched herk/gemm per tile group per
// step and syncs its queues after each op (internal_herk.cc:491-530).
#include "internal.hh"
#include "spread.hh"
#include "../kernels/kernels.hh"

#include <algorithm>
#include <numeric>

namespace slate {

namespace {

template <typename T>
int64_t potrf_lower(BaseMatrix<T> A, Target target, int64_t la) {
    using namespace internal;
    auto& g = *A.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t nt = A.nt();
    if (nt == 0) return 0;
    slate_error_if_msg(A.mb() != A.nb(), "potrf requires square tiles");
    slate_error_if_msg(!A.aligned(), "potrf requires a tile-aligned matrix");
    const int64_t nb = A.nb();

    LocalBlock<T> L = A.local(loc, true);
    T* a = L.ptr;
    const int64_t lda = L.ld, mloc = L.m;

    Sched S(target);
    const int R = int(std::max<int64_t>(2, la + 2));   // workspace ring depth
    // panel row-broadcast buffers and transposed-operand buffers
    std::vector<Work<T>> W(R), Wt(R), Dk(R), Ws(R);
    const int64_t lcm = std::lcm(int64_t(p), int64_t(q));
    const int64_t maxcnt = ceildiv(nt, lcm) + 1;
    // Transposed tiles arrive in two all-gathers: first the lookahead columns'
    // (a prefix of every process row's list: c1(k) tiles, region 1 of Wt),
    // so the next panel's update does not wait for the whole set; then the
    // rest (region 2).  Same layout on every rank of the process column.
    // SLATE_POTRF_SPLIT=0: one all-gather of every tile (round 5)
    static const bool split_env = [] {
        const char* e = std::getenv("SLATE_POTRF_SPLIT");
        return !e || std::atoi(e) != 0;
    }();
    const int64_t la_tiles = std::max<int64_t>(la, 1);
    const int64_t R1 = int64_t(p) * la_tiles * nb * nb;
    auto c1_of = [&](int64_t k) {
        int64_t c1 = 0;
        if (!split_env) return c1;
        std::vector<int64_t> cnt(p, 0);
        for (int64_t J = k + 1; J < std::min(nt, k + 1 + la); ++J)
            if (A.scol_owner(J) == mycol) c1 = std::max(c1, ++cnt[A.srow_owner(J)]);
        return c1;
    };
    // element offset in Wt of tile idx of process row r's list at step k
    auto toff = [&, R1](int64_t c1, int r, int64_t idx) -> int64_t {
        return idx < c1 ? (int64_t(r) * c1 + idx) * nb * nb : R1 + (int64_t(r) * (maxcnt - c1) + idx - c1) * nb * nb;
    };
    for (int r = 0; r < R; ++r) {
        if (q > 1) W[r].resize(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
        if (p > 1) {
            Wt[r].resize(target, size_t(R1) + size_t(p) * maxcnt * nb * nb);
            Ws[r].resize(target, size_t(maxcnt) * nb * nb);
            Dk[r].resize(target, size_t(nb) * nb);
        }
    }
    // ---- staircase single-launch updates on p x q > 1 (see header)
    // local row / column tile t of the view is view tile prow + t p / pcol + t q
    // on a block-cyclic layout; verified here, else the per-tile-column path
    const int64_t nloc = L.n;
    std::vector<int64_t> rtiles, ctiles;     // view tile of each local row / column tile
    for (int64_t i = 0; i < A.mt(); ++i) if (A.srow_owner(i) == myrow) rtiles.push_back(i);
    for (int64_t j = 0; j < nt; ++j) if (A.scol_owner(j) == mycol) ctiles.push_back(j);
    bool stair = (p * q > 1) && target == Target::Devices && !is_complex_v<T> && nb % 128 == 0;
    if (stair) {
        for (size_t t = 0; t < rtiles.size() && stair; ++t)
            stair = rtiles[t] == rtiles[0] + int64_t(t) * p && lrow_of(A, rtiles[t]) == int64_t(t) * nb &&
                    (rtiles[t] == A.mt() - 1 || A.tileMb(rtiles[t]) == nb);
        for (size_t t = 0; t < ctiles.size() && stair; ++t)
            stair = ctiles[t] == ctiles[0] + int64_t(t) * q && lcol_of(A, ctiles[t]) == int64_t(t) * nb &&
                    (ctiles[t] == nt - 1 || A.tileNb(ctiles[t]) == nb);
        stair = stair && (rtiles.empty() || rtiles[0] < p) && (ctiles.empty() || ctiles[0] < q);
    }
    const int prow0 = rtiles.empty() ? myrow : int(rtiles[0]), pcol0 = ctiles.empty() ? mycol : int(ctiles[0]);
    const int64_t nlt = int64_t(ctiles.size());
    // btab[k][t]: offset of local column tile t's B^T rows in step k's operand
    // (p == 1: rows of W_k, ld ldW; p > 1: tiles of the gathered Wt, ld nb)
    Work<int64_t> btab;
    if (stair && nlt > 0) {
        std::vector<int64_t> tab(size_t(nt) * nlt, 0);
        for (int64_t k = 0; k + 1 < nt; ++k) {
            const int64_t lr_k1 = lrow_of(A, k + 1), c1 = c1_of(k);
            std::vector<int64_t> seen(p, 0);
            for (int64_t J = k + 1; J < nt; ++J) {
                if (A.scol_owner(J) != mycol) continue;
                const int64_t t = (lcol_of(A, J)) / nb;
                const int r = A.srow_owner(J);
                tab[size_t(k) * nlt + t] = (p == 1) ? lrow_of(A, J) - lr_k1 : toff(c1, r, seen[r]);
                ++seen[r];
            }
        }
        btab.resize(target, tab.size());
        device::memcpy_async(btab.data(), tab.data(), tab.size() * sizeof(int64_t), S.ctx(1).stream);
        slate_hip_call(hipStreamSynchronize(S.ctx(1).stream));
    }
    (void)nloc;

    // Panel messages (diagonal tile down the column, L panel along the row,
    // transposed tiles over the column) are all on the critical path: they go
    // on the panel queue over the fast-lane (duplicate) communicators
    // (as getrf / geqrf), so step k+1's panel chain is one stream with no
    // cross-queue hops; SLATE_POTRF_COMM_QUEUE=1 keeps them on the comm queue.
    static const bool comm_q_env = [] {
        const char* e = std::getenv("SLATE_POTRF_COMM_QUEUE");
        return e && std::atoi(e) != 0;
    }();
    const bool fast = !comm_q_env;   // (the fast comms alias row() / col() without a duplicate)
    const int qM = fast ? 1 : device::kCommQueue;
    Comm& rowM = fast ? g.row_fast() : g.row();
    Comm& colM = fast ? g.col_fast() : g.col();

    Work<int> dinfo(target, 1);
    {
        lb::Ctx c0 = S.ctx(1);
        if (c0.dev()) device::memset_async(dinfo.data(), 0, sizeof(int), c0.stream);
        else dinfo.data()[0] = 0;
    }

    // 1x1 device grid: once the remaining matrix is at most `tail` wide, factor
    // it with ONE recursive device potrf (local_blas.cc: 64-column leaves,
    // two launches each) instead of nb-wide steps, whose per-step panel,
    // trsm and lookahead hops dominate when the trailing update has shrunk to
    // a few hundred microseconds.  SLATE_POTRF_TAIL = width (0: off); config 2
    // (n = 32768, nb = 512): round 4 237.4 ms at 0, 234.2 at 4096, 233.0 at
    // 8192; round 5 (leaf kernels) 4096 214.0-214.7 ms against 215.2-216.2 at
    // 8192 and 248-250 at 16384 (profiles/r5_potrf_tail_ab.txt).
    static const int64_t tail_env = [] {
        const char* e = std::getenv("SLATE_POTRF_TAIL");
        return e ? std::atoll(e) : int64_t(4096);
    }();
    const bool tail_ok = p * q == 1 && target == Target::Devices && tail_env > 0;
    for (int64_t k = 0; k < nt; ++k) {
        const int64_t kb = A.tileNb(k);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        if (tail_ok && k > 0 && A.n() - grow_of(A, k) <= std::max(tail_env, nb)) {
            const int64_t kk0 = grow_of(A, k), rest = A.n() - kk0;
            std::vector<int64_t> cols;
            for (int64_t j = k; j < nt; ++j) cols.push_back(Sched::col(j));
            T* akk0 = a + lrow_of(A, k) + lcol_of(A, k) * lda;
            S.task(1, cols, cols, [&, akk0, rest, kk0](lb::Ctx const& c) {
                trace::Block tb("potrf_tail");
                lb::potrf(c, Uplo::Lower, rest, akk0, lda, dinfo.data(), kk0);
            });
            break;
        }
        const int64_t lr_k = lrow_of(A, k), lr_k1 = lrow_of(A, k + 1);
        const int64_t mrows = mloc - lr_k1;
        const int slot = int(k % R);
        const int64_t kk = grow_of(A, k);
        const bool in_col = (mycol == qk);
        const int64_t lc_k = in_col ? lcol_of(A, k) : 0;
        T* akk = a + lr_k + lc_k * lda;          // diag tile (if mine)
        T* apan = a + lr_k1 + lc_k * lda;        // my rows below the diagonal

        const int64_t tDiag = Sched::tok(5, slot), tBc = Sched::bcast(slot), tLa = Sched::tok(6, slot);

        // ---- panel: potrf(A(k,k))
        if (in_col && myrow == pk) {
            S.task(1, {}, {Sched::col(k)}, [&, akk, kb, kk](lb::Ctx const& c) {
                trace::Block tb("potrf_diag");
                lb::potrf(c, Uplo::Lower, kb, akk, lda, dinfo.data(), kk);
            });
        }
        // ---- diag tile down the process column
        T* Lkk = akk;
        int64_t ldL = lda;
        if (in_col && p > 1) {
            T* D = Dk[slot].data();
            S.task(qM, {Sched::col(k)}, {tDiag}, [&, D, akk, kb, pk](lb::Ctx const& c) {
                trace::Block tb("bcast_diag");
                if (myrow == pk) pack(c, kb, kb, akk, lda, D);
                bcast(colM, D, size_t(kb * kb), pk, c);
            });
            Lkk = D; ldL = kb;
        }
        // ---- panel trsm: A(k+1:, k) = A(k+1:, k) L(k,k)^{-H}
        if (in_col && mrows > 0) {
            S.task(1, {tDiag}, {Sched::col(k)}, [&, Lkk, ldL, apan, mrows, kb](lb::Ctx const& c) {
                trace::Block tb("potrf_trsm");
                lb::trsm(c, Side::Right, Uplo::Lower, Op::ConjTrans, Diag::NonUnit, mrows, kb, T(1),
                         Lkk, ldL, apan, lda);
            });
        }
        if (k == nt - 1) break;

        // ---- broadcast the panel along process rows, transposed tiles along columns
        T* Wk = (q > 1) ? W[slot].data() : apan;
        const int64_t ldW = (q > 1) ? std::max<int64_t>(mrows, 1) : lda;
        // tiles J > k that my process column needs, grouped by owning process row
        std::vector<std::vector<int64_t>> lists(p);
        for (int64_t J = k + 1; J < nt; ++J)
            if (A.scol_owner(J) == mycol) lists[A.srow_owner(J)].push_back(J);
        const int64_t c1 = p > 1 ? c1_of(k) : 0;
        // pack my tiles [i0, i1) of my list (rows of Wk) and all-gather them
        auto gather_t = [&, Wk, ldW, kb, slot, lists, lr_k1](lb::Ctx const& c, int64_t i0, int64_t i1, T* dst) {
            if (i1 <= i0) return;
            T* Sb = Ws[slot].data();
            auto const& mine = lists[myrow];
            for (int64_t i = i0; i < std::min<int64_t>(i1, int64_t(mine.size())); ++i) {
                const int64_t J = mine[size_t(i)];
                lb::copy2d(c, A.tileMb(J), kb, Wk + (lrow_of(A, J) - lr_k1), ldW, Sb + (i - i0) * nb * nb, nb);
            }
            colM.allgather(Sb, dst, size_t((i1 - i0) * nb * nb), scalar_type<T>(), c.loc(), c.stream);
        };
        // (tBc as an output too: the slot's W / Wt reuse waits for step k - R's trailing readers)
        S.task(qM, {Sched::col(k)}, {tLa, tBc}, [&, Wk, apan, mrows, kb, qk, slot, c1, gather_t](lb::Ctx const& c) {
            trace::Block tb("bcast_panel");
            if (q > 1) {
                if (mycol == qk) pack(c, mrows, kb, apan, lda, Wk);
                bcast(rowM, Wk, size_t(mrows * kb), qk, c);
            }
            if (p > 1 && split_env) gather_t(c, 0, c1, Wt[slot].data());    // the lookahead columns' tiles
            if (p > 1 && !split_env) gather_t(c, 0, maxcnt, Wt[slot].data() + R1);
        });
        if (p > 1 && split_env) {
            S.task(qM, {tLa}, {tBc}, [&, slot, c1, gather_t, R1](lb::Ctx const& c) {
                trace::Block tb("bcast_transposed");
                gather_t(c, c1, maxcnt, Wt[slot].data() + R1);   // the rest
            });
        }

        // ---- trailing updates
        auto update = [&, Wk, ldW, kb, slot, lists, lr_k1, k](lb::Ctx const& c, int64_t j0, int64_t j1) {
            trace::Block tb("potrf_update");
            if (stair && c.dev()) {
                if constexpr (!is_complex_v<T>) {
                    const int64_t c0 = lcol_of(A, j0), nc = lcol_of(A, j1) - c0;
                    const int64_t r0 = lrow_of(A, j0), nrows = mloc - r0;
                    if (nc <= 0 || nrows <= 0) return;
                    slate_amd::dev::StairMap sm;
                    sm.btab = btab.data() + k * nlt + c0 / nb;
                    sm.c0 = c0; sm.r0 = r0; sm.nb = int(nb); sm.p = p; sm.q = q; sm.prow = prow0; sm.pcol = pcol0;
                    const T* Bb = (p == 1) ? Wk : Wt[slot].data();
                    slate_amd::dev::gemm_stair_real<T>(nrows, nc, kb, T(-1), Wk + (r0 - lr_k1), ldW, Bb,
                                                       p == 1 ? ldW : nb, sm, T(1), a + r0 + c0 * lda, lda, c.stream);
                }
                return;
            }
            // fast path: 1x1 grid, contiguous range -> one herk over [j0, j1) x [j0, ...)
            if (p == 1 && q == 1) {
                int64_t r0 = lrow_of(A, j0), c0 = lcol_of(A, j0), c1 = lcol_of(A, j1);
                int64_t ncols = c1 - c0, nrows = mloc - r0;
                T const* Wr = Wk + (r0 - lr_k1);
                // diagonal square block: herk; rows below: gemm
                lb::herk(c, Uplo::Lower, Op::NoTrans, ncols, kb, real_type<T>(-1), Wr, ldW, real_type<T>(1),
                         a + r0 + c0 * lda, lda);
                if (nrows > ncols)
                    lb::gemm(c, Op::NoTrans, Op::ConjTrans, nrows - ncols, ncols, kb, T(-1), Wr + ncols, ldW,
                             Wr, ldW, T(1), a + r0 + ncols + c0 * lda, lda);
                return;
            }
            for (int64_t J = j0; J < j1; ++J) {
                if (A.scol_owner(J) != mycol) continue;
                int64_t jb = A.tileNb(J);
                int64_t rJ = lrow_of(A, J), cJ = lcol_of(A, J);
                int64_t nrows = mloc - rJ;
                if (nrows <= 0) continue;
                // transposed operand L(J, k): jb x kb
                T const* Bt; int64_t ldB;
                if (p == 1) { Bt = Wk + (lrow_of(A, J) - lr_k1); ldB = ldW; }
                else {
                    int r = A.srow_owner(J);
                    auto const& lst = lists[r];
                    int64_t idx = std::find(lst.begin(), lst.end(), J) - lst.begin();
                    Bt = Wt[slot].data() + toff(c1_of(k), r, idx); ldB = nb;
                }
                T const* Ar = Wk + (rJ - lr_k1);
                T* Cc = a + rJ + cJ * lda;
                if (A.srow_owner(J) == myrow) {
                    // diagonal tile is local: herk on it, gemm below
                    lb::gemm_tri(c, Uplo::Lower, Op::NoTrans, Op::ConjTrans, jb, kb, T(-1), Ar, ldW, Bt, ldB, T(1), Cc, lda);
                    if (nrows > jb)
                        lb::gemm(c, Op::NoTrans, Op::ConjTrans, nrows - jb, jb, kb, T(-1), Ar + jb, ldW, Bt, ldB,
                                 T(1), Cc + jb, lda);
                } else {
                    lb::gemm(c, Op::NoTrans, Op::ConjTrans, nrows, jb, kb, T(-1), Ar, ldW, Bt, ldB, T(1), Cc, lda);
                }
            }
        };
        int64_t jla_end = std::min(nt, k + 1 + la);
        for (int64_t j = k + 1; j < jla_end; ++j) {
            int qi = device::kLookaheadQueue;
            S.task(qi, {tLa}, {Sched::col(j)}, [&, update, j](lb::Ctx const& c) { update(c, j, j + 1); });
        }
        if (jla_end < nt) {
            std::vector<int64_t> outs;
            for (int64_t j = jla_end; j < nt; ++j) outs.push_back(Sched::col(j));
            S.task(device::kTrailQueue, {tBc}, outs, [&, update, jla_end](lb::Ctx const& c) { update(c, jla_end, nt); });
        }
    }
    S.wait_all();
    int64_t info = fetch_info(target, dinfo.data());
    return reduce_info(info, g.world());
}

/// Upper storage A = U^H U, in place (the reference factors the conjugate
/// transpose as a shallow view, potrf.cc:45-47; here the mirror of
/// potrf_lower with block ROWS): per step the diagonal tile along process
/// row pk, the row panel U(k, k+1:) = U(k,k)^{-H} A(k, k+1:) solved there
/// and broadcast down the process columns, the tiles U(k, I) each process
/// needs for its local ROWS all-gathered over the process row, and the upper
/// trapezoid of every local column range updated by C -= U(k, rows)^H
/// U(k, cols) (on a 1 x 1 grid one herk + one gemm per range).
template <typename T>
int64_t potrf_upper(BaseMatrix<T> A, Target target, int64_t la) {
    using namespace internal;
    auto& g = *A.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t nt = A.nt();
    if (nt == 0) return 0;
    slate_error_if_msg(A.mb() != A.nb(), "potrf requires square tiles");
    slate_error_if_msg(!A.aligned(), "potrf requires a tile-aligned matrix");
    const int64_t nb = A.nb();
    LocalBlock<T> L = A.local(loc, true);
    T* a = L.ptr;
    const int64_t lda = L.ld, nloc = L.n;
    Sched S(target);
    const int R = int(std::max<int64_t>(2, la + 2));
    std::vector<Work<T>> W(R), Wt(R), Dk(R), Ws(R), X(R);
    const int64_t lcm = std::lcm(int64_t(p), int64_t(q));
    const int64_t maxcnt = ceildiv(nt, lcm) + 1;
    const int64_t mloc = L.m;
    for (int r = 0; r < R; ++r) {
        if (p > 1) W[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
        if (q > 1) {
            Wt[r].resize(target, size_t(q) * maxcnt * nb * nb);
            Ws[r].resize(target, size_t(maxcnt) * nb * nb);
            Dk[r].resize(target, size_t(nb) * nb);
        }
        if (p * q > 1) X[r].resize(target, size_t(nb) * std::max<int64_t>(mloc, 1));
    }
    Work<int> dinfo(target, 1);
    {
        lb::Ctx c0 = S.ctx(1);
        if (c0.dev()) device::memset_async(dinfo.data(), 0, sizeof(int), c0.stream);
        else dinfo.data()[0] = 0;
    }
    for (int64_t k = 0; k < nt; ++k) {
        const int64_t kb = A.tileNb(k);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const int64_t lr_k = lrow_of(A, k), lr_k1 = lrow_of(A, k + 1);
        const int64_t lc_k1 = lcol_of(A, k + 1), ncols = nloc - lc_k1;
        const int slot = int(k % R);
        const int64_t kk = grow_of(A, k);
        const bool in_row = (myrow == pk);
        const int64_t lc_k = (mycol == qk) ? lcol_of(A, k) : 0;
        T* akk = a + lr_k + lc_k * lda;
        T* apan = a + lr_k + lc_k1 * lda;     // my columns right of the diagonal, row k
        const int64_t tDiag = Sched::tok(5, slot), tBc = Sched::bcast(slot);
        if (in_row && mycol == qk)
            S.task(1, {}, {Sched::row(k)}, [&, akk, kb, kk](lb::Ctx const& c) {
                trace::Block tb("potrf_diag");
                lb::potrf(c, Uplo::Upper, kb, akk, lda, dinfo.data(), kk);
            });
        T* Ukk = akk;
        int64_t ldU = lda;
        if (in_row && q > 1) {
            T* D = Dk[slot].data();
            S.task(1, {Sched::row(k)}, {tDiag}, [&, D, akk, kb, qk](lb::Ctx const& c) {
                trace::Block tb("bcast_diag");
                if (mycol == qk) pack(c, kb, kb, akk, lda, D);
                bcast(g.row_fast(), D, size_t(kb * kb), qk, c);
            });
            Ukk = D; ldU = kb;
        }
        if (in_row && ncols > 0)
            S.task(1, {tDiag}, {Sched::row(k)}, [&, Ukk, ldU, apan, ncols, kb](lb::Ctx const& c) {
                trace::Block tb("potrf_trsm");
                lb::trsm(c, Side::Left, Uplo::Upper, Op::ConjTrans, Diag::NonUnit, kb, ncols, T(1), Ukk, ldU, apan, lda);
            });
        if (k == nt - 1) break;
        // row panel down the process columns; the tiles of my local rows over the row
        T* Wk = (p > 1) ? W[slot].data() : apan;
        const int64_t ldW = (p > 1) ? kb : lda;
        std::vector<std::vector<int64_t>> lists(q);     // tiles I > k of my process ROW, by column owner
        for (int64_t I = k + 1; I < nt; ++I)
            if (A.srow_owner(I) == myrow) lists[A.scol_owner(I)].push_back(I);
        T* Xk = (p * q > 1) ? X[slot].data() : nullptr;   // U(k, my rows > k) as kb x rows
        S.task(1, {Sched::row(k)}, {tBc}, [&, Wk, ldW, apan, ncols, kb, pk, slot, lists, Xk, lr_k1](lb::Ctx const& c) {
            trace::Block tb("bcast_panel");
            if (p > 1) {
                if (in_row) lb::copy2d(c, kb, ncols, apan, lda, Wk, ldW);
                bcast(g.col_fast(), Wk, size_t(kb * ncols), pk, c);
            }
            if (Xk) {
                if (q > 1) {
                    // my column tiles J that row owner r needs: pack, all-gather over the row
                    T* Sb = Ws[slot].data();
                    int64_t cnt = 0;
                    for (int64_t J = k + 1; J < nt; ++J) {
                        if (A.scol_owner(J) != mycol || A.srow_owner(J) != myrow) continue;
                        lb::copy2d(c, kb, A.tileNb(J), Wk + (lcol_of(A, J) - lc_k1) * ldW, ldW, Sb + cnt * nb * nb, kb);
                        ++cnt;
                    }
                    g.row_fast().allgather(Sb, Wt[slot].data(), size_t(maxcnt * nb * nb), scalar_type<T>(), c.loc(),
                                           c.stream);
                    for (int cc = 0; cc < q; ++cc)
                        for (size_t t = 0; t < lists[cc].size(); ++t) {
                            const int64_t I = lists[cc][t];
                            lb::copy2d(c, kb, A.tileMb(I), Wt[slot].data() + (int64_t(cc) * maxcnt + int64_t(t)) * nb * nb,
                                       kb, Xk + (lrow_of(A, I) - lr_k1) * kb, kb);
                        }
                } else {
                    // q == 1: my columns are every column; my rows' tiles sit in Wk
                    for (int64_t I = k + 1; I < nt; ++I)
                        if (A.srow_owner(I) == myrow)
                            lb::copy2d(c, kb, A.tileMb(I), Wk + (lcol_of(A, I) - lc_k1) * ldW, ldW,
                                       Xk + (lrow_of(A, I) - lr_k1) * kb, kb);
                }
            }
        });
        // trailing update by ROW tiles [i0, i1) (the mirror of the lower
        // factor's column lookahead: step k+1's panel needs block ROW k+1
        // across every column, so the rows k+1 .. k+la go first on the
        // lookahead queue, the rest on the trailing queue): for each row tile
        // I, C(I, J > I) -= U(k, I)^H U(k, J) and the upper triangle of C(I, I)
        auto update = [&, Wk, ldW, Xk, kb, lr_k1, lc_k1](lb::Ctx const& c, int64_t i0, int64_t i1) {
            trace::Block tb("potrf_update");
            if (p * q == 1) {
                const int64_t r0 = lrow_of(A, i0), r1 = lrow_of(A, i1), nr = r1 - r0, nright = nloc - r1;
                T const* Wr = Wk + (r0 - lc_k1) * ldW;
                lb::herk(c, Uplo::Upper, Op::ConjTrans, nr, kb, real_type<T>(-1), Wr, ldW, real_type<T>(1),
                         a + r0 + r0 * lda, lda);
                if (nright > 0)
                    lb::gemm(c, Op::ConjTrans, Op::NoTrans, nr, nright, kb, T(-1), Wr, ldW, Wk + (r1 - lc_k1) * ldW,
                             ldW, T(1), a + r0 + r1 * lda, lda);
                return;
            }
            for (int64_t I = i0; I < i1; ++I) {
                if (A.srow_owner(I) != myrow) continue;
                const int64_t ib = A.tileMb(I), rI = lrow_of(A, I);
                T const* XI = Xk + (rI - lr_k1) * kb;
                const int64_t cR = lcol_of(A, I + 1), nright = nloc - cR;
                if (nright > 0)
                    lb::gemm(c, Op::ConjTrans, Op::NoTrans, ib, nright, kb, T(-1), XI, kb, Wk + (cR - lc_k1) * ldW, ldW,
                             T(1), a + rI + cR * lda, lda);
                if (A.scol_owner(I) == mycol) {
                    const int64_t cI = lcol_of(A, I);
                    lb::gemm_tri(c, Uplo::Upper, Op::ConjTrans, Op::NoTrans, ib, kb, T(-1), XI, kb,
                                 Wk + (cI - lc_k1) * ldW, ldW, T(1), a + rI + cI * lda, lda);
                }
            }
        };
        const int64_t ila_end = std::min(nt, k + 1 + la);
        for (int64_t i = k + 1; i < ila_end; ++i)
            S.task(device::kLookaheadQueue, {tBc}, {Sched::row(i)}, [&, update, i](lb::Ctx const& c) { update(c, i, i + 1); });
        if (ila_end < nt) {
            std::vector<int64_t> outs;
            for (int64_t i = ila_end; i < nt; ++i) outs.push_back(Sched::row(i));
            S.task(device::kTrailQueue, {tBc}, outs, [&, update, ila_end](lb::Ctx const& c) { update(c, ila_end, nt); });
        }
    }
    S.wait_all();
    int64_t info = fetch_info(target, dinfo.data());
    return reduce_info(info, g.world());
}

}  // namespace

template <typename T>
int64_t potrf(HermitianMatrix<T>& A_in, Options const& opts) {
    {   // one process, several GPUs: in-process ranks (spread.hh)
        int64_t info = 0;
        const Uplo u = A_in.uplo();
        if (internal::spread<T>(opts, {{&A_in, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
                HermitianMatrix<T> H(u, M[0]);
                const int64_t i = potrf(H, opts);
                if (rank == 0) info = i;
            }))
            return info;
    }
    if (A_in.arbitrary_layout()) {
        HermitianMatrix<T> Ab(A_in.uplo(), internal::block_cyclic(A_in, opts));
        int64_t info = potrf(Ab, opts);
        slate::copy<T, T>(Ab, A_in, opts);
        return info;
    }
    trace::Block tb("potrf");
    internal::DriverScope ds_;
    Target target = internal::resolve_target(opts);
    int64_t la = get_option<int64_t>(opts, Option::Lookahead, 1);
    BaseMatrix<T> A = A_in;
    if (A.op() != Op::NoTrans) A = A.transpose_view(A.op() == Op::ConjTrans);  // physical view
    int64_t info;
    if (A_in.uplo_physical() == Uplo::Lower) {
        info = potrf_lower(A, target, la);
    } else {
        info = potrf_upper(A, target, la);   // in place, no transposed copy
    }
    internal::finish_origin(A, opts);
    return info;
}

template int64_t potrf<float>(HermitianMatrix<float>&, Options const&);
template int64_t potrf<double>(HermitianMatrix<double>&, Options const&);
template int64_t potrf<std::complex<float>>(HermitianMatrix<std::complex<float>>&, Options const&);
template int64_t potrf<std::complex<double>>(HermitianMatrix<std::complex<double>>&, Options const&);

}  // namespace slate
