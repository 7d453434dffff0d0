// Distributed LU factorization with partial pivoting (reference src/getrf.cc,
// src/getrf_tntpiv.cc, src/getrf_nopiv.cc, src/internal/internal_swap.cc).
//
// Per block column k:
//   panel (queue 1): the whole m x nb panel is factored ON THE DEVICE by the
//     recursive LU kernel (device pivot search, in-kernel row swaps across the
//     panel, trsm/gemm recursion) -- no host round trip per column.  With
//     p = 1 the panel is local to its process column.  With p > 1 the panel
//     rows are gathered to the diagonal process over the column communicator,
//     factored there and scattered back (exact partial pivoting).
//   The panel's row permutation is turned into (dst, src) row pairs on the
//   device; they travel with the pivots in one broadcast, and every process
//   permutes its local columns with ONE gather/scatter kernel per column
//   range (column-major rows are moved whole), instead of the reference's one
//   blas::swap per pivot (internal_swap.cc:674).
//   U row: trsm on process row pk, broadcast down columns; trailing update
//   A22 -= L21 U12 as one MFMA GEMM per process; lookahead columns on their
//   own queues.
// getrf_tntpiv (CALU) shares this driver: its panel (gathered to the diagonal
// process when p > 1) selects the pivots of every 32-column narrow block by a
// tournament over 256-row leaves on the device (kernels/tslu.hip), then
// factors that block without further pivoting.
#include "internal.hh"
#include "../kernels/kernels.hh"

#include <algorithm>
#include <numeric>
#include <unordered_map>

namespace slate {

using namespace internal;

namespace {

/// Global row permutation pairs (dst <- src), both view-relative row indices.
struct RowPairs {
    std::vector<int64_t> dst, src;
    size_t size() const { return dst.size(); }
};

/// Sequential interchanges ipiv (global, view-relative, applied in order for
/// rows r0, r0+1, ...) -> (dst, src) pairs of the resulting permutation.
RowPairs pairs_from_ipiv(int64_t r0, std::vector<int64_t> const& ipiv) {
    std::unordered_map<int64_t, int64_t> pos;   // row -> original row now there
    auto get = [&](int64_t r) { auto it = pos.find(r); return it == pos.end() ? r : it->second; };
    for (size_t t = 0; t < ipiv.size(); ++t) {
        int64_t a = r0 + int64_t(t), b = ipiv[t];
        if (a == b) continue;
        int64_t va = get(a), vb = get(b);
        pos[a] = vb; pos[b] = va;
    }
    RowPairs P;
    for (auto& kv : pos)
        if (kv.first != kv.second) { P.dst.push_back(kv.first); P.src.push_back(kv.second); }
    return P;
}

/// Apply row pairs to the local columns [c0, c1) of view A (rows distributed
/// over the column communicator).  Synchronous.  Reads all sources before
/// writing any destination.
template <typename T>
void permute_rows_dist(BaseMatrix<T> const& A, RowPairs const& P, int64_t c0, int64_t c1, lb::Ctx const& c) {
    auto& s = *A.storage();
    auto& g = *s.grid;
    const int p = g.p(), me = g.myrow();
    const int64_t ncols = c1 - c0;
    if (P.size() == 0) return;
    LocalBlock<T> la = A.local_raw(c.loc());
    auto owner_row = [&](int64_t gr) { return s.row_owner((A.row0() + gr) / s.mb); };
    auto lrow = [&](int64_t gr) { return g2l(A.row0() + gr, s.mb, p) - A.lrow_begin(); };
    // every process walks the pair list in the same order
    std::vector<std::vector<int64_t>> send_src(p), recv_dst(p);
    std::vector<int64_t> loc_src, loc_dst;
    for (size_t t = 0; t < P.size(); ++t) {
        int od = owner_row(P.dst[t]), os = owner_row(P.src[t]);
        if (od == me && os == me) { loc_src.push_back(P.src[t]); loc_dst.push_back(P.dst[t]); }
        else if (os == me) send_src[od].push_back(P.src[t]);
        else if (od == me) recv_dst[os].push_back(P.dst[t]);
    }
    size_t nsend = 0, nrecv = 0;
    for (int r = 0; r < p; ++r) { nsend += send_src[r].size(); nrecv += recv_dst[r].size(); }
    size_t nloc = loc_src.size();
    Work<T> buf(c.dev() ? Target::Devices : Target::HostTask, std::max<size_t>(1, (nsend + nrecv + nloc) * std::max<int64_t>(ncols, 1)));
    T* sb = buf.data();
    T* lb_ = sb + nsend * ncols;
    T* rb = lb_ + nloc * ncols;
    // row lists: send rows (grouped by destination), local moves, received rows
    std::vector<int64_t> snd, lsrc, ldst, rcv;
    for (int r = 0; r < p; ++r) for (int64_t gr : send_src[r]) snd.push_back(lrow(gr));
    for (size_t t = 0; t < nloc; ++t) { lsrc.push_back(lrow(loc_src[t])); ldst.push_back(lrow(loc_dst[t])); }
    for (int r = 0; r < p; ++r) for (int64_t gr : recv_dst[r]) rcv.push_back(lrow(gr));
    T* Ablk = la.ptr + c0 * la.ld;
    // packed buffers are (rows x ncols) with ld = rows: message r is then not
    // contiguous, so pack per destination / source block into its own slab
    if (c.dev()) {
        Work<int64_t> didx(Target::Devices, std::max<size_t>(1, snd.size() + 2 * nloc + rcv.size()));
        std::vector<int64_t> all;
        all.insert(all.end(), snd.begin(), snd.end());
        all.insert(all.end(), lsrc.begin(), lsrc.end());
        all.insert(all.end(), ldst.begin(), ldst.end());
        all.insert(all.end(), rcv.begin(), rcv.end());
        if (!all.empty()) device::memcpy_async(didx.data(), all.data(), all.size() * sizeof(int64_t), c.stream);
        int64_t* d_snd = didx.data();
        int64_t* d_lsrc = d_snd + snd.size();
        int64_t* d_ldst = d_lsrc + nloc;
        int64_t* d_rcv = d_ldst + nloc;
        using DT = slate_amd::dev::dev_t<T>;
        auto pk = [&](int64_t* idx, size_t cnt, T* buf, bool scat) {
            if (cnt) slate_amd::dev::rows_pack<DT>(ncols, slate_amd::dev::dptr(Ablk), la.ld, idx, int(cnt),
                                                   slate_amd::dev::dptr(buf), scat, c.stream);
        };
        // per-peer slabs so each message is contiguous
        size_t so = 0;
        for (int r = 0; r < p; ++r) { pk(d_snd + so, send_src[r].size(), sb + so * ncols, false); so += send_src[r].size(); }
        pk(d_lsrc, nloc, lb_, false);
        if (p > 1 && ncols > 0) {
            std::vector<Comm::P2P> ops;
            size_t s2 = 0, r2 = 0;
            for (int r = 0; r < p; ++r) {
                if (!send_src[r].empty()) ops.push_back({sb + s2 * ncols, send_src[r].size() * ncols, r, true});
                s2 += send_src[r].size();
            }
            for (int r = 0; r < p; ++r) {
                if (!recv_dst[r].empty()) ops.push_back({rb + r2 * ncols, recv_dst[r].size() * ncols, r, false});
                r2 += recv_dst[r].size();
            }
            g.col().exchange(ops, scalar_type<T>(), c.loc(), c.stream);
        }
        pk(d_ldst, nloc, lb_, true);
        size_t ro = 0;
        for (int r = 0; r < p; ++r) { pk(d_rcv + ro, recv_dst[r].size(), rb + ro * ncols, true); ro += recv_dst[r].size(); }
        slate_hip_call(hipStreamSynchronize(c.stream));
        return;
    }
    // host: same slab layout, plain loops
    auto hpk = [&](int64_t const* idx, size_t cnt, T* buf, bool scat) {
        for (int64_t j = 0; j < ncols; ++j)
            for (size_t t = 0; t < cnt; ++t) {
                T& a = Ablk[idx[t] + j * la.ld];
                T& b = buf[t + j * cnt];
                if (scat) a = b; else b = a;
            }
    };
    size_t so = 0;
    for (int r = 0; r < p; ++r) { hpk(snd.data() + so, send_src[r].size(), sb + so * ncols, false); so += send_src[r].size(); }
    hpk(lsrc.data(), nloc, lb_, false);
    if (p > 1 && ncols > 0) {
        std::vector<Comm::P2P> ops;
        size_t s2 = 0, r2 = 0;
        for (int r = 0; r < p; ++r) {
            if (!send_src[r].empty()) ops.push_back({sb + s2 * ncols, send_src[r].size() * ncols, r, true});
            s2 += send_src[r].size();
        }
        for (int r = 0; r < p; ++r) {
            if (!recv_dst[r].empty()) ops.push_back({rb + r2 * ncols, recv_dst[r].size() * ncols, r, false});
            r2 += recv_dst[r].size();
        }
        g.col().exchange(ops, scalar_type<T>(), c.loc(), c.stream);
    }
    hpk(ldst.data(), nloc, lb_, true);
    size_t ro = 0;
    for (int r = 0; r < p; ++r) { hpk(rcv.data() + ro, recv_dst[r].size(), rb + ro * ncols, true); ro += recv_dst[r].size(); }
}

enum class PanelMode { Partial, Tournament, NoPiv };

template <typename T>
int64_t getrf_impl(Matrix<T>& A_in, Pivots& pivots, Options const& opts, PanelMode mode) {
    trace::Block tb("getrf");
    Target target = resolve_target(opts);
    const int64_t la = get_option<int64_t>(opts, Option::Lookahead, 1);
    slate_error_if_msg(A_in.op() != Op::NoTrans, "getrf: NoTrans view required");
    slate_error_if_msg(!A_in.aligned(), "getrf: tile-aligned matrix required");
    slate_error_if_msg(A_in.mb() != A_in.nb(), "getrf: square tiles required");
    BaseMatrix<T> A = A_in;
    auto& g = *A.grid();
    const int p = g.p(), q = g.q(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t mt = A.mt(), nt = A.nt(), m = A.m(), n = A.n();
    const int64_t kt = std::min(mt, nt);
    const int64_t nb = A.nb();
    LocalBlock<T> L = A.local(loc, true);
    T* a = L.ptr;
    const int64_t lda = L.ld, mloc = L.m, nloc = L.n;
    const bool pivot = (mode != PanelMode::NoPiv);
    const bool tnt = (mode == PanelMode::Tournament);

    Sched S(target);
    const int R = int(std::max<int64_t>(2, la + 2));
    std::vector<Work<T>> W(R), WU(R);
    std::vector<Work<int64_t>> PV(R);      // [ipiv(kb) | dst(2kb) | src(2kb) | count]
    for (int r = 0; r < R; ++r) {
        W[r].resize(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
        WU[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
        PV[r].resize(target, size_t(5 * nb + 8));
    }
    Work<int64_t> perm(target, size_t(std::max<int64_t>(m, 1)));
    Work<int> dinfo(target, 1);
    std::vector<int64_t> ipiv_all(std::min(m, n), 0);    // host copy (global rows)
    std::vector<Work<int64_t>> ipiv_dev(kt);              // device per-step pivots (p == 1)
    {
        lb::Ctx c0 = S.ctx(1);
        if (c0.dev()) device::memset_async(dinfo.data(), 0, sizeof(int), c0.stream);
        else dinfo.data()[0] = 0;
    }
    int host_info = 0;
    std::vector<RowPairs> host_pairs(kt);

    for (int64_t k = 0; k < kt; ++k) {
        const int64_t kb = A.tileNb(k);
        const int64_t kk = grow_of(A, k);
        const int64_t M = m - kk;                         // panel rows (global)
        const int64_t kd = std::min(kb, M);                // pivots this step
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const bool in_col = (mycol == qk);
        const int64_t lr_k = lrow_of(A, k), lr_k1 = lrow_of(A, k + 1);
        const int64_t lc_k = in_col ? lcol_of(A, k) : 0;
        const int slot = int(k % R);
        int64_t* pv = PV[slot].data();
        int64_t* pv_ipiv = pv;
        int64_t* pv_dst = pv + nb;
        int64_t* pv_src = pv + 3 * nb;
        const int64_t tPanel = Sched::tok(6, slot), tBc = Sched::bcast(slot);

        // ------------------------------------------------------------ panel
        if (p == 1) {
            if (in_col) {
                S.task(1, {}, {Sched::col(k), tPanel}, [&, k, kb, kk, M, kd, lr_k, lc_k, pv_ipiv, pv_dst, pv_src](lb::Ctx const& c) {
                    trace::Block t2("getrf_panel");
                    T* ap = a + lr_k + lc_k * lda;
                    lb::getrf_panel(c, M, kb, ap, lda, pv_ipiv, perm.data(), dinfo.data(), kk, pivot, tnt);
                    if (c.dev()) {
                        slate_amd::dev::perm_pairs(kd, perm.data(), pv_ipiv, pv_dst, pv_src, c.stream);
                    } else {
                        // host: pairs from sequential pivots
                        std::vector<int64_t> ip(pv_ipiv, pv_ipiv + kd);
                        for (auto& x : ip) x += kk;
                        RowPairs P = pairs_from_ipiv(kk, ip);
                        int64_t cnt = int64_t(P.size());
                        for (int64_t t = 0; t < 2 * kd; ++t) {
                            pv_dst[t] = t < cnt ? P.dst[t] - kk : 0;
                            pv_src[t] = t < cnt ? P.src[t] - kk : 0;
                        }
                        pv[5 * nb] = cnt;
                    }
                });
            }
        } else {
            // p > 1: gather the panel to the diagonal process row, factor, scatter back
            if (in_col) {
                S.task(device::kCommQueue, {}, {Sched::col(k), tPanel}, [&, k, kb, kk, M, kd, lr_k, lc_k, pv_ipiv, pk](lb::Ctx const& c) {
                    trace::Block t2("getrf_panel_gather");
                    // local rows >= kk of the panel
                    int64_t mr = mloc - lr_k;
                    T* ap = a + lr_k + lc_k * lda;
                    auto& st = *A.storage();
                    // which global tile rows belong to which process row
                    std::vector<std::vector<int64_t>> rows_of(p);   // global row starts of tiles
                    std::vector<int64_t> cnt(p, 0);
                    for (int64_t i = k; i < mt; ++i) {
                        int r = A.srow_owner(i);
                        rows_of[r].push_back(i);
                        cnt[r] += A.tileMb(i);
                    }
                    Work<T> full(target, size_t(std::max<int64_t>(M, 1)) * kb);
                    Work<T> mine(target, size_t(std::max<int64_t>(mr, 1)) * kb);
                    pack(c, mr, kb, ap, lda, mine.data());
                    // gather to pk
                    std::vector<Comm::P2P> ops;
                    std::vector<Work<T>> rbufs(p);
                    if (myrow == pk) {
                        for (int r = 0; r < p; ++r) {
                            if (r == pk || cnt[r] == 0) continue;
                            rbufs[r].resize(target, size_t(cnt[r]) * kb);
                            ops.push_back({rbufs[r].data(), size_t(cnt[r] * kb), r, false});
                        }
                    } else if (mr > 0) {
                        ops.push_back({mine.data(), size_t(mr * kb), pk, true});
                    }
                    g.col().exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                    if (myrow == pk) {
                        // assemble in global order
                        std::vector<int64_t> off(p, 0);
                        for (int64_t i = k; i < mt; ++i) {
                            int r = A.srow_owner(i);
                            int64_t ib = A.tileMb(i);
                            T const* src = (r == pk) ? mine.data() + off[r] : rbufs[r].data() + off[r];
                            int64_t lds = (r == pk) ? std::max<int64_t>(mr, 1) : cnt[r];
                            lb::copy2d(c, ib, kb, src, lds, full.data() + (grow_of(A, i) - kk), std::max<int64_t>(M, 1));
                            off[r] += ib;
                        }
                        lb::getrf_panel(c, M, kb, full.data(), std::max<int64_t>(M, 1), pv_ipiv, nullptr,
                                        dinfo.data(), kk, pivot, tnt);
                        // scatter back (same layout)
                        std::fill(off.begin(), off.end(), 0);
                        for (int64_t i = k; i < mt; ++i) {
                            int r = A.srow_owner(i);
                            int64_t ib = A.tileMb(i);
                            T* dst = (r == pk) ? mine.data() + off[r] : rbufs[r].data() + off[r];
                            int64_t ldd = (r == pk) ? std::max<int64_t>(mr, 1) : cnt[r];
                            lb::copy2d(c, ib, kb, full.data() + (grow_of(A, i) - kk), std::max<int64_t>(M, 1), dst, ldd);
                            off[r] += ib;
                        }
                    }
                    ops.clear();
                    if (myrow == pk) {
                        for (int r = 0; r < p; ++r)
                            if (r != pk && cnt[r] > 0) ops.push_back({rbufs[r].data(), size_t(cnt[r] * kb), r, true});
                    } else if (mr > 0) {
                        ops.push_back({mine.data(), size_t(mr * kb), pk, false});
                    }
                    g.col().exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                    lb::copy2d(c, mr, kb, mine.data(), std::max<int64_t>(mr, 1), ap, lda);
                    // pivots to every process of the column
                    g.col().bcast(pv_ipiv, size_t(kd), scalar_type<int64_t>(), pk, c.loc(), c.stream);
                    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
                    (void)st;
                });
            }
        }

        // ------------------------------------------- pivots to every process
        // p == 1: (ipiv, pairs) along the process row, stays on the device.
        // p > 1: ipiv to every rank (world bcast from the diagonal owner), pairs
        //        computed on the host (the row exchange needs host counts).
        S.task(device::kCommQueue, {tPanel}, {tBc}, [&, k, kd, kk, qk, pk, pv_ipiv, slot](lb::Ctx const& c) {
            trace::Block t2("getrf_bcast_piv");
            if (p == 1) {
                bcast(g.row(), PV[slot].data(), size_t(5 * nb + 8), qk, c);
            } else {
                int root = g.rank_of(pk, qk);
                g.world().bcast(pv_ipiv, size_t(kd), scalar_type<int64_t>(), root, c.loc(), c.stream);
                std::vector<int64_t> ip(kd);
                if (c.dev()) {
                    device::memcpy_async(ip.data(), pv_ipiv, kd * sizeof(int64_t), c.stream);
                    slate_hip_call(hipStreamSynchronize(c.stream));
                } else std::copy(pv_ipiv, pv_ipiv + kd, ip.begin());
                for (auto& x : ip) x += kk;
                host_pairs[k] = pairs_from_ipiv(kk, ip);
            }
        });

        // ----------------------------------------- L panel along process rows
        T* Wk = W[slot].data();
        const int64_t mrows_k = mloc - lr_k;     // my rows >= kk
        S.task(device::kCommQueue, {Sched::col(k), tBc}, {Sched::tok(7, slot)}, [&, lr_k, lc_k, kb, qk, Wk, mrows_k](lb::Ctx const& c) {
            trace::Block t2("getrf_bcast_L");
            if (mycol == qk) pack(c, mrows_k, kb, a + lr_k + lc_k * lda, lda, Wk);
            if (q > 1) bcast(g.row(), Wk, size_t(mrows_k * kb), qk, c);
        });
        const int64_t tL = Sched::tok(7, slot);

        // -------------------------------------- column ranges: permute, U, update
        // apply the step's row permutation to local columns [c0, c1)
        auto permute = [&, k, kk, kd, slot](lb::Ctx const& c, int64_t c0, int64_t c1) {
            if (c1 <= c0 || !pivot) return;
            if (p == 1) {
                // rows: local == global; pairs relative to kk
                int64_t* pvv = PV[slot].data();
                if (c.dev()) {
                    slate_amd::dev::permute_rows(c1 - c0, slate_amd::dev::dptr(a + kk + c0 * lda), lda,
                                                 pvv + nb, pvv + 3 * nb, nullptr, int(2 * kd), c.stream);
                } else {
                    int64_t cnt = pvv[5 * nb];
                    std::vector<T> tmp(cnt);
                    for (int64_t j = c0; j < c1; ++j) {
                        T* col = a + kk + j * lda;
                        for (int64_t t = 0; t < cnt; ++t) tmp[t] = col[pvv[3 * nb + t]];
                        for (int64_t t = 0; t < cnt; ++t) col[pvv[nb + t]] = tmp[t];
                    }
                }
            } else {
                permute_rows_dist(A, host_pairs[k], c0, c1, c);
            }
        };
        // columns of tiles [j0, j1) local to me
        auto lcols = [&](int64_t j0, int64_t j1) { return std::make_pair(lcol_of(A, j0), lcol_of(A, j1)); };
        T* WUk = WU[slot].data();
        // U row height is kd = tileMb(k) (< kb only for the last block row of a
        // wide matrix; rows beyond it are not part of the matrix)
        auto urow = [&, k, kd, lr_k, pk, Wk, WUk](lb::Ctx const& c, int64_t j0, int64_t j1) {
            auto [c0, c1] = lcols(j0, j1);
            if (c1 <= c0) return;
            if (myrow == pk) {
                // U(k, j0:j1) = L(k,k)^{-1} A(k, j0:j1); L(k,k) = top kd rows of W_k
                lb::trsm(c, Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, kd, c1 - c0, T(1),
                         Wk, std::max<int64_t>(mrows_k, 1), a + lr_k + c0 * lda, lda);
            }
        };
        auto ubcast = [&, k, kb, kd, lr_k, pk, WUk](lb::Ctx const& c, int64_t j0, int64_t j1) {
            auto [c0, c1] = lcols(j0, j1);
            int64_t nc = c1 - c0;
            if (nc <= 0) return;
            T* dst = WUk + c0 * kb;
            if (myrow == pk) lb::copy2d(c, kd, nc, a + lr_k + c0 * lda, lda, dst, kb);
            if (p > 1) bcast(g.col(), dst, size_t(kb * nc), pk, c);
        };
        auto update = [&, k, kb, lr_k1, lr_k, Wk, WUk](lb::Ctx const& c, int64_t j0, int64_t j1) {
            auto [c0, c1] = lcols(j0, j1);
            int64_t nc = c1 - c0, nr = mloc - lr_k1;
            if (nc <= 0 || nr <= 0) return;
            trace::Block t2("getrf_update");
            lb::gemm(c, Op::NoTrans, Op::NoTrans, nr, nc, kb, T(-1), Wk + (lr_k1 - lr_k), std::max<int64_t>(mrows_k, 1),
                     WUk + c0 * kb, kb, T(1), a + lr_k1 + c0 * lda, lda);
        };

        auto range_tasks = [&](int queue, int64_t j0, int64_t j1) {
            std::vector<int64_t> cols;
            for (int64_t j = j0; j < j1; ++j) cols.push_back(Sched::col(j));
            std::vector<int64_t> in = {tBc, tL};
            int pq = (p == 1) ? queue : device::kCommQueue;
            S.task(pq, in, cols, [&, j0, j1](lb::Ctx const& c) {
                auto [c0, c1] = lcols(j0, j1);
                permute(c, c0, c1);
            });
            S.task(queue, in, cols, [&, urow, j0, j1](lb::Ctx const& c) { urow(c, j0, j1); });
            const int64_t tU = Sched::tok(10 + queue, slot);
            S.task(device::kCommQueue, cols, {tU}, [&, ubcast, j0, j1](lb::Ctx const& c) { ubcast(c, j0, j1); });
            std::vector<int64_t> in2 = {tU, tL};
            S.task(queue, in2, cols, [&, update, j0, j1](lb::Ctx const& c) { update(c, j0, j1); });
        };
        int64_t jla_end = std::min(nt, k + 1 + la);
        for (int64_t j = k + 1; j < jla_end; ++j)
            range_tasks(device::kLookaheadQueue, j, j + 1);
        if (jla_end < nt) range_tasks(device::kTrailQueue, jla_end, nt);

        // left columns [0, k): apply the step's interchanges (deferred queue)
        if (k > 0 && pivot) {
            int lq = (p == 1) ? device::kTrailQueue : device::kCommQueue;
            S.task(lq, {tBc}, {Sched::tok(11, 0), Sched::col(k - 1)}, [&, k](lb::Ctx const& c) {
                auto [c0, c1] = lcols(0, k);
                permute(c, c0, c1);
            });
        }
        // host copy of this step's pivots (global rows)
        S.task(device::kCommQueue, {tBc}, {}, [&, k, kk, kd, pv_ipiv](lb::Ctx const& c) {
            std::vector<int64_t> ip(kd);
            if (c.dev()) {
                device::memcpy_async(ip.data(), pv_ipiv, kd * sizeof(int64_t), c.stream);
                slate_hip_call(hipStreamSynchronize(c.stream));
            } else std::copy(pv_ipiv, pv_ipiv + kd, ip.begin());
            for (int64_t t = 0; t < kd; ++t) ipiv_all[kk + t] = ip[t] + (p == 1 ? kk : kk);
        });
    }
    S.wait_all();
    (void)host_info;
    // pivots -> reference Pivots structure: (tile index relative to k, offset)
    pivots.assign(kt, {});
    for (int64_t k = 0; k < kt; ++k) {
        int64_t kk = grow_of(A, k), kd = std::min(A.tileNb(k), m - kk);
        pivots[k].resize(kd);
        for (int64_t t = 0; t < kd; ++t) {
            int64_t r = ipiv_all[kk + t];
            // tile index relative to k and offset within the tile
            int64_t ti = 0;
            while (ti + k + 1 < mt && grow_of(A, k + ti + 1) <= r) ++ti;
            pivots[k][t] = Pivot(ti, r - grow_of(A, k + ti));
        }
    }
    int64_t info = fetch_info(target, dinfo.data());
    info = reduce_info(info, g.world());
    A.storage()->update_origin();
    return info;
}

}  // namespace

template <typename T>
int64_t getrf(Matrix<T>& A, Pivots& pivots, Options const& opts) {
    Method m = get_option<int64_t>(opts, Option::MethodLU, MethodLU::PartialPiv);
    return getrf_impl(A, pivots, opts, m == MethodLU::NoPiv ? PanelMode::NoPiv :
                      (m == MethodLU::CALU ? PanelMode::Tournament : PanelMode::Partial));
}

template <typename T>
int64_t getrf_tntpiv(Matrix<T>& A, Pivots& pivots, Options const& opts) {
    return getrf_impl(A, pivots, opts, PanelMode::Tournament);
}

template <typename T>
int64_t getrf_nopiv(Matrix<T>& A, Options const& opts) {
    Pivots piv;
    return getrf_impl(A, piv, opts, PanelMode::NoPiv);
}

//------------------------------------------------------------------------------
namespace internal {

/// Apply pivots (forward or backward) to the rows of B.
template <typename T>
void apply_pivots(Pivots const& pivots, BaseMatrix<T> const& A, Matrix<T>& B, Target target, bool forward) {
    std::vector<int64_t> ip;
    for (size_t k = 0; k < pivots.size(); ++k) {
        int64_t kk = grow_of(A, int64_t(k));
        for (auto const& pv : pivots[k])
            ip.push_back(grow_of(A, int64_t(k) + pv.tileIndex()) + pv.elementOffset());
        (void)kk;
    }
    if (!forward) {
        // inverse permutation: apply interchanges in reverse order
        std::unordered_map<int64_t, int64_t> pos;
        auto get = [&](int64_t r) { auto it = pos.find(r); return it == pos.end() ? r : it->second; };
        for (int64_t t = int64_t(ip.size()) - 1; t >= 0; --t) {
            int64_t a = t, b = ip[t];
            if (a == b) continue;
            int64_t va = get(a), vb = get(b);
            pos[a] = vb; pos[b] = va;
        }
        RowPairs P;
        for (auto& kv : pos) if (kv.first != kv.second) { P.dst.push_back(kv.first); P.src.push_back(kv.second); }
        lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
        B.storage()->get(loc_of(target), true);
        permute_rows_dist(B, P, 0, B.lcol_end() - B.lcol_begin(), c);
        return;
    }
    RowPairs P = pairs_from_ipiv(0, ip);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    B.storage()->get(loc_of(target), true);
    permute_rows_dist(B, P, 0, B.lcol_end() - B.lcol_begin(), c);
}

template void apply_pivots<float>(Pivots const&, BaseMatrix<float> const&, Matrix<float>&, Target, bool);
template void apply_pivots<double>(Pivots const&, BaseMatrix<double> const&, Matrix<double>&, Target, bool);
template void apply_pivots<std::complex<float>>(Pivots const&, BaseMatrix<std::complex<float>> const&, Matrix<std::complex<float>>&, Target, bool);
template void apply_pivots<std::complex<double>>(Pivots const&, BaseMatrix<std::complex<double>> const&, Matrix<std::complex<double>>&, Target, bool);

}  // namespace internal

#define SLATE_GETRF_INST(T)                                                                  \
    template int64_t getrf<T>(Matrix<T>&, Pivots&, Options const&);                         \
    template int64_t getrf_tntpiv<T>(Matrix<T>&, Pivots&, Options const&);                  \
    template int64_t getrf_nopiv<T>(Matrix<T>&, Options const&);

SLATE_GETRF_INST(float)
SLATE_GETRF_INST(double)
SLATE_GETRF_INST(std::complex<float>)
SLATE_GETRF_INST(std::complex<double>)

}  // namespace slate
