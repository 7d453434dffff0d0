// Distributed LU factorization with partial pivoting (reference src/getrf.cc,
// src/getrf_tntpiv.cc, src/getrf_nopiv.cc, src/internal/internal_swap.cc).
//
// Per block column k:
//   panel (queue 1): the whole m x nb panel is factored ON THE DEVICE by the
//     recursive LU kernel (device pivot search, in-kernel row swaps across the
//     panel, trsm/gemm recursion) -- no host round trip per column.  With
//     p = 1 the panel is local to its process column.  With p > 1 (see
//     getrf_dist) partial pivoting all-gathers the panel rows over the column
//     (ONE collective per panel) and factors the assembled panel redundantly on
//     every process of the column; tournament pivoting (CALU) runs a
//     cross-process tree.
//   The panel's row permutation is turned into (dst, src) row pairs on the
//   device; they travel with the pivots in one broadcast, and every process
//   permutes its local columns with ONE gather/scatter kernel per column
//   range (column-major rows are moved whole), instead of the reference's one
//   blas::swap per pivot (internal_swap.cc:674).
//   U row: trsm on process row pk, broadcast down columns; trailing update
//   A22 -= L21 U12 as one MFMA GEMM per process; lookahead columns on their
//   own queues.
// getrf_tntpiv (CALU) shares this driver: its panel selects the pivots of
// every 32-column narrow block by a tournament over 256-row leaves on the
// device (kernels/tslu.hip), then factors that block without further pivoting.
#include "internal.hh"
#include "spread.hh"
#include "lu_dist.hh"
#include "../kernels/kernels.hh"

#include <atomic>
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

/// Per-process counters of the exact row exchange (tests / diagnostics):
/// elements this process sent, and the rows behind them (summed over ranges).
// updated by every rank thread of an in-process grid: atomics (TSan, make tsan)
struct RowXStats { std::atomic<int64_t> elems{0}, rows{0}; };
RowXStats& rowx_stats() { static RowXStats s; return s; }

/// Exact row exchange of one LU step on a p > 1 grid.  The slot lists of the
/// step (slot s < kd: U row s <- winner ssrc[s]; s >= kd: displaced row
/// ssrc[s] -> sdst[s]) are on the host, so every message carries exactly the
/// rows that change process: the winner rows I own go to every other process
/// of the column (each needs the whole U block row for its U12 and GEMM), the
/// displaced rows only to the owner of their destination.  The reference
/// moves the remote pivot rows the same way (internal_swap.cc:511-805).
/// with_u = false (the left columns): every slot is a plain row move.
struct RowXPlan {
    int p = 1;
    std::vector<std::vector<int64_t>> sU, sD, rU, rD;   // per peer
    std::vector<int64_t> lUsrc, lUslot, lDsrc, lDdst;   // my own rows
    std::vector<int64_t> flat;                          // all lists, host
    std::vector<size_t> o_sU, o_sD, o_rU, o_rD;
    size_t o_lUsrc = 0, o_lUslot = 0, o_lDsrc = 0, o_lDdst = 0;
    int64_t sends = 0, recvs = 0;                       // rows per column
    size_t slab(int r) const { return sU[r].size() + sD[r].size(); }
    size_t rslab(int r) const { return rU[r].size() + rD[r].size(); }
};

RowXPlan rowx_plan(slate_amd::dev::RowDist const& rd, int64_t kd, int64_t const* ssrc, int64_t const* sdst,
                   bool with_u) {
    namespace kdv = slate_amd::dev;
    RowXPlan P;
    const int p = rd.p, me = rd.myrow;
    P.p = p;
    P.sU.assign(p, {}); P.sD.assign(p, {}); P.rU.assign(p, {}); P.rD.assign(p, {});
    for (int64_t s = 0; s < 2 * kd; ++s) {
        const int64_t src = ssrc[s], dst = sdst[s];
        if (src < 0 || dst < 0) continue;
        const int os = kdv::rd_owner(rd, src), od = kdv::rd_owner(rd, dst);
        if (with_u && s < kd) {
            if (os == me) {
                P.lUsrc.push_back(kdv::rd_lrow(rd, src));
                P.lUslot.push_back(s);
                for (int r = 0; r < p; ++r) if (r != me) P.sU[r].push_back(kdv::rd_lrow(rd, src));
            } else {
                P.rU[os].push_back(s);
            }
            continue;
        }
        if (src == dst) continue;
        if (os == me && od == me) { P.lDsrc.push_back(kdv::rd_lrow(rd, src)); P.lDdst.push_back(kdv::rd_lrow(rd, dst)); }
        else if (os == me) P.sD[od].push_back(kdv::rd_lrow(rd, src));
        else if (od == me) P.rD[os].push_back(kdv::rd_lrow(rd, dst));
    }
    auto put = [&](std::vector<int64_t> const& v) { size_t o = P.flat.size(); P.flat.insert(P.flat.end(), v.begin(), v.end()); return o; };
    for (int r = 0; r < p; ++r) {
        P.o_sU.push_back(put(P.sU[r])); P.o_sD.push_back(put(P.sD[r]));
        P.o_rU.push_back(put(P.rU[r])); P.o_rD.push_back(put(P.rD[r]));
        P.sends += int64_t(P.slab(r));
        P.recvs += int64_t(P.rslab(r));
    }
    P.o_lUsrc = put(P.lUsrc); P.o_lUslot = put(P.lUslot); P.o_lDsrc = put(P.lDsrc); P.o_lDdst = put(P.lDdst);
    if (P.flat.empty()) P.flat.push_back(0);
    return P;
}

/// Execute a plan on local columns [0, nc) of A (ld lda): pack, exchange over
/// `cm`, unpack.  U rows land in buf (ld ldu, slot s at row s); idx: the
/// plan's flat lists where the context can read them (device copy on the
/// device); SB (>= sends x nc), RB (>= recvs x nc), TB (>= 2 kd x nc) scratch.
template <typename T>
void rowx_run(lb::Ctx const& c, RowXPlan const& P, int64_t const* idx, int64_t nc, T* A, int64_t lda, T* buf,
              int64_t ldu, T* SB, T* RB, T* TB, Comm& cm, int phase) {
    if (nc <= 0) return;
    auto mv = [&](int64_t const* ix, size_t cnt, T* M, int64_t ldm, T* slab, bool scatter) {
        if (cnt == 0) return;
        if (c.dev()) {
            using DT = slate_amd::dev::dev_t<T>;
            slate_amd::dev::rows_pack<DT>(nc, slate_amd::dev::dptr(M), ldm, ix, int(cnt), slate_amd::dev::dptr(slab),
                                          scatter, c.stream);
            return;
        }
        for (int64_t j = 0; j < nc; ++j)
            for (size_t t = 0; t < cnt; ++t) {
                T& a = M[ix[t] + j * ldm];
                T& b = slab[t + j * cnt];
                if (scatter) a = b; else b = a;
            }
    };
    const int p = P.p;
    // phase 1: reads (every source row before any destination is written)
    if (phase & 1) {
        size_t off = 0;
        for (int r = 0; r < p; ++r) {
            mv(idx + P.o_sU[r], P.sU[r].size(), A, lda, SB + off * nc, false);
            mv(idx + P.o_sD[r], P.sD[r].size(), A, lda, SB + (off + P.sU[r].size()) * nc, false);
            off += P.slab(r);
        }
        mv(idx + P.o_lUsrc, P.lUsrc.size(), A, lda, TB, false);
        mv(idx + P.o_lDsrc, P.lDsrc.size(), A, lda, TB + P.lUsrc.size() * nc, false);
    }
    // phase 2: the messages (one send / one receive per peer that has rows)
    if (phase & 2) {
        std::vector<Comm::P2P> ops;
        size_t so = 0, ro = 0;
        for (int r = 0; r < p; ++r) {
            if (P.slab(r)) ops.push_back({SB + so * nc, P.slab(r) * nc, r, true});
            if (P.rslab(r)) ops.push_back({RB + ro * nc, P.rslab(r) * nc, r, false});
            so += P.slab(r);
            ro += P.rslab(r);
        }
        if (!ops.empty()) cm.exchange(ops, scalar_type<T>(), c.loc(), c.stream);
        rowx_stats().elems += int64_t(so) * nc;
        rowx_stats().rows += int64_t(so);
    }
    // phase 4: writes
    if (phase & 4) {
        size_t ro = 0;
        for (int r = 0; r < p; ++r) {
            mv(idx + P.o_rU[r], P.rU[r].size(), buf, ldu, RB + ro * nc, true);
            mv(idx + P.o_rD[r], P.rD[r].size(), A, lda, RB + (ro + P.rU[r].size()) * nc, true);
            ro += P.rslab(r);
        }
        mv(idx + P.o_lUslot, P.lUslot.size(), buf, ldu, TB, true);
        mv(idx + P.o_lDdst, P.lDdst.size(), A, lda, TB + P.lUsrc.size() * nc, true);
    }
}

enum class PanelMode { Partial, Tournament, NoPiv };

//------------------------------------------------------------------------------
/// LU on a p x q grid with p > 1.  No host synchronization inside the k-loop:
/// every pivot-dependent quantity stays on the device and every message size
/// is known on the host from the distribution alone.
///
/// Panel (process column qk, rows spread over the p process rows):
///   Tournament (CALU, reference internal_getrf_tntpiv.cc:479-633): every
///     process selects kd candidate rows from its local panel rows with the
///     device tournament panel (a local LU on a copy); the candidates of
///     process rows meet in a binary tree rooted at the diagonal process pk
///     (ncclSend/Recv of kd x kb ORIGINAL rows + their global indices over the
///     column communicator, partial-pivoting LU of the stacked 2kd x kb block);
///     the root's final LU gives the winners and [L11\U11].  Winners and LU11
///     go down the column; the panel rows are permuted (slot all-reduce) and
///     L21 = A21 U11^{-1} is a local trsm on every process.
///   Partial (PPLU, reference Tile_getrf.hh:162-450 does one MPI_Allreduce
///     MAXLOC per column): ONE all-gather of the panel rows over the column
///     communicator; every process of the column assembles the M x kb panel in
///     global row order, factors it with the device partial-pivoting panel
///     (identical, deterministic result on every process: exact partial
///     pivoting, the same pivots as on one GPU) and keeps its own rows.
///     1 collective per panel instead of nb.
///   NoPiv: pk factors the diagonal block, the column solves L21 locally.
/// Row permutation of every other column range: an exact point-to-point
/// exchange (the default, SLATE_LU_EXACT_SWAP=1): only the rows that change
/// process move, each once, with grouped send / recv over the column
/// communicator; the pivot-row owners then broadcast the U block row to the
/// column, where U12 = L11^{-1} (...) is computed redundantly instead of
/// broadcast solved.  SLATE_LU_EXACT_SWAP=0 keeps the older slot scheme
/// (lu_dist.hip: pack -> all-reduce over the column communicator -> unpack,
/// which delivers the unsolved U block row to every process at once).
/// Two communication lanes (Grid::row_fast / col_fast): every message on the
/// critical path -- tournament / panel gather, LU11 + pivots + L panel
/// broadcasts, and the row exchange of the lookahead columns -- is issued on
/// the high-priority panel queue over duplicate communicators; the trailing
/// chunks' row exchanges and the left-column swaps stay on the comm queue
/// over the plain communicators.  So step k+1's panel never waits behind
/// step k's bulk traffic (reference priorities: src/getrf.cc:92,124,175-186).
/// Every communicator sees its operations in the same order on every rank
/// (one program order, and a task only waits on earlier tasks), so the lanes
/// cannot deadlock.  Trailing columns are processed in chunks so the
/// all-reduce of chunk c+1 overlaps the GEMM of chunk c.
/// Option::PivotThreshold in (0, 1] (reference src/getrf.cc:39): partial
/// pivoting keeps the diagonal while |a_jj| >= threshold * column max
inline double pivot_threshold(Options const& opts) {
    double t = get_option<double>(opts, Option::PivotThreshold, 1.0);
    slate_error_if_msg(!(t > 0.0 && t <= 1.0), "PivotThreshold must be in (0, 1]");
    return t;
}

template <typename T>
int64_t getrf_dist(BaseMatrix<T>& A, Pivots& pivots, Options const& opts, PanelMode mode, Target target) {
    using namespace internal::ludist;
    trace::Block tb("getrf_dist");
    internal::DriverScope ds_;
    const int64_t la = get_option<int64_t>(opts, Option::Lookahead, 1);
    const double thresh = pivot_threshold(opts);
    auto& g = *A.grid();
    const int p = g.p(), myrow = g.myrow(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t mt = A.mt(), nt = A.nt(), m = A.m(), n = A.n();
    const int64_t kt = std::min(mt, nt), nb = A.nb();
    slate_error_if_msg(nb > 1024, "getrf on a p > 1 grid: tile size above 1024");
    LocalBlock<T> L = A.local(loc, true);
    T* a = L.ptr;
    const int64_t lda = L.ld, mloc = L.m, nloc = L.n;
    const bool pivot = mode != PanelMode::NoPiv;
    const RowDist rd = row_dist(A);
    const int qC = device::kCommQueue, qP = 1;
    // critical-path lane (panel queue, duplicate comms) / bulk lane (comm queue)
    Comm& colF = g.col_fast();
    Comm& rowF = g.row_fast();
    auto& st = *A.storage();

    Sched S(target);
    const int R = int(std::max<int64_t>(3, la + 2));
    std::vector<Work<T>> W(R), LU(R);
    std::vector<Work<int64_t>> PV(R);        // [win nb | ipiv nb | slot_src 2nb | slot_dst 2nb]
    for (int r = 0; r < R; ++r) {
        W[r].resize(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
        LU[r].resize(target, size_t(nb) * nb);
        PV[r].resize(target, size_t(6 * nb));
    }
    const size_t ubn = size_t(2 * nb) * size_t(std::max<int64_t>(nloc, 1));
    Work<T> UB(target, ubn), LB(pivot ? target : Target::HostTask, pivot ? ubn : 1), PB(target, size_t(nb) * nb);
    // panel scratch
    Work<T> Wsel(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
    Work<T> Cb(target, size_t(nb) * nb), Cr(target, size_t(nb) * nb), Sb(target, size_t(2 * nb) * nb),
        Fb(target, size_t(2 * nb) * nb);
    Work<int64_t> ids(target, nb), idr(target, nb), idS(target, 2 * nb),
        perm(target, size_t(std::max<int64_t>(mode == PanelMode::Partial ? m : mloc, 2 * nb))), pip(target, nb);
    // partial pivoting: my packed panel rows / all-gathered rows / assembled panel
    Work<T> PS, PG, PP;
    const int64_t maxloc_rows = ceildiv(std::max<int64_t>(m, 1), st.mb * p) * st.mb;
    if (mode == PanelMode::Partial) {
        slate_error_if_msg(p > 16, "getrf partial pivoting: more than 16 process rows");
        PS.resize(target, size_t(maxloc_rows) * nb);
        PG.resize(target, size_t(p) * maxloc_rows * nb);
        PP.resize(target, size_t(std::max<int64_t>(m, 1)) * nb);
    }
    Work<int64_t> ipiv_all(target, size_t(std::max<int64_t>(kt, 1)) * nb);
    // exact row exchange (default; SLATE_LU_EXACT_SWAP=0: the slot all-reduce):
    // the step's pivot slots come to the host once per step (after the pivot
    // broadcast) and every trailing / left row move is a point-to-point
    // message of exactly the rows that change process (see RowXPlan)
    static const bool exact_env = [] {
        const char* e = std::getenv("SLATE_LU_EXACT_SWAP");
        return e ? std::atoi(e) != 0 : true;
    }();
    const bool exact = pivot && exact_env;
    std::vector<RowXPlan> RPl(R), LPl(R);
    std::vector<Work<int64_t>> PX(R), PXL(R);
    Work<T> XS, XR, XT, XLS, XLR, XLT;
    int64_t* hpv = nullptr;
    const size_t pxn = size_t(p + 4) * 2 * nb + 16;
    if (exact) {
        for (int r = 0; r < R; ++r) { PX[r].resize(target, pxn); PXL[r].resize(target, pxn); }
        const size_t nl = size_t(std::max<int64_t>(nloc, 1));
        XS.resize(target, size_t(p) * nb * nl); XR.resize(target, 2 * size_t(nb) * nl); XT.resize(target, 2 * size_t(nb) * nl);
        XLS.resize(target, size_t(p) * nb * nl); XLR.resize(target, 2 * size_t(nb) * nl); XLT.resize(target, 2 * size_t(nb) * nl);
        if (target == Target::Devices) hpv = static_cast<int64_t*>(device::malloc_host(6 * nb * sizeof(int64_t)));
    }
    struct HostFree { int64_t* p; ~HostFree() { if (p) device::free_host(p); } } hpv_free{hpv};
    Work<int> dinfo(target, 2);               // [info, dummy]
    {
        lb::Ctx c0 = S.ctx(qP);
        if (c0.dev()) device::memset_async(dinfo.data(), 0, 2 * sizeof(int), c0.stream);
        else dinfo.data()[0] = dinfo.data()[1] = 0;
    }
    int* info_real = dinfo.data();
    int* info_dummy = dinfo.data() + 1;
    auto lcols = [&](int64_t j0, int64_t j1) { return std::make_pair(lcol_of(A, j0), lcol_of(A, j1)); };
    const int64_t tSel = Sched::tok(30, 0), tPB = Sched::tok(33, 0), tLeft = Sched::tok(34, 0);

    // left-column interchanges of step k2 on tile columns [0, k2)
    auto left = [&](int64_t k2) {
        if (!pivot || k2 <= 0) return;
        int64_t nc = lcol_of(A, k2);
        if (nc <= 0) return;
        const int s2 = int(k2 % R);
        if (exact) {
            const int qL = device::kTrailQueue;
            RowXPlan const* P = &LPl[s2];
            int64_t const* ix = target == Target::Devices ? PXL[s2].data() : LPl[s2].flat.data();
            S.task(qL, {Sched::tok(31, s2), Sched::col(k2 - 1)}, {tLeft}, [&, nc, P, ix](lb::Ctx const& c) {
                trace::Block t2("getrf_left_pack");
                rowx_run<T>(c, *P, ix, nc, a, lda, (T*)nullptr, 0, XLS.data(), XLR.data(), XLT.data(), g.col(), 1);
            });
            S.task(qC, {}, {tLeft}, [&, nc, P, ix](lb::Ctx const& c) {
                trace::Block t2("getrf_left_swap");
                rowx_run<T>(c, *P, ix, nc, a, lda, (T*)nullptr, 0, XLS.data(), XLR.data(), XLT.data(), g.col(), 2);
            });
            S.task(qL, {Sched::tok(31, s2)}, {tLeft, Sched::col(k2 - 1)}, [&, nc, P, ix](lb::Ctx const& c) {
                trace::Block t2("getrf_left_unpack");
                rowx_run<T>(c, *P, ix, nc, a, lda, (T*)nullptr, 0, XLS.data(), XLR.data(), XLT.data(), g.col(), 4);
            });
            return;
        }
        const int64_t kd2 = std::min(A.tileNb(k2), m - grow_of(A, k2));
        int64_t* pv2 = PV[s2].data();
        // pack / unpack on a compute queue, only the all-reduce on the comm
        // queue (tLeft chains the three and the next step's use of LB)
        const int ns = int(2 * kd2);
        const int qL = device::kTrailQueue;
        S.task(qL, {Sched::tok(31, s2), Sched::col(k2 - 1)}, {tLeft}, [&, nc, ns, pv2](lb::Ctx const& c) {
            trace::Block t2("getrf_left_pack");
            slots_pack(c, 0, ns, nc, pv2 + 2 * nb, a, lda, rd, LB.data(), ns);
        });
        S.task(qC, {}, {tLeft}, [&, nc, ns](lb::Ctx const& c) {
            trace::Block t2("getrf_left_swap");
            g.col().allreduce(LB.data(), size_t(ns) * nc, ReduceOp::Sum, c.loc(), c.stream);
        });
        // (reads PV[s2] too: the token makes its next writer wait for it)
        S.task(qL, {Sched::tok(31, s2)}, {tLeft, Sched::col(k2 - 1)}, [&, nc, ns, pv2](lb::Ctx const& c) {
            trace::Block t2("getrf_left_unpack");
            slots_unpack(c, 0, ns, nc, pv2 + 4 * nb, LB.data(), ns, a, lda, rd);
        });
    };

    for (int64_t k = 0; k < kt; ++k) {
        const int64_t kb = A.tileNb(k), kk = grow_of(A, k), M = m - kk, kd = std::min(kb, M);
        const int pk = A.srow_owner(k), qk = A.scol_owner(k);
        const bool in_col = (mycol == qk), diag = (myrow == pk);
        const int64_t lr_k = lrow_of(A, k);
        // first local row below the diagonal block T = rows [kk, kk + kd) (on pk
        // T starts tile k; kd < tileMb(k) in the last block column)
        const int64_t lr_k1 = diag ? lr_k + kd : lr_k;
        const int64_t lc_k = in_col ? lcol_of(A, k) : 0;
        const int64_t mr = mloc - lr_k, ldw = std::max<int64_t>(mr, 1);
        const int slot = int(k % R);
        int64_t* pv = PV[slot].data();
        int64_t* win = pv;
        int64_t* ipv = pv + nb;
        int64_t* ssrc = pv + 2 * nb;
        int64_t* sdst = pv + 4 * nb;
        T* LUk = LU[slot].data();
        T* Wk = W[slot].data();
        T* ap = a + lr_k + lc_k * lda;        // my panel rows (>= kk)
        T* apc = a + lc_k * lda;               // panel column, local row 0
        const int64_t tPV = Sched::tok(31, slot), tW = Sched::tok(32, slot);
        // rows of the panel (global rows >= kk) per process row: host-known
        std::vector<int64_t> rows_r(p, 0);
        for (int64_t i = k; i < mt; ++i) rows_r[A.srow_owner(i)] += A.tileMb(i);

        // ================================================================ panel
        if (in_col && mode == PanelMode::Tournament) {
            // tree over the process rows holding panel rows, rooted at pk
            std::vector<int> part;
            for (int d = 0; d < p; ++d) { int r = (pk + d) % p; if (rows_r[r] > 0) part.push_back(r); }
            const int np = int(part.size());
            std::vector<int64_t> cnt(np);
            for (int i = 0; i < np; ++i) cnt[i] = std::min(rows_r[part[i]], kd);
            int ix = -1;
            for (int i = 0; i < np; ++i) if (part[i] == myrow) ix = i;
            struct Round { bool recv; int peer; int64_t mine, theirs; bool final; };
            std::vector<Round> rounds;
            for (int l = 1; l < np; l *= 2) {
                for (int i = 0; i + l < np; i += 2 * l) {
                    if (i == ix) rounds.push_back({true, part[i + l], cnt[i], cnt[i + l], false});
                    if (i + l == ix) rounds.push_back({false, part[i], cnt[i + l], 0, false});
                    cnt[i] = std::min(cnt[i] + cnt[i + l], kd);
                }
            }
            if (diag && !rounds.empty()) rounds.back().final = true;
            const bool sel_final = diag && rounds.empty();
            if (ix >= 0) {
                const int64_t cme = std::min(mr, kd);
                S.task(qP, {Sched::col(k)}, {tSel}, [&, ap, mr, kb, kk, cme, sel_final, lr_k](lb::Ctx const& c) {
                    trace::Block t2("getrf_tnt_local");
                    lb::copy2d(c, mr, kb, ap, lda, Wsel.data(), mr);
                    lb::getrf_panel(c, mr, kb, Wsel.data(), mr, pip.data(), perm.data(),
                                    sel_final ? info_real : info_dummy, kk, true, true);
                    gather_rows_ids(c, cme, kb, perm.data(), ap, lda, Cb.data(), cme, (int64_t const*)nullptr,
                                    ids.data(), rd, lr_k);
                });
                int64_t cur = cme;
                T const* lastF = Wsel.data();
                int64_t ldF = mr;
                for (auto const& rd_ : rounds) {
                    if (!rd_.recv) {
                        S.task(qP, {tSel}, {tSel}, [&, rd_, kb](lb::Ctx const& c) {
                            trace::Block t2("getrf_tnt_send");
                            std::vector<Comm::P2P> ops{{Cb.data(), size_t(rd_.mine * kb), rd_.peer, true}};
                            colF.exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                            std::vector<Comm::P2P> ops2{{ids.data(), size_t(rd_.mine), rd_.peer, true}};
                            colF.exchange(ops2, scalar_type<int64_t>(), c.loc(), c.stream);
                        });
                        break;
                    }
                    S.task(qP, {}, {tSel}, [&, rd_, kb](lb::Ctx const& c) {
                        trace::Block t2("getrf_tnt_recv");
                        std::vector<Comm::P2P> ops{{Cr.data(), size_t(rd_.theirs * kb), rd_.peer, false}};
                        colF.exchange(ops, scalar_type<T>(), c.loc(), c.stream);
                        std::vector<Comm::P2P> ops2{{idr.data(), size_t(rd_.theirs), rd_.peer, false}};
                        colF.exchange(ops2, scalar_type<int64_t>(), c.loc(), c.stream);
                    });
                    const int64_t ms = rd_.mine + rd_.theirs, c2 = std::min(ms, kd);
                    S.task(qP, {}, {tSel}, [&, rd_, kb, kk, ms, c2](lb::Ctx const& c) {
                        trace::Block t2("getrf_tnt_merge");
                        // stacked originals S = [mine; theirs], F = LU(S) with partial pivoting
                        lb::copy2d(c, rd_.mine, kb, Cb.data(), rd_.mine, Sb.data(), ms);
                        lb::copy2d(c, rd_.theirs, kb, Cr.data(), rd_.theirs, Sb.data() + rd_.mine, ms);
                        lb::copy2d(c, rd_.mine, int64_t(1), ids.data(), rd_.mine, idS.data(), ms);
                        lb::copy2d(c, rd_.theirs, int64_t(1), idr.data(), rd_.theirs, idS.data() + rd_.mine, ms);
                        lb::copy2d(c, ms, kb, Sb.data(), ms, Fb.data(), ms);
                        // tournament inside the merge too (tslu narrow blocks): a 2kd x kb
                        // partial-pivoting LU would cost two launches per column
                        lb::getrf_panel(c, ms, kb, Fb.data(), ms, pip.data(), perm.data(),
                                        rd_.final ? info_real : info_dummy, kk, true, true);
                        gather_rows_ids(c, c2, kb, perm.data(), Sb.data(), ms, Cb.data(), c2, idS.data(), ids.data(),
                                        rd, 0);
                    });
                    cur = c2;
                    lastF = Fb.data();
                    ldF = ms;
                }
                if (diag) {
                    S.task(qP, {tSel}, {tPV}, [&, lastF, ldF, kd, kb, LUk, win](lb::Ctx const& c) {
                        lb::copy2d(c, kd, kb, lastF, ldF, LUk, kd);
                        lb::copy2d(c, kd, int64_t(1), ids.data(), kd, win, kd);
                    });
                }
                (void)cur;
            }
            // winners and [L11\U11] down the panel column
            S.task(qP, {}, {tPV}, [&, kd, kb, pk, LUk, win](lb::Ctx const& c) {
                trace::Block t2("getrf_bcast_winners");
                bcast(colF, win, size_t(kd), pk, c);
                bcast(colF, LUk, size_t(kd * kb), pk, c);
            });
            S.task(qP, {}, {tPV}, [&, k, kk, kd, win, ipv, ssrc, sdst](lb::Ctx const& c) {
                perm_slots(c, 0, kk, int(kd), win, 0, ipv, ssrc, sdst);
            });
            // panel rows: displaced rows to the vacated winner positions
            S.task(qP, {tPV}, {Sched::col(k), tPB}, [&, kd, kb, apc, ssrc, sdst](lb::Ctx const& c) {
                trace::Block t2("getrf_panel_perm");
                slots_pack(c, int(kd), int(2 * kd), kb, ssrc, apc, lda, rd, PB.data(), kd);
                colF.allreduce(PB.data(), size_t(kd * kb), ReduceOp::Sum, c.loc(), c.stream);
                slots_unpack(c, int(kd), int(2 * kd), kb, sdst, PB.data(), kd, apc, lda, rd);
            });
        } else if (in_col && mode == PanelMode::Partial) {
            // exact partial pivoting with ONE all-gather per panel (see above):
            // pack my panel rows, all-gather over the column, assemble the
            // M x kb panel in global row order, factor it on the device (the
            // same deterministic result on every process of the column), keep
            // my rows, LU11 and the pivot slots
            const int64_t maxr = *std::max_element(rows_r.begin(), rows_r.end());
            PanelBases pb{};
            for (int r = 0; r < p; ++r) pb.base[r] = g2l_ceil(A.row0() + kk, st.mb, (r - st.rsrc + p) % p, p);
            S.task(qP, {Sched::col(k)}, {Sched::col(k), tPV}, [&, k, kk, kd, kb, M, mr, maxr, pb, diag, ap, LUk, ipv, ssrc, sdst](lb::Ctx const& c) {
                trace::Block t2("getrf_pp_panel");
                lb::copy2d(c, mr, kb, ap, lda, PS.data(), maxr);
                colF.allgather(PS.data(), PG.data(), size_t(maxr * kb), scalar_type<T>(), c.loc(), c.stream);
                panel_xfer<T>(c, M, kb, kk, rd, pb, maxr, PG.data(), PP.data(), M, nullptr, 1, 0);
                lb::getrf_panel(c, M, kb, PP.data(), M, pip.data(), perm.data(), diag ? info_real : info_dummy, kk,
                                true, false, thresh);
                panel_xfer<T>(c, M, kb, kk, rd, pb, maxr, nullptr, PP.data(), M, ap, lda, 1);
                lb::copy2d(c, kd, kb, PP.data(), M, LUk, kd);
                perm_slots(c, 1, kk, int(kd), pip.data(), kk, ipv, ssrc, sdst);
            });
        } else if (in_col) {
            // no pivoting: pk factors the diagonal block
            if (diag) {
                S.task(qP, {Sched::col(k)}, {Sched::col(k), tPV}, [&, kk, kd, kb, ap, LUk](lb::Ctx const& c) {
                    lb::getrf_panel(c, kd, kb, ap, lda, pip.data(), (int64_t*)nullptr, info_real, kk, false, false);
                    lb::copy2d(c, kd, kb, ap, lda, LUk, kd);
                });
            }
            S.task(qP, {}, {tPV}, [&, kd, kb, pk, LUk](lb::Ctx const& c) { bcast(colF, LUk, size_t(kd * kb), pk, c); });
        }
        // L21 = A21 U11^{-1} (tournament / no pivoting: the panel rows are still
        // original; partial: already factored by pk) and the L panel for the row
        if (in_col) {
            const bool solve = (mode != PanelMode::Partial);
            S.task(qP, {tPV, tPB}, {Sched::col(k), tW}, [&, solve, kd, kb, ap, mr, lr_k1, lc_k, LUk, Wk, diag](lb::Ctx const& c) {
                trace::Block t2("getrf_l21");
                if (solve) {
                    if (diag && mode != PanelMode::NoPiv) lb::copy2d(c, kd, kb, LUk, kd, ap, lda);
                    lb::trsm(c, Side::Right, Uplo::Upper, Op::NoTrans, Diag::NonUnit, mloc - lr_k1, kd, T(1), LUk, kd,
                             a + lr_k1 + lc_k * lda, lda);
                }
                if (mr > 0) pack(c, mr, kb, ap, lda, Wk);
            });
        }
        // pivots + LU11 and the L panel along the process rows
        S.task(qP, {}, {tPV}, [&, k, kd, kb, qk, pv, ipv, LUk](lb::Ctx const& c) {
            trace::Block t2("getrf_bcast_row");
            if (pivot) {
                bcast(rowF, pv, size_t(6 * nb), qk, c);
                lb::copy2d(c, kd, int64_t(1), ipv, kd, ipiv_all.data() + k * nb, kd);
            }
            bcast(rowF, LUk, size_t(kd * kb), qk, c);
        });
        if (exact) {
            // the step's pivot slots on the host (one wait per step: the panel
            // queue drains, the trailing queues keep running), then the exact
            // exchange plans of the trailing ranges and of the left columns
            int64_t const* hp = pv;
            if (target == Target::Devices) {
                device::memcpy_async(hpv, pv, 6 * nb * sizeof(int64_t), S.ctx(qP).stream);
                // allowed host wait: the step's pivot slots (exact row exchange)
                slate_hip_call(hipStreamSynchronize(S.ctx(qP).stream));
                hp = hpv;
            }
            RPl[slot] = rowx_plan(rd, kd, hp + 2 * nb, hp + 4 * nb, true);
            LPl[slot] = rowx_plan(rd, kd, hp + 2 * nb, hp + 4 * nb, false);
            if (target == Target::Devices)
                S.task(qP, {}, {tPV}, [&, slot](lb::Ctx const& c) {
                    slate_error_if_msg(RPl[slot].flat.size() > pxn || LPl[slot].flat.size() > pxn, "getrf: row plan size");
                    device::memcpy_async(PX[slot].data(), RPl[slot].flat.data(), RPl[slot].flat.size() * sizeof(int64_t),
                                         c.stream);
                    device::memcpy_async(PXL[slot].data(), LPl[slot].flat.data(),
                                         LPl[slot].flat.size() * sizeof(int64_t), c.stream);
                });
        }
        S.task(qP, {}, {tW}, [&, kb, qk, mr, Wk](lb::Ctx const& c) {
            trace::Block t2("getrf_bcast_L");
            bcast(rowF, Wk, size_t(mr * kb), qk, c);
        });

        // ============================================== column ranges: U + update
        const int64_t ldu = pivot ? 2 * kd : kd;
        auto range = [&, k, kd, kb, pk, diag, lr_k, lr_k1, ldu, ssrc, sdst, LUk, Wk, ldw, tPV, tW](int queue, int64_t j0,
                                                                                                   int64_t j1) {
            const auto cc = lcols(j0, j1);
            const int64_t c0 = cc.first, nc = cc.second - cc.first;
            if (nc <= 0) return;
            std::vector<int64_t> cols;
            for (int64_t j = j0; j < j1; ++j) cols.push_back(Sched::col(j));
            T* buf = UB.data() + c0 * ldu;
            // permuted block row k of these columns -> buf (every process of
            // the column); lookahead columns on the critical-path lane
            const bool crit = (queue == device::kLookaheadQueue);
            Comm& cc_ = crit ? colF : g.col();
            if (pivot && exact) {
                RowXPlan const* P = &RPl[slot];
                int64_t const* ix = target == Target::Devices ? PX[slot].data() : RPl[slot].flat.data();
                T* sb = XS.data() + c0 * (p * nb);
                T* rb = XR.data() + c0 * (2 * nb);
                T* tb = XT.data() + c0 * (2 * nb);
                if (crit) {
                    S.task(qP, {tPV}, cols, [&, c0, nc, buf, P, ix, sb, rb, tb](lb::Ctx const& c) {
                        trace::Block t2("getrf_rows_exchange");
                        rowx_run<T>(c, *P, ix, nc, a + c0 * lda, lda, buf, ldu, sb, rb, tb, colF, 7);
                    });
                } else {
                    S.task(queue, {tPV}, cols, [&, c0, nc, buf, P, ix, sb, rb, tb](lb::Ctx const& c) {
                        trace::Block t2("getrf_rows_pack");
                        rowx_run<T>(c, *P, ix, nc, a + c0 * lda, lda, buf, ldu, sb, rb, tb, g.col(), 1);
                    });
                    S.task(qC, {}, cols, [&, c0, nc, buf, P, ix, sb, rb, tb](lb::Ctx const& c) {
                        trace::Block t2("getrf_rows_exchange");
                        rowx_run<T>(c, *P, ix, nc, a + c0 * lda, lda, buf, ldu, sb, rb, tb, g.col(), 2);
                    });
                    S.task(queue, {tPV}, cols, [&, c0, nc, buf, P, ix, sb, rb, tb](lb::Ctx const& c) {
                        trace::Block t2("getrf_rows_unpack");
                        rowx_run<T>(c, *P, ix, nc, a + c0 * lda, lda, buf, ldu, sb, rb, tb, g.col(), 4);
                    });
                }
            } else
            if (!crit && pivot) {
                // bulk lane: slot pack / unpack on the range's compute queue,
                // only the all-reduce on the comm queue (the cols tokens
                // order the three)
                S.task(queue, {tPV}, cols, [&, c0, nc, buf](lb::Ctx const& c) {
                    trace::Block t2("getrf_rows_pack");
                    slots_pack(c, 0, int(2 * kd), nc, ssrc, a + c0 * lda, lda, rd, buf, ldu);
                });
                S.task(qC, {}, cols, [&, nc, buf](lb::Ctx const& c) {
                    trace::Block t2("getrf_rows_exchange");
                    cc_.allreduce(buf, size_t(ldu * nc), ReduceOp::Sum, c.loc(), c.stream);
                });
                S.task(queue, {tPV}, cols, [&, c0, nc, buf](lb::Ctx const& c) {
                    trace::Block t2("getrf_rows_unpack");
                    slots_unpack(c, int(kd), int(2 * kd), nc, sdst, buf + kd, ldu, a + c0 * lda, lda, rd);
                });
            } else
            S.task(crit ? qP : qC, {tPV}, cols, [&, c0, nc, buf](lb::Ctx const& c) {
                trace::Block t2("getrf_rows_exchange");
                if (pivot) {
                    slots_pack(c, 0, int(2 * kd), nc, ssrc, a + c0 * lda, lda, rd, buf, ldu);
                    cc_.allreduce(buf, size_t(ldu * nc), ReduceOp::Sum, c.loc(), c.stream);
                    slots_unpack(c, int(kd), int(2 * kd), nc, sdst, buf + kd, ldu, a + c0 * lda, lda, rd);
                } else {
                    if (diag) lb::copy2d(c, kd, nc, a + lr_k + c0 * lda, lda, buf, ldu);
                    bcast(cc_, buf, size_t(ldu * nc), pk, c);
                }
            });
            std::vector<int64_t> in{tPV, tW};
            S.task(queue, in, cols, [&, c0, nc, buf](lb::Ctx const& c) {
                trace::Block t2("getrf_update");
                lb::trsm(c, Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, kd, nc, T(1), LUk, kd, buf, ldu);
                if (diag) lb::copy2d(c, kd, nc, buf, ldu, a + lr_k + c0 * lda, lda);
                lb::gemm(c, Op::NoTrans, Op::NoTrans, mloc - lr_k1, nc, kd, T(-1), Wk + (lr_k1 - lr_k), ldw,
                         buf, ldu, T(1), a + lr_k1 + c0 * lda, lda);
            });
        };
        const int64_t jla_end = std::min(nt, k + 1 + la);
        for (int64_t j = k + 1; j < jla_end; ++j) range(device::kLookaheadQueue, j, j + 1);
        if (jla_end < nt) {
            const int64_t ntr = nt - jla_end;
            const int64_t nch = std::min<int64_t>(4, ntr);
            for (int64_t ch = 0; ch < nch; ++ch)
                range(device::kTrailQueue, jla_end + ch * ntr / nch, jla_end + (ch + 1) * ntr / nch);
        }
        // interchanges of the previous step on its left columns
        left(k - 1);
    }
    left(kt - 1);
    S.wait_all();

    // pivots -> Pivots (tile index relative to k, offset within the tile)
    std::vector<int64_t> ip(size_t(std::max<int64_t>(kt, 1)) * nb, 0);
    if (target == Target::Devices) {
        if (pivot) device::memcpy_async(ip.data(), ipiv_all.data(), ip.size() * sizeof(int64_t), S.ctx(qP).stream);
        slate_hip_call(hipStreamSynchronize(S.ctx(qP).stream));
    } else if (pivot) {
        std::copy(ipiv_all.data(), ipiv_all.data() + ip.size(), ip.begin());
    }
    pivots.assign(kt, {});
    for (int64_t k = 0; k < kt; ++k) {
        int64_t kk = grow_of(A, k), kd = std::min(A.tileNb(k), m - kk);
        pivots[k].resize(kd);
        for (int64_t t = 0; t < kd; ++t) {
            int64_t r = pivot ? ip[k * nb + t] : kk + t;
            int64_t ti = 0;
            while (ti + k + 1 < mt && grow_of(A, k + ti + 1) <= r) ++ti;
            pivots[k][t] = Pivot(ti, r - grow_of(A, k + ti));
        }
    }
    int64_t info = fetch_info(target, info_real);
    info = reduce_info(info, g.world());
    internal::finish_origin(A, opts);
    (void)n;
    return info;
}

template <typename T>
int64_t getrf_impl(Matrix<T>& A_in, Pivots& pivots, Options const& opts, PanelMode mode) {
    trace::Block tb("getrf");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    const int64_t la = get_option<int64_t>(opts, Option::Lookahead, 1);
    const double thresh = pivot_threshold(opts);
    slate_error_if_msg(A_in.op() != Op::NoTrans, "getrf: NoTrans view required");
    slate_error_if_msg(!A_in.aligned(), "getrf: tile-aligned matrix required");
    slate_error_if_msg(A_in.mb() != A_in.nb(), "getrf: square tiles required");
    BaseMatrix<T> A = A_in;
    auto& g = *A.grid();
    if (g.p() > 1) return getrf_dist(A, pivots, opts, mode, target);
    // ---- p == 1: the panel column is local to one process; pivots travel
    // along the process row as device (dst, src) row pairs
    const int q = g.q(), mycol = g.mycol();
    const Loc loc = loc_of(target);
    const int64_t mt = A.mt(), nt = A.nt(), m = A.m();
    const int64_t kt = std::min(mt, nt);
    const int64_t nb = A.nb();
    LocalBlock<T> L = A.local(loc, true);
    T* a = L.ptr;
    const int64_t lda = L.ld, mloc = L.m, nloc = L.n;
    const bool pivot = (mode != PanelMode::NoPiv);
    const bool tnt = (mode == PanelMode::Tournament);

    Sched S(target);
    const int R = int(std::max<int64_t>(2, la + 2));
    // SLATE_GETRF_LINV=1: L(k,k)^{-1} once per step, shared by the range
    // tasks' U solves.  Off by default: neutral for fp64 (same-box A/B, 3450 vs
    // 3454 ms at n=65536) and, applied to the fp32 factor of dgesv_mixed, the
    // inverse-based U rows cost accuracy: 24-29 instead of 9 refinement
    // iterations (profiles/r2_ab_linv.txt)
    static const bool linv_env = [] {
        const char* e = std::getenv("SLATE_GETRF_LINV");
        return e ? std::atoi(e) != 0 : false;
    }();
    const bool use_linv = linv_env && target == Target::Devices;
    // SLATE_UPDATE_TN=1: trailing update as a TN product against a once-per-
    // step transposed copy of L21 (both operands K-contiguous, rotated 8-wave
    // MFMA tile) instead of the NT form
    static const bool tn_env = [] {
        const char* e = std::getenv("SLATE_UPDATE_TN");
        return e && std::atoi(e) != 0;
    }();
    const bool use_tn = tn_env && !is_complex_v<T> && target == Target::Devices;
    std::vector<Work<T>> W(R), WU(R), WI(R), WLT(R);
    // pivot slots live in a deeper ring than the panel buffers: the left
    // swaps of step k (comm queue, off the critical path) read PV up to RP
    // steps later before panel k + RP may rewrite it (token tPV, WAR)
    const int RP = R + 8;
    std::vector<Work<int64_t>> PV(RP);     // [ipiv(kb) | dst(2kb) | src(2kb) | count]
    for (int r = 0; r < R; ++r) {
        W[r].resize(target, size_t(std::max<int64_t>(mloc, 1)) * nb);
        WU[r].resize(target, size_t(nb) * std::max<int64_t>(nloc, 1));
        WI[r].resize(target, size_t(nb) * nb);
        if (use_tn) WLT[r].resize(target, size_t(nb) * std::max<int64_t>(mloc, 1));
        (void)0;
    }
    for (int r = 0; r < RP; ++r) PV[r].resize(target, size_t(5 * nb + 8));
    Work<int64_t> perm(target, size_t(std::max<int64_t>(m, 1)));
    Work<int> dinfo(target, 1);
    // every step's panel-relative pivots, copied to the host once at the end
    Work<int64_t> ipiv_all(target, size_t(std::max<int64_t>(kt, 1)) * nb);
    {
        lb::Ctx c0 = S.ctx(1);
        if (c0.dev()) device::memset_async(dinfo.data(), 0, sizeof(int), c0.stream);
        else dinfo.data()[0] = 0;
    }
    // left columns [0, k): apply the step's interchanges.  Off the trailing
    // queue (the comm queue is idle on a p == 1 grid): nothing on the
    // critical path reads these columns again, so the memory-bound swaps
    // overlap the trailing GEMM instead of serializing before it
    static const int left_q = [] {
        const char* e = std::getenv("SLATE_LU_LEFT_TRAIL");   // A/B: 1 = back on the trailing queue
        return (e && std::atoi(e)) ? device::kTrailQueue : device::kCommQueue;
    }();
    // 1x1 device grid, square: once the remaining matrix is at most `tail_w`
    // wide, factor it with ONE recursive device panel (32-column tournament /
    // partial-pivoting narrow blocks, trsm + GEMM recursion) instead of
    // nb-wide steps whose panels are exposed once the trailing GEMM has shrunk
    // (at nb = 2048 the last panels cost ~20 ms each beside < 1 ms of GEMM).
    // SLATE_GETRF_TAIL = width (0: off); the left-column permutation of the
    // tail is one LDS-staged pass, so the width is capped at 64 KB of rows.
    static const int64_t tail_env = [] {
        const char* e = std::getenv("SLATE_GETRF_TAIL");
        return e ? std::atoll(e) : int64_t(0);
    }();
    const int64_t tail_w = std::min<int64_t>(tail_env, int64_t(65536 / sizeof(T)));
    const bool tail_ok = q == 1 && target == Target::Devices && pivot && tail_w > 0 && m == A.n();
    int64_t tail_k = kt;                     // first tile of the tail (kt: none)
    Work<int64_t> tpv;                       // [ipiv(w) | dst(2w) | src(2w)]
    if (tail_ok) tpv.resize(target, size_t(5 * tail_w + 8));
    // Deferred left interchanges: once the remaining matrix is at most m / D
    // tall (SLATE_LU_DEFER_LEFT = D, default 2, 0 = off), the steps' row
    // interchanges are no longer applied to the left columns [0, k_def) step
    // by step -- in the tail those swaps of up to 2 kb rows across almost the
    // whole width ran beside trailing GEMMs too small to hide them
    // (profiles/r6_final_trace_dgetrf.txt: 136 ms of permute_rows in the last
    // decile's GEMM-idle windows) -- but composed on the host at the end and
    // applied once: each moved row of those columns is gathered and scattered
    // a single time.  n = 65536: dgetrf 3203-3207 ms (off) -> 3174 ms (D = 2),
    // 3191 ms (D = 4), interleaved (profiles/r6_lu_defer_left_ab.txt).
    static const double defer_div = [] {
        const char* e = std::getenv("SLATE_LU_DEFER_LEFT");
        return e ? std::atof(e) : 2.0;
    }();
    int64_t k_def = kt;
    if (pivot && target == Target::Devices && defer_div >= 1.0 && !tail_ok)
        for (int64_t k = 1; k < kt; ++k)
            if (double(m - grow_of(A, k)) * defer_div <= double(m)) { k_def = k; break; }

    for (int64_t k = 0; k < kt; ++k) {
        const int64_t kb = A.tileNb(k);
        const int64_t kk = grow_of(A, k);
        const int64_t M = m - kk;                         // panel rows (global)
        const int64_t kd = std::min(kb, M);                // pivots this step
        const int qk = A.scol_owner(k);
        if (tail_ok && k > 0 && M <= tail_w) {
            tail_k = k;
            std::vector<int64_t> cols;
            for (int64_t j = k; j < nt; ++j) cols.push_back(Sched::col(j));
            std::vector<int64_t> outs = cols;
            const int64_t tT = Sched::tok(15, 0);
            outs.push_back(tT);
            int64_t* tp = tpv.data();
            S.task(1, cols, outs, [&, k, kk, M, tp](lb::Ctx const& c) {
                trace::Block t2("getrf_tail");
                lb::getrf_panel(c, M, M, a + kk + kk * lda, lda, tp, perm.data(), dinfo.data(), kk, pivot, tnt,
                                thresh);
                // square: the first M pairs (t <- perm[t]) already cover every row
                slate_amd::dev::perm_pairs(M, perm.data(), tp, tp + tail_w, tp + 3 * tail_w, c.stream);
                lb::copy2d(c, M, int64_t(1), tp, M, ipiv_all.data() + k * nb, M);
            });
            S.task(left_q, {tT}, {Sched::tok(11, 0), Sched::col(k - 1)}, [&, kk, M, tp](lb::Ctx const& c) {
                slate_amd::dev::permute_rows(kk, slate_amd::dev::dptr(a + kk), lda, tp + tail_w, tp + 3 * tail_w,
                                             nullptr, int(M), c.stream);
            });
            break;
        }
        const bool in_col = (mycol == qk);
        const int64_t lr_k = lrow_of(A, k), lr_k1 = lrow_of(A, k + 1);
        const int64_t lc_k = in_col ? lcol_of(A, k) : 0;
        const int slot = int(k % R);
        const int pvs = int(k % RP);
        int64_t* pv = PV[pvs].data();
        const int64_t tPV = Sched::tok(14, pvs);
        int64_t* pv_ipiv = pv;
        int64_t* pv_dst = pv + nb;
        int64_t* pv_src = pv + 3 * nb;
        const int64_t tPanel = Sched::tok(6, slot), tBc = Sched::bcast(slot);

        // ------------------------------------------------------------ panel
        if (in_col) {
            // (writes PV[pvs]: tPV orders it after that slot's last readers)
            S.task(1, {}, {Sched::col(k), tPanel, tPV}, [&, k, kb, kk, M, kd, lr_k, lc_k, pv_ipiv, pv_dst, pv_src](lb::Ctx const& c) {
                trace::Block t2("getrf_panel");
                T* ap = a + lr_k + lc_k * lda;
                lb::getrf_panel(c, M, kb, ap, lda, pv_ipiv, perm.data(), dinfo.data(), kk, pivot, tnt, thresh);
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

        // ------------------------------- (ipiv, pairs) along the process row
        // (critical path: on the panel queue over the fast-lane row comm)
        S.task(1, {tPanel}, {tBc, tPV}, [&, k, kd, pvs, pv_ipiv](lb::Ctx const& c) {
            trace::Block t2("getrf_bcast_piv");
            bcast(g.row_fast(), PV[pvs].data(), size_t(5 * nb + 8), qk, c);
            if (pivot) lb::copy2d(c, kd, int64_t(1), pv_ipiv, kd, ipiv_all.data() + k * nb, kd);
        });

        // ----------------------------------------- L panel along process rows
        T* Wk = W[slot].data();
        const int64_t mrows_k = mloc - lr_k;     // my rows >= kk
        S.task(1, {Sched::col(k), tBc}, {Sched::tok(7, slot)}, [&, lr_k, lc_k, kb, qk, Wk, mrows_k](lb::Ctx const& c) {
            trace::Block t2("getrf_bcast_L");
            if (mycol == qk) pack(c, mrows_k, kb, a + lr_k + lc_k * lda, lda, Wk);
            if (q > 1) bcast(g.row_fast(), Wk, size_t(mrows_k * kb), qk, c);
        });
        const int64_t tL = Sched::tok(7, slot);
        // L(k,k)^{-1} once per step (device): every column range's U solve is
        // then one GEMM instead of re-inverting the triangle (~10 launches)
        // in each of the lookahead and trailing tasks
        T* Ltk = use_tn ? WLT[slot].data() : nullptr;
        const int64_t tLt = Sched::tok(13, slot);
        if (use_tn && mloc > lr_k1)
            S.task(1, {tL}, {tLt}, [&, kd, Wk, Ltk, mrows_k, lr_k, lr_k1](lb::Ctx const& c) {
                trace::Block t2("getrf_lt");
                lb::copy<T, T>(c, Uplo::General, Op::Trans, kd, mloc - lr_k1, Wk + (lr_k1 - lr_k),
                               std::max<int64_t>(mrows_k, 1), Ltk, kd);
            });
        T* Lik = WI[slot].data();
        const int64_t tLi = Sched::tok(12, slot);
        if (use_linv)
            S.task(1, {tL}, {tLi}, [&, kd, Wk, Lik, mrows_k](lb::Ctx const& c) {
                trace::Block t2("getrf_linv");
                lb::trtri_to(c, Uplo::Lower, Diag::Unit, kd, Wk, std::max<int64_t>(mrows_k, 1), Lik, kd);
            });

        // -------------------------------------- column ranges: permute, U, update
        // apply the step's row permutation to local columns [c0, c1)
        auto permute = [&, kk, kd, pvs](lb::Ctx const& c, int64_t c0, int64_t c1) {
            if (c1 <= c0 || !pivot) return;
            // rows: local == global; pairs relative to kk
            int64_t* pvv = PV[pvs].data();
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
        };
        // columns of tiles [j0, j1) local to me
        auto lcols = [&](int64_t j0, int64_t j1) { return std::make_pair(lcol_of(A, j0), lcol_of(A, j1)); };
        T* WUk = WU[slot].data();
        // U row height is kd = tileMb(k) (< kb only for the last block row of a
        // wide matrix; rows beyond it are not part of the matrix)
        auto urow = [&, kd, lr_k, Wk, Lik, WUk, use_linv](lb::Ctx const& c, int64_t j0, int64_t j1) {
            auto cc = lcols(j0, j1);
            int64_t c0 = cc.first, c1 = cc.second;
            if (c1 <= c0) return;
            if (use_linv) {
                // U = L^{-1} A(k, cols) through a copy in this range's slice of WU
                const int64_t nc = c1 - c0;
                T* Ac = a + lr_k + c0 * lda;
                T* tmp = WUk + c0 * kd;
                lb::copy2d(c, kd, nc, Ac, lda, tmp, kd);
                lb::gemm(c, Op::NoTrans, Op::NoTrans, kd, nc, kd, T(1), Lik, kd, tmp, kd, T(0), Ac, lda);
                return;
            }
            // U(k, j0:j1) = L(k,k)^{-1} A(k, j0:j1); L(k,k) = top kd rows of W_k
            lb::trsm(c, Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, kd, c1 - c0, T(1),
                     Wk, std::max<int64_t>(mrows_k, 1), a + lr_k + c0 * lda, lda);
        };
        auto update = [&, kb, kd, lr_k1, lr_k, Wk, WUk, Ltk, use_tn](lb::Ctx const& c, int64_t j0, int64_t j1) {
            auto cc = lcols(j0, j1);
            int64_t c0 = cc.first, nc = cc.second - cc.first, nr = mloc - lr_k1;
            if (nc <= 0 || nr <= 0) return;
            trace::Block t2("getrf_update");
            // U rows of these columns live in A itself (process row 0 owns them)
            if (use_tn) {
                lb::gemm(c, Op::Trans, Op::NoTrans, nr, nc, kd, T(-1), Ltk, kd, a + lr_k + c0 * lda, lda, T(1),
                         a + lr_k1 + c0 * lda, lda);
                return;
            }
            if (!is_complex_v<T> && c.dev() && update_nt()) {
                // NT product against U^T (nc x kd, ld nc) in this range's own
                // slice of the slot's WU buffer
                T* Ut = WUk + c0 * kd;
                lb::copy<T, T>(c, Uplo::General, Op::Trans, nc, kd, a + lr_k + c0 * lda, lda, Ut, nc);
                lb::gemm(c, Op::NoTrans, Op::Trans, nr, nc, kd, T(-1), Wk + (lr_k1 - lr_k),
                         std::max<int64_t>(mrows_k, 1), Ut, nc, T(1), a + lr_k1 + c0 * lda, lda);
                return;
            }
            lb::gemm(c, Op::NoTrans, Op::NoTrans, nr, nc, kb, T(-1), Wk + (lr_k1 - lr_k), std::max<int64_t>(mrows_k, 1),
                     a + lr_k + c0 * lda, lda, T(1), a + lr_k1 + c0 * lda, lda);
        };

        auto range_tasks = [&](int queue, int64_t j0, int64_t j1) {
            std::vector<int64_t> cols;
            for (int64_t j = j0; j < j1; ++j) cols.push_back(Sched::col(j));
            std::vector<int64_t> in = {tBc, tL, tPV};
            if (use_linv) in.push_back(tLi);
            if (use_tn && mloc > lr_k1) in.push_back(tLt);
            S.task(queue, in, cols, [&, j0, j1](lb::Ctx const& c) {
                auto cc = lcols(j0, j1);
                permute(c, cc.first, cc.second);
                urow(c, j0, j1);
                update(c, j0, j1);
            });
        };
        int64_t jla_end = std::min(nt, k + 1 + la);
        for (int64_t j = k + 1; j < jla_end; ++j)
            range_tasks(device::kLookaheadQueue, j, j + 1);
        // 1x1 device grid: the trailing range in two parts, A (the first
        // 1/split_div of it) on the trailing queue and B on the idle comm
        // queue, B starting once A's row interchanges and U rows are done.
        // The interchanges are memory-bound scattered-row gathers (one 128-byte
        // line per moved element: ~3 ms a step at n = 65536) that otherwise
        // serialize before the one trailing GEMM; here only A's are exposed,
        // B's run under A's GEMM.  SLATE_LU_TRAIL_SPLIT = split_div (0: off,
        // the default: same-box n = 65536 dgetrf 54.8 TFLOP/s unsplit against
        // 53.4-53.8 at 4 / 8 / 16, dgesv_mixed neutral -- two concurrent
        // trailing GEMMs lose more than the hidden interchanges gain;
        // profiles/r4_lu_split_potrf_rec.txt).
        static const int64_t split_div = [] {
            const char* e = std::getenv("SLATE_LU_TRAIL_SPLIT");
            return e ? std::atoll(e) : int64_t(0);
        }();
        const int64_t nrest = nt - jla_end;
        if (nrest >= 2 && split_div > 0 && q == 1 && target == Target::Devices && pivot) {
            const int64_t ja = jla_end + std::max<int64_t>(1, nrest / split_div);
            const int64_t tA = Sched::tok(16, slot);
            std::vector<int64_t> colsA, colsB;
            for (int64_t j = jla_end; j < ja; ++j) colsA.push_back(Sched::col(j));
            for (int64_t j = ja; j < nt; ++j) colsB.push_back(Sched::col(j));
            std::vector<int64_t> in = {tBc, tL, tPV};
            if (use_linv) in.push_back(tLi);
            if (use_tn && mloc > lr_k1) in.push_back(tLt);
            std::vector<int64_t> outA = colsA;
            outA.push_back(tA);
            S.task(device::kTrailQueue, in, outA, [&, jla_end, ja](lb::Ctx const& c) {
                auto cc = lcols(jla_end, ja);
                permute(c, cc.first, cc.second);
                urow(c, jla_end, ja);
            });
            S.task(device::kTrailQueue, in, colsA, [&, jla_end, ja](lb::Ctx const& c) { update(c, jla_end, ja); });
            std::vector<int64_t> inB = in;
            inB.push_back(tA);
            S.task(device::kCommQueue, inB, colsB, [&, ja](lb::Ctx const& c) {
                auto cc = lcols(ja, nt);
                permute(c, cc.first, cc.second);
                urow(c, ja, nt);
                update(c, ja, nt);
            });
        } else if (jla_end < nt) {
            range_tasks(device::kTrailQueue, jla_end, nt);
        }

        if (k > 0 && pivot && k != k_def) {
            // reads PV[pvs] (tPV): the panel that next rewrites the slot, RP
            // steps later, waits for it (write-after-read across queues)
            S.task(left_q, {tPV}, {Sched::tok(11, 0), Sched::col(k - 1)}, [&, k](lb::Ctx const& c) {
                auto cc = lcols(k > k_def ? k_def : 0, k);   // [0, k_def) deferred
                permute(c, cc.first, cc.second);
            });
        }
    }
    S.wait_all();
    // pivots -> reference Pivots structure: (tile index relative to k, offset)
    std::vector<int64_t> ip(size_t(std::max<int64_t>(kt, 1)) * nb, 0);
    if (pivot) {
        if (target == Target::Devices) {
            hipStream_t s1 = S.ctx(1).stream;
            device::memcpy_async(ip.data(), ipiv_all.data(), ip.size() * sizeof(int64_t), s1);
            slate_hip_call(hipStreamSynchronize(s1));
        } else {
            std::copy(ipiv_all.data(), ipiv_all.data() + ip.size(), ip.begin());
        }
    }
    if (k_def < kt) {
        // the deferred interchanges of steps k_def.. on local columns [0, k_def):
        // compose them (row i of the result holds original row where[i]),
        // then gather the moved rows and scatter them to their places
        const int64_t r0 = grow_of(A, k_def), R = m - r0;
        std::vector<int64_t> where(static_cast<size_t>(R), int64_t(0));
        std::iota(where.begin(), where.end(), int64_t(0));
        for (int64_t k = k_def; k < kt; ++k) {
            const int64_t kk = grow_of(A, k) - r0, kd = std::min(A.tileNb(k), m - r0 - kk);
            for (int64_t t = 0; t < kd; ++t) std::swap(where[kk + t], where[kk + ip[k * nb + t]]);
        }
        std::vector<int64_t> idx;   // [src rows | dst rows], relative to r0
        for (int64_t i = 0; i < R; ++i) if (where[i] != i) idx.push_back(where[i]);
        const int64_t cnt = int64_t(idx.size());
        for (int64_t i = 0; i < R; ++i) if (where[i] != i) idx.push_back(i);
        const int64_t ncl = lcol_of(A, k_def);
        if (cnt > 0 && ncl > 0) {
            lb::Ctx c = S.ctx(left_q);
            Work<int64_t> didx(target, idx.size());
            device::memcpy_async(didx.data(), idx.data(), idx.size() * sizeof(int64_t), c.stream);
            const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(ncl, 32768));
            Work<T> buf(target, size_t(cnt) * chunk);
            for (int64_t j0 = 0; j0 < ncl; j0 += chunk) {
                const int64_t nc = std::min(chunk, ncl - j0);
                T* a0 = a + r0 + j0 * lda;
                slate_amd::dev::rows_pack(nc, slate_amd::dev::dptr(a0), lda, didx.data(), int(cnt),
                                          slate_amd::dev::dptr(buf.data()), false, c.stream);
                slate_amd::dev::rows_pack(nc, slate_amd::dev::dptr(a0), lda, didx.data() + cnt, int(cnt),
                                          slate_amd::dev::dptr(buf.data()), true, c.stream);
            }
            slate_hip_call(hipStreamSynchronize(c.stream));
        }
    }
    pivots.assign(kt, {});
    for (int64_t k = 0; k < kt; ++k) {
        int64_t kk = grow_of(A, k), kd = std::min(A.tileNb(k), m - kk);
        // the tail's pivots are relative to its first row
        const int64_t base = k >= tail_k ? grow_of(A, tail_k) : kk;
        pivots[k].resize(kd);
        for (int64_t t = 0; t < kd; ++t) {
            int64_t r = pivot ? ip[k * nb + t] + base : kk + t;
            // tile index relative to k and offset within the tile
            int64_t ti = 0;
            while (ti + k + 1 < mt && grow_of(A, k + ti + 1) <= r) ++ti;
            pivots[k][t] = Pivot(ti, r - grow_of(A, k + ti));
        }
    }
    int64_t info = fetch_info(target, dinfo.data());
    info = reduce_info(info, g.world());
    internal::finish_origin(A, opts);
    return info;
}

}  // namespace

template <typename T>
int64_t getrf(Matrix<T>& A, Pivots& pivots, Options const& opts) {
    {   // one process, several GPUs: in-process ranks (spread.hh)
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
                Pivots P;
                const int64_t i = getrf(M[0], P, opts);
                if (rank == 0) { info = i; pivots = P; }
            }))
            return info;
    }
    if (A.arbitrary_layout()) {
        Matrix<T> Ab = internal::block_cyclic(A, opts);
        int64_t info = getrf(Ab, pivots, opts);
        slate::copy<T, T>(Ab, A, opts);
        return info;
    }
    Method m = get_option<int64_t>(opts, Option::MethodLU, MethodLU::PartialPiv);
    return getrf_impl(A, pivots, opts, m == MethodLU::NoPiv ? PanelMode::NoPiv :
                      (m == MethodLU::CALU ? PanelMode::Tournament : PanelMode::Partial));
}

template <typename T>
int64_t getrf_tntpiv(Matrix<T>& A, Pivots& pivots, Options const& opts) {
    {
        int64_t info = 0;
        if (internal::spread<T>(opts, {{&A, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
                Pivots P;
                const int64_t i = getrf_tntpiv(M[0], P, opts);
                if (rank == 0) { info = i; pivots = P; }
            }))
            return info;
    }
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

/// Counters of the exact LU row exchange on this process (elements sent,
/// rows sent summed over column ranges); reset with lu_rowx_reset().
void lu_rowx_stats(int64_t& elems, int64_t& rows) { elems = rowx_stats().elems; rows = rowx_stats().rows; }
void lu_rowx_reset() { rowx_stats().elems = 0; rowx_stats().rows = 0; }

#define SLATE_GETRF_INST(T)                                                                  \
    template int64_t getrf<T>(Matrix<T>&, Pivots&, Options const&);                         \
    template int64_t getrf_tntpiv<T>(Matrix<T>&, Pivots&, Options const&);                  \
    template int64_t getrf_nopiv<T>(Matrix<T>&, Options const&);

SLATE_GETRF_INST(float)
SLATE_GETRF_INST(double)
SLATE_GETRF_INST(std::complex<float>)
SLATE_GETRF_INST(std::complex<double>)

}  // namespace slate
