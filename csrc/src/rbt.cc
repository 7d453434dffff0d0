// Random butterfly transforms (reference src/gerbt.cc, gesv_rbt.cc,
// internal_gerbt.cc, internal_rbt_generate.cc; Parker 1995, Baboulin, Dongarra,
// Herrmann & Tomov 2013): A' = U^T A V with recursive butterflies U, V of
// depth d, so that LU WITHOUT pivoting of A' is stable with high probability;
// x = V y, then iterative refinement against the original A.
//
// U = L_{d-1} ... L_0, where level l splits the index range into 2^l blocks
// and pairs index i with i + h inside each block (h = half the block):
//   L = 1/sqrt(2) [D0  D1; D0  -D1]   (D0, D1 random diagonals near 1).
// Every level is therefore a per-index combination x_i <- ca_i x_i + cp_i x_pi
// of an index with its partner: O(m n) work per level (O(n^2 d) in total)
// applied by the rbt.hip kernels, with ONE grouped exchange of the partner
// rows (columns) over the column (row) communicator when the partner lives on
// another process.  The random values come from a counter-based hash of
// (seed, level, index), so U and V never depend on the process grid.
#include "internal.hh"
#include "../kernels/kernels.hh"

#include <algorithm>
#include <cmath>

namespace slate {

using namespace internal;

namespace {

namespace kd = slate_amd::dev;
using kd::dptr;

inline double rbt_rand(uint64_t seed, uint64_t level, uint64_t idx) {
    // SplitMix64 on (seed, level, idx) -> r in [-0.5, 0.5]; entry exp(r / 10)
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + level * 0xBF58476D1CE4E5B9ull + idx * 0x94D049BB133111EBull;
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    double r = double(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    return std::exp(r / 10.0);
}

/// index gi of a length-N butterfly at level lev: its partner and the
/// coefficients of  x_gi <- ca x_gi + cp x_partner  for L (trans = false) or
/// L^T (trans = true).  A middle index of an odd block is left alone.
struct BflyEntry { int64_t partner; double ca, cp; };
inline BflyEntry bfly_entry(int64_t N, int lev, int64_t gi, uint64_t seed, bool trans) {
    const int64_t nblk = int64_t(1) << lev;
    int64_t b = gi * nblk / N;
    while (b + 1 < nblk && N * (b + 1) / nblk <= gi) ++b;
    while (b > 0 && N * b / nblk > gi) --b;
    const int64_t r0 = N * b / nblk, r1 = N * (b + 1) / nblk, h = (r1 - r0) / 2, r = gi - r0;
    if (r >= 2 * h) return {gi, 1.0, 0.0};
    const double s2 = 1.0 / std::sqrt(2.0);
    const bool top = r < h;
    const int64_t ip = top ? gi : gi - h;
    const double R0 = rbt_rand(seed, lev, 2 * ip), R1 = rbt_rand(seed, lev, 2 * ip + 1);
    // L:   top' = s2 (R0 top + R1 bot),  bot' = s2 (R0 top - R1 bot)
    // L^T: top' = s2 R0 (top + bot),     bot' = s2 R1 (top - bot)
    if (top) return {gi + h, s2 * R0, s2 * (trans ? R0 : R1)};
    return {ip, -s2 * R1, s2 * (trans ? R1 : R0)};
}

/// One butterfly level on the rows (by_rows) or columns of X (NoTrans, whole
/// matrix: row0 = col0 = 0).
template <typename T>
void bfly_level(Matrix<T>& X, bool by_rows, int lev, uint64_t seed, bool trans, Target target) {
    using R = real_type<T>;
    const int64_t N = by_rows ? X.m() : X.n();
    if (N < 2) return;
    auto& g = *X.grid();
    const Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    LocalBlock<T> lx = X.local(loc, true);
    const int64_t nl = by_rows ? lx.m : lx.n, len = by_rows ? lx.n : lx.m;
    const int me = by_rows ? g.myrow() : g.mycol(), np = by_rows ? g.p() : g.q();
    const int64_t tsz = by_rows ? X.mb() : X.nb(), ntl = by_rows ? X.mt() : X.nt();
    auto owner = [&](int64_t t) { return by_rows ? X.srow_owner(t) : X.scol_owner(t); };
    auto lstart = [&](int64_t t) { return by_rows ? lrow_of(X, t) : lcol_of(X, t); };
    std::vector<R> ca(size_t(std::max<int64_t>(nl, 1)), R(1)), cp(ca.size(), R(0));
    std::vector<int64_t> self_dst, self_src;
    std::vector<std::vector<std::pair<int64_t, int64_t>>> per(np);   // (pair key, my local index)
    for (int64_t t = 0; t < ntl; ++t) {
        if (owner(t) != me) continue;
        const int64_t sz = by_rows ? X.tileMb(t) : X.tileNb(t), l0 = lstart(t);
        for (int64_t o = 0; o < sz; ++o) {
            const int64_t gi = t * tsz + o, li = l0 + o;
            BflyEntry e = bfly_entry(N, lev, gi, seed, trans);
            ca[li] = R(e.ca);
            cp[li] = R(e.cp);
            const int po = owner(e.partner / tsz);
            if (po == me) {
                self_dst.push_back(li);
                self_src.push_back(lstart(e.partner / tsz) + e.partner % tsz);
            } else {
                per[po].push_back({std::min(gi, e.partner), li});
            }
        }
    }
    std::vector<int64_t> off(np + 1, 0), sidx;
    for (int o = 0; o < np; ++o) {
        std::sort(per[o].begin(), per[o].end());
        off[o + 1] = off[o] + int64_t(per[o].size());
        for (auto& kv : per[o]) sidx.push_back(kv.second);
    }
    const int64_t nself = int64_t(self_dst.size()), nsend = off[np];
    const int64_t ldp = std::max<int64_t>(lx.m, 1);
    Work<T> P(target, size_t(ldp) * std::max<int64_t>(lx.n, 1));
    Work<T> tmp(target, size_t(std::max<int64_t>(nself, 1)) * std::max<int64_t>(len, 1));
    Work<T> sb(target, size_t(std::max<int64_t>(nsend, 1)) * std::max<int64_t>(len, 1));
    Work<T> rb(target, sb.size());
    if (!c.dev()) {
        auto at = [&](T* A, int64_t ld, int64_t idx, int64_t k) -> T& { return by_rows ? A[idx + k * ld] : A[k + idx * ld]; };
        for (int64_t t = 0; t < nself; ++t)
            for (int64_t k = 0; k < len; ++k) at(P.data(), ldp, self_dst[t], k) = at(lx.ptr, lx.ld, self_src[t], k);
        for (int o = 0; o < np; ++o) {
            const int64_t cnt = off[o + 1] - off[o];
            T* seg = sb.data() + off[o] * len;
            for (int64_t t = 0; t < cnt; ++t)
                for (int64_t k = 0; k < len; ++k)
                    (by_rows ? seg[t + k * cnt] : seg[k + t * len]) = at(lx.ptr, lx.ld, sidx[off[o] + t], k);
        }
    } else {
        std::vector<int64_t> hidx(self_dst);
        hidx.insert(hidx.end(), self_src.begin(), self_src.end());
        hidx.insert(hidx.end(), sidx.begin(), sidx.end());
        Work<int64_t> didx(target, std::max<size_t>(hidx.size(), 1));
        Work<R> dco(target, 2 * ca.size());
        if (!hidx.empty()) device::memcpy_async(didx.data(), hidx.data(), hidx.size() * sizeof(int64_t), c.stream);
        device::memcpy_async(dco.data(), ca.data(), ca.size() * sizeof(R), c.stream);
        device::memcpy_async(dco.data() + ca.size(), cp.data(), cp.size() * sizeof(R), c.stream);
        const int64_t* d_dst = didx.data();
        const int64_t* d_src = didx.data() + nself;
        const int64_t* d_snd = didx.data() + 2 * nself;
        kd::rbt_gather(by_rows, false, nself, len, d_src, dptr(lx.ptr), lx.ld, dptr(tmp.data()),
                       by_rows ? std::max<int64_t>(nself, 1) : len, c.stream);
        kd::rbt_gather(by_rows, true, nself, len, d_dst, dptr(P.data()), ldp, dptr(tmp.data()),
                       by_rows ? std::max<int64_t>(nself, 1) : len, c.stream);
        for (int o = 0; o < np; ++o) {
            const int64_t cnt = off[o + 1] - off[o];
            kd::rbt_gather(by_rows, false, cnt, len, d_snd + off[o], dptr(lx.ptr), lx.ld,
                           dptr(sb.data() + off[o] * len), by_rows ? cnt : len, c.stream);
        }
        // exchange, unpack and combine below run on the same stream
        std::vector<Comm::P2P> ops;
        for (int o = 0; o < np; ++o) {
            const int64_t cnt = off[o + 1] - off[o];
            if (cnt == 0) continue;
            ops.push_back({sb.data() + off[o] * len, size_t(cnt * len), o, true});
            ops.push_back({rb.data() + off[o] * len, size_t(cnt * len), o, false});
        }
        if (!ops.empty()) (by_rows ? g.col() : g.row()).exchange(ops, scalar_type<T>(), loc, c.stream);
        for (int o = 0; o < np; ++o) {
            const int64_t cnt = off[o + 1] - off[o];
            kd::rbt_gather(by_rows, true, cnt, len, d_snd + off[o], dptr(P.data()), ldp,
                           dptr(rb.data() + off[o] * len), by_rows ? cnt : len, c.stream);
        }
        kd::rbt_combine(by_rows, lx.m, lx.n, dptr(lx.ptr), lx.ld, dptr(P.data()), ldp, dco.data(),
                        dco.data() + ca.size(), c.stream);
        slate_hip_call(hipStreamSynchronize(c.stream));
        return;
    }
    // host: exchange, unpack, combine
    std::vector<Comm::P2P> ops;
    for (int o = 0; o < np; ++o) {
        const int64_t cnt = off[o + 1] - off[o];
        if (cnt == 0) continue;
        ops.push_back({sb.data() + off[o] * len, size_t(cnt * len), o, true});
        ops.push_back({rb.data() + off[o] * len, size_t(cnt * len), o, false});
    }
    if (!ops.empty()) (by_rows ? g.col() : g.row()).exchange(ops, scalar_type<T>(), loc, nullptr);
    for (int o = 0; o < np; ++o) {
        const int64_t cnt = off[o + 1] - off[o];
        T const* seg = rb.data() + off[o] * len;
        for (int64_t t = 0; t < cnt; ++t) {
            const int64_t li = sidx[off[o] + t];
            for (int64_t k = 0; k < len; ++k)
                (by_rows ? P.data()[li + k * ldp] : P.data()[k + li * ldp]) = by_rows ? seg[t + k * cnt] : seg[k + t * len];
        }
    }
    for (int64_t j = 0; j < lx.n; ++j)
        for (int64_t i = 0; i < lx.m; ++i) {
            const int64_t r = by_rows ? i : j;
            lx.ptr[i + j * lx.ld] = lx.ptr[i + j * lx.ld] * ca[r] + P.data()[i + j * ldp] * cp[r];
        }
}

/// X := op(W) X (by_rows) or X op(W) (columns) for the depth-d butterfly W of
/// `seed`: trans applies W^T from the left / W from the right (levels d-1..0),
/// otherwise W from the left (levels 0..d-1).
template <typename T>
void apply_butterfly(Matrix<T>& X, bool by_rows, int depth, uint64_t seed, bool trans, Target target) {
    for (int t = 0; t < depth; ++t) bfly_level(X, by_rows, trans ? depth - 1 - t : t, seed, trans, target);
}

/// whole-matrix NoTrans working copy (bfly_level's requirement) when needed
template <typename T>
bool is_whole(Matrix<T> const& A) { return A.op() == Op::NoTrans && A.row0() == 0 && A.col0() == 0; }

}  // namespace

/// A := U^T A V (reference gerbt(U, A, V)); U and V from (seed, depth).
template <typename T>
void gerbt(Matrix<T>& A, int depth, uint64_t seed_u, uint64_t seed_v, Options const& opts) {
    trace::Block tb("gerbt");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    if (!is_whole(A)) {
        Matrix<T> W(A.m(), A.n(), A.mb(), A.nb(), A.grid());
        W.insertLocalTiles(target);
        slate::copy<T, T>(A, W, opts);
        gerbt(W, depth, seed_u, seed_v, opts);
        slate::copy<T, T>(W, A, opts);
        return;
    }
    apply_butterfly(A, true, depth, seed_u, true, target);
    apply_butterfly(A, false, depth, seed_v, true, target);
    internal::finish_origin(A, opts);
}

template <typename T>
int64_t gesv_rbt(Matrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts) {
    trace::Block tb("gesv_rbt");
    internal::DriverScope ds_;
    using R = real_type<T>;
    Target target = resolve_target(opts);
    const int depth = int(get_option<int64_t>(opts, Option::Depth, 2));
    const int itermax = int(get_option<int64_t>(opts, Option::MaxIterations, 10));
    const bool fallback = get_option<int64_t>(opts, Option::UseFallbackSolver, 1) != 0;
    const int64_t n = A.n();
    const uint64_t su = 0x5eed0001, sv = 0x5eed0002;
    R Anorm = norm(Norm::Inf, A, opts);
    const R cte = Anorm * std::numeric_limits<R>::epsilon() * std::sqrt(R(n));
    // A' = U^T A V on a working copy (A is kept for the residuals)
    Matrix<T> Ap(A.m(), A.n(), A.mb(), A.nb(), A.grid());
    Ap.insertLocalTiles(target);
    slate::copy<T, T>(A, Ap, opts);
    apply_butterfly(Ap, true, depth, su, true, target);
    apply_butterfly(Ap, false, depth, sv, true, target);
    int64_t info = getrf_nopiv(Ap, opts);
    iter = 0;
    auto solve = [&](Matrix<T> const& Rhs, Matrix<T>& Out) {
        // Out = V (A')^{-1} U^T Rhs
        Matrix<T> Y(Rhs.m(), Rhs.n(), Ap.mb(), Rhs.nb(), Ap.grid());
        Y.insertLocalTiles(target);
        slate::copy<T, T>(Rhs, Y, opts);
        apply_butterfly(Y, true, depth, su, true, target);
        getrs_nopiv(Ap, Y, opts);
        apply_butterfly(Y, true, depth, sv, false, target);
        slate::copy<T, T>(Y, Out, opts);
    };
    if (info == 0) {
        solve(B, X);
        Matrix<T> Rm = B.emptyLike();
        Rm.insertLocalTiles(target);
        Matrix<T> D = X.emptyLike();
        D.insertLocalTiles(target);
        const int64_t nrhs = B.n();
        std::vector<R> rnorm(nrhs), xnorm(nrhs);
        for (int it = 0; it <= itermax; ++it) {
            slate::copy<T, T>(B, Rm, opts);
            gemm(T(-1), A, X, T(1), Rm, opts);
            colNorms(Norm::Max, X, xnorm.data(), opts);
            colNorms(Norm::Max, Rm, rnorm.data(), opts);
            bool ok = true;
            for (int64_t j = 0; j < nrhs; ++j) ok = ok && rnorm[j] <= xnorm[j] * cte;
            if (ok) { iter = it; return 0; }
            if (it == itermax) break;
            solve(Rm, D);
            add(T(1), D, T(1), X, opts);
        }
        iter = -itermax - 1;
    } else {
        iter = -3;
    }
    if (!fallback) return info;
    slate::copy<T, T>(B, X, opts);
    Pivots piv;
    return gesv(A, piv, X, opts);
}

#define SLATE_RBT_INST(T)                                                                         \
    template void gerbt<T>(Matrix<T>&, int, uint64_t, uint64_t, Options const&);                 \
    template int64_t gesv_rbt<T>(Matrix<T>&, Matrix<T>&, Matrix<T>&, int&, Options const&);

SLATE_RBT_INST(float)
SLATE_RBT_INST(double)
SLATE_RBT_INST(std::complex<float>)
SLATE_RBT_INST(std::complex<double>)

}  // namespace slate
