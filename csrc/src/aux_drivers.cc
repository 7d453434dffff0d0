// Auxiliary distributed drivers: copy (with precision conversion and
// transposition), add, scale, set, gather, redistribute, norms, and the
// info reduction helpers.  Reference: src/copy.cc, add.cc, scale.cc,
// scale_row_col.cc, set.cc, set_lambdas.cc, redistribute.cc, norm.cc,
// colNorms.cc, internal_reduce_info.cc.
#include "internal.hh"
#include "spread.hh"

#include <algorithm>

#include <cstring>
#include <functional>
#include <numeric>

namespace slate {
namespace internal {

int64_t reduce_info(int64_t info, Comm& comm) {
    if (comm.size() == 1) return info;
    int64_t v = info == 0 ? INT64_MAX : info;
    v = comm.allreduce_scalar<int64_t>(v, ReduceOp::Min);
    return v == INT64_MAX ? 0 : v;
}

int64_t fetch_info(Target t, int* info) {
    if (t != Target::Devices) return info[0];
    int h = 0;
    slate_hip_call(hipMemcpy(&h, info, sizeof(int), hipMemcpyDeviceToHost));
    return h;
}

namespace {

/// true if every tile of A and B has the same size and owner
template <typename Ta, typename Tb>
bool same_layout(BaseMatrix<Ta> const& A, BaseMatrix<Tb> const& B) {
    if (A.m() != B.m() || A.n() != B.n() || A.mt() != B.mt() || A.nt() != B.nt()) return false;
    if (!A.grid()->same_processes(*B.grid())) return false;
    for (int64_t i = 0; i < A.mt(); ++i) if (A.tileMb(i) != B.tileMb(i)) return false;
    for (int64_t j = 0; j < A.nt(); ++j) if (A.tileNb(j) != B.tileNb(j)) return false;
    for (int64_t j = 0; j < A.nt(); ++j)
        for (int64_t i = 0; i < A.mt(); ++i)
            if (A.tileRank(i, j) != B.tileRank(i, j)) return false;
    return true;
}

inline bool is_trapezoid_kind(MatrixKind k) {
    return k == MatrixKind::Trapezoid || k == MatrixKind::Triangular ||
           k == MatrixKind::Symmetric || k == MatrixKind::Hermitian;
}

/// Calls fn(uplo, r, c, m, n) for the parts of an mb x nb tile whose (0, 0)
/// element is view element (ri, cj) that lie in trapezoid `u` of the view
/// (Lower keeps i >= j, Upper i <= j).  Handles views whose diagonal does not
/// run through tile corners (slices with row0 != col0): at most one General
/// strip plus one triangular sub-block per tile.
template <typename F>
void tz_tile_parts(Uplo u, int64_t ri, int64_t cj, int64_t mb, int64_t nb, F&& fn) {
    if (u == Uplo::General) { fn(Uplo::General, 0, 0, mb, nb); return; }
    const int64_t k = cj - ri;  // tile element (r, c) is on the view diagonal iff r - c == k
    if (u == Uplo::Upper) {
        if (k >= 0) {
            if (k > 0) fn(Uplo::General, 0, 0, std::min(k, mb), nb);
            if (k < mb) fn(Uplo::Upper, k, 0, mb - k, nb);
        } else if (-k < nb) {
            fn(Uplo::Upper, 0, -k, mb, nb + k);
        }
    } else {
        if (k >= 0) {
            if (k < mb) fn(Uplo::Lower, k, 0, mb - k, nb);
        } else {
            fn(Uplo::General, 0, 0, mb, std::min(-k, nb));
            if (-k < nb) fn(Uplo::Lower, 0, -k, mb, nb + k);
        }
    }
}

/// Visit the local tiles of storage-oriented view A (NoTrans) that touch its
/// trapezoid `u`, with each tile's view element origin.
template <typename T, typename F>
void for_tz_tiles(BaseMatrix<T> const& A, Uplo u, F&& fn) {
    std::vector<int64_t> r0(A.mt() + 1, 0), c0(A.nt() + 1, 0);
    for (int64_t i = 0; i < A.mt(); ++i) r0[i + 1] = r0[i] + A.tileMb(i);
    for (int64_t j = 0; j < A.nt(); ++j) c0[j + 1] = c0[j] + A.tileNb(j);
    for (int64_t j = 0; j < A.nt(); ++j)
        for (int64_t i = 0; i < A.mt(); ++i) {
            if (!A.tileIsLocal(i, j)) continue;
            // skip tiles entirely outside the trapezoid
            if (u == Uplo::Lower && r0[i + 1] - 1 < c0[j]) continue;
            if (u == Uplo::Upper && r0[i] > c0[j + 1] - 1) continue;
            fn(i, j, r0[i], c0[j]);
        }
}

/// iterate over the local tiles of a view (logical indices), giving storage pointers
template <typename T, typename F>
void for_local_tiles(BaseMatrix<T> const& A, Loc loc, F f) {
    for (int64_t j = 0; j < A.nt(); ++j)
        for (int64_t i = 0; i < A.mt(); ++i)
            if (A.tileIsLocal(i, j)) f(i, j, A.tile(i, j, loc));
}

}  // namespace

/// B = op(A) over p2p for any pair of distributions AND tilings (reference
/// redistribute.cc).  The unit of transfer is a cell of the union of both
/// tile grids: each cell lies in exactly one tile of A and one tile of B, so
/// with equal tilings cells are tiles (one message per tile).  For a
/// triangular mask the row and column breakpoints are merged so diagonal
/// cells are square blocks on the diagonal.
template <typename Ts, typename Td>
void redistribute_any(BaseMatrix<Ts> const& A, BaseMatrix<Td>& B, Target target, Uplo mask) {
    slate_error_if_msg(A.m() != B.m() || A.n() != B.n(), "redistribute: dimension mismatch");
    Comm& world = A.grid()->world();
    slate_error_if_msg(!A.grid()->same_processes(*B.grid()) && world.size() > 1,
                       "redistribute: A and B must live on the same processes");
    const int me = world.rank();
    const Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    A.storage()->get(loc, false);
    B.storage()->get(loc, true);
    // tile boundaries (logical, op applied) and their union
    auto bounds = [](int64_t nt, auto size) {
        std::vector<int64_t> v(1, 0);
        for (int64_t t = 0; t < nt; ++t) v.push_back(v.back() + size(t));
        return v;
    };
    std::vector<int64_t> ar = bounds(A.mt(), [&](int64_t t) { return A.tileMb(t); });
    std::vector<int64_t> ac = bounds(A.nt(), [&](int64_t t) { return A.tileNb(t); });
    std::vector<int64_t> br = bounds(B.mt(), [&](int64_t t) { return B.tileMb(t); });
    std::vector<int64_t> bc = bounds(B.nt(), [&](int64_t t) { return B.tileNb(t); });
    auto merge = [](std::vector<std::vector<int64_t> const*> const& lists, int64_t lim) {
        std::vector<int64_t> u;
        for (auto* l : lists) for (int64_t x : *l) if (x <= lim) u.push_back(x);
        u.push_back(lim);
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end()), u.end());
        return u;
    };
    std::vector<int64_t> ur, uc;
    if (mask == Uplo::General) { ur = merge({&ar, &br}, A.m()); uc = merge({&ac, &bc}, A.n()); }
    else { ur = merge({&ar, &br, &ac, &bc}, A.m()); uc = merge({&ar, &br, &ac, &bc}, A.n()); }
    auto tile_of = [](std::vector<int64_t> const& b, int64_t x) {
        return int64_t(std::upper_bound(b.begin(), b.end(), x) - b.begin()) - 1;
    };
    // sub-block (rows r0.., cols c0..) of an op-applied tile view
    auto sub = [](auto const& t, int64_t r, int64_t cc) {
        return t.op == Op::NoTrans ? t.data + r + cc * t.stride : t.data + cc + r * t.stride;
    };
    struct Xfer { int64_t r0, c0, mb, nb; int peer; size_t off; bool diag; };
    std::vector<Xfer> sends, recvs;
    size_t soff = 0, roff = 0;
    for (size_t jc = 0; jc + 1 < uc.size(); ++jc)
        for (size_t ic = 0; ic + 1 < ur.size(); ++ic) {
            const int64_t r0 = ur[ic], c0 = uc[jc], mb = ur[ic + 1] - r0, nb = uc[jc + 1] - c0;
            const bool diag = mask != Uplo::General && r0 == c0;
            if (mask == Uplo::Lower && r0 < c0 && !diag) continue;
            if (mask == Uplo::Upper && r0 > c0 && !diag) continue;
            const int64_t ia = tile_of(ar, r0), ja = tile_of(ac, c0), ib = tile_of(br, r0), jb = tile_of(bc, c0);
            const int src = A.tileRank(ia, ja), dst = B.tileRank(ib, jb);
            if (src == me && dst == me) {
                Tile<Ts> ta = A.tile(ia, ja, loc);
                Tile<Td> tb = B.tile(ib, jb, loc);
                lb::copy(c, diag ? mask : Uplo::General, ta.op, mb, nb, sub(ta, r0 - ar[ia], c0 - ac[ja]), ta.stride,
                         sub(tb, r0 - br[ib], c0 - bc[jb]), tb.stride);
            } else if (src == me) {
                sends.push_back({r0, c0, mb, nb, dst, soff, diag}); soff += size_t(mb) * nb;
            } else if (dst == me) {
                recvs.push_back({r0, c0, mb, nb, src, roff, diag}); roff += size_t(mb) * nb;
            }
        }
    if (world.size() == 1) {
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        return;
    }
    Work<Ts> sbuf(target, std::max<size_t>(soff, 1));
    Work<Ts> rbuf(target, std::max<size_t>(roff, 1));
    for (auto& x : sends) {
        const int64_t ia = tile_of(ar, x.r0), ja = tile_of(ac, x.c0);
        Tile<Ts> ta = A.tile(ia, ja, loc);
        // pack the op(A) cell as a dense mb x nb block
        lb::copy(c, Uplo::General, ta.op, x.mb, x.nb, sub(ta, x.r0 - ar[ia], x.c0 - ac[ja]), ta.stride,
                 sbuf.data() + x.off, x.mb);
    }
    std::vector<Comm::P2P> ops;
    for (auto& x : sends) ops.push_back({sbuf.data() + x.off, size_t(x.mb * x.nb), x.peer, true});
    for (auto& x : recvs) ops.push_back({rbuf.data() + x.off, size_t(x.mb * x.nb), x.peer, false});
    world.exchange(ops, scalar_type<Ts>(), loc, c.stream);
    for (auto& x : recvs) {
        const int64_t ib = tile_of(br, x.r0), jb = tile_of(bc, x.c0);
        Tile<Td> tb = B.tile(ib, jb, loc);
        lb::copy(c, x.diag ? mask : Uplo::General, Op::NoTrans, x.mb, x.nb, rbuf.data() + x.off, x.mb,
                 sub(tb, x.r0 - br[ib], x.c0 - bc[jb]), tb.stride);
    }
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
}

template <typename T>
void redistribute_op(BaseMatrix<T> const& A, BaseMatrix<T>& B, Target target) {
    redistribute_any<T, T>(A, B, target, Uplo::General);
}

template void redistribute_op<float>(BaseMatrix<float> const&, BaseMatrix<float>&, Target);
template void redistribute_op<double>(BaseMatrix<double> const&, BaseMatrix<double>&, Target);
template void redistribute_op<std::complex<float>>(BaseMatrix<std::complex<float>> const&, BaseMatrix<std::complex<float>>&, Target);
template void redistribute_op<std::complex<double>>(BaseMatrix<std::complex<double>> const&, BaseMatrix<std::complex<double>>&, Target);

}  // namespace internal

using namespace internal;

//------------------------------------------------------------------------------
/// same process grid, tile sizes and first-tile owner (local elements match)
template <typename Ts, typename Td>
bool co_located(BaseMatrix<Ts> const& A, BaseMatrix<Td> const& B) {
    auto &sa = *A.storage(), &sb = *B.storage();
    return A.op() == Op::NoTrans && B.op() == Op::NoTrans && A.grid().get() == B.grid().get() && sa.mb == sb.mb &&
           sa.nb == sb.nb && sa.rsrc == sb.rsrc && sa.csrc == sb.csrc && A.row0() == B.row0() &&
           A.col0() == B.col0() && A.m() == B.m() && A.n() == B.n();
}

template <typename Ts, typename Td>
void copy(BaseMatrix<Ts> const& A, BaseMatrix<Td>& B, Options const& opts) {
    if (A.is_multi_device() || B.is_multi_device()) {
        internal::copy_multi<Ts, Td>(A, B, opts);
        return;
    }
    trace::Block tb("copy");
    internal::DriverScope ds_;
    if (A.storage()->banded || B.storage()->banded) {
        // band-only storage on either side: element copy on the host between
        // co-located matrices (entries outside a source band are zero,
        // entries outside a destination band are not stored)
        slate_error_if_msg(!co_located(A, B), "copy: band-only storage needs co-located operands");
        auto& sa = *A.storage();
        auto& g = *sa.grid;
        sa.get(Loc::Host, false);
        Uplo mask = is_trapezoid_kind(B.matrix_kind()) ? B.uplo() : Uplo::General;
        for_each_stored(B, true, [&](int64_t i, int64_t j, Td& v) {
            if (mask == Uplo::Lower ? i < j : (mask == Uplo::Upper ? i > j : false)) return;
            const int64_t gr = A.row0() + i, gc = A.col0() + j;
            Ts const* e = sa.local_ptr(Loc::Host, g2l(gr, sa.mb, g.p()), g2l(gc, sa.nb, g.q()));
            v = e ? Td(*e) : Td(0);
        });
        if (resolve_target(opts) == Target::Devices) B.storage()->get(Loc::Device, false);
        internal::finish_origin(B, opts);
        return;
    }
    Target target = resolve_target(opts);
    Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    Uplo mask = Uplo::General;
    if (is_trapezoid_kind(B.matrix_kind())) mask = B.uplo();
    if (A.grid()->size() == 1 && B.grid()->size() == 1 && !A.arbitrary_layout() && !B.arbitrary_layout() &&
        (B.op() == Op::NoTrans || (A.op() == Op::NoTrans && mask == Uplo::General))) {
        // one process holds both: one (transposing) device copy of the local
        // blocks instead of the tile-by-tile redistribution
        LocalBlock<Ts> la = A.local(loc, false);
        LocalBlock<Td> lbk = B.local(loc, true);
        if (B.op() == Op::NoTrans)
            lb::copy(c, mask, A.op(), B.m(), B.n(), la.ptr, la.ld, lbk.ptr, lbk.ld);
        else   // B_storage = op_B(A) for a transposed destination view
            lb::copy(c, Uplo::General, B.op(), B.n(), B.m(), la.ptr, la.ld, lbk.ptr, lbk.ld);
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        internal::finish_origin(B, opts);
        return;
    }
    if (A.op() == Op::NoTrans && B.op() == Op::NoTrans && !A.arbitrary_layout() && !B.arbitrary_layout() && same_layout(A, B) &&
        A.aligned() && B.aligned()) {
        LocalBlock<Ts> la = A.local(loc, false);
        LocalBlock<Td> lbk = B.local(loc, true);
        if (mask == Uplo::General || A.grid()->size() == 1) {
            lb::copy(c, mask, Op::NoTrans, la.m, la.n, la.ptr, la.ld, lbk.ptr, lbk.ld);
        } else {
            // trapezoid on a distributed grid: copy tiles in the triangle
            for (int64_t j = 0; j < A.nt(); ++j)
                for (int64_t i = 0; i < A.mt(); ++i) {
                    if (!A.tileIsLocal(i, j)) continue;
                    if (mask == Uplo::Lower ? i < j : i > j) continue;
                    Tile<Ts> ta = A.tile(i, j, loc);
                    Tile<Td> tbt = B.tile(i, j, loc);
                    lb::copy(c, i == j ? mask : Uplo::General, Op::NoTrans, ta.mb, ta.nb, ta.data, ta.stride,
                             tbt.data, tbt.stride);
                }
        }
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    } else {
        redistribute_any<Ts, Td>(A, B, target, mask);
    }
    internal::finish_origin(B, opts);
}

template <typename T>
void redistribute(Matrix<T> const& A, Matrix<T>& B, Options const& opts) {
    copy<T, T>(A, B, opts);
}

template <typename T>
void add(T alpha, Matrix<T> const& A, T beta, Matrix<T>& B, Options const& opts) {
    if (internal::spread<T>(opts, {{&A, false}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int) {
            add(alpha, M[0], beta, M[1], opts);
        }, false))
        return;
    if (A.arbitrary_layout() || B.arbitrary_layout()) {
        Matrix<T> Ab = bc_operand(A, opts), Bb = block_cyclic(B, opts);
        add(alpha, Ab, beta, Bb, opts);
        slate::copy<T, T>(Bb, B, opts);
        return;
    }
    trace::Block tb("add");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    Loc loc = loc_of(target);
    slate_error_if_msg(!same_layout(A, B) || A.op() != B.op(), "add: matrices must share a layout");
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    LocalBlock<T> la = A.local(loc, false);
    LocalBlock<T> lbk = B.local(loc, true);
    lb::add(c, Uplo::General, la.m, la.n, alpha, la.ptr, la.ld, beta, lbk.ptr, lbk.ld);
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    internal::finish_origin(B, opts);
}

template <typename T>
void add(T alpha, BaseTrapezoidMatrix<T> const& A, T beta, BaseTrapezoidMatrix<T>& B, Options const& opts) {
    if (internal::spread<T>(opts, {{&A, false}, {&B, true}}, [&](std::vector<Matrix<T>>& M, int) {
            auto Ar = internal::rewrap(A, M[0]);
            auto Br = internal::rewrap(B, M[1]);
            add(alpha, Ar, beta, Br, opts);
        }, false))
        return;
    trace::Block tb("tzadd");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    Loc loc = loc_of(target);
    slate_error_if_msg(!same_layout(A, B), "add: matrices must share a layout");
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    A.storage()->get(loc, false);
    B.storage()->get(loc, true);
    // storage orientation: both views share op (same_layout)
    BaseMatrix<T> As = A.op() == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(A.op() == Op::ConjTrans);
    BaseMatrix<T> Bs = B.op() == Op::NoTrans ? BaseMatrix<T>(B) : B.transpose_view(B.op() == Op::ConjTrans);
    Uplo u = Bs.uplo();
    for_tz_tiles(Bs, u, [&](int64_t i, int64_t j, int64_t ri, int64_t cj) {
        Tile<T> ta = As.tile(i, j, loc), tbt = Bs.tile(i, j, loc);
        tz_tile_parts(u, ri, cj, ta.mb, ta.nb, [&](Uplo pu, int64_t r, int64_t cc, int64_t m, int64_t n) {
            lb::add(c, pu, m, n, alpha, ta.data + r + cc * ta.stride, ta.stride, beta,
                    tbt.data + r + cc * tbt.stride, tbt.stride);
        });
    });
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    internal::finish_origin(B, opts);
}

template <typename T>
void scale(real_type<T> numer, real_type<T> denom, BaseMatrix<T>& A, Options const& opts) {
    if (A.is_multi_device()) {
        A.storage()->group->run([&](int r, GridPtr const&) {
            BaseMatrix<T> Ar = A.on_part(r);
            scale(numer, denom, Ar, opts);
        });
        return;
    }
    if (A.arbitrary_layout()) {
        Matrix<T> B = block_cyclic(A, opts);
        BaseMatrix<T>& Bb = B;
        scale(numer, denom, Bb, opts);
        slate::copy<T, T>(B, A, opts);
        return;
    }
    trace::Block tb("scale");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    bool trap = is_trapezoid_kind(A.matrix_kind());
    A.storage()->get(loc, true);
    if (!trap || (A.grid()->size() == 1 && A.row0() == A.col0())) {
        LocalBlock<T> la = A.local_raw(loc);
        lb::scale(c, trap ? A.uplo_physical() : Uplo::General, la.m, la.n, numer, denom, la.ptr, la.ld);
    } else {
        BaseMatrix<T> As = A.op() == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(A.op() == Op::ConjTrans);
        Uplo u = As.uplo();
        for_tz_tiles(As, u, [&](int64_t i, int64_t j, int64_t ri, int64_t cj) {
            Tile<T> t = As.tile(i, j, loc);
            tz_tile_parts(u, ri, cj, t.mb, t.nb, [&](Uplo pu, int64_t r, int64_t cc, int64_t m, int64_t n) {
                lb::scale(c, pu, m, n, numer, denom, t.data + r + cc * t.stride, t.stride);
            });
        });
    }
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    internal::finish_origin(A, opts);
}

template <typename T>
void scale_row_col(Equed equed, std::vector<real_type<T>> const& R, std::vector<real_type<T>> const& C,
                   Matrix<T>& A, Options const& opts) {
    trace::Block tb("scale_row_col");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    slate_error_if_msg(A.op() != Op::NoTrans, "scale_row_col: NoTrans view required");
    LocalBlock<T> la = A.local(loc, true);
    using Rt = real_type<T>;
    // local slices of R and C
    std::vector<Rt> r(la.m), cs(la.n);
    auto& s = *A.storage();
    for (int64_t il = 0; il < la.m; ++il) {
        int64_t g = l2g(A.lrow_begin() + il, s.mb, s.rrel(), s.grid->p()) - A.row0();
        r[il] = (equed == Equed::Row || equed == Equed::Both) ? R[g] : Rt(1);
    }
    for (int64_t jl = 0; jl < la.n; ++jl) {
        int64_t g = l2g(A.lcol_begin() + jl, s.nb, s.crel(), s.grid->q()) - A.col0();
        cs[jl] = (equed == Equed::Col || equed == Equed::Both) ? C[g] : Rt(1);
    }
    if (c.dev()) {
        Work<Rt> dr(target, r.size() + 1), dc(target, cs.size() + 1);
        device::memcpy_async(dr.data(), r.data(), r.size() * sizeof(Rt), c.stream);
        device::memcpy_async(dc.data(), cs.data(), cs.size() * sizeof(Rt), c.stream);
        lb::scale_row_col(c, la.m, la.n, dr.data(), dc.data(), la.ptr, la.ld);
        slate_hip_call(hipStreamSynchronize(c.stream));
    } else {
        lb::scale_row_col(c, la.m, la.n, r.data(), cs.data(), la.ptr, la.ld);
    }
    internal::finish_origin(A, opts);
}

template <typename T>
void set(T offdiag, T diag, BaseMatrix<T>& A, Options const& opts) {
    if (A.is_multi_device()) {
        A.storage()->group->run([&](int r, GridPtr const&) {
            internal::TargetScope ts(Target::Devices);
            BaseMatrix<T> Ar = A.on_part(r);
            set(offdiag, diag, Ar, opts);
        });
        return;
    }
    if (A.arbitrary_layout()) {
        Matrix<T> B = block_cyclic(A, opts);
        B.set_uplo(A.uplo());
        BaseMatrix<T>& Bb = B;
        set(offdiag, diag, Bb, opts);
        slate::copy<T, T>(B, A, opts);
        return;
    }
    trace::Block tb("set");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    if (A.storage()->banded) {
        // band-only storage: the stored band elements (host), then the device
        slate_error_if_msg(A.op() != Op::NoTrans, "set: band-only storage needs a NoTrans view");
        for_each_stored(A, true, [&](int64_t i, int64_t j, T& v) { v = (i == j) ? diag : offdiag; });
        if (target == Target::Devices) A.storage()->get(Loc::Device, false);
        internal::finish_origin(A, opts);
        return;
    }
    Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    bool trap = is_trapezoid_kind(A.matrix_kind());
    A.storage()->get(loc, true);
    // storage orientation; a transposed view stores op(value) (set is symmetric
    // in i, j, but conj_transpose views store conjugated values)
    bool cj_ = A.op() == Op::ConjTrans;
    BaseMatrix<T> As = A.op() == Op::NoTrans ? BaseMatrix<T>(A) : A.transpose_view(cj_);
    if (cj_) { offdiag = slate::conj(offdiag); diag = slate::conj(diag); }
    Uplo u = trap ? As.uplo() : Uplo::General;
    // whole local block in ONE launch when no diagonal bookkeeping is needed
    // (a general matrix with diag == offdiag, on any grid) or the local block
    // is the whole view with its diagonal on the storage diagonal (one
    // process, row0 == col0): the tile loop below launched a kernel per tile
    // -- 16384 launches for an 8192^2 matrix in 64-wide tiles (the svd's
    // vector matrices), ~79 ms of the n = 8192 svd
    if (!A.storage()->banded && A.op() == Op::NoTrans &&
        ((u == Uplo::General && diag == offdiag) || (A.grid()->size() == 1 && A.row0() == A.col0()))) {
        LocalBlock<T> la = A.local_raw(loc);
        if (la.m > 0 && la.n > 0) lb::set(c, u, la.m, la.n, offdiag, diag, la.ptr, la.ld);
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        internal::finish_origin(A, opts);
        return;
    }
    for_tz_tiles(As, u, [&](int64_t i, int64_t j, int64_t ri, int64_t cj) {
        Tile<T> t = As.tile(i, j, loc);
        if (u == Uplo::General) {
            // whole tile, then the diagonal run r - c == cj - ri (if any) through a sub-block
            const int64_t k = cj - ri, r = std::max<int64_t>(k, 0), cc = std::max<int64_t>(-k, 0);
            const bool has_diag = r < t.mb && cc < t.nb;
            lb::set(c, Uplo::General, t.mb, t.nb, offdiag, offdiag, t.data, t.stride);
            if (has_diag && !(diag == offdiag))
                lb::set(c, Uplo::General, t.mb - r, t.nb - cc, offdiag, diag, t.data + r + cc * t.stride, t.stride);
            return;
        }
        // trapezoid: General strips hold no diagonal element; triangular parts
        // have the view diagonal as their own
        tz_tile_parts(u, ri, cj, t.mb, t.nb, [&](Uplo pu, int64_t r, int64_t cc, int64_t m, int64_t n) {
            lb::set(c, pu, m, n, offdiag, pu == Uplo::General ? offdiag : diag, t.data + r + cc * t.stride, t.stride);
        });
    });
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    internal::finish_origin(A, opts);
}

template <typename T>
void set(std::function<T(int64_t, int64_t)> const& value, BaseMatrix<T>& A, Options const&) {
    if (A.is_multi_device()) {
        A.storage()->group->run([&](int r, GridPtr const&) {
            BaseMatrix<T> Ar = A.on_part(r);
            set(value, Ar, Options{});
        });
        return;
    }
    trace::Block tb("set_lambda");
    internal::DriverScope ds_;
    // evaluated on the host instance, then marked modified
    auto& s = *A.storage();
    T* base = s.get(Loc::Host, true);
    int64_t ld = s.ld(Loc::Host);
    LocalBlock<T> la = A.local_raw(Loc::Host);
    (void)base;
    for (int64_t jl = 0; jl < la.n; ++jl) {
        int64_t gc = l2g(A.lcol_begin() + jl, s.nb, s.crel(), s.grid->q()) - A.col0();
        for (int64_t il = 0; il < la.m; ++il) {
            int64_t gr = l2g(A.lrow_begin() + il, s.mb, s.rrel(), s.grid->p()) - A.row0();
            int64_t i = A.op() == Op::NoTrans ? gr : gc, j = A.op() == Op::NoTrans ? gc : gr;
            T v = value(i, j);
            if (A.op() == Op::ConjTrans) v = slate::conj(v);
            la.ptr[il + jl * ld] = v;
        }
    }
}

template <typename T>
void gather(BaseMatrix<T> const& A, std::vector<T>& full, Options const& opts) {
    if (A.is_multi_device()) {
        A.storage()->group->run([&](int r, GridPtr const&) {
            std::vector<T> f;
            gather(A.on_part(r), f, opts);
            if (r == 0) full.swap(f);
        });
        return;
    }
    trace::Block tb("gather");
    internal::DriverScope ds_;
    (void)opts;
    int64_t m = A.m(), n = A.n();
    full.assign(size_t(m) * n, T(0));
    auto& s = *A.storage();
    if (s.banded) {
        // band-only storage: scatter the stored elements, sum over ranks
        // (every element has one owner; zeros elsewhere)
        BaseMatrix<T> As = A.op() == Op::NoTrans ? A : A.transpose_view(A.op() == Op::ConjTrans);
        const bool tr = A.op() != Op::NoTrans, cj = A.op() == Op::ConjTrans;
        for_each_stored(As, false, [&](int64_t i, int64_t j, T& v) {
            if (tr) full[j + i * m] = cj ? slate::conj(v) : v;
            else full[i + j * m] = v;
        });
        Comm& w = A.grid()->world();
        if (w.size() > 1) {
            using R = real_type<T>;
            allreduce_host<R>(w, reinterpret_cast<R*>(full.data()), full.size() * (is_complex_v<T> ? 2 : 1),
                              ReduceOp::Sum);
        }
        return;
    }
    // host instance of the local data
    T* base = s.get(Loc::Host, false);
    (void)base;
    LocalBlock<T> la = A.local_raw(Loc::Host);
    Comm& world = A.grid()->world();
    // pack my local block (storage orientation) with its global indices
    std::vector<T> mine(size_t(la.m) * la.n);
    for (int64_t j = 0; j < la.n; ++j)
        for (int64_t i = 0; i < la.m; ++i) mine[i + j * la.m] = la.ptr[i + j * la.ld];
    int size = world.size();
    std::vector<int64_t> dims(2 * size);
    int64_t md[2] = {la.m, la.n};
    world.allgather(md, dims.data(), 2, ScalarType::Int64, Loc::Host, nullptr);
    int64_t mx = 1;
    for (int r = 0; r < size; ++r) mx = std::max(mx, dims[2 * r] * dims[2 * r + 1]);
    std::vector<T> sendb(mx), recvb(size_t(mx) * size);
    std::copy(mine.begin(), mine.end(), sendb.begin());
    world.allgather(sendb.data(), recvb.data(), size_t(mx), scalar_type<T>(), Loc::Host, nullptr);
    auto& g = *s.grid;
    for (int r = 0; r < size; ++r) {
        int pr = g.row_of(r), pc = g.col_of(r);
        int rrel = (pr - s.rsrc + g.p()) % g.p(), crel = (pc - s.csrc + g.q()) % g.q();
        int64_t rb = g2l_ceil(A.row0(), s.mb, rrel, g.p()), cb = g2l_ceil(A.col0(), s.nb, crel, g.q());
        int64_t lm = dims[2 * r], ln = dims[2 * r + 1];
        T const* src = recvb.data() + size_t(mx) * r;
        for (int64_t j = 0; j < ln; ++j) {
            int64_t gc = l2g(cb + j, s.nb, crel, g.q()) - A.col0();
            for (int64_t i = 0; i < lm; ++i) {
                int64_t gr = l2g(rb + i, s.mb, rrel, g.p()) - A.row0();
                T v = src[i + j * lm];
                if (A.op() == Op::NoTrans) full[gr + gc * m] = v;
                else full[gc + gr * m] = A.op() == Op::ConjTrans ? slate::conj(v) : v;
            }
        }
    }
}

//------------------------------------------------------------------------------
// norms
namespace {

template <typename T>
struct NormParts {
    using R = real_type<T>;
    std::vector<R> colsum, rowsum;  // global-length vectors (storage orientation)
    R maxv = 0, scale = 0, sumsq = 1;
};

/// local partial norms of the view in storage orientation with mask
template <typename T>
void local_parts(BaseMatrix<T> const& A, Target target, char kind, Uplo mask, Diag diag,
                 int64_t kl, int64_t ku, NormParts<T>& P) {
    using R = real_type<T>;
    Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    auto& s = *A.storage();
    A.storage()->get(loc, false);
    int64_t M = A.srows(), N = A.scols();
    if (kind == '1') P.colsum.assign(N, 0);
    if (kind == 'I') P.rowsum.assign(M, 0);
    bool band = kl >= 0 || ku >= 0;
    const int p = s.grid->p(), q = s.grid->q();
    // On a 1 x 1 grid the local block is the view itself, so trapezoid masks
    // and unit diagonals apply to it directly (view-relative offsets 0, 0).
    const bool whole = mask == Uplo::General && diag == Diag::NonUnit;
    if (!band && (whole || (p == 1 && q == 1)) && A.aligned()) {
        // the whole local block (ScaLAPACK-layout local array) in one kernel
        // launch and one sync, instead of one of each per tile
        LocalBlock<T> la = A.local(loc, false);
        if (la.empty()) return;
        std::vector<R> out(kind == 'I' ? la.m : (kind == 'F' ? 2 * la.n : la.n));
        lb::norm_partial(c, kind, mask, diag, la.m, la.n, la.ptr, la.ld, 0, 0, out.data());
        auto gcol = [&](int64_t jl) { return l2g(A.lcol_begin() + jl, s.nb, s.crel(), q) - A.col0(); };
        auto grow = [&](int64_t il) { return l2g(A.lrow_begin() + il, s.mb, s.rrel(), p) - A.row0(); };
        if (kind == 'M') for (R v : out) P.maxv = max_nan(P.maxv, v);
        else if (kind == '1') for (int64_t jl = 0; jl < la.n; ++jl) P.colsum[gcol(jl)] += out[jl];
        else if (kind == 'I') for (int64_t il = 0; il < la.m; ++il) P.rowsum[grow(il)] += out[il];
        else for (int64_t jl = 0; jl < la.n; ++jl) combine_sumsq(P.scale, P.sumsq, out[2 * jl], out[2 * jl + 1]);
        return;
    }
    // per local tile (for trapezoid / band masks the global offsets matter)
    int64_t smt = A.op() == Op::NoTrans ? A.mt() : A.nt();
    int64_t snt = A.op() == Op::NoTrans ? A.nt() : A.mt();
    BaseMatrix<T> As = A.op() == Op::NoTrans ? A : A.transpose_view(A.op() == Op::ConjTrans);
    for (int64_t j = 0; j < snt; ++j)
        for (int64_t i = 0; i < smt; ++i) {
            if (!As.tileIsLocal(i, j)) continue;
            if (mask == Uplo::Lower && i < j) continue;
            if (mask == Uplo::Upper && i > j) continue;
            int64_t gr = grow_of(As, i), gc = gcol_of(As, j);
            Tile<T> t = As.tile(i, j, loc);
            if (band) {
                // skip tiles entirely outside the band
                if (gr - (gc + t.nb - 1) > kl) continue;
                if (gc - (gr + t.mb - 1) > ku) continue;
            }
            std::vector<R> out(kind == 'I' ? t.mb : (kind == 'F' ? 2 * t.nb : t.nb));
            if (band) {
                // host-side masked evaluation on a copy (band tiles are few)
                std::vector<T> h(size_t(t.mb) * t.nb);
                if (c.dev()) {
                    device::memcpy2d_async(h.data(), t.mb * sizeof(T), t.data, t.stride * sizeof(T), t.mb * sizeof(T), t.nb, c.stream);
                    slate_hip_call(hipStreamSynchronize(c.stream));
                } else {
                    for (int64_t jj = 0; jj < t.nb; ++jj) for (int64_t ii = 0; ii < t.mb; ++ii) h[ii + jj * t.mb] = t.data[ii + jj * t.stride];
                }
                for (int64_t jj = 0; jj < t.nb; ++jj) for (int64_t ii = 0; ii < t.mb; ++ii) {
                    int64_t gi = gr + ii, gj = gc + jj;
                    if (gi - gj > kl || gj - gi > ku) h[ii + jj * t.mb] = T(0);
                }
                lb::norm_partial(lb::Ctx::host(), kind, mask, diag, t.mb, t.nb, h.data(), t.mb, gr, gc, out.data());
            } else {
                lb::norm_partial(c, kind, mask, diag, t.mb, t.nb, t.data, t.stride, gr, gc, out.data());
            }
            if (kind == 'M') for (R v : out) P.maxv = max_nan(P.maxv, v);
            else if (kind == '1') for (int64_t jj = 0; jj < t.nb; ++jj) P.colsum[gc + jj] += out[jj];
            else if (kind == 'I') for (int64_t ii = 0; ii < t.mb; ++ii) P.rowsum[gr + ii] += out[ii];
            else for (int64_t jj = 0; jj < t.nb; ++jj) combine_sumsq(P.scale, P.sumsq, out[2 * jj], out[2 * jj + 1]);
        }
    (void)s;
}

template <typename T>
real_type<T> finish_norm(BaseMatrix<T> const& A, char kind, NormParts<T>& P) {
    using R = real_type<T>;
    Comm& w = A.grid()->world();
    if (kind == 'M') {
        R v = P.maxv;
        if (w.size() > 1) {
            // NaN-propagating max: allreduce max on values with NaN mapped to +inf marker
            R nanflag = std::isnan(v) ? R(1) : R(0);
            nanflag = w.allreduce_scalar<R>(nanflag, ReduceOp::Max);
            v = w.allreduce_scalar<R>(std::isnan(v) ? R(0) : v, ReduceOp::Max);
            if (nanflag > 0) v = std::numeric_limits<R>::quiet_NaN();
        }
        return v;
    }
    if (kind == '1' || kind == 'I') {
        auto& vec = kind == '1' ? P.colsum : P.rowsum;
        allreduce_host(w, vec.data(), vec.size(), ReduceOp::Sum);
        R v = 0;
        for (R x : vec) v = max_nan(v, x);
        return v;
    }
    // Frobenius: gather (scale, sumsq) pairs
    if (w.size() > 1) {
        std::vector<R> pairs(2 * w.size());
        R mine[2] = {P.scale, P.sumsq};
        w.allgather(mine, pairs.data(), 2, scalar_type<R>(), Loc::Host, nullptr);
        R sc = 0, sq = 1;
        for (int r = 0; r < w.size(); ++r) combine_sumsq(sc, sq, pairs[2 * r], pairs[2 * r + 1]);
        P.scale = sc; P.sumsq = sq;
    }
    return P.scale * std::sqrt(P.sumsq);
}

/// Norm of a matrix with band-only storage: host pass over the stored
/// band elements, masked to the logical band / triangle (General, Band,
/// TriangularBand, HermitianBand kinds), then one world reduction.
template <typename T>
real_type<T> norm_band_stored(Norm in_norm, BaseMatrix<T> const& A) {
    using R = real_type<T>;
    Norm nrm = in_norm;
    if (A.op() != Op::NoTrans) nrm = nrm == Norm::One ? Norm::Inf : (nrm == Norm::Inf ? Norm::One : nrm);
    BaseMatrix<T> As = A.op() == Op::NoTrans ? A : A.transpose_view(A.op() == Op::ConjTrans);
    const MatrixKind k = A.matrix_kind();
    const bool herm = (k == MatrixKind::HermitianBand);
    const bool unit = (k == MatrixKind::TriangularBand && As.diag() == Diag::Unit);
    int64_t kl = As.kl(), ku = As.ku();
    if (k == MatrixKind::General) { kl = As.m(); ku = As.n(); }
    const int64_t m = As.m(), n = As.n();
    R mx = 0, scale = 0, sumsq = 1;
    std::vector<R> colsum(nrm == Norm::One || herm ? n : 0, R(0)), rowsum(nrm == Norm::Inf || herm ? m : 0, R(0));
    bool nan = false;
    auto add = [&](int64_t i, int64_t j, R a, bool twice) {
        if (std::isnan(a)) nan = true;
        mx = std::max(mx, a);
        if (!colsum.empty()) { colsum[j] += a; if (twice) colsum[i] += a; }
        if (!rowsum.empty()) { rowsum[i] += a; if (twice) rowsum[j] += a; }
        if (nrm == Norm::Fro && a != R(0)) {
            for (int t = 0; t < (twice ? 2 : 1); ++t) {
                if (scale < a) { sumsq = 1 + sumsq * (scale / a) * (scale / a); scale = a; }
                else sumsq += (a / scale) * (a / scale);
            }
        }
    };
    for_each_stored(As, false, [&](int64_t i, int64_t j, T& v) {
        if (i - j > kl || j - i > ku) return;
        if (i == j && unit) { add(i, j, R(1), false); return; }
        R a = (herm && i == j) ? std::abs(std::real(v)) : std::abs(v);
        add(i, j, a, herm && i != j);
    });
    Comm& w = As.grid()->world();
    if (w.size() > 1) {
        nan = w.allreduce_scalar<R>(nan ? R(1) : R(0), ReduceOp::Max) > 0;
        mx = w.allreduce_scalar<R>(mx, ReduceOp::Max);
        if (!colsum.empty()) allreduce_host(w, colsum.data(), colsum.size(), ReduceOp::Sum);
        if (!rowsum.empty()) allreduce_host(w, rowsum.data(), rowsum.size(), ReduceOp::Sum);
        if (nrm == Norm::Fro) {
            // combine (scale, sumsq) pairs through the world max scale
            R smax = w.allreduce_scalar<R>(scale, ReduceOp::Max);
            R part = smax > 0 ? sumsq * (scale / smax) * (scale / smax) : R(0);
            part = w.allreduce_scalar<R>(part, ReduceOp::Sum);
            scale = smax; sumsq = part;
        }
    }
    if (nan) return std::numeric_limits<R>::quiet_NaN();
    switch (nrm) {
        case Norm::Max: return mx;
        case Norm::One: return colsum.empty() ? R(0) : *std::max_element(colsum.begin(), colsum.end());
        case Norm::Inf: return rowsum.empty() ? R(0) : *std::max_element(rowsum.begin(), rowsum.end());
        case Norm::Fro: return scale * std::sqrt(sumsq);
        default: slate_not_implemented("two-norm of a band matrix");
    }
    return 0;
}

}  // namespace

template <typename T>
real_type<T> norm(Norm in_norm, BaseMatrix<T> const& A, Options const& opts) {
    if (A.is_multi_device()) {
        real_type<T> v = 0;
        A.storage()->group->run([&](int r, GridPtr const&) {
            internal::TargetScope ts(Target::Devices);
            const real_type<T> x = norm(in_norm, A.on_part(r), opts);
            if (r == 0) v = x;
        });
        return v;
    }
    if (A.arbitrary_layout()) {
        Matrix<T> B = block_cyclic(A, opts);
        B.set_kind(A.matrix_kind());
        B.set_uplo(A.uplo());
        B.set_diag(A.diag());
        B.set_band(A.kl(), A.ku());
        return norm(in_norm, BaseMatrix<T>(B), opts);
    }
    trace::Block tb("norm");
    internal::DriverScope ds_;
    using R = real_type<T>;
    Target target = resolve_target(opts);
    if (A.storage()->banded) return norm_band_stored(in_norm, A);
    // normalize: work in storage orientation; One<->Inf swap for transposed views
    Norm nrm = in_norm;
    if (A.op() != Op::NoTrans) {
        if (nrm == Norm::One) nrm = Norm::Inf;
        else if (nrm == Norm::Inf) nrm = Norm::One;
    }
    BaseMatrix<T> As = A.op() == Op::NoTrans ? A : A.transpose_view(A.op() == Op::ConjTrans);
    MatrixKind k = A.matrix_kind();
    char kind = nrm == Norm::Max ? 'M' : nrm == Norm::One ? '1' : nrm == Norm::Inf ? 'I' : 'F';
    if (nrm == Norm::Two) slate_not_implemented("two-norm of a matrix");
    int64_t kl = -1, ku = -1;
    if (k == MatrixKind::Band || k == MatrixKind::TriangularBand || k == MatrixKind::HermitianBand) {
        kl = As.kl(); ku = As.ku();
    }
    bool sym = (k == MatrixKind::Symmetric || k == MatrixKind::Hermitian || k == MatrixKind::HermitianBand);
    Uplo mask = (k == MatrixKind::General || k == MatrixKind::Band) ? Uplo::General : As.uplo_physical();
    Diag diag = (k == MatrixKind::Triangular || k == MatrixKind::Trapezoid || k == MatrixKind::TriangularBand)
              ? As.diag() : Diag::NonUnit;
    if (k == MatrixKind::HermitianBand) { kl = ku = std::max(As.kl(), As.ku()); }
    if (!sym) {
        NormParts<T> P;
        local_parts(As, target, kind, mask, diag, kl, ku, P);
        return finish_norm(As, kind, P);
    }
    // symmetric/Hermitian from one triangle
    if (kind == 'M') {
        const int64_t n = std::min(As.srows(), As.scols());
        if (is_complex_v<T> && k == MatrixKind::Hermitian && kl < 0 && n >= 1) {
            // Hermitian: the diagonal counts with its real part only (LAPACK
            // lanhe): max over the strict triangle (a shifted slice of the
            // stored one) and the |Re| of the diagonal
            // (n == 1: the strict triangle is empty)
            R v = 0;
            if (n > 1) {
                BaseMatrix<T> St = mask == Uplo::Lower ? As.slice(1, n - 1, 0, n - 2) : As.slice(0, n - 2, 1, n - 1);
                NormParts<T> P;
                local_parts(St, target, 'M', mask, diag, kl, ku, P);
                v = finish_norm(St, 'M', P);
            }
            Loc loc = loc_of(target);
            lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
            R dmax = 0;
            for (int64_t i = 0; i < std::min(As.mt(), As.nt()); ++i) {
                if (!As.tileIsLocal(i, i)) continue;
                Tile<T> t = As.tile(i, i, loc);
                int64_t nd = std::min(t.mb, t.nb);
                std::vector<T> h(nd);
                if (c.dev()) {
                    device::memcpy2d_async(h.data(), sizeof(T), t.data, (t.stride + 1) * sizeof(T), sizeof(T), nd, c.stream);
                    slate_hip_call(hipStreamSynchronize(c.stream));
                } else for (int64_t ii = 0; ii < nd; ++ii) h[ii] = t.data[ii * (t.stride + 1)];
                for (int64_t ii = 0; ii < nd; ++ii) dmax = max_nan(dmax, R(std::abs(std::real(h[ii]))));
            }
            Comm& w = As.grid()->world();
            if (w.size() > 1) {
                R nanflag = std::isnan(dmax) ? R(1) : R(0);
                nanflag = w.allreduce_scalar<R>(nanflag, ReduceOp::Max);
                dmax = w.allreduce_scalar<R>(std::isnan(dmax) ? R(0) : dmax, ReduceOp::Max);
                if (nanflag > 0) dmax = std::numeric_limits<R>::quiet_NaN();
            }
            return max_nan(v, dmax);
        }
        NormParts<T> P;
        local_parts(As, target, 'M', mask, diag, kl, ku, P);
        return finish_norm(As, 'M', P);
    }
    if (kind == '1' || kind == 'I') {
        NormParts<T> Pc, Pr, Pd;
        local_parts(As, target, '1', mask, diag, kl, ku, Pc);
        local_parts(As, target, 'I', mask, diag, kl, ku, Pr);
        Comm& w = As.grid()->world();
        allreduce_host(w, Pc.colsum.data(), Pc.colsum.size(), ReduceOp::Sum);
        allreduce_host(w, Pr.rowsum.data(), Pr.rowsum.size(), ReduceOp::Sum);
        // diagonal magnitudes (counted in both); a Hermitian diagonal counts
        // with its real part only, as LAPACK lanhe does
        const bool herm = is_complex_v<T> && k != MatrixKind::Symmetric;
        std::vector<R> d(As.srows(), 0), dre(As.srows(), 0);
        {
            // diagonal: gather via per-tile host reads
            Loc loc = loc_of(target);
            lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
            for (int64_t i = 0; i < std::min(As.mt(), As.nt()); ++i) {
                if (!As.tileIsLocal(i, i)) continue;
                Tile<T> t = As.tile(i, i, loc);
                int64_t nd = std::min(t.mb, t.nb);
                std::vector<T> h(nd);
                if (c.dev()) {
                    device::memcpy2d_async(h.data(), sizeof(T), t.data, (t.stride + 1) * sizeof(T), sizeof(T), nd, c.stream);
                    slate_hip_call(hipStreamSynchronize(c.stream));
                } else for (int64_t ii = 0; ii < nd; ++ii) h[ii] = t.data[ii * (t.stride + 1)];
                for (int64_t ii = 0; ii < nd; ++ii) {
                    d[grow_of(As, i) + ii] = std::abs(h[ii]);
                    dre[grow_of(As, i) + ii] = std::abs(std::real(h[ii]));
                }
            }
            allreduce_host(w, d.data(), d.size(), ReduceOp::Sum);
            allreduce_host(w, dre.data(), dre.size(), ReduceOp::Sum);
        }
        R v = 0;
        for (size_t j = 0; j < d.size(); ++j)
            v = max_nan(v, herm ? Pc.colsum[j] + Pr.rowsum[j] - 2 * d[j] + dre[j] : Pc.colsum[j] + Pr.rowsum[j] - d[j]);
        return v;
    }
    // Frobenius: 2 * |triangle|^2 - |diag|^2
    NormParts<T> Pt;
    local_parts(As, target, 'F', mask, diag, kl, ku, Pt);
    R tri = finish_norm(As, 'F', Pt);
    // diagonal Frobenius
    NormParts<T> Pd, Pdr;
    const bool herm_f = is_complex_v<T> && k != MatrixKind::Symmetric;
    {
        Loc loc = loc_of(target);
        lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
        for (int64_t i = 0; i < std::min(As.mt(), As.nt()); ++i) {
            if (!As.tileIsLocal(i, i)) continue;
            Tile<T> t = As.tile(i, i, loc);
            int64_t nd = std::min(t.mb, t.nb);
            std::vector<T> h(nd);
            if (c.dev()) {
                device::memcpy2d_async(h.data(), sizeof(T), t.data, (t.stride + 1) * sizeof(T), sizeof(T), nd, c.stream);
                slate_hip_call(hipStreamSynchronize(c.stream));
            } else for (int64_t ii = 0; ii < nd; ++ii) h[ii] = t.data[ii * (t.stride + 1)];
            for (int64_t ii = 0; ii < nd; ++ii) {
                add_sumsq(Pd.scale, Pd.sumsq, R(std::abs(h[ii])));
                add_sumsq(Pdr.scale, Pdr.sumsq, R(std::abs(std::real(h[ii]))));
            }
        }
    }
    R dg = finish_norm(As, 'F', Pd);
    // Hermitian: the diagonal counts with its real part only (LAPACK lanhe)
    R dr = herm_f ? finish_norm(As, 'F', Pdr) : R(0);
    R v2 = herm_f ? 2 * tri * tri - 2 * dg * dg + dr * dr : 2 * tri * tri - dg * dg;
    return std::sqrt(std::max<R>(v2, 0));
}

template <typename T>
void colNorms(Norm in_norm, Matrix<T> const& A, real_type<T>* values, Options const& opts) {
    if (A.is_multi_device()) {
        A.storage()->group->run([&](int r, GridPtr const&) {
            internal::TargetScope ts(Target::Devices);
            std::vector<real_type<T>> v(size_t(A.n()));
            colNorms(in_norm, Matrix<T>(A.on_part(r)), v.data(), opts);
            if (r == 0) std::copy(v.begin(), v.end(), values);
        });
        return;
    }
    trace::Block tb("colNorms");
    internal::DriverScope ds_;
    using R = real_type<T>;
    Target target = resolve_target(opts);
    slate_error_if_msg(in_norm != Norm::Max, "colNorms: only Norm::Max is supported (as the reference)");
    slate_error_if_msg(A.op() != Op::NoTrans, "colNorms: NoTrans view required");
    Loc loc = loc_of(target);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    int64_t n = A.n();
    std::vector<R> v(n, 0);
    LocalBlock<T> la = A.local(loc, false);
    auto& s = *A.storage();
    if (!la.empty()) {
        std::vector<R> out(la.n);
        lb::norm_partial(c, 'M', Uplo::General, Diag::NonUnit, la.m, la.n, la.ptr, la.ld, 0, 0, out.data());
        for (int64_t jl = 0; jl < la.n; ++jl)
            v[l2g(A.lcol_begin() + jl, s.nb, s.crel(), s.grid->q()) - A.col0()] = out[jl];
    }
    allreduce_host(A.grid()->world(), v.data(), v.size(), ReduceOp::Max);
    std::copy(v.begin(), v.end(), values);
}

void sync() { if (device::available()) device::sync_all(); }

//------------------------------------------------------------------------------
#define SLATE_AUX_INST(T)                                                                               \
    template void redistribute<T>(Matrix<T> const&, Matrix<T>&, Options const&);                       \
    template void add<T>(T, Matrix<T> const&, T, Matrix<T>&, Options const&);                          \
    template void add<T>(T, BaseTrapezoidMatrix<T> const&, T, BaseTrapezoidMatrix<T>&, Options const&); \
    template void scale<T>(real_type<T>, real_type<T>, BaseMatrix<T>&, Options const&);                 \
    template void scale_row_col<T>(Equed, std::vector<real_type<T>> const&, std::vector<real_type<T>> const&, Matrix<T>&, Options const&); \
    template void set<T>(T, T, BaseMatrix<T>&, Options const&);                                          \
    template void set<T>(std::function<T(int64_t, int64_t)> const&, BaseMatrix<T>&, Options const&);     \
    template void gather<T>(BaseMatrix<T> const&, std::vector<T>&, Options const&);                     \
    template real_type<T> norm<T>(Norm, BaseMatrix<T> const&, Options const&);                           \
    template void colNorms<T>(Norm, Matrix<T> const&, real_type<T>*, Options const&);

SLATE_AUX_INST(float)
SLATE_AUX_INST(double)
SLATE_AUX_INST(std::complex<float>)
SLATE_AUX_INST(std::complex<double>)

#define SLATE_COPY_INST(Ts, Td) template void copy<Ts, Td>(BaseMatrix<Ts> const&, BaseMatrix<Td>&, Options const&);
SLATE_COPY_INST(float, float)
SLATE_COPY_INST(double, double)
SLATE_COPY_INST(float, double)
SLATE_COPY_INST(double, float)
SLATE_COPY_INST(std::complex<float>, std::complex<float>)
SLATE_COPY_INST(std::complex<double>, std::complex<double>)
SLATE_COPY_INST(std::complex<float>, std::complex<double>)
SLATE_COPY_INST(std::complex<double>, std::complex<float>)

}  // namespace slate
