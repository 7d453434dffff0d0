// Band drivers (reference src/gbtrf.cc, gbtrs.cc, gbsv.cc, pbtrf.cc, pbtrs.cc,
// pbsv.cc, gbmm.cc, hbmm.cc, tbsm.cc, internal_gbnorm.cc / hbnorm.cc).
//
// gbtrf / pbtrf are blocked and distributed: the band (O(n * bandwidth)
// entries, never O(n^2)) is laid out as dense block-column slabs, block
// column J on world rank J % P, each slab holding only the rows of that block
// column that the band (plus LU fill) can reach.  Step J: the owner factors
// its (nb + kl) x nb panel (device LU panel kernel / potrf + trsm), one world
// broadcast ships the panel (and pivots) to the owners of the few block
// columns it reaches, which apply the swaps, the triangular solve and the
// GEMM update to their slabs -- the reference's tile-band algorithm with
// whole-panel collectives instead of per-tile messages.  gbmm / hbmm / tbsm,
// pbtrs and gbtrs work chunk by chunk on the band's sub-views with the
// distributed GEMM / TRSM (no dense operand, no replicated right-hand side).
#include "internal.hh"
#include "../kernels/kernels.hh"

#include <cmath>

namespace slate {

using namespace internal;

namespace {

/// Visit every local element of A (NoTrans view) with its global (i, j)
/// relative to the view; f(i, j, T& value).  Host instance, optionally for write.
template <typename T, typename F>
void for_each_local(BaseMatrix<T> const& A, bool write, F&& f) {
    for_each_stored(A, write, std::forward<F>(f));
}

//------------------------------------------------------------------------------
// host band kernels (LAPACK gbtf2 / gbtrs / pbtf2 / pbtrs semantics)
template <typename T>
int64_t gbtf2(int64_t n, int64_t kl, int64_t ku, T* ab, int64_t ldab, int64_t* ipiv) {
    const int64_t kv = ku + kl;
    auto A = [&](int64_t i, int64_t j) -> T& { return ab[(kv + i - j) + j * ldab]; };
    int64_t info = 0, ju = 0;
    for (int64_t j = 0; j < n; ++j) {
        const int64_t km = std::min(kl, n - 1 - j);
        int64_t jp = 0;
        real_type<T> mx = -1;
        for (int64_t i = 0; i <= km; ++i) {
            real_type<T> a = std::abs(std::real(A(j + i, j))) + std::abs(std::imag(A(j + i, j)));
            if (a > mx) { mx = a; jp = i; }
        }
        ipiv[j] = j + jp;
        if (A(j + jp, j) != T(0)) {
            ju = std::max(ju, std::min(j + ku + jp, n - 1));
            if (jp != 0)
                for (int64_t c = j; c <= ju; ++c) std::swap(A(j + jp, c), A(j, c));
            if (km > 0) {
                T r = T(1) / A(j, j);
                for (int64_t i = 1; i <= km; ++i) A(j + i, j) *= r;
                for (int64_t c = j + 1; c <= ju; ++c) {
                    T t = A(j, c);
                    if (t == T(0)) continue;
                    for (int64_t i = 1; i <= km; ++i) A(j + i, c) -= A(j + i, j) * t;
                }
            }
        } else if (info == 0) {
            info = j + 1;
        }
    }
    return info;
}

/// Lower band Cholesky: ab(i - j, j) = A(i, j), ldab >= kd + 1.
template <typename T>
int64_t pbtf2(int64_t n, int64_t kd, T* ab, int64_t ldab) {
    auto L = [&](int64_t i, int64_t j) -> T& { return ab[(i - j) + j * ldab]; };
    for (int64_t j = 0; j < n; ++j) {
        real_type<T> ajj = std::real(L(j, j));
        if (!(ajj > 0)) return j + 1;
        ajj = std::sqrt(ajj);
        L(j, j) = T(ajj);
        int64_t kn = std::min(kd, n - 1 - j);
        for (int64_t i = 1; i <= kn; ++i) L(j + i, j) /= T(ajj);
        for (int64_t c = 1; c <= kn; ++c) {
            T lc = slate::conj(L(j + c, j));
            for (int64_t r = c; r <= kn; ++r) L(j + r, j + c) -= L(j + r, j) * lc;
        }
    }
    return 0;
}

/// Dense block-column slabs of a band matrix distributed 1-D over the world
/// (block column J on rank J % P): rows [J nb - top, J nb + nb + bot) of the
/// block column, H = top + nb + bot rows, zero outside the band.
template <typename T>
struct BandSlabs {
    int64_t n = 0, nb = 0, top = 0, bot = 0, H = 0, nblk = 0;
    int P = 1, me = 0;
    Target target = Target::HostTask;
    std::vector<int64_t> lidx;     // block column -> my slab index, -1 if not mine
    Work<T> buf;

    BandSlabs(int64_t n_, int64_t nb_, int64_t top_, int64_t bot_, Comm& w, Target t)
        : n(n_), nb(nb_), top(top_), bot(bot_), H(top_ + nb_ + bot_), P(w.size()), me(w.rank()), target(t) {
        nblk = ceildiv(n, nb);
        lidx.assign(nblk, -1);
        int64_t cnt = 0;
        for (int64_t J = 0; J < nblk; ++J) if (J % P == me) lidx[J] = cnt++;
        buf.resize(target, size_t(std::max<int64_t>(cnt, 1)) * H * nb);
    }
    int owner(int64_t J) const { return int(J % P); }
    bool mine(int64_t J) const { return lidx[J] >= 0; }
    T* slab(int64_t J) const { return buf.data() + size_t(lidx[J]) * H * nb; }
    int64_t width(int64_t J) const { return std::min(nb, n - J * nb); }
    int64_t row0(int64_t J) const { return J * nb - top; }
    /// fill my slabs from replicated band storage: A(i, j) = ab[(r0 + i - j) + j ldab] for -up <= i - j <= lo
    void load(std::vector<T> const& ab, int64_t r0, int64_t ldab, int64_t lo, int64_t up) {
        std::vector<T> h(size_t(H) * nb);
        for (int64_t J = 0; J < nblk; ++J) {
            if (!mine(J)) continue;
            std::fill(h.begin(), h.end(), T(0));
            for (int64_t jj = 0; jj < width(J); ++jj) {
                const int64_t j = J * nb + jj;
                for (int64_t i = std::max<int64_t>(0, j - up); i <= std::min(n - 1, j + lo); ++i) {
                    const int64_t r = i - row0(J);
                    if (r >= 0 && r < H) h[r + jj * H] = ab[(r0 + i - j) + j * ldab];
                }
            }
            if (target == Target::Devices)
                device::memcpy_async(slab(J), h.data(), h.size() * sizeof(T), device::queue(0));
            else
                std::copy(h.begin(), h.end(), slab(J));
        }
        if (target == Target::Devices) slate_hip_call(hipStreamSynchronize(device::queue(0)));
    }
    /// my slabs' band entries into (zeroed) replicated band storage, then summed over the world
    void store(std::vector<T>& ab, int64_t r0, int64_t ldab, int64_t lo, int64_t up, Comm& w) {
        std::fill(ab.begin(), ab.end(), T(0));
        std::vector<T> h(size_t(H) * nb);
        for (int64_t J = 0; J < nblk; ++J) {
            if (!mine(J)) continue;
            if (target == Target::Devices) {
                device::memcpy_async(h.data(), slab(J), h.size() * sizeof(T), device::queue(0));
                slate_hip_call(hipStreamSynchronize(device::queue(0)));
            } else {
                std::copy(slab(J), slab(J) + h.size(), h.begin());
            }
            for (int64_t jj = 0; jj < width(J); ++jj) {
                const int64_t j = J * nb + jj;
                for (int64_t i = std::max<int64_t>(0, j - up); i <= std::min(n - 1, j + lo); ++i) {
                    const int64_t r = i - row0(J);
                    if (r >= 0 && r < H) ab[(r0 + i - j) + j * ldab] = h[r + jj * H];
                }
            }
        }
        if (w.size() > 1) {
            using R = real_type<T>;
            allreduce_host<R>(w, reinterpret_cast<R*>(ab.data()), ab.size() * (is_complex_v<T> ? 2 : 1), ReduceOp::Sum);
        }
    }
};

/// Distributed blocked band LU with partial pivoting on the slabs (top = nb *
/// ceil((kl + ku + nb - 1) / nb) rows for the U fill, bot = kl); ipiv absolute.
template <typename T>
int64_t gbtrf_slabs(BandSlabs<T>& S_, int64_t kl, int64_t ku, Comm& w, std::vector<int64_t>& ipiv) {
    const int64_t n = S_.n, nb = S_.nb, H = S_.H, top = S_.top;
    const Target target = S_.target;
    Sched S(target);
    const int R = 3;
    std::vector<Work<T>> PB(R);
    std::vector<Work<int64_t>> PI(R);
    for (int r = 0; r < R; ++r) {
        PB[r].resize(target, size_t(nb + kl) * nb);
        PI[r].resize(target, size_t(nb + nb + kl));      // [ipiv nb | perm nb + kl]
    }
    Work<int64_t> ipiv_all(target, size_t(std::max<int64_t>(n, 1)));
    Work<int> dinfo(target, 1);
    {
        lb::Ctx c0 = S.ctx(1);
        if (c0.dev()) device::memset_async(dinfo.data(), 0, sizeof(int), c0.stream);
        else dinfo.data()[0] = 0;
    }
    for (int64_t J = 0; J < S_.nblk; ++J) {
        const int64_t wJ = S_.width(J), jj0 = J * nb;
        const int64_t mrows = std::min(wJ + kl, n - jj0);
        const int slot = int(J % R);
        T* Pb = PB[slot].data();
        int64_t* Pi = PI[slot].data();
        const int64_t tP = Sched::bcast(slot);
        if (S_.mine(J)) {
            T* pan = S_.slab(J) + top;                 // rows [jj0, jj0 + mrows)
            S.task(1, {Sched::col(J)}, {Sched::col(J), tP}, [&, pan, mrows, wJ, jj0, Pb, Pi](lb::Ctx const& c) {
                trace::Block t2("gbtrf_panel");
                lb::getrf_panel(c, mrows, wJ, pan, H, Pi, Pi + nb, dinfo.data(), jj0, true, false);
                lb::copy2d(c, mrows, wJ, pan, H, Pb, mrows);
                // the broadcast copy keeps the getrf convention for the updates;
                // the stored factor gets gbtrs's (no later swaps on earlier columns)
                if (c.dev()) {
                    slate_amd::dev::undo_left_swaps(wJ, slate_amd::dev::dptr(pan), H, Pi, c.stream);
                } else {
                    for (int64_t col = 0; col < wJ; ++col)
                        for (int64_t jj = wJ - 1; jj > col; --jj)
                            if (Pi[jj] != jj) std::swap(pan[jj + col * H], pan[Pi[jj] + col * H]);
                }
            });
        }
        S.task(device::kCommQueue, {}, {tP}, [&, J, mrows, wJ, jj0, Pb, Pi](lb::Ctx const& c) {
            trace::Block t2("gbtrf_bcast");
            if (w.size() > 1) {
                w.bcast(Pb, size_t(mrows * wJ), S_.owner(J), c.loc(), c.stream);
                w.bcast(Pi, size_t(nb + mrows), S_.owner(J), c.loc(), c.stream);
            }
            lb::copy2d(c, std::min(wJ, mrows), int64_t(1), Pi, nb, ipiv_all.data() + jj0, nb);
        });
        // block columns the panel reaches (U fill: kl + ku past the diagonal)
        const int64_t Jlast = std::min(S_.nblk - 1, (jj0 + wJ - 1 + kl + ku) / nb);
        for (int64_t J2 = J + 1; J2 <= Jlast; ++J2) {
            if (!S_.mine(J2)) continue;
            const int64_t w2 = S_.width(J2);
            T* blk = S_.slab(J2) + (jj0 - S_.row0(J2));    // rows [jj0, jj0 + mrows) of block column J2
            const int q = (J2 == J + 1) ? int(device::kLookaheadQueue) : int(device::kTrailQueue);
            S.task(q, {tP}, {Sched::col(J2)}, [&, blk, mrows, wJ, w2, Pb, Pi](lb::Ctx const& c) {
                trace::Block t2("gbtrf_update");
                lb::apply_perm(c, std::min(wJ, mrows), Pi + nb, Pi, w2, blk, H);
                lb::trsm(c, Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, wJ, w2, T(1), Pb, mrows, blk, H);
                if (mrows > wJ)
                    lb::gemm(c, Op::NoTrans, Op::NoTrans, mrows - wJ, w2, wJ, T(-1), Pb + wJ, mrows, blk, H, T(1),
                             blk + wJ, H);
            });
        }
    }
    S.wait_all();
    ipiv.assign(n, 0);
    if (target == Target::Devices) {
        device::memcpy_async(ipiv.data(), ipiv_all.data(), n * sizeof(int64_t), device::queue(0));
        slate_hip_call(hipStreamSynchronize(device::queue(0)));
    } else {
        std::copy(ipiv_all.data(), ipiv_all.data() + n, ipiv.begin());
    }
    for (int64_t J = 0; J < S_.nblk; ++J)
        for (int64_t t = 0; t < S_.width(J) && J * nb + t < n; ++t) ipiv[J * nb + t] += J * nb;
    int64_t info = fetch_info(target, dinfo.data());
    return reduce_info(info, w);
}

/// Distributed blocked band Cholesky (lower, bandwidth kd) on the slabs (top = 0, bot = kd).
template <typename T>
int64_t pbtrf_slabs(BandSlabs<T>& S_, int64_t kd, Comm& w) {
    const int64_t n = S_.n, nb = S_.nb, H = S_.H;
    const Target target = S_.target;
    Sched S(target);
    const int R = 3;
    std::vector<Work<T>> PB(R);
    for (int r = 0; r < R; ++r) PB[r].resize(target, size_t(nb + kd) * nb);
    Work<int> dinfo(target, 1);
    {
        lb::Ctx c0 = S.ctx(1);
        if (c0.dev()) device::memset_async(dinfo.data(), 0, sizeof(int), c0.stream);
        else dinfo.data()[0] = 0;
    }
    for (int64_t J = 0; J < S_.nblk; ++J) {
        const int64_t wJ = S_.width(J), jj0 = J * nb;
        const int64_t mrows = std::min(wJ + kd, n - jj0);
        const int slot = int(J % R);
        T* Pb = PB[slot].data();
        const int64_t tP = Sched::bcast(slot);
        if (S_.mine(J)) {
            T* pan = S_.slab(J);
            S.task(1, {Sched::col(J)}, {Sched::col(J), tP}, [&, pan, mrows, wJ, jj0, Pb](lb::Ctx const& c) {
                trace::Block t2("pbtrf_panel");
                lb::potrf(c, Uplo::Lower, wJ, pan, H, dinfo.data(), jj0);
                if (mrows > wJ)
                    lb::trsm(c, Side::Right, Uplo::Lower, Op::ConjTrans, Diag::NonUnit, mrows - wJ, wJ, T(1), pan, H,
                             pan + wJ, H);
                lb::copy2d(c, mrows, wJ, pan, H, Pb, mrows);
            });
        }
        S.task(device::kCommQueue, {}, {tP}, [&, J, mrows, wJ, Pb](lb::Ctx const& c) {
            trace::Block t2("pbtrf_bcast");
            if (w.size() > 1) w.bcast(Pb, size_t(mrows * wJ), S_.owner(J), c.loc(), c.stream);
        });
        const int64_t Jlast = std::min(S_.nblk - 1, (jj0 + mrows - 1) / nb);
        for (int64_t J2 = J + 1; J2 <= Jlast; ++J2) {
            if (!S_.mine(J2)) continue;
            const int64_t w2 = S_.width(J2), ra = J2 * nb - jj0;    // panel row of J2's first column
            const int64_t nr = mrows - ra;                           // rows [J2 nb, jj0 + mrows) of block column J2
            const int64_t wc = std::min(w2, nr);                     // J2 columns the panel reaches
            T* blk = S_.slab(J2);
            const int q = (J2 == J + 1) ? int(device::kLookaheadQueue) : int(device::kTrailQueue);
            S.task(q, {tP}, {Sched::col(J2)}, [&, blk, mrows, wJ, ra, nr, wc, Pb](lb::Ctx const& c) {
                trace::Block t2("pbtrf_update");
                // lower part of A(J2 rows.., J2 cols) -= L(rows, J) L(cols, J)^H
                lb::gemm_tri(c, Uplo::Lower, Op::NoTrans, Op::ConjTrans, wc, wJ, T(-1), Pb + ra, mrows, Pb + ra,
                             mrows, T(1), blk, H);
                if (nr > wc)
                    lb::gemm(c, Op::NoTrans, Op::ConjTrans, nr - wc, wc, wJ, T(-1), Pb + ra + wc, mrows, Pb + ra,
                             mrows, T(1), blk + wc, H);
            });
        }
    }
    S.wait_all();
    int64_t info = fetch_info(target, dinfo.data());
    return reduce_info(info, w);
}

/// Pivots (reference layout: per tile column, (tile offset from k, row offset))
template <typename T>
void pivots_from_ipiv(BaseMatrix<T> const& A, std::vector<int64_t> const& ipiv, Pivots& pivots) {
    const int64_t kt = std::min(A.mt(), A.nt());
    pivots.assign(kt, {});
    for (int64_t k = 0; k < kt; ++k) {
        int64_t kk = grow_of(A, k), kd = std::min(A.tileNb(k), int64_t(ipiv.size()) - kk);
        for (int64_t t = 0; t < kd; ++t) {
            int64_t r = ipiv[kk + t];
            int64_t ti = 0;
            while (ti + k + 1 < A.mt() && grow_of(A, k + ti + 1) <= r) ++ti;
            pivots[k].push_back(Pivot(ti, r - grow_of(A, k + ti)));
        }
    }
}

template <typename T>
std::vector<int64_t> ipiv_from_pivots(BaseMatrix<T> const& A, Pivots const& pivots) {
    std::vector<int64_t> ipiv;
    for (int64_t k = 0; k < int64_t(pivots.size()); ++k)
        for (auto const& p : pivots[k]) ipiv.push_back(grow_of(A, k + p.tileIndex()) + p.elementOffset());
    return ipiv;
}

}  // namespace

//------------------------------------------------------------------------------
// Band BLAS (reference src/gbmm.cc, hbmm.cc, tbsm.cc, work on the tiles inside
// the band only).  Here the band is walked in chunks of block columns: each
// chunk's band part -- at most (chunk + bandwidth) x chunk elements, entries
// outside the band zeroed -- is copied out of the storage and applied with one
// distributed GEMM / TRSM on the sub-views of B and C it touches.  Flops are
// O(n * bandwidth * nrhs) and the temporaries O(nb * bandwidth) per chunk, not
// the dense product's O(n^2 * nrhs) / O(n^2).
namespace {

template <typename T>
int64_t row_off(BaseMatrix<T> const& A, int64_t i) {
    int64_t o = 0;
    for (int64_t t = 0; t < i; ++t) o += A.tileMb(t);
    return o;
}

template <typename T>
int64_t col_off(BaseMatrix<T> const& A, int64_t j) {
    int64_t o = 0;
    for (int64_t t = 0; t < j; ++t) o += A.tileNb(t);
    return o;
}

/// logical tile row holding element row r (0 <= r < m)
template <typename T>
int64_t tile_row_of(BaseMatrix<T> const& A, int64_t r) {
    int64_t o = 0;
    for (int64_t t = 0; t < A.mt(); ++t) {
        o += A.tileMb(t);
        if (r < o) return t;
    }
    return A.mt() - 1;
}

template <typename T>
int64_t tile_col_of(BaseMatrix<T> const& A, int64_t c) {
    int64_t o = 0;
    for (int64_t t = 0; t < A.nt(); ++t) {
        o += A.tileNb(t);
        if (c < o) return t;
    }
    return A.nt() - 1;
}

/// Copy of the tiles [i0..i1] x [k0..k1] of the physical (NoTrans) band
/// storage Ap keeping only dmin <= i - j <= dmax (global element indices of
/// Ap); real_diag drops the imaginary part on the diagonal (Hermitian band).
/// Same distribution as the sub-view, O(chunk) storage.
template <typename T>
Matrix<T> band_chunk(BaseMatrix<T> const& Ap, int64_t i0, int64_t i1, int64_t k0, int64_t k1, int64_t dmin,
                     int64_t dmax, bool real_diag, Target target) {
    Matrix<T> S(Ap.sub(i0, i1, k0, k1));
    S.set_uplo(Uplo::General);
    Matrix<T> D = S.emptyLike();
    D.insertLocalTiles(Target::Host);
    const int64_t ro = row_off(Ap, i0), co = col_off(Ap, k0);
    if (Ap.storage()->banded) {
        // band-only storage: D is co-located with the sub-view, so every
        // local element of D is a local element of Ap (stored or outside)
        auto& st = *Ap.storage();
        st.get(Loc::Host, false);
        auto& g = *st.grid;
        const int64_t R0 = Ap.row0() + ro, C0 = Ap.col0() + co;
        for_each_local(D, true, [&](int64_t i, int64_t j, T& v) {
            const int64_t gr = R0 + i, gc = C0 + j;
            T* e = st.local_ptr(Loc::Host, g2l(gr, st.mb, g.p()), g2l(gc, st.nb, g.q()));
            v = e ? *e : T(0);
        });
    } else {
        Options oh = {{Option::Target, Target::Host}};
        slate::copy<T, T>(S, D, oh);
    }
    for_each_local(D, true, [&](int64_t i, int64_t j, T& v) {
        const int64_t d = (ro + i) - (co + j);
        if (d < dmin || d > dmax) v = T(0);
        else if (real_diag && d == 0) v = T(std::real(v));
    });
    if (target == Target::Devices) D.insertLocalTiles(Target::Devices);
    return D;
}

template <typename T>
Matrix<T> op_view(Op op, Matrix<T> const& D) {
    if (op == Op::NoTrans) return D;
    return op == Op::Trans ? transpose(D) : conj_transpose(D);
}

/// Physical (NoTrans) view of a possibly transposed band operand.
template <typename T>
BaseMatrix<T> physical(BaseMatrix<T> const& A) {
    return A.op() == Op::NoTrans ? A : A.transpose_view(A.op() == Op::ConjTrans);
}

/// C = beta C (beta = 0 writes zeros, so NaNs in C do not propagate)
template <typename T>
void scale_by(T beta, Matrix<T>& C, Options const& opts) {
    if (beta == T(1)) return;
    if (beta == T(0)) slate::set(T(0), T(0), C, opts);
    else slate::add(beta, C, T(0), C, opts);
}

/// C += alpha op(A) B (Left) or alpha B op(A) (Right), A the band part
/// dmin <= i - j <= dmax of the physical storage Ap, applied block-column
/// chunk by chunk of Ap.
template <typename T>
void band_apply(Side side, Op op, T alpha, BaseMatrix<T> const& Ap, int64_t dmin, int64_t dmax, bool real_diag,
                Matrix<T> const& B, Matrix<T>& C, Options const& opts) {
    const Target target = resolve_target(opts);
    const int64_t m = Ap.m(), nt = Ap.nt(), nb = std::max<int64_t>(1, Ap.nb());
    const int64_t kc = std::max<int64_t>(1, ceildiv(std::max<int64_t>(-dmin, 0) + std::max<int64_t>(dmax, 0), nb));
    for (int64_t k0 = 0; k0 < nt; k0 += kc) {
        const int64_t k1 = std::min(nt - 1, k0 + kc - 1);
        const int64_t c0 = col_off(Ap, k0), c1 = col_off(Ap, k1) + Ap.tileNb(k1) - 1;
        const int64_t r_lo = std::max<int64_t>(0, c0 + dmin), r_hi = std::min(m - 1, c1 + dmax);
        if (r_lo > r_hi) continue;
        const int64_t i0 = tile_row_of(Ap, r_lo), i1 = tile_row_of(Ap, r_hi);
        Matrix<T> D = op_view(op, band_chunk(Ap, i0, i1, k0, k1, dmin, dmax, real_diag, target));
        // tile ranges of op(A)'s chunk: rows [a0..a1] x cols [b0..b1]
        const int64_t a0 = op == Op::NoTrans ? i0 : k0, a1 = op == Op::NoTrans ? i1 : k1;
        const int64_t b0 = op == Op::NoTrans ? k0 : i0, b1 = op == Op::NoTrans ? k1 : i1;
        if (side == Side::Left) {
            Matrix<T> Cs = C.sub(a0, a1, 0, C.nt() - 1);
            gemm(alpha, D, B.sub(b0, b1, 0, B.nt() - 1), T(1), Cs, opts);
        } else {
            Matrix<T> Cs = C.sub(0, C.mt() - 1, b0, b1);
            gemm(alpha, B.sub(0, B.mt() - 1, a0, a1), D, T(1), Cs, opts);
        }
    }
}

/// op(A) X = B (B overwritten) for a triangular band A, by a blocked
/// substitution over chunks of ~kd columns: a TRSM with the chunk's diagonal
/// triangle, then one GEMM with the band block that couples it to the next
/// rows (reference src/tbsm.cc / work_trsm's band form).
template <typename T>
void tbsm_left(Op op, BaseMatrix<T> const& Ap, Uplo u, Diag diag, int64_t kd, Matrix<T>& B, Options const& opts) {
    const Target target = resolve_target(opts);
    const int64_t nt = Ap.nt(), n = Ap.n(), nb = std::max<int64_t>(1, Ap.nb());
    const int64_t kc = std::max<int64_t>(1, ceildiv(kd, nb));
    const int64_t dmin = u == Uplo::Lower ? 0 : -kd, dmax = u == Uplo::Lower ? kd : 0;
    const bool forward = (u == Uplo::Lower) == (op == Op::NoTrans);
    // op(A)'s band block rows [r0..r1] x cols [c0..c1] (tiles)
    auto block = [&](int64_t r0, int64_t r1, int64_t c0, int64_t c1) {
        return op == Op::NoTrans ? band_chunk(Ap, r0, r1, c0, c1, dmin, dmax, false, target)
                                 : op_view(op, band_chunk(Ap, c0, c1, r0, r1, dmin, dmax, false, target));
    };
    const int64_t nchunks = ceildiv(nt, kc);
    for (int64_t s = 0; s < nchunks; ++s) {
        const int64_t cidx = forward ? s : nchunks - 1 - s;
        const int64_t k0 = cidx * kc, k1 = std::min(nt - 1, k0 + kc - 1);
        Matrix<T> Bk = B.sub(k0, k1, 0, B.nt() - 1);
        {
            Matrix<T> D = band_chunk(Ap, k0, k1, k0, k1, dmin, dmax, false, target);
            TriangularMatrix<T> Tk(u, diag, D);
            if (op == Op::NoTrans) trsm(Side::Left, T(1), Tk, Bk, opts);
            else if (op == Op::Trans) trsm(Side::Left, T(1), transpose(Tk), Bk, opts);
            else trsm(Side::Left, T(1), conj_transpose(Tk), Bk, opts);
        }
        const int64_t e0 = col_off(Ap, k0), e1 = col_off(Ap, k1) + Ap.tileNb(k1) - 1;
        if (forward && k1 + 1 < nt && kd > 0) {
            const int64_t r1 = tile_col_of(Ap, std::min(n - 1, e1 + kd));
            Matrix<T> Bs = B.sub(k1 + 1, r1, 0, B.nt() - 1);
            gemm(T(-1), block(k1 + 1, r1, k0, k1), Bk, T(1), Bs, opts);
        } else if (!forward && k0 > 0 && kd > 0) {
            const int64_t r0 = tile_col_of(Ap, std::max<int64_t>(0, e0 - kd));
            Matrix<T> Bs = B.sub(r0, k0 - 1, 0, B.nt() - 1);
            gemm(T(-1), block(r0, k0 - 1, k0, k1), Bk, T(1), Bs, opts);
        }
    }
}

}  // namespace

//------------------------------------------------------------------------------
template <typename T>
int64_t gbtrf(BandMatrix<T>& A, Pivots& pivots, Options const& opts) {
    trace::Block tb("gbtrf");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kl = A.lowerBandwidth(), ku = A.upperBandwidth();
    slate_error_if_msg(A.m() != n, "gbtrf: square band matrix required");
    const int64_t ldab = 2 * kl + ku + 1, kv = kl + ku;
    // AB(kv + i - j, j) = A(i, j); rows [0, kl) receive the fill
    std::vector<T> ab = band_gather<T>(A, kl, ku, kv, ldab);
    Target target = resolve_target(opts);
    Comm& w = A.grid()->world();
    const int64_t nb = std::max<int64_t>(1, A.nb());
    BandSlabs<T> sl(n, nb, nb * ceildiv(kl + ku + nb - 1, nb), kl, w, target);
    sl.load(ab, kv, ldab, kl, ku);
    std::vector<int64_t> ipiv;
    int64_t info = gbtrf_slabs<T>(sl, kl, ku, w, ipiv);
    sl.store(ab, kv, ldab, kl, kv, w);
    // factors: L (kl below) and U (kl + ku above); the matrix's storage holds the fill
    band_scatter<T>(A, ab, kl, kv, kv, ldab);
    A.set_band(kl, kl + ku);
    pivots_from_ipiv(A, ipiv, pivots);
    if (target == Target::Devices) A.storage()->get(Loc::Device, false);
    return info;
}

template <typename T>
void gbtrs(BandMatrix<T> const& A, Pivots const& pivots, Matrix<T>& B, Options const& opts) {
    trace::Block tb("gbtrs");
    internal::DriverScope ds_;
    // after gbtrf the stored upper bandwidth is kl + ku (the fill)
    const int64_t n = A.n(), kl = A.lowerBandwidth(), kuf = A.upperBandwidth();
    const Target target = resolve_target(opts);
    if (kl > 0 && n > 0) {
        // L with the interleaved row swaps (LAPACK gbtrs convention): the
        // swaps and eliminations of block column [j0, j1) only touch rows
        // [j0, j1 + kl).  Their product M (tile-padded, identity outside) is
        // formed on the host from the O(n * kl) L band and applied to those
        // rows of B by one distributed GEMM per block column (reference
        // src/gbtrs.cc: tbsm with pivots).
        std::vector<T> abl = band_gather<T>(A, kl, 0, 0, kl + 1);   // abl(i - j, j) = L(i, j)
        std::vector<int64_t> ipiv = ipiv_from_pivots(A, pivots);
        const int64_t nt = A.nt();
        for (int64_t k = 0; k < nt; ++k) {
            const int64_t j0 = col_off<T>(A, k), j1 = j0 + A.tileNb(k);
            const int64_t kr = tile_row_of<T>(A, std::min(n, j1 + kl) - 1);
            const int64_t R0 = row_off<T>(A, k), Rn = row_off<T>(A, kr) + A.tileMb(kr) - R0;
            // M = (swap, eliminate)_j1-1 ... (swap, eliminate)_j0 applied to
            // the identity, one column at a time (columns are independent;
            // contiguous axpys, skipped where the pivot row entry is zero).
            // Rows at or past Ct are never touched, so those columns stay e_c.
            const int64_t Ct = std::min(Rn, j1 - R0 + kl);
            std::vector<T> M(size_t(Rn) * Rn, T(0));
            #pragma omp parallel for schedule(dynamic, 16)
            for (int64_t c = 0; c < Rn; ++c) {
                T* col = M.data() + c * Rn;
                col[c] = T(1);
                if (c >= Ct) continue;
                for (int64_t j = j0; j < j1; ++j) {
                    const int64_t lj = j - R0, lp = ipiv[j] - R0;
                    if (lp != lj) std::swap(col[lj], col[lp]);
                    const T b = col[lj];
                    if (b == T(0)) continue;
                    const int64_t km = std::min(kl, n - 1 - j);
                    T const* l = abl.data() + 1 + j * (kl + 1);
                    T* y = col + lj + 1;
                    for (int64_t i = 0; i < km; ++i) y[i] -= l[i] * b;
                }
            }
            Matrix<T> Ms(BaseMatrix<T>(A).sub(k, kr, k, kr));
            Matrix<T> Mm = Ms.emptyLike();
            Mm.insertLocalTiles(Target::Host);
            for_each_local(Mm, true, [&](int64_t i, int64_t j, T& v) { v = M[i + j * Rn]; });
            if (target == Target::Devices) Mm.insertLocalTiles(Target::Devices);
            Matrix<T> Bs = B.sub(k, kr, 0, B.nt() - 1);
            Matrix<T> Bt = Bs.emptyLike();
            Bt.insertLocalTiles(target);
            slate::copy<T, T>(Bs, Bt, opts);
            gemm(T(1), Mm, Bt, T(0), Bs, opts);
        }
    }
    TriangularBandMatrix<T> U(Uplo::Upper, Diag::NonUnit, kuf, BaseMatrix<T>(A));
    tbsm(Side::Left, T(1), U, B, opts);
}

template <typename T>
int64_t gbsv(BandMatrix<T>& A, Pivots& pivots, Matrix<T>& B, Options const& opts) {
    trace::Block tb("gbsv");
    internal::DriverScope ds_;
    int64_t info = gbtrf(A, pivots, opts);
    if (info == 0) gbtrs(A, pivots, B, opts);
    return info;
}

template <typename T>
int64_t pbtrf(HermitianBandMatrix<T>& A, Options const& opts) {
    trace::Block tb("pbtrf");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kd = A.bandwidth();
    const bool upper = A.uplo() == Uplo::Upper;
    // lower band storage ab(i - j, j) = L(i, j); an Upper matrix is read as U^H
    std::vector<T> ab = upper ? band_gather<T>(A, 0, kd, 0, kd + 1, true) : band_gather<T>(A, kd, 0, 0, kd + 1);
    Target target = resolve_target(opts);
    Comm& w = A.grid()->world();
    BandSlabs<T> sl(n, std::max<int64_t>(1, A.nb()), 0, kd, w, target);
    sl.load(ab, 0, kd + 1, kd, 0);
    int64_t info = pbtrf_slabs<T>(sl, kd, w);
    sl.store(ab, 0, kd + 1, kd, 0, w);
    if (upper) band_scatter<T>(A, ab, 0, kd, 0, kd + 1, true);
    else band_scatter<T>(A, ab, kd, 0, 0, kd + 1);
    if (resolve_target(opts) == Target::Devices) A.storage()->get(Loc::Device, false);
    return info;
}

template <typename T>
void pbtrs(HermitianBandMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("pbtrs");
    internal::DriverScope ds_;
    // two distributed band triangular solves with the factor (reference
    // src/pbtrs.cc): A = L L^H (Lower) or U^H U (Upper)
    const Uplo u = A.uplo();
    TriangularBandMatrix<T> F(u, Diag::NonUnit, A.bandwidth(), BaseMatrix<T>(A));
    if (u == Uplo::Lower) {
        tbsm(Side::Left, T(1), F, B, opts);
        tbsm(Side::Left, T(1), conj_transpose(F), B, opts);
    } else {
        tbsm(Side::Left, T(1), conj_transpose(F), B, opts);
        tbsm(Side::Left, T(1), F, B, opts);
    }
}

template <typename T>
int64_t pbsv(HermitianBandMatrix<T>& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("pbsv");
    internal::DriverScope ds_;
    int64_t info = pbtrf(A, opts);
    if (info == 0) pbtrs(A, B, opts);
    return info;
}


template <typename T>
void gbmm(T alpha, BandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts) {
    trace::Block tb("gbmm");
    internal::DriverScope ds_;
    BaseMatrix<T> Ap = physical<T>(A);
    scale_by(beta, C, opts);
    if (alpha != T(0)) band_apply(Side::Left, A.op(), alpha, Ap, -Ap.ku(), Ap.kl(), false, B, C, opts);
}

template <typename T>
void hbmm(Side side, T alpha, HermitianBandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts) {
    trace::Block tb("hbmm");
    internal::DriverScope ds_;
    const int64_t kd = A.bandwidth();
    BaseMatrix<T> Ap = physical<T>(A);
    scale_by(beta, C, opts);
    if (alpha == T(0)) return;
    // A = S + E^H: S the stored triangle with a real diagonal, E its strict part
    const bool lower = A.uplo_physical() == Uplo::Lower;
    const Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
    if (lower) {
        band_apply(side, Op::NoTrans, alpha, Ap, 0, kd, true, B, C, opts);
        if (kd > 0) band_apply(side, cT, alpha, Ap, 1, kd, false, B, C, opts);
    } else {
        band_apply(side, Op::NoTrans, alpha, Ap, -kd, 0, true, B, C, opts);
        if (kd > 0) band_apply(side, cT, alpha, Ap, -kd, -1, false, B, C, opts);
    }
}

template <typename T>
void tbsm(Side side, T alpha, TriangularBandMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("tbsm");
    internal::DriverScope ds_;
    BaseMatrix<T> Ap = physical<T>(A);
    const Uplo u = A.uplo_physical();
    const int64_t kd = A.bandwidth();
    if (side == Side::Left) {
        scale_by(alpha, B, opts);
        tbsm_left(A.op(), Ap, u, A.diag(), kd, B, opts);
        return;
    }
    // X op(A) = alpha B  <=>  t(op(A)) t(X) = alpha' t(B), t = conj-transpose
    // (transpose for a Trans view of complex data), solved on a transposed copy
    const Op t = (is_complex_v<T> && A.op() == Op::Trans) ? Op::Trans : (is_complex_v<T> ? Op::ConjTrans : Op::Trans);
    const Op op2 = (A.op() == Op::NoTrans) ? t : Op::NoTrans;
    const T alpha2 = t == Op::ConjTrans ? slate::conj(alpha) : alpha;
    Matrix<T> Bt = B.emptyLike(0, 0, Op::Trans);
    Bt.insertLocalTiles(resolve_target(opts));
    slate::copy<T, T>(op_view(t, B), Bt, opts);
    scale_by(alpha2, Bt, opts);
    tbsm_left(op2, Ap, u, A.diag(), kd, Bt, opts);
    slate::copy<T, T>(op_view(t, Bt), B, opts);
}

/// tbsm with the pivots of gbtrf (reference src/tbsmPivots.cc): op(A) X =
/// alpha B (Left) or X op(A) = alpha B (Right) where the row interchanges of
/// tile k are applied to B(k:mt-1, :) just before tile k's solve on a
/// forward sweep (op(A) lower: the L factor of gbtrf) or right after it on a
/// backward sweep (op(A) upper: L^T).  Tile by tile: the diagonal tile's band
/// part by one trsm, the band below / above it by one gemm; empty pivots:
/// plain tbsm.
template <typename T>
void tbsm(Side side, T alpha, TriangularBandMatrix<T> const& A, Pivots const& pivots, Matrix<T>& B,
          Options const& opts) {
    if (pivots.empty()) { tbsm(side, alpha, A, B, opts); return; }
    trace::Block tb("tbsm_pivots");
    internal::DriverScope ds_;
    if (side == Side::Right) {
        // X op(A) = alpha B  <=>  t(op(A)) t(X) = alpha' t(B), on a transposed copy of B
        const Op t = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
        const T alpha2 = t == Op::ConjTrans ? slate::conj(alpha) : alpha;
        Matrix<T> Bt = B.emptyLike(0, 0, Op::Trans);
        Bt.insertLocalTiles(resolve_target(opts));
        slate::copy<T, T>(op_view(t, B), Bt, opts);
        TriangularBandMatrix<T> At = t == Op::ConjTrans ? conj_transpose(A) : transpose(A);
        tbsm(Side::Left, alpha2, At, pivots, Bt, opts);
        slate::copy<T, T>(op_view(t, Bt), B, opts);
        return;
    }
    const Target target = resolve_target(opts);
    BaseMatrix<T> Ap = physical<T>(A);
    const Uplo u = A.uplo_physical();
    const Op op = A.op();
    const int64_t kd = A.bandwidth(), nt = Ap.nt(), n = Ap.n();
    const int64_t dmin = u == Uplo::Lower ? 0 : -kd, dmax = u == Uplo::Lower ? kd : 0;
    const bool forward = (u == Uplo::Lower) == (op == Op::NoTrans);
    slate_error_if_msg(B.mt() != nt, "tbsm: B's tile rows must match A's tiles");
    scale_by(alpha, B, opts);
    auto block = [&](int64_t r0, int64_t r1, int64_t c0, int64_t c1) {
        return op == Op::NoTrans ? band_chunk(Ap, r0, r1, c0, c1, dmin, dmax, false, target)
                                 : op_view(op, band_chunk(Ap, c0, c1, r0, r1, dmin, dmax, false, target));
    };
    auto swaps = [&](int64_t k, bool fwd) {
        if (k >= int64_t(pivots.size()) || pivots[k].empty()) return;
        Matrix<T> Bk = B.sub(k, B.mt() - 1, 0, B.nt() - 1);
        internal::apply_pivots(Pivots{pivots[k]}, BaseMatrix<T>(Bk), Bk, target, fwd);
    };
    for (int64_t s = 0; s < nt; ++s) {
        const int64_t k = forward ? s : nt - 1 - s;
        if (forward) swaps(k, true);
        Matrix<T> Bk = B.sub(k, k, 0, B.nt() - 1);
        const int64_t e0 = col_off(Ap, k), e1 = e0 + Ap.tileNb(k) - 1;
        if (!forward && k + 1 < nt && kd > 0) {
            // B(k) -= op(A)(k, k+1 : k_end) B(k+1 : k_end)
            const int64_t c1 = tile_col_of(Ap, std::min(n - 1, e1 + kd));
            Matrix<T> Bs = B.sub(k + 1, c1, 0, B.nt() - 1);
            gemm(T(-1), block(k, k, k + 1, c1), Bs, T(1), Bk, opts);
        }
        {
            Matrix<T> D = band_chunk(Ap, k, k, k, k, dmin, dmax, false, target);
            TriangularMatrix<T> Tk(u, A.diag(), D);
            if (op == Op::NoTrans) trsm(Side::Left, T(1), Tk, Bk, opts);
            else if (op == Op::Trans) trsm(Side::Left, T(1), transpose(Tk), Bk, opts);
            else trsm(Side::Left, T(1), conj_transpose(Tk), Bk, opts);
        }
        if (forward && k + 1 < nt && kd > 0) {
            // B(k+1 : i_end) -= op(A)(k+1 : i_end, k) B(k)
            const int64_t r1 = tile_col_of(Ap, std::min(n - 1, e1 + kd));
            Matrix<T> Bs = B.sub(k + 1, r1, 0, B.nt() - 1);
            gemm(T(-1), block(k + 1, r1, k, k), Bk, T(1), Bs, opts);
        }
        if (!forward) swaps(k, false);
    }
}

#define SLATE_BAND_INST(T)                                                                                 \
    template int64_t gbtrf<T>(BandMatrix<T>&, Pivots&, Options const&);                                   \
    template void gbtrs<T>(BandMatrix<T> const&, Pivots const&, Matrix<T>&, Options const&);              \
    template int64_t gbsv<T>(BandMatrix<T>&, Pivots&, Matrix<T>&, Options const&);                        \
    template int64_t pbtrf<T>(HermitianBandMatrix<T>&, Options const&);                                   \
    template void pbtrs<T>(HermitianBandMatrix<T> const&, Matrix<T>&, Options const&);                    \
    template int64_t pbsv<T>(HermitianBandMatrix<T>&, Matrix<T>&, Options const&);                        \
    template void gbmm<T>(T, BandMatrix<T> const&, Matrix<T> const&, T, Matrix<T>&, Options const&);      \
    template void tbsm<T>(Side, T, TriangularBandMatrix<T> const&, Pivots const&, Matrix<T>&, Options const&); \
    template void hbmm<T>(Side, T, HermitianBandMatrix<T> const&, Matrix<T> const&, T, Matrix<T>&,        \
                          Options const&);                                                                 \
    template void tbsm<T>(Side, T, TriangularBandMatrix<T> const&, Matrix<T>&, Options const&);

SLATE_BAND_INST(float)
SLATE_BAND_INST(double)
SLATE_BAND_INST(std::complex<float>)
SLATE_BAND_INST(std::complex<double>)

}  // namespace slate
