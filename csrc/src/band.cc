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
// whole-panel collectives instead of per-tile messages.  The solves and band
// multiplies keep the band form on the host / a band-masked operand.
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
    slate_error_if_msg(A.op() != Op::NoTrans, "band: NoTrans view required");
    auto& s = *A.storage();
    s.get(Loc::Host, write);
    const int64_t ld = s.ld(Loc::Host);
    LocalBlock<T> la = A.local_raw(Loc::Host);
    std::vector<int64_t> gr(la.m);
    for (int64_t il = 0; il < la.m; ++il)
        gr[il] = l2g(A.lrow_begin() + il, s.mb, s.rrel(), s.grid->p()) - A.row0();
    for (int64_t jl = 0; jl < la.n; ++jl) {
        int64_t gc = l2g(A.lcol_begin() + jl, s.nb, s.crel(), s.grid->q()) - A.col0();
        for (int64_t il = 0; il < la.m; ++il) f(gr[il], gc, la.ptr[il + jl * ld]);
    }
}

/// Replicated LAPACK band storage: AB(r0 + i - j, j) = A(i, j) for
/// -ku <= i - j <= kl; ldab >= r0 + kl + 1.  conj_upper: read A's upper
/// band (i < j) as the conj-transposed lower band (Hermitian band, Upper).
template <typename T>
std::vector<T> gather_band(BaseMatrix<T> const& A, int64_t kl, int64_t ku, int64_t r0, int64_t ldab,
                           bool upper_as_lower = false) {
    const int64_t n = A.n();
    std::vector<T> ab(size_t(ldab) * n, T(0));
    for_each_local(A, false, [&](int64_t i, int64_t j, T& v) {
        if (upper_as_lower) {
            if (j >= i && j - i <= ku) ab[(r0 + j - i) + i * ldab] = slate::conj(v);   // (j, i) of the lower band
        } else if (i - j <= kl && j - i <= ku) {
            ab[(r0 + i - j) + j * ldab] = v;
        }
    });
    // every band entry is owned by exactly one rank
    Comm& w = A.grid()->world();
    if (w.size() > 1) {
        using R = real_type<T>;
        size_t mult = is_complex_v<T> ? 2 : 1;
        allreduce_host<R>(w, reinterpret_cast<R*>(ab.data()), ab.size() * mult, ReduceOp::Sum);
    }
    return ab;
}

template <typename T>
void scatter_band(BaseMatrix<T>& A, std::vector<T> const& ab, int64_t kl, int64_t ku, int64_t r0, int64_t ldab,
                  bool upper_as_lower = false) {
    for_each_local(A, true, [&](int64_t i, int64_t j, T& v) {
        if (upper_as_lower) {
            if (j >= i && j - i <= ku) v = slate::conj(ab[(r0 + j - i) + i * ldab]);
        } else if (i - j <= kl && j - i <= ku) {
            v = ab[(r0 + i - j) + j * ldab];
        }
    });
}

/// Dense (replicated, column-major) copy of a distributed matrix.
template <typename T>
std::vector<T> gather_dense(BaseMatrix<T> const& B, Options const& opts) {
    std::vector<T> b;
    gather(B, b, opts);
    return b;
}

template <typename T>
void scatter_dense(Matrix<T>& B, std::vector<T> const& b, int64_t ldb) {
    for_each_local(B, true, [&](int64_t i, int64_t j, T& v) { v = b[i + j * ldb]; });
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

template <typename T>
void gbtrs_host(int64_t n, int64_t kl, int64_t ku, int64_t nrhs, T const* ab, int64_t ldab, int64_t const* ipiv,
                T* b, int64_t ldb) {
    const int64_t kv = ku + kl;
    auto A = [&](int64_t i, int64_t j) { return ab[(kv + i - j) + j * ldab]; };
    #pragma omp parallel for schedule(static) if (nrhs > 1)
    for (int64_t c = 0; c < nrhs; ++c) {
        T* x = b + c * ldb;
        for (int64_t j = 0; j < n; ++j) {
            if (ipiv[j] != j) std::swap(x[j], x[ipiv[j]]);
            int64_t km = std::min(kl, n - 1 - j);
            for (int64_t i = 1; i <= km; ++i) x[j + i] -= A(j + i, j) * x[j];
        }
        for (int64_t j = n - 1; j >= 0; --j) {
            x[j] /= A(j, j);
            int64_t lo = std::max<int64_t>(0, j - kv);
            for (int64_t i = lo; i < j; ++i) x[i] -= A(i, j) * x[j];
        }
    }
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

template <typename T>
void pbtrs_host(int64_t n, int64_t kd, int64_t nrhs, T const* ab, int64_t ldab, T* b, int64_t ldb) {
    auto L = [&](int64_t i, int64_t j) { return ab[(i - j) + j * ldab]; };
    #pragma omp parallel for schedule(static) if (nrhs > 1)
    for (int64_t c = 0; c < nrhs; ++c) {
        T* x = b + c * ldb;
        for (int64_t j = 0; j < n; ++j) {
            x[j] /= L(j, j);
            int64_t kn = std::min(kd, n - 1 - j);
            for (int64_t i = 1; i <= kn; ++i) x[j + i] -= L(j + i, j) * x[j];
        }
        for (int64_t j = n - 1; j >= 0; --j) {
            int64_t kn = std::min(kd, n - 1 - j);
            T s = x[j];
            for (int64_t i = 1; i <= kn; ++i) s -= slate::conj(L(j + i, j)) * x[j + i];
            x[j] = s / slate::conj(L(j, j));
        }
    }
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

/// General copy of a band matrix with out-of-band entries zeroed.
template <typename T>
Matrix<T> band_dense(BaseMatrix<T> const& A, int64_t kl, int64_t ku, Options const& opts, bool herm = false,
                     Uplo uplo = Uplo::General) {
    Target target = resolve_target(opts);
    Matrix<T> G(A);
    G.set_uplo(Uplo::General);
    Matrix<T> D = G.emptyLike();
    D.insertLocalTiles(Target::Host);
    Options oh = {{Option::Target, Target::Host}};
    slate::copy<T, T>(G, D, oh);
    if (herm) {
        // Hermitian band stored in one triangle: mirror it
        Matrix<T> Dh = D.emptyLike();
        Dh.insertLocalTiles(Target::Host);
        slate::copy<T, T>(conj_transpose(D), Dh, oh);
        D.storage()->get(Loc::Host, true);
        // combine: D(i,j) = stored-triangle value, other triangle from Dh
        LocalBlock<T> ld = D.local_raw(Loc::Host), lh = Dh.local_raw(Loc::Host);
        auto& s = *D.storage();
        for (int64_t jl = 0; jl < ld.n; ++jl) {
            int64_t gc = l2g(D.lcol_begin() + jl, s.nb, s.crel(), s.grid->q()) - D.col0();
            for (int64_t il = 0; il < ld.m; ++il) {
                int64_t gr = l2g(D.lrow_begin() + il, s.mb, s.rrel(), s.grid->p()) - D.row0();
                bool stored = (uplo == Uplo::Lower) ? gr >= gc : gr <= gc;
                T v = stored ? ld.ptr[il + jl * ld.ld] : lh.ptr[il + jl * lh.ld];
                if (gr == gc) v = T(std::real(v));
                ld.ptr[il + jl * ld.ld] = v;
            }
        }
    }
    for_each_local(D, true, [&](int64_t i, int64_t j, T& v) {
        if (i - j > kl || j - i > ku) v = T(0);
    });
    if (target == Target::Devices) D.insertLocalTiles(Target::Devices);
    return D;
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
    std::vector<T> ab = gather_band<T>(A, kl, ku, kv, ldab);
    Target target = resolve_target(opts);
    Comm& w = A.grid()->world();
    const int64_t nb = std::max<int64_t>(1, A.nb());
    BandSlabs<T> sl(n, nb, nb * ceildiv(kl + ku + nb - 1, nb), kl, w, target);
    sl.load(ab, kv, ldab, kl, ku);
    std::vector<int64_t> ipiv;
    int64_t info = gbtrf_slabs<T>(sl, kl, ku, w, ipiv);
    sl.store(ab, kv, ldab, kl, kv, w);
    // factors: L (kl below) and U (kl + ku above); the matrix's storage holds the fill
    scatter_band<T>(A, ab, kl, kv, kv, ldab);
    A.set_band(kl, kl + ku);
    pivots_from_ipiv(A, ipiv, pivots);
    if (target == Target::Devices) A.storage()->get(Loc::Device, false);
    return info;
}

template <typename T>
void gbtrs(BandMatrix<T> const& A, Pivots const& pivots, Matrix<T>& B, Options const& opts) {
    trace::Block tb("gbtrs");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kl = A.lowerBandwidth(), ku_f = A.upperBandwidth();
    // after gbtrf the stored upper bandwidth is kl + ku (fill)
    const int64_t ku = std::max<int64_t>(ku_f - kl, 0);
    const int64_t ldab = 2 * kl + ku + 1;
    std::vector<T> ab = gather_band<T>(A, kl, kl + ku, kl + ku, ldab);
    std::vector<int64_t> ipiv = ipiv_from_pivots(A, pivots);
    std::vector<T> b = gather_dense(B, opts);
    gbtrs_host<T>(n, kl, ku, B.n(), ab.data(), ldab, ipiv.data(), b.data(), n);
    scatter_dense(B, b, n);
    if (resolve_target(opts) == Target::Devices) B.storage()->get(Loc::Device, false);
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
    std::vector<T> ab = upper ? gather_band<T>(A, 0, kd, 0, kd + 1, true) : gather_band<T>(A, kd, 0, 0, kd + 1);
    Target target = resolve_target(opts);
    Comm& w = A.grid()->world();
    BandSlabs<T> sl(n, std::max<int64_t>(1, A.nb()), 0, kd, w, target);
    sl.load(ab, 0, kd + 1, kd, 0);
    int64_t info = pbtrf_slabs<T>(sl, kd, w);
    sl.store(ab, 0, kd + 1, kd, 0, w);
    if (upper) scatter_band<T>(A, ab, 0, kd, 0, kd + 1, true);
    else scatter_band<T>(A, ab, kd, 0, 0, kd + 1);
    if (resolve_target(opts) == Target::Devices) A.storage()->get(Loc::Device, false);
    return info;
}

template <typename T>
void pbtrs(HermitianBandMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("pbtrs");
    internal::DriverScope ds_;
    const int64_t n = A.n(), kd = A.bandwidth();
    const bool upper = A.uplo() == Uplo::Upper;
    std::vector<T> ab = upper ? gather_band<T>(A, 0, kd, 0, kd + 1, true) : gather_band<T>(A, kd, 0, 0, kd + 1);
    std::vector<T> b = gather_dense(B, opts);
    pbtrs_host<T>(n, kd, B.n(), ab.data(), kd + 1, b.data(), n);
    scatter_dense(B, b, n);
    if (resolve_target(opts) == Target::Devices) B.storage()->get(Loc::Device, false);
}

template <typename T>
int64_t pbsv(HermitianBandMatrix<T>& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("pbsv");
    internal::DriverScope ds_;
    int64_t info = pbtrf(A, opts);
    if (info == 0) pbtrs(A, B, opts);
    return info;
}

//------------------------------------------------------------------------------
template <typename T>
void gbmm(T alpha, BandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts) {
    trace::Block tb("gbmm");
    internal::DriverScope ds_;
    Matrix<T> D = band_dense<T>(A, A.lowerBandwidth(), A.upperBandwidth(), opts);
    gemm(alpha, D, B, beta, C, opts);
}

template <typename T>
void hbmm(Side side, T alpha, HermitianBandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts) {
    trace::Block tb("hbmm");
    internal::DriverScope ds_;
    const int64_t kd = A.bandwidth();
    Matrix<T> D = band_dense<T>(A, kd, kd, opts, true, A.uplo());
    if (side == Side::Left) gemm(alpha, D, B, beta, C, opts);
    else gemm(alpha, B, D, beta, C, opts);
}

template <typename T>
void tbsm(Side side, T alpha, TriangularBandMatrix<T> const& A, Matrix<T>& B, Options const& opts) {
    trace::Block tb("tbsm");
    internal::DriverScope ds_;
    Matrix<T> D = band_dense<T>(A, A.kl(), A.ku(), opts);
    TriangularMatrix<T> Tm(A.uplo(), A.diag(), D);
    trsm(side, alpha, Tm, B, opts);
}

#define SLATE_BAND_INST(T)                                                                                 \
    template int64_t gbtrf<T>(BandMatrix<T>&, Pivots&, Options const&);                                   \
    template void gbtrs<T>(BandMatrix<T> const&, Pivots const&, Matrix<T>&, Options const&);              \
    template int64_t gbsv<T>(BandMatrix<T>&, Pivots&, Matrix<T>&, Options const&);                        \
    template int64_t pbtrf<T>(HermitianBandMatrix<T>&, Options const&);                                   \
    template void pbtrs<T>(HermitianBandMatrix<T> const&, Matrix<T>&, Options const&);                    \
    template int64_t pbsv<T>(HermitianBandMatrix<T>&, Matrix<T>&, Options const&);                        \
    template void gbmm<T>(T, BandMatrix<T> const&, Matrix<T> const&, T, Matrix<T>&, Options const&);      \
    template void hbmm<T>(Side, T, HermitianBandMatrix<T> const&, Matrix<T> const&, T, Matrix<T>&,        \
                          Options const&);                                                                 \
    template void tbsm<T>(Side, T, TriangularBandMatrix<T> const&, Matrix<T>&, Options const&);

SLATE_BAND_INST(float)
SLATE_BAND_INST(double)
SLATE_BAND_INST(std::complex<float>)
SLATE_BAND_INST(std::complex<double>)

}  // namespace slate
