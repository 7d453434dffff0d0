// Driver-internal helpers: distribution math over a view, panel broadcasts
// and tile exchanges.  These replace the reference's listBcast / listReduce /
// tileSend / tileRecv (BaseMatrix.hh:1762-2456) with whole-panel collectives:
// one contiguous buffer per panel per communicator instead of one message
// per tile.
#pragma once

#include "slate_amd/slate.hh"
#include "slate_amd/runtime.hh"
#include "slate_amd/trace.hh"

#include <cstdlib>
#include <functional>
#include <vector>

namespace slate {
namespace internal {
/// Working precision of the mixed-precision solvers' factorization.
template <typename T> struct lower_prec { using type = T; };
template <> struct lower_prec<double> { using type = float; };
template <> struct lower_prec<std::complex<double>> { using type = std::complex<float>; };

/// GMRES-IR continuation of a mixed-precision solve (gmres.cc): each column
/// of X (the current estimate) is refined by restarted GMRES on A x = b with
/// the low-precision factors as right preconditioner (solve_lo, in place on a
/// low-precision vector); residual(R, V) computes R -= A V.  Returns true when
/// every column met the classical stopping test; iters = the largest GMRES
/// iteration count over the columns.
template <typename T>
bool gmres_refine(Matrix<T>& B, Matrix<T>& X, real_type<T> Anorm, int itermax, int& iters,
                  std::function<void(Matrix<T>&, Matrix<T>&)> const& residual,
                  std::function<void(Matrix<typename lower_prec<T>::type>&)> const& solve_lo, Options const& opts);
}  // namespace internal

namespace internal {

/// Real trailing updates C -= X Y as NT products against a transposed copy of
/// Y (the 4-wave rotated MFMA tile, measured faster than the NN 8-wave tile
/// on large shapes); SLATE_UPDATE_NT=0 keeps the NN form.
inline bool update_nt() {
    static const bool v = [] {
        const char* e = std::getenv("SLATE_UPDATE_NT");
        return e ? std::atoi(e) != 0 : true;
    }();
    return v;
}

/// Local row offset within `A`'s local block for view row-tile index i (first
/// local row whose global index is >= start of tile i).
template <typename T>
inline int64_t lrow_of(BaseMatrix<T> const& A, int64_t i) {
    auto& s = *A.storage();
    int64_t g = (i < A.mt() ? std::max<int64_t>(0, (A.row0() / s.mb + i) * s.mb - A.row0()) : A.srows());
    return g2l_ceil(A.row0() + std::min(g, A.srows()), s.mb, s.rrel(), s.grid->p()) - A.lrow_begin();
}
template <typename T>
inline int64_t lcol_of(BaseMatrix<T> const& A, int64_t j) {
    auto& s = *A.storage();
    int64_t g = (j < A.nt() ? std::max<int64_t>(0, (A.col0() / s.nb + j) * s.nb - A.col0()) : A.scols());
    return g2l_ceil(A.col0() + std::min(g, A.scols()), s.nb, s.crel(), s.grid->q()) - A.lcol_begin();
}

/// Global row/col (within view) where tile i/j starts.
template <typename T>
inline int64_t grow_of(BaseMatrix<T> const& A, int64_t i) {
    auto& s = *A.storage();
    if (i >= A.mt()) return A.srows();
    return std::max<int64_t>(0, (A.row0() / s.mb + i) * s.mb - A.row0());
}
template <typename T>
inline int64_t gcol_of(BaseMatrix<T> const& A, int64_t j) {
    auto& s = *A.storage();
    if (j >= A.nt()) return A.scols();
    return std::max<int64_t>(0, (A.col0() / s.nb + j) * s.nb - A.col0());
}

/// Dense device/host buffer sized for panels.
template <typename T>
class Work {
public:
    Work() = default;
    Work(Target t, size_t n) { resize(t, n); }
    void resize(Target t, size_t n) {
        dev_ = (t == Target::Devices);
        if (n <= n_) return;
        release();
        n_ = std::max<size_t>(n, 1);
        if (dev_) p_ = static_cast<T*>(device::malloc(n_ * sizeof(T)));
        else { h_.assign(n_, T(0)); p_ = h_.data(); }
    }
    ~Work() { release(); }
    Work(Work&& o) noexcept { *this = std::move(o); }
    Work& operator=(Work&& o) noexcept {
        release();
        p_ = o.p_; n_ = o.n_; dev_ = o.dev_; h_ = std::move(o.h_);
        if (!dev_) p_ = h_.data();
        o.p_ = nullptr; o.n_ = 0;
        return *this;
    }
    T* data() const { return p_; }
    size_t size() const { return n_; }
private:
    void release() {
        if (dev_ && p_) device::free(p_);
        p_ = nullptr; n_ = 0; h_.clear();
    }
    T* p_ = nullptr;
    size_t n_ = 0;
    bool dev_ = false;
    std::vector<T> h_;
};

/// Location of a target.
inline Loc loc_of(Target t) { return t == Target::Devices ? Loc::Device : Loc::Host; }

/// Normalize a HostTask/HostNest/HostBatch/Host target; Devices requires a GPU.
inline Target resolve_target(Options const& opts) {
    Target t = get_target(opts, Target::HostTask);
    if (t == Target::Devices && !device::available())
        slate_error("Target::Devices requested but no HIP device is available");
    return t;
}

/// Driver nesting depth on this thread.  Option::HoldLocalWorkspace = false
/// (the default, reference src/potrf.cc:42,198) frees a matrix's non-origin
/// instance -- the device copy of a host-origin matrix, i.e. SLATE's
/// workspace tiles -- when the OUTERMOST driver finishes, so composite drivers
/// (gesv = getrf + getrs, posv, gels, ...) keep it between their stages.
inline int& driver_depth() { thread_local int d = 0; return d; }
struct DriverScope {
    DriverScope() { ++driver_depth(); }
    ~DriverScope() { --driver_depth(); }
    DriverScope(DriverScope const&) = delete;
    DriverScope& operator=(DriverScope const&) = delete;
};

/// End of a driver for an output matrix: write back to the origin instance
/// (tileUpdateAllOrigin) and release the workspace instance unless held.
template <typename T>
inline void finish_origin(BaseMatrix<T> const& A, Options const& opts) {
    A.storage()->update_origin();
    if (driver_depth() <= 1 && !get_option<bool>(opts, Option::HoldLocalWorkspace, false))
        A.storage()->release_workspace();
}

/// Block-cyclic working copy of an arbitrary-distribution (lambda
/// constructor) matrix or of a view of one: the drivers' contiguous local
/// arrays need the 2-D block-cyclic layout, while the reference drivers
/// consume any layout tile by tile.  Same processes; the largest tile of A
/// becomes the uniform tile.  The copy is the tile-by-tile redistribution.
template <typename T>
Matrix<T> block_cyclic(BaseMatrix<T> const& A, Options const& opts) {
    const int64_t b = std::max<int64_t>(1, std::max(A.storage()->mb, A.storage()->nb));
    Matrix<T> B(A.m(), A.n(), b, b, A.grid());
    B.insertLocalTiles(resolve_target(opts));
    slate::copy<T, T>(A, B, opts);
    return B;
}
/// A itself, or its block-cyclic copy when A has an arbitrary distribution
template <typename T>
Matrix<T> bc_operand(BaseMatrix<T> const& A, Options const& opts) {
    return A.arbitrary_layout() ? block_cyclic(A, opts) : Matrix<T>(A);
}
/// Block-cyclic copy of B whose row tiles are those of the (block-cyclic)
/// factor F, on F's grid: the right-hand side of a solve with F's factors.
template <typename T>
Matrix<T> block_cyclic_rows_of(BaseMatrix<T> const& F, BaseMatrix<T> const& B, Options const& opts) {
    Matrix<T> Bb(B.m(), B.n(), F.mb(), F.mb(), F.grid());
    Bb.insertLocalTiles(resolve_target(opts));
    slate::copy<T, T>(B, Bb, opts);
    return Bb;
}
/// Pivots / T factors of an arbitrary-layout matrix are expressed in the
/// tiling of its block-cyclic working copy (block_cyclic(), tile size = the
/// largest tile of A), which is deterministic; the solve-side drivers (getrs,
/// getri, unmqr, unmlq) re-create that copy, so factor and solve agree.
template <typename T>
bool needs_bc(BaseMatrix<T> const& A, BaseMatrix<T> const& B) {
    return A.arbitrary_layout() || B.arbitrary_layout();
}

/// Visit every STORED local element of the NoTrans view A on the host
/// instance (dense: the whole local block; band-only storage: the stored band
/// tiles) with its view-relative global (i, j): f(i, j, T& value).
template <typename T, typename F>
void for_each_stored(BaseMatrix<T> const& A, bool write, F&& f) {
    slate_error_if_msg(A.op() != Op::NoTrans, "for_each_stored: NoTrans view required");
    auto& s = *A.storage();
    s.get(Loc::Host, write);
    const int64_t r0 = A.lrow_begin(), r1 = A.lrow_end();
    const int p = s.grid->p(), q = s.grid->q();
    for (int64_t lc = A.lcol_begin(); lc < A.lcol_end(); ++lc) {
        const int64_t gc = l2g(lc, s.nb, s.crel(), q) - A.col0();
        int64_t a = r0, b = r1;
        if (s.banded) {
            const int64_t lj = lc / s.nb;
            a = std::max(r0, s.boff[lj]);
            b = std::min(r1, s.bend[lj]);
        }
        if (b <= a) continue;
        T* col = s.local_ptr(Loc::Host, a, lc);
        for (int64_t lr = a; lr < b; ++lr) f(l2g(lr, s.mb, s.rrel(), p) - A.row0(), gc, col[lr - a]);
    }
}

/// Broadcast a contiguous buffer over `comm` from `root` (stream-ordered).
template <typename T>
inline void bcast(Comm& comm, T* buf, size_t count, int root, lb::Ctx const& c) {
    if (comm.size() == 1 || count == 0) return;
    comm.bcast(buf, count, root, c.loc(), c.stream);
}

/// Pack a strided block into a dense buffer (ld = m).
template <typename T>
inline void pack(lb::Ctx const& c, int64_t m, int64_t n, T const* A, int64_t lda, T* W) {
    lb::copy2d(c, m, n, A, lda, W, m);
}

/// Reduce info across ranks (reference internal_reduce_info.cc): min over
/// nonzero values.
int64_t reduce_info(int64_t info, Comm& comm);

/// Read a device (or host) int info.
int64_t fetch_info(Target t, int* info);

/// All-gather of per-column norms etc. helper: allreduce on host vector.
template <typename R>
inline void allreduce_host(Comm& comm, R* v, size_t n, ReduceOp op) {
    if (comm.size() == 1 || n == 0) return;
    comm.allreduce(v, v, n, scalar_type<R>(), op, Loc::Host, nullptr);
}

/// Replicated LAPACK band storage: AB(r0 + i - j, j) = A(i, j) for
/// -ku <= i - j <= kl; ldab >= r0 + kl + 1.  conj_upper: read A's upper
/// band (i < j) as the conj-transposed lower band (Hermitian band, Upper).
template <typename T>
std::vector<T> band_gather(BaseMatrix<T> const& A, int64_t kl, int64_t ku, int64_t r0, int64_t ldab,
                           bool upper_as_lower = false) {
    const int64_t n = A.n();
    std::vector<T> ab(size_t(ldab) * n, T(0));
    for_each_stored(A, false, [&](int64_t i, int64_t j, T& v) {
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
void band_scatter(BaseMatrix<T>& A, std::vector<T> const& ab, int64_t kl, int64_t ku, int64_t r0, int64_t ldab,
                  bool upper_as_lower = false) {
    for_each_stored(A, true, [&](int64_t i, int64_t j, T& v) {
        if (upper_as_lower) {
            if (j >= i && j - i <= ku) v = slate::conj(ab[(r0 + j - i) + i * ldab]);
        } else if (i - j <= kl && j - i <= ku) {
            v = ab[(r0 + i - j) + j * ldab];
        }
    });
}

/// General redistribution B = op(A) between two matrices over the same world
/// (any grids / tile sizes with equal element counts), tile by tile over p2p.
template <typename T>
void redistribute_op(BaseMatrix<T> const& A, BaseMatrix<T>& B, Target target);

/// Distributed tridiagonal eigensolvers (eig_dist.cc): divide and conquer
/// with Q on its 2-D grid, and QL with the rotations applied to each rank's
/// rows of Z.  d, e replicated; eigenvalues ascending in d.
template <typename R>
void stedc_dist(std::vector<R>& d, std::vector<R> const& e, Matrix<R>& Q, Options const& opts);
template <typename T>
int64_t steqr2_dist(std::vector<real_type<T>>& d, std::vector<real_type<T>>& e, Matrix<T>& Z, Options const& opts);

/// Apply LU pivots to the rows of B (forward: P B; backward: P^T B).
template <typename T>
void apply_pivots(Pivots const& pivots, BaseMatrix<T> const& A, Matrix<T>& B, Target target, bool forward);

}  // namespace internal
}  // namespace slate
