// Transparent single-process multi-GPU for the C++ / C / Python drivers.
//
// Reference: one MPI rank drives all of its GPUs -- MatrixStorage gives tile
// (i, j) to device func::device_1d_grid(GridOrder::Row, q, num_devices())
// (include/slate/internal/MatrixStorage.hh:503-506), so a plain
// slate::potrf(A, {Target::Devices}) on one process uses every GPU.
//
// Here a GPU is a rank of the ordinary p x q machinery (inproc.hh): when a
// driver is called with Target::Devices on matrices of a 1 x 1 grid, by a
// thread that is not itself an in-process rank, and the process may use
// more than one GPU (inproc_ranks(): every visible GPU unless a launcher
// started one process per GPU or the program picked its device;
// $SLATE_INPROC_RANKS), the driver runs on a p x q grid of in-process ranks
// over 2-D block-cyclic copies of its operands (each rank copies its own
// tiles in from the caller's storage over xGMI peer reads and its output
// tiles back), and the caller's matrices stay where they were.
// $SLATE_SPREAD=0 turns it off; problems under kSpreadMinN rows
// ($SLATE_SPREAD_MIN_N) stay on one GPU.
#pragma once

#include "slate_amd/inproc.hh"
#include "internal.hh"

#include <cstdlib>
#include <functional>
#include <type_traits>
#include <vector>

namespace slate {
namespace internal {

constexpr int64_t kSpreadMinN = 2048;

template <typename T>
struct SpreadArg {
    BaseMatrix<T> const* M;
    bool out;
};

inline bool spread_allowed(Options const& opts) {
    static const bool on = [] {
        const char* e = std::getenv("SLATE_SPREAD");
        return !e || std::atoi(e) != 0;
    }();
    // only the outermost driver spreads: a driver called by another driver
    // (gesv_mixed's getrf / getrs, GMRES's gemm, rbt, condest) runs where its
    // caller runs instead of re-scattering its operands on every call
    if (!on || in_inproc_rank() || driver_depth() > 0) return false;
    if (get_target(opts, Target::HostTask) != Target::Devices || !device::available()) return false;
    return inproc_ranks() > 1;
}

/// Runs body(per-rank matrices, rank) on in-process ranks and returns true,
/// or returns false (the caller takes its one-GPU path).
///
/// Multi-device operands (Matrix::multiDevice / fromDevices(Aarray,
/// num_devices)): the body runs on their group's ranks directly on the parts
/// -- the same view (offsets, op, uplo, ...) on every rank's local storage,
/// no copies -- whatever the driver nesting; every multi-device operand must
/// live on the same group.  One-GPU operands of such a call (full views on a
/// 1 x 1 grid) are copied in (and out, for outputs) around the body.
///
/// Otherwise (spread_allowed: Target::Devices, an outermost driver, several
/// GPUs usable) every argument must be a full, non-transposed, block-cyclic
/// view with square tiles on a 1 x 1 grid and the first argument must have at
/// least kSpreadMinN rows and a tile row per rank: the body then runs on the
/// inproc_ranks() group over block-cyclic copies of the operands.
///
/// copy_path = false (drivers whose outputs cannot be copied back, e.g. QR T
/// factors): only the multi-device case.  Arguments without storage (empty
/// matrices, e.g. no eigenvectors) reach the body as empty matrices.
template <typename T>
bool spread(Options const& opts, std::vector<SpreadArg<T>> const& args,
            std::function<void(std::vector<Matrix<T>>&, int)> const& body, bool copy_path = true) {
    if (args.empty()) return false;
    std::shared_ptr<InprocGroup> group;
    for (auto const& a : args)
        if (a.M->storage() && a.M->is_multi_device()) {
            auto const& g = a.M->storage()->group;
            slate_error_if_msg(group && group != g,
                               "multi-device operands must live on the same devices (one in-process group)");
            group = g;
        }
    const bool multi = group != nullptr;
    auto full_view = [](BaseMatrix<T> const& M) {
        auto st = M.storage();
        return st && !st->multi() && !M.arbitrary_layout() && M.grid()->size() == 1 && M.op() == Op::NoTrans &&
               M.row0() == 0 && M.col0() == 0 && M.srows() == st->m && M.scols() == st->n && M.mb() == M.nb();
    };
    if (!multi) {
        if (!copy_path || !spread_allowed(opts)) return false;
        for (auto const& a : args)
            if (!full_view(*a.M)) return false;
        const int nr = inproc_ranks();
        auto const& A0 = *args[0].M;
        static const int64_t min_n = [] {
            const char* e = std::getenv("SLATE_SPREAD_MIN_N");
            return e ? std::atoll(e) : kSpreadMinN;
        }();
        if (A0.m() < min_n || (A0.m() + A0.nb() - 1) / A0.nb() < nr) return false;
        group = InprocGroup::of_size(nr);
    } else {
        for (auto const& a : args)
            slate_error_if_msg(a.M->storage() && !a.M->is_multi_device() && !full_view(*a.M),
                               "a one-GPU operand of a multi-device call must be a whole matrix with square tiles");
    }
    // the caller's one-GPU operands: where each one is valid (its device, else host)
    struct Src { T* ptr = nullptr; int64_t ld = 0; };
    std::vector<Src> src(args.size());
    bool copies = false;
    for (size_t i = 0; i < args.size(); ++i) {
        auto const& a = args[i];
        if (!a.M->storage() || a.M->is_multi_device()) continue;
        auto const& st = *a.M->storage();
        const Loc loc = st.has(Loc::Device) && st.state(Loc::Device) != Invalid ? Loc::Device : Loc::Host;
        LocalBlock<T> L = a.M->local(loc, a.out);   // for outputs: the other instance goes stale
        src[i] = {L.ptr, L.ld};
        copies = true;
    }
    if (copies && device::available()) device::sync_all();   // the caller's queued work on its operands is done
    const bool dev = device::available();
    const Target tgt = dev ? Target::Devices : Target::Host;
    group->run([&](int rank, GridPtr const& g) {
        // multi-device parts live on the devices: drivers given no target use them there
        struct TargetScope {
            Target prev;
            explicit TargetScope(Target t) : prev(thread_default_target()) { thread_default_target() = t; }
            ~TargetScope() { thread_default_target() = prev; }
        } ts(multi && dev ? Target::Devices : thread_default_target());
        std::vector<Matrix<T>> X;
        for (size_t i = 0; i < args.size(); ++i) {
            auto const& M = *args[i].M;
            if (!M.storage()) { X.push_back(Matrix<T>()); continue; }
            if (M.is_multi_device()) {
                X.push_back(Matrix<T>(M.on_part(rank)));
                continue;
            }
            Matrix<T> C(M.m(), M.n(), M.nb(), g);
            C.insertLocalTiles(tgt);
            scatter_from_host(static_cast<T const*>(src[i].ptr), src[i].ld, C, tgt);
            X.push_back(C);
        }
        body(X, rank);
        for (size_t i = 0; i < args.size(); ++i)
            if (args[i].out && args[i].M->storage() && !args[i].M->is_multi_device())
                gather_to_host(X[i], src[i].ptr, src[i].ld);
    });
    return true;
}

/// Default target of the calling (rank) thread for a scope: multi-device
/// parts live on the devices.
struct TargetScope {
    Target prev;
    explicit TargetScope(Target t) : prev(thread_default_target()) {
        thread_default_target() = device::available() ? t : Target::Host;
    }
    ~TargetScope() { thread_default_target() = prev; }
    TargetScope(TargetScope const&) = delete;
    TargetScope& operator=(TargetScope const&) = delete;
};

/// copy() with a multi-device source and / or destination: part by part when
/// both live on one group; a whole one-GPU matrix scattered into a whole
/// multi-device one (the data-loading path) or gathered out of one.
template <typename Ts, typename Td>
void copy_multi(BaseMatrix<Ts> const& A, BaseMatrix<Td>& B, Options const& opts) {
    auto whole = [](auto const& M) {
        auto st = M.storage();
        return M.op() == Op::NoTrans && M.row0() == 0 && M.col0() == 0 && M.srows() == st->m &&
               M.scols() == st->n && !M.arbitrary_layout() && !st->banded;
    };
    if (A.is_multi_device() && B.is_multi_device()) {
        slate_error_if_msg(A.storage()->group != B.storage()->group,
                           "copy: multi-device matrices on different devices");
        A.storage()->group->run([&](int r, GridPtr const&) {
            TargetScope ts(Target::Devices);
            BaseMatrix<Td> Br = B.on_part(r);
            slate::copy<Ts, Td>(A.on_part(r), Br, opts);
        });
        return;
    }
    if constexpr (std::is_same_v<Ts, Td>) {
        using T = Ts;
        const bool dev = device::available();
        if (B.is_multi_device()) {
            slate_error_if_msg(!whole(A) || !whole(B) || A.grid()->size() != 1 || A.m() != B.m() || A.n() != B.n(),
                               "copy into a multi-device matrix: whole matrices of one process");
            auto const& st = *A.storage();
            const Loc loc = st.has(Loc::Device) && st.state(Loc::Device) != Invalid ? Loc::Device : Loc::Host;
            LocalBlock<T> L = A.local(loc, false);
            if (dev) device::sync_all();
            B.storage()->group->run([&](int r, GridPtr const&) {
                Matrix<T> Br(B.on_part(r));
                scatter_from_host(static_cast<T const*>(L.ptr), L.ld, Br, dev ? Target::Devices : Target::Host);
                Br.storage()->modified(dev ? Loc::Device : Loc::Host);
            });
            return;
        }
        slate_error_if_msg(!whole(A) || !whole(B) || B.grid()->size() != 1 || A.m() != B.m() || A.n() != B.n(),
                           "copy out of a multi-device matrix: whole matrices of one process");
        auto const& st = *B.storage();
        const Loc loc = st.has(Loc::Device) ? Loc::Device : Loc::Host;
        LocalBlock<T> L = B.local(loc, true);
        if (dev) device::sync_all();
        A.storage()->group->run([&](int r, GridPtr const&) {
            Matrix<T> Ar(A.on_part(r));
            gather_to_host(Ar, L.ptr, L.ld);
        });
        internal::finish_origin(B, opts);
    } else {
        slate_error("copy between a multi-device and a one-GPU matrix of different precisions: copy within one "
                    "precision first");
    }
}

/// A's type and meta-data (kind, uplo, diag, bands) on the body's per-rank
/// matrix X (a multi-device part, which already has A's view, or a
/// block-cyclic copy of a whole one-GPU A).
template <typename MT, typename T>
MT rewrap(MT const& A, Matrix<T> const& X) {
    MT r = A;
    static_cast<BaseMatrix<T>&>(r) = static_cast<BaseMatrix<T> const&>(X);
    r.set_uplo(A.uplo());
    r.set_diag(A.diag());
    r.set_kind(A.matrix_kind());
    r.set_band(A.kl(), A.ku());
    return r;
}

/// Caller-side multi-device T factors from each rank's factors.
template <typename T>
std::vector<Matrix<T>> factors_from_parts(std::shared_ptr<InprocGroup> const& grp,
                                          std::vector<std::vector<Matrix<T>>> const& per_rank) {
    std::vector<Matrix<T>> out;
    for (size_t i = 0; i < per_rank[0].size(); ++i) {
        std::vector<Matrix<T>> parts;
        for (auto const& v : per_rank) parts.push_back(v.at(i));
        out.push_back(Matrix<T>::fromParts(grp, parts));
    }
    return out;
}

/// args plus the T factors (inputs) of a QR / LQ application
template <typename T>
std::vector<SpreadArg<T>> with_factors(std::initializer_list<SpreadArg<T>> args, std::vector<Matrix<T>> const& Tf) {
    std::vector<SpreadArg<T>> v(args);
    for (auto const& t : Tf) {
        slate_error_if_msg(!t.is_multi_device(), "QR / LQ factors of a multi-device matrix must come from its "
                                                 "geqrf / gelqf (multi-device T)");
        v.push_back({&t, false});
    }
    return v;
}

/// Group of the multi-device operands among args (nullptr: none).
template <typename T>
std::shared_ptr<InprocGroup> multi_group(std::initializer_list<BaseMatrix<T> const*> args) {
    for (auto* a : args) if (a && a->storage() && a->is_multi_device()) return a->storage()->group;
    return nullptr;
}

}  // namespace internal
}  // namespace slate
