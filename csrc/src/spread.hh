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
    if (!on || in_inproc_rank()) return false;
    if (get_target(opts, Target::HostTask) != Target::Devices || !device::available()) return false;
    return inproc_ranks() > 1;
}

/// Runs body(copies, rank) on inproc_ranks() in-process ranks; false (the
/// caller takes its one-GPU path) unless every argument is a full,
/// non-transposed, block-cyclic view with square tiles on a 1 x 1 grid and
/// the first argument has at least kSpreadMinN rows and a tile row per rank.
template <typename T>
bool spread(Options const& opts, std::vector<SpreadArg<T>> const& args,
            std::function<void(std::vector<Matrix<T>>&, int)> const& body) {
    if (args.empty() || !spread_allowed(opts)) return false;
    for (auto const& a : args) {
        auto const& M = *a.M;
        auto st = M.storage();
        if (!st || M.arbitrary_layout() || M.grid()->size() != 1 || M.op() != Op::NoTrans || M.row0() != 0 ||
            M.col0() != 0 || M.srows() != st->m || M.scols() != st->n || M.mb() != M.nb())
            return false;
    }
    const int nr = inproc_ranks();
    auto const& A0 = *args[0].M;
    static const int64_t min_n = [] {
        const char* e = std::getenv("SLATE_SPREAD_MIN_N");
        return e ? std::atoll(e) : kSpreadMinN;
    }();
    if (A0.m() < min_n || (A0.m() + A0.nb() - 1) / A0.nb() < nr) return false;
    int p, q;
    inproc_grid_shape(nr, p, q);
    // the caller's operands: where each one is valid (its device, else host)
    struct Src { T* ptr; int64_t ld; };
    std::vector<Src> src;
    for (auto const& a : args) {
        auto const& st = *a.M->storage();
        const Loc loc = st.has(Loc::Device) && st.state(Loc::Device) != Invalid ? Loc::Device : Loc::Host;
        LocalBlock<T> L = a.M->local(loc, a.out);   // for outputs: the other instance goes stale
        src.push_back({L.ptr, L.ld});
    }
    device::sync_all();   // the caller's queued work on its operands is done
    run_in_process(p, q, [&](int rank, GridPtr const& g) {
        std::vector<Matrix<T>> X;
        for (size_t i = 0; i < args.size(); ++i) {
            auto const& M = *args[i].M;
            Matrix<T> C(M.m(), M.n(), M.nb(), g);
            C.insertLocalTiles(Target::Devices);
            scatter_from_host(static_cast<T const*>(src[i].ptr), src[i].ld, C, Target::Devices);
            X.push_back(C);
        }
        body(X, rank);
        for (size_t i = 0; i < args.size(); ++i)
            if (args[i].out) gather_to_host(X[i], src[i].ptr, src[i].ld);
    });
    return true;
}

}  // namespace internal
}  // namespace slate
