// Shared helpers of the C++ examples (reference examples/util.hh).
// Every example runs on 1 process, or on N processes with a torchrun-style
// launcher:  python -m torch.distributed.run --nproc-per-node 4 \
//                --master-addr 127.0.0.1 build/examples/ex05_blas
// Target: SLATE_TARGET=d|h (default: the GPU when one is visible).
#pragma once

#include "slate_amd/slate.hh"
#include "slate_amd/inproc.hh"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>

namespace ex {

inline slate::Target target() {
    const char* e = std::getenv("SLATE_TARGET");
    if (e && (e[0] == 'h' || e[0] == 'H')) return slate::Target::HostTask;
    if (e && (e[0] == 'd' || e[0] == 'D')) return slate::Target::Devices;
    return slate::device::available() ? slate::Target::Devices : slate::Target::HostTask;
}

inline slate::Options opts() { return {{slate::Option::Target, target()}}; }

/// Deterministic, distribution-independent random fill of a distributed
/// matrix (the counter-based matgen: same values for any p x q).
template <typename T>
void random_fill(slate::Matrix<T>& A, uint64_t seed) {
    A.insertLocalTiles(target());
    slate::BaseMatrix<T>& B = A;
    slate::generate_matrix(std::string("rand"), B, seed, -1, opts());
}

inline int rank() { return slate::default_grid()->rank(); }

inline void banner(const char* name) {
    if (rank() == 0)
        std::printf("== %s: slate %s, %d process(es), target %s\n", name, slate::version(),
                    slate::default_grid()->size(), target() == slate::Target::Devices ? "devices" : "host");
}

/// Print PASS/FAIL on rank 0 and accumulate the exit status.
inline int check(const char* what, double err, double tol) {
    bool ok = std::isfinite(err) && err <= tol;
    if (rank() == 0) std::printf("  %-44s error %.2e  %s\n", what, err, ok ? "pass" : "FAILED");
    return ok ? 0 : 1;
}

/// ||B - A X||_1 / (n ||A||_1 ||X||_1) with A, X, B distributed (reference
/// test_gesv.cc residual).
template <typename T>
double solve_residual(slate::Matrix<T> const& A, slate::Matrix<T> const& X, slate::Matrix<T> const& B) {
    auto o = opts();
    slate::Matrix<T> R = B.emptyLike();
    R.insertLocalTiles(target());
    slate::copy<T, T>(B, R, o);
    slate::gemm(T(-1), A, X, T(1), R, o);
    double rn = slate::norm(slate::Norm::One, R, o);
    double an = slate::norm(slate::Norm::One, A, o), xn = slate::norm(slate::Norm::One, X, o);
    return rn / (double(A.n()) * an * xn);
}

template <typename T>
slate::Matrix<T> copy_of(slate::Matrix<T> const& A) {
    slate::Matrix<T> C = A.emptyLike();
    C.insertLocalTiles(target());
    slate::copy<T, T>(A, C, opts());
    return C;
}

inline int finish(int fails) {
    int total = int(slate::default_grid()->world().allreduce_scalar<int32_t>(fails, slate::ReduceOp::Sum));
    // drivers that ran on in-process ranks (one process, several GPUs: spread.hh)
    if (rank() == 0 && slate::inproc_run_count() > 0) {
        int p = 0, q = 0;
        slate::inproc_last_shape(p, q);
        std::printf("  in-process multi-GPU driver runs: %lld (last grid %d x %d)\n",
                    (long long)slate::inproc_run_count(), p, q);
    }
    if (rank() == 0) std::printf("  %s\n", total ? "FAILED" : "all passed");
    slate::finalize();
    return total ? 1 : 0;
}

}  // namespace ex
