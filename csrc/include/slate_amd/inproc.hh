// Intra-process multi-GPU: one process drives every GPU of the node.
//
// Reference: an MPI rank spreads its tiles over all of its GPUs
// (tileDevice = func::device_1d_grid, include/slate/internal/
// MatrixStorage.hh:503-511) and its LAPACK shim switches to the device
// target when GPUs exist (lapack_api/lapack_slate.hh).  Here every GPU is a
// rank of the ordinary p x q machinery: run_in_process starts one thread per
// rank, binds it to its own device context (streams, events, allocator) and
// an in-process communicator (thread_comm.cc: peer copies over xGMI ordered
// by events), and runs the same driver code as a one-process-per-GPU job.
#pragma once

#include "matrix.hh"
#include "grid.hh"

#include <functional>
#include <vector>

namespace slate {

/// A persistent p x q group of in-process ranks: the rank threads' grids and
/// communicators (thread_comm.cc) are made once and reused by every run, so
/// matrices whose storage lives on the group's devices (multi-device
/// matrices, MatrixStorage::parts) keep valid grids from one driver call to
/// the next.  Groups are cached per (p, q, order, devices).
class InprocGroup {
public:
    /// the cached group of p x q ranks (devices: one per rank, default r % device count)
    static std::shared_ptr<InprocGroup> get(int p, int q, std::vector<int> devices = {},
                                            GridOrder order = GridOrder::Col);
    /// the group of n ranks on the first n devices with the near-square
    /// shape of inproc_grid_shape (n = 0: inproc_ranks())
    static std::shared_ptr<InprocGroup> of_size(int n = 0);
    int p() const { return p_; }
    int q() const { return q_; }
    int size() const { return p_ * q_; }
    GridOrder order() const { return order_; }
    GridPtr const& grid(int rank) const { return grids_[rank]; }
    /// device of rank r (-1 in host mode)
    int device(int rank) const { return devices_.empty() ? -1 : devices_[rank]; }
    /// fn(rank, grid) on every rank thread (serialized with run_in_process)
    void run(std::function<void(int, GridPtr const&)> const& fn);

    InprocGroup(int p, int q, GridOrder order, std::vector<int> devices);
private:
    int p_, q_;
    GridOrder order_;
    std::vector<int> devices_;
    std::vector<GridPtr> grids_;
};
using InprocGroupPtr = std::shared_ptr<InprocGroup>;

/// Bytes the single-process paths copied between a caller's operand and the
/// in-process ranks (scatter_from_host + gather_to_host): zero for drivers
/// called on multi-device matrices (tests pin that no re-scatter happens).
int64_t inproc_copy_bytes();

/// Run fn(rank, grid) on p*q in-process ranks (threads; rank r on device
/// devices[r], default r % device count; host mode when no GPU is visible).
/// Each thread sees `grid` as its default grid.  The first exception of any
/// rank is rethrown after every thread has stopped (the others are woken by
/// aborting their communicators).  Calls are serialized.
void run_in_process(int p, int q, std::function<void(int, GridPtr const&)> const& fn,
                    std::vector<int> devices = {}, GridOrder order = GridOrder::Col);

/// Number of run_in_process calls so far (tests: did a call take the
/// in-process multi-rank path?) and the grid shape of the last one.
int64_t inproc_run_count();
void inproc_last_shape(int& p, int& q);

/// Ranks the single-process APIs (LAPACK-compatible shim, and the drivers
/// called on a 1 x 1 grid) spread work over: $SLATE_INPROC_RANKS if set;
/// else 1 in a multi-process job (WORLD_SIZE / LOCAL_RANK / MPI / Slurm
/// environment), after set_device, or with a > 1-rank default grid; else
/// the number of visible GPUs (1 without).
int inproc_ranks();
/// True when the environment shows a launcher started several processes.
bool multi_process_job();
/// Is the calling thread one of run_in_process's rank threads?
bool in_inproc_rank();
/// Near-square p x q with p <= q for n ranks (1x1, 1x2, 2x2, 2x4, ...).
void inproc_grid_shape(int n, int& p, int& q);

/// Copy this rank's tiles of M from / to a global column-major array A (lda)
/// that every in-process rank can read (scatter) or write (gather, disjoint
/// tiles): the data path of the single-process APIs.
template <typename T>
void scatter_from_host(T const* A, int64_t lda, Matrix<T>& M, Target target);
template <typename T>
void gather_to_host(Matrix<T>& M, T* A, int64_t lda);

}  // namespace slate
