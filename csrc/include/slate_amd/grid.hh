// Process grid: p x q processes, one GPU each, with row and column
// communicators.  Reference: the p x q MPI grid of func::process_2d_grid
// (func.hh:179) plus the implicit row/column rank sets used by listBcast.
#pragma once

#include "comm.hh"

#include <memory>

namespace slate {

class Grid {
public:
    /// world: all p*q ranks; row: my process row (size q, rank = my column);
    /// col: my process column (size p, rank = my row).
    Grid(int p, int q, GridOrder order, CommPtr world, CommPtr row, CommPtr col);

    /// 1 x 1 grid on a SelfComm.
    static std::shared_ptr<Grid> self();

    int p() const { return p_; }
    int q() const { return q_; }
    GridOrder order() const { return order_; }
    int rank() const { return world_->rank(); }
    int size() const { return p_ * q_; }
    int myrow() const { return myrow_; }
    int mycol() const { return mycol_; }

    /// world rank of process (r, c)
    int rank_of(int r, int c) const {
        return order_ == GridOrder::Col ? r + c * p_ : r * q_ + c;
    }
    int row_of(int rank) const { return order_ == GridOrder::Col ? rank % p_ : rank / q_; }
    int col_of(int rank) const { return order_ == GridOrder::Col ? rank / p_ : rank % q_; }

    Comm& world() const { return *world_; }
    Comm& row()   const { return *row_; }
    Comm& col()   const { return *col_; }
    CommPtr world_ptr() const { return world_; }
    CommPtr row_ptr() const { return row_; }
    CommPtr col_ptr() const { return col_; }

    /// Critical-path ("fast lane") row / column communicators: duplicates of
    /// row() / col() over the same processes (a second ncclCommSplit for RCCL).
    /// Panel, tournament, TSQR and lookahead messages travel on these, issued
    /// on the high-priority panel queue, so they never wait behind the bulk
    /// trailing-update traffic that the plain comms carry on the comm queue
    /// (the reference gives panel / lookahead tasks priority 1 and the
    /// trailing update priority 0, src/getrf.cc:92,124,175-186).  Without
    /// duplicates (host transports, which are synchronous anyway) they alias
    /// row() / col().
    Comm& row_fast() const { return *(row_fast_ ? row_fast_ : row_); }
    Comm& col_fast() const { return *(col_fast_ ? col_fast_ : col_); }
    CommPtr row_fast_ptr() const { return row_fast_ ? row_fast_ : row_; }
    CommPtr col_fast_ptr() const { return col_fast_ ? col_fast_ : col_; }
    bool has_fast_lane() const { return row_fast_ != nullptr || col_fast_ != nullptr; }
    void set_fast(CommPtr row_fast, CommPtr col_fast) { row_fast_ = row_fast; col_fast_ = col_fast; }

    /// The same processes viewed as a q x p grid (tile (i,j) of a matrix on
    /// the transposed grid lives where tile (j,i) lives on this grid);
    /// reference func::transpose_grid (func.hh:230).
    std::shared_ptr<Grid> transposed() const;

    bool same_processes(Grid const& o) const { return world_.get() == o.world_.get(); }

private:
    int p_, q_;
    GridOrder order_;
    int myrow_, mycol_;
    CommPtr world_, row_, col_;
    CommPtr row_fast_, col_fast_;
};

using GridPtr = std::shared_ptr<Grid>;

/// Default grid for new matrices when none is given (1 x 1 self unless the
/// embedding runtime installed one).  A thread may override it for itself
/// (in-process ranks: each rank thread sees its own grid).
GridPtr default_grid();
void set_default_grid(GridPtr g);
void set_thread_default_grid(GridPtr g);   // nullptr: back to the process default

/// p x q grid of in-process ranks (thread_comm.cc): one Grid per rank, world
/// rank r = element r.  `devices` (one entry per rank, may repeat) selects
/// device mode and enables peer access between them; empty = host mode.
std::vector<GridPtr> make_thread_grids(int p, int q, GridOrder order, std::vector<int> const& devices);
/// Abort every in-process communicator of g (see thread_comm_abort).
void thread_grid_abort(Grid const& g);
/// Clear the aborted state of g's in-process communicators (all of the
/// group's rank threads have stopped), so a persistent group runs again.
void thread_grid_reset(Grid const& g);

}  // namespace slate
