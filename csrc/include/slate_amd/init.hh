// Native process-grid bootstrap for standalone C++ / C / Fortran programs
// (the role MPI_Init + a p x q BLACS-style grid play for the reference,
// test/test.cc:593-599, func::process_2d_grid func.hh:179).
//
// Launch one process per GPU with any launcher that sets the torchrun-style
// environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT), e.g.
//     python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 ./my_prog
// then call slate::init_grid(p, q).  Ranks rendezvous over TCP
// (SLATE_MASTER_PORT, default MASTER_PORT + 17), exchange the RCCL unique id
// and build RCCL world/row/column communicators ("rccl", the default when a
// GPU is visible) or use the native TCP host transport ("tcp": CPU runs,
// SLATE_COMM=host).
#pragma once

#include "grid.hh"

#include <string>

namespace slate {

/// Create the p x q grid over all WORLD_SIZE ranks and install it as the
/// default grid.  p = q = 0 picks the most square p <= q.  transport:
/// "auto", "rccl" or "tcp".  WORLD_SIZE = 1 gives the 1 x 1 self grid.
GridPtr init_grid(int p = 0, int q = 0, GridOrder order = GridOrder::Col, std::string transport = "auto");

/// Barrier, then tear down the default grid (MPI_Finalize analog).
void finalize();

/// The TCP world communicator of this job (created on first use).
CommPtr make_tcp_world(double timeout_s = 120.0);
/// Sub-communicator of a TCP communicator (collective over `parent`).
CommPtr tcp_split(CommPtr const& parent, int color, int key);

int env_world_rank();
int env_world_size();

}  // namespace slate
