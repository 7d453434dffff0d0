"""Process grids and communicators.

One process per GPU.  The p x q process grid gets a world communicator plus
row/column communicators (the rank sets the reference's listBcast derives per
tile, include/slate/BaseMatrix.hh:1999-2212).  Two transports:

* ``rccl``  - native RCCL communicators over xGMI (production, GPU buffers,
  stream-ordered).  Bootstrapped with an RCCL unique id that rank 0 creates
  and torch.distributed (gloo) distributes; subcommunicators via ncclCommSplit.
* ``host``  - torch.distributed (gloo) callbacks on host buffers; device
  buffers are staged through pinned host memory (the reference's
  non-GPU-aware-MPI path).  Used for CPU multi-process tests and for
  multi-rank runs sharing one GPU.
* ``tcp``   - the native C++ socket-mesh transport (csrc/src/tcp_comm.cc,
  no torch needed; the same one standalone C++/C/Fortran programs use
  through slate::init_grid).  Host buffers, staged like ``host``.

``init_grid(p, q)`` returns the Grid and installs it as the default grid.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .. import _slate
from .._core import GridOrder

__all__ = ["init_grid", "TorchHostComm", "world_size", "world_rank", "choose_grid", "self_grid"]


def world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def world_rank() -> int:
    return int(os.environ.get("RANK", "0"))


def self_grid():
    return _slate.Grid.self()


def choose_grid(n: int):
    """Default p x q for n processes: as square as possible with p <= q
    (2x4 for 8, 2x2 for 4, 1x2 for 2)."""
    p = int(np.floor(np.sqrt(n)))
    while n % p:
        p -= 1
    return p, n // p


_DTYPES = {"s": "float32", "d": "float64", "c": "complex64", "z": "complex128",
           "i": "int32", "l": "int64", "b": "uint8"}


def _view(ptr: int, nbytes: int):
    import torch
    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8)
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    return torch.frombuffer(buf, dtype=torch.uint8)


def _typed(ptr: int, count: int, code: str):
    import torch
    t = {"s": torch.float32, "d": torch.float64, "c": torch.float32, "z": torch.float64,
         "i": torch.int32, "l": torch.int64, "b": torch.uint8}[code]
    mult = 2 if code in "cz" else 1
    esize = torch.empty(0, dtype=t).element_size()
    return _view(ptr, count * mult * esize).view(t)


class TorchHostComm(_slate.HostComm):
    """Host communicator over a torch.distributed process group (gloo)."""

    def __init__(self, ranks, group=None):
        super().__init__()
        import torch.distributed as dist
        self._dist = dist
        self._ranks = list(ranks)
        self._group = group
        me = dist.get_rank()
        self._rank = self._ranks.index(me)
        self._pending = None

    def rank(self):
        return self._rank

    def size(self):
        return len(self._ranks)

    def bcast_raw(self, ptr, nbytes, code, root):
        if nbytes == 0:
            return
        self._dist.broadcast(_view(ptr, nbytes), src=self._ranks[root], group=self._group)

    def allreduce_raw(self, ptr, count, code, op):
        if count == 0:
            return
        d = self._dist
        rop = {"s": d.ReduceOp.SUM, "x": d.ReduceOp.MAX, "n": d.ReduceOp.MIN}[op]
        d.all_reduce(_typed(ptr, count, code), op=rop, group=self._group)

    def allgather_raw(self, sptr, rptr, nbytes):
        if nbytes == 0:
            return
        s = _view(sptr, nbytes).clone()
        r = _view(rptr, nbytes * len(self._ranks))
        outs = list(r.view(len(self._ranks), nbytes).unbind(0))
        self._dist.all_gather(outs, s, group=self._group)

    def send_raw(self, ptr, nbytes, peer):
        t = _view(ptr, nbytes)
        if self._pending is not None:
            self._pending.append(self._dist.isend(t, dst=self._ranks[peer], group=self._group))
        else:
            self._dist.send(t, dst=self._ranks[peer], group=self._group)

    def recv_raw(self, ptr, nbytes, peer):
        t = _view(ptr, nbytes)
        if self._pending is not None:
            self._pending.append(self._dist.irecv(t, src=self._ranks[peer], group=self._group))
        else:
            self._dist.recv(t, src=self._ranks[peer], group=self._group)

    def group_start(self):
        self._pending = []

    def group_end(self):
        pend, self._pending = self._pending or [], None
        for w in pend:
            w.wait()

    def barrier(self):
        self._dist.barrier(group=self._group)


_GRID = None
_KEEP = []


def _ensure_dist(backend="gloo"):
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group(backend=backend, rank=world_rank(), world_size=world_size())
    return dist


def init_grid(p: int | None = None, q: int | None = None, order=GridOrder.Col, transport: str = "auto"):
    """Create the p x q process grid over all ranks and make it the default.

    transport: 'auto' (rccl when a GPU is visible and world > 1, else host),
    'rccl', 'host' (torch.distributed/gloo) or 'tcp' (native socket mesh).
    """
    global _GRID
    n = world_size()
    if p is None or q is None:
        p, q = choose_grid(n)
    if p * q != n:
        raise ValueError(f"grid {p}x{q} does not match world size {n}")
    if n == 1:
        _GRID = _slate.Grid.self()
        _slate.set_default_grid(_GRID)
        return _GRID
    if transport == "tcp":
        _GRID = _slate.native_init_grid(p, q, order, "tcp")
        return _GRID
    dist = _ensure_dist("gloo")
    rank = dist.get_rank()
    if order == GridOrder.Col:
        rc = lambda r: (r % p, r // p)
        rank_of = lambda i, j: i + j * p
    else:
        rc = lambda r: (r // q, r % q)
        rank_of = lambda i, j: i * q + j
    myrow, mycol = rc(rank)
    if transport == "auto":
        transport = "rccl" if (_slate.device_available() and os.environ.get("SLATE_COMM", "") != "host") else "host"
    if transport == "rccl":
        uid = [_slate.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        world = _slate.make_rccl_comm(uid[0], n, rank)
        rowc = _slate.rccl_split(world, myrow, mycol)
        colc = _slate.rccl_split(world, p + mycol, myrow)
        # critical-path duplicates (Grid.set_fast): panel / lookahead messages
        # on the panel queue, bulk trailing traffic on the comm queue
        fast = (_slate.rccl_split(world, myrow, mycol), _slate.rccl_split(world, p + mycol, myrow))
    else:
        world = TorchHostComm(list(range(n)), None)
        rowc = colc = None
        # every process creates every group in the same order
        for i in range(p):
            ranks = [rank_of(i, j) for j in range(q)]
            g = dist.new_group(ranks)
            if i == myrow:
                rowc = TorchHostComm(ranks, g)
        for j in range(q):
            ranks = [rank_of(i, j) for i in range(p)]
            g = dist.new_group(ranks)
            if j == mycol:
                colc = TorchHostComm(ranks, g)
    _KEEP.extend([world, rowc, colc])
    _GRID = _slate.Grid(p, q, order, world, rowc, colc)
    if transport == "rccl" and os.environ.get("SLATE_FAST_LANE", "1") != "0":
        _KEEP.extend(fast)
        _GRID.set_fast(*fast)
    _slate.set_default_grid(_GRID)
    return _GRID


def reshape_grid(p: int, q: int, order=GridOrder.Col):
    """Another p x q grid over the SAME processes as the current grid (its
    world communicator; new row / column -- and fast-lane -- communicators
    split from it).  Every rank must call it, in the same order.  Used to
    run each routine on its best grid shape in one job (bench.py)."""
    g = current_grid()
    n = world_size()
    if p * q != n:
        raise ValueError(f"grid {p}x{q} does not match world size {n}")
    if n == 1 or (g.p == p and g.q == q and g.order == order):
        return g
    world = g.world
    rank = world.rank()
    myrow, mycol = (rank % p, rank // p) if order == GridOrder.Col else (rank // q, rank % q)
    if world.name() == "rccl":
        rowc = _slate.rccl_split(world, myrow, mycol)
        colc = _slate.rccl_split(world, p + mycol, myrow)
        grid = _slate.Grid(p, q, order, world, rowc, colc)
        _KEEP.extend([rowc, colc])
        if os.environ.get("SLATE_FAST_LANE", "1") != "0":
            fast = (_slate.rccl_split(world, myrow, mycol), _slate.rccl_split(world, p + mycol, myrow))
            _KEEP.extend(fast)
            grid.set_fast(*fast)
        return grid
    if world.name() == "tcp":
        rowc = _slate.tcp_split(world, myrow, mycol)
        colc = _slate.tcp_split(world, p + mycol, myrow)
        _KEEP.extend([rowc, colc])
        return _slate.Grid(p, q, order, world, rowc, colc)
    import torch.distributed as dist
    rank_of = (lambda i, j: i + j * p) if order == GridOrder.Col else (lambda i, j: i * q + j)
    rowc = colc = None
    for i in range(p):
        ranks = [rank_of(i, j) for j in range(q)]
        gg = dist.new_group(ranks)
        if i == myrow:
            rowc = TorchHostComm(ranks, gg)
    for j in range(q):
        ranks = [rank_of(i, j) for i in range(p)]
        gg = dist.new_group(ranks)
        if j == mycol:
            colc = TorchHostComm(ranks, gg)
    _KEEP.extend([rowc, colc])
    return _slate.Grid(p, q, order, world, rowc, colc)


def finalize():
    """Tear down the grid and the torch.distributed process group (the
    reference's MPI_Finalize point).  Call before exit in multi-process runs:
    destroying gloo groups during interpreter shutdown can abort."""
    global _GRID
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        _slate.native_finalize()
        _GRID = None
        _KEEP.clear()
        return
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
    _slate.set_default_grid(_slate.Grid.self())
    _GRID = None
    _KEEP.clear()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def current_grid():
    return _GRID if _GRID is not None else _slate.default_grid()
