"""Core Python layer: dtype dispatch and matrix helpers over the native
library (``_slate``).  Mirrors the reference's C++ API surface
(include/slate/slate.hh) with Pythonic wrappers; all heavy lifting is in
C++/HIP.
"""
from __future__ import annotations

import os
import numpy as np

from . import _slate

Target = _slate.Target
Op = _slate.Op
Uplo = _slate.Uplo
Job = _slate.Job
Diag = _slate.Diag
Side = _slate.Side
Norm = _slate.Norm
GridOrder = _slate.GridOrder
Layout = _slate.Layout
Equed = _slate.Equed
Grid = _slate.Grid

_SUFFIX = {
    np.dtype(np.float32): "s",
    np.dtype(np.float64): "d",
    np.dtype(np.complex64): "c",
    np.dtype(np.complex128): "z",
}
_DTYPE = {v: k for k, v in _SUFFIX.items()}


def suffix_of(obj) -> str:
    """Precision suffix ('s','d','c','z') of a native matrix object or dtype."""
    if isinstance(obj, str):
        return obj
    try:
        return _SUFFIX[np.dtype(obj)]
    except TypeError:
        pass
    name = type(obj).__name__
    return name.rsplit("_", 1)[-1]


def dtype_of(obj) -> np.dtype:
    return _DTYPE[suffix_of(obj)]


def native(name: str, obj):
    """The native function `name_<suffix>` for a matrix object."""
    return getattr(_slate, f"{name}_{suffix_of(obj)}")


def _cls(kind: str, dtype):
    return getattr(_slate, f"{kind}_{suffix_of(dtype)}")


def target_of(t) -> Target:
    if t is None:
        return Target.Devices if (os.environ.get("SLATE_TARGET", "").lower() in ("d", "devices")) else Target.HostTask
    if isinstance(t, Target):
        return t
    return {"h": Target.Host, "host": Target.Host, "t": Target.HostTask, "task": Target.HostTask,
            "n": Target.HostNest, "b": Target.HostBatch, "d": Target.Devices,
            "dev": Target.Devices, "devices": Target.Devices}[str(t).lower()]


def opts(target=None, **kw) -> dict:
    o = dict(kw)
    if target is not None:
        o["target"] = target_of(target)
    return o


# ---------------------------------------------------------------- matrices
def Matrix(m, n, nb=256, dtype=np.float64, grid=None, mb=None):
    """Distributed m x n matrix with mb x nb tiles on `grid` (no storage yet)."""
    return _cls("Matrix", dtype)(int(m), int(n), int(mb or nb), int(nb), grid)


def HermitianMatrix(uplo, A):
    return _cls("HermitianMatrix", A)(uplo, A)


def SymmetricMatrix(uplo, A):
    return _cls("SymmetricMatrix", A)(uplo, A)


def TriangularMatrix(uplo, diag, A):
    return _cls("TriangularMatrix", A)(uplo, diag, A)


def TrapezoidMatrix(uplo, diag, A):
    return _cls("TrapezoidMatrix", A)(uplo, diag, A)


def BandMatrix(kl, ku, A):
    return _cls("BandMatrix", A)(kl, ku, A)


def band_matrix(m, n, kl, ku, nb, dtype=np.float64, grid=None, target=None):
    """Band matrix with band-only storage (only the tiles that intersect the
    band plus gbtrf's fill are allocated: O(n * (2 kl + ku)) memory)."""
    B = getattr(_slate, f"BandMatrix_{_SUFFIX[np.dtype(dtype)]}").banded(m, n, kl, ku, nb, grid)
    B.insertLocalTiles(target_of(target) if target is not None else Target.Host)
    return B


def hermitian_band_matrix(uplo, n, kd, nb, dtype=np.float64, grid=None, target=None):
    """Hermitian band matrix with band-only storage."""
    B = getattr(_slate, f"HermitianBandMatrix_{_SUFFIX[np.dtype(dtype)]}").banded(uplo, n, kd, nb, grid)
    B.insertLocalTiles(target_of(target) if target is not None else Target.Host)
    return B


def TriangularBandMatrix(uplo, diag, kd, A):
    return _cls("TriangularBandMatrix", A)(uplo, diag, kd, A)


def HermitianBandMatrix(uplo, kd, A):
    return _cls("HermitianBandMatrix", A)(uplo, kd, A)


def general(A):
    """General Matrix view of any matrix object (drops uplo/diag meta)."""
    return _cls("Matrix", A)(A)


def from_numpy(full: np.ndarray, nb=256, grid=None, target=None, dtype=None, mb=None):
    """Distribute a full (replicated) numpy array: each rank keeps its local
    tiles.  Storage is allocated at the target's location."""
    full = np.asarray(full)
    if dtype is None:
        dtype = full.dtype if full.dtype in _SUFFIX else np.float64
    full = full.astype(dtype, copy=False)
    if full.ndim == 1:
        full = full.reshape(-1, 1)
    m, n = full.shape
    A = Matrix(m, n, nb, dtype, grid, mb=mb)
    A.insertLocalTiles(Target.Host)
    rows = A.local_row_indices()
    cols = A.local_col_indices()
    if len(rows) and len(cols):
        A.set_local(np.asfortranarray(full[np.ix_(rows, cols)]))
    if target_of(target) == Target.Devices:
        A.insertLocalTiles(Target.Devices)
    return A


def matrix_layout(m, n, tile_mb, tile_nb, tile_rank, dtype=np.float64, grid=None, target=None):
    """Matrix with an arbitrary distribution and non-uniform tiles (reference
    Matrix(m, n, tileMb, tileNb, tileRank, tileDevice, comm)): tile_mb(i) /
    tile_nb(j) give tile sizes (or lists), tile_rank(i, j) the owning world
    rank (or an mt x nt list).  Drivers run on a block-cyclic copy."""
    def sizes(f, total):
        out, acc = [], 0
        while acc < total:
            b = int(f[len(out)] if not callable(f) else f(len(out)))
            out.append(b)
            acc += b
        return out
    rs, cs = sizes(tile_mb, m), sizes(tile_nb, n)
    own = tile_rank if not callable(tile_rank) else [[int(tile_rank(i, j)) for j in range(len(cs))]
                                                     for i in range(len(rs))]
    cls = getattr(_slate, "Matrix_" + _SUFFIX[np.dtype(dtype)])
    A = cls.with_layout(m, n, rs, cs, own, grid)
    A.insertLocalTiles(target_of(target) if target is not None else Target.Host)
    return A


def multi_device(m, n, nb=256, dtype=np.float64, num_devices=0, mb=None):
    """New multi-device matrix: 2-D block-cyclic over num_devices in-process
    ranks of this process (0: every GPU it may use; 8 GPUs -> 2 x 4), storage
    on the devices.  Drivers called with it run on those GPUs in place
    (reference: one MPI rank spreads its tiles over all of its GPUs,
    MatrixStorage.hh:503-506)."""
    cls = getattr(_slate, "Matrix_" + _SUFFIX[np.dtype(dtype)])
    return cls.multiDevice(m, n, mb or nb, nb, num_devices)


def to_multi_device(full: np.ndarray, nb=256, num_devices=0, dtype=None):
    """Copy a numpy array into a new multi-device matrix (one scatter)."""
    full = np.asarray(full)
    if dtype is None:
        dtype = full.dtype if full.dtype in _SUFFIX else np.float64
    full = np.asfortranarray(full.astype(dtype, copy=False))
    if full.ndim == 1:
        full = full.reshape(-1, 1)
    m, n = full.shape
    src = Matrix(m, n, nb, dtype, _slate.Grid.self())
    src.insertLocalTiles(Target.Host)
    src.set_local(full)
    A = multi_device(m, n, nb, dtype, num_devices)
    native("copy", A)(src, A, opts())
    return A


def from_devices(m, n, ptrs, lda, nb, dtype=np.float64, mb=None):
    """Reference fromDevices(m, n, Aarray, num_devices, lda, mb, nb): one
    device pointer per GPU, tile column j on device j % len(ptrs)."""
    cls = getattr(_slate, "Matrix_" + _SUFFIX[np.dtype(dtype)])
    return cls.fromDevicesArray(m, n, [int(p) for p in ptrs], lda, mb or nb, nb)


def to_numpy(A) -> np.ndarray:
    """Gather a distributed matrix (logical view) to a full numpy array on every rank."""
    return A.gather()


def empty_like(A, target=None):
    B = _cls("Matrix", A)(A).emptyLike()
    B.insertLocalTiles(target_of(target) if target is not None else Target.Host)
    return B


def local_tensor(A, device=True):
    """Zero-copy torch view of this rank's local block (column-major)."""
    import torch
    return torch.utils.dlpack.from_dlpack(A.local_dlpack(device))


def transpose(A):
    return A.transpose()


def conj_transpose(A):
    return A.conj_transpose()


def version() -> str:
    return _slate.version()
