"""slate_d35_amd: an MI355X-native distributed dense linear-algebra framework
with the capabilities of SLATE (liamscarlett/slate-d35).

Native core (C++ runtime + gfx950 HIP kernels + RCCL) in ``_slate``;
this package adds dtype dispatch, grid bootstrap and torch interop.

    import slate_d35_amd as slate
    grid = slate.init_grid()                 # p x q over torchrun ranks (1x1 alone)
    A = slate.from_numpy(a, nb=512, target="d")
    info = slate.potrf(slate.HermitianMatrix(slate.Uplo.Lower, A), target="d")
"""
try:
    # Load torch's HIP runtime first: its libamdhip64/librccl carry the same
    # SONAMEs as the system ROCm ones, so the native library then binds to
    # the already-loaded copies and the process has ONE HIP runtime.
    import torch as _torch  # noqa: F401
except Exception:  # torch is optional for the native library
    _torch = None
from . import _slate
from ._core import (Target, Op, Uplo, Diag, Side, Norm, GridOrder, Layout, Equed, Grid, Job,  # noqa: F401
                    Matrix, HermitianMatrix, SymmetricMatrix, TriangularMatrix, TrapezoidMatrix,
                    BandMatrix, TriangularBandMatrix, HermitianBandMatrix, general, band_matrix,
                    hermitian_band_matrix,
                    from_numpy, to_numpy, multi_device, to_multi_device, from_devices, matrix_layout, empty_like, local_tensor, transpose, conj_transpose,
                    version, suffix_of, dtype_of, opts, target_of)
from .parallel import init_grid, choose_grid, TorchHostComm, current_grid, finalize  # noqa: F401
from .models import *  # noqa: F401,F403
from . import utils  # noqa: F401
from . import ops  # noqa: F401

trace = _slate.trace
sync = _slate.sync
timers = _slate.timers
device_available = _slate.device_available

__version__ = _slate.version()
