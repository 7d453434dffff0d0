"""Debug utilities (reference src/auxiliary/Debug.hh:18-75): tile maps with
MOSI states, tile liveness / layout checks, LAPACK-matrix tile diffs and the
device allocator's block report.  All of it runs in libslate_amd
(csrc/src/debug.cc); Debug.on() (or SLATE_DEBUG=1) also echoes the reports."""
import numpy as np

from .. import _slate
from .._core import suffix_of


def on():
    _slate.debug_on()


def off():
    _slate.debug_off()


def enabled():
    return _slate.debug_enabled()


def print_tiles(A):
    """Per-tile map: owner rank and host/device MOSI letters of local tiles."""
    return getattr(_slate, "debug_print_tiles_" + suffix_of(A))(A)


def check_tiles_lives(A):
    """Number of local tiles without a live, valid instance (0 = healthy)."""
    return getattr(_slate, "debug_check_tiles_lives_" + suffix_of(A))(A)


def check_tiles_layout(A):
    return getattr(_slate, "debug_check_tiles_layout_" + suffix_of(A))(A)


_SUF = {np.dtype(np.float32): "s", np.dtype(np.float64): "d",
        np.dtype(np.complex64): "c", np.dtype(np.complex128): "z"}


def diff_lapack_matrices(A, B, mb, nb, tol=0.0):
    """(number of differing tiles, tile map) of two column-major arrays."""
    A = np.asfortranarray(A)
    B = np.asfortranarray(B, dtype=A.dtype)
    return getattr(_slate, "debug_diff_lapack_" + _SUF[A.dtype])(A, B, mb, nb, tol)


def mem_report():
    """Device allocator blocks / bytes in use and cached (printNumFreeMemBlocks)."""
    return _slate.debug_mem_report()


def device_memory_leaks():
    return _slate.debug_device_leaks()


def host_memory_leaks():
    return _slate.debug_host_leaks()
