"""Direct access to the gfx950 kernels on torch tensors (single process).

These bypass the distributed matrix classes and call the local BLAS layer
(csrc/src/local_blas.cc) on device pointers; used by kernel numerics tests
and micro-benchmarks.  Tensors are interpreted column-major: pass the
transpose of a row-major torch tensor, or use the helpers below which take
care of layout.
"""
from __future__ import annotations

from .. import _slate

__all__ = ["have_native_ops", "gemm", "gemm_async", "herk", "trsm", "potrf", "getrf_panel", "geqrf_panel", "lu_sign",
           "set_queue", "queue_sync"]


def set_queue(q: int):
    """HIP queue of the calls below (0 default; 1 = the high-priority panel queue)."""
    _slate.set_ops_queue(q)


def queue_sync(q: int):
    _slate.queue_sync(q)


def have_native_ops() -> bool:
    return hasattr(_slate, "lb_gemm_d")


def _suffix(t):
    import torch
    return {torch.float32: "s", torch.float64: "d", torch.complex64: "c", torch.complex128: "z"}[t.dtype]


def _cm(t):
    """(ptr, m, n, ld) of a torch tensor viewed as a column-major matrix:
    a row-major (n x m) contiguous tensor is an m x n column-major matrix.
    Synchronizes torch's stream first: the native kernels run on the
    framework's own HIP queues."""
    import torch
    assert t.dim() == 2 and t.stride(1) == 1, "row-major contiguous rows expected"
    if t.is_cuda:
        # torch's own stream only: a device-wide synchronize would also wait
        # for work queued on the framework's queues (e.g. gemm_async)
        torch.cuda.current_stream(t.device).synchronize()
    return t.data_ptr(), t.shape[1], t.shape[0], t.stride(0)


def gemm(opA: str, opB: str, alpha, A, B, beta, C):
    """Column-major C = alpha op(A) op(B) + beta C on the device, where a
    row-major torch tensor X (r x c) represents the column-major c x r matrix X^T."""
    fn = getattr(_slate, f"lb_gemm_{_suffix(C)}")
    pa, ma, na, lda = _cm(A)
    pb, mb, nb, ldb = _cm(B)
    pc, mc, nc, ldc = _cm(C)
    k = na if opA == "N" else ma
    fn(opA, opB, mc, nc, k, alpha, pa, lda, pb, ldb, beta, pc, ldc)


def gemm_async(queue: int, opA: str, opB: str, alpha, A, B, beta, C):
    """gemm launched on `queue` without waiting for it (queue_sync(queue))."""
    fn = getattr(_slate, f"lb_gemm_async_{_suffix(C)}")
    pa, ma, na, lda = _cm(A)
    pb, mb, nb, ldb = _cm(B)
    pc, mc, nc, ldc = _cm(C)
    k = na if opA == "N" else ma
    fn(queue, opA, opB, mc, nc, k, alpha, pa, lda, pb, ldb, beta, pc, ldc)


def herk(uplo: str, op: str, alpha, A, beta, C):
    fn = getattr(_slate, f"lb_herk_{_suffix(C)}")
    pa, ma, na, lda = _cm(A)
    pc, n, _, ldc = _cm(C)
    k = na if op == "N" else ma
    fn(uplo, op, n, k, alpha, pa, lda, beta, pc, ldc)


def trsm(side: str, uplo: str, op: str, diag: str, alpha, A, B):
    fn = getattr(_slate, f"lb_trsm_{_suffix(B)}")
    pa, _, _, lda = _cm(A)
    pb, m, n, ldb = _cm(B)
    fn(side, uplo, op, diag, m, n, alpha, pa, lda, pb, ldb)


def potrf(uplo: str, A):
    fn = getattr(_slate, f"lb_potrf_{_suffix(A)}")
    pa, n, _, lda = _cm(A)
    return fn(uplo, n, pa, lda)


def getrf_panel(A, tournament: bool = False):
    """LU of a column-major m x n panel; returns (info, ipiv).  Partial pivoting
    per column, or tournament (CALU) pivoting per 32-column block."""
    fn = getattr(_slate, f"lb_getrf_panel_{_suffix(A)}")
    pa, m, n, lda = _cm(A)
    return fn(m, n, pa, lda, tournament)


def geqrf_panel(A):
    """Householder QR of a column-major m x n panel; returns (tau, T) as torch tensors."""
    fn = getattr(_slate, f"lb_geqrf_panel_{_suffix(A)}")
    pa, m, n, lda = _cm(A)
    return fn(m, n, pa, lda)


def lu_sign(A):
    """Sign-modified LU without pivoting of a column-major n x n block in
    place (the Householder reconstruction step of the CholeskyQR / TSQR QR
    panels, lu_dist.cc): L U = A + diag(s), s_k = the unit phase of the k-th
    pivot; returns s."""
    fn = getattr(_slate, f"lb_lu_sign_{_suffix(A)}")
    pa, m, n, lda = _cm(A)
    return fn(n, pa, lda)
