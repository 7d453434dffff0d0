"""Test-matrix generation (reference matgen/generate_matrix_*.cc).

Values come from a counter-based generator keyed by (global i, global j,
seed), so a matrix is identical for any process grid (reference
matgen/random.cc:53-110 uses Philox-2x64 for the same property).  The
native generator (`generate_matrix` in C++) fills local tiles directly on
the device; this module holds the host reference and kind dispatch."""
from __future__ import annotations

import numpy as np

__all__ = ["random_matrix", "spd_matrix", "diag_dominant_matrix", "generate", "KINDS"]

KINDS = ["rand", "rands", "randn", "randb", "randr", "zeros", "identity", "ij", "jordan", "diag",
         "poev", "heev", "spd", "diag_dominant", "orthog", "riemann", "kms", "fiedler", "circul", "chebspec"]


def _hash(i, j, seed):
    # SplitMix64 of a (i, j, seed) key: grid-independent element values
    x = (np.asarray(i, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
         ^ (np.asarray(j, dtype=np.uint64) + np.uint64(0x632BE59BD9B4E019)) * np.uint64(0xD1B54A32D192ED03)
         ^ np.uint64(seed) * np.uint64(0x94D049BB133111EB))
    x = x ^ (x >> np.uint64(30)); x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27)); x = x * np.uint64(0x94D049BB133111EB)
    x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(11)).astype(np.float64) / float(1 << 53)


def random_matrix(m, n, seed=42, dtype=np.float64, kind="rands"):
    with np.errstate(over="ignore"):
        i, j = np.meshgrid(np.arange(m, dtype=np.uint64), np.arange(n, dtype=np.uint64), indexing="ij")
        u = _hash(i, j, seed)
        if np.issubdtype(np.dtype(dtype), np.complexfloating):
            v = _hash(i, j, seed + 7919)
    if kind == "rand":
        a = u
    elif kind == "randn":
        u2 = _hash(i, j, seed + 104729)
        a = np.sqrt(-2 * np.log(np.maximum(u, 1e-300))) * np.cos(2 * np.pi * u2)
    elif kind == "randb":
        a = (u > 0.5).astype(np.float64)
    elif kind == "randr":
        a = np.where(u > 0.5, 1.0, -1.0)
    else:
        a = 2 * u - 1
    if np.issubdtype(np.dtype(dtype), np.complexfloating):
        a = a + 1j * (2 * v - 1)
    return a.astype(dtype)


def spd_matrix(n, seed=42, dtype=np.float64):
    """Hermitian positive definite: random symmetric + n*I (reference 'rands' + diag shift)."""
    a = random_matrix(n, n, seed, dtype)
    a = (a + a.conj().T) / 2
    a += n * np.eye(n, dtype=dtype)
    return a


def diag_dominant_matrix(n, seed=42, dtype=np.float64):
    a = random_matrix(n, n, seed, dtype)
    a += n * np.eye(n, dtype=dtype)
    return a


def generate(kind, m, n=None, seed=42, dtype=np.float64, cond=None):
    n = m if n is None else n
    if kind in ("rand", "rands", "randn", "randb", "randr"):
        return random_matrix(m, n, seed, dtype, kind)
    if kind == "zeros":
        return np.zeros((m, n), dtype)
    if kind == "identity":
        return np.eye(m, n, dtype=dtype)
    if kind == "ij":
        i, j = np.meshgrid(np.arange(m), np.arange(n), indexing="ij")
        return (i + j / 10 ** np.ceil(np.log10(max(n, 2)))).astype(dtype)
    if kind == "jordan":
        return (np.eye(m, n, dtype=dtype) + np.eye(m, n, 1, dtype=dtype))
    if kind in ("spd", "poev"):
        return spd_matrix(n, seed, dtype)
    if kind == "diag_dominant":
        return diag_dominant_matrix(n, seed, dtype)
    if kind == "diag":
        return np.diag(np.linspace(1, n, n)).astype(dtype)
    if kind == "heev":
        q, _ = np.linalg.qr(random_matrix(n, n, seed, np.float64))
        cond = cond or 1e3
        d = np.logspace(0, -np.log10(cond), n)
        return (q @ np.diag(d) @ q.T).astype(dtype)
    if kind == "orthog":
        i, j = np.meshgrid(np.arange(1, m + 1), np.arange(1, n + 1), indexing="ij")
        return (np.sqrt(2.0 / (n + 1)) * np.sin(i * j * np.pi / (n + 1))).astype(dtype)
    if kind == "riemann":
        i, j = np.meshgrid(np.arange(2, m + 2), np.arange(2, n + 2), indexing="ij")
        return np.where(j % i == 0, i - 1, -1).astype(dtype)
    if kind == "kms":
        i, j = np.meshgrid(np.arange(m), np.arange(n), indexing="ij")
        return (0.5 ** np.abs(i - j)).astype(dtype)
    if kind == "fiedler":
        i, j = np.meshgrid(np.arange(m), np.arange(n), indexing="ij")
        return np.abs(i - j).astype(dtype)
    if kind == "circul":
        i, j = np.meshgrid(np.arange(m), np.arange(n), indexing="ij")
        return ((j - i) % n + 1).astype(dtype)
    if kind == "chebspec":
        x = np.cos(np.pi * np.arange(n) / (n - 1)) if n > 1 else np.zeros(1)
        c = np.ones(n); c[0] = c[-1] = 2; c *= (-1.0) ** np.arange(n)
        X = np.tile(x, (n, 1)).T
        dX = X - X.T
        D = np.outer(c, 1 / c) / (dX + np.eye(n))
        D -= np.diag(D.sum(axis=1))
        return D[:m].astype(dtype)
    raise ValueError(f"unknown matrix kind {kind!r}")
