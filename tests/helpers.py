import numpy as np

import slate_d35_amd as s

DTYPES = [np.float32, np.float64, np.complex64, np.complex128]


def tol(dtype):
    return {np.float32: 2e-4, np.float64: 1e-11, np.complex64: 3e-4, np.complex128: 1e-11}[np.dtype(dtype).type]


def rnd(m, n, dtype, seed):
    return s.utils.random_matrix(m, n, seed=seed, dtype=dtype)


def relerr(x, ref):
    d = np.linalg.norm(np.asarray(x) - np.asarray(ref))
    r = np.linalg.norm(np.asarray(ref))
    return d / max(r, 1e-300)
