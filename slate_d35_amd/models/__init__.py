"""Routine families (the reference's "model families" are linear-algebra
routine groups, src/*.cc): level-3 BLAS, auxiliary, norms, Cholesky, LU,
QR/LQ/least squares, eigenvalue and SVD drivers.  Each function dispatches on
the matrix precision to the native driver; options are keyword arguments
(target='d'|'h', lookahead=..., ...)."""
from .blas3 import *      # noqa: F401,F403
from .aux import *        # noqa: F401,F403
from .cholesky import *   # noqa: F401,F403
from .lu import *         # noqa: F401,F403
from .qr import *         # noqa: F401,F403
from .eig import *        # noqa: F401,F403
from .factor import *     # noqa: F401,F403
