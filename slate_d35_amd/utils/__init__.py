"""Utilities: LAWN-41 flop counts (reference docs/latex/flops.py), timing,
test-matrix generation (reference matgen/)."""
from .flops import *   # noqa: F401,F403
from .matgen import *  # noqa: F401,F403
from . import debug  # noqa: F401
