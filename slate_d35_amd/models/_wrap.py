"""Helpers to build dtype-dispatching wrappers around native drivers."""
from __future__ import annotations

from .. import _slate
from .._core import native, opts, suffix_of


def call(name, key, *args, target=None, **kw):
    """Call native `name_<suffix of key>` with args + an options dict."""
    fn = getattr(_slate, f"{name}_{suffix_of(key)}", None)
    if fn is None:
        raise NotImplementedError(f"{name} is not available for precision {suffix_of(key)!r}")
    return fn(*args, opts(target, **kw))
