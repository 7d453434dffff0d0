"""Source check: the factorization k-loops never block the host.

The distributed drivers enqueue every step on HIP streams with event
dependencies (runtime.hh); a host synchronization inside the k-loop would stop
DAG construction so step k+1's panel could not be enqueued while step k waits
(reference drivers block per op: internal_gemm.cc:510 queue->sync()).  This
test scans each driver's k-loop body -- from the `for (int64_t k = 0; k < kt`
header to the loop's closing `S.wait_all()` -- for synchronizing calls."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYNC = re.compile(r"hip(Stream|Event|Device)Synchronize|hipMemcpy\(|fetch_info|\.barrier\(")

# (file, function) pairs whose k-loops must stay asynchronous
DRIVERS = [
    ("csrc/src/getrf.cc", "getrf_dist"),
    ("csrc/src/getrf.cc", "getrf_impl"),
    ("csrc/src/potrf.cc", "potrf_lower"),
    ("csrc/src/qr.cc", "geqrf_impl"),
]


LOOP = re.compile(r"for \(int64_t k = 0; k < \w+; \+\+k\) \{")


def loop_bodies(text, func):
    """Body of the first step loop of `func` up to its S.wait_all()."""
    i = text.find(func + "(")
    assert i >= 0, func
    m = LOOP.search(text, i)
    if not m:
        return []
    end = text.find("S.wait_all()", m.start())
    assert end > m.start()
    return [text[m.start():end]]


@pytest.mark.parametrize("path,func", DRIVERS)
def test_k_loop_has_no_host_sync(path, func):
    text = open(os.path.join(ROOT, path)).read()
    bodies = loop_bodies(text, func)
    assert bodies, (path, func)
    for b in bodies:
        # strip comments
        code = re.sub(r"//[^\n]*", "", b)
        hits = SYNC.findall(code)
        assert not hits, f"{path}:{func}: host synchronization inside the k-loop: {hits}"
