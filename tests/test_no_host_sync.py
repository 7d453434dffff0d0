"""Source check: the factorization k-loops never block the host.

The distributed drivers enqueue every step on HIP streams with event
dependencies (runtime.hh); a host synchronization inside the k-loop would stop
DAG construction so step k+1's panel could not be enqueued while step k waits
(reference drivers block per op: internal_gemm.cc:510 queue->sync()).  This
test scans each driver's k-loop body -- from the `for (int64_t k = 0; k < kt`
header to the loop's closing `S.wait_all()` -- for synchronizing calls.

The one deliberate exception is a wait tagged `// allowed host wait:` on the
line before it (the p x q LU's per-step fetch of its pivot slots, which the
exact point-to-point row exchange needs on the host: the panel queue drains,
the trailing queues keep computing); the test pins that there is at most one
such wait per loop."""
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
        lines = b.split("\n")
        hits, allowed = [], 0
        for i, line in enumerate(lines):
            code = re.sub(r"//[^\n]*", "", line)
            if not SYNC.search(code):
                continue
            if i > 0 and "allowed host wait:" in lines[i - 1]:
                allowed += 1
                continue
            hits.append(code.strip())
        assert not hits, f"{path}:{func}: host synchronization inside the k-loop: {hits}"
        assert allowed <= 1, f"{path}:{func}: {allowed} tagged host waits (at most one per step)"
