"""Development probe: the depth-limit heap sort (k_tie_heap) alone on one large segment (depth 0: the
whole input is one heap), timed per call and checked against the oracle's literal restatement.
    python3 tools/heap_big.py [sizes...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pfilter-noetic_amd"), os.path.join(ROOT, "oracle")]
import pfilter_amd as pa  # noqa: E402
import pfref  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [20000, 60000, 200000, 850000]
rng = np.random.default_rng(11)


def make_keys(n, kind):
    if kind == "repeats":
        return rng.integers(0, n - n // 50, n).astype(np.uint32)      # equal keys: the heap sort
    if kind == "distinct":
        return rng.permutation(n).astype(np.uint32)                   # the bitonic network
    keys = np.arange(n, dtype=np.uint32)                              # nearly sorted, distinct
    for x in rng.integers(0, n, n // 250):
        y = (x + 7) % n
        keys[x], keys[y] = keys[y], keys[x]
    return keys


for n in sizes:
    for kind in ("repeats", "distinct", "nearly_sorted"):
        keys = make_keys(n, kind)
        ts = []
        for r in range(3):
            t = time.perf_counter()
            out = pa.tie_sort(keys, depth=0, levels=0)
            ts.append(time.perf_counter() - t)
        ok = bool(np.array_equal(out, pfref.sort_perm(keys, "literal", 0)))
        tm = sorted(ts)[1]
        print("heap n %7d %-13s %9.2f ms  %.3f us/key  parity %s" % (n, kind, tm * 1e3, tm * 1e6 / n, ok), flush=True)
