"""Development probe (variant build with -DPF_TIE_PROF, loaded through PFILTER_HIP_LIB): k_tie_heap's
phases on one depth-limit segment of n keys (depth limit 0: the whole input is heap-sorted).
    python3 tools/heap_prof.py [n...]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
import pfilter_amd as pa  # noqa: E402

L = pa.lib()
PROF = hasattr(L, "pf_dev_tie_prof")          # the -DPF_TIE_PROF build; without it the sorts just run
if PROF:
    L.pf_dev_tie_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
rng = np.random.default_rng(7)
for n in [int(a) for a in sys.argv[1:]] or [500, 3000, 7000]:
    keys = rng.integers(0, n // 3, n).astype(np.uint32)
    for rep in range(3):
        pa.tie_sort(keys, depth=0)
    if not PROF:
        print("n %d: 3 sorts (no prof build)" % n)
        continue
    buf = np.zeros(1024, np.uint64)
    assert L.pf_dev_tie_prof(buf.ctypes.data, 1024) == 0
    b = buf.astype(np.int64)
    mk = (b[961] - b[960]) / 100.0
    so = (b[962] - b[961]) / 100.0
    clk = (b[966] - b[965]) / ((b[962] - b[960]) / 100.0)
    steps = b[964]
    print("n %d make %.1f us sort %.1f us steps %d (%.2f per pop) %.0f cycles/step %.0f cycles/pop clock %.0f MHz"
          % (b[963], mk, so, steps, steps / max(1, n - 1), so * clk / max(1, steps), so * clk / max(1, n - 1), clk))
    if b[967] or b[968]:                  # per-step cycles of the two steps of a pair (s_memtime)
        print("   step A %.0f cycles, step B %.0f cycles" % (2 * b[967] / max(1, steps), 2 * b[968] / max(1, steps)))
