"""Development probe (variant build with -DPF_TIE_PROF, loaded through PFILTER_HIP_LIB): per-level
phase times of the partition tiers and k_tie_local's first job on a synthetic key set, or on the keys of a
real sort call the oracle dumped.  python3 tools/tie_prof.py [n] [per] | [dump file] [call]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
import pfilter_amd as pa  # noqa: E402

rng = np.random.default_rng(5)
if len(sys.argv) > 1 and os.path.exists(sys.argv[1]):
    # keys of a real sort call dumped by the oracle (PFREF_SORT_DUMP / PFREF_SORT_DUMP_MIN: count, keys ...)
    raw = np.fromfile(sys.argv[1], np.uint32)
    want = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    i = c = 0
    while True:
        cnt = int(raw[i])
        if c == want:
            keys = raw[i + 1:i + 1 + cnt].copy()
            break
        i += 1 + cnt
        c += 1
    n, per = keys.size, 0
else:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 11000
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 13
if per == 0:
    pass
elif per > 0:
    keys = rng.integers(0, max(1, n // per), n).astype(np.uint32)
else:                             # rgbds-like: a sorted distinct map plus -per appended points on it
    napp = -per
    m = np.sort(rng.choice(1 << 24, n - napp, replace=False))
    keys = np.concatenate([m, rng.choice(m, napp)]).astype(np.uint32)
L = pa.lib()
L.pf_dev_tie_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
for rep in range(3):
    pa.tie_sort(keys, levels=0)
buf = np.zeros(1024, np.uint64)
assert L.pf_dev_tie_prof(buf.ctypes.data, 1024) == 0
t0 = int(buf[0])
lev = int(buf[3])
print("shader clock %.0f MHz" % ((int(buf[5]) - int(buf[4])) / ((int(buf[1]) - t0) / 100.0)))
print("jobs", int(buf[6]), "mid items", int(buf[7]))
print("n", n, "levels", lev, "loop %.1f us" % ((int(buf[1]) - t0) / 100.0), "output %.1f us" % ((int(buf[2]) - int(buf[1])) / 100.0))
def tier(base, name, nlev=16):
    for k in range(nlev):
        b = buf[base + 8 * k: base + 8 * k + 8].astype(np.int64)
        if b[0] == 0:
            break
        if b[1] == 0 or b[7] == 0:
            print("%s lev %2d ns %4d" % (name, k, b[7]))
            break
        ph = [(b[i + 1] - b[i]) / 100.0 for i in range(5)]
        print("%s lev %2d ns %4d  ranks %6.2f  count %6.2f  cut %6.2f  swaps %6.2f  children %6.2f us"
              % (name, k, b[7], *ph))


tier(256, "medium", 32)
tier(512, "mid")
for k in range(lev + 1):
    b = buf[8 + 8 * k: 8 + 8 * k + 6].astype(np.int64)
    if k == lev:
        print("lev %2d ns %4d" % (k, b[5]))
        break
    b = buf[8 + 8 * k: 8 + 8 * k + 8].astype(np.int64)
    t = [b[0], b[1], b[2], b[3], b[4], b[6]]
    ph = [(t[i + 1] - t[i]) / 100.0 for i in range(5)]
    print("lev %2d ns %4d  ranks %6.2f  lists %6.2f  search %6.2f  swaps %6.2f  children %6.2f us" % (k, b[5], *ph))
