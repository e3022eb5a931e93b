"""Development probe: device memory per handle (hipMemGetInfo before / after creating handles; the
library allocates everything at create): ES and BPF at the default capacities (max_points 300000,
map_capacity 1 << 22) in the default (reference tie) order and in the stable order, and ES at a small
map_capacity.  python3 tools/mem_probe.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pfilter-noetic_amd")]
import pfilter_amd as pa  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def free_bytes():
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)) == 0
    return f.value


def measure(cls, tie, cap, k=2):
    base = free_bytes()
    hs = []
    for _ in range(k):
        o = cls(device=0, max_points=300000, map_capacity=cap, tie_order=tie)
        o.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
        hs.append(o)
    used = base - free_bytes()
    del hs
    import gc
    gc.collect()
    return used / k


out = {}
lid = pa.make_lidar(64, 3.0, 90.0)
hip.hipSetDevice(0)
for name, cls in (("es", pa.Odom_ES_EstimationClass), ("bpf", pa.Odom_BPF_EstimationClass)):
    for tie in (None, False):
        b = measure(cls, tie, 1 << 22)
        out["%s_%s_cap4M" % (name, "tie" if tie is None else "stable")] = round(b / 2**30, 3)
out["es_tie_cap256k"] = round(measure(pa.Odom_ES_EstimationClass, None, 1 << 18) / 2**30, 3)
print(json.dumps({"GiB_per_handle": out}))
