"""Development probe: the dependence flags of frame k's rgbds with the small and the full table."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pfilter-noetic_amd"), os.path.join(ROOT, "pfilter-noetic_amd", "synth")]
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
seq = pfsynth.Sequence("S64", n_frames=K + 1, seed=0)
buf, cnt = seq.frames(0, K + 1, threads=16)
db = pa.DeviceBuffer(buf.nbytes)
db.upload(buf)
L = pa.lib()
L.pf_dev_dep_flags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
res = []
for full in (False, True):
    od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 21, tie_order=True)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    od.set_dep_full(full)
    for i in range(K + 1):
        od.frame_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
    od.sync()
    f = np.zeros(1 << 22, np.uint8)
    n = ctypes.c_int()
    assert L.pf_dev_dep_flags(od._h, f.ctypes.data, f.size, ctypes.byref(n)) == 0
    st = od.stats()
    res.append((f[:n.value].copy(), st))
a, b = res[0][0], res[1][0]
print("n", a.size, b.size, "free small", int(a.sum()), "free full", int(b.sum()))
d = np.nonzero(a != b)[0]
print("differ", d.size, "first", d[:20], "small", a[d[:20]], "full", b[d[:20]])
st = res[0][1]
print({k: st[k] for k in ("n_edge_map", "n_surf_map", "n_edge_ds", "n_surf_ds")})
