"""Development probe: configs[4] (S128 scans against a seeded 2M-point surf map) frame by frame: the
synchronous time of each frame and the map merge's counters (updates that fell back to the full sort,
largest appended-point count of a bucket).  python3 tools/c4_probe.py [frames] [tie|stable] [graph|eager]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pfilter-noetic_amd"), os.path.join(ROOT, "pfilter-noetic_amd", "synth")]
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 30
ORDER = sys.argv[2] if len(sys.argv) > 2 else "stable"
GRAPH = (sys.argv[3] if len(sys.argv) > 3 else "graph") == "graph"
seq = pfsynth.Sequence("S128", n_frames=N, speed=1.0)
buf, counts = seq.frames(0, N, threads=16)
db = pa.DeviceBuffer(buf.nbytes)
db.upload(buf)
ptrs = [(db.ptr + i * buf.shape[1] * 16, int(counts[i])) for i in range(N)]
od = pa.Odom_ES_EstimationClass(max_points=300000, map_capacity=1 << 22)
od.init(pa.make_lidar(128, 3.0, 90.0, 0.1, ring_model=(15.0, -25.0)), 0.4, 0, 0.0, 0, 0)
od.set_tie_order(ORDER == "tie")
od.set_graph(GRAPH)
od.frame_device(*ptrs[0])
od.sync()
m = pfsynth.voxel_map(2_000_000, 0.8, seed=5)
od.set_map(1, m, np.zeros((m.shape[0], 2), np.uint8))
prev = od.merge_stats()
for k in range(1, N):
    t = time.perf_counter()
    od.frame_device(*ptrs[k])
    od.sync()
    el = (time.perf_counter() - t) * 1e3
    ms = od.merge_stats()
    st = od.stats()
    print("frame %3d %8.3f ms  full_sorts +%d  max_appended %d  n_map %s n_ds %s" % (
        k, el, ms[0] - prev[0], ms[1], st["n_map"][:2], st["n_ds"][:2]), flush=True)
    prev = ms
