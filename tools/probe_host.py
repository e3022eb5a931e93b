"""Development probe: host-side submission cost of pf_odom_frame_device (graph replay) versus the
device frame rate. Prints per-call host microseconds (no synchronisation inside the loop)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 600
seq = pfsynth.Sequence("S64", n_frames=N, seed=0)
buf, counts = seq.frames(0, N, threads=8)
db = pa.DeviceBuffer(buf.nbytes)
db.upload(buf)
stride = buf.shape[1] * 16
od = pa.Odom_ES_EstimationClass(max_points=300000, map_capacity=1 << 22)
od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
for k in range(40):
    od.frame_device(db.ptr + k * stride, int(counts[k]))
od.sync()
calls = []
t0 = time.perf_counter()
for k in range(40, N):
    a = time.perf_counter()
    od.frame_device(db.ptr + k * stride, int(counts[k]))
    calls.append(time.perf_counter() - a)
t1 = time.perf_counter()
od.sync()
t2 = time.perf_counter()
c = np.array(calls) * 1e6
print("frames %d  host us/call median %.1f p90 %.1f  enqueue total %.1f ms  until idle %.1f ms  -> %.1f us/frame"
      % (len(calls), np.median(c), np.percentile(c, 90), (t1 - t0) * 1e3, (t2 - t0) * 1e3,
         (t2 - t0) * 1e6 / len(calls)))
print("call us (frames 300..340):", " ".join("%.0f" % x for x in c[260:300]))
del od
import gc
gc.collect()
