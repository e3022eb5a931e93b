"""Development probe: per-bucket phase times of k_rgm_bucket (PF_PROBE timestamps, 100 MHz) on the
last frame of a short S64 run, and each bucket's appended-point count.  python3 tools/rgm_probe.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
os.environ["PF_PROBE"] = "1"
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
R = 512                                   # kRgmBuckets
seq = pfsynth.Sequence("S64", n_frames=N)
buf, cnt = seq.frames(0, N, threads=16)
db = pa.DeviceBuffer(buf.nbytes)
db.upload(buf)
od = pa.Odom_ES_EstimationClass()
od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
L = pa.lib()
L.pf_dev_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
names = ["keys", "apps", "sort", "voxels", "scan"]
acc = []
for k in range(N):
    od.frame_device(db.ptr + k * buf.shape[1] * 16, int(cnt[k]))
    if k >= N - 20:
        od.sync()
        t = np.zeros(8192, np.uint64)
        assert L.pf_dev_probe(od._h, t.ctypes.data, 8192) == 0
        r = t[64:64 + 10 * R].astype(np.int64).reshape(R, 10)
        acc.append(r)
a = np.array(acc)                         # [frames, bucket, 10]
t0 = a[:, :, 0].min(axis=1)[:, None]
for i, nm in enumerate(names):
    d = (a[:, :, i + 1] - a[:, :, i]) / 100.0
    print("%-9s us: median over buckets %.2f, max %.2f" % (nm, np.median(d), np.median(d.max(axis=1))))
span = (a[:, :, 5].max(axis=1) - a[:, :, 0].min(axis=1)) / 100.0
start = (a[:, :, 0].max(axis=1) - a[:, :, 0].min(axis=1)) / 100.0
print("bucket start spread us (median) %.2f; first start -> last mark %.2f" % (np.median(start), np.median(span)))
print("appended points per bucket (last frame): max %d, mean %.1f" % (a[-1, :, 9].max(), a[-1, :, 9].mean()))
