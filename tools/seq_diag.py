"""Development: the full S64 sequence through pf_odom_frame_device, synchronised every 128 frames, to
locate a frame that raises a device error word (prints the window, the merge statistics and the
words).  python3 tools/seq_diag.py [frames]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4541
seq = pfsynth.Sequence("S64", n_frames=N, seed=0)
od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22)
od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
for f0 in range(0, N, 128):
    nf = min(128, N - f0)
    buf, cnt = seq.frames(f0, nf, threads=16)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    for i in range(nf):
        od.frame_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
    try:
        od.sync()
    except pa.PFError as e:
        print("frames %d..%d: %s; merge stats %s" % (f0, f0 + nf - 1, e, od.merge_stats()), flush=True)
        sys.exit(1)
    db.free()
    if f0 % 1024 == 0:
        print("frames to %d ok, merge stats %s" % (f0 + nf - 1, od.merge_stats()), flush=True)
print("all %d frames ok, merge stats %s" % (N, od.merge_stats()))
