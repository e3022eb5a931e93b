"""Global-map probe: LaserMappingClass updates (pf_map_update_device) over S64 edge + surf clouds along
the synthetic trajectory, plus one getMap; prints ms per update.   python3 tools/map_probe.py [--frames N]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pfilter-noetic_amd"), os.path.join(ROOT, "pfilter-noetic_amd", "synth")]
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=200)
a = ap.parse_args()
seq = pfsynth.Sequence("S64", n_frames=a.frames, seed=0)
fe = pa.LaserProcessingClass()
fe.init(pa.make_lidar(64, 3.0, 90.0))
clouds, poses = [], []
for k in range(a.frames):
    e, s = fe.featureExtraction(seq.frame(k))
    clouds.append(np.concatenate([e, s]).astype(np.float32))
    poses.append(np.ascontiguousarray(seq.gt_pose(k), np.float64))
stride = 16 * max(c.shape[0] for c in clouds)
buf = pa.DeviceBuffer(stride * a.frames)
for k, c in enumerate(clouds):
    buf.upload(c, k * stride)
m = pa.LaserMappingClass(max_points=1 << 24, max_scan=stride // 16)
m.init(0.4)
t0 = time.perf_counter()
for k, c in enumerate(clouds):
    rc = pa.lib().pf_map_update_device(m._h, buf.ptr + k * stride, c.shape[0], poses[k].ctypes.data)
    assert rc == 0, rc
el = time.perf_counter() - t0
out = m.getMap()
print("%d updates, %.3f ms per update (synchronous, incl. the host round trip), map %d points, %.1f k points per scan"
      % (a.frames, el / a.frames * 1e3, out.shape[0], np.mean([c.shape[0] for c in clouds]) / 1e3))
