"""Development probe: after every frame of a tie-order run, whether two map points share an rgbds voxel
(the premise of the dependence table's small path, pf_odom.hip DepTab), and the first frame whose map
differs between the small and the full table.   python3 tools/dep_diag.py [frames]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pfilter-noetic_amd"), os.path.join(ROOT, "pfilter-noetic_amd", "synth")]
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 6
seq = pfsynth.Sequence("S64", n_frames=N, seed=0)
buf, cnt = seq.frames(0, N, threads=16)
db = pa.DeviceBuffer(buf.nbytes)
db.upload(buf)
runs = []
for full in (False, True):
    od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 21, tie_order=True)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    od.set_dep_full(full)
    maps = []
    for i in range(N):
        od.frame_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
        od.sync()
        maps.append([od._map(w) for w in (0, 1)])
    runs.append(maps)
for i in range(N):
    line = "frame %d" % i
    for w, leaf in ((0, 0.4), (1, 0.8)):
        xyz = runs[0][i][w][0].astype(np.float32)
        vox = np.floor(xyz / np.float32(leaf)).astype(np.int64)
        _, c = np.unique(vox, axis=0, return_counts=True)
        same = runs[0][i][w][0].shape == runs[1][i][w][0].shape and \
            np.array_equal(runs[0][i][w][0].view(np.uint32), runs[1][i][w][0].view(np.uint32))
        line += "  map%d n %d dup-voxels %d same %s" % (w, xyz.shape[0], int((c > 1).sum()), same)
    print(line, flush=True)
