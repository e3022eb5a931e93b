"""Development probe: device timestamps inside k_lm_solve (block 0) for a steady-state frame."""
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

seq = pfsynth.Sequence("S64", n_frames=40)
od = pa.Odom_ES_EstimationClass()
od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
od.set_graph(False)
L = pa.lib()
L.pf_dev_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
for k in range(30):
    od.frame_host(seq.frame(k))
    if k >= 25:
        t = np.zeros(64, np.uint64)
        L.pf_dev_probe(od._h, t.ctypes.data, 64)
        t = t.astype(np.int64)
        out = []
        prev = t[0]
        for ev in range(5):
            a = t[1 + 4 * ev: 5 + 4 * ev]
            if a[0] == 0:
                break
            out.append("ev%d eval %.1f red %.1f wait %.1f gather %.1f step %.1f" % (
                ev, (a[0] - prev) / 100, (a[1] - a[0]) / 100, (a[2] - a[1]) / 100, (t[40 + ev] - a[2]) / 100,
                (a[3] - t[40 + ev]) / 100))
            prev = a[3]
        print("frame", k, " | ".join(out), flush=True)
        p = t[21:26]
        print("   step ev1: load %.2f accept %.2f try_step %.2f se3+shfl %.2f next %.2f" % (
            (p[4] - t[40 + 1]) / 100, (p[0] - p[4]) / 100, (p[1] - p[0]) / 100, (p[2] - p[1]) / 100,
            (p[3] - p[2]) / 100))
