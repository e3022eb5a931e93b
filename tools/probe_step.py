import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd")); sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
os.environ["PF_PROBE"] = "1"
import pfilter_amd as pa, pfsynth
seq = pfsynth.Sequence("S64", n_frames=40)
od = pa.Odom_ES_EstimationClass(); od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0); od.set_graph(False)
L = pa.lib(); L.pf_dev_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
for k in range(30):
    od.frame_host(seq.frame(k))
    if k >= 26:
        t = np.zeros(64, np.uint64); L.pf_dev_probe(od._h, t.ctypes.data, 64); t = t.astype(np.int64)
        names = {47: "start", 48: "accepted", 54: "gradchk", 49: "after_grad", 50: "A_built", 51: "solved", 52: "mcc", 53: "se3"}
        seq_ = [(k2, t[k2]) for k2 in (47, 48, 54, 49, 50, 51, 52, 53) if t[k2] > 0]
        seq_.sort(key=lambda a: a[1])
        base = seq_[0][1]
        print("frame", k, " ".join("%s=%.2f" % (names[a], (b - base) / 100) for a, b in seq_), " total_step=%.2f" % ((t[4 + 8] - t[40 + 2]) / 100))
