"""Per-evaluation timeline of k_lm_solve from its device probe (s_memrealtime, 100 MHz), block 0:
home-chunk reduction, arrival wait, partial gather, LM step; and for evaluation 1 the step's parts
(core load, lm_try_step, the two SE(3) updates, the rest).  python3 tools/probe_lm2.py"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd")); sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
os.environ["PF_PROBE"] = "1"
import pfilter_amd as pa, pfsynth
NF = int(os.environ.get("PF_PROBE_FRAMES", "60"))
seq = pfsynth.Sequence("S64", n_frames=NF)
od = pa.Odom_ES_EstimationClass(); od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0); od.set_graph(False)
L = pa.lib(); L.pf_dev_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
acc = []
for k in range(NF):
    od.frame_host(seq.frame(k))
    if k < 30:
        continue
    t = np.zeros(64, np.uint64); L.pf_dev_probe(od._h, t.ctypes.data, 64); t = t.astype(np.int64)
    prev = t[0]
    row = []
    for ev in range(5):
        if t[4 + 4 * ev] == 0 or t[4 + 4 * ev] < prev:
            break
        red, wait, gat, step = t[1 + 4 * ev] - prev, t[3 + 4 * ev] - t[1 + 4 * ev], t[40 + ev] - t[3 + 4 * ev], t[4 + 4 * ev] - t[40 + ev]
        row.append((red, wait, gat, step))
        prev = t[4 + 4 * ev]
    parts = (t[25] - t[40 + 1], t[21] - t[25], t[22] - t[21], t[23] - t[22], t[24] - t[23])
    acc.append((row, parts, prev - t[0], (t[55] - t[0], t[50] - t[55], t[51] - t[50], t[52] - t[51], t[53] - t[52], t[54] - t[53], t[1] - t[54])))
    t[:] = 0
ev_stats = {}
for row, parts, tot, _o in acc:
    for i, r in enumerate(row):
        ev_stats.setdefault(i, []).append(r)
for i in sorted(ev_stats):
    a = np.array(ev_stats[i]) / 100.0
    print("eval %d (n=%d) us: reduce %.2f wait %.2f gather %.2f step %.2f" % ((i, len(a)) + tuple(np.median(a, 0))))
p = np.array([x[1] for x in acc]) / 100.0
print("eval 1 step parts us (median): load %.2f try_step %.2f se3 %.2f tail %.2f | core total %.2f" % tuple(np.median(p, 0)[[0, 2, 3, 4]].tolist() + [np.median(p[:, 1:].sum(1))]))
o = np.array([x[3] for x in acc]) / 100.0
print("eval 0 observe us (median): prologue %.2f  observe loads+eval %.2f  claim sync %.2f  commits issued %.2f  commits complete+sync %.2f  count/s_mine %.2f  home reduce %.2f" % tuple(np.median(o, 0)))
sp = np.array([x[2] for x in acc]) / 100.0
print("launch span us (median): %.2f  mean %.2f  n %d  lib %s" % (np.median(sp), sp.mean(), len(sp), os.environ.get("PFILTER_HIP_LIB", "in-tree")))
