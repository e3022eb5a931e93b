"""Per-workgroup k_lm_solve timeline from the device probe (PF_PROBE, s_memrealtime at 100 MHz): every
workgroup's start, and per evaluation each home chunk's publish and each workgroup's end of the
arrival wait.  Splits the arrival wait into skew (last publish - block 0's publish) and visibility
(block 0's wait end - last publish).  python3 tools/probe_lm3.py"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd")); sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
os.environ["PF_PROBE"] = "1"
import pfilter_amd as pa, pfsynth
W, B, E = 8192, 32, 5
P0 = W - 512
seq = pfsynth.Sequence("S64", n_frames=60)
od = pa.Odom_ES_EstimationClass(); od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0); od.set_graph(False)
L = pa.lib(); L.pf_dev_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
rows = []
for k in range(60):
    od.frame_host(seq.frame(k))
    if k < 30:
        continue
    t = np.zeros(W, np.uint64); L.pf_dev_probe(od._h, t.ctypes.data, W); t = t.astype(np.int64)
    st = t[P0 + 2 * E * B: P0 + 2 * E * B + B]
    t0 = st.min()
    pub = t[P0: P0 + 2 * E * B: 2].reshape(E, B)
    wend = t[P0 + 1: P0 + 2 * E * B: 2].reshape(E, B)
    rows.append((st - t0, pub, wend, t0))
starts = np.array([r[0] for r in rows]) / 100.0
print("workgroup start spread us: median %.2f  max %.2f" % (np.median(starts.max(1)), starts.max()))
for ev in range(E):
    sk, vis, last_b = [], [], []
    for st, pub, wend, t0 in rows:
        if pub[ev].min() < t0 or wend[ev, 0] < pub[ev].max():
            continue
        sk.append(pub[ev].max() - pub[ev, 0]); vis.append(wend[ev, 0] - pub[ev].max()); last_b.append(int(pub[ev].argmax()))
    if not sk:
        continue
    print("eval %d (n=%d) us: skew (last publish - block 0) median %.2f  visibility (block 0 wait end - last publish) median %.2f  last block %s"
          % (ev, len(sk), np.median(sk) / 100, np.median(vis) / 100, np.bincount(last_b, minlength=B).argsort()[::-1][:4].tolist()))
