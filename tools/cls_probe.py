"""Front-end probe for rocprofv3: the BPF front end (pf_cls_extract) on S64 frames, repeated.
  python3 tools/cls_probe.py [--iters N]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pfilter-noetic_amd"), os.path.join(ROOT, "pfilter-noetic_amd", "synth")]
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--dcvc", action="store_true", help="curvedfilter on (DCVC between ground_seg and featureExtract)")
a = ap.parse_args()
seq = pfsynth.Sequence("S64", n_frames=8, seed=0)
frames = [seq.frame(k) for k in range(8)]
fe = pa.BPFFrontEnd(max_points=300000)
if a.dcvc:
    fe.set_dcvc(True)
fe.extract(frames[0])
t = time.perf_counter()
for i in range(a.iters):
    r = fe.extract(frames[i % 8])
el = time.perf_counter() - t
print({k: len(v) for k, v in r.items()}, "%.3f ms/frame (host API, incl. H2D/D2H)" % (el / a.iters * 1e3))
