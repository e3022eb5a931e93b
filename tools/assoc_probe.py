"""Association-kNN-only workload for the PMC passes of bench.py's configs4 leg: configs[4]'s state (synthetic
S128 scans at 1 m/s, the 2,000,000-point voxel_map surf map seeded after frame 0, a few frames run), then
pf_odom_probe_assoc (k_assoc's exact 5-NN on the last frame's queries against its maps) --iters times.

  python3 tools/assoc_probe.py [--frames N] [--iters N]
Run under one `rocprofv3 --pmc` counter per pass; the kernels are k_assoc_probe_t16 / _t8."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pfilter-noetic_amd"), os.path.join(ROOT, "pfilter-noetic_amd", "synth")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import pfilter_amd as pa
    import pfsynth
    seq = pfsynth.Sequence("S128", n_frames=a.frames, speed=1.0)
    buf, counts = seq.frames(0, a.frames, threads=16)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    od = pa.Odom_ES_EstimationClass(max_points=300000, map_capacity=1 << 22)
    od.init(pa.make_lidar(128, 3.0, 90.0, 0.1, ring_model=(15.0, -25.0)), 0.4, 0, 0.0, 0, 0)
    for k in range(a.frames):
        od.frame_device(db.ptr + k * buf.shape[1] * 16, int(counts[k]))
        od.sync()
        if k == 0:
            m = pfsynth.voxel_map(2_000_000, 0.8, seed=5)
            od.set_map(1, m, np.zeros((m.shape[0], 2), np.uint8))
    ms, alg, nq = od.probe_assoc(iters=a.iters)[:3]
    print(json.dumps({"avg_kernel_ms": ms, "alg_bytes_per_launch": alg, "queries": nq}))


if __name__ == "__main__":
    main()
