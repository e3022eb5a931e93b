"""Full-sequence parity report (CPU; oracle = test infrastructure): the committed GPU trajectory
(tests/golden/odom_s64_full.npz, which the -m gpu test test_full_sequence_bench_path shows the device
reproduces) against (a) the oracle's reference-faithful option set (opts=0: libstdc++ std::sort tie
order in VoxelGrid / rgbds / the sector sort, Householder-QR LM, FLANN-style kd-tree) and (b) the
generator's ground truth, per frame and as drift, and the same for the faithful trajectory.

  python3 tools/parity_report.py [--frames N] [--out profiles/parity_r02.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("pfilter-noetic_amd/synth", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))


def drift(poses, gt):
    """translation error at the end / path length, and the mean per-frame position error (m)"""
    e = np.linalg.norm(poses[:, 4:7] - gt[:, 4:7], axis=1)
    path = np.sum(np.linalg.norm(np.diff(gt[:, 4:7], axis=0), axis=1))
    return {"final_pos_err_m": float(e[-1]), "path_m": float(path), "final_drift_pct": float(100 * e[-1] / path),
            "mean_pos_err_m": float(e.mean()), "max_pos_err_m": float(e.max())}


def main():
    import pfsynth
    import pfref
    from _util import pose_err
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "parity_r02.json"))
    a = ap.parse_args()
    g = np.load(os.path.join(ROOT, "tests", "golden", "odom_s64_full.npz"))
    gpu = g["poses"]
    n = a.frames or gpu.shape[0]
    gpu = gpu[:n]
    seq = pfsynth.Sequence("S64", n_frames=gpu.shape[0] if not a.frames else n, seed=0)
    gt = np.array([seq.gt_pose(k) for k in range(n)])
    orc = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=0)
    faith = np.empty((n, 7))
    t0 = time.time()
    for f0 in range(0, n, 256):
        nf = min(256, n - f0)
        buf, cnt = seq.frames(f0, nf, threads=8)
        for i in range(nf):
            faith[f0 + i] = orc.frame(buf[i, :cnt[i]])
    el = time.time() - t0
    e = np.array([pose_err(gpu[k], faith[k]) for k in range(n)])
    first = {str(th): (int(np.argmax(e[:, 0] > th)) if (e[:, 0] > th).any() else None) for th in (1e-12, 1e-9, 1e-6, 1e-4)}
    out = {"frames": n, "sequence": "S64 seed 0 (configs[1] parameters)",
           "gpu_vs_faithful": {"first_frame_above_m": first,
                               "frames_within_1e-4m_1e-5rad": int(np.sum((e[:, 0] < 1e-4) & (e[:, 1] < 1e-5))),
                               "median_m": float(np.median(e[:, 0])), "max_m": float(e[:, 0].max()),
                               "max_rad": float(e[:, 1].max())},
           "gpu_vs_ground_truth": drift(gpu, gt), "faithful_vs_ground_truth": drift(faith, gt),
           "oracle_seconds": round(el, 1)}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
