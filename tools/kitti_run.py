"""Run the device odometry over a KITTI odometry sequence and score it.

  python tools/kitti_run.py --root $PF_KITTI_ROOT --seq 0 --out results/00_pred.txt

Scans are read from <root>/sequences/<seq>/velodyne/*.bin, staged in HBM and run through
pf_odom_frame_device (featureExtraction + Odom_ES_EstimationClass, configs[1] parameters unless set)
or, with --estimator bpf, pf_bpf_frame_scan_device (ground_seg + PCA featureExtract +
Odom_BPF_EstimationClass: the additionNode -> odomEstimationNode chain without the DCVC stage);
poses are written in the KITTI format (camera frame when <root>/sequences/<seq>/calib.txt exists),
and scored against <root>/poses/<seq>.txt when present (kitti.evaluate). Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", required=True)
    ap.add_argument("--seq", type=int, default=0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--lines", type=int, default=64)
    ap.add_argument("--min-dist", type=float, default=3.0)
    ap.add_argument("--max-dist", type=float, default=90.0)
    ap.add_argument("--map-res", type=float, default=0.4)
    ap.add_argument("--k-new", type=int, default=0)
    ap.add_argument("--theta-p", type=float, default=0.4)
    ap.add_argument("--theta-max", type=int, default=75)
    ap.add_argument("--weight-type", type=int, default=0)
    ap.add_argument("--max-frames", type=int, default=0)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--estimator", choices=["es", "bpf"], default="es")
    a = ap.parse_args()
    import kitti
    import pfilter_amd as pa
    paths = kitti.sequence_scans(a.root, a.seq)
    if a.max_frames:
        paths = paths[:a.max_frames]
    if not paths:
        raise SystemExit("no scans under %s" % a.root)
    scans = [kitti.read_velodyne(p) for p in paths]
    cap = max(s.shape[0] for s in scans)
    buf = np.zeros((len(scans), cap, 4), np.float32)
    for i, s in enumerate(scans):
        buf[i, :s.shape[0]] = s
    db = pa.DeviceBuffer(buf.nbytes, device=a.device)
    db.upload(buf)
    cls = pa.Odom_BPF_EstimationClass if a.estimator == "bpf" else pa.Odom_ES_EstimationClass
    od = cls(device=a.device, max_points=max(cap, 1024))
    od.init(pa.make_lidar(a.lines, a.min_dist, a.max_dist), a.map_res, a.k_new, a.theta_p, a.theta_max,
            a.weight_type)
    step = od.frame_scan_device if a.estimator == "bpf" else od.frame_device
    t0 = time.perf_counter()
    for i, s in enumerate(scans):
        step(db.ptr + i * cap * 16, s.shape[0])
    od.sync()
    el = time.perf_counter() - t0
    poses = od.poses()
    seqdir = os.path.join(a.root, "sequences", "%02d" % a.seq)
    calib = os.path.join(seqdir, "calib.txt")
    tr = kitti.read_calib_tr(calib) if os.path.exists(calib) else None
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    kitti.write_poses(a.out, poses, tr)
    res = {"seq": "%02d" % a.seq, "estimator": a.estimator, "frames": len(scans), "seconds": round(el, 4),
           "frames_per_s": round(len(scans) / el, 2), "out": a.out, "camera_frame": tr is not None}
    gt = os.path.join(a.root, "poses", "%02d.txt" % a.seq)
    if os.path.exists(gt):
        res["eval"] = kitti.evaluate(kitti.read_poses(gt), kitti.read_poses(a.out))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
