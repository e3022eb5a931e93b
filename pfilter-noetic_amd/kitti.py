"""KITTI odometry I/O and evaluation around the device pipeline.

The reference evaluates by replaying KITTI sequences through its ROS nodes and scoring the written
trajectories with the external KITTI_odometry_evaluation_tool (runkitti.py:111-157: `<seq>_pred.txt`
against `ground_truth_pose/<seq>.txt`). This module is the same round trip without ROS:

  read_velodyne / sequence_scans   velodyne/*.bin scans (float32 x, y, z, reflectance)
  read_calib_tr                    Tr (velodyne -> left camera) of calib.txt
  poses_to_kitti / write_poses     per-frame odometry poses {qx,qy,qz,qw,tx,ty,tz} (lidar frame 0) as
                                   KITTI rows: 12 values of [R | t] in the camera frame,
                                   T_cam = Tr T_lidar Tr^-1 (Tr = I without calibration)
  read_poses                       KITTI pose files back to (n, 4, 4)
  evaluate                         the evaluation tool's published metric: for every first frame
                                   (step 10) and segment length 100 .. 800 m, the relative pose error
                                   between the frame and the first frame that far along the ground
                                   truth path; translation error in % of the length, rotation error
                                   in deg / 100 m, averaged over all segments; plus the absolute
                                   trajectory RMSE
"""
import glob
import os

import numpy as np

LENGTHS = (100, 200, 300, 400, 500, 600, 700, 800)


def read_velodyne(path):
    """One KITTI scan: (n, 4) float32 x, y, z, reflectance."""
    return np.fromfile(path, dtype=np.float32).reshape(-1, 4)


def sequence_scans(root, seq):
    """Sorted scan paths of sequence `seq` (int or "00") under root/sequences/<seq>/velodyne."""
    d = os.path.join(root, "sequences", "%02d" % int(seq), "velodyne")
    return sorted(glob.glob(os.path.join(d, "*.bin")))


def read_calib_tr(path):
    """Tr of a KITTI odometry calib.txt as a 4x4 matrix."""
    with open(path) as f:
        for line in f:
            if line.startswith("Tr:"):
                v = np.array([float(x) for x in line.split()[1:13]])
                T = np.eye(4)
                T[:3, :4] = v.reshape(3, 4)
                return T
    raise ValueError("no Tr in %s" % path)


def quat_to_mat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def pose7_to_mat(p):
    T = np.eye(4)
    T[:3, :3] = quat_to_mat(p[:4])
    T[:3, 3] = p[4:7]
    return T


def poses_to_kitti(poses7, tr=None):
    """(n, 7) odometry poses -> (n, 12) KITTI rows in the camera frame."""
    tr = np.eye(4) if tr is None else np.asarray(tr, np.float64)
    tri = np.linalg.inv(tr)
    out = np.empty((len(poses7), 12))
    for i, p in enumerate(np.asarray(poses7, np.float64)):
        out[i] = (tr @ pose7_to_mat(p) @ tri)[:3, :4].reshape(12)
    return out


def write_poses(path, poses7, tr=None):
    np.savetxt(path, poses_to_kitti(poses7, tr), fmt="%.9e")


def read_poses(path):
    v = np.loadtxt(path, ndmin=2)
    T = np.tile(np.eye(4), (v.shape[0], 1, 1))
    T[:, :3, :4] = v.reshape(-1, 3, 4)
    return T


def _path_dist(gt):
    d = np.zeros(len(gt))
    d[1:] = np.cumsum(np.linalg.norm(np.diff(gt[:, :3, 3], axis=0), axis=1))
    return d


def _rot_angle(R):
    return float(np.arccos(np.clip((np.trace(R) - 1) / 2, -1.0, 1.0)))


def evaluate(gt, pred, step=10, lengths=LENGTHS):
    """Segment errors of the KITTI odometry benchmark and the absolute trajectory RMSE.

    gt, pred: (n, 4, 4) poses of the same frames. Returns {"t_rel_pct", "r_rel_deg_per_100m",
    "segments", "ate_rmse_m"}; the relative metrics are None when the path is shorter than 100 m."""
    gt = np.asarray(gt, np.float64)
    pred = np.asarray(pred, np.float64)
    n = min(len(gt), len(pred))
    gt, pred = gt[:n], pred[:n]
    dist = _path_dist(gt)
    t_err, r_err = [], []
    for first in range(0, n, step):
        for L in lengths:
            last = int(np.searchsorted(dist, dist[first] + L))
            if last >= n:
                continue
            dg = np.linalg.inv(gt[first]) @ gt[last]
            dp = np.linalg.inv(pred[first]) @ pred[last]
            e = np.linalg.inv(dp) @ dg
            t_err.append(np.linalg.norm(e[:3, 3]) / L)
            r_err.append(_rot_angle(e[:3, :3]) / L)
    ate = float(np.sqrt(np.mean(np.sum((gt[:, :3, 3] - pred[:, :3, 3]) ** 2, axis=1))))
    if not t_err:
        return {"t_rel_pct": None, "r_rel_deg_per_100m": None, "segments": 0, "ate_rmse_m": ate}
    return {"t_rel_pct": 100.0 * float(np.mean(t_err)),
            "r_rel_deg_per_100m": float(np.degrees(np.mean(r_err)) * 100.0),
            "segments": len(t_err), "ate_rmse_m": ate}
