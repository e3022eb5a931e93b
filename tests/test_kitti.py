"""KITTI I/O and the evaluation metric (runkitti.py:111-157 scores `<seq>_pred.txt`
with the external KITTI odometry evaluation tool, whose published segment metric kitti.evaluate
restates). CPU tests use synthetic trajectories; the GPU test runs tools/kitti_run.py over a synthetic
sequence written as KITTI .bin scans."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _traj(n=400, speed=1.0, yaw_rate=0.01):
    """a planar drive: 1 m per frame, slowly turning; poses {qx,qy,qz,qw,tx,ty,tz}"""
    out = np.zeros((n, 7))
    yaw, x, y = 0.0, 0.0, 0.0
    for i in range(n):
        out[i] = [0, 0, np.sin(yaw / 2), np.cos(yaw / 2), x, y, 0]
        x += speed * np.cos(yaw)
        y += speed * np.sin(yaw)
        yaw += yaw_rate
    return out


def test_pose_file_round_trip(tmp_path):
    import kitti
    p = _traj(50)
    rng = np.random.default_rng(0)
    tr = kitti.pose7_to_mat(np.r_[rng.normal(size=4), rng.normal(size=3)] / np.r_[np.ones(4) * 2, np.ones(3)])
    q = rng.normal(size=4)
    tr[:3, :3] = kitti.quat_to_mat(q / np.linalg.norm(q))
    kitti.write_poses(tmp_path / "a.txt", p, tr)
    T = kitti.read_poses(tmp_path / "a.txt")
    assert T.shape == (50, 4, 4)
    for i in (0, 17, 49):
        back = np.linalg.inv(tr) @ T[i] @ tr
        np.testing.assert_allclose(back, kitti.pose7_to_mat(p[i]), atol=1e-7)
    kitti.write_poses(tmp_path / "b.txt", p)          # no calibration: the lidar poses themselves
    np.testing.assert_allclose(kitti.read_poses(tmp_path / "b.txt")[5], kitti.pose7_to_mat(p[5]), atol=1e-8)


def test_velodyne_reader(tmp_path):
    import kitti
    x = np.random.default_rng(1).normal(size=(1000, 4)).astype(np.float32)
    d = tmp_path / "sequences" / "03" / "velodyne"
    d.mkdir(parents=True)
    for k in (2, 0, 1):
        x[k:].tofile(d / ("%06d.bin" % k))
    paths = kitti.sequence_scans(tmp_path, 3)
    assert [os.path.basename(p) for p in paths] == ["000000.bin", "000001.bin", "000002.bin"]
    np.testing.assert_array_equal(kitti.read_velodyne(paths[1]), x[1:])


def test_evaluate_metric():
    import kitti
    p = _traj(900)
    gt = np.array([kitti.pose7_to_mat(v) for v in p])
    r = kitti.evaluate(gt, gt)
    assert r["segments"] > 0 and r["t_rel_pct"] < 1e-9 and r["r_rel_deg_per_100m"] < 1e-6 and r["ate_rmse_m"] == 0
    straight = np.array([kitti.pose7_to_mat(v) for v in _traj(900, yaw_rate=1e-4)])
    scaled = straight.copy()
    scaled[:, :3, 3] *= 1.01        # 1 % scale drift: 1 % of the chord on every segment (chord ~ length here)
    r = kitti.evaluate(straight, scaled)
    assert abs(r["t_rel_pct"] - 1.0) < 1e-3 and r["r_rel_deg_per_100m"] < 1e-6
    short = kitti.evaluate(gt[:50], gt[:50])         # path shorter than 100 m: no segments
    assert short["segments"] == 0 and short["t_rel_pct"] is None


@pytest.mark.gpu
def test_kitti_runner_on_synthetic_sequence(pa, pfsynth, tmp_path):
    """tools/kitti_run.py over a synthetic S64 sequence written as KITTI scans + ground truth: the
    same poses as the in-process pipeline, a written KITTI pose file and a small segment error."""
    import kitti
    n = 120
    seq = pfsynth.Sequence("S64", n_frames=n)
    d = tmp_path / "sequences" / "00" / "velodyne"
    d.mkdir(parents=True)
    for k in range(n):
        seq.frame(k).astype(np.float32).tofile(d / ("%06d.bin" % k))
    (tmp_path / "poses").mkdir()
    kitti.write_poses(tmp_path / "poses" / "00.txt", np.array([seq.gt_pose(k) for k in range(n)]))
    out = tmp_path / "00_pred.txt"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kitti_run.py"), "--root", str(tmp_path),
                        "--seq", "0", "--out", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["frames"] == n and not res["camera_frame"]
    od = pa.Odom_ES_EstimationClass()
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    for k in range(n):
        od.frame_host(seq.frame(k), want_pose=False)
    np.testing.assert_allclose(kitti.read_poses(out)[:, :3, :4].reshape(n, 12), kitti.poses_to_kitti(od.poses()),
                               atol=2e-9)
    ev = res["eval"]
    assert ev["segments"] > 0 and ev["t_rel_pct"] < 2.0 and ev["ate_rmse_m"] < 1.0


@pytest.mark.gpu
def test_kitti_runner_bpf_chain(pa, pfsynth, tmp_path):
    """tools/kitti_run.py --estimator bpf: raw KITTI-format scans through the front end and the BPF
    estimator; the same poses as the in-process raw-scan pipeline, and a bounded segment error."""
    import kitti
    n = 120
    seq = pfsynth.Sequence("S64", n_frames=n)
    d = tmp_path / "sequences" / "00" / "velodyne"
    d.mkdir(parents=True)
    for k in range(n):
        seq.frame(k).astype(np.float32).tofile(d / ("%06d.bin" % k))
    (tmp_path / "poses").mkdir()
    kitti.write_poses(tmp_path / "poses" / "00.txt", np.array([seq.gt_pose(k) for k in range(n)]))
    out = tmp_path / "00_pred.txt"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kitti_run.py"), "--root", str(tmp_path),
                        "--seq", "0", "--out", str(out), "--estimator", "bpf"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["frames"] == n and res["estimator"] == "bpf"
    od = pa.Odom_BPF_EstimationClass()
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    for k in range(n):
        od.frame_host(seq.frame(k), want_pose=False)
    od.sync()
    np.testing.assert_allclose(kitti.read_poses(out)[:, :3, :4].reshape(n, 12), kitti.poses_to_kitti(od.poses()),
                               atol=2e-9)
    ev = res["eval"]
    print("bpf chain on synthetic S64:", ev)
    assert ev["segments"] > 0 and ev["t_rel_pct"] < 5.0
