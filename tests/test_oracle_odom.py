"""CPU: the oracle's whole odometry path on synthetic sequences (no GPU).

Checks that the restatement tracks (drift against the generator's ground truth), that the pose
stays a unit quaternion through the constant-velocity prediction — Eigen 3.3's
Isometry3d::rotation() re-orthonormalises (SVD polar factor); using linear() instead lets |q|-1
grow ~3x per frame once the heading passes 90 degrees and the odometry diverges — and that the
option bits that separate the GPU-equivalent mode from the reference-faithful one only move the
pose by tie-order / summation-order noise."""
import numpy as np

from _util import pose_err


def yaw(q):
    return 2 * np.arctan2(q[2], q[3])


def test_tracks_and_keeps_unit_quaternion(pfref, pfsynth):
    seq = pfsynth.Sequence("S64", n_frames=60, az_steps=1000)
    od = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=pfref.GPU_EQUIV)
    for k in range(40):
        p = od.frame(seq.frame(k))
        assert abs(np.linalg.norm(p[:4]) - 1) < 1e-14
    gt = seq.gt_pose(39)
    assert np.linalg.norm(p[4:] - gt[4:]) < 0.2
    st = od.stats()
    assert st["n_edge_res"] > 100 and st["n_surf_res"] > 100 and not st["map_too_small"]


def test_heading_beyond_90_degrees(pfref, pfsynth):
    """Start the odometry at a world heading of 2.0 rad: the same scans must give the same
    trajectory rotated by 2.0 rad (this is where a linear()-based rotation() diverged)."""
    y0 = 2.0
    seq = pfsynth.Sequence("S64", n_frames=80, az_steps=900)
    od = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=pfref.GPU_EQUIV)
    q0 = np.array([0, 0, np.sin(y0 / 2), np.cos(y0 / 2), 0, 0, 0.0])
    od.set_state(q0, q0)
    for k in range(70):
        p = od.frame(seq.frame(k))
        err = (yaw(p) - y0 - yaw(seq.gt_pose(k)) + np.pi) % (2 * np.pi) - np.pi
        assert abs(err) < 0.01, (k, err)
        assert abs(np.linalg.norm(p[:4]) - 1) < 1e-14


def test_option_bits_are_tie_noise(pfref, pfsynth):
    """opts=0 (std::sort ties, dense QR LM, kd-tree) vs GPU_EQUIV: same counts, poses within
    the north-star tolerance over a short sequence."""
    seq = pfsynth.Sequence("S64", n_frames=20, az_steps=1000)
    a = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=0)
    b = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=pfref.GPU_EQUIV)
    for k in range(10):
        x = seq.frame(k)
        dt, dr = pose_err(a.frame(x), b.frame(x))
        assert dt < 1e-4 and dr < 1e-5


def test_map_state_invariants(pfref, pfsynth):
    """Ages (r) and p-index (g) bytes: g <= 255, every map point inside the 100 m crop box."""
    seq = pfsynth.Sequence("S64", n_frames=20, az_steps=900)
    od = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=pfref.GPU_EQUIV)
    for k in range(8):
        p = od.frame(seq.frame(k))
    for which in (0, 1):
        xyz, rg = od.get_map(which)
        assert xyz.shape[0] > 100
        assert np.all(np.abs(xyz - p[4:].astype(np.float32)) <= 100.0 + 1e-3)
        assert rg[:, 1].max() >= 1            # p-index observed at least once


def test_bpf_tracks_and_reduces_to_es_structure(pfref, pfsynth):
    """Odom_BPF_EstimationClass restated (src/odomEstimationClass.cpp:649-1306): three maps in class
    order beam / pillar / facade, each with its own p-index bookkeeping. It tracks the generator's
    trajectory like the ES estimator on the same scans, and each class reports its own counts."""
    seq = pfsynth.Sequence("S64", n_frames=30, az_steps=1000)
    lid = pfref.make_lidar(64, 3.0, 90.0)
    od = pfref.OdomBPF(lid, 0.4, 0, 0.4, 75, 0, opts=pfref.GPU_EQUIV)
    for k in range(25):
        e, s = pfref.feature_extraction(seq.frame(k), lid, opts=pfref.FE_STABLE_TIES)
        cl = pfsynth.bpf_split(e, s)
        if k == 0:
            od.init_map(*cl)
            st = od.stats()
            assert st["n_map"] == [len(c) for c in cl]
            continue
        p = od.update(*cl)
        assert abs(np.linalg.norm(p[:4]) - 1) < 1e-14
    st = od.stats()
    assert all(n > 50 for n in st["n_res"]) and not st["map_too_small"]
    assert st["n_edge_res"] == st["n_res"][0] and st["n_surf_res"] == st["n_res"][1]
    assert np.linalg.norm(p[4:] - seq.gt_pose(24)[4:]) < 0.2
    # the per-class maps stay separate: each rgbds output is voxel-unique at its own leaf
    for c, leaf in ((0, 0.4), (1, 0.4), (2, 0.8)):
        xyz, rg = od.get_map(c)
        assert xyz.shape[0] == st["n_map"][c] and (rg[:, 0] >= 2).all()


def test_synced_parity_worker_reproduces_a_free_run(pfref, pfsynth):
    """The synced parity test's worker (tests/_parity_worker.py) rebuilds a fresh oracle from a state
    (maps with their r / g bytes, odom / last_odom poses, optimization_count) and runs one frame: fed
    the states of a free-running faithful oracle it must give that oracle's next frame (to the 1e-16
    the quaternion round trip of the state leaves), counts and map bytes identical."""
    import _parity_worker as pw
    from _util import pose_err
    n = 14
    lid, prm = (64, 3.0, 90.0), (0.4, 0, 0.4, 75, 0)
    pw.init("S64", n, 0, lid, None, prm, 0)
    seq = pfsynth.Sequence("S64", n_frames=n, seed=0)
    orc = pfref.Odom(pfref.make_lidar(*lid), *prm, opts=0)
    poses = [orc.frame(seq.frame(0))]
    report = dict(frames=0, worst_t=0.0, worst_r=0.0, worst_xyz=0.0, xyz_bitexact_frames=0, pose_bad=[],
                  count_bad=[], map_bad=[])
    for k in range(1, n):
        maps = [orc.get_map(0), orc.get_map(1)]
        opt = 12 if k == 1 else max(2, 13 - k)
        task = (k, maps, poses[k - 1], poses[max(k - 2, 0)], opt)
        pose = orc.frame(seq.frame(k))
        poses.append(pose)
        st = orc.stats()
        _, wp, wc, wm = pw.run(task)
        pw.compare(k, (pose, {c: int(st[c]) for c in pw.COUNTS}, [orc.get_map(0), orc.get_map(1)]),
                   (wp, wc, wm), report, 1e-12, 1e-12, pose_err, tol_xyz=1e-4)
    assert report["frames"] == n - 1 and report["worst_xyz"] < 1e-4
    assert not report["pose_bad"] and not report["count_bad"] and not report["map_bad"]
