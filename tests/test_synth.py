"""CPU: the synthetic workload generator (KITTI-like scans; no network for KITTI itself).

Parity tests regenerate their inputs from (preset, seed, frame), so the generator must be
deterministic: independent of thread count and of the sequence length."""
import numpy as np


def test_prefix_and_thread_invariance(pfsynth):
    a = pfsynth.Sequence("S64", n_frames=20, az_steps=600)
    b = pfsynth.Sequence("S64", n_frames=400, az_steps=600)
    for k in (0, 7, 19):
        np.testing.assert_array_equal(a.frame(k), b.frame(k))
        np.testing.assert_array_equal(a.gt_pose(k), b.gt_pose(k))
    buf1, c1 = a.frames(3, 4, threads=1)
    buf4, c4 = a.frames(3, 4, threads=4)
    np.testing.assert_array_equal(c1, c4)
    for i in range(4):
        n = int(c1[i])
        np.testing.assert_array_equal(buf1[i, :n], buf4[i, :n])
        np.testing.assert_array_equal(buf1[i, :n], a.frame(3 + i))


def test_scan_geometry(pfsynth):
    s = pfsynth.Sequence("S32", n_frames=5, az_steps=900)
    x, ring = s.frame(2, with_ring=True)
    assert x.dtype == np.float32 and x.shape[1] == 4
    assert ring.min() >= 0 and ring.max() < 32
    r = np.linalg.norm(x[:, :3], axis=1)
    assert r.max() < 130.0 and r.min() > 0.5
    elev = np.degrees(np.arctan2(x[:, 2], np.hypot(x[:, 0], x[:, 1])))
    assert elev.min() > -31.5 and elev.max() < 12.0


def test_trajectory_is_smooth(pfsynth):
    s = pfsynth.Sequence("S64", n_frames=50, az_steps=400)
    p = np.array([s.gt_pose(k) for k in range(50)])
    np.testing.assert_allclose(np.linalg.norm(p[:, :4], axis=1), 1.0, atol=1e-12)
    step = np.linalg.norm(np.diff(p[:, 4:], axis=0), axis=1)
    assert np.all(step < 1.5) and np.all(step > 0.5)       # 10 m/s at 10 Hz


def test_dense_map_and_queries(pfsynth):
    m = pfsynth.dense_map(20000, seed=5)
    q = pfsynth.dense_queries(m, 1000, sigma=0.3, seed=6)
    assert m.shape == (20000, 4) and q.shape == (1000, 4)
    np.testing.assert_array_equal(m, pfsynth.dense_map(20000, seed=5))
    assert np.isfinite(q).all()
