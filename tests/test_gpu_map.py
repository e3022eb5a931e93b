"""GPU: LaserMappingClass (src/laserMappingClass.cpp) through the C ABI (pf_map_*) against the oracle.
Transform, cube assignment, per-cube VoxelGrid and getMap order are float/integer work restated
operation for operation on both sides, so the maps must be identical bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _filtered(pfref, x):
    """/velodyne_points_filtered: featureExtraction's edge + surf (src/laserProcessingNode.cpp:82-84)"""
    e, s = pfref.feature_extraction(x, pfref.make_lidar(64, 3.0, 90.0), opts=pfref.FE_STABLE_TIES)
    return np.concatenate([e, s]).astype(np.float32)


def _pair(pa, pfref, leaf=0.4):
    g = pa.LaserMappingClass(max_points=1 << 22, max_scan=200000)
    g.init(leaf)
    return g, pfref.GlobalMap(leaf)


def test_sequence_matches_oracle(pa, pfref, pfsynth):
    seq = pfsynth.Sequence("S64", n_frames=40, az_steps=1000)
    g, o = _pair(pa, pfref)
    for k in range(0, 40, 3):                        # 13 frames, ~36 m of travel
        x, p = _filtered(pfref, seq.frame(k)), seq.gt_pose(k)
        g.updateCurrentPointsToMap(x, p)
        assert o.update(x, p) == 0
        if k % 9 == 0 or k == 39:
            np.testing.assert_array_equal(g.getMap(), o.get())
    np.testing.assert_array_equal(g.getMap(), o.get())
    assert len(o.get()) > 5000


def test_far_travel_and_leafs(pa, pfref):
    """Poses crossing cube boundaries (neighbourhood moves, earlier cubes stay as they are), a coarse
    and a fine leaf, and a scan reaching an allocated cube outside the current neighbourhood."""
    rng = np.random.default_rng(5)
    for leaf in (1.0, 0.2):
        g, o = _pair(pa, pfref, leaf)
        for f in range(8):
            yaw = 0.4 * f
            pose = np.array([0, 0, np.sin(yaw / 2), np.cos(yaw / 2), 30.0 * f, -12.0 * f, 0.5 * f])
            r, a = rng.uniform(3, 90, 3000), rng.uniform(0, 2 * np.pi, 3000)   # within max_dis, as the node's input
            x = np.c_[r * np.cos(a), r * np.sin(a), rng.uniform(-3, 10, 3000), rng.uniform(0, 1, 3000)]
            x = x.astype(np.float32)
            g.updateCurrentPointsToMap(x, pose)
            assert o.update(x, pose) == 0
        np.testing.assert_array_equal(g.getMap(), o.get())
        back = np.array([[-10.0, 0, 0, 0]], np.float32)              # cube (1, ...) from a later pose: allocated
        pose = np.array([0, 0, 0, 1, 200.0, -84.0, 3.5])
        g.updateCurrentPointsToMap(back, pose)
        assert o.update(back, pose) == 0
        np.testing.assert_array_equal(g.getMap(), o.get())


def test_rejects_unallocated_cube(pa, pfref):
    g, o = _pair(pa, pfref)
    x = np.array([[1.0, 2.0, 0.0, 0.0]], np.float32)
    ident = np.array([0, 0, 0, 1, 0, 0, 0.0])
    g.updateCurrentPointsToMap(x, ident)
    o.update(x, ident)
    far = np.array([[400.0, 0, 0, 0]], np.float32)
    with pytest.raises(pa.PFError):
        g.updateCurrentPointsToMap(far, ident)
    assert o.update(far, ident) == -1
    np.testing.assert_array_equal(g.getMap(), o.get())               # unchanged


def test_device_entry_point(pa, pfref, pfsynth):
    seq = pfsynth.Sequence("S64", n_frames=6, az_steps=800)
    a = pa.LaserMappingClass(max_points=1 << 21, max_scan=200000)
    a.init(0.4)
    b = pa.LaserMappingClass(max_points=1 << 21, max_scan=200000)
    b.init(0.4)
    buf = pa.DeviceBuffer(16 * 200000)
    for k in range(6):
        x, p = _filtered(pfref, seq.frame(k)), seq.gt_pose(k)
        a.updateCurrentPointsToMap(x, p)
        buf.upload(np.ascontiguousarray(x, np.float32))
        pose = np.ascontiguousarray(p, np.float64)
        assert pa.lib().pf_map_update_device(b._h, buf.ptr, x.shape[0], pose.ctypes.data) == 0
    np.testing.assert_array_equal(a.getMap(), b.getMap())


def test_edge_cases(pa, pfref):
    """Empty scans, a scan above max_scan and a map above max_points (PF_ECAPACITY, map unchanged)."""
    g, o = _pair(pa, pfref)
    ident = np.array([0, 0, 0, 1, 0, 0, 0.0])
    empty = np.zeros((0, 4), np.float32)
    g.updateCurrentPointsToMap(empty, ident)
    assert o.update(empty, ident) == 0
    assert g.getMap().shape == (0, 4)
    rng = np.random.default_rng(9)
    x = np.c_[rng.uniform(-20, 20, (500, 3)), np.zeros(500)].astype(np.float32)
    g.updateCurrentPointsToMap(x, ident)
    o.update(x, ident)
    np.testing.assert_array_equal(g.getMap(), o.get())
    small = pa.LaserMappingClass(max_points=100, max_scan=50)
    small.init(0.4)
    with pytest.raises(pa.PFError):
        small.updateCurrentPointsToMap(x[:60], ident)                  # above max_scan
    small.updateCurrentPointsToMap(x[:50], ident)
    small.updateCurrentPointsToMap(x[50:100], ident)
    n = small.getMap().shape[0]
    with pytest.raises(pa.PFError):
        for k in range(2, 10):                                        # the map outgrows max_points
            small.updateCurrentPointsToMap(x[50 * k:50 * k + 50] + np.float32(0.01 * k), ident)
    assert small.getMap().shape[0] >= n
