"""GPU: Odom_ES_EstimationClass (src/odomEstimationClass.cpp:182-647) through the C ABI against the
oracle. The handles run the library default, the reference tie order (std::sort's order of equal keys
in VoxelGrid / rgbds / the sector sort), against the oracle with the same sort order and the device's
normal-equation LM step (opts = LM_NORMAL_EQ); tests marked "stable" run the stable-sort mode
(pf_odom_set_tie_order off) against GPU_EQUIV (stable tie orders + normal-equation LM).

Tolerances (BASELINE.json north_star): pose within 1e-4 m / 1e-5 rad per frame. Integer work —
down-sampled counts, residual counts, map sizes, ages / p-index bytes — must be identical. Map
coordinates are f32 results of f64 pose arithmetic: they agree within the pose tolerance (the only
arithmetic difference is the summation order of the 6x6 normal equations, ~1e-12 relative per
frame, so most map coordinates are bit-identical)."""
import ctypes

import numpy as np
import pytest

from _util import pose_err

pytestmark = pytest.mark.gpu

TOL_T, TOL_R = 1e-4, 1e-5
COUNTS = ("n_edge_ds", "n_surf_ds", "n_edge_map", "n_surf_map", "n_edge_res", "n_surf_res", "n_edge_valid",
          "n_surf_valid", "outer_iterations", "map_too_small")


def _pair(pa, pfref, lines=64, map_res=0.4, k_new=0, theta_p=0.4, theta_max=75, wt=0, mn=3.0, mx=90.0, order="tie"):
    tie = order == "tie"
    od = pa.Odom_ES_EstimationClass(device=0, tie_order=None if tie else False)
    od.init(pa.make_lidar(lines, mn, mx), map_res, k_new, theta_p, theta_max, wt)
    orc = pfref.Odom(pfref.make_lidar(lines, mn, mx), map_res, k_new, theta_p, theta_max, wt,
                     opts=pfref.LM_NORMAL_EQ if tie else pfref.GPU_EQUIV)
    return od, orc


def _compare_maps(od, orc):
    for which, (gx, grg) in ((0, od.laserCloudCornerMap), (1, od.laserCloudSurfMap)):
        rx, rrg = orc.get_map(which)
        assert gx.shape == rx.shape, (which, gx.shape, rx.shape)
        np.testing.assert_allclose(gx, rx, rtol=0, atol=TOL_T)
        np.testing.assert_array_equal(grg, rrg)


def _run(od, orc, seq, frames, check_maps_every=0):
    worst = (0.0, 0.0)
    for i, k in enumerate(frames):
        x = seq.frame(k)
        pg = od.frame_host(x)
        pr = orc.frame(x)
        dt, dr = pose_err(pg, pr)
        worst = (max(worst[0], dt), max(worst[1], dr))
        assert dt < TOL_T and dr < TOL_R, "frame %d: %.3e m %.3e rad" % (k, dt, dr)
        if i > 0:
            sg, sr = od.stats(), orc.stats()
            for c in COUNTS:
                assert sg[c] == sr[c], (k, c, sg[c], sr[c])
        if check_maps_every and i % check_maps_every == 0:
            _compare_maps(od, orc)
    return worst


@pytest.mark.parametrize("order", ["tie", "stable"])
def test_pose_and_map_parity_kitti_config(pa, pfref, pfsynth, order):
    """configs[1]: 64 lines, k_new 0, theta_p 0.4, theta_max 75, weightType 0, map_res 0.4."""
    seq = pfsynth.Sequence("S64", n_frames=60)
    od, orc = _pair(pa, pfref, order=order)
    worst = _run(od, orc, seq, range(40), check_maps_every=13)
    _compare_maps(od, orc)
    assert worst[0] < 1e-6 and worst[1] < 1e-7


@pytest.mark.parametrize("wt", [1, 2, 12])
def test_weight_types(pa, pfref, pfsynth, wt):
    """weightType 1 / 2 / 12 (include/odomEstimationClass.h:111-126; 2 is pfilter_kitti.launch:7's
    default) free-running against the oracle over 120 frames, maps every 17th; weightType 2 also has a
    whole-sequence synced case (tests/test_gpu_parity_synced.py configs1_S64_wt2)."""
    seq = pfsynth.Sequence("S64", n_frames=130, az_steps=1200)
    od, orc = _pair(pa, pfref, wt=wt)
    _run(od, orc, seq, range(120), check_maps_every=17)
    _compare_maps(od, orc)


@pytest.mark.parametrize("k_new,theta_p,theta_max", [(0, 0.0, 0), (2, 0.4, 75), (1, 0.8, 30)])
def test_pindex_configs(pa, pfref, pfsynth, k_new, theta_p, theta_max):
    """theta_p 0 = plain FLOAM map (no p-index filter); k_new > 0 keeps young map points."""
    seq = pfsynth.Sequence("S64", n_frames=20, az_steps=1200)
    od, orc = _pair(pa, pfref, k_new=k_new, theta_p=theta_p, theta_max=theta_max)
    _run(od, orc, seq, range(12), check_maps_every=11)


def test_campus_32_line(pa, pfref, pfsynth):
    """configs[2]: 32-line campus scan (launch/pfilter.launch: min/max 3/90), theta_p 1, theta_max 200."""
    seq = pfsynth.Sequence("S32", n_frames=20)
    od, orc = _pair(pa, pfref, lines=32, theta_p=1.0, theta_max=200)
    _run(od, orc, seq, range(12), check_maps_every=11)


@pytest.mark.parametrize("map_res", [0.15, 0.25])
def test_rgbds_key_grids(pa, pfref, pfsynth, map_res):
    """The two rgbds key paths of addPointsToMap (pf_odom.hip): map_res 0.25 keys on the crop box's
    voxel grid in the fused append+keys launch; at 0.15 that grid would overflow the 30 key bits
    (rg_fused_keys), so the min/max pass and the reference's own key grid run. Both sort as the
    reference does: counts, maps and poses against the oracle."""
    seq = pfsynth.Sequence("S64", n_frames=20, az_steps=1200)
    od, orc = _pair(pa, pfref, map_res=map_res)
    _run(od, orc, seq, range(12), check_maps_every=11)
    _compare_maps(od, orc)


@pytest.mark.parametrize("theta_p,theta_max", [(0.4, 75), (0.0, 0)])
def test_dense_vegetation_scene(pa, pfref, pfsynth, theta_p, theta_max):
    """S64V (bench.py's dense legs): porous tree crowns, hedges and rough ground give about twice the
    down-sampled surf points of S64 and, at theta = 0, maps of 4e4-9e4 points (SURVEY §8 KITTI sizes)."""
    seq = pfsynth.Sequence("S64V", n_frames=40)
    od, orc = _pair(pa, pfref, theta_p=theta_p, theta_max=theta_max)
    _run(od, orc, seq, range(30), check_maps_every=14)
    _compare_maps(od, orc)


def test_per_frame_parity_vs_reference_faithful_oracle(pa, pfref, pfsynth):
    """The north star's per-frame criterion against the oracle's reference-faithful option set
    (opts=0: libstdc++ std::sort tie order in VoxelGrid / rgbds / the sector sort as PCL and
    src/odomEstimationClass.cpp:74 call it, Householder-QR LM as Ceres DENSE_QR, the FLANN-style
    kd-tree): on identical input clouds and an identical estimator state, the device pose within
    1e-4 m / 1e-5 rad. The faithful oracle runs the sequence itself; before every sampled frame its
    maps (with the age / p-index bytes) and its odom / last_odom / optimization_count are loaded into
    the device handle (pf_odom_set_map, pf_odom_set_state) and into the oracle alike, then both run
    the frame. (Over whole sequences the two tie orders make trajectories separate after ~50 frames,
    as any change of sort implementation would make the reference's own: tools/parity_report.py.)"""
    n = 300
    sample = set(range(12, n, 12))
    seq = pfsynth.Sequence("S64", n_frames=n)
    lid = 64, 3.0, 90.0
    orc = pfref.Odom(pfref.make_lidar(*lid), 0.4, 0, 0.4, 75, 0, opts=0)
    od = pa.Odom_ES_EstimationClass(device=0)
    od.init(pa.make_lidar(*lid), 0.4, 0, 0.4, 75, 0)
    poses, worst, same_counts = [], (0.0, 0.0), 0
    for k in range(n):
        x = seq.frame(k)
        if k in sample:
            for which in (0, 1):
                xyz, rg = orc.get_map(which)
                od.set_map(which, xyz, rg)
            od.set_state(poses[-1], poses[-2], 2)
            orc.set_state(poses[-1], poses[-2])
            orc.set_opt_count(2)
            pg = od.frame_host(x)
        pr = orc.frame(x)
        poses.append(pr)
        if k in sample:
            dt, dr = pose_err(pg, pr)
            worst = (max(worst[0], dt), max(worst[1], dr))
            assert dt < TOL_T and dr < TOL_R, "frame %d: %.3e m %.3e rad" % (k, dt, dr)
            sg, sr = od.stats(), orc.stats()
            same_counts += all(sg[c] == sr[c] for c in ("n_edge_ds", "n_surf_ds", "n_edge_map", "n_surf_map"))
    print("per-frame parity vs the faithful oracle: %d frames, worst %.3e m %.3e rad, counts identical in %d"
          % (len(sample), worst[0], worst[1], same_counts))
    assert same_counts == len(sample)


def test_stage_timing(pa, pfsynth):
    """pf_odom_set_stage_timing / pf_odom_stage_times: per-stage device time over the frames since
    enable; results unchanged by the event records."""
    seq = pfsynth.Sequence("S64", n_frames=30, az_steps=1500)
    buf, counts = seq.frames(0, 30)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    ptr = lambda k: (db.ptr + k * buf.shape[1] * 16, int(counts[k]))
    runs = []
    for timing in (False, True):
        od = pa.Odom_ES_EstimationClass(device=0)
        od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
        for k in range(12):
            od.frame_device(*ptr(k))
        if timing:
            od.set_stage_timing(True)
        for k in range(12, 30):
            od.frame_device(*ptr(k))
        od.sync()
        runs.append(od.poses())
        if timing:
            st = od.stage_times()
            assert st["frames"] == 18
            assert 5.0 < st["a_us"] < 5e4 and 5.0 < st["b_us"] < 5e4, st
            od.set_stage_timing(False)
            assert od.stage_times()["frames"] == 0
    np.testing.assert_array_equal(runs[0], runs[1])


def test_update_api_matches_oracle(pa, pfref, pfsynth):
    """initMapWithPoints / updatePointsToMap with host-side features (the node's call pattern)."""
    seq = pfsynth.Sequence("S64", n_frames=10, az_steps=1500)
    lid = pfref.make_lidar(64, 3.0, 90.0)
    od, orc = _pair(pa, pfref)
    for k in range(6):
        e, s = pfref.feature_extraction(seq.frame(k), lid, opts=pfref.FE_STABLE_TIES)
        if k == 0:
            od.initMapWithPoints(e, s)
            orc.init_map(e, s)
            continue
        pg = od.updatePointsToMap(e, s)
        pr = orc.update(e, s)
        dt, dr = pose_err(pg, pr)
        assert dt < TOL_T and dr < TOL_R
        np.testing.assert_array_equal(pg, od.odom)
    _compare_maps(od, orc)


def test_small_capacity_handle_tie_order(pa, pfref, pfsynth):
    """A handle with small caps (max_points 2000, map_capacity 10000: rgbds sort capacity 24000, so the
    dependence table's own size would be 2^15 slots, below the 2^16 the small-table path hashes into)
    in the default tie order, fed sub-sampled features through the update API for 12 frames: poses,
    every count and both maps (xyz within the tolerance, age / p-index bytes identical) against the
    oracle, and the same bits as a default-capacity handle (the table is now never smaller
    than the small path's 2^16 slots)."""
    seq = pfsynth.Sequence("S64", n_frames=12, az_steps=1000)
    lid = pfref.make_lidar(64, 3.0, 90.0)
    small = pa.Odom_ES_EstimationClass(device=0, max_points=2000, map_capacity=10000)
    small.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    big, orc = _pair(pa, pfref)
    for k in range(12):
        e, s = pfref.feature_extraction(seq.frame(k), lid, opts=0)
        e = e[:: max(1, -(-len(e) // 1500))][:2000]
        s = s[:: max(1, -(-len(s) // 1500))][:2000]
        if k == 0:
            for od in (small, big):
                od.initMapWithPoints(e, s)
            orc.init_map(e, s)
            continue
        ps = small.updatePointsToMap(e, s)
        pb = big.updatePointsToMap(e, s)
        pr = orc.update(e, s)
        np.testing.assert_array_equal(ps, pb)
        dt, dr = pose_err(ps, pr)
        assert dt < TOL_T and dr < TOL_R, (k, dt, dr)
        ss, sr = small.stats(), orc.stats()
        for c in COUNTS:
            assert ss[c] == sr[c], (k, c, ss[c], sr[c])
        assert ss["errors"] == 0
    _compare_maps(small, orc)
    for a, b in ((small.laserCloudCornerMap, big.laserCloudCornerMap),
                 (small.laserCloudSurfMap, big.laserCloudSurfMap)):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


def test_device_pipeline_graph_equals_eager(pa, pfsynth):
    """hipGraph replay of the steady-state frame gives the same bits as eager launches, for every
    graph mode (pf_odom_set_graph: stage A, stage B, both)."""
    seq = pfsynth.Sequence("S64", n_frames=30, az_steps=1500)
    buf, counts = seq.frames(0, 30)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    stride = buf.shape[1] * 16
    res = []
    for graph in (3, 1, 2, 0):
        od = pa.Odom_ES_EstimationClass(device=0)
        od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
        od.set_graph(graph)
        for k in range(30):
            od.frame_device(db.ptr + k * stride, counts[k])
        od.sync()
        res.append((od.poses(), od.laserCloudSurfMap))
    for r in res[:-1]:
        np.testing.assert_array_equal(r[0], res[-1][0])
        np.testing.assert_array_equal(r[1][0], res[-1][1][0])
        np.testing.assert_array_equal(r[1][1], res[-1][1][1])


def test_map_too_small_warning(pa, pfref):
    """|M_e| <= 10 or |M_s| <= 50: the solve is skipped and the prediction kept (.cpp:247, 274-277)."""
    rng = np.random.default_rng(0)
    e = np.zeros((5, 4), np.float32)
    e[:, :3] = rng.uniform(-5, 5, (5, 3))
    s = np.zeros((30, 4), np.float32)
    s[:, :3] = rng.uniform(-5, 5, (30, 3))
    od, orc = _pair(pa, pfref)
    od.initMapWithPoints(e, s)
    orc.init_map(e, s)
    pg = od.updatePointsToMap(e, s)
    pr = orc.update(e, s)
    assert od.last_status == pa.PF_W_MAP_TOO_SMALL
    assert od.stats()["map_too_small"] == 1 and orc.stats()["map_too_small"] == 1
    np.testing.assert_allclose(pg, pr, atol=1e-12)


def test_set_get_map_roundtrip(pa):
    od = pa.Odom_ES_EstimationClass(device=0)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    rng = np.random.default_rng(1)
    xyz = rng.uniform(-50, 50, (1000, 3)).astype(np.float32)
    rg = rng.integers(0, 256, (1000, 2)).astype(np.uint8)
    od.set_map(1, xyz, rg)
    gx, grg = od.laserCloudSurfMap
    np.testing.assert_array_equal(gx, xyz)
    np.testing.assert_array_equal(grg, rg)
    assert od.laserCloudCornerMap[0].shape[0] == 0


def test_invalid_arguments(pa):
    od = pa.Odom_ES_EstimationClass(device=0)
    with pytest.raises(pa.PFError) as ei:
        od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 3)      # weightType 3
    assert ei.value.code == pa.PF_EINVAL
    od = pa.Odom_ES_EstimationClass(device=0, max_points=500)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    with pytest.raises(pa.PFError) as ei:
        od.frame_host(np.ones((501, 4), np.float32))
    assert ei.value.code == pa.PF_ECAPACITY
    L = pa.lib()
    assert L.pf_odom_update(None, None, 0, 16, None, 0, 16, None) == pa.PF_EINVAL
    assert L.pf_odom_get_map(od._h, 2, None, None, 0, ctypes.byref(ctypes.c_size_t())) == pa.PF_EINVAL


def test_long_sequence_matches_oracle(pa, pfref, pfsynth):
    """Full-size S64 through the device pipeline (hipGraph replay): 400 frames with the heading
    passing 90 degrees, every pose within the north-star tolerance of the oracle, |q| = 1."""
    n = 400
    seq = pfsynth.Sequence("S64", n_frames=n)
    od = pa.Odom_ES_EstimationClass(device=0)           # the library default: reference tie order
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    orc = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=pfref.LM_NORMAL_EQ)
    ref = []
    for f0 in range(0, n, 100):
        buf, counts = seq.frames(f0, 100)
        db = pa.DeviceBuffer(buf.nbytes)
        db.upload(buf)
        for i in range(100):
            od.frame_device(db.ptr + i * buf.shape[1] * 16, counts[i])
            ref.append(orc.frame(buf[i, :counts[i]]))
        od.sync()
        db.free()
    p = od.poses()
    assert p.shape == (n, 7)
    for k in range(n):
        dt, dr = pose_err(p[k], ref[k])
        assert dt < TOL_T and dr < TOL_R, "frame %d: %.3e m %.3e rad" % (k, dt, dr)
    np.testing.assert_allclose(np.linalg.norm(p[:, :4], axis=1), 1.0, atol=1e-12)
    gt = np.array([seq.gt_pose(k) for k in range(n)])
    assert np.max(2 * np.arctan2(gt[:, 2], gt[:, 3])) > 1.5          # heading passed 90 degrees
    assert np.linalg.norm(p[-1, 4:6] - gt[-1, 4:6]) < 0.01 * 400.0     # planar drift < 1 %


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_full_sequence_bench_path(pa, pfsynth):
    """Stable order. configs[1] end to end through bench.py's own path: all 4541 S64 seed-0 scans HBM-resident,
    pf_odom_frame_device per frame with hipGraph replay, no host round trip. Against the committed
    oracle trajectory (tests/golden/odom_s64_full.npz, GPU_EQUIV): every frame's pose within the
    north-star 1e-4 m / 1e-5 rad (the design target is bit-identity: the device's LM reduction tree
    and SE(3) sincos are restated in the oracle), every frame's counts identical (a second handle
    reads them after each frame) and the final maps identical byte for byte."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "odom_s64_full.npz"))
    n = g["poses"].shape[0]
    names = [str(c) for c in g["count_names"]]
    seq = pfsynth.Sequence("S64", n_frames=n, seed=0)
    lid = pa.make_lidar(64, 3.0, 90.0)
    bench_h = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22, tie_order=False)
    bench_h.init(lid, 0.4, 0, 0.4, 75, 0)
    count_h = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22, tie_order=False)
    count_h.init(lid, 0.4, 0, 0.4, 75, 0)
    checks = dict(zip((int(k) for k in g["input_frames"]), (str(h) for h in g["input_sha"])))
    bufs, bad_counts = [], []
    for f0 in range(0, n, 256):
        nf = min(256, n - f0)
        buf, cnt = seq.frames(f0, nf, threads=16)
        for i in range(nf):
            if f0 + i in checks:
                assert _sha(buf[i, :cnt[i]]) == checks[f0 + i], "generator output changed at frame %d" % (f0 + i)
        db = pa.DeviceBuffer(buf.nbytes)
        db.upload(buf)
        bufs.append(db)
        stride = buf.shape[1] * 16
        for i in range(nf):
            bench_h.frame_device(db.ptr + i * stride, int(cnt[i]))
            count_h.frame_device(db.ptr + i * stride, int(cnt[i]))
            st = count_h.stats()
            got = [st[c] for c in names]
            if f0 + i > 0 and got != list(g["counts"][f0 + i]) and len(bad_counts) < 5:
                bad_counts.append((f0 + i, got, list(g["counts"][f0 + i])))
    bench_h.sync()
    p = bench_h.poses()
    assert p.shape == (n, 7)
    ref = g["poses"]
    errs = np.array([pose_err(p[k], ref[k]) for k in range(n)])
    exact = int(np.sum(np.all(p == ref, axis=1)))
    first = next((k for k in range(n) if not np.array_equal(p[k], ref[k])), None)
    print("full sequence: %d / %d frames bit-identical (first difference: %s); worst %.3e m %.3e rad"
          % (exact, n, first, errs[:, 0].max(), errs[:, 1].max()))
    bad = np.nonzero((errs[:, 0] >= TOL_T) | (errs[:, 1] >= TOL_R))[0]
    assert bad.size == 0, "frame %d: %.3e m %.3e rad" % (bad[0], errs[bad[0], 0], errs[bad[0], 1])
    assert not bad_counts, bad_counts
    np.testing.assert_array_equal(count_h.poses(), p)                 # per-frame reads change nothing
    ex, er = bench_h.laserCloudCornerMap
    sx, sr = bench_h.laserCloudSurfMap
    assert [ex.shape[0], sx.shape[0]] == list(g["map_sizes"])
    assert [_sha(ex), _sha(er), _sha(sx), _sha(sr)] == [str(h) for h in g["map_sha"]]
    for db in bufs:
        db.free()


def test_golden_trajectory(pa):
    """Stable order: the device pipeline against the committed GPU_EQUIV oracle trajectory
    (tests/golden/odom_s64_24f.npz)."""
    import os
    import pfsynth
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "odom_s64_24f.npz"))
    seq = pfsynth.Sequence("S64", n_frames=30, az_steps=1000)
    od = pa.Odom_ES_EstimationClass(device=0, tie_order=False)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    for k in range(24):
        p = od.frame_host(seq.frame(k))
        dt, dr = pose_err(p, g["gpu_equiv_poses"][k])
        assert dt < TOL_T and dr < TOL_R, (k, dt, dr)
        st = od.stats()
        got = [st[c] for c in ("n_edge_in", "n_surf_in", "n_edge_ds", "n_surf_ds", "n_edge_map", "n_surf_map",
                               "n_edge_res", "n_surf_res")]
        if k > 0:
            assert got == list(g["gpu_equiv_counts"][k]), (k, got)


def test_reset_replays_like_a_fresh_handle(pa, pfsynth):
    """pf_odom_reset: the same frames after a reset give the bits of a fresh handle."""
    seq = pfsynth.Sequence("S64", n_frames=12, az_steps=1200)
    frames = [seq.frame(k) for k in range(12)]
    od = pa.Odom_ES_EstimationClass(device=0)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    first = [od.frame_host(x) for x in frames]
    od.reset()
    again = [od.frame_host(x) for x in frames]
    np.testing.assert_array_equal(np.array(first), np.array(again))
    assert od.poses().shape == (12, 7)


def _run_handle(pa, db, row_floats, counts, reserve=None):
    od = pa.Odom_ES_EstimationClass(device=0)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    if reserve is not None:
        od.set_stage_a_reserve(reserve)
    for i in range(len(counts)):
        od.frame_device(db.ptr + i * row_floats * 4, counts[i])
    od.sync()                                       # raises on any sticky device error
    poses = od.poses()
    assert od.stats()["errors"] == 0
    return od, poses


@pytest.mark.parametrize("reserve", [None, 0])
def test_concurrent_handles_match_solo_runs(pa, pfsynth, reserve):
    """configs[3] mode: 12 handles (one sequence each, own host thread, own streams) on one device at
    once — more LM solves in flight than the CUs could hold as co-resident 32-workgroup grids, the
    case that deadlocked before the LM claimed its chunks dynamically (pf_odom.hip k_lm_solve). Every
    trajectory is bit-identical to the same sequence run alone; no sticky error word is raised.
    reserve None = the default stage-A CU mask (128 CUs kept free), 0 = unrestricted."""
    import threading
    n_handles, n_frames = 12, 40
    seqs = []
    for s in range(n_handles):
        seq = pfsynth.Sequence("S64", n_frames=n_frames, az_steps=900, seed=s)
        buf, counts = seq.frames(0, n_frames)
        db = pa.DeviceBuffer(buf.nbytes)
        db.upload(buf)
        seqs.append((db, buf.shape[1] * 4, counts))
    solo = []
    for db, row, counts in seqs:
        od, p = _run_handle(pa, db, row, counts, reserve)
        solo.append(p)
        del od
    out = [None] * n_handles
    errs = []
    start = threading.Barrier(n_handles)

    def work(k):
        try:
            db, row, counts = seqs[k]
            od = pa.Odom_ES_EstimationClass(device=0)
            od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
            if reserve is not None:
                od.set_stage_a_reserve(reserve)
            start.wait()
            for i in range(len(counts)):
                od.frame_device(db.ptr + i * row * 4, counts[i])
            od.sync()
            out[k] = od.poses()
            assert od.stats()["errors"] == 0
            del od
        except Exception as e:                      # reported below, in the main thread
            errs.append((k, repr(e)))

    th = [threading.Thread(target=work, args=(k,)) for k in range(n_handles)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a handle thread did not finish"
    assert not errs, errs
    for k in range(n_handles):
        np.testing.assert_array_equal(out[k], solo[k], err_msg="handle %d" % k)
    for db, _, _ in seqs:
        db.free()


def test_stage_a_reservation_does_not_change_results(pa, pfsynth):
    """The stage-A CU mask (default 128 reserved CUs, pf_odom_set_stage_a_reserve) only moves work
    between CUs: the same 16 frames give the same bits with the default, with 0 and with 64."""
    seq = pfsynth.Sequence("S64", n_frames=16, az_steps=1000)
    buf, counts = seq.frames(0, 16)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    runs = []
    for reserve in (None, 0, 64):
        od = pa.Odom_ES_EstimationClass(device=0)
        od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
        if reserve is not None:
            od.set_stage_a_reserve(reserve)
        for i in range(16):
            od.frame_device(db.ptr + i * buf.shape[1] * 16, counts[i])
        od.sync()
        runs.append(od.poses())
        del od
    np.testing.assert_array_equal(runs[0], runs[1])
    np.testing.assert_array_equal(runs[0], runs[2])
    with pytest.raises(pa.PFError):
        od = pa.Odom_ES_EstimationClass(device=0)
        od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
        od.set_stage_a_reserve(-1)


def test_s128_odometry_with_2m_point_map(pa, pfref, pfsynth):
    """configs[4] as a pipeline: synthetic 128-line scans (~200k points) through featureExtraction
    with the linear beam-model extension (pf_odom_set_ring_model(15, -25): the reference has no
    128-line ring formula) and updatePointsToMap against a 2,000,000-point surf
    map seeded by pf_odom_set_map (voxel centroids of the dense synthetic block at the 0.8 m surf leaf,
    a fixed point of rgbds). FLOAM parameters (theta_p 0) keep the map at its size. Poses within the
    tolerance and every count identical per frame; both maps compared at the end. Stable order (the
    reference tie order at this size: tests/test_gpu_parity_synced.py::test_synced_parity_s128_2m_point_map_tie)."""
    seq = pfsynth.Sequence("S128", n_frames=16)
    od = pa.Odom_ES_EstimationClass(device=0, tie_order=False)
    od.init(pa.make_lidar(128, 3.0, 90.0, ring_model=(15.0, -25.0)), 0.4, 0, 0.0, 0, 0)
    orc = pfref.Odom(pfref.make_lidar(128, 3.0, 90.0, ring_model=(15.0, -25.0)), 0.4, 0, 0.0, 0, 0,
                     opts=pfref.GPU_EQUIV)
    x = seq.frame(0)
    assert x.shape[0] > 150000
    od.frame_host(x)
    orc.frame(x)
    m = pfref.rgbds(pfsynth.dense_map(7_000_000, seed=5), 0.8)[:2_000_000, :3]
    assert m.shape[0] == 2_000_000
    rg = np.zeros((m.shape[0], 2), np.uint8)
    od.set_map(1, m, rg)
    orc.set_map(1, m, rg)
    worst = _run(od, orc, seq, range(1, 13))
    st = od.stats()
    assert st["n_surf_map"] > 1_900_000 and st["n_surf_res"] > 500 and st["n_edge_res"] > 500
    _compare_maps(od, orc)
    assert worst[0] < TOL_T and worst[1] < TOL_R


def test_snapshot_restore_continues_bit_identically(pa, pfsynth):
    """pf_odom_snapshot after frame 6, pf_odom_restore into a fresh handle: frames 7..13 give the
    bits of the uninterrupted run (poses, both maps with their age / p-index bytes, the
    OdomBaseClass members); a snapshot does not load into a handle with other parameters."""
    seq = pfsynth.Sequence("S64", n_frames=14, az_steps=1200)
    frames = [seq.frame(k) for k in range(14)]
    a = pa.Odom_ES_EstimationClass(device=0)
    a.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    for k in range(7):
        a.frame_host(frames[k])
    blob = a.snapshot()
    st6, pose6 = a.state(), a.odom
    want = [a.frame_host(x) for x in frames[7:]]
    b = pa.Odom_ES_EstimationClass(device=0)
    b.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    b.restore(blob)
    np.testing.assert_array_equal(b.odom, pose6)
    s = b.state()
    np.testing.assert_array_equal(s["parameters"], st6["parameters"])
    assert s["optimization_count"] == st6["optimization_count"]
    got = [b.frame_host(x) for x in frames[7:]]
    np.testing.assert_array_equal(np.array(got), np.array(want))
    for which in (0, 1):
        np.testing.assert_array_equal(b._map(which)[0], a._map(which)[0])
        np.testing.assert_array_equal(b._map(which)[1], a._map(which)[1])
    c = pa.Odom_ES_EstimationClass(device=0)
    c.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.0, 0, 0)           # other theta_p / theta_max
    with pytest.raises(pa.PFError):
        c.restore(blob)


def test_map_export_equals_get_map(pa, pfsynth):
    """pf_odom_set_map_export: the maps written into pinned host memory at the end of every frame
    (graph replay and the update API) equal pf_odom_get_map's copy, every frame."""
    seq = pfsynth.Sequence("S64", n_frames=12, az_steps=1000)
    od = pa.Odom_ES_EstimationClass(device=0)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    od.set_map_export(True)
    for k in range(12):
        od.frame_host(seq.frame(k))
        for which in (0, 1):
            ex, er = od.map_export(which)
            gx, gr = od._map(which)
            np.testing.assert_array_equal(ex, gx)
            np.testing.assert_array_equal(er, gr)


def test_probe_assoc_knn(pa, pfref, pfsynth):
    """pf_odom_probe_assoc: the association's kNN alone on the last frame changes nothing (the next
    frames give the bits of an unprobed run), and its algorithmic bytes are SURVEY 8(d)'s formula over
    the queries it returns, against each query class's own map (the grid the frame searched)."""
    seq = pfsynth.Sequence("S64", n_frames=10, az_steps=1500)
    frames = [seq.frame(k) for k in range(10)]
    runs = []
    for probe in (False, True):
        od = pa.Odom_ES_EstimationClass(device=0)
        od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
        for k in range(5):
            od.frame_host(frames[k])
        maps = [od._map(0)[0], od._map(1)[0]]                 # frame 5's grid is built from these
        od.frame_host(frames[5])
        if probe:
            ms, alg, nq, q = od.probe_assoc(iters=3, queries=True)
        for k in range(6, 10):
            od.frame_host(frames[k])
        runs.append(od.poses())
    np.testing.assert_array_equal(runs[0], runs[1])
    assert ms > 0 and nq == q.shape[0] > 1000
    cls = q[:, 3].view(np.int32)
    assert set(np.unique(cls)) == {0, 1}
    pop = sum(pfref.knn_cellpop(np.c_[maps[c], np.zeros(len(maps[c]), np.float32)],
                                np.c_[q[cls == c, :3], np.zeros(int((cls == c).sum()), np.float32)]) for c in (0, 1))
    assert alg == (16 + 40 + 216) * nq + 16 * pop


@pytest.mark.parametrize("preset,frames,bpf", [("S64", 300, False), ("S64V", 200, False), ("S64", 120, True)])
def test_fused_observe_equals_separate_launch(pa, pfsynth, preset, frames, bpf):
    """weightType 0 runs the observe pass inside k_lm_solve (chunk by chunk, k_observe not launched):
    poses, maps (r / g bytes included) and the per-frame counts must be those of the separate
    k_observe launch (development switch pf_dev_set_fuse_observe), under graph replay of both stages."""
    seq = pfsynth.Sequence(preset, n_frames=frames, seed=0)
    buf, cnt = seq.frames(0, frames, threads=16)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    out = []
    try:
        for fused in (True, False):
            if bpf:
                od = pa.Odom_BPF_EstimationClass(device=0)
            else:
                od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 21)
            od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
            od.set_graph(3)
            od.set_fuse_observe(fused)
            stats = []
            for i in range(frames):
                if bpf:
                    od.frame_scan_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
                else:
                    od.frame_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
                if i % 50 == 49:
                    st = od.stats()
                    stats.append((st["n_res"], st["n_valid"], st["n_map"], st["errors"]))
            od.sync()
            out.append((od.poses(), [od._map(w) for w in range(3 if bpf else 2)], stats))
    finally:
        db.free()
    assert np.array_equal(out[0][0], out[1][0])
    for w in range(len(out[0][1])):
        assert np.array_equal(out[0][1][w][0].view(np.uint32), out[1][1][w][0].view(np.uint32)), w
        assert np.array_equal(out[0][1][w][1], out[1][1][w][1]), w
    assert out[0][2] == out[1][2]
    assert all(s[3] == 0 for s in out[0][2])
