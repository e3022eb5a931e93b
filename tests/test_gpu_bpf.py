"""GPU: Odom_BPF_EstimationClass (src/odomEstimationClass.cpp:649-1306) through the C ABI against the
oracle with the device's default sort order (libstdc++ std::sort's order of equal keys, the reference
tie order) and its normal-equation LM step (opts = LM_NORMAL_EQ). Beam / pillar / facade inputs come from pfsynth.bpf_split (a deterministic
stand-in for the reference's PCA classifier, which is outside this path: SURVEY §8(f) rank 3).

Tolerances as for the ES estimator (BASELINE.json north_star): pose within 1e-4 m / 1e-5 rad per
frame; per-class down-sampled counts, residual counts, map sizes and age / p-index bytes identical."""
import ctypes

import numpy as np
import pytest

from _util import pose_err

pytestmark = pytest.mark.gpu

TOL_T, TOL_R = 1e-4, 1e-5
CLASS_COUNTS = ("n_ds", "n_map", "n_res", "n_valid")


def _pair(pa, pfref, map_res=0.4, k_new=0, theta_p=0.4, theta_max=75, wt=0):
    od = pa.Odom_BPF_EstimationClass(device=0)
    od.init(pa.make_lidar(64, 3.0, 90.0), map_res, k_new, theta_p, theta_max, wt)
    orc = pfref.OdomBPF(pfref.make_lidar(64, 3.0, 90.0), map_res, k_new, theta_p, theta_max, wt,
                        opts=pfref.LM_NORMAL_EQ)
    return od, orc


def _inputs(pfref, pfsynth, seq, k):
    e, s = pfref.feature_extraction(seq.frame(k), pfref.make_lidar(64, 3.0, 90.0), opts=pfref.FE_STABLE_TIES)
    return pfsynth.bpf_split(e, s)


def _compare_maps(od, orc):
    for c, (gx, grg) in enumerate((od.laserCloudBeamMap, od.laserCloudPillarMap, od.laserCloudFacadeMap)):
        rx, rrg = orc.get_map(c)
        assert gx.shape == rx.shape, (c, gx.shape, rx.shape)
        np.testing.assert_allclose(gx, rx, rtol=0, atol=TOL_T)
        np.testing.assert_array_equal(grg, rrg)


def _run(od, orc, pfref, pfsynth, seq, frames, check_maps_every=0):
    worst = (0.0, 0.0)
    for i, k in enumerate(frames):
        cl = _inputs(pfref, pfsynth, seq, k)
        if i == 0:
            od.initMapWithPoints(*cl)
            orc.init_map(*cl)
            continue
        pg = od.updatePointsToMap(*cl)
        pr = orc.update(*cl)
        dt, dr = pose_err(pg, pr)
        worst = (max(worst[0], dt), max(worst[1], dr))
        assert dt < TOL_T and dr < TOL_R, "frame %d: %.3e m %.3e rad" % (k, dt, dr)
        sg, sr = od.stats(), orc.stats()
        for c in CLASS_COUNTS:
            assert sg[c] == sr[c], (k, c, sg[c], sr[c])
        assert sg["outer_iterations"] == sr["outer_iterations"] and sg["map_too_small"] == sr["map_too_small"]
        if check_maps_every and i % check_maps_every == 0:
            _compare_maps(od, orc)
    return worst


def test_bpf_parity(pa, pfref, pfsynth):
    """configs[1] parameters on the three-map estimator, 25 frames, maps compared every 8 frames."""
    seq = pfsynth.Sequence("S64", n_frames=30)
    od, orc = _pair(pa, pfref)
    worst = _run(od, orc, pfref, pfsynth, seq, range(25), check_maps_every=8)
    _compare_maps(od, orc)
    assert worst[0] < 1e-6 and worst[1] < 1e-7


@pytest.mark.parametrize("wt,k_new,theta_p,theta_max", [(2, 0, 0.4, 75), (12, 1, 0.8, 30), (0, 0, 0.0, 0)])
def test_bpf_configs(pa, pfref, pfsynth, wt, k_new, theta_p, theta_max):
    seq = pfsynth.Sequence("S64", n_frames=14, az_steps=1200)
    od, orc = _pair(pa, pfref, wt=wt, k_new=k_new, theta_p=theta_p, theta_max=theta_max)
    _run(od, orc, pfref, pfsynth, seq, range(12), check_maps_every=11)


def test_bpf_device_frames_match_update_api(pa, pfref, pfsynth):
    """pf_bpf_frame_device (HBM-resident clouds, two-stage pipeline, graph replay) gives the same bits
    as the host-input update API."""
    seq = pfsynth.Sequence("S64", n_frames=24, az_steps=1500)
    clouds = [_inputs(pfref, pfsynth, seq, k) for k in range(24)]
    host = pa.Odom_BPF_EstimationClass(device=0)
    host.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    poses_h = []
    for k, cl in enumerate(clouds):
        if k == 0:
            host.initMapWithPoints(*cl)
            poses_h.append(host.odom)
        else:
            poses_h.append(host.updatePointsToMap(*cl))
    bufs = []
    dev = pa.Odom_BPF_EstimationClass(device=0)
    dev.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    for cl in clouds:
        ptrs = []
        for c in cl:
            b = pa.DeviceBuffer(max(c.nbytes, 16))
            b.upload(np.ascontiguousarray(c, np.float32))
            bufs.append(b)
            ptrs.append(b.ptr)
        dev.frame_device(ptrs, [c.shape[0] for c in cl])
    dev.sync()
    np.testing.assert_array_equal(dev.poses(), np.array(poses_h))
    for c in range(3):
        gx, grg = dev._map(c)
        hx, hrg = host._map(c)
        np.testing.assert_array_equal(gx, hx)
        np.testing.assert_array_equal(grg, hrg)


def _front_clouds(pfref, x):
    r = pfref.bpf_preprocess(x, pfref.cls_params())
    return [np.c_[x[r[k], :3], np.zeros(len(r[k]))].astype(np.float32) for k in ("beam", "pillar", "facade")]


def test_bpf_scan_pipeline(pa, pfref, pfsynth):
    """Raw-scan mode (pf_bpf_frame_scan_device: the front end, VoxelGrid and odometry in the two-stage
    pipeline, graph replay from frame 11): the same bits as the update API fed the oracle front end's
    clouds, and within the pose tolerance of the oracle's whole chain (front end + OdomBPF)."""
    nf = 16
    seq = pfsynth.Sequence("S64", n_frames=nf, az_steps=1500)
    scans = [seq.frame(k) for k in range(nf)]
    clouds = [_front_clouds(pfref, x) for x in scans]
    host = pa.Odom_BPF_EstimationClass(device=0)
    host.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    orc = pfref.OdomBPF(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=pfref.LM_NORMAL_EQ)
    poses_h = []
    for k, cl in enumerate(clouds):
        if k == 0:
            host.initMapWithPoints(*cl)
            orc.init_map(*cl)
            poses_h.append(host.odom)
            continue
        poses_h.append(host.updatePointsToMap(*cl))
        dt, dr = pose_err(poses_h[-1], orc.update(*cl))
        assert dt < TOL_T and dr < TOL_R, (k, dt, dr)
    dev = pa.Odom_BPF_EstimationClass(device=0)
    dev.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    n = max(x.shape[0] for x in scans)
    buf = pa.DeviceBuffer(16 * n * nf)
    for k, x in enumerate(scans):
        buf.upload(x, 16 * n * k)
    for k, x in enumerate(scans):
        dev.frame_scan_device(buf.ptr + 16 * n * k, x.shape[0])
    dev.sync()
    np.testing.assert_array_equal(dev.poses(), np.array(poses_h))
    st = dev.stats()
    assert all(st["n_in"][c] == clouds[-1][c].shape[0] for c in range(3))
    # frame_host stages through a device buffer: same result on a fresh handle
    dev2 = pa.Odom_BPF_EstimationClass(device=0)
    dev2.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    last = [dev2.frame_host(x) for x in scans[:4]][-1]
    np.testing.assert_array_equal(last, poses_h[3])


@pytest.mark.parametrize("dcvc", [False, True])
def test_bpf_front_lanes_identical(pa, pfsynth, dcvc):
    """Two front-end lanes (pf_bpf_set_front_lanes(2), what the auto default picks for a lone handle: consecutive frames' front ends on
    two streams with an instance each) give the bits of one lane, with and without the curvedfilter
    (whose first-call defaults belong to frame 0 on lane 0), through graph replay, and again after
    pf_odom_reset on the same handle."""
    nf = 24
    seq = pfsynth.Sequence("S64", n_frames=nf, az_steps=1500)
    scans = [seq.frame(k) for k in range(nf)]
    n = max(x.shape[0] for x in scans)
    buf = pa.DeviceBuffer(16 * n * nf)
    for k, x in enumerate(scans):
        buf.upload(x, 16 * n * k)

    def run(lanes, od=None):
        if od is None:
            od = pa.Odom_BPF_EstimationClass(device=0)
            od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
            od.set_front_lanes(lanes)
            if dcvc:
                od.set_dcvc(True)
        for k, x in enumerate(scans):
            od.frame_scan_device(buf.ptr + 16 * n * k, x.shape[0])
        od.sync()
        return od, od.poses(), [od._map(c) for c in range(3)]

    _, p1, m1 = run(1)
    od2, p2, m2 = run(2)
    np.testing.assert_array_equal(p1, p2)
    for a, b in zip(m1, m2):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
    od2.reset()
    _, p3, _ = run(2, od2)
    np.testing.assert_array_equal(p1, p3)
    # the lane mode changed mid-sequence (as the auto mode does when a second handle appears)
    od3 = pa.Odom_BPF_EstimationClass(device=0)
    od3.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    if dcvc:
        od3.set_dcvc(True)
    for k, x in enumerate(scans):
        if k in (7, 13, 18):
            od3.set_front_lanes({7: 1, 13: 2, 18: 0}[k])
        od3.frame_scan_device(buf.ptr + 16 * n * k, x.shape[0])
    od3.sync()
    np.testing.assert_array_equal(p1, od3.poses())
    if dcvc:
        # the curvedfilter switched on after an odd number of frames: its first call (the 5 m ring
        # start) is that frame's, on whichever lane runs it, as with one lane
        def late(lanes, when):
            od = pa.Odom_BPF_EstimationClass(device=0)
            od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
            od.set_front_lanes(lanes)
            for k, x in enumerate(scans):
                if k == when:
                    od.set_dcvc(True)
                od.frame_scan_device(buf.ptr + 16 * n * k, x.shape[0])
            od.sync()
            return od.poses()
        for when in (5, 6):
            np.testing.assert_array_equal(late(1, when), late(2, when), err_msg="DCVC from frame %d" % when)


def test_bpf_scan_edge_cases(pa, pfsynth):
    """Raw-scan mode with an empty scan and a scan of a few points (the front end yields empty class
    clouds; the estimator warns that the map is too small, as the reference prints and continues), a
    scan above max_points (PF_ECAPACITY) and front-end parameters outside the supported range."""
    od = pa.Odom_BPF_EstimationClass(device=0, max_points=200000)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    buf = pa.DeviceBuffer(16 * 200000)
    x = pfsynth.Sequence("S64", n_frames=2, az_steps=800).frame(0)
    buf.upload(x)
    od.frame_scan_device(buf.ptr, x.shape[0])                          # seeds the maps
    for n in (0, 5):
        pose = np.empty(7)
        rc = pa.lib().pf_bpf_frame_scan_device(od._h, buf.ptr, n, pose.ctypes.data)
        assert rc >= 0 and np.all(np.isfinite(pose))
    assert pa.lib().pf_bpf_frame_scan_device(od._h, buf.ptr, 200001, None) == pa.PF_ECAPACITY
    bad = pa.cls_params(k=40)
    assert pa.lib().pf_bpf_set_front_end(od._h, ctypes.byref(bad)) == pa.PF_EINVAL


def test_bpf_rejects_es_entry_points(pa):
    od = pa.Odom_BPF_EstimationClass(device=0)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    z = np.zeros((4, 4), np.float32)
    assert pa.lib().pf_odom_init_map(od._h, z.ctypes.data, 4, 16, z.ctypes.data, 4, 16) == pa.PF_EINVAL
    assert pa.lib().pf_odom_frame_host(od._h, z.ctypes.data, 4, 16, None) == pa.PF_EINVAL
    assert pa.lib().pf_odom_classes(od._h) == 3
    es = pa.Odom_ES_EstimationClass(device=0)
    es.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    assert pa.lib().pf_bpf_init_map(es._h, z.ctypes.data, 4, 16, z.ctypes.data, 4, 16, z.ctypes.data, 4,
                                    16) == pa.PF_EINVAL
    assert pa.lib().pf_odom_classes(es._h) == 2
