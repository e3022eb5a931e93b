"""GPU: curvedVoxel (DCVC, src/additionClass.cpp:1-497) through the C ABI (pf_dcvc_*, pf_cls_set_dcvc,
pf_bpf_set_dcvc).

The reference runs DCVC's loops under OpenMP with shared temporaries, so its output is not a function
of its input; its deterministic reading is the serial one (oracle/pfref_dcvc.cpp, mode 0), a greedy
pass that leaves some neighbours of a processed point unlabelled. The device computes the connected
components of the same curved-voxel neighbourhood (searchKNN with its quirks). Bars:
  * bit-exact against the oracle's components mode (mode 1): kept points in the published order and
    every point's cluster rank (integer / index work);
  * statistical against the serial reading, per frame: the kept point sets overlap with IoU >= 0.95
    and the clusterings of the points both keep agree with adjusted Rand index >= 0.9 (measured
    0.96-0.9999 and 0.95-1.0 on S64 / S32 / S64V frames when this bar was set)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ari(a, b):
    """adjusted Rand index of two labellings"""
    from collections import Counter
    n = len(a)
    if n < 2:
        return 1.0
    comb = lambda x: x * (x - 1) / 2.0
    pairs = Counter(zip(a.tolist(), b.tolist()))
    sa, sb = Counter(a.tolist()), Counter(b.tolist())
    idx = sum(comb(v) for v in pairs.values())
    ea, eb = sum(comb(v) for v in sa.values()), sum(comb(v) for v in sb.values())
    exp = ea * eb / comb(n)
    mx = 0.5 * (ea + eb)
    return 1.0 if mx == exp else (idx - exp) / (mx - exp)


def _nonground(pfref, x):
    g, u = pfref.ground_seg(x[:, :3])
    return x[u]


@pytest.mark.parametrize("preset,frame", [("S64", 5), ("S64", 40), ("S32", 3), ("S64V", 30)])
def test_dcvc_matches_components_oracle_and_serial_statistics(pa, pfref, pfsynth, preset, frame):
    U = _nonground(pfref, pfsynth.Sequence(preset, n_frames=frame + 1).frame(frame))
    dc = pa.Dcvc(max_points=200000)
    dc.run(U[:100])                                   # the first call starts the rings at 5 m: not this one
    idx, lab = dc.run(U)
    oidx, olab = pfref.dcvc(U, components=True)
    np.testing.assert_array_equal(idx, oidx)
    np.testing.assert_array_equal(lab, olab)
    sidx, slab = pfref.dcvc(U)                        # the serial reading
    ks, kg = slab > 0, lab > 0
    iou = (ks & kg).sum() / max(1, (ks | kg).sum())
    both = ks & kg
    ari = _ari(slab[both], lab[both])
    assert iou >= 0.95 and ari >= 0.9, (iou, ari)
    assert len(idx) > 0.8 * len(U)


@pytest.mark.parametrize("kw", [dict(delta_a=1.0, delta_p=0.8), dict(delta_a=0.1, delta_p=0.2, min_seg=20),
                                dict(start_r=0.5, delta_r=0.001)])
def test_dcvc_other_grids(pa, pfref, pfsynth, kw):
    """Grids other than config.yaml's: width 361 (azimuth 301..360 search the clamped column 300, a
    one-way neighbourhood the unions must take from its only side), an index space too large for the
    device's voxel table (binary-search lookups), finer rings. Bit-exact against the components mode."""
    U = _nonground(pfref, pfsynth.Sequence("S64", n_frames=8).frame(7))
    dc = pa.Dcvc(max_points=200000, **kw)
    dc.run(U[:50])
    idx, lab = dc.run(U)
    oidx, olab = pfref.dcvc(U, pfref.dcvc_params(**kw), components=True)
    np.testing.assert_array_equal(idx, oidx)
    np.testing.assert_array_equal(lab, olab)
    assert len(idx) > 0


def test_dcvc_first_frame_and_reset(pa, pfref, pfsynth):
    """The first call of a handle (and the first after reset) starts the range rings at the member
    default 5 m (include/additionClass.hpp:105-106), later calls at 0 m (resetParams :445-449)."""
    U = _nonground(pfref, pfsynth.Sequence("S32", n_frames=2).frame(1))
    dc = pa.Dcvc(max_points=100000)
    a = dc.run(U)
    b = dc.run(U)
    dc.reset()
    c = dc.run(U)
    oa = pfref.dcvc(U, first_frame=True, components=True)
    ob = pfref.dcvc(U, first_frame=False, components=True)
    for got, want in ((a, oa), (b, ob), (c, oa)):
        np.testing.assert_array_equal(got[0], want[0])
        np.testing.assert_array_equal(got[1], want[1])


def test_dcvc_edge_cases(pa, pfref):
    dc = pa.Dcvc(max_points=10000, min_seg=2)
    idx, lab = dc.run(np.zeros((0, 3), np.float32))
    assert len(idx) == 0
    rng = np.random.default_rng(3)
    pts = np.concatenate([rng.normal([10, 0, 0], 0.05, (20, 3)), rng.normal([0, 10, 1], 0.05, (5, 3)),
                          [[0.2, 0.1, 0.0], [200.0, 0, 0]]]).astype(np.float32)   # out of range: (0, 0, 0) voxel
    dc.run(pts)
    idx, lab = dc.run(pts)
    oidx, olab = pfref.dcvc(pts, pfref.dcvc_params(min_seg=2), components=True)
    np.testing.assert_array_equal(idx, oidx)
    np.testing.assert_array_equal(lab, olab)
    assert lab[:20].min() == 1                        # the larger cluster first


def test_front_end_with_curvedfilter(pa, pfref, pfsynth):
    """pf_cls_set_dcvc: ground_seg -> DCVC -> featureExtract (src/additionNode.cpp:21-45 with curvedfilter
    on, the KITTI launch's default) equals the oracle chain with DCVC's components reading, list for
    list; the ground list is unchanged by the filter."""
    fe = pa.BPFFrontEnd(max_points=300000, device=0)
    fe.set_dcvc(True)
    seq = pfsynth.Sequence("S64", n_frames=4)
    for k in range(3):
        x = seq.frame(k)
        got = fe.extract(x)
        want = pfref.bpf_preprocess(x, pfref.cls_params(), dcvc=pfref.dcvc_params(), first_frame=(k == 0),
                                    components=True)
        for key in ("beam", "pillar", "facade", "ground"):
            np.testing.assert_array_equal(got[key], want[key], err_msg="%d %s" % (k, key))
    fe.set_dcvc(False)
    np.testing.assert_array_equal(fe.extract(x)["facade"], pfref.bpf_preprocess(x, pfref.cls_params())["facade"])


def test_bpf_scan_pipeline_with_curvedfilter(pa, pfsynth):
    """pf_bpf_set_dcvc: the raw-scan BPF pipeline with DCVC runs, graph replay equals eager, and the
    class clouds it feeds the estimator are the front end's (same frames, same parameters)."""
    seq = pfsynth.Sequence("S64", n_frames=30, az_steps=1500)
    buf, counts = seq.frames(0, 30)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    out = []
    for graph in (3, 0):
        od = pa.Odom_BPF_EstimationClass(device=0)
        od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
        od.set_graph(graph)
        od.set_dcvc(True)
        for k in range(30):
            od.frame_scan_device(db.ptr + k * buf.shape[1] * 16, int(counts[k]))
        od.sync()
        out.append(od.poses())
        assert od.stats()["errors"] == 0
    np.testing.assert_array_equal(out[0], out[1])
    assert np.isfinite(out[0]).all() and np.linalg.norm(out[0][-1, 4:6]) > 1.0


def _isolated_points():
    """6,000 single-point clusters: every third azimuth bin, every third 1 m range ring, two pitch
    layers 9.6 degrees apart, so no two points share a 27-voxel neighbourhood (> kDcMaxClusters)"""
    az = np.deg2rad(np.arange(0, 360, 3.6))
    rng = 10.0 + 3.0 * np.arange(30)
    pit = np.deg2rad([2.0, 11.6])
    a, r, p = np.meshgrid(az, rng, pit, indexing="ij")
    xyz = np.stack([r * np.cos(p) * np.cos(a), r * np.cos(p) * np.sin(a), r * np.sin(p)], -1).reshape(-1, 3)
    return xyz.astype(np.float32)


def test_curvedfilter_overflow_does_not_stick(pa, pfref, pfsynth):
    """a frame whose kept clusters exceed the device's cluster table raises PF_ECAPACITY for
    that frame only; the next frames run normally again (the DCVC error word is per call) and equal the
    oracle chain, and so does a frame after pf_dcvc-style reset of the sequence."""
    fe = pa.BPFFrontEnd(max_points=300000, device=0, ground_filter=0)
    fe.set_dcvc(True, min_seg=0)
    seq = pfsynth.Sequence("S64", n_frames=3)
    x0 = seq.frame(0)
    fe.extract(x0)                                      # first call: rings from 5 m
    with pytest.raises(pa.PFError) as ei:
        fe.extract(_isolated_points())
    assert ei.value.code == pa.PF_ECAPACITY
    for k in (1, 2):
        x = seq.frame(k)
        got = fe.extract(x)
        want = pfref.bpf_preprocess(x, pfref.cls_params(ground_filter=0), dcvc=pfref.dcvc_params(min_seg=0),
                                    components=True)
        for key in ("beam", "pillar", "facade"):
            np.testing.assert_array_equal(got[key], want[key], err_msg="%d %s" % (k, key))


def test_dcvc_rejects_rings_that_never_reach_max_range(pa):
    """start_r - k * delta_r reaches 0 at about 166 m with the default widths: a max_range past that
    is refused at create (the reference would loop forever building its ring bounds, :127-134)."""
    with pytest.raises(pa.PFError) as ei:
        pa.Dcvc(max_points=1000, max_range=200.0)
    assert ei.value.code == pa.PF_EINVAL
    pa.Dcvc(max_points=1000, max_range=150.0)


def test_front_end_dcvc_rejects_rings_that_never_reach_max_range(pa):
    """The same parameter check for the curvedfilter inside the front end and the BPF pipeline
    (pf_cls_set_dcvc / pf_bpf_set_dcvc), so an accepted configuration cannot overflow the ring bounds
    on every frame."""
    fe = pa.BPFFrontEnd(max_points=1000, device=0)
    with pytest.raises(pa.PFError) as ei:
        fe.set_dcvc(True, max_range=200.0)
    assert ei.value.code == pa.PF_EINVAL
    fe.set_dcvc(True, max_range=150.0)
    od = pa.Odom_BPF_EstimationClass(device=0)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    with pytest.raises(pa.PFError) as ei:
        od.set_dcvc(True, max_range=200.0)
    assert ei.value.code == pa.PF_EINVAL
