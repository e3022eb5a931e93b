"""GPU: the C++ drop-in classes (pfilter-noetic_amd/shim) driven like the ROS nodes
(tests/shim/shim_driver.cpp), against the same frames through the Python binding of the same C ABI:
identical poses and map sizes."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shim_matches_python_binding(pa, pfref, pfsynth, tmp_path):
    exe = str(tmp_path / "shim_driver")
    lib = os.path.join(ROOT, "pfilter-noetic_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "shim", "shim_driver.cpp"), "-o", exe, "-L", lib,
                           "-lpfilter_hip", "-Wl,-rpath," + lib, "-Wl,-rpath-link,/opt/rocm/lib"])
    seq = pfsynth.Sequence("S64", n_frames=8, az_steps=1200)
    frames = [seq.frame(k) for k in range(8)]
    with open(tmp_path / "frames.bin", "wb") as f:
        for x in frames:
            np.array([x.shape[0]], np.int64).tofile(f)
            x.astype(np.float32).tofile(f)
    subprocess.check_call([exe, str(tmp_path / "frames.bin"), str(tmp_path / "poses.txt")], timeout=120)
    got = np.loadtxt(tmp_path / "poses.txt")
    lines = open(tmp_path / "poses.txt").read().splitlines()
    lid = pa.make_lidar(64, 3.0, 90.0)
    fe = pa.LaserProcessingClass()
    fe.init(lid)
    od = pa.Odom_ES_EstimationClass()
    od.init(lid, 0.4, 0, 0.4, 75, 0)
    for k, x in enumerate(frames):
        e, s = fe.featureExtraction(x)
        if k == 0:
            od.initMapWithPoints(e, s)
        else:
            od.updatePointsToMap(e, s)
        np.testing.assert_array_equal(got[k, :7], od.odom)
        assert got[k, 7] == od.laserCloudCornerMap[0].shape[0]
        assert got[k, 8] == od.laserCloudSurfMap[0].shape[0]
        st = od.state()                                      # OdomBaseClass members through the shim
        np.testing.assert_array_equal(got[k, 9:16], st["parameters"])
        np.testing.assert_array_equal(got[k, 16:19], st["last_odom"][:, 3])
        assert got[k, 19] == st["optimization_count"]
        cs = 0
        for r, g in od.laserCloudSurfMap[1]:
            cs = (cs * 1000003 + int(r) * 256 + int(g)) % (1 << 64)
        assert int(lines[k].split()[20]) == cs


def test_shim_default_is_reference_order_against_faithful_trajectory(pa, pfsynth, tmp_path):
    """The drop-in as the unchanged ROS nodes build it -- shim classes with their default settings, driven
    like src/laserProcessingNode.cpp:71-78 + src/odomEstimationNode copy.cpp:86-107 -- against the
    reference-faithful oracle's own free run of the headline sequence (tests/golden/odom_s64_faithful.npz:
    pfref opts=0, libstdc++ std::sort tie orders, Householder-QR LM, FLANN-style kd-tree): every frame's
    pose within 1e-4 m / 1e-5 rad and both map sizes equal. The shims default to the reference tie order
    (reference_tie_order = true, pf_odom_set_tie_order / pf_fe_set_tie_order), so no node change is needed
    for the reference's results."""
    import hashlib
    from _util import pose_err
    g = np.load(os.path.join(ROOT, "tests", "golden", "odom_s64_faithful.npz"))
    n = 400
    exe = str(tmp_path / "shim_driver")
    lib = os.path.join(ROOT, "pfilter-noetic_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "shim", "shim_driver.cpp"), "-o", exe, "-L", lib,
                           "-lpfilter_hip", "-Wl,-rpath," + lib, "-Wl,-rpath-link,/opt/rocm/lib"])
    seq = pfsynth.Sequence("S64", n_frames=n, seed=0)
    checks = dict(zip((int(k) for k in g["input_frames"]), (str(h) for h in g["input_sha"])))
    with open(tmp_path / "frames.bin", "wb") as f:
        for k in range(n):
            x = np.ascontiguousarray(seq.frame(k), np.float32)
            if k in checks:
                assert hashlib.sha256(x.tobytes()).hexdigest() == checks[k], "generator changed at frame %d" % k
            np.array([x.shape[0]], np.int64).tofile(f)
            x.tofile(f)
    subprocess.check_call([exe, str(tmp_path / "frames.bin"), str(tmp_path / "poses.txt")], timeout=600)
    got = np.loadtxt(tmp_path / "poses.txt")
    assert got.shape[0] == n
    names = [str(c) for c in g["count_names"]]
    ie, is_ = names.index("n_edge_map"), names.index("n_surf_map")
    worst = 0.0
    for k in range(n):
        dt, dr = pose_err(got[k, :7], g["poses"][k])
        worst = max(worst, dt)
        assert dt < 1e-4 and dr < 1e-5, (k, dt, dr)
        if k > 0:
            assert (got[k, 7], got[k, 8]) == (g["counts"][k][ie], g["counts"][k][is_]), k
    print("shim (default settings) vs faithful oracle: %d frames, worst %.3e m" % (n, worst))


def test_bpf_shim_matches_python_binding(pa, pfref, pfsynth, tmp_path):
    """Odom_BPF_EstimationClass drop-in (shim) driven like src/odomEstimationNode.cpp:254-264."""
    exe = str(tmp_path / "shim_bpf_driver")
    lib = os.path.join(ROOT, "pfilter-noetic_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "shim", "shim_bpf_driver.cpp"), "-o", exe, "-L", lib,
                           "-lpfilter_hip", "-Wl,-rpath," + lib, "-Wl,-rpath-link,/opt/rocm/lib"])
    seq = pfsynth.Sequence("S64", n_frames=8, az_steps=1200)
    lid = pfref.make_lidar(64, 3.0, 90.0)
    clouds = [pfsynth.bpf_split(*pfref.feature_extraction(seq.frame(k), lid, opts=pfref.FE_STABLE_TIES))
              for k in range(8)]
    with open(tmp_path / "clouds.bin", "wb") as f:
        for cl in clouds:
            for c in cl:
                np.array([c.shape[0]], np.int64).tofile(f)
                c.astype(np.float32).tofile(f)
    subprocess.check_call([exe, str(tmp_path / "clouds.bin"), str(tmp_path / "poses.txt")], timeout=120)
    got = np.loadtxt(tmp_path / "poses.txt")
    od = pa.Odom_BPF_EstimationClass()
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    for k, cl in enumerate(clouds):
        if k == 0:
            od.initMapWithPoints(*cl)
        else:
            od.updatePointsToMap(*cl)
        np.testing.assert_array_equal(got[k, :7], od.odom)
        sizes = [m[0].shape[0] for m in (od.laserCloudBeamMap, od.laserCloudPillarMap, od.laserCloudFacadeMap)]
        assert list(got[k, 7:10]) == sizes and got[k, 10] == sum(sizes)


def test_front_end_shim_matches_python_binding(pa, pfsynth, tmp_path):
    """groundSeg + nongroundExtract drop-in (shim) driven like src/additionNode.cpp:21-45: the published
    beam / pillar / facade clouds equal the C ABI's index lists applied to the scan, and carry the
    PCA normals assign_normal writes (include/preProcess.hpp:327-346) as pf_cls_normals reports them."""
    exe = str(tmp_path / "shim_cls_driver")
    lib = os.path.join(ROOT, "pfilter-noetic_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "shim", "shim_cls_driver.cpp"), "-o", exe, "-L", lib,
                           "-lpfilter_hip", "-Wl,-rpath," + lib, "-Wl,-rpath-link,/opt/rocm/lib"])
    seq = pfsynth.Sequence("S64", n_frames=3, az_steps=1500)
    scans = [seq.frame(k) for k in range(3)]
    with open(tmp_path / "scans.bin", "wb") as f:
        for x in scans:
            np.array([x.shape[0]], np.int64).tofile(f)
            x.astype(np.float32).tofile(f)
    subprocess.check_call([exe, str(tmp_path / "scans.bin"), str(tmp_path / "out.bin")], timeout=120)
    raw = open(tmp_path / "out.bin", "rb").read()
    fe = pa.BPFFrontEnd(max_points=200000)
    off = 0
    for x in scans:
        sz = np.frombuffer(raw, np.int64, 5, off)
        off += 40
        r = fe.extract(x)
        g, u = fe.ground_seg(x)
        assert list(sz) == [len(g), len(u), len(r["beam"]), len(r["pillar"]), len(r["facade"])]
        np.testing.assert_array_equal(g, r["ground"])
        U = x[u]
        cls, _, nrm = fe.classify(U, normals=True)
        for k, code in (("beam", 2), ("pillar", 1), ("facade", 3)):
            rec = np.frombuffer(raw, np.float32, 7 * len(r[k]), off).reshape(-1, 7)
            off += 28 * len(r[k])
            np.testing.assert_array_equal(rec[:, :3], x[r[k], :3])
            np.testing.assert_array_equal(rec[:, 3:].view(np.uint32), nrm[cls == code].view(np.uint32))


def test_mapping_shim_matches_python_binding(pa, pfref, pfsynth, tmp_path):
    """LaserMappingClass drop-in (shim) driven like src/laserMappingNode.cpp:72-86, the pose as the
    Isometry3d matrix: the same map as the pose-quaternion entry point."""
    exe = str(tmp_path / "shim_map_driver")
    lib = os.path.join(ROOT, "pfilter-noetic_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "shim", "shim_map_driver.cpp"), "-o", exe, "-L", lib,
                           "-lpfilter_hip", "-Wl,-rpath," + lib, "-Wl,-rpath-link,/opt/rocm/lib"])
    seq = pfsynth.Sequence("S64", n_frames=10, az_steps=800)
    lid = pfref.make_lidar(64, 3.0, 90.0)
    m = pa.LaserMappingClass(max_points=1 << 21, max_scan=100000)
    m.init(0.4)
    with open(tmp_path / "frames.bin", "wb") as f:
        for k in range(0, 10, 2):
            e, s = pfref.feature_extraction(seq.frame(k), lid, opts=pfref.FE_STABLE_TIES)
            x = np.concatenate([e, s]).astype(np.float32)
            p = seq.gt_pose(k)
            qx, qy, qz, qw = p[:4]
            tx, ty, tz = 2 * qx, 2 * qy, 2 * qz
            R = np.array([[1 - (ty * qy + tz * qz), ty * qx - tz * qw, tz * qx + ty * qw],
                          [ty * qx + tz * qw, 1 - (tx * qx + tz * qz), tz * qy - tx * qw],
                          [tz * qx - ty * qw, tz * qy + tx * qw, 1 - (tx * qx + ty * qy)]])
            T = np.c_[R, p[4:]].astype(np.float64)
            np.array([x.shape[0]], np.int64).tofile(f)
            T.tofile(f)
            x.tofile(f)
            m.updateCurrentPointsToMap(x, p)
    subprocess.check_call([exe, str(tmp_path / "frames.bin"), str(tmp_path / "map.bin")], timeout=120)
    got = np.fromfile(tmp_path / "map.bin", np.float32).reshape(-1, 4)
    np.testing.assert_array_equal(got, m.getMap())


def test_curved_voxel_shim_matches_c_abi(pa, pfsynth, tmp_path):
    """curvedVoxel drop-in (pfilter_hip::CurvedVoxelT, the class shim/additionClass.hpp gives
    additionNode.cpp) driven per frame like src/additionNode.cpp:29-39: pointCloudSegPtr and labelRecords
    equal pf_dcvc_run's kept points and cluster ranks bit for bit, the first frame included (rings from
    5 m, then from 0, through the device handle the object's copies share); clusterBoxes() (the bounds
    colorSegmentation publishes, src/additionClass.cpp:364-416) equal each cluster run's min / max."""
    exe = str(tmp_path / "shim_dcvc_driver")
    lib = os.path.join(ROOT, "pfilter-noetic_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "shim", "shim_dcvc_driver.cpp"), "-o", exe, "-L", lib,
                           "-lpfilter_hip", "-Wl,-rpath," + lib, "-Wl,-rpath-link,/opt/rocm/lib"])
    seq = pfsynth.Sequence("S64", n_frames=4, az_steps=1500)
    frames = [seq.frame(k) for k in range(4)]
    with open(tmp_path / "frames.bin", "wb") as f:
        for x in frames:
            np.array([x.shape[0]], np.int64).tofile(f)
            x.astype(np.float32).tofile(f)
    subprocess.check_call([exe, str(tmp_path / "frames.bin"), str(tmp_path / "out.bin")], timeout=120)
    raw = open(tmp_path / "out.bin", "rb").read()
    dc = pa.Dcvc(max_points=300000)
    off = 0
    for x in frames:
        idx, lab = dc.run(x[:, :3])
        nk, nc = np.frombuffer(raw, np.int64, 2, off)
        off += 16
        xyz = np.frombuffer(raw, np.float32, 3 * nk, off).reshape(-1, 3)
        off += 12 * nk
        rec = np.frombuffer(raw, np.int32, 3 * nc, off).reshape(-1, 3)
        off += 12 * nc
        assert nk == idx.size and nk > 1000
        np.testing.assert_array_equal(xyz.view(np.uint32), x[idx, :3].view(np.uint32))
        ranks, sizes = np.unique(lab[lab > 0], return_counts=True)
        np.testing.assert_array_equal(rec[:, 0], ranks)
        np.testing.assert_array_equal(rec[:, 1], sizes)
        starts = np.cumsum(np.r_[0, sizes[:-1]])
        np.testing.assert_array_equal(rec[:, 2], idx[starts])
        box = np.frombuffer(raw, np.float32, 6 * nc, off).reshape(-1, 6)       # colorSegmentation's bounds
        off += 24 * nc
        for c in range(nc):
            run = xyz[starts[c]:starts[c] + sizes[c]]
            np.testing.assert_array_equal(box[c, :3], run.min(0))
            np.testing.assert_array_equal(box[c, 3:], run.max(0))
    assert off == len(raw)
