"""Regenerate tests/golden/*.npz: oracle (pfref) outputs on seeded synthetic inputs.

The reference ships no fixtures and cannot be built here, so these vectors pin the
oracle against regressions and give the GPU tests an oracle-free comparison; they are NOT outputs of
the reference itself ("parity unpinned" at the PCL/Eigen/FLANN/Ceres boundary).
Inputs are regenerated from the seeded generator at test time and checked against the stored hash.

  python tools/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "pfilter-noetic_amd", "synth")):
    sys.path.insert(0, p)
import pfref  # noqa: E402
import pfsynth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def fe_case():
    seq = pfsynth.Sequence("S32", n_frames=6, az_steps=600)
    x = seq.frame(3)
    e, s = pfref.feature_extraction(x, pfref.make_lidar(32, 3.0, 90.0), opts=pfref.FE_STABLE_TIES)
    np.savez_compressed(os.path.join(OUT, "fe_s32_f3.npz"), input_sha=sha(x), n_in=x.shape[0], edge=e, surf=s,
                        spec=np.array(["S32", "n_frames=6", "az_steps=600", "frame=3", "lines=32", "3-90 m",
                                       "opts=FE_STABLE_TIES"]))
    print("fe", x.shape, e.shape, s.shape)


def odom_case():
    seq = pfsynth.Sequence("S64", n_frames=30, az_steps=1000)
    frames = [seq.frame(k) for k in range(24)]
    out = {"input_sha": np.array([sha(x) for x in frames])}
    for name, opts in (("gpu_equiv", pfref.GPU_EQUIV), ("faithful", 0)):
        od = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=opts)
        poses, counts = [], []
        for x in frames:
            poses.append(od.frame(x))
            st = od.stats()
            counts.append([st[k] for k in ("n_edge_in", "n_surf_in", "n_edge_ds", "n_surf_ds", "n_edge_map",
                                           "n_surf_map", "n_edge_res", "n_surf_res")])
        out[name + "_poses"] = np.array(poses)
        out[name + "_counts"] = np.array(counts, np.int64)
        ex, er = od.get_map(0)
        sx, sr = od.get_map(1)
        out[name + "_map_sha"] = np.array([sha(ex), sha(er), sha(sx), sha(sr)])
    np.savez_compressed(os.path.join(OUT, "odom_s64_24f.npz"), **out,
                        spec=np.array(["S64", "n_frames=30", "az_steps=1000", "frames 0-23", "lines=64",
                                       "3-90 m", "map 0.4", "k_new 0", "theta_p 0.4", "theta_max 75", "weight 0"]))
    print("odom", out["gpu_equiv_poses"][-1])


FULL_COUNTS = ("n_edge_in", "n_surf_in", "n_edge_ds", "n_surf_ds", "n_edge_map", "n_surf_map", "n_edge_res",
               "n_surf_res", "n_edge_valid", "n_surf_valid")


def odom_full_case(n=4541):
    """configs[1] over the whole bench sequence (S64 seed 0, 4541 frames, bench.py's generator
    call): the GPU_EQUIV trajectory, every frame's counts and the final maps' hashes. The GPU test
    (tests/test_gpu_odom.py::test_full_sequence_bench_path) replays it through the bench's path."""
    seq = pfsynth.Sequence("S64", n_frames=n, seed=0)
    od = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=pfref.GPU_EQUIV)
    poses = np.zeros((n, 7))
    counts = np.zeros((n, len(FULL_COUNTS)), np.int32)
    in_sha = []
    for f0 in range(0, n, 256):
        nf = min(256, n - f0)
        buf, cnt = seq.frames(f0, nf, threads=8)
        for i in range(nf):
            k = f0 + i
            x = buf[i, :cnt[i]]
            if k % 500 == 0 or k == n - 1:
                in_sha.append((k, sha(x)))
            poses[k] = od.frame(x)
            st = od.stats()
            counts[k] = [st[c] for c in FULL_COUNTS]
        print("frame", f0 + nf, poses[f0 + nf - 1][4:], flush=True)
    ex, er = od.get_map(0)
    sx, sr = od.get_map(1)
    np.savez_compressed(os.path.join(OUT, "odom_s64_full.npz"), poses=poses, counts=counts,
                        count_names=np.array(FULL_COUNTS), input_frames=np.array([k for k, _ in in_sha]),
                        input_sha=np.array([h for _, h in in_sha]),
                        map_sha=np.array([sha(ex), sha(er), sha(sx), sha(sr)]),
                        map_sizes=np.array([ex.shape[0], sx.shape[0]]),
                        spec=np.array(["S64", "n_frames=%d" % n, "seed=0", "lines=64", "3-90 m", "map 0.4",
                                       "k_new 0", "theta_p 0.4", "theta_max 75", "weight 0", "opts=GPU_EQUIV"]))
    print("odom_full", poses[-1], ex.shape, sx.shape)


def faithful_traj(preset, n, theta, name, lines=64, seed=0):
    """A whole sequence through the reference-faithful oracle (opts=0: libstdc++ std::sort tie orders,
    Householder-QR LM, FLANN-style kd-tree), free-running: every frame's pose and counts and the final
    maps' hashes. The GPU test (tests/test_gpu_parity_free.py) runs the device free-running in the
    reference-tie-order mode against it."""
    seq = pfsynth.Sequence(preset, n_frames=n, seed=seed)
    od = pfref.Odom(pfref.make_lidar(lines, 3.0, 90.0), 0.4, 0, theta[0], theta[1], 0, opts=0)
    poses = np.zeros((n, 7))
    counts = np.zeros((n, len(FULL_COUNTS)), np.int32)
    in_sha = []
    for f0 in range(0, n, 256):
        nf = min(256, n - f0)
        buf, cnt = seq.frames(f0, nf, threads=8)
        for i in range(nf):
            k = f0 + i
            x = buf[i, :cnt[i]]
            if k % 500 == 0 or k == n - 1:
                in_sha.append((k, sha(x)))
            poses[k] = od.frame(x)
            st = od.stats()
            counts[k] = [st[c] for c in FULL_COUNTS]
        print(name, "frame", f0 + nf, poses[f0 + nf - 1][4:], flush=True)
    ex, er = od.get_map(0)
    sx, sr = od.get_map(1)
    gt = np.array([seq.gt_pose(k) for k in range(n)])
    np.savez_compressed(os.path.join(OUT, "odom_%s_faithful.npz" % name), poses=poses, counts=counts, gt=gt,
                        count_names=np.array(FULL_COUNTS), input_frames=np.array([k for k, _ in in_sha]),
                        input_sha=np.array([h for _, h in in_sha]),
                        map_sha=np.array([sha(ex), sha(er), sha(sx), sha(sr)]),
                        map_sizes=np.array([ex.shape[0], sx.shape[0]]),
                        spec=np.array([preset, "n_frames=%d" % n, "seed=%d" % seed, "lines=%d" % lines, "3-90 m",
                                       "map 0.4", "k_new 0", "theta_p %g" % theta[0], "theta_max %d" % theta[1],
                                       "weight 0", "opts=0 (faithful)"]))
    print(name, "faithful", poses[-1], ex.shape, sx.shape)


def faithful_s64_case():
    faithful_traj("S64", 4541, (0.4, 75), "s64")


def faithful_s64t_case():
    faithful_traj("S64T", 4541, (0.4, 75), "s64t")


def knn_case():
    rng = np.random.default_rng(11)
    mp = np.zeros((3000, 4), np.float32)
    mp[:, :3] = rng.uniform(-8, 8, (3000, 3))
    mp[:800, 2] = 0.0
    q = np.zeros((400, 4), np.float32)
    q[:, :3] = rng.uniform(-9, 9, (400, 3))
    idx, d2 = pfref.knn(mp, q, 5, opts=pfref.KNN_BRUTE)
    np.savez_compressed(os.path.join(OUT, "knn_3000x400.npz"), map=mp, queries=q, idx=idx, d2=d2)
    print("knn", idx.shape)


def grid_case():
    rng = np.random.default_rng(12)
    xyz = rng.uniform(-3, 3, (2500, 3)).astype(np.float32)
    xyz[:400] = np.round(xyz[:400] * 2.5) / np.float32(2.5)
    r = rng.integers(0, 256, 2500)
    g = rng.integers(0, 256, 2500)
    pts = pfref.pack_rgb(xyz, r=r, g=g)
    vg = pfref.voxel_grid(pts, 0.8, opts=pfref.VG_STABLE)
    rg = pfref.rgbds(pts, 0.4, opts=pfref.VG_STABLE)
    np.savez_compressed(os.path.join(OUT, "voxel_2500.npz"), points=pts, voxel_grid_08=vg, rgbds_04=rg)
    print("voxel", vg.shape, rg.shape)


def cls_case():
    """BPF front end (ground_seg + featureExtract) on one S32 frame: index lists."""
    x = pfsynth.Sequence("S32", n_frames=3, az_steps=900).frame(2)
    r = pfref.bpf_preprocess(x, pfref.cls_params())
    g, u = pfref.ground_seg(x, pfref.cls_params())
    cls, num = pfref.pca_classify(x[u], pfref.cls_params())
    np.savez_compressed(os.path.join(OUT, "cls_s32_f2.npz"), input_sha=sha(x), unground=u, pt_num=num, cls=cls,
                        **r)
    print("cls", {k: len(v) for k, v in r.items()})


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:] or ["fe", "odom", "knn", "grid", "cls"]
    for w in which:
        globals()[w + "_case"]()
