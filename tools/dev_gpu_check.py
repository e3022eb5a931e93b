"""Exploratory GPU parity/timing check (development tool; the gated tests live in tests/)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd")); sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pfilter_amd as pa, pfsynth, pfref

def log(*a):
    print(*a, flush=True)

rng = np.random.default_rng(0)
# 1. kNN parity
M = 20000
mp = np.zeros((M, 4), np.float32); mp[:, :3] = rng.uniform(-10, 10, (M, 3)).astype(np.float32)
mp[:5000, 2] = 0.0  # plane with ties
Q = 5000
q = np.zeros((Q, 4), np.float32); q[:, :3] = rng.uniform(-11, 11, (Q, 3)).astype(np.float32)
kn = pa.Knn(M, Q); kn.set_map(mp); gi, gd = kn.query(q)
ri, rd = pfref.knn(mp, q, 5, opts=pfref.KNN_BRUTE)
valid = rd[:, 4] < 1.0
ok = np.array_equal(gi[valid], ri[valid]) and np.array_equal(gd[valid].view(np.uint32), rd[valid].view(np.uint32))
log("knn: valid", valid.sum(), "exact", ok, "gpu found5", (gi[:, 4] >= 0).sum())

# 2. feature extraction parity
seq = pfsynth.Sequence("S64", n_frames=60)
lid = pa.make_lidar(64, 3.0, 90.0)
fe = pa.LaserProcessingClass(); fe.init(lid)
x = seq.frame(3)
t = time.time(); ge, gs = fe.featureExtraction(x); tg = time.time() - t
re_, rs_ = pfref.feature_extraction(x, pfref.make_lidar(64, 3.0, 90.0), opts=pfref.FE_STABLE_TIES)
log("fe: gpu", ge.shape, gs.shape, "ref", re_.shape, rs_.shape, "edge exact", np.array_equal(ge.view(np.uint32), re_.view(np.uint32)),
    "surf exact", np.array_equal(gs.view(np.uint32), rs_.view(np.uint32)), "t %.2f ms" % (tg * 1e3))

# 3. odometry parity over frames (host path, whole frame)
NF = int(os.environ.get("NF", "40"))
od = pa.OdomEstimationClass(); od.init(lid, 0.4, 0, 0.4, 75, 0)
orc = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=pfref.GPU_EQUIV)
worst_t = worst_r = 0.0
for k in range(NF):
    x = seq.frame(k)
    pg = od.frame_host(x)
    pr = orc.frame(x)
    dt = np.linalg.norm(pg[4:] - pr[4:])
    dq = pg[:4] * np.sign(np.dot(pg[:4], pr[:4]))
    dr = 2 * np.linalg.norm(dq - pr[:4])
    worst_t = max(worst_t, dt); worst_r = max(worst_r, dr)
    if k < 4 or k % 10 == 0:
        sg, so = od.stats(), orc.stats()
        log(k, "dt %.3e dr %.3e" % (dt, dr), "gpu", {kk: sg[kk] for kk in ("n_edge_ds", "n_surf_ds", "n_edge_map", "n_surf_map", "n_edge_res", "n_surf_res", "lm_iterations")},
            "ref", {kk: so[kk] for kk in ("n_edge_ds", "n_surf_ds", "n_edge_map", "n_surf_map", "n_edge_res", "n_surf_res", "lm_iterations")})
log("odom worst dt %.3e dr %.3e" % (worst_t, worst_r))

# 4. timing of the device pipeline
NT = int(os.environ.get("NT", "200"))
seq2 = pfsynth.Sequence("S64", n_frames=12 + NT)
buf, counts = seq2.frames(0, 12 + NT)
od2 = pa.OdomEstimationClass(); od2.init(lid, 0.4, 0, 0.4, 75, 0)
db = pa.DeviceBuffer(buf.nbytes); db.upload(buf)
stride = buf.shape[1] * 16
for k in range(12):
    od2.frame_device(db.ptr + k * stride, counts[k])
od2.sync()
t = time.time()
for k in range(12, 12 + NT):
    od2.frame_device(db.ptr + k * stride, counts[k])
od2.sync()
el = time.time() - t
log("pipeline: %d frames %.3f s -> %.1f fps, %.3f ms/frame" % (NT, el, NT / el, el / NT * 1e3))
p = od2.poses()
gt = np.array([seq2.gt_pose(k) for k in range(p.shape[0])])
log("pipeline drift: final pos err %.3f m over %.1f m" % (np.linalg.norm(p[-1, 4:] - gt[-1, 4:]), np.linalg.norm(gt[-1, 4:])))
