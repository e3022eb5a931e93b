"""GPU: free-running parity against the reference-faithful oracle over whole sequences (VERDICT r02
next-2, r03 next-2b). The device runs a sequence on its own (HBM-resident scans, graph replay) in the
reference-tie-order mode (pf_odom_set_tie_order: VoxelGrid / rgbds order equal voxel keys as
libstdc++'s std::sort, src/odomEstimationClass.cpp:74, so every centroid is summed in the reference's
order); the committed trajectory tests/golden/odom_<name>_faithful.npz is the faithful oracle's own
free run (opts=0: std::sort, Householder-QR LM, FLANN-style kd-tree; tools/make_golden.py). The
remaining arithmetic differences are rounding: the LM's normal equations against QR, sums in another
order, the deterministic sincos against libm (~1e-14 m per frame, tests/test_gpu_parity_synced.py).

Round 3's device took getTransformFromSe3's (1 - cos(theta)) / theta^2 and (theta - sin(theta)) / theta^3
by half-angle identities, exact where the source's form cancels: up to ~1e-8 relative apart at small
theta, and on S64T (the town) an ill-conditioned stretch amplified that into a count flip at frame 338.
The device now takes the source's form (pf_geom.h se3_exp); the oracle's restatement of the device's LM
then tracks the faithful oracle on every one of the 4541 frames of both sequences (2.1e-11 m at worst
on S64T, profiles/r04_drift/), while rounding-level perturbations of the faithful path itself (QR or cost
sums reversed, libm's last bit) stay at 1e-14 m. Both scenes are therefore held to the tolerance on every
frame with every count identical. Without the tie order the runs separate at frame 47 (S64) / 7
(S64T)."""
import hashlib
import json
import os

import numpy as np
import pytest

from _util import pose_err

pytestmark = pytest.mark.gpu

TOL_T, TOL_R = 1e-4, 1e-5
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def free_run(pa, pfsynth, name, preset, theta, tie_order=True, lines=64):
    g = np.load(os.path.join(GOLDEN, "odom_%s_faithful.npz" % name))
    ref = g["poses"]
    n = ref.shape[0]
    names = [str(c) for c in g["count_names"]]
    checks = dict(zip((int(k) for k in g["input_frames"]), (str(h) for h in g["input_sha"])))
    seq = pfsynth.Sequence(preset, n_frames=n, seed=0)
    od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22)
    od.init(pa.make_lidar(lines, 3.0, 90.0), 0.4, 0, theta[0], theta[1], 0)
    od.set_tie_order(tie_order)
    cnt_h = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22)
    cnt_h.init(pa.make_lidar(lines, 3.0, 90.0), 0.4, 0, theta[0], theta[1], 0)
    cnt_h.set_tie_order(tie_order)
    first_count = None
    for f0 in range(0, n, 256):
        nf = min(256, n - f0)
        buf, cnt = seq.frames(f0, nf, threads=16)
        for i in range(nf):
            if f0 + i in checks:
                assert _sha(buf[i, :cnt[i]]) == checks[f0 + i], "generator output changed at frame %d" % (f0 + i)
        db = pa.DeviceBuffer(buf.nbytes)
        db.upload(buf)
        for i in range(nf):
            od.frame_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
            if first_count is None:                       # a second handle reads the counts per frame
                cnt_h.frame_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
                st = cnt_h.stats()
                if f0 + i > 0 and [st[c] for c in names] != list(g["counts"][f0 + i]):
                    first_count = f0 + i
        od.sync()
        db.free()
    p = od.poses()
    errs = np.array([pose_err(p[k], ref[k]) for k in range(n)])
    bad = np.nonzero((errs[:, 0] >= TOL_T) | (errs[:, 1] >= TOL_R))[0]
    gt = g["gt"]
    path = float(np.sum(np.linalg.norm(np.diff(gt[:, 4:7], axis=0), axis=1)))
    rep = {"name": name, "preset": preset, "theta": list(theta), "tie_order": tie_order, "frames": n,
           "first_frame_past_tolerance": int(bad[0]) if bad.size else None, "frames_past_tolerance": int(bad.size),
           "first_count_mismatch": first_count,
           "worst_m_within_first_1000": float(errs[:1000, 0].max()), "worst_m": float(errs[:, 0].max()),
           "worst_m_before_first_count_mismatch": float(errs[:first_count if first_count else n, 0].max()),
           "worst_rad": float(errs[:, 1].max()),
           "bit_identical_frames": int(np.sum(np.all(p == ref, axis=1))),
           "device_drift_pct": float(100 * np.linalg.norm(p[-1, 4:7] - gt[-1, 4:7]) / path),
           "faithful_drift_pct": float(100 * np.linalg.norm(ref[-1, 4:7] - gt[-1, 4:7]) / path),
           "path_m": path}
    print(json.dumps(rep))
    out = os.environ.get("PF_PARITY_OUT")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_free_%s%s.json" % (name, "_tie" if tie_order else "")), "w") as f:
            json.dump(rep, f, indent=1)
    return rep


def test_free_running_s64t(pa, pfsynth):
    """The town, configs[1] parameters, 4541 frames free-running in tie mode: every frame within the
    1e-4 m / 1e-5 rad tolerance of the faithful oracle's own run and every count identical (round 3:
    a count flip at frame 338 from the half-angle SE(3) form; profiles/r04_drift/)."""
    rep = free_run(pa, pfsynth, "s64t", "S64T", (0.4, 75))
    assert rep["first_count_mismatch"] is None, rep
    assert rep["frames_past_tolerance"] == 0, rep


def test_free_running_s64_headline_scene(pa, pfsynth):
    """configs[1] on S64 (the headline's street canyon), 4541 frames free-running in tie mode: every
    frame within the tolerance of the faithful oracle's free run, every count identical (measured: a
    worst 5.9e-12 m over the sequence, profiles/r03_parity_free/)."""
    rep = free_run(pa, pfsynth, "s64", "S64", (0.4, 75))
    assert rep["frames_past_tolerance"] == 0, rep
    assert rep["first_count_mismatch"] is None, rep


@pytest.mark.parametrize("name,preset", [("s64", "S64"), ("s64t", "S64T")])
def test_free_running_stable_order(pa, pfsynth, name, preset):
    """The default (stable radix) order, free-running: the last bits of the centroids differ from the
    reference's from frame 1 on, so the trajectories separate; where is recorded."""
    rep = free_run(pa, pfsynth, name, preset, (0.4, 75), tie_order=False)
    assert rep["frames"] == 4541
