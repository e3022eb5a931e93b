"""GPU: per-frame parity against the reference-faithful oracle on EVERY frame of whole sequences
(VERDICT r02 next-1). The north star's criterion is per frame on identical input clouds: so before
each frame k the device handle and the oracle (opts=0: libstdc++ std::sort tie orders as PCL's
VoxelGrid and src/odomEstimationClass.cpp:74 call them, Householder-QR LM as Ceres DENSE_QR, the
FLANN-style kd-tree) are put into the same estimator state -- the local maps with their age / p-index
bytes (pf_odom_get_map), odom, last_odom and optimization_count (pf_odom_set_state; the oracle gets
the same poses) -- and both run frame k of the scan sequence (featureExtraction + updatePointsToMap,
src/odomEstimationClass.cpp:229-282). The states come from the device's own run (the device's maps
after frame k - 1 are frame k's input), so every oracle frame is independent and the frames run in
parallel worker processes.

Per frame: the pose within 1e-4 m / 1e-5 rad, every count identical (input, down-sampled, map,
residual and association counts), the map's age / p-index bytes identical byte for byte (integer
work) and the map coordinates within 1e-4 m (f32 centroids summed in std::sort's order). The run's
worst case is written to $PF_PARITY_OUT/parity_synced_<name>.json when that variable is set."""
import json
import os
import sys

import numpy as np
import pytest

import _parity_worker as pw
from _util import pose_err

pytestmark = pytest.mark.gpu

TOL_T, TOL_R = 1e-4, 1e-5
INFLIGHT = 96


def _workers():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 4
    return max(2, min(16, n))


def synced_run(pa, pfsynth, name, preset, n, theta, lines=64, seed=0, ring_model=None, seed_map=None, every=1,
               tie_order=False, wt=0, k_new=0):
    from multiprocessing import get_context
    lid = (lines, 3.0, 90.0)
    prm = (0.4, k_new, theta[0], theta[1], wt)
    ctx = get_context("spawn")
    pool = ctx.Pool(_workers(), initializer=pw.init, initargs=(preset, n, seed, lid, ring_model, prm, 0))
    od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22)
    od.init(pa.make_lidar(*lid, ring_model=ring_model), *prm)
    od.set_tie_order(tie_order)
    seq = pfsynth.Sequence(preset, n_frames=n, seed=seed)
    report = dict(name=name, preset=preset, theta=list(theta), weight_type=wt, frames=0, worst_t=0.0, worst_r=0.0, worst_xyz=0.0,
                  xyz_bitexact_frames=0, pose_bad=[], count_bad=[], map_bad=[], tie_order=tie_order)
    pending, dev = {}, {}
    poses = []

    def drain(block, everything=False):
        """compare the finished oracle frames whose device maps are in; block: wait for the oldest ones
        until at most INFLIGHT / 2 remain (everything: until none remains)"""
        for k in sorted(pending):
            if len(dev[k]) < 3:                              # its maps arrive with the next frame
                continue
            r = pending[k]
            wait = everything or (block and len(pending) > INFLIGHT // 2)
            if not wait and not r.ready():
                continue
            _, pose, counts, maps = r.get(timeout=600)
            del pending[k]
            pw.compare(k, dev.pop(k), (pose, counts, maps), report, TOL_T, TOL_R, pose_err)

    try:
        prev_maps, task_pose = None, None
        for f0 in range(0, n, 128):
            nf = min(128, n - f0)
            buf, cnt = seq.frames(f0, nf, threads=16)
            for i in range(nf):
                k = f0 + i
                x = buf[i, :cnt[i]]
                checked = k > 0 and k % every == 0
                if k > 0 and (checked or k - 1 in dev):
                    maps = [od._map(0), od._map(1)]                 # S_{k-1}
                    if k - 1 in dev:
                        dev[k - 1] = dev[k - 1] + (maps,)
                if checked:
                    opt = od.state()["optimization_count"]
                    p1, p2 = poses[k - 1], poses[max(k - 2, 0)]
                    od.set_state(p1, p2, opt)
                    task_pose = (maps, p1, p2, opt)
                pose = od.frame_host(x)
                if k == 0 and seed_map is not None:
                    od.set_map(1, *seed_map)
                poses.append(pose)
                if checked:
                    st = od.stats()
                    dev[k] = (pose, {c: int(st[c]) for c in pw.COUNTS})
                    maps, p1, p2, opt = task_pose
                    pending[k] = pool.apply_async(pw.run, ((k, maps, p1, p2, opt),))
                if len(pending) > INFLIGHT:
                    drain(True)
                else:
                    drain(False)
                if k % 500 == 0:
                    print("%s: frame %d, compared %d, pose worst %.3e m, %d count / %d map mismatches"
                          % (name, k, report["frames"], report["worst_t"], len(report["count_bad"]),
                             len(report["map_bad"])), file=sys.stderr, flush=True)
        last = n - 1
        if last in dev:
            dev[last] = dev[last] + ([od._map(0), od._map(1)],)
        drain(True, everything=True)
    finally:
        pool.terminate()
        pool.join()
    out = os.environ.get("PF_PARITY_OUT")
    summary = dict(report, pose_bad=report["pose_bad"][:20], count_bad=report["count_bad"][:20],
                   map_bad=report["map_bad"][:20], n_pose_bad=len(report["pose_bad"]),
                   n_count_bad=len(report["count_bad"]), n_map_bad=len(report["map_bad"]))
    print(json.dumps(summary, default=str))
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_synced_%s.json" % name), "w") as f:
            json.dump(summary, f, default=str, indent=1)
    return report


def _check(rep, n_expected):
    assert rep["frames"] == n_expected
    assert not rep["pose_bad"], rep["pose_bad"][:5]
    assert not rep["count_bad"], rep["count_bad"][:5]
    assert not rep["map_bad"], rep["map_bad"][:5]


CONFIGS = [
    # name, preset, frames, (theta_p, theta_max), lines, weightType, map xyz NOT bit-identical at most
    ("configs1_S64", "S64", 4541, (0.4, 75), 64, 0, 10),      # configs[1]: the headline workload, every frame
    ("configs0_S64", "S64", 4541, (0.0, 0), 64, 0, 10),       # configs[0]: FLOAM-equivalent parameters
    ("configs2_S32", "S32", 3000, (1.0, 200), 32, 0, 10),     # configs[2]: 32-line campus, theta 1 / 200
    ("dense_S64V", "S64V", 1000, (0.4, 75), 64, 0, 10),       # dense vegetation scene, KITTI-like map sizes
    ("town_S64T", "S64T", 4541, (0.4, 75), 64, 0, 10),        # the well-conditioned town (free-running scene)
    ("configs1_S64_wt2", "S64", 4541, (0.4, 75), 64, 2, 10),  # weightType 2: pfilter_kitti.launch:7's default
    ("configs1_S64_wt1", "S64", 4541, (0.4, 75), 64, 1, 10),  # weightType 1: the observe weight alone
    ("configs1_S64_wt12", "S64", 4541, (0.4, 75), 64, 12, 10),  # weightType 12: observe and sparsity averaged
]


@pytest.mark.parametrize("name,preset,n,theta,lines,wt,xyz_off", CONFIGS)
def test_synced_parity_every_frame(pa, pfsynth, name, preset, n, theta, lines, wt, xyz_off):
    """Reference tie order on (pf_odom_set_tie_order): the strict per-frame bar on every frame, plus the
    map coordinates' bits. The permutation the tie order reproduces is integer work and its observable is
    the f32 centroid bits, so the maps must come out bit-identical on (nearly) every frame: a wrong order of
    an order-dependent voxel group moves its centroid by an ulp on every frame it recurs. The only other
    source of an ulp is the pose: the device's normal-equation LM and the oracle's Householder QR agree to
    ~1e-12 m, and an appended point whose exact transformed coordinate lies within that of an f32
    rounding boundary rounds the other way (about 1e-7 per coordinate; a handful over a 4540-frame
    sequence of ~7k appended points per frame: r03 saw 0 of 9080 maps on configs[0]/[1]/[2] and S64V and
    1 on S64T, round 6 2 on configs[0]). At most 10 of the 2 x frames maps may differ, each within the
    tolerance."""
    rep = synced_run(pa, pfsynth, name + "_tie", preset, n, theta, lines=lines, tie_order=True, wt=wt)
    _check(rep, n - 1)
    if xyz_off is not None:
        assert rep["xyz_bitexact_frames"] >= 2 * rep["frames"] - xyz_off, (rep["xyz_bitexact_frames"], rep["frames"])


@pytest.mark.parametrize("k_new,theta", [(2, (0.4, 75)), (1, (0.8, 30))])
def test_synced_parity_pindex_variants(pa, pfsynth, k_new, theta):
    """The p-index filter's other parameters (k_new > 0 keeps map points younger than k_new rounds,
    src/odomEstimationClass.cpp:350-353) over the whole S64 sequence in the tie order, every frame synced:
    the strict bar of test_synced_parity_every_frame."""
    rep = synced_run(pa, pfsynth, "pindex_k%d_S64_tie" % k_new, "S64", 4541, theta, tie_order=True, k_new=k_new)
    _check(rep, 4540)
    assert rep["xyz_bitexact_frames"] >= 2 * rep["frames"] - 10, (rep["xyz_bitexact_frames"], rep["frames"])


@pytest.mark.parametrize("name,preset,n,theta,lines", [c[:5] for c in CONFIGS if c[5] == 0])
def test_synced_statistics_stable_order(pa, pfsynth, name, preset, n, theta, lines):
    """A statistics run, not a parity check: the stable-order mode (VoxelGrid / rgbds sorted stably,
    pf_odom_set_tie_order off) does NOT meet the per-frame bar -- its centroids differ from the
    reference's in the last bits, which tips a residual or map count on a few per cent of frames and a
    few poses past 1e-4 m (profiles/r03_parity_synced/). Every 4th frame is compared and the summary
    recorded; what is asserted is the envelope that deviation stayed in (r03: worst 1.44e-4 m /
    1.4e-5 rad, count differences on 1.9 % of compared frames): 10x the pose tolerance and 5 % of frames."""
    rep = synced_run(pa, pfsynth, name, preset, n, theta, lines=lines, every=4)
    assert rep["frames"] == len(range(4, n, 4))
    assert rep["worst_t"] < 10 * TOL_T and rep["worst_r"] < 10 * TOL_R, (rep["worst_t"], rep["worst_r"])
    assert len(rep["count_bad"]) <= 0.05 * rep["frames"], len(rep["count_bad"])


def _seed_map_2m(pfref, pfsynth):
    m = pfref.rgbds(pfsynth.dense_map(7_000_000, seed=5), 0.8)[:2_000_000, :3]
    return (np.ascontiguousarray(m), np.zeros((m.shape[0], 2), np.uint8))


def test_synced_parity_s128_2m_point_map_tie(pa, pfref, pfsynth):
    """configs[4] in the reference tie order, the mode bench.py runs it in: synthetic 128-line scans
    (~200k points, the linear beam-model extension) against a 2,000,000-point surf map (voxel centroids of
    the dense block at the 0.8 m leaf, seeded after frame 0), theta 0 so the map keeps its size; every
    frame synced against the faithful oracle (opts=0), the strict bar: every count identical, both maps'
    r / g bytes identical, pose and map coordinates within the tolerance. Each rgbds sort of the ~2M-point
    voxel-ordered map plus the appended points reaches libstdc++'s depth limit on a ~820k-key segment and
    runs the big partition levels and the heap tier's global path at their full size
    (src/odomEstimationClass.cpp:74, 606-626). 100 frames: the frames bench.py's configs4 leg times
    (VERDICT r05 next-4)."""
    rep = synced_run(pa, pfsynth, "configs4_S128_2M_tie", "S128", 101, (0.0, 0), lines=128,
                     ring_model=(15.0, -25.0), seed_map=_seed_map_2m(pfref, pfsynth), tie_order=True)
    _check(rep, 100)


def test_synced_parity_s128_2m_point_map_stable(pa, pfref, pfsynth):
    """configs[4] in the stable-sort mode, every frame synced: within the strict bar on these 12 frames
    (round 3), although the stable mode does not meet it in general (test_synced_statistics_stable_order)."""
    rep = synced_run(pa, pfsynth, "configs4_S128_2M", "S128", 13, (0.0, 0), lines=128, ring_model=(15.0, -25.0),
                     seed_map=_seed_map_2m(pfref, pfsynth), tie_order=False)
    _check(rep, 12)
