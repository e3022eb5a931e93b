"""GPU: per-frame parity of Odom_BPF_EstimationClass (src/odomEstimationClass.cpp:649-1306) against the
reference-faithful oracle (pfref.OdomBPF, opts=0: libstdc++ std::sort tie orders, Householder-QR LM, the
FLANN-style kd-tree) on every frame, with the device in the reference tie order
(pf_odom_set_tie_order). As tests/test_gpu_parity_synced.py for the ES estimator: before frame k both
sides get the same state (the device's three maps with their age / p-index bytes after frame k - 1,
odom / last_odom / optimization_count), both run frame k, and everything is compared: pose within
1e-4 m / 1e-5 rad, every per-class count identical, every map's age / p-index bytes identical, map
coordinates within 1e-4 m. The oracle frames are independent and run in worker processes.

Two feeds: the raw-scan chain (pf_bpf_frame_scan_device: the device's own front end, bit-exact with the
oracle front end the workers run, tests/test_gpu_cls.py) over 1000 frames, and the update API
(pf_bpf_update) fed the oracle front end's clouds. The run's summary goes to
$PF_PARITY_OUT/parity_synced_bpf_<name>.json when that variable is set."""
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


def synced_bpf(pa, pfsynth, name, preset, n, raw_scan=True):
    from multiprocessing import get_context
    lid = (64, 3.0, 90.0)
    prm = (0.4, 0, 0.4, 75, 0)
    ctx = get_context("spawn")
    pool = ctx.Pool(_workers(), initializer=pw.init, initargs=(preset, n, 0, lid, None, prm, 0))
    od = pa.Odom_BPF_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22)
    od.init(pa.make_lidar(*lid), *prm)
    od.set_tie_order(True)
    seq = pfsynth.Sequence(preset, n_frames=n)
    clouds = pool.map(pw.bpf_clouds, range(n), chunksize=4) if not raw_scan else None
    report = dict(name=name, preset=preset, feed="raw scan" if raw_scan else "update API", frames=0, worst_t=0.0,
                  worst_r=0.0, worst_xyz=0.0, xyz_bitexact_frames=0, pose_bad=[], count_bad=[], map_bad=[])
    pending, dev, poses = {}, {}, []

    def drain(block, everything=False):
        for k in sorted(pending):
            if len(dev[k]) < 3:
                continue
            r = pending[k]
            if not (everything or (block and len(pending) > INFLIGHT // 2)) and not r.ready():
                continue
            _, pose, counts, maps = r.get(timeout=600)
            del pending[k]
            pw.compare_bpf(k, dev.pop(k), (pose, counts, maps), report, TOL_T, TOL_R, pose_err)

    try:
        for f0 in range(0, n, 128):
            nf = min(128, n - f0)
            buf, cnt = seq.frames(f0, nf, threads=16) if raw_scan else (None, None)
            for i in range(nf):
                k = f0 + i
                task = None
                if k > 0:
                    maps = [od._map(c) for c in range(3)]                  # S_{k-1}
                    if k - 1 in dev:
                        dev[k - 1] = dev[k - 1] + (maps,)
                    opt = od.state()["optimization_count"]
                    p1, p2 = poses[k - 1], poses[max(k - 2, 0)]
                    od.set_state(p1, p2, opt)
                    task = (k, maps, p1, p2, opt)
                if raw_scan:
                    pose = od.frame_host(buf[i, :cnt[i]])
                elif k == 0:
                    od.initMapWithPoints(*clouds[0])
                    pose = od.odom
                else:
                    pose = od.updatePointsToMap(*clouds[k])
                poses.append(np.asarray(pose))
                if task is not None:
                    dev[k] = (pose, pw.bpf_counts(od.stats()))
                    pending[k] = pool.apply_async(pw.run_bpf, (task,))
                drain(len(pending) > INFLIGHT)
                if k % 250 == 0:
                    print("%s: frame %d, compared %d, pose worst %.3e m, %d count / %d map mismatches"
                          % (name, k, report["frames"], report["worst_t"], len(report["count_bad"]),
                             len(report["map_bad"])), file=sys.stderr, flush=True)
        if n - 1 in dev:
            dev[n - 1] = dev[n - 1] + ([od._map(c) for c in range(3)],)
        drain(True, everything=True)
    finally:
        pool.terminate()
        pool.join()
    summary = dict(report, pose_bad=report["pose_bad"][:20], count_bad=report["count_bad"][:20],
                   map_bad=report["map_bad"][:20], n_pose_bad=len(report["pose_bad"]),
                   n_count_bad=len(report["count_bad"]), n_map_bad=len(report["map_bad"]))
    print(json.dumps(summary, default=str))
    out = os.environ.get("PF_PARITY_OUT")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_synced_bpf_%s.json" % name), "w") as f:
            json.dump(summary, f, default=str, indent=1)
    return report


def _check(rep, n_expected):
    assert rep["frames"] == n_expected
    assert not rep["pose_bad"], rep["pose_bad"][:5]
    assert not rep["count_bad"], rep["count_bad"][:5]
    assert not rep["map_bad"], rep["map_bad"][:5]


def test_bpf_synced_parity_raw_scan_chain(pa, pfsynth):
    """configs[1] parameters, the BPF raw-scan chain, every frame of the whole sequence (S64, 4541)"""
    _check(synced_bpf(pa, pfsynth, "S64_raw", "S64", 4541, raw_scan=True), 4540)


def test_bpf_synced_parity_update_api(pa, pfsynth):
    """the update API (pf_bpf_update) fed the oracle front end's clouds, every frame of 1000 (S64T)"""
    _check(synced_bpf(pa, pfsynth, "S64T_update", "S64T", 1000, raw_scan=False), 999)
