"""GPU: configs[3] (KITTI 00-10 as independent streams) through bench.py's multi-sequence path against the
reference-faithful oracle.

The path under test is bench.run_kitti11's: the eleven sequences (synthetic S64, seed = sequence number,
their KITTI frame counts scaled down here) assigned to 4 concurrent host threads by LPT, each thread owning
one handle (library default: the reference tie order; stage-A CU reservation 0, graph mode auto, as the
bench sets them) that runs its sequences back to back with pf_odom_reset between them -- the reference runs
every sequence through a fresh estimator (/root/reference/runkitti.py:86-108). Every other frame goes through
pf_odom_frame_device asynchronously, as in the bench. Every 8th frame of every sequence k > 0 is sampled: the
thread waits for the handle, takes its state (both maps with age / p-index bytes, odom and last_odom from
the pose array, optimization_count), runs frame k, and takes the pose, the counts and the maps after it.
The oracle (pfref, opts=0: libstdc++ std::sort tie orders, Householder-QR LM, FLANN-style kd-tree) runs the
same frame from the same state in worker processes (tests/_parity_worker.py), the transfer of
tests/test_gpu_parity_synced.py.

Bar (the strict one of the synced tests): the pose within 1e-4 m / 1e-5 rad, every count identical, both
maps' age / p-index bytes identical byte for byte and their coordinates within 1e-4 m. The summary is
written to $PF_PARITY_OUT/parity_synced_kitti11.json when that variable is set."""
import json
import os
import sys
import threading

import numpy as np
import pytest

import _parity_worker as pw
from _util import pose_err

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL_T, TOL_R = 1e-4, 1e-5
EVERY = 8
SCALE = 20              # KITTI frame counts / SCALE (at least MIN_FRAMES): 1166 frames over the 11 sequences
MIN_FRAMES = 40


def _workers():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 4
    return max(2, min(16, n))


def test_kitti11_multi_sequence_path_against_oracle(pa, pfsynth):
    sys.path.insert(0, ROOT)
    import bench
    from multiprocessing import get_context
    lengths = [max(MIN_FRAMES, n // SCALE) for n in bench.KITTI_SEQ_FRAMES]
    lid = (64, 3.0, 90.0)
    cfg = bench.ODOM_CFG
    prm = (cfg["map_resolution"], cfg["k_new"], cfg["theta_p"], cfg["theta_max"], cfg["weightType"])
    ctx = get_context("spawn")
    pool = ctx.Pool(_workers(), initializer=pw.init_multi,
                    initargs=("S64", {sq: n for sq, n in enumerate(lengths)}, lid, None, prm, 0))
    try:
        # every sequence HBM-resident first (bench.run_kitti11: load_frames per sequence)
        bufs, ptrs = [], {}
        for sq, n in enumerate(lengths):
            buf, counts = pfsynth.Sequence("S64", n_frames=n, seed=sq).frames(0, n, threads=16)
            db = pa.DeviceBuffer(buf.nbytes)
            db.upload(buf)
            bufs.append(db)
            ptrs[sq] = [(db.ptr + i * buf.shape[1] * 16, int(counts[i])) for i in range(n)]
        concurrent = 4
        shares = [[] for _ in range(concurrent)]             # LPT over the threads, as the bench
        loads = [0] * concurrent
        for sq in bench.lpt_assign(lengths, 1)[0]:
            j = loads.index(min(loads))
            shares[j].append(sq)
            loads[j] += lengths[sq]
        handles = []
        for _ in range(concurrent):
            od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22)
            od.init(pa.make_lidar(*lid, 0.1), **cfg)
            od.set_graph(4)
            od.set_stage_a_reserve(0)
            handles.append(od)
        tasks, dev, errors = [], {}, []
        lock = threading.Lock()

        def drive(od, items):
            try:
                for i, sq in enumerate(items):
                    if i:
                        od.sync()
                        od.reset()
                    for k, (ptr, n) in enumerate(ptrs[sq]):
                        if k == 0 or k % EVERY:
                            od.frame_device(ptr, n)
                            continue
                        od.sync()
                        poses = od.poses()
                        maps = [od._map(0), od._map(1)]
                        task = (sq, k, maps, poses[k - 1], poses[max(k - 2, 0)], od.state()["optimization_count"])
                        od.frame_device(ptr, n)
                        od.sync()
                        st = od.stats()
                        got = (od.poses()[k], {c: int(st[c]) for c in pw.COUNTS}, [od._map(0), od._map(1)])
                        with lock:
                            tasks.append(pool.apply_async(pw.run_multi, (task,)))
                            dev[(sq, k)] = got
                od.sync()
                assert od.stats()["errors"] == 0
            except Exception as e:                       # re-raised in the main thread
                errors.append(repr(e))

        ths = [threading.Thread(target=drive, args=(handles[j], shares[j])) for j in range(concurrent)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=600)
        assert not any(th.is_alive() for th in ths), "a sequence thread did not finish"
        assert not errors, errors
        report = dict(name="kitti11", frames=0, worst_t=0.0, worst_r=0.0, worst_xyz=0.0, xyz_bitexact_frames=0,
                      pose_bad=[], count_bad=[], map_bad=[], sequences=len(lengths), frames_per_sequence=lengths,
                      every=EVERY, concurrent=concurrent)
        for r in tasks:
            sq, k, pose, counts, maps = r.get(timeout=600)
            pw.compare((sq, k), dev[(sq, k)], (pose, counts, maps), report, TOL_T, TOL_R, pose_err)
    finally:
        pool.terminate()
        pool.join()
    expected = sum(len(range(EVERY, n, EVERY)) for n in lengths)
    summary = dict(report, pose_bad=report["pose_bad"][:20], count_bad=report["count_bad"][:20],
                   map_bad=report["map_bad"][:20])
    print(json.dumps(summary, default=str))
    out = os.environ.get("PF_PARITY_OUT")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_synced_kitti11.json"), "w") as f:
            json.dump(summary, f, default=str, indent=1)
    assert report["frames"] == expected
    assert not report["pose_bad"], report["pose_bad"][:5]
    assert not report["count_bad"], report["count_bad"][:5]
    assert not report["map_bad"], report["map_bad"][:5]
