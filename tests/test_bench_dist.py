"""CPU: the multi-GPU harness of bench.py at world size 2 over gloo (the GPU box uses RCCL):
max-over-ranks time, summed frames, and the all-gather of every rank's pose array (ragged)."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    poses = np.arange(7 * (3 + rank), dtype=np.float64).reshape(-1, 7) + 100 * rank
    el, frames, allp = bench.reduce_results(dist, 1.0 + rank, 10 + rank, poses, "cpu")
    out[rank] = (el, frames, [a.tolist() for a in allp])
    dist.destroy_process_group()


def test_reduce_results_gloo_world2():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    for rank in (0, 1):
        el, frames, allp = res[rank]
        assert el == 2.0 and frames == 21
        assert len(allp) == 2
        for r in (0, 1):
            exp = np.arange(7 * (3 + r), dtype=np.float64).reshape(-1, 7) + 100 * r
            np.testing.assert_array_equal(np.array(allp[r]), exp)


def test_lpt_assignment_of_kitti_sequences():
    """configs[3]: the 11 KITTI sequences over 1/2/4/8 ranks by longest processing time; every
    sequence exactly once, and at 8 ranks the makespan is seq 02's length."""
    sys.path.insert(0, ROOT)
    import bench
    L = bench.KITTI_SEQ_FRAMES
    for world in (1, 2, 4, 8):
        a = bench.lpt_assign(L, world)
        assert sorted(s for r in a for s in r) == list(range(11))
        loads = [sum(L[s] for s in r) for r in a]
        assert max(loads) - min(loads) <= max(L)
    a8 = bench.lpt_assign(L, 8)
    assert max(sum(L[s] for s in r) for r in a8) == L[2] == 4661
    assert bench.lpt_assign(L, 1) == [[2, 0, 8, 5, 9, 10, 1, 6, 7, 3, 4]]


def _bcast_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    arr = np.arange(24, dtype=np.float32).reshape(6, 4) if rank == 0 else None
    got = bench.broadcast_array(dist, arr, 0, "cpu")
    out[rank] = (got.tolist(), bench.shard_bounds(200_000, world, rank))
    dist.destroy_process_group()


def test_knn_shard_broadcast_and_bounds_gloo_world2():
    """configs[4] multi-GPU kNN: the map reaches every rank by one broadcast; the query shards tile
    [0, Q) exactly."""
    sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 3, 8):
        bounds = [bench.shard_bounds(200_003, world, r) for r in range(world)]
        assert bounds[0][0] == 0 and bounds[-1][1] == 200_003
        assert all(bounds[i][1] == bounds[i + 1][0] for i in range(world - 1))
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_bcast_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    for rank in (0, 1):
        np.testing.assert_array_equal(np.array(res[rank][0]), np.arange(24, dtype=np.float32).reshape(6, 4))
    assert res[0][1] == (0, 100_000) and res[1][1] == (100_000, 200_000)


def test_gpus_flag_launches_the_ranks():
    """`python bench.py --gpus 2` outside torch.distributed.run launches 2 ranks itself (gloo and a
    stubbed pipeline here): n_gpus 2, frames summed over ranks, time = the slowest rank's."""
    import json
    import subprocess
    env = dict(os.environ, PF_BENCH_BACKEND="gloo", PF_BENCH_STUB="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "10",
                        "--warmup", "0", "--no-cpu"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["stub"]
    assert abs(out["value"] - 20 / 2.0) < 1e-9           # 2 x 10 frames over the slower rank's 2 s


def test_gpus_flag_must_match_world():
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse(["--gpus", "4"])
    assert bench.resolve_world(a, {}) == (4, True)
    assert bench.resolve_world(a, {"WORLD_SIZE": "4"}) == (4, False)
    assert bench.resolve_world(bench.parse([]), {"WORLD_SIZE": "2"}) == (2, False)
    assert bench.resolve_world(bench.parse([]), {}) == (1, False)
    import pytest
    with pytest.raises(SystemExit):
        bench.resolve_world(a, {"WORLD_SIZE": "2"})


def _launch(extra):
    import json
    import subprocess
    env = dict(os.environ, PF_BENCH_BACKEND="gloo", PF_BENCH_STUB="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + extra, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_kitti11_mode_gloo_world2(tmp_path):
    """configs[3] (`--sequences kitti11`) at 2 ranks over gloo with the stubbed pipeline: one JSON line,
    n_gpus 2, all 23,201 frames of the 11 sequences counted once, time = the slowest rank's; every
    sequence's trajectory all-gathered and written as KITTI pose files (runkitti.py:111-157)."""
    out = _launch(["--sequences", "kitti11", "--warmup", "0", "--poses-out", str(tmp_path)])
    assert out["n_gpus"] == 2 and out["stub"] and out["scaling"] == "strong"
    assert out["steps"] == sum(bench_frames()) == 23201
    assert abs(out["value"] - 23201 / 2.0) < 1e-6
    assert sorted(s for r in out["config"]["assignment"] for s in r) == list(range(11))
    # the pose all-gather: every sequence's stub trajectory reaches rank 0 complete and in order
    assert out["poses"]["sequences"] == list(range(11))
    assert out["poses"]["frames"] == bench_frames()
    assert out["poses"]["stub_match"] is True
    sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
    import kitti
    for sq, n in enumerate(bench_frames()):
        m = kitti.read_poses(str(tmp_path / ("%02d.txt" % sq)))
        assert m.shape[0] == n
        assert np.allclose(m[:, 0, 3], np.arange(n)) and np.allclose(m[:, 1, 3], sq)


def bench_frames():
    sys.path.insert(0, ROOT)
    import bench
    return bench.KITTI_SEQ_FRAMES


def test_knn_shard_mode_gloo_world2():
    """configs[4] kNN over 2 ranks (`--knn-shard`) over gloo with the stubbed kernel: the map and queries
    are broadcast from rank 0, the slowest rank's time and the summed algorithmic bytes reduced."""
    out = _launch(["--knn-shard"])
    assert out["n_gpus"] == 2 and out["stub"]
    assert abs(out["ms_per_step"] - 2.0) < 1e-9                  # rank 1's 2 ms
    assert abs(out["value"] - 2000 / 2e-3) < 1e-3
    assert abs(out["aggregate_alg_GBps"] - 2000 * 1000.0 / 2e-3 / 1e9) < 0.1


def test_sort_order_flags():
    """The headline runs in the reference tie order by default (the mode whose results are the
    reference's frame by frame); the other order is reported beside it; configs[4]'s leg runs in the tie
    order too (its depth-limit segment of ~820k distinct keys is sorted by one device-wide radix sort,
    DESIGN.md section 4)."""
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse([])
    assert a.order == "tie" and a.configs4_order == "tie" and a.other_order_frames > 0
    b = bench.parse(["--order", "stable", "--configs4-order", "stable", "--other-order-frames", "0"])
    assert b.order == "stable" and b.configs4_order == "stable" and b.other_order_frames == 0


def test_cpu_baseline_sample_order():
    """bench.py's CPU baseline times one frame per stratum of the headline's frames, strata in van der
    Corput order: a permutation of the strata whose every prefix is spread over the whole sequence, so a
    budget that ends the sample early still covers early and late frames alike."""
    sys.path.insert(0, ROOT)
    import bench
    for n in (1, 2, 7, 64, 512, 1000):
        o = bench.vdc_order(n)
        assert sorted(o) == list(range(n))
    o = bench.vdc_order(512)
    for m in (8, 32, 128):
        pre = sorted(o[:m])
        assert pre[0] < 512 // m and pre[-1] >= 512 - 512 // m      # both ends covered
        assert max(np.diff(pre)) <= 2 * 512 // m                    # no gap above twice the stride
    a = np.array([0.0, 0.0, 0.0, 1.0, 1.0, 2.0, 3.0])
    b = a.copy()
    b[4] += 1e-5
    dt, dr = bench.pose_diff(a, b)
    assert abs(dt - 1e-5) < 1e-12 and dr == 0.0
    c = a.copy()
    c[:4] = -c[:4]                                                  # q and -q are the same rotation
    assert bench.pose_diff(a, c) == (0.0, 0.0)


def test_kitti11_hw_queues_raised_only_for_concurrent_sequences():
    """configs[3] with several sequences per GPU raises the process's hardware queues to 16 before the HIP
    runtime starts (bench.kitti11_hw_queues); never lowers a larger value, leaves other runs alone."""
    import bench
    env = {"GPU_MAX_HW_QUEUES": "4"}
    assert bench.kitti11_hw_queues(bench.parse(["--sequences", "kitti11", "--concurrent", "4"]), env) == 16
    assert env["GPU_MAX_HW_QUEUES"] == "16"
    env = {"GPU_MAX_HW_QUEUES": "24"}
    assert bench.kitti11_hw_queues(bench.parse(["--sequences", "kitti11", "--concurrent", "4"]), env) == 24
    env = {}
    assert bench.kitti11_hw_queues(bench.parse(["--sequences", "kitti11", "--concurrent", "1"]), env) is None
    assert bench.kitti11_hw_queues(bench.parse([]), env) is None and env == {}
