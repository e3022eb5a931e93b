"""Benchmark: LiDAR frames/sec (scan -> pose) on a KITTI-00-like 64-line sequence, MI355X.

A "step" is one frame of the hot path: featureExtraction + updatePointsToMap (the reference's timed
boundary, src/laserProcessingNode.cpp:71-78 + src/odomEstimationNode copy.cpp:92-100). Workload =
BASELINE.json configs[1]: 64 lines, min_dis 3 / max_dis 90, k_new=0 theta_p=0.4 theta_max=75,
weightType 0, map_resolution 0.4, on the synthetic S64 sequence (ray-cast urban scene, KITTI-00
length 4541 frames; no network for KITTI itself, real .bin scans are used when PF_KITTI_ROOT is set).
All scans are resident in HBM before the timed region. Per-frame poses stay on the device.

  python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1: one process per GPU (torch.distributed.run), one independent sequence per rank (weak
scaling); RCCL all-gather of the per-rank pose arrays after the timed region. Run as
`python bench.py --gpus N` outside torch.distributed.run, the script launches the N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU) and exits with its code.

Extra legs (rank 0, N=1 only, outside the timed region):
  roofline     exact 5-NN kernel on config 5 (2M-point map, 200k queries) timed with HIP events on
               its own stream; achieved = algorithmic bytes / avg kernel time
  cpu_baseline the pfref oracle (single thread, reference-faithful options) on a bounded sample of
               the same frames
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "pfilter-noetic_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(PKG, "synth"))

METRIC = "LiDAR frames/sec (scan→pose) on KITTI-00 64-line; kNN HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
KITTI00_FRAMES = 4541


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks). Without WORLD_SIZE in the environment and N > 1, the ranks are "
                         "launched here; under torch.distributed.run it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=KITTI00_FRAMES - 20)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-roofline", action="store_true", help="skip the kNN roofline leg")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--graph-mode", type=int, default=4,
                    help="pf_odom_set_graph: bit 0 stage A, bit 1 stage B, 4 = auto (the default: stage A, and "
                         "stage B when the process holds several handles)")
    ap.add_argument("--sequences", default="one", choices=["one", "kitti11"],
                    help="one: an independent sequence per rank (weak scaling, the default); kitti11: "
                         "configs[3], KITTI 00-10 LPT-assigned to the ranks (strong scaling)")
    ap.add_argument("--knn-shard", action="store_true",
                    help="configs[4] kNN leg over the ranks: map broadcast once (RCCL), queries sharded")
    ap.add_argument("--order", default="tie", choices=["tie", "stable"],
                    help="sort order of every leg: tie = libstdc++ std::sort's order of equal keys (the "
                         "reference's results frame by frame, pf_odom_set_tie_order), stable = stable sorts")
    ap.add_argument("--other-order-frames", type=int, default=1000,
                    help="frames of the headline workload run again in the other sort order (0: skip)")
    ap.add_argument("--poses-out", default=None,
                    help="kitti11: directory for the gathered trajectories, one KITTI pose file per sequence "
                         "(NN.txt, 3x4 row-major per frame, runkitti.py's layout)")
    ap.add_argument("--concurrent", type=int, default=4,
                    help="kitti11: host threads per GPU, each driving its share of the sequences on its own "
                         "handle and streams")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 PMC passes that measure the kNN kernel's fabric traffic")
    ap.add_argument("--bpf-frames", type=int, default=1000,
                    help="frames of the Odom_BPF_EstimationClass leg (SURVEY §8(f) rank 1); 0 = skip")
    ap.add_argument("--leg-frames", type=int, default=1000,
                    help="frames of each extra ES leg (configs[0] theta=0 on S64; the S64V dense scene at "
                         "configs[1] and at theta=0); 0 = skip them")
    ap.add_argument("--leg-cpu-seconds", type=float, default=8.0, help="CPU baseline sample of each extra leg")
    ap.add_argument("--only-headline", action="store_true",
                    help="the headline line alone (no roofline, CPU, BPF, ES, PCIe, node, pageable or configs4 "
                         "legs): for profiling the frame path")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the PCIe-inclusive leg (the headline's frames from pinned host RAM through "
                         "pf_odom_frame_host; reported as pcie_inclusive, never as value)")
    ap.add_argument("--pageable-frames", type=int, default=500,
                    help="frames of pf_odom_frame_host from pageable memory (pcie_pageable); 0 = skip")
    ap.add_argument("--configs4-frames", type=int, default=100,
                    help="frames of the configs[4] pipeline leg (S128 scans, 2M-point map); 0 = skip")
    ap.add_argument("--configs4-order", default="tie", choices=["tie", "stable"],
                    help="sort order of the configs[4] leg (default the reference's tie order: the 2M-point "
                         "voxel-ordered map with a few thousand appended points drives introsort to its "
                         "depth limit on a ~820k-key segment of distinct keys, which k_tie_heap sorts by a "
                         "bitonic network; DESIGN.md section 5)")
    ap.add_argument("--node-frames", type=int, default=1000,
                    help="frames of the node call pattern (pf_fe_extract -> pf_odom_update); 0 = skip")
    ap.add_argument("--full-frames", type=int, default=KITTI00_FRAMES - 20,
                    help="full_sequence object: the headline workload over this many timed frames after 20 "
                         "warm-up frames whatever --steps is (the KITTI-00 length by default), with its own "
                         "stage times, stratified CPU baseline and node call patterns; 0 = skip")
    ap.add_argument("--full-cpu-seconds", type=float, default=40.0,
                    help="CPU budget of the full sequence's stratified baseline (512 strata take ~12 s)")
    a = ap.parse_args(argv)
    if a.only_headline:
        a.no_roofline = a.no_cpu = a.no_pcie = True
        a.bpf_frames = a.leg_frames = a.pageable_frames = a.node_frames = a.configs4_frames = a.full_frames = 0
    return a


def resolve_world(args, env):
    """(world, launch): the rank count and whether this process must launch the ranks itself.
    Refuses a --gpus that disagrees with a torch.distributed.run world."""
    env_world = env.get("WORLD_SIZE")
    if env_world is not None:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
        return world, False
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return n, n > 1


def launch_ranks(n, argv, port=None):
    """Runs this script under torch.distributed.run with n ranks (a child process: nothing here has
    touched the GPU) and returns its exit code."""
    import socket
    import subprocess
    if port is None:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def lidar_cfg():
    import pfilter_amd as pa
    return pa.make_lidar(64, 3.0, 90.0, 0.1)


ODOM_CFG = dict(map_resolution=0.4, k_new=0, theta_p=0.4, theta_max=75, weightType=0)
# the sort order of VoxelGrid / rgbds / the featureExtraction sectors in every leg of the run (--order):
# "tie" = libstdc++ std::sort's order of equal keys (pf_odom_set_tie_order, the reference's own results
# frame by frame), "stable" = stable radix sorts and rgbds by merge (faster, last bits of the centroids
# differ). ORDER[0] is read by every handle the bench creates.
ORDER = ["tie"]


def set_order(h):
    """apply the run's sort order to a freshly initialised odometry handle"""
    h.set_tie_order(ORDER[0] == "tie")


# KITTI odometry sequences 00-10 (frame counts)
KITTI_SEQ_FRAMES = [4541, 1101, 4661, 801, 271, 2761, 1101, 1101, 4071, 1591, 1201]


def lpt_assign(lengths, world):
    """Longest-processing-time assignment of sequences to ranks: longest first, each to the least
    loaded rank (ties to the lowest rank). Returns the sequence indices of every rank."""
    loads = [0] * world
    out = [[] for _ in range(world)]
    for sq in sorted(range(len(lengths)), key=lambda i: (-lengths[i], i)):
        r = min(range(world), key=lambda k: (loads[k], k))
        out[r].append(sq)
        loads[r] += lengths[sq]
    return out


def load_frames(seq_id, total, threads, preset="S64"):
    """Yields (frame_index, [nf,cap,4] chunk, counts, description) of sequence `seq_id` (synthetic
    `preset` with seed = seq_id, or KITTI sequence seq_id under PF_KITTI_ROOT)."""
    import pfsynth
    rank = seq_id
    kroot = os.environ.get("PF_KITTI_ROOT")
    if kroot:
        seqdir = os.path.join(kroot, "sequences", "%02d" % rank, "velodyne")
        files = sorted(f for f in os.listdir(seqdir) if f.endswith(".bin"))[:total]
        frames = [np.fromfile(os.path.join(seqdir, f), np.float32).reshape(-1, 4) for f in files]
        cap = max(f.shape[0] for f in frames)
        buf = np.zeros((len(frames), cap, 4), np.float32)
        counts = np.zeros(len(frames), np.int64)
        for i, f in enumerate(frames):
            buf[i, :f.shape[0]] = f
            counts[i] = f.shape[0]
        yield 0, buf, counts, "kitti-%02d" % rank
        return
    seq = pfsynth.Sequence(preset, n_frames=total, seed=rank)
    chunk = 256
    for f0 in range(0, total, chunk):
        nf = min(chunk, total - f0)
        buf, counts = seq.frames(f0, nf, threads=threads)
        yield f0, buf, counts, "synthetic %s seed %d" % (preset, rank)


GRAPH_NAMES = {0: "none", 1: "stage A", 2: "stage B", 3: "stages A and B", 4: "auto"}


def graph_mode(args):
    """pf_odom_set_graph mode: --no-graph = eager launches in both stages"""
    return 0 if args.no_graph else args.graph_mode


def run_gpu(rank, local_rank, world, steps, warmup, threads, use_graph, barrier, keep_host=False):
    """The headline: every scan HBM-resident before the timed region. keep_host: the scans also stay in
    pinned host RAM (pf_host_alloc; the HBM copies are uploaded from there) for the PCIe-inclusive and
    node-pattern legs, which read the same frames."""
    import pfilter_amd as pa
    total = warmup + steps
    lid = lidar_cfg()
    od = pa.Odom_ES_EstimationClass(device=local_rank, max_points=300000, map_capacity=1 << 22)
    od.init(lid, **ODOM_CFG)
    set_order(od)
    od.set_graph(use_graph)
    if os.environ.get("PF_BENCH_STAGE_A_RESERVE"):           # development sweep of the stage-A CU mask
        od.set_stage_a_reserve(int(os.environ["PF_BENCH_STAGE_A_RESERVE"]))
    # stage every scan in HBM (untimed)
    bufs, ptrs, hbufs, hptrs = [], [], [], []
    data_desc = None
    npts = []
    for f0, buf, counts, desc in load_frames(rank, total, threads):
        data_desc = desc
        src = buf
        if keep_host:
            hb = pa.HostBuffer(buf.nbytes)
            src = hb.view(buf.shape)
            src[...] = buf
            hbufs.append(hb)
        db = pa.DeviceBuffer(buf.nbytes, device=local_rank)
        db.upload(src)
        stride = buf.shape[1] * 16
        for i in range(buf.shape[0]):
            ptrs.append((db.ptr + i * stride, int(counts[i])))
            if keep_host:
                hptrs.append((hb.ptr + i * stride, int(counts[i])))
            npts.append(int(counts[i]))
        bufs.append(db)
        del buf, src
    for k in range(min(warmup, len(ptrs))):
        od.frame_device(*ptrs[k])
    od.sync()
    barrier()
    t0 = time.perf_counter()
    for k in range(warmup, len(ptrs)):
        od.frame_device(*ptrs[k])
    t_enq = time.perf_counter()    # the host's enqueue time (frames are submitted asynchronously)
    od.sync()                      # raises on a sticky device error: a failed frame is never counted
    barrier()
    t1 = time.perf_counter()
    poses = od.poses()
    stats = od.stats()
    if stats["errors"]:
        raise RuntimeError("device error words 0x%x during the timed region" % stats["errors"])
    nframes = len(ptrs) - warmup
    return dict(elapsed=t1 - t0, frames=nframes, poses=poses, stats=stats, data=data_desc, enqueue=t_enq - t0,
                mean_points=float(np.mean(npts)) if npts else 0.0, od=od, bufs=bufs, ptrs=ptrs, hbufs=hbufs,
                hptrs=hptrs)


def run_kitti11(rank, local_rank, world, warmup, threads, use_graph, barrier, concurrent=1):
    """Config 4: KITTI 00-10 (frame counts of the real sequences) as independent streams, LPT-assigned
    to the ranks. On a rank, `concurrent` host threads (at most the handles a device admits) each own
    one handle and run their share of the rank's sequences back to back, pf_odom_reset between
    sequences (a fresh map and pose, as the reference restarts its nodes per sequence: runkitti.py).
    Scans are HBM-resident before the timed region; `warmup` frames run on every handle first."""
    import threading
    import pfilter_amd as pa
    mine = lpt_assign(KITTI_SEQ_FRAMES, world)[rank]
    seqs = []                      # (frame pointers, buffers) per sequence, in LPT order
    for sq in mine:
        bufs, ptrs = [], []
        for f0, buf, counts, desc in load_frames(sq, KITTI_SEQ_FRAMES[sq], threads):
            db = pa.DeviceBuffer(buf.nbytes, device=local_rank)
            db.upload(buf)
            stride = buf.shape[1] * 16
            ptrs += [(db.ptr + i * stride, int(counts[i])) for i in range(buf.shape[0])]
            bufs.append(db)
        seqs.append((ptrs, bufs))
        log("kitti11: sequence %02d staged in HBM (%d frames)" % (sq, len(ptrs)))   # progress on a long staging
    nthreads = max(1, min(concurrent, len(seqs)))
    handles = []
    for _ in range(nthreads):
        od = pa.Odom_ES_EstimationClass(device=local_rank, max_points=300000, map_capacity=1 << 22)
        od.init(lidar_cfg(), **ODOM_CFG)
        set_order(od)
        od.set_graph(use_graph)
        if concurrent > 1:
            od.set_stage_a_reserve(0)      # several sequences share the GPU: stage A may use every CU
        for ptr, n in seqs[0][0][:warmup]:
            od.frame_device(ptr, n)
        od.sync()
        od.reset()
        handles.append(od)
    shares = [[] for _ in range(nthreads)]         # LPT again over the threads
    loads = [0] * nthreads
    for sq, (ptrs, _) in zip(mine, seqs):
        j = loads.index(min(loads))
        shares[j].append((sq, ptrs))
        loads[j] += len(ptrs)

    errors = []
    poses = {}                     # sequence -> its trajectory (n, 7), read before the handle's reset

    def drive(od, items):          # ctypes releases the GIL inside every C call
        try:
            for k, (sq, ptrs) in enumerate(items):
                if k:
                    od.sync()          # raises on a sticky device error of the finished sequence
                    poses[items[k - 1][0]] = od.poses()
                    od.reset()
                for ptr, n in ptrs:
                    od.frame_device(ptr, n)
                log("kitti11: sequence %02d enqueued (%.1f s)" % (sq, time.perf_counter() - t0))
            od.sync()
            if items:
                poses[items[-1][0]] = od.poses()
        except Exception as e:     # re-raised in the main thread: a failed frame is never counted
            errors.append(repr(e))

    log("kitti11: %d handles ready" % nthreads)
    barrier()
    t0 = time.perf_counter()
    ths = [threading.Thread(target=drive, args=(handles[j], shares[j])) for j in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    barrier()
    el = time.perf_counter() - t0
    if errors:
        raise RuntimeError("kitti11: device errors on rank %d: %s" % (rank, errors))
    for od in handles:
        assert od.stats()["errors"] == 0
    return dict(elapsed=el, frames=sum(len(p) for p, _ in seqs), sequences=["%02d" % sq for sq in mine],
                poses=poses)


def stub_poses(sq, n):
    """the stubbed pipeline's trajectory of sequence sq (pose7 = qx qy qz qw tx ty tz): identity
    rotations, x = frame, y = sequence"""
    p = np.zeros((n, 7))
    p[:, 3] = 1.0
    p[:, 4] = np.arange(n)
    p[:, 5] = sq
    return p


def gather_poses(poses, world, rank, dist, dev):
    """configs[3]'s one collective (after the timed region): every rank's per-sequence trajectories to
    every rank, as one padded float64 all_gather (each rank's sequences and their frame counts follow
    from the LPT assignment, so no sizes travel). Returns {sequence: (n, 7)} of every sequence."""
    assign = lpt_assign(KITTI_SEQ_FRAMES, world)
    sizes = [sum(KITTI_SEQ_FRAMES[sq] for sq in assign[r]) for r in range(world)]
    mine = np.zeros((max(sizes), 7))
    o = 0
    for sq in assign[rank]:
        n = KITTI_SEQ_FRAMES[sq]
        p = poses[sq]
        if p.shape != (n, 7):
            raise RuntimeError("sequence %02d: %s poses, expected %d" % (sq, p.shape, n))
        mine[o:o + n] = p
        o += n
    if dist is None:
        parts = [mine]
    else:
        import torch
        t = torch.from_numpy(mine).to(dev)
        got = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(got, t)
        parts = [g.cpu().numpy() for g in got]
    out = {}
    for r in range(world):
        o = 0
        for sq in assign[r]:
            n = KITTI_SEQ_FRAMES[sq]
            out[sq] = parts[r][o:o + n].copy()
            o += n
    return out


def shard_bounds(n, world, rank):
    """contiguous shard [a, b) of n items for `rank` (sizes differ by at most one)"""
    base, extra = divmod(n, world)
    a = rank * base + min(rank, extra)
    return a, a + base + (1 if rank < extra else 0)


def broadcast_array(dist, arr, src, device):
    """rank `src`'s float32 array to every rank (one collective; RCCL over xGMI on the GPU box)"""
    import torch
    shape = torch.tensor(list(arr.shape) if arr is not None else [0, 0], dtype=torch.int64, device=device)
    dist.broadcast(shape, src)
    t = (torch.from_numpy(np.ascontiguousarray(arr, np.float32)).to(device) if arr is not None
         else torch.empty(tuple(shape.tolist()), dtype=torch.float32, device=device))
    dist.broadcast(t, src)
    return t.cpu().numpy()


def main_knn_shard(args, rank, local_rank, world, dist, barrier, dev="cuda", stub=False):
    """configs[4] at N GPUs: the 2M-point map is generated on rank 0 and broadcast once; every rank runs
    the exact 5-NN kernel on its contiguous shard of the 200k queries (timed with HIP events on its
    stream, as the roofline leg); value = all queries / the slowest rank's kernel time. stub (the CPU
    test of the rank plumbing): a 20k-point map and 2k queries go through the same broadcasts and
    reductions, and rank r 'takes' 1 + r ms per launch."""
    import pfsynth
    nmap, nq, iters = (20_000, 2_000, 5) if stub else (2_000_000, 200_000, 50)
    mp = q = None
    if rank == 0:
        mp = pfsynth.dense_map(nmap, seed=5)
        q = pfsynth.dense_queries(mp, nq, sigma=0.3, seed=6)
    if dist is not None:
        mp = broadcast_array(dist, mp, 0, dev)
        q = broadcast_array(dist, q, 0, dev)
    a, b = shard_bounds(nq, world, rank)
    if stub:
        assert mp.shape == (nmap, 4) and q.shape == (nq, 4)
        ms, alg = 1.0 + rank, float(b - a) * 1000.0
    else:
        import pfilter_amd as pa
        kn = pa.Knn(nmap, max(1, b - a), device=local_rank)
        kn.set_map(mp)
        kn.query(q[a:b])
        barrier()
        ms, alg = kn.bench(iters)
    worst_ms, tot_alg = ms, alg
    if dist is not None:
        import torch
        t = torch.tensor([ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        g = torch.tensor([alg], dtype=torch.float64, device=dev)
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        worst_ms, tot_alg = float(t.item()), float(g.item())
    if rank == 0:
        out = {"metric": "exact 5-NN queries/s (configs[4]: 2M-point map, 200k queries)",
               "value": round(nq / (worst_ms * 1e-3), 1), "unit": "queries/s", "n_gpus": world, "steps": iters,
               "warmup": 2, "ms_per_step": round(worst_ms, 5), "higher_is_better": True, "scaling": "strong",
               "vs_baseline": None, "dtype": "f32", "data": "synthetic",
               "config": {"workload": "configs[4] kNN: dense map replicated by broadcast, queries sharded",
                          "parallelism": "queries over GPUs"},
               "aggregate_alg_GBps": round(tot_alg / (worst_ms * 1e-3) / 1e9, 1)}
        if stub:
            out["stub"] = True
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def knn_roofline(device=0, nmap=2_000_000, nq=200_000, iters=50, pmc=True):
    """Config 5: exact 5-NN of 200k jittered queries against a 2M-point dense map."""
    import pfilter_amd as pa
    import pfsynth
    mp = pfsynth.dense_map(nmap, seed=5)
    q = pfsynth.dense_queries(mp, nq, sigma=0.3, seed=6)
    kn = pa.Knn(nmap, nq, device=device)
    kn.set_map(mp)
    idx, d2 = kn.query(q)
    ms, alg = kn.bench(iters)
    achieved = alg / (ms * 1e-3) / 1e9
    found = int((idx[:, 4] >= 0).sum())
    out = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
           "kernel": "k_knn_thick (exact radius-gated 5-NN, 1 m cell grid, thick-row layout)",
           "workload": "config 5: map %d pts, %d queries, %d with 5 neighbours" % (nmap, nq, found),
           "alg_bytes_per_launch": alg, "avg_kernel_ms": round(ms, 5)}
    if pmc:
        t = knn_pmc_traffic()
        if t is not None:
            out["traffic"] = t["bytes_per_launch"]
            out["traffic_frac"] = round(t["bytes_per_launch"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            out["traffic_source"] = t["source"]
    return out


def knn_pmc_traffic(timeout_s=90, probe=("knn_probe.py", "--iters", "5"), kernel="k_knn_thick"):
    """HBM (fabric) bytes per launch of k_knn_thick (the standalone query's kernel; or `kernel` of the
    `probe` script), measured now: two rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE: they do not fit
    one pass) over tools/<probe> as child processes.
    MI355X_MICROARCH.md: FETCH_SIZE is doubled on gfx950 (128-B requests tallied at 64 B); WRITE_SIZE
    is exact. None when rocprofv3 is unavailable or a pass fails (never a stale number)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None
    vals = {}
    tmp = tempfile.mkdtemp(prefix="pf_pmc_")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = ["timeout", "-s", "KILL", str(timeout_s), "rocprofv3", "--pmc", ctr, "-d", d, "-o", "run",
                   "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "tools", probe[0])] + list(probe[1:])
            env = dict(os.environ, TMPDIR="/tmp")
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env, cwd="/tmp")
            if r.returncode != 0:
                log("pmc pass %s failed (rc %d): %s" % (ctr, r.returncode, r.stderr[-400:]))
                return None
            xs = []
            for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
                for row in csv.DictReader(open(f)):
                    if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                        xs.append(float(row["Counter_Value"]))
            if not xs:
                return None
            vals[ctr] = float(np.median(xs)) * 1024.0          # kB -> bytes, per launch
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    rd, wr = 2.0 * vals["FETCH_SIZE"], vals["WRITE_SIZE"]
    return {"bytes_per_launch": round(rd + wr), "read": round(rd), "write": round(wr),
            "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, measured in this run "
                      "(tools/%s, median over launches)" % probe[0]}


def pcie_leg(device, hptrs, warmup, use_graph=True):
    """The headline's frames again, fed from pinned host RAM through pf_odom_frame_host (the scan's H2D
    DMA inside the timed region, on the handle's copy stream, overlapping the previous frames' kernels;
    pose_out NULL as the headline's frame_device). SURVEY 8(d)'s frame boundary: scans preloaded in
    pinned host RAM, H2D included."""
    import pfilter_amd as pa
    od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lidar_cfg(), **ODOM_CFG)
    set_order(od)
    od.set_graph(use_graph)
    for ptr, n in hptrs[:warmup]:
        od.frame_host_ptr(ptr, n)
    od.sync()
    t0 = time.perf_counter()
    for ptr, n in hptrs[warmup:]:
        od.frame_host_ptr(ptr, n)
    t_enq = time.perf_counter()
    od.sync()
    el = time.perf_counter() - t0
    assert od.stats()["errors"] == 0
    nf = len(hptrs) - warmup
    return {"value": round(nf / el, 2), "unit": "frames/s", "frames": nf, "ms_per_step": round(el / nf * 1e3, 4),
            "host_us_per_frame": round((t_enq - t0) / nf * 1e6, 1), "poses": od.poses(),
            "note": "pf_odom_frame_host over the headline's frames from pinned host RAM (pf_host_alloc): "
                    "H2D DMA of every scan inside the timed region"}


def pageable_leg(device, nframes, threads, warmup=20, use_graph=True):
    """pf_odom_frame_host from ordinary (pageable) numpy memory: each scan repacked into the handle's
    pinned staging, then the same DMA path (frames warmup .. warmup + nframes of the headline sequence)."""
    import pfilter_amd as pa
    import pfsynth
    seq = pfsynth.Sequence("S64", n_frames=nframes + warmup, seed=0)
    buf, counts = seq.frames(0, nframes + warmup, threads=threads)
    scans = [np.ascontiguousarray(buf[k, :counts[k]]) for k in range(nframes + warmup)]
    del buf
    od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lidar_cfg(), **ODOM_CFG)
    set_order(od)
    od.set_graph(use_graph)
    for k in range(warmup):
        od.frame_host(scans[k], want_pose=False)
    od.sync()
    t0 = time.perf_counter()
    for k in range(warmup, nframes + warmup):
        od.frame_host(scans[k], want_pose=False)
    od.sync()
    el = time.perf_counter() - t0
    return {"value": round(nframes / el, 2), "unit": "frames/s", "frames": nframes,
            "note": "pf_odom_frame_host from pageable numpy memory (repacked into pinned staging per frame)"}


def node_pattern_leg(device, hptrs, warmup, nframes):
    """The drop-in call pattern of the reference's nodes: laserProcessingNode's featureExtraction
    (src/laserProcessingNode.cpp:62-78) returns the edge / surf clouds to the host, and the odometry
    node hands them to updatePointsToMap (src/odomEstimationNode copy.cpp:74-100), which returns the
    pose: pf_fe_extract -> pf_odom_update per frame, both synchronous, clouds in pinned host RAM. The
    reference's two timers are reported as fe_us / odom_us."""
    import ctypes
    import pfilter_amd as pa
    L = pa.lib()
    lid = lidar_cfg()
    fe = ctypes.c_void_p()
    pa._check("pf_fe_create", L.pf_fe_create(ctypes.byref(lid), device, 300000, ctypes.byref(fe)))
    pa._check("pf_fe_set_tie_order", L.pf_fe_set_tie_order(fe, int(ORDER[0] == "tie")))
    od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lid, **ODOM_CFG)
    set_order(od)
    eb, sb = pa.HostBuffer(300000 * 16), pa.HostBuffer(300000 * 16)
    ne, ns = ctypes.c_size_t(), ctypes.c_size_t()
    pose = np.empty(7)
    t_fe = t_od = 0.0
    total = min(len(hptrs), warmup + nframes)
    for k in range(total):
        ptr, n = hptrs[k]
        a = time.perf_counter()
        pa._check("pf_fe_extract", L.pf_fe_extract(fe, ptr, n, 16, eb.ptr, ctypes.byref(ne), sb.ptr,
                                                   ctypes.byref(ns), 300000))
        b = time.perf_counter()
        if k == 0:
            pa._check("pf_odom_init_map", L.pf_odom_init_map(od._h, eb.ptr, ne.value, 16, sb.ptr, ns.value, 16))
        else:
            pa._check("pf_odom_update", L.pf_odom_update(od._h, eb.ptr, ne.value, 16, sb.ptr, ns.value, 16,
                                                         pose.ctypes.data))
        c = time.perf_counter()
        if k >= warmup:
            t_fe += b - a
            t_od += c - b
    L.pf_fe_destroy(fe)
    nf = total - warmup
    return {"value": round(nf / (t_fe + t_od), 2), "unit": "frames/s", "frames": nf,
            "fe_us": round(t_fe / nf * 1e6, 1), "odom_us": round(t_od / nf * 1e6, 1), "poses": od.poses(),
            "note": "pf_fe_extract -> pf_odom_update per frame (the nodes' synchronous calls), clouds in "
                    "pinned host RAM; frames %d..%d of the headline sequence" % (warmup, total - 1)}


def configs4_leg(device, nframes, threads, warmup=3, timing_frames=20, use_graph=True, order=None, pmc=False):
    """BASELINE.json configs[4] as a pipeline: synthetic 128-line scans (~200k points; the reference has
    no 128-line ring formula, so the linear beam-model extension pf_odom_set_ring_model(15, -25) bins
    them) against a 2,000,000-point surf map (pfsynth.voxel_map: voxel centroids
    of the dense block at the 0.8 m surf leaf) seeded by pf_odom_set_map after frame 0; FLOAM
    parameters (theta 0: no stability filter, the map keeps its size), scans HBM-resident, graph replay.
    Then the association's kNN alone on the last frame (pf_odom_probe_assoc: the exact 5-NN of k_assoc
    against the 2M-point grid, HIP events, algorithmic bytes per SURVEY 8(d)) and, for comparison, the
    standalone thick-row kNN (k_knn_thick) on the same surf map and the same surf queries.
    order: "tie" / "stable" for this leg alone (default: the run's --order)"""
    import pfilter_amd as pa
    import pfsynth
    total = 1 + warmup + nframes + timing_frames
    # 1 m/s: the seeded map (+-103 m around the start) stays inside the +-100 m crop box of every pose
    # of the run (12 m of travel), so the surf map keeps ~2M points instead of emptying as at 10 m/s
    seq = pfsynth.Sequence("S128", n_frames=total, speed=1.0)
    bufs, ptrs = [], []
    for f0 in range(0, total, 64):
        nf = min(64, total - f0)
        buf, counts = seq.frames(f0, nf, threads=threads)
        db = pa.DeviceBuffer(buf.nbytes, device=device)
        db.upload(buf)
        ptrs += [(db.ptr + i * buf.shape[1] * 16, int(counts[i])) for i in range(nf)]
        bufs.append(db)
        del buf
    lid = pa.make_lidar(128, 3.0, 90.0, 0.1, ring_model=(15.0, -25.0))
    od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lid, 0.4, 0, 0.0, 0, 0)
    od.set_tie_order((order or ORDER[0]) == "tie")
    od.set_graph(use_graph)
    od.frame_device(*ptrs[0])
    od.sync()
    m = pfsynth.voxel_map(2_000_000, 0.8, seed=5)
    od.set_map(1, m, np.zeros((m.shape[0], 2), np.uint8))
    for k in range(1, 1 + warmup):
        od.frame_device(*ptrs[k])
    od.sync()
    fs0 = od.merge_stats()[0]
    t0 = time.perf_counter()
    for k in range(1 + warmup, 1 + warmup + nframes):
        od.frame_device(*ptrs[k])
    od.sync()
    el = time.perf_counter() - t0
    fs1 = od.merge_stats()[0]
    st = od.stats()
    assert st["errors"] == 0
    od.set_stage_timing(True)
    for k in range(1 + warmup + nframes, total):
        od.frame_device(*ptrs[k])
    stg = od.stage_times()
    od.set_stage_timing(False)
    ms, alg, nq, q = od.probe_assoc(iters=20, queries=True)
    out = {"value": round(nframes / el, 2), "unit": "frames/s", "frames": nframes,
           "ms_per_step": round(el / nframes * 1e3, 4),
           "workload": "configs[4]: S128 synthetic 128-line scans (linear beam model 15..-25 deg, 1 m/s), "
                       "2,000,000-point surf map seeded after frame 0, k_new 0 theta_p 0 theta_max 0, weightType 0, "
                       "map_res 0.4",
           "mean_points_per_frame": round(float(np.mean([n for _, n in ptrs])), 1),
           "stage_us": {"A_features_voxelgrid": round(stg["a_us"], 1), "B_odometry": round(stg["b_us"], 1),
                        "frames": stg["frames"]},
           "last_frame": {k: st[k] for k in ("n_in", "n_ds", "n_map", "n_res")},
           # rgbds updates of the timed frames that fell back to the full sort (the first update after
           # the host map write does, in the warm-up: the seeded map is not in voxel order)
           "full_sort_updates_timed": fs1 - fs0}
    ach = alg / (ms * 1e-3) / 1e9
    out["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                       "kernel": "k_assoc's exact 5-NN (knn5_team on the 1 m grid of the frame's maps), "
                                 "pf_odom_probe_assoc on the last frame",
                       "queries": nq, "alg_bytes_per_launch": alg, "avg_kernel_ms": round(ms, 5)}
    if pmc:
        # the same kernel's fabric bytes per launch, from tools/assoc_probe.py (configs[4]'s state rebuilt in
        # a child process: a few frames against the same seeded map, so the query set is similar, not equal)
        t = knn_pmc_traffic(timeout_s=240, probe=("assoc_probe.py", "--frames", "4", "--iters", "5"),
                            kernel="k_assoc_probe")
        if t is not None:
            out["roofline"]["traffic"] = t["bytes_per_launch"]
            out["roofline"]["traffic_source"] = t["source"]
    surf = q[q[:, 3].view(np.int32) == 1]
    mxyz = od._map(1)[0]
    if surf.shape[0] and mxyz.shape[0]:
        kn = pa.Knn(mxyz.shape[0], surf.shape[0], device=device)
        kn.set_map(np.c_[mxyz, np.zeros(mxyz.shape[0], np.float32)])
        kn.query(np.c_[surf[:, :3], np.zeros(surf.shape[0], np.float32)])
        tms, talg = kn.bench(20)
        # the frame's surf queries only, against the surf map (k_assoc's launch above also holds the
        # edge queries against the edge map, so its query count and bytes are not this one's)
        out["thick_knn_surf_queries"] = {"avg_kernel_ms": round(tms, 5), "alg_bytes_per_launch": talg,
                                         "frac": round(talg / (tms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                         "queries": int(surf.shape[0]), "map_points": int(mxyz.shape[0]),
                                         "assoc_queries_edge_and_surf": int(nq),
                                         "kernel": "k_knn_thick (standalone pf_knn, thick-row layout) on the "
                                                   "last frame's surf queries and the surf map"}
    for db in bufs:
        db.free()
    return out


def bpf_leg(device, nframes, threads, warmup=20, cpu_seconds=10.0, with_cpu=True, use_graph=True, dcvc=False):
    """The BPF chain frames/s on the same S64 sequence with configs[1]'s odometry parameters: raw scan ->
    groundSeg::ground_seg + nongroundExtract::featureExtract (include/preProcess.hpp:398-505, 646-689) ->
    Odom_BPF_EstimationClass (src/odomEstimationClass.cpp:649-1306), i.e. the additionNode ->
    odomEstimationNode path without ROS. All scans are HBM-resident before the timed region; the timed
    loop is pf_bpf_frame_scan_device per frame (front end + VoxelGrid in stage A, odometry in stage B)."""
    import pfilter_amd as pa
    import pfsynth
    total = warmup + nframes
    seq = pfsynth.Sequence("S64", n_frames=total, seed=0)
    stride = 128000 * 16                         # bytes per frame slot (S64: <= 128,000 rays)
    scans = pa.DeviceBuffer(stride * total, device=device)
    counts = []
    for f0 in range(0, total, 256):
        nf = min(256, total - f0)
        buf, cnt = seq.frames(f0, nf, threads=threads)
        for i in range(nf):
            scans.upload(np.ascontiguousarray(buf[i, :cnt[i]], np.float32), (f0 + i) * stride)
            counts.append(int(cnt[i]))
    od = pa.Odom_BPF_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lidar_cfg(), **ODOM_CFG)
    set_order(od)
    od.set_graph(use_graph)
    if dcvc:
        od.set_dcvc(True)                        # curvedfilter on, as launch/pfilter_kitti.launch:8

    def run(k):
        od.frame_scan_device(scans.ptr + k * stride, counts[k])

    for k in range(warmup):
        run(k)
    od.sync()
    t0 = time.perf_counter()
    for k in range(warmup, total):
        run(k)
    od.sync()
    el = time.perf_counter() - t0
    st = od.stats()
    out = {"value": round(nframes / el, 2), "unit": "frames/s", "frames": nframes,
           "ms_per_step": round(el / nframes * 1e3, 4),
           "workload": "raw S64 seed 0 scan -> ground_seg + %sPCA featureExtract (reference defaults) -> "
                       "Odom_BPF_EstimationClass (configs[1] parameters)" % ("DCVC (curvedfilter) + " if dcvc else ""),
           "last_frame": {"n_in": st["n_in"], "n_ds": st["n_ds"], "n_map": st["n_map"], "n_res": st["n_res"]}}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pfref
        lid = pfref.make_lidar(64, 3.0, 90.0)
        cp = pfref.cls_params()
        dp = pfref.dcvc_params() if dcvc else None
        orc = pfref.OdomBPF(lid, 0.4, 0, 0.4, 75, 0, opts=0)
        cw = min(warmup, 11)                     # optimization_count reaches its steady 2 after 10 frames
        n, el, k = 0, 0.0, 0
        pc = pinned_core().__enter__()
        while k < total and (el < cpu_seconds or k < cw):
            x = seq.frame(k)
            t = time.perf_counter()
            r = pfref.bpf_preprocess(x, cp, dcvc=dp, first_frame=(k == 0))
            cl = [np.c_[x[r[c], :3], np.zeros(len(r[c]))].astype(np.float32) for c in ("beam", "pillar", "facade")]
            if k == 0:
                orc.init_map(*cl)
            else:
                orc.update(*cl)
            if k >= cw:
                el += time.perf_counter() - t
                n += 1
            k += 1
        host = pc.host()
        pc.__exit__(None, None, None)
        out["cpu_baseline"] = {"value": round(n / el, 3), "unit": "frames/s", "cores": 1, "kind": "port", "host": host,
                               "sample": "pfref front end (radius k-NN over a hash grid, PCA) + OdomBPF "
                                         "(reference-faithful opts=0), frames %d..%d, single thread (the "
                                         "reference's PCA loop uses up to 6 OpenMP threads, preProcess.hpp:207), "
                                         "%.1f s of CPU time" % (cw, k - 1, el)}
        out["speedup_vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 2)
    return out


class pinned_core:
    """Run the CPU baseline on one core (single thread, pinned like `taskset -c 0`), and
    describe the host: the CPU model and the cores this process may use."""

    def __enter__(self):
        self.saved = None
        try:
            self.saved = os.sched_getaffinity(0)
            self.core = min(self.saved)
            os.sched_setaffinity(0, {self.core})
        except (AttributeError, OSError):
            self.core = None
        return self

    def __exit__(self, *exc):
        if self.saved:
            os.sched_setaffinity(0, self.saved)
        return False

    def host(self):
        model = "unknown"
        try:
            with open("/proc/cpuinfo") as f:
                for line in f:
                    if line.startswith("model name"):
                        model = line.split(":", 1)[1].strip()
                        break
        except OSError:
            pass
        return {"cpu_model": model, "pinned_core": self.core,
                "cores_available": len(self.saved) if self.saved else os.cpu_count()}


def _cpu_baseline(budget_s, warmup, preset="S64", theta=(0.4, 75), max_frames=2000, lines=64, wt=0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pfref
    import pfsynth
    seq = pfsynth.Sequence(preset, n_frames=warmup + max_frames, seed=0)
    orc = pfref.Odom(pfref.make_lidar(lines, 3.0, 90.0), 0.4, 0, theta[0], theta[1], wt, opts=0)
    for k in range(warmup):
        orc.frame(seq.frame(k))
    n, el, k = 0, 0.0, warmup
    while el < budget_s and n < max_frames:
        x = seq.frame(k)
        t = time.perf_counter()
        orc.frame(x)
        el += time.perf_counter() - t
        n += 1
        k += 1
    return {"value": round(n / el, 3), "unit": "frames/s", "cores": 1, "kind": "port", "frames": [warmup, k],
            "sample": "pfref (oracle/, reference-faithful opts=0) frames %d..%d of the same %s seed-0 sequence "
                      "after %d warm-up frames, single thread, %.1f s of CPU time" % (warmup, k - 1, preset, warmup, el)}


def vdc_order(n):
    """0 .. n-1 in van der Corput (bit-reversed) order: every prefix is spread over the whole range"""
    bits = max(1, (n - 1).bit_length())
    out = []
    for i in range(1 << bits):
        r = int(format(i, "0%db" % bits)[::-1], 2)
        if r < n:
            out.append(r)
    return out


def cpu_baseline_synced(device, ptrs, warmup, budget_s, use_graph=True, strata=512, preset="S64", seed=0):
    """pfref (oracle/, reference-faithful opts=0) timed per frame on a stratified sample of the headline's
    own frames [warmup, len(ptrs)): one frame per stratum (its middle), strata visited in van der Corput
    order so that the frames timed before the budget ran out are spread over the whole sequence.

    The oracle is not run through the sequence: before each sampled frame k it is given the device's
    estimator state after frame k - 1 -- both local maps with their age / p-index bytes, odom, last_odom,
    optimization_count, the transfer of the synced parity test (tests/test_gpu_parity_synced.py) -- from
    a capture pass of the device pipeline over the same frames (outside every timed region). Only the
    oracle's frame call (featureExtraction + updatePointsToMap, the reference's timed boundary:
    src/laserProcessingNode.cpp:71-78 + src/odomEstimationNode copy.cpp:92-100) is timed, single thread,
    pinned to one core. Each timed frame's oracle pose is also compared with the device's pose of that
    frame from the same state (`parity`)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pfilter_amd as pa
    import pfref
    import pfsynth
    from_ = warmup
    total = len(ptrs)
    span = total - from_
    strata = max(1, min(strata, span))
    frames = sorted({from_ + (2 * s + 1) * span // (2 * strata) for s in range(strata)})
    want = set(frames)
    # capture pass: the device pipeline in frame order, the state taken before every sampled frame
    od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lidar_cfg(), **ODOM_CFG)
    set_order(od)
    od.set_graph(use_graph)
    states, dev_pose = {}, {}
    poses_so_far = None
    for k in range(total):
        if k in want and k > 0:
            poses_so_far = od.poses()
            p1, p2 = poses_so_far[k - 1], poses_so_far[max(k - 2, 0)]
            opt = od.state()["optimization_count"]
            states[k] = ([od._map(0), od._map(1)], p1, p2, opt)
        od.frame_device(*ptrs[k])
        if k in want:
            od.sync()
    allp = od.poses()
    assert od.stats()["errors"] == 0
    del od
    for k in states:
        dev_pose[k] = allp[k]
    # the CPU pass
    seq = pfsynth.Sequence(preset, n_frames=total, seed=seed)
    orc = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), ODOM_CFG["map_resolution"], ODOM_CFG["k_new"],
                     ODOM_CFG["theta_p"], ODOM_CFG["theta_max"], ODOM_CFG["weightType"], opts=0)
    order = [frames[i] for i in vdc_order(len(frames))]
    n, el = 0, 0.0
    worst_t = worst_r = 0.0
    timed = []
    with pinned_core() as pc:
        for k in order:
            if el >= budget_s:
                break
            if k not in states:
                continue
            maps, p1, p2, opt = states[k]
            for c, (xyz, rg) in enumerate(maps):
                orc.set_map(c, xyz, rg)
            orc.set_state(p1, p2)
            orc.set_opt_count(opt)
            x = seq.frame(k)
            t = time.perf_counter()
            pose = orc.frame(x)
            el += time.perf_counter() - t
            n += 1
            timed.append(k)
            dt, dr = pose_diff(pose, dev_pose[k])
            worst_t, worst_r = max(worst_t, dt), max(worst_r, dr)
        host = pc.host()
    timed.sort()
    return {"value": round(n / el, 3), "unit": "frames/s", "cores": 1, "kind": "port", "host": host,
            "frames_timed": n, "strata": len(frames), "frame_range": [from_, total - 1],
            "first_last_timed": [timed[0], timed[-1]] if timed else None,
            "sample": "pfref (oracle/, reference-faithful opts=0), single thread pinned to one core: %d frames "
                      "of the headline's own frames %d..%d (one per stratum of %d, strata in van der Corput "
                      "order until %.1f s of CPU time), each from the device's estimator state before it "
                      "(maps with age / p-index bytes, odom, last_odom, optimization_count)"
                      % (n, from_, total - 1, len(frames), el),
            "parity": {"frames": n, "worst_t_m": worst_t, "worst_r_rad": worst_r,
                       "note": "oracle pose vs the device's pose of the same frame from the same state"}}


def pose_diff(a, b):
    """(translation m, rotation rad) between two {qx, qy, qz, qw, tx, ty, tz} poses"""
    dt = float(np.linalg.norm(np.asarray(a[4:7]) - np.asarray(b[4:7])))
    q = np.asarray(a[:4]) * (1.0 if float(np.dot(a[:4], b[:4])) >= 0 else -1.0)
    return dt, float(2.0 * np.linalg.norm(q - np.asarray(b[:4])))     # tests/_util.py pose_err


ES_LEGS = {
    # name: (preset, theta_p, theta_max, what it is[, weightType])
    "theta0": ("S64", 0.0, 0, "configs[0] parameters (k_new=0 theta_p=0 theta_max=0, FLOAM-equivalent) on S64"),
    "weight2": ("S64", 0.4, 75, "configs[1] parameters with weightType 2 (launch/pfilter_kitti.launch:7's default; "
                                "SURVEY 8(d) config 2's secondary run) on S64", 2),
    "campus32": ("S32", 1.0, 200, "configs[2]: 32-line campus scans (S32, 2 m/s), k_new=0 theta_p=1 theta_max=200"),
    "dense": ("S64V", 0.4, 75, "configs[1] parameters on S64V: residential scene with vegetation and rough "
                               "ground, denser features and maps than S64 (KITTI-00-like sizes)"),
    "dense_theta0": ("S64V", 0.0, 0, "configs[0] parameters on S64V (the largest maps: no stability filter)"),
}


def es_leg(name, device, nframes, threads, cpu_seconds, warmup=20, use_graph=True, with_cpu=True):
    """One extra ES line: the device pipeline over `nframes` frames of the leg's sequence (scans
    HBM-resident, graph replay, timed like the headline), then the same frames again on a fresh handle
    with per-stage device timing (pf_odom_set_stage_timing: stage A = featureExtraction + VoxelGrid,
    stage B = odometry), and the CPU port on the leg's first frames after the same warm-up."""
    import pfilter_amd as pa
    preset, tp, tm, what = ES_LEGS[name][:4]
    wt = ES_LEGS[name][4] if len(ES_LEGS[name]) > 4 else 0
    cfg = dict(ODOM_CFG, theta_p=tp, theta_max=tm, weightType=wt)
    lines = 32 if preset == "S32" else 64
    total = warmup + nframes
    bufs, ptrs = [], []
    for _, buf, counts, _ in load_frames(0, total, threads, preset):
        db = pa.DeviceBuffer(buf.nbytes, device=device)
        db.upload(buf)
        ptrs += [(db.ptr + i * buf.shape[1] * 16, int(counts[i])) for i in range(buf.shape[0])]
        bufs.append(db)

    def run(timing):
        od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
        od.init(pa.make_lidar(lines, 3.0, 90.0, 0.1), **cfg)
        set_order(od)
        od.set_graph(use_graph)
        for k in range(warmup):
            od.frame_device(*ptrs[k])
        od.sync()
        if timing:
            od.set_stage_timing(True)
        t0 = time.perf_counter()
        for k in range(warmup, total):
            od.frame_device(*ptrs[k])
        od.sync()
        el = time.perf_counter() - t0
        st = od.stats()
        assert st["errors"] == 0
        return el, st, (od.stage_times() if timing else None)

    el, st, _ = run(False)
    _, _, stg = run(True)
    out = {"value": round(nframes / el, 2), "unit": "frames/s", "frames": nframes, "ms_per_step": round(el / nframes * 1e3, 4),
           "workload": what, "sequence": "synthetic %s seed 0" % preset,
           "stage_us": {"A_features_voxelgrid": round(stg["a_us"], 1), "B_odometry": round(stg["b_us"], 1),
                        "frames": stg["frames"]},
           "last_frame": {k: st[k] for k in ("n_in", "n_ds", "n_map", "n_res")}}
    if with_cpu:
        with pinned_core() as pc:
            cb = _cpu_baseline(cpu_seconds, warmup, preset=preset, theta=(tp, tm), max_frames=nframes, lines=lines,
                               wt=wt)
            cb["host"] = pc.host()
        f0, f1 = cb.pop("frames")
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu"] = round(out["value"] / cb["value"], 2)
    return out


def stage_pass(device, ptrs, warmup, nframes, use_graph=True):
    """Per-stage device time of the headline workload: the first `nframes` timed frames again on a
    fresh handle with pf_odom_set_stage_timing (outside the timed region)."""
    import pfilter_amd as pa
    od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lidar_cfg(), **ODOM_CFG)
    set_order(od)
    od.set_graph(use_graph)
    for k in range(warmup):
        od.frame_device(*ptrs[k])
    od.sync()
    od.set_stage_timing(True)
    for k in range(warmup, min(len(ptrs), warmup + nframes)):
        od.frame_device(*ptrs[k])
    st = od.stage_times()
    return {"A_features_voxelgrid": round(st["a_us"], 1), "B_odometry": round(st["b_us"], 1), "frames": st["frames"]}


def node_threads_leg(device, hptrs, warmup, nframes):
    """The nodes as ROS runs them: laserProcessingNode and odomEstimationNode are separate processes
    joined by a topic, so frame k + 1's featureExtraction runs while frame k's updatePointsToMap does.
    Two host threads, each with its own handle, joined by a two-deep queue of edge / surf clouds in
    pinned host RAM (the subscriber queue): pf_fe_extract on one, pf_odom_update on the other, both
    synchronous calls as in the nodes."""
    import ctypes
    import queue
    import threading
    import pfilter_amd as pa
    L = pa.lib()
    lid = lidar_cfg()
    fe = ctypes.c_void_p()
    pa._check("pf_fe_create", L.pf_fe_create(ctypes.byref(lid), device, 300000, ctypes.byref(fe)))
    pa._check("pf_fe_set_tie_order", L.pf_fe_set_tie_order(fe, int(ORDER[0] == "tie")))
    od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lid, **ODOM_CFG)
    set_order(od)
    total = min(len(hptrs), warmup + nframes)
    slots = [(pa.HostBuffer(300000 * 16), pa.HostBuffer(300000 * 16)) for _ in range(3)]
    full, free = queue.Queue(), queue.Queue()
    for i in range(3):
        free.put(i)
    errors, marks = [], {}

    def extract():
        try:
            ne, ns = ctypes.c_size_t(), ctypes.c_size_t()
            for k in range(total):
                i = free.get()
                eb, sb = slots[i]
                ptr, n = hptrs[k]
                pa._check("pf_fe_extract", L.pf_fe_extract(fe, ptr, n, 16, eb.ptr, ctypes.byref(ne), sb.ptr,
                                                           ctypes.byref(ns), 300000))
                full.put((k, i, ne.value, ns.value))
        except Exception as e:
            errors.append(repr(e))
            full.put(None)

    def odometry():
        try:
            pose = np.empty(7)
            for _ in range(total):
                item = full.get()
                if item is None:
                    return
                k, i, ne, ns = item
                eb, sb = slots[i]
                if k == 0:
                    pa._check("pf_odom_init_map", L.pf_odom_init_map(od._h, eb.ptr, ne, 16, sb.ptr, ns, 16))
                else:
                    pa._check("pf_odom_update", L.pf_odom_update(od._h, eb.ptr, ne, 16, sb.ptr, ns, 16,
                                                                 pose.ctypes.data))
                free.put(i)
                if k == warmup - 1 or (warmup == 0 and k == 0):
                    marks["t0"] = time.perf_counter()
                if k == total - 1:
                    marks["t1"] = time.perf_counter()
        except Exception as e:
            errors.append(repr(e))

    ths = [threading.Thread(target=extract), threading.Thread(target=odometry)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    L.pf_fe_destroy(fe)
    if errors:
        raise RuntimeError("node threads: %s" % errors)
    nf = total - max(warmup, 1)
    el = marks["t1"] - marks["t0"]
    return {"value": round(nf / el, 2), "unit": "frames/s", "frames": nf, "poses": od.poses(),
            "note": "two host threads as the two ROS nodes: pf_fe_extract -> 2-deep queue of pinned clouds -> "
                    "pf_odom_update, every call synchronous; frames %d..%d" % (warmup, total - 1)}


def order_leg(device, ptrs, warmup, nframes, order, use_graph=True):
    """The headline workload's first `nframes` timed frames in the given sort order on a fresh handle,
    timed like the headline (HBM-resident scans, one sync at the end), then once more with per-stage
    device timing."""
    import pfilter_amd as pa
    total = min(len(ptrs), warmup + nframes)

    def run(timing):
        od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
        od.init(lidar_cfg(), **ODOM_CFG)
        od.set_tie_order(order == "tie")
        od.set_graph(use_graph)
        for k in range(warmup):
            od.frame_device(*ptrs[k])
        od.sync()
        if timing:
            od.set_stage_timing(True)
        t0 = time.perf_counter()
        for k in range(warmup, total):
            od.frame_device(*ptrs[k])
        od.sync()
        el = time.perf_counter() - t0
        assert od.stats()["errors"] == 0
        return el, (od.stage_times() if timing else None)

    el, _ = run(False)
    _, st = run(True)
    nf = total - warmup
    return {"order": order, "value": round(nf / el, 2), "unit": "frames/s", "frames": nf,
            "stage_us": {"A_features_voxelgrid": round(st["a_us"], 1), "B_odometry": round(st["b_us"], 1),
                         "frames": st["frames"]}}


def gpu_window(device, f0, f1, threads, use_graph=True):
    """The GPU pipeline timed over exactly frames [f0, f1) of S64 seed 0 (frames 0..f0-1 run untimed
    first, as the CPU baseline's warm-up): the CPU baseline's own window, for a like-for-like ratio."""
    import pfilter_amd as pa
    od = pa.Odom_ES_EstimationClass(device=device, max_points=300000, map_capacity=1 << 22)
    od.init(lidar_cfg(), **ODOM_CFG)
    set_order(od)
    od.set_graph(use_graph)
    bufs, ptrs = [], []
    for _, buf, counts, _ in load_frames(0, f1, threads):
        db = pa.DeviceBuffer(buf.nbytes, device=device)
        db.upload(buf)
        ptrs += [(db.ptr + i * buf.shape[1] * 16, int(counts[i])) for i in range(buf.shape[0])]
        bufs.append(db)
    for k in range(f0):
        od.frame_device(*ptrs[k])
    od.sync()
    t0 = time.perf_counter()
    for k in range(f0, f1):
        od.frame_device(*ptrs[k])
    od.sync()
    el = time.perf_counter() - t0
    return {"value": round((f1 - f0) / el, 2), "frames": [f0, f1]}


def full_sequence_leg(local_rank, threads, use_graph, nframes, cpu_seconds, with_cpu, head=None, head_cpu=None,
                      node=True):
    """The north star's number over the whole sequence, whatever the headline's --steps: the headline
    workload (configs[1], S64 seed 0) over `nframes` timed frames after 20 warm-up frames (the KITTI-00
    length by default), timed like the headline; the per-stage device times over the same frames; the
    stratified synced CPU baseline over them (512 strata, cpu_baseline_synced); the ratio; and the
    nodes' synchronous call pattern (node_pattern, node_threads) over all of them. head: the headline's
    own run when it already covers these frames (then it is reused, not re-run)."""
    warm = 20
    if head is not None and head["frames"] == nframes:
        r = head
        reused = True
    else:
        r = run_gpu(0, local_rank, 1, nframes, warm, threads, use_graph, lambda: None, keep_host=node)
        reused = False
    value = r["frames"] / r["elapsed"]
    out = {"value": round(value, 2), "unit": "frames/s", "frames": r["frames"], "warmup": warm,
           "frame_range": [warm, warm + r["frames"] - 1], "ms_per_step": round(r["elapsed"] / r["frames"] * 1e3, 4),
           "sequence": r["data"], "same_run_as_value": reused,
           "host_enqueue_us_per_frame": round(r.get("enqueue", 0.0) / max(1, r["frames"]) * 1e6, 1)}
    out["stage_us"] = stage_pass(local_rank, r["ptrs"], warm, r["frames"], use_graph)
    log("full_sequence: %s" % out)
    if node and r.get("hptrs"):
        try:
            nd = node_pattern_leg(local_rank, r["hptrs"], warm, r["frames"])
            npo = nd.pop("poses")
            nd["poses_equal_pipeline"] = bool(np.array_equal(npo, r["poses"][:npo.shape[0]]))
            nd["ratio_to_pipeline"] = round(nd["value"] / value, 4)
            out["node_pattern"] = nd
            nt = node_threads_leg(local_rank, r["hptrs"], warm, r["frames"])
            ntp = nt.pop("poses")
            nt["poses_equal_pipeline"] = bool(np.array_equal(ntp, r["poses"][:ntp.shape[0]]))
            nt["ratio_to_pipeline"] = round(nt["value"] / value, 4)
            out["node_threads"] = nt
            log("full_sequence node legs: %s / %s" % (nd["value"], nt["value"]))
        except Exception as e:  # report, never hide
            log("full-sequence node legs failed: %r" % (e,))
    if with_cpu:
        cb = head_cpu if (reused and head_cpu is not None) else \
            cpu_baseline_synced(local_rank, r["ptrs"], warm, cpu_seconds, use_graph)
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu"] = round(value / cb["value"], 2)
    return out


def stub_run(rank, steps):
    """Stand-in for run_gpu in the CPU test of the rank plumbing: rank r 'takes' 1 + r seconds."""
    poses = np.tile(np.array([0, 0, 0, 1, rank, 0, 0], np.float64), (steps, 1))
    return dict(elapsed=1.0 + rank, frames=steps, poses=poses, stats={}, data="stub", mean_points=0.0)


def reduce_results(dist, elapsed, frames, poses, device):
    """Across ranks: the max elapsed time, the total frame count and every rank's pose array. The
    pose all-gather is the design's only collective (RCCL over xGMI on the GPU box; any
    torch.distributed backend here)."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    f = torch.tensor([frames], dtype=torch.int64, device=device)
    dist.all_reduce(f, op=dist.ReduceOp.SUM)
    p = torch.from_numpy(np.ascontiguousarray(poses, dtype=np.float64)).to(device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, torch.tensor([p.shape[0]], dtype=torch.int64, device=device))
    cap = int(max(int(x.item()) for x in sizes))
    padded = torch.zeros((cap, 7), dtype=torch.float64, device=device)
    padded[:p.shape[0]] = p
    gathered = [torch.empty_like(padded) for _ in range(dist.get_world_size())]
    dist.all_gather(gathered, padded)
    poses_all = [g[:int(n.item())].cpu().numpy() for g, n in zip(gathered, sizes)]
    return float(t.item()), int(f.item()), poses_all


KITTI11_HW_QUEUES = 16


def kitti11_hw_queues(args, env):
    """configs[3] with several concurrent sequences per GPU: the HIP runtime's hardware queues per process
    raised to KITTI11_HW_QUEUES (before the runtime starts; never lowered). At the image's default of 4, the
    2-3 streams of every handle share the queues: in the tie order K = 4 ran 1286-1764 frames/s and K = 6
    stalled (cross-stream waits queued behind each other's kernels); at 16 queues K = 4 ran 2198 and K = 6
    2183-2208 (profiles/r06/k11conc/). Returns the value set, or None."""
    if args.sequences != "kitti11" or args.concurrent <= 1:
        return None
    try:
        cur = int(env.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        cur = 4
    if cur < KITTI11_HW_QUEUES:
        env["GPU_MAX_HW_QUEUES"] = str(KITTI11_HW_QUEUES)
    return int(env["GPU_MAX_HW_QUEUES"])


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    ORDER[0] = args.order
    hw_queues = kitti11_hw_queues(args, os.environ)   # before anything starts the HIP runtime
    world, launch = resolve_world(args, os.environ)
    if launch:                     # nothing has touched the GPU yet
        sys.exit(launch_ranks(world, argv))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # PF_BENCH_BACKEND=gloo / PF_BENCH_STUB=1: the CPU test of the rank plumbing (tests/test_bench_dist.py)
    backend = os.environ.get("PF_BENCH_BACKEND", "nccl")
    stub = os.environ.get("PF_BENCH_STUB") == "1"
    dev = "cuda" if backend == "nccl" else "cpu"
    dist = None
    if world > 1:
        import torch  # noqa: F401  (loaded before the HIP library: one HIP runtime per process)
        import torch.distributed as tdist
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend, init_method="env://")
        dist = tdist

    def barrier():
        if dist is not None:
            dist.barrier()

    threads = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    if args.knn_shard:
        return main_knn_shard(args, rank, local_rank, world, dist, barrier, dev, stub)
    if args.sequences == "kitti11":
        return main_kitti11(args, rank, local_rank, world, dist, barrier, threads, dev, stub, hw_queues)
    host_legs = world == 1 and not stub and (not args.no_pcie or args.node_frames > 0)
    if stub:
        r = stub_run(rank, args.steps)
    else:
        r = run_gpu(rank, local_rank, world, args.steps, args.warmup, threads, graph_mode(args), barrier,
                    keep_host=host_legs)
    elapsed, frames = r["elapsed"], r["frames"]
    if dist is not None:
        elapsed, total_frames, _ = reduce_results(dist, elapsed, frames, r["poses"][-frames:], dev)
    else:
        total_frames = frames
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    value = total_frames / elapsed
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / max(1, frames) * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32/f64",
        "data": "synthetic" if not os.environ.get("PF_KITTI_ROOT") else "kitti",
        "config": {"workload": "KITTI-00 64-line (configs[1]): S64 synthetic scans, k_new=0 theta_p=0.4 "
                               "theta_max=75, weightType 0, map_res 0.4, min/max dis 3/90",
                   "sequence": r["data"], "frames_per_rank": frames,
                   "mean_points_per_frame": round(r["mean_points"], 1),
                   "parallelism": "one independent sequence per GPU" if world > 1 else "single sequence",
                   "graph": GRAPH_NAMES[graph_mode(args)],
                   "sort_order": args.order + (" (libstdc++ std::sort's order of equal keys in featureExtraction's "
                                               "sectors, VoxelGrid and rgbds: the reference's results frame by "
                                               "frame)" if args.order == "tie" else
                                               " (stable sorts: centroids differ from the reference's in the "
                                               "last bits)")},
    }
    log("pipeline: %d frames in %.3f s (host enqueue %.3f s), last-frame stats %s"
        % (frames, elapsed, r.get("enqueue", 0.0), r["stats"]))
    if "enqueue" in r:
        out["config"]["host_enqueue_us_per_frame"] = round(r["enqueue"] / max(1, frames) * 1e6, 1)
    if world == 1 and not stub:
        # over the same frames as `value` (every timed frame)
        out["stage_us"] = stage_pass(local_rank, r["ptrs"], args.warmup, frames, graph_mode(args))
    if world == 1 and not stub and args.other_order_frames > 0:
        other = "stable" if args.order == "tie" else "tie"
        try:
            log("other-order leg (%s) ..." % other)
            oo = order_leg(local_rank, r["ptrs"], args.warmup, args.other_order_frames, other, graph_mode(args))
            oo["ratio_to_value"] = round(oo["value"] / value, 4)
            out["other_order"] = oo
            log("other_order: %s" % oo)
        except Exception as e:  # report, never hide
            log("other-order leg failed: %r" % (e,))
            out["other_order"] = None
    if stub:
        out["stub"] = True
    elif world == 1 and not args.no_roofline:
        try:
            log("roofline leg ...")
            out["roofline"] = knn_roofline(local_rank, pmc=not args.no_pmc)
        except Exception as e:  # report, never hide
            log("roofline leg failed: %r" % (e,))
            out["roofline"] = None
    if world == 1 and args.bpf_frames > 0 and not stub:
        for name, dc in (("bpf", False), ("bpf_dcvc", True)):
            try:
                log("%s leg ..." % name)
                out[name] = bpf_leg(local_rank, args.bpf_frames, threads, with_cpu=not args.no_cpu,
                                    use_graph=graph_mode(args), dcvc=dc)
            except Exception as e:  # report, never hide
                log("%s leg failed: %r" % (name, e))
                out[name] = None
    if world == 1 and args.leg_frames > 0 and not stub:
        for name in ES_LEGS:
            try:
                log("%s leg ..." % name)
                out[name] = es_leg(name, local_rank, args.leg_frames, threads, args.leg_cpu_seconds,
                                   use_graph=graph_mode(args), with_cpu=not args.no_cpu)
            except Exception as e:  # report, never hide
                log("%s leg failed: %r" % (name, e))
                out[name] = None
    if host_legs and not args.no_pcie:
        pc = pcie_leg(local_rank, r["hptrs"], args.warmup, graph_mode(args))
        pp = pc.pop("poses")
        pc["ratio_to_value"] = round(pc["value"] / value, 4)
        pc["poses_equal_headline"] = bool(np.array_equal(pp, r["poses"]))
        out["pcie_inclusive"] = pc
        log("pcie_inclusive: %s" % pc)
    if host_legs and args.node_frames > 0:
        # the device pipeline (value's path) over exactly the node legs' frames, for like-for-like ratios
        gw = gpu_window(local_rank, args.warmup, min(frames + args.warmup, args.warmup + args.node_frames), threads,
                        graph_mode(args))
        nd = node_pattern_leg(local_rank, r["hptrs"], args.warmup, args.node_frames)
        nd["pipeline_same_frames"] = gw
        nd["ratio_to_pipeline_same_frames"] = round(nd["value"] / gw["value"], 4)
        npo = nd.pop("poses")
        nd["poses_equal_headline"] = bool(np.array_equal(npo, r["poses"][:npo.shape[0]]))
        out["node_pattern"] = nd
        log("node_pattern: %s" % nd)
        try:
            nt = node_threads_leg(local_rank, r["hptrs"], args.warmup, args.node_frames)
            ntp = nt.pop("poses")
            nt["poses_equal_headline"] = bool(np.array_equal(ntp, r["poses"][:ntp.shape[0]]))
            nt["ratio_to_pipeline_same_frames"] = round(nt["value"] / gw["value"], 4)
            out["node_threads"] = nt
            log("node_threads: %s" % nt)
        except Exception as e:  # report, never hide
            log("node-threads leg failed: %r" % (e,))
            out["node_threads"] = None
    if world == 1 and not stub and args.configs4_frames > 0:
        try:
            log("configs4 leg (%s order) ..." % args.configs4_order)
            # PF_GRAPH_AUTO replays stage B's graph only while a process holds several handles; here the
            # headline's handle is still alive (the CPU baseline syncs from it later), which a configs[4]
            # user's single handle would not have: run the leg as AUTO runs one handle (stage A's graph,
            # stage B eager, its radix route on the side stream)
            g4 = graph_mode(args)
            g4 = 1 if g4 == 4 else g4
            out["configs4"] = configs4_leg(local_rank, args.configs4_frames, threads, use_graph=g4,
                                           order=args.configs4_order, pmc=not args.no_pmc)
            out["configs4"]["order"] = args.configs4_order
            out["configs4"]["graph_mode"] = g4
            log("configs4: %s" % out["configs4"])
        except Exception as e:  # report, never hide
            log("configs4 leg failed: %r" % (e,))
            out["configs4"] = None
    if world == 1 and not stub and args.pageable_frames > 0:
        log("pageable leg ...")
        out["pcie_pageable"] = pageable_leg(local_rank, args.pageable_frames, threads, use_graph=graph_mode(args))
    if world == 1 and not args.no_cpu and not stub:
        log("cpu baseline (stratified over the headline's frames, device state synced) ...")
        cb = cpu_baseline_synced(local_rank, r["ptrs"], args.warmup, args.cpu_seconds, graph_mode(args))
        out["cpu_baseline"] = cb
        # like for like: both rates are over the same population of frames (every timed frame for the GPU,
        # a stratified sample of those frames for the CPU)
        out["speedup_vs_cpu"] = round(value / cb["value"], 2)
        log("cpu_baseline: %s" % cb)
    if world == 1 and not stub and args.full_frames > 0:
        log("full sequence (%d frames) ..." % args.full_frames)
        same = args.warmup == 20 and frames == args.full_frames
        head = dict(r) if same else None
        del r                                    # the headline's scans leave HBM / pinned RAM first
        try:
            out["full_sequence"] = full_sequence_leg(local_rank, threads, graph_mode(args), args.full_frames,
                                                     args.full_cpu_seconds, not args.no_cpu, head=head,
                                                     head_cpu=out.get("cpu_baseline"))
            log("full_sequence: %s" % out["full_sequence"])
        except Exception as e:  # report, never hide
            log("full-sequence leg failed: %r" % (e,))
            out["full_sequence"] = None
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main_kitti11(args, rank, local_rank, world, dist, barrier, threads, dev="cuda", stub=False, hw_queues=None):
    if stub:                       # CPU test of the rank plumbing: rank r 'takes' 1 + r seconds
        mine = lpt_assign(KITTI_SEQ_FRAMES, world)[rank]
        r = dict(elapsed=1.0 + rank, frames=sum(KITTI_SEQ_FRAMES[sq] for sq in mine),
                 sequences=["%02d" % sq for sq in mine],
                 poses={sq: stub_poses(sq, KITTI_SEQ_FRAMES[sq]) for sq in mine})
    else:
        r = run_kitti11(rank, local_rank, world, args.warmup, threads, graph_mode(args), barrier, args.concurrent)
    elapsed, frames = r["elapsed"], r["frames"]
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        f = torch.tensor([frames], dtype=torch.int64, device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.SUM)
        elapsed, total = float(t.item()), int(f.item())
    else:
        total = frames
    # the trajectories of all eleven sequences to every rank (runkitti.py:111-157 evaluates them together)
    allp = gather_poses(r["poses"], world, rank, dist, dev)
    pose_info = {"sequences": sorted(allp), "frames": [int(allp[sq].shape[0]) for sq in sorted(allp)],
                 "dir": None}
    if rank == 0:
        if args.poses_out:
            import kitti
            os.makedirs(args.poses_out, exist_ok=True)
            for sq in sorted(allp):
                kitti.write_poses(os.path.join(args.poses_out, "%02d.txt" % sq), allp[sq])
            pose_info["dir"] = args.poses_out
        if stub:
            pose_info["stub_match"] = all(np.array_equal(allp[sq], stub_poses(sq, KITTI_SEQ_FRAMES[sq]))
                                          for sq in allp)
        out = {"metric": METRIC, "value": round(total / elapsed, 2), "unit": "frames/s", "n_gpus": world,
               "steps": total, "warmup": args.warmup, "ms_per_step": round(elapsed / max(1, total) * 1e3, 4),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32/f64",
               "data": "synthetic" if not os.environ.get("PF_KITTI_ROOT") else "kitti",
               "config": {"workload": "configs[3]: KITTI 00-10 (real frame counts, S64 synthetic scans seeded "
                                      "by sequence) as independent streams, LPT-assigned to the GPUs",
                          "assignment": lpt_assign(KITTI_SEQ_FRAMES, world), "rank0_sequences": r["sequences"],
                          "parallelism": "sequences over GPUs", "concurrent_per_gpu": args.concurrent,
                          "hw_queues_per_process": hw_queues,
                          "graph": GRAPH_NAMES[graph_mode(args)]},
               "poses": pose_info}
        if stub:
            out["stub"] = True
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
