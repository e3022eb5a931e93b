"""Worker of the synced per-frame parity test (tests/test_gpu_parity_synced.py). TEST INFRASTRUCTURE:
runs ONE frame of the reference-faithful oracle (pfref, opts=0: libstdc++ std::sort tie orders,
Householder-QR LM, FLANN-style kd-tree) from a given estimator state. Imported by spawned worker
processes, which load pfref and pfsynth only, never the HIP library."""
import numpy as np

COUNTS = ("n_edge_in", "n_surf_in", "n_edge_ds", "n_surf_ds", "n_edge_map", "n_surf_map", "n_edge_res",
          "n_surf_res", "n_edge_valid", "n_surf_valid", "outer_iterations", "map_too_small")

_ctx = {}


def init(preset, n_frames, seed, lidar, ring_model, params, opts):
    import pfsynth
    _ctx["seq"] = pfsynth.Sequence(preset, n_frames=n_frames, seed=seed)
    _ctx["args"] = (lidar, ring_model, params, opts)


def init_multi(preset, n_by_seed, lidar, ring_model, params, opts):
    """several sequences in one pool (configs[3]: KITTI 00-10 as seeds 0..10): built on first use"""
    _ctx["multi"] = (preset, dict(n_by_seed))
    _ctx["seqs"] = {}
    _ctx["args"] = (lidar, ring_model, params, opts)


def run_multi(task):
    """task = (seed, k, maps, odom pose, last_odom pose, optimization_count) -> (seed, k, pose, counts, maps)"""
    import pfsynth
    seed, k = task[0], task[1]
    if seed not in _ctx["seqs"]:
        preset, nbs = _ctx["multi"]
        _ctx["seqs"][seed] = pfsynth.Sequence(preset, n_frames=nbs[seed], seed=seed)
    _ctx["seq"] = _ctx["seqs"][seed]
    return (seed,) + run(task[1:])


def run(task):
    """task = (k, [(xyz, rg) per map class] before frame k, odom pose, last_odom pose, optimization_count)
    -> (k, pose after frame k, counts, [(xyz, rg) per map class] after frame k)"""
    import pfref
    k, maps, odom_pose, last_pose, opt = task
    lid, ring_model, prm, opts = _ctx["args"]
    orc = pfref.Odom(pfref.make_lidar(*lid, ring_model=ring_model), *prm, opts=opts)
    for c, (xyz, rg) in enumerate(maps):
        orc.set_map(c, xyz, rg)
    orc.set_state(odom_pose, last_pose)
    orc.set_opt_count(opt)
    pose = orc.frame(_ctx["seq"].frame(k))
    st = orc.stats()
    return k, pose, {c: int(st[c]) for c in COUNTS}, [orc.get_map(c) for c in range(len(maps))]


def compare(k, dev, ref, report, tol_t, tol_r, pose_err, tol_xyz=None):
    """dev / ref = (pose, counts, maps after frame k); accumulates into report (a dict)"""
    tol_xyz = tol_t if tol_xyz is None else tol_xyz
    dt, dr = pose_err(dev[0], ref[0])
    report["worst_t"] = max(report["worst_t"], dt)
    report["worst_r"] = max(report["worst_r"], dr)
    report["frames"] += 1
    if not (dt < tol_t and dr < tol_r):
        report["pose_bad"].append((k, dt, dr))
    bad = {c: (dev[1][c], ref[1][c]) for c in COUNTS if dev[1][c] != ref[1][c]}
    if bad:
        report["count_bad"].append((k, bad))
    for c, ((gx, grg), (rx, rrg)) in enumerate(zip(dev[2], ref[2])):
        if gx.shape != rx.shape:
            report["map_bad"].append((k, c, "size", gx.shape[0], rx.shape[0]))
            continue
        if not np.array_equal(grg, rrg):
            report["map_bad"].append((k, c, "rg", int(np.sum(np.any(grg != rrg, axis=1)))))
        if gx.size:
            d = float(np.max(np.abs(gx.astype(np.float64) - rx)))
            report["worst_xyz"] = max(report["worst_xyz"], d)
            report["xyz_bitexact_frames"] += int(np.array_equal(gx.view(np.uint32), rx.view(np.uint32)))
            if d >= tol_xyz:
                report["map_bad"].append((k, c, "xyz", d))


# ---- Odom_BPF_EstimationClass (src/odomEstimationClass.cpp:649-1306) ----
BPF_COUNTS = ("n_ds", "n_map", "n_res", "n_valid", "outer_iterations", "map_too_small")


def bpf_clouds(k):
    """frame k's beam / pillar / facade clouds by the oracle front end (ground_seg + featureExtract,
    include/preProcess.hpp), xyz + 0 as the node publishes them; the device's front end is bit-exact
    with it (tests/test_gpu_cls.py)"""
    import pfref
    x = _ctx["seq"].frame(k)
    r = pfref.bpf_preprocess(x, pfref.cls_params())
    return [np.c_[x[r[c], :3], np.zeros(len(r[c]))].astype(np.float32) for c in ("beam", "pillar", "facade")]


def bpf_counts(st):
    return {c: (list(st[c]) if isinstance(st[c], (list, tuple)) else int(st[c])) for c in BPF_COUNTS}


def run_bpf(task):
    """task = (k, [(xyz, rg) x 3] before frame k, odom, last_odom, optimization_count) -> (k, pose, counts,
    maps after frame k) of the faithful OdomBPF on frame k's classified clouds"""
    import pfref
    k, maps, odom_pose, last_pose, opt = task
    lid, ring_model, prm, opts = _ctx["args"]
    orc = pfref.OdomBPF(pfref.make_lidar(*lid, ring_model=ring_model), *prm, opts=opts)
    for c, (xyz, rg) in enumerate(maps):
        orc.set_map(c, xyz, rg)
    orc.set_state(odom_pose, last_pose)
    orc.set_opt_count(opt)
    orc.inited = True
    pose = orc.update(*bpf_clouds(k))
    return k, pose, bpf_counts(orc.stats()), [orc.get_map(c) for c in range(3)]


def compare_bpf(k, dev, ref, report, tol_t, tol_r, pose_err):
    """as compare(), over the three map classes"""
    dt, dr = pose_err(dev[0], ref[0])
    report["worst_t"] = max(report["worst_t"], dt)
    report["worst_r"] = max(report["worst_r"], dr)
    report["frames"] += 1
    if not (dt < tol_t and dr < tol_r):
        report["pose_bad"].append((k, dt, dr))
    bad = {c: (dev[1][c], ref[1][c]) for c in BPF_COUNTS if dev[1][c] != ref[1][c]}
    if bad:
        report["count_bad"].append((k, bad))
    for c, ((gx, grg), (rx, rrg)) in enumerate(zip(dev[2], ref[2])):
        if gx.shape != rx.shape:
            report["map_bad"].append((k, c, "size", gx.shape[0], rx.shape[0]))
            continue
        if not np.array_equal(grg, rrg):
            report["map_bad"].append((k, c, "rg", int(np.sum(np.any(grg != rrg, axis=1)))))
        if gx.size:
            d = float(np.max(np.abs(gx.astype(np.float64) - rx)))
            report["worst_xyz"] = max(report["worst_xyz"], d)
            report["xyz_bitexact_frames"] += int(np.array_equal(gx.view(np.uint32), rx.view(np.uint32)))
            if d >= tol_t:
                report["map_bad"].append((k, c, "xyz", d))
