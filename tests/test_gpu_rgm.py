"""GPU: rgbds by merge (the default order; pf_odom.hip k_rgm_keys / k_rgm_merge / k_rg_tail64). The map
that an update writes is in voxel order, so the next update sorts only its appended points (runs of
4096 in LDS) and merges them into the map by binary searches; the map is re-sorted whole only when it
is not in voxel order (after initMapWithPoints or pf_odom_set_map, or a centroid that rounded into a
neighbouring voxel) or more than 65536 points are appended. The stable order it produces -- voxel
index, then element index (map points before appended points) -- is the stable radix sort's, so the
frames must be bit-identical to the full radix sort of every element (the development switch
pf_dev_set_rg_radix, the path before the merge): poses, map coordinates and the map's r / g bytes,
under graph replay. The oracle comparisons of the default order (tests/test_gpu_odom.py,
tests/test_gpu_parity_synced.py) run on this path too."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _es_run(pa, pfsynth, preset, frames, radix, theta=(0.4, 75), lines=64, shuffle_at=None):
    seq = pfsynth.Sequence(preset, n_frames=frames, seed=0)
    od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 21, tie_order=False)
    od.init(pa.make_lidar(lines, 3.0, 90.0), 0.4, 0, theta[0], theta[1], 0)
    od.set_rg_radix(radix)
    buf, cnt = seq.frames(0, frames, threads=16)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    try:
        for i in range(frames):
            if shuffle_at is not None and i == shuffle_at:     # a map out of voxel order (set_map)
                od.sync()
                for which in (0, 1):
                    xyz, rg = od._map(which)
                    perm = np.random.default_rng(which).permutation(xyz.shape[0])
                    od.set_map(which, xyz[perm], rg[perm])
            od.frame_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
        od.sync()
        return od.poses(), [od._map(w) for w in (0, 1)], od.merge_stats()
    finally:
        db.free()


def _same(a, b):
    pa_, ma, _ = a
    pb_, mb, _ = b
    assert pa_.shape == pb_.shape
    bad = np.nonzero(np.any(pa_ != pb_, axis=1))[0]
    assert bad.size == 0, "poses differ from frame %d" % bad[0]
    for w in (0, 1):
        assert ma[w][0].shape == mb[w][0].shape, (w, ma[w][0].shape, mb[w][0].shape)
        assert np.array_equal(ma[w][0].view(np.uint32), mb[w][0].view(np.uint32)), w
        assert np.array_equal(ma[w][1], mb[w][1]), w


@pytest.mark.parametrize("preset,frames,theta,lines", [
    ("S64", 800, (0.4, 75), 64),        # configs[1]
    ("S64", 300, (0.0, 0), 64),         # configs[0]
    ("S32", 300, (1.0, 200), 32),       # configs[2]
    ("S64V", 300, (0.4, 75), 64),       # the dense scene: more appended points per frame
    ("S64T", 300, (0.4, 75), 64),       # the town
])
def test_merge_equals_full_radix_sort(pa, pfsynth, preset, frames, theta, lines):
    m = _es_run(pa, pfsynth, preset, frames, False, theta, lines)
    r = _es_run(pa, pfsynth, preset, frames, True, theta, lines)
    _same(m, r)
    full, most = m[2]
    print("%s: full sorts %d, most appended %d" % (preset, full, most))
    assert full >= 1                      # the first update: the map is the raw first scan's features
    assert full <= 1 + frames // 50       # otherwise the map stays in voxel order
    assert 0 < most <= 65536


def test_merge_after_set_map_out_of_order(pa, pfsynth):
    """pf_odom_set_map with the maps shuffled mid-sequence: the next update detects the order and
    sorts every element; the frames stay identical to the radix path's."""
    m = _es_run(pa, pfsynth, "S64", 200, False, shuffle_at=120)
    r = _es_run(pa, pfsynth, "S64", 200, True, shuffle_at=120)
    _same(m, r)
    assert m[2][0] >= 2


def test_merge_bpf_three_classes(pa, pfsynth):
    """The BPF estimator (beam / pillar / facade maps) through the raw-scan chain."""
    seq = pfsynth.Sequence("S64", n_frames=150, seed=0)
    buf, cnt = seq.frames(0, 150, threads=16)
    out = []
    for radix in (False, True):
        od = pa.Odom_BPF_EstimationClass(device=0, tie_order=False)
        od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
        od.set_rg_radix(radix)
        db = pa.DeviceBuffer(buf.nbytes)
        db.upload(buf)
        for i in range(150):
            od.frame_scan_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
        od.sync()
        out.append((od.poses(), [od._map(w) for w in (0, 1, 2)]))
        db.free()
    assert np.array_equal(out[0][0], out[1][0])
    for w in range(3):
        assert np.array_equal(out[0][1][w][0].view(np.uint32), out[1][1][w][0].view(np.uint32)), w
        assert np.array_equal(out[0][1][w][1], out[1][1][w][1]), w


# ---- the tie order's dependence table (pf_odom.hip DepTab) --------------------------------------------
# While the map holds one centroid per voxel (no host write since the last rgbds, no centroid rounded
# across a voxel face), a group of three or more holds two appended points, so only the appended points
# go into a small table and the map points probe it; the full table takes every element. The flags are
# the heap tier's pop bound, so any difference shows in the map bytes: both runs must be bit-identical.
def _tie_run(pa, pfsynth, preset, frames, full, theta=(0.4, 75), lines=64, set_map_at=None, big_map=False):
    seq = pfsynth.Sequence(preset, n_frames=frames, seed=0)
    od = pa.Odom_ES_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22, tie_order=True)
    if lines == 128:
        od.init(pa.make_lidar(128, 3.0, 90.0, 0.1, ring_model=(15.0, -25.0)), 0.4, 0, theta[0], theta[1], 0)
    else:
        od.init(pa.make_lidar(lines, 3.0, 90.0), 0.4, 0, theta[0], theta[1], 0)
    od.set_dep_full(full)
    buf, cnt = seq.frames(0, frames, threads=16)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    try:
        for i in range(frames):
            if set_map_at is not None and i == set_map_at:
                od.sync()
                if big_map:                          # configs[4]: the 2M-point surf map
                    m = pfsynth.voxel_map(2_000_000, 0.8, seed=5)
                    od.set_map(1, m, np.zeros((m.shape[0], 2), np.uint8))
                else:                                # a host write: shuffled, several frames later
                    for which in (0, 1):
                        xyz, rg = od._map(which)
                        perm = np.random.default_rng(which).permutation(xyz.shape[0])
                        od.set_map(which, xyz[perm], rg[perm])
            od.frame_device(db.ptr + i * buf.shape[1] * 16, int(cnt[i]))
        od.sync()
        return od.poses(), [od._map(w) for w in (0, 1)], None
    finally:
        db.free()


@pytest.mark.parametrize("preset,frames,theta,lines,set_map_at", [
    ("S64", 600, (0.4, 75), 64, None),    # configs[1]
    ("S64", 200, (0.0, 0), 64, 120),      # configs[0], a host map write half way
    ("S64V", 200, (0.4, 75), 64, None),   # the dense scene
])
def test_dep_small_table_equals_full(pa, pfsynth, preset, frames, theta, lines, set_map_at):
    a = _tie_run(pa, pfsynth, preset, frames, False, theta, lines, set_map_at)
    b = _tie_run(pa, pfsynth, preset, frames, True, theta, lines, set_map_at)
    _same(a, b)


def test_dep_small_table_configs4(pa, pfsynth):
    """configs[4]: S128 scans against the 2M-point surf map (set after frame 1), 12 frames"""
    a = _tie_run(pa, pfsynth, "S128", 12, False, (0.0, 0), 128, set_map_at=1, big_map=True)
    b = _tie_run(pa, pfsynth, "S128", 12, True, (0.0, 0), 128, set_map_at=1, big_map=True)
    _same(a, b)
