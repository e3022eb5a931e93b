"""GPU: exact radius-gated 5-NN (k_knn_query) against the oracle's brute-force search.

Bit-exact: the same 5 indices (ties by map index) and the same f32 squared distances
(accumulated x -> y -> z) wherever the oracle's neighbour lies within the 1 m^2 gate that
src/odomEstimationClass.cpp:299-300 / :447-451 apply; beyond the gate the GPU reports -1 / inf."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(pa, pfref, mp, q):
    kn = pa.Knn(mp.shape[0], q.shape[0])
    kn.set_map(mp)
    gi, gd = kn.query(q)
    ri, rd = pfref.knn(mp, q, 5, opts=pfref.KNN_BRUTE)
    inside = rd < 1.0
    np.testing.assert_array_equal(np.where(inside, ri, -1), gi)
    np.testing.assert_array_equal(gd[inside].view(np.uint32), rd[inside].view(np.uint32))
    assert np.all(np.isinf(gd[~inside]))
    return gi


def test_knn_random_with_ties(pa, pfref):
    rng = np.random.default_rng(0)
    mp = np.zeros((30000, 4), np.float32)
    mp[:, :3] = rng.uniform(-12, 12, (30000, 3))
    mp[:8000, 2] = 0.0                               # plane
    mp[8000:9000, :3] = np.round(mp[8000:9000, :3])   # lattice points, duplicated distances
    mp[9000:9100] = mp[9100:9200]                     # exact duplicates
    q = np.zeros((6000, 4), np.float32)
    q[:, :3] = rng.uniform(-13, 13, (6000, 3))
    q[:500, :3] = np.round(q[:500, :3]) + 0.5         # equidistant from lattice neighbours
    gi = _check(pa, pfref, mp, q)
    assert (gi[:, 4] >= 0).sum() > 1000


def test_knn_dense_map(pa, pfref, pfsynth):
    mp = pfsynth.dense_map(200000, seed=5)
    q = pfsynth.dense_queries(mp, 3000, sigma=0.3, seed=6)
    gi = _check(pa, pfref, mp, q)
    assert (gi[:, 4] >= 0).mean() > 0.3


def test_knn_far_and_negative_coordinates(pa, pfref):
    rng = np.random.default_rng(1)
    mp = np.zeros((5000, 4), np.float32)
    mp[:, :3] = rng.uniform(-2000, -1990, (5000, 3))
    q = np.zeros((800, 4), np.float32)
    q[:, :3] = rng.uniform(-2002, -1988, (800, 3))
    q[:50, :3] = 1e4                                   # nothing anywhere near
    gi = _check(pa, pfref, mp, q)
    assert np.all(gi[:50] == -1)


def test_knn_tiny_map(pa, pfref):
    mp = np.array([[0, 0, 0, 0], [0.5, 0, 0, 0], [0, 0.5, 0, 0]], np.float32)
    q = np.array([[0.1, 0.1, 0, 0], [5, 5, 5, 0]], np.float32)
    kn = pa.Knn(3, 2)
    kn.set_map(mp)
    gi, gd = kn.query(q)
    assert list(gi[0, :3]) == [0, 1, 2] and np.all(gi[0, 3:] == -1)
    assert np.all(gi[1] == -1)


def test_knn_golden(pa):
    """Against the committed vectors (tests/golden/knn_3000x400.npz): gated neighbours bit-exact."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "knn_3000x400.npz"))
    kn = pa.Knn(g["map"].shape[0], g["queries"].shape[0])
    kn.set_map(g["map"])
    gi, gd = kn.query(g["queries"])
    inside = g["d2"] < 1.0
    np.testing.assert_array_equal(np.where(inside, g["idx"], -1), gi)
    np.testing.assert_array_equal(gd[inside].view(np.uint32), g["d2"][inside].view(np.uint32))


def test_knn_config5_full_size(pa, pfref, pfsynth):
    """configs[4] at full size: the 2M-point dense map and the 200k jittered queries of the roofline
    leg (bench.py knn_roofline), every gated idx / d^2 bit-exact against the oracle's kd-tree (itself
    checked against brute force on every 100th query), and the kernel's algorithmic byte count built
    from the GPU's own |C(q)| (k_knn_cellpop) equal to the oracle's count."""
    mp = pfsynth.dense_map(2_000_000, seed=5)
    q = pfsynth.dense_queries(mp, 200_000, sigma=0.3, seed=6)
    kn = pa.Knn(mp.shape[0], q.shape[0])
    kn.set_map(mp)
    gi, gd = kn.query(q)
    ri, rd = pfref.knn(mp, q, 5)                      # kd-tree
    bi, bd = pfref.knn(mp, q[::100], 5, opts=pfref.KNN_BRUTE)
    ins = bd < 1.0
    np.testing.assert_array_equal(np.where(ins, bi, -1), np.where(ins, ri[::100], -1))
    inside = rd < 1.0
    np.testing.assert_array_equal(np.where(inside, ri, -1), gi)
    np.testing.assert_array_equal(gd[inside].view(np.uint32), rd[inside].view(np.uint32))
    assert np.all(np.isinf(gd[~inside]))
    assert (gi[:, 4] >= 0).sum() == 181836
    _, alg = kn.bench(1)
    pop = pfref.knn_cellpop(mp, q)
    assert alg == q.shape[0] * (16 + 40 + 27 * 8) + 16 * pop


def test_knn_thick_layout_equals_grid_walk(pa, pfsynth):
    """The standalone kNN's thick-row layout (every cell holding its z - 1, z, z + 1 layers, pf_knn.h)
    gives the same bits as the 9-row walk of the plain cell grid, including queries one layer below
    and above the map's bounding box and outside it."""
    import ctypes
    mp = pfsynth.dense_map(300000, seed=5)
    q = pfsynth.dense_queries(mp, 20000, sigma=0.3, seed=6)
    lo, hi = mp[:, :3].min(0), mp[:, :3].max(0)
    q[:300, 2] = lo[2] - np.linspace(0.01, 1.5, 300)              # below the grid, in and out of reach
    q[300:600, 2] = hi[2] + np.linspace(0.01, 1.5, 300)           # above it
    q[600:700, :2] = lo[:2] - 0.5                                  # off a corner
    out = []
    for layout in (1, 0):
        kn = pa.Knn(mp.shape[0], q.shape[0])
        assert pa.lib().pf_knn_set_layout(ctypes.c_void_p(kn._h), layout) == 0
        kn.set_map(mp)
        out.append(kn.query(q))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1].view(np.uint32), out[1][1].view(np.uint32))
    assert (out[0][0][:600, 0] >= 0).sum() > 50                      # some off-grid queries found neighbours


def test_knn_gate_boundary_both_layouts(pa, pfref):
    """d^2 == 1.0 exactly is outside the gate (the empty list slot is keyed (1.0, index 0), pf_knn.h):
    map point 0 and others at exactly 1 m along the axes are never reported, points just inside are,
    in the thick-row layout and in the 9-row walk alike."""
    import ctypes
    just_in = np.nextafter(np.float32(1.0), np.float32(0.0))
    mp = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, -1, 0], [just_in, 0, 0, 0], [0, -just_in, 0, 0],
                   [0.5, 0.5, 0.5, 0], [3, 3, 3, 0]], np.float32)
    q = np.array([[0, 0, 0, 0], [2, 0, 0, 0], [1, 1, 0, 0]], np.float32)
    ri, rd = pfref.knn(mp, q, 5, opts=pfref.KNN_BRUTE)
    inside = rd < 1.0
    for layout in (1, 0):
        kn = pa.Knn(mp.shape[0], q.shape[0])
        assert pa.lib().pf_knn_set_layout(ctypes.c_void_p(kn._h), layout) == 0
        kn.set_map(mp)
        gi, gd = kn.query(q)
        np.testing.assert_array_equal(np.where(inside, ri, -1), gi)
        np.testing.assert_array_equal(gd[inside].view(np.uint32), rd[inside].view(np.uint32))
        assert sorted(gi[0][gi[0] >= 0]) == [3, 4, 5]          # the exact-1 m points 0, 1, 2 are out
        assert 0 not in gi[1]                                  # (2,0,0) -> point 0 at exactly 1 m
