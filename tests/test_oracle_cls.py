"""CPU: the oracle's BPF front end — groundSeg::ground_seg and nongroundExtract::featureExtract
(include/preProcess.hpp:398-505, :646-689; chained as src/additionNode.cpp:21-45).

The reference ships no tests or fixtures for these either, so the C oracle is pinned by
(1) a second, independent restatement in plain Python loops of ground_seg on small clouds, (2) a
numpy restatement of the PCA decision (float32 sequential sums, the shared eigensolver) with a
brute-force radius search, and (3) known-answer geometry: points on a vertical line are pillars,
on a horizontal line above beam_height_min beams, on a vertical plane facades, on the ground plane
nothing, and the edge cases of the reference's loops (cells below gf_grid_pt_num_thre dropped,
high points pushed first, the 3x3 neighbour minimum, the strict radius gate, the k cap)."""
import math

import numpy as np
import pytest

F32_MAX = float(np.finfo(np.float32).max)


def f32(x):
    return float(np.float32(x))


def ground_seg_py(xyz, p):
    """include/preProcess.hpp:398-505 in plain Python (float32 where the reference uses float)."""
    n = len(xyz)
    if n == 0:
        return [], []
    xs = [float(v) for v in xyz[:, 0]]
    ys = [float(v) for v in xyz[:, 1]]
    zs = [f32(v) for v in xyz[:, 2]]
    min_x, max_x, min_y, max_y = min(xs), max(xs), min(ys), max(ys)
    res = float(np.float32(p.gf_grid_res))
    row = math.ceil((max_y - min_y) / res)
    col = math.ceil((max_x - min_x) / res)
    num = row * col
    cnt = [0] * num
    ids = [[] for _ in range(num)]
    minz = [F32_MAX] * num
    nbz = [F32_MAX] * num
    ground, unground = [], []
    maxg, ming = f32(p.gf_max_ground_height), f32(p.gf_min_ground_height)
    for j in range(n):
        tc = math.floor((xs[j] - min_x) / res)
        tr = math.floor((ys[j] - min_y) / res)
        tid = tr * col + tc
        if not (0 <= tid < num):
            continue
        cnt[tid] += 1
        if zs[j] > maxg:
            unground.append(j)
        else:
            ids[tid].append(j)
            if zs[j] < minz[tid] and zs[j] > ming:
                minz[tid] = nbz[tid] = zs[j]
    for m in range(num):
        r, c = divmod(m, col)
        if 1 <= r <= row - 2 and 1 <= c <= col - 2:
            for dj in (-1, 0, 1):
                for dk in (-1, 0, 1):
                    if nbz[m] > minz[m + dj * col + dk]:
                        nbz[m] = minz[m + dj * col + dk]
    for i in range(num):
        if cnt[i] < p.gf_min_grid_pts:
            continue
        if f32(np.float32(minz[i]) - np.float32(nbz[i])) < f32(p.gf_neighbor_height_diff):
            for j in ids[i]:
                if f32(np.float32(zs[j]) - np.float32(minz[i])) < f32(p.gf_max_height_diff) and zs[j] > ming:
                    ground.append(j)
                else:
                    unground.append(j)
        else:
            unground.extend(ids[i])
    return ground, unground


def pca_code_np(pfref, pts, nb, qz, p):
    """:653-688 / :283-323 with float32 sequential sums and the oracle's eigensolver."""
    n = len(nb)
    if not (n > p.k_min) or n <= 3:
        return 0
    P = pts[nb].astype(np.float32)
    s = np.zeros(3, np.float32)
    for e in range(n):
        s = s + P[e]
    m = s / np.float32(n)
    c = np.zeros(6, np.float32)
    for e in range(n):
        d = P[e] - m
        c = c + np.array([d[0] * d[0], d[0] * d[1], d[0] * d[2], d[1] * d[1], d[1] * d[2], d[2] * d[2]], np.float32)
    ev, V = pfref.eigen_sym3(c.astype(np.float64))
    l1, l2, l3 = (np.float32(ev[2]), np.float32(ev[1]), np.float32(ev[0]))
    v0 = V[:, 2].astype(np.float32)
    v1 = V[:, 1].astype(np.float32)
    nv = np.array([v0[1] * v1[2] - v0[2] * v1[1], v0[2] * v1[0] - v0[0] * v1[2], v0[0] * v1[1] - v0[1] * v1[0]],
                  np.float32)
    for v in (v0, nv):
        sq = np.float32(np.float32(v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
        if sq > 0:
            v /= np.sqrt(sq)
    lin = (float(l1) - float(l2)) / float(l1)
    pla = (float(l2) - float(l3)) / float(l1)
    if lin > f32(p.edge_thre):
        if abs(v0[2]) > np.float32(p.linear_vsin_high):
            return 1
        if abs(v0[2]) < np.float32(p.linear_vsin_low) and qz < np.float32(p.beam_h_max) and qz > np.float32(p.beam_h_min):
            return 2
    elif pla > f32(p.planar_thre):
        if abs(nv[2]) < np.float32(p.planar_vsin_low):
            return 3
    return 0


def radius_knn_brute(pts, i, r2, k):
    d = np.zeros(len(pts), np.float32)
    for a in range(3):
        t = (pts[i, a] - pts[:, a]).astype(np.float32)
        d = (d + t * t).astype(np.float32)
    sel = np.nonzero(d < np.float32(r2))[0]
    order = np.lexsort((sel, d[sel]))
    return sel[order][:k]


def scene(seed, n=1500):
    """ground + a wall + a pole + a beam + clutter, with some points above 5 m"""
    rng = np.random.default_rng(seed)
    parts = [
        np.c_[rng.uniform(-15, 15, (n, 2)), rng.normal(-1.7, 0.02, n)],                   # ground
        np.c_[rng.uniform(2, 8, n // 3), np.full(n // 3, 6.0) + rng.normal(0, 0.01, n // 3),
              rng.uniform(-1.7, 6.5, n // 3)],                                             # facade
        np.c_[rng.normal(-4, 0.01, 200), rng.normal(-4, 0.01, 200), rng.uniform(-1.7, 4, 200)],  # pole
        np.c_[rng.uniform(-10, -6, 200), rng.normal(3, 0.01, 200), rng.normal(3.0, 0.01, 200)],  # beam
        rng.uniform([-15, -15, -2], [15, 15, 8], (150, 3)),                               # clutter
    ]
    xyz = np.concatenate(parts).astype(np.float32)
    return xyz[rng.permutation(len(xyz))]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ground_seg_matches_python_restatement(pfref, seed):
    xyz = scene(seed, 1200)
    p = pfref.cls_params()
    g, u = pfref.ground_seg(xyz, p)
    g2, u2 = ground_seg_py(xyz, p)
    assert list(g) == g2 and list(u) == u2
    assert len(g) > 500 and len(u) > 400


def test_ground_seg_order_and_edge_cases(pfref):
    p = pfref.cls_params()
    rng = np.random.default_rng(3)
    flat = np.c_[rng.uniform(0, 12, (400, 2)), np.full(400, -1.7)].astype(np.float32)
    high = np.array([[1, 1, 6.0], [5, 5, 7.0]], np.float32)          # above gf_max_ground_height
    sparse = np.array([[20.5, 20.5, -1.7]] * 3, np.float32)          # a cell with 3 < 8 points
    xyz = np.concatenate([flat, high, sparse])
    g, u = pfref.ground_seg(xyz, p)
    assert list(u[:2]) == [400, 401]                                  # high points first, input order
    assert not set(range(402, 405)) & set(g) and not set(range(402, 405)) & set(u)   # dropped
    # points pushed cell by cell, input order inside a cell
    assert sorted(g) != list(g) or len(g) < 2
    # a raised cell (min z 2 m above its neighbours) is all non-ground
    box = np.c_[rng.uniform(4.5, 5.5, (30, 2)), np.full(30, 0.5)].astype(np.float32)
    g2, u2 = pfref.ground_seg(np.concatenate([flat, box]), p)
    assert not set(range(400, 430)) & set(g2)
    g0, u0 = pfref.ground_seg(np.zeros((0, 3), np.float32), p)
    assert len(g0) == 0 and len(u0) == 0


def test_pca_classify_matches_numpy_restatement(pfref):
    xyz = scene(4, 700)
    p = pfref.cls_params()
    cls, num = pfref.pca_classify(xyz, p)
    for i in range(0, len(xyz), 3):
        nb = radius_knn_brute(xyz, i, 1.0, 25)
        assert num[i] == len(nb)
        assert cls[i] == pca_code_np(pfref, xyz, nb, xyz[i, 2], p), i
    assert set(np.unique(cls)) == {0, 1, 2, 3}


def test_pca_known_geometry(pfref):
    p = pfref.cls_params()
    t = np.linspace(0, 4, 81, dtype=np.float32)
    pole = np.c_[np.zeros(81), np.zeros(81), t - 1].astype(np.float32)
    beam_hi = np.c_[t + 10, np.zeros(81), np.full(81, 2.0)].astype(np.float32)
    beam_lo = np.c_[t + 20, np.zeros(81), np.full(81, 0.2)].astype(np.float32)   # below beam_h_min
    rng = np.random.default_rng(7)
    u, v = rng.uniform(0, 3, (2, 2000))
    wall = np.c_[u + 30, np.full(u.size, 5.0), v].astype(np.float32)
    floor = np.c_[u + 40, v, np.full(u.size, -1.0)].astype(np.float32)
    interior = (u > 0.4) & (u < 2.6) & (v > 0.4) & (v < 2.6)
    for cloud, want in ((pole, 1), (beam_hi, 2), (beam_lo, 0)):      # 1-D: l2 = l3 = 0, linear_2 = 1
        cls, num = pfref.pca_classify(cloud, p)
        inner = num > p.k_min
        assert inner.sum() > 10 and np.all(cls[inner] == want) and np.all(cls[~inner] == 0)
    # 2-D: 25 random neighbours give planar_2 = l2 / l1 above or below 0.65 by sampling noise; a
    # vertical plane is facade or nothing (never beam), a horizontal one never facade
    cls, num = pfref.pca_classify(wall, p)
    assert np.all(cls[interior] != 2) and np.mean(cls[interior] == 3) > 0.4
    cls, num = pfref.pca_classify(floor, p)
    assert not np.any(cls == 3) and not np.any(cls == 2)
    # k caps the neighbourhood; the gate is strict
    cls, num = pfref.pca_classify(pole, pfref.cls_params(k=5))
    assert num.max() == 5
    two = np.array([[0, 0, 0], [1, 0, 0], [0.5, 0, 0]], np.float32)
    _, num = pfref.pca_classify(two, p)
    assert list(num) == [2, 2, 3]                                    # d^2 = 1 exactly is outside


def test_pca_normals_known_geometry(pfref):
    """assign_normal (include/preProcess.hpp:327-346): a pole's points carry the principal direction
    (+-z) with linear_2 = 1 in the fourth float, a wall's facade points the wall normal (+-y) with
    planar_2 there. Every other point with more than 3 neighbours keeps what get_pc_pca_feature wrote
    (:238-239): its PCA normal direction and planar_2 (about 0 on a pole); points with 0-3 neighbours
    carry the zero-initialised feature's zeros."""
    p = pfref.cls_params()
    t = np.linspace(0, 4, 81, dtype=np.float32)
    pole = np.c_[np.zeros(81), np.zeros(81), t - 1].astype(np.float32)
    cls, num, nrm = pfref.pca_classify(pole, p, normals=True)
    on = cls == 1
    assert on.sum() > 10
    np.testing.assert_allclose(np.abs(nrm[on, 2]), 1.0, atol=1e-6)
    np.testing.assert_allclose(nrm[on, 3], 1.0, atol=1e-6)
    sparse = np.c_[np.zeros(14), np.zeros(14), np.arange(14) * 0.3 - 1].astype(np.float32)
    cls, num, nrm = pfref.pca_classify(sparse, p, normals=True)
    rest = (num > 3) & (cls == 0)                  # 4-7 neighbours: unclassified (k_min 8) but normal set
    assert rest.sum() > 5
    np.testing.assert_allclose(np.linalg.norm(nrm[rest, :3], axis=1), 1.0, atol=1e-5)
    assert np.all(np.abs(nrm[rest, 3]) < 1e-3)
    few = np.c_[np.zeros(3), np.zeros(3), np.arange(3) * 0.3].astype(np.float32)
    cls, num, nrm = pfref.pca_classify(few, p, normals=True)
    assert list(num) == [3, 3, 3] and np.all(nrm == 0)          # the point itself counts
    rng = np.random.default_rng(7)
    u, v = rng.uniform(0, 3, (2, 2000))
    wall = np.c_[u + 30, np.full(u.size, 5.0), v].astype(np.float32)
    cls, num, nrm = pfref.pca_classify(wall, p, normals=True)
    f = cls == 3
    assert f.sum() > 100
    np.testing.assert_allclose(np.abs(nrm[f, 1]), 1.0, atol=1e-5)
    assert np.all((nrm[f, 3] > 0.65) & (nrm[f, 3] <= 1.0))
    c2, n2 = pfref.pca_classify(wall, p)                       # the plain entry point: same classes
    np.testing.assert_array_equal(c2, cls)


def test_preprocess_chain(pfref, pfsynth):
    x = pfsynth.Sequence("S32", n_frames=2, az_steps=500).frame(1)
    p = pfref.cls_params()
    r = pfref.bpf_preprocess(x, p)
    g, u = pfref.ground_seg(x, p)
    np.testing.assert_array_equal(r["ground"], g)
    cls, _ = pfref.pca_classify(x[u], p)
    np.testing.assert_array_equal(r["pillar"], u[cls == 1])
    np.testing.assert_array_equal(r["beam"], u[cls == 2])
    np.testing.assert_array_equal(r["facade"], u[cls == 3])
    assert len(r["facade"]) > 100 and len(r["pillar"]) > 10
    off = pfref.bpf_preprocess(x, pfref.cls_params(ground_filter=0))
    cls0, _ = pfref.pca_classify(x, p)
    np.testing.assert_array_equal(off["facade"], np.nonzero(cls0 == 3)[0])
    assert len(off["ground"]) == 0
