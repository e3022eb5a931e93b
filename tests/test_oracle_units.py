"""CPU: the oracle's building blocks against independent numpy restatements and known answers.

The reference ships no unit tests or fixtures, so the oracle is pinned here by
properties of the functions it restates: src/lidarOptimization.cpp (Plus, getTransformFromSe3,
Edge/SurfNormAnalyticCostFunction), the Eigen 3.3 eigensolver / QR / polar factor, PCL VoxelGrid and
OdomBaseClass::rgbds (src/odomEstimationClass.cpp:34-134), FLANN-style exact kNN.
"""
import numpy as np
import pytest

from _util import quat_to_mat, rand_quat, skew


def np_se3_plus(x, d):
    """getTransformFromSe3 + Plus (src/lidarOptimization.cpp:80-143) in numpy."""
    w, u = np.asarray(d[:3], float), np.asarray(d[3:], float)
    th = np.linalg.norm(w)
    W = skew(w)
    if th < 1e-10:
        imag = 0.5 - 0.0208333 * th ** 2 + 0.000260417 * th ** 4
        dq = np.array([imag * w[0], imag * w[1], imag * w[2], np.cos(th / 2)])
        J = quat_to_mat(dq)
    else:
        dq = np.r_[np.sin(th / 2) / th * w, np.cos(th / 2)]
        J = np.eye(3) + (1 - np.cos(th)) / th ** 2 * W + (th - np.sin(th)) / th ** 3 * W @ W
    dt = J @ u
    q = x[:4]
    # Hamilton product dq * q, (x, y, z, w) storage
    a, b = dq, q
    prod = np.array([a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1],
                     a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2],
                     a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0],
                     a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]])
    return np.r_[prod, quat_to_mat(dq) @ x[4:] + dt]


def test_se3_plus_matches_exp_map(pfref):
    rng = np.random.default_rng(1)
    for _ in range(50):
        x = np.r_[rand_quat(rng), rng.normal(size=3) * 10]
        d = rng.normal(size=6) * 0.3
        np.testing.assert_allclose(pfref.se3_plus(x, d), np_se3_plus(x, d), atol=1e-12)


def test_se3_plus_small_angle_branch(pfref):
    x = np.array([0, 0, 0, 1.0, 1, 2, 3])
    d = np.array([1e-12, 0, 0, 0.1, 0.2, 0.3])
    out = pfref.se3_plus(x, d)
    np.testing.assert_allclose(out[4:], [1.1, 2.2, 3.3], atol=1e-12)
    np.testing.assert_allclose(pfref.se3_plus(x, np.zeros(6)), x, atol=0)


def test_det_sincos_accuracy(pfref):
    """The deterministic sincos (GPU_EQUIV, pf_geom.h det_sincos) is within 2 ulp of libm over the
    LM's range (half-angles up to pi) and stays close out to 1e4; NaN in gives NaN out."""
    rng = np.random.default_rng(3)
    xs = np.r_[0.0, 1e-300, 1e-12, 1e-6, np.pi / 4, np.pi / 2, np.pi, -np.pi / 3,
               rng.uniform(0, np.pi, 2000), rng.uniform(-50, 50, 500), rng.uniform(-1e4, 1e4, 200)]
    for x in xs:
        s, c = pfref.det_sincos(x)
        tol = 2 * np.spacing(1.0) if abs(x) <= np.pi else 1e-12 * max(1.0, abs(x))
        assert abs(s - np.sin(x)) <= max(tol, 2 * np.spacing(abs(np.sin(x)))), x
        assert abs(c - np.cos(x)) <= max(tol, 2 * np.spacing(abs(np.cos(x)))), x
    assert pfref.det_sincos(0.0) == (0.0, 1.0)
    s, c = pfref.det_sincos(float("nan"))
    assert np.isnan(s) and np.isnan(c)


def test_se3_plus_device_form_matches_faithful(pfref):
    """GPU_EQUIV's SE(3) update (pf_geom.h se3_exp: the source's (1 - cos(theta)) / theta^2 and
    (theta - sin(theta)) / theta^3 on the deterministic sincos) is the faithful getTransformFromSe3 bit for
    bit at LM step sizes, and within an ulp of det_sincos at large angles. Round 3's half-angle identities
    differed by up to ~1e-8 relative in those coefficients at small theta (the source's 1 - cos cancels),
    the difference tools/drift_probe.py traced the S64T free-run separation to."""
    rng = np.random.default_rng(4)
    for scale in (1e-11, 1e-6, 1e-3, 0.3, 2.0):
        for _ in range(40):
            x = np.r_[rand_quat(rng), rng.normal(size=3) * 50]
            d = rng.normal(size=6) * scale
            a, b = pfref.se3_plus_half(x, d), pfref.se3_plus(x, d)
            if scale <= 1e-3:
                np.testing.assert_array_equal(a, b)
            assert np.all(np.abs(a - b) <= 1e-13 * (1 + np.abs(b))), (scale, a - b)


def _fd_jac(f, x, eps=1e-7):
    J = np.zeros(6)
    for i in range(6):
        d = np.zeros(6)
        d[i] = eps
        J[i] = (f(x, d) - f(x, -d)) / (2 * eps)
    return J


def test_edge_residual_and_jacobian(pfref):
    rng = np.random.default_rng(2)
    for _ in range(20):
        x = np.r_[rand_quat(rng), rng.normal(size=3)]
        cur = rng.normal(size=3) * 5
        R = quat_to_mat(x[:4])
        p = R @ cur + x[4:]
        dirn = rng.normal(size=3)
        a, b = p + 0.3 * dirn, p - 0.2 * dirn
        r0, _ = pfref.edge_eval(x, cur, a, b)
        assert abs(r0) < 1e-12                       # point on the line
        off = np.cross(dirn, rng.normal(size=3))
        a2, b2 = a + off, b + off
        r, J = pfref.edge_eval(x, cur, a2, b2)
        assert r == pytest.approx(np.linalg.norm(off), rel=1e-9)
        f = lambda xx, d: pfref.edge_eval(pfref.se3_plus(xx, d), cur, a2, b2)[0]
        np.testing.assert_allclose(J[:6], _fd_jac(f, x), atol=1e-6)
        assert J[6] == 0.0


def test_surf_residual_and_jacobian(pfref):
    rng = np.random.default_rng(3)
    for _ in range(20):
        x = np.r_[rand_quat(rng), rng.normal(size=3)]
        cur = rng.normal(size=3) * 5
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        p = quat_to_mat(x[:4]) @ cur + x[4:]
        r0, _ = pfref.surf_eval(x, cur, n, -n @ p)
        assert abs(r0) < 1e-12
        d = -n @ p + 0.25
        r, J = pfref.surf_eval(x, cur, n, d)
        assert r == pytest.approx(0.25, abs=1e-12)
        f = lambda xx, dd: pfref.surf_eval(pfref.se3_plus(xx, dd), cur, n, d)[0]
        np.testing.assert_allclose(J[:6], _fd_jac(f, x), atol=1e-6)


@pytest.mark.parametrize("w", [1.0, 2.0, 12.0])
def test_weight_scales_residual_only(pfref, w):
    """weightType 1/2/12 multiply the residual but not the Jacobian (lidarOptimization.cpp:25-43,66-76)."""
    x = np.array([0, 0, 0.1, np.sqrt(1 - 0.01), 0.5, -0.2, 0.1])
    cur, a, b = np.array([3.0, 1, 0.5]), np.array([1.0, 2, 3]), np.array([2.0, 2.5, 2])
    r0, J0 = pfref.edge_eval(x, cur, a, b, 0.0)
    r1, J1 = pfref.edge_eval(x, cur, a, b, w)
    assert r1 == pytest.approx(w * r0, rel=1e-15)
    np.testing.assert_array_equal(J0, J1)
    n = np.array([0.0, 0.6, 0.8])
    s0, K0 = pfref.surf_eval(x, cur, n, 0.3, 0.0)
    s1, K1 = pfref.surf_eval(x, cur, n, 0.3, w)
    assert s1 == pytest.approx(w * s0, rel=1e-15)
    np.testing.assert_array_equal(K0, K1)


def test_eigen_sym3_matches_numpy(pfref):
    rng = np.random.default_rng(4)
    for _ in range(100):
        A = rng.normal(size=(3, 3))
        A = A @ A.T
        a6 = [A[0, 0], A[0, 1], A[0, 2], A[1, 1], A[1, 2], A[2, 2]]
        ev, V = pfref.eigen_sym3(a6)
        ref = np.linalg.eigvalsh(A)
        np.testing.assert_allclose(ev, ref, rtol=1e-12, atol=1e-12)
        assert np.all(np.diff(ev) >= 0)
        np.testing.assert_allclose(A @ V, V * ev, atol=1e-10)


def test_plane_fit_matches_lstsq(pfref):
    rng = np.random.default_rng(5)
    for _ in range(100):
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        c = rng.normal(size=3) * 20
        t1 = np.cross(n, [1, 0, 0])
        t1 /= np.linalg.norm(t1)
        t2 = np.cross(n, t1)
        A = c + rng.normal(size=(5, 1)) * t1 + rng.normal(size=(5, 1)) * t2 + rng.normal(size=(5, 1)) * 0.01 * n
        got = pfref.plane_fit(A)
        ref = np.linalg.lstsq(A, -np.ones(5), rcond=None)[0]
        np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-12)


def test_rotation_polar(pfref):
    """Isometry3d::rotation() in Eigen 3.3 = orthogonal polar factor (SVD)."""
    rng = np.random.default_rng(6)
    for _ in range(100):
        R = quat_to_mat(rand_quat(rng))
        np.testing.assert_allclose(pfref.rotation_polar(R), R, atol=2e-15)
        M = R + rng.normal(size=(3, 3)) * 1e-6
        U, _, Vt = np.linalg.svd(M)
        P = U @ Vt
        got = pfref.rotation_polar(M)
        np.testing.assert_allclose(got, P, atol=1e-13)
        np.testing.assert_allclose(got @ got.T, np.eye(3), atol=1e-14)


def _np_voxel_grid(pts, leaf):
    """PCL VoxelGrid<PointXYZRGB>: f32 keys from the inverse leaf, stable order."""
    xyz = pts[:, :3].astype(np.float32)
    inv = np.float32(1.0) / np.float32(leaf)
    mn, mx = xyz.min(0), xyz.max(0)
    minb = np.floor(mn * inv).astype(np.int64)
    maxb = np.floor(mx * inv).astype(np.int64)
    div = maxb - minb + 1
    ijk = (np.floor(xyz * inv) - minb.astype(np.float32)).astype(np.int64)
    key = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = np.argsort(key, kind="stable")
    out = []
    k = key[order]
    starts = np.r_[0, np.nonzero(np.diff(k))[0] + 1, len(k)]
    for s, e in zip(starts[:-1], starts[1:]):
        acc = np.zeros(3, np.float32)
        for i in order[s:e]:
            acc = (acc + xyz[i]).astype(np.float32)
        out.append(acc / np.float32(e - s))
    return np.array(out, np.float32)


def test_voxel_grid_matches_numpy(pfref):
    rng = np.random.default_rng(7)
    xyz = rng.uniform(-20, 20, size=(3000, 3)).astype(np.float32)
    xyz[:500] = np.round(xyz[:500] * 2.5) / np.float32(2.5)      # exact boundary hits
    pts = pfref.pack_rgb(xyz)
    got = pfref.voxel_grid(pts, 0.8, opts=pfref.VG_STABLE)
    ref = _np_voxel_grid(pts, 0.8)
    assert got.shape[0] == ref.shape[0]
    np.testing.assert_array_equal(got[:, :3].view(np.uint32), ref.view(np.uint32))


def test_voxel_grid_overflow_copies_input(pfref):
    """Leaf too small for int32 voxel ids: PCL warns and returns the input unchanged."""
    xyz = np.array([[-1000, -1000, -1000], [1000, 1000, 1000], [0, 0, 0]], np.float32)
    pts = pfref.pack_rgb(xyz)
    got = pfref.voxel_grid(pts, 0.001)
    np.testing.assert_array_equal(got, pts)


def test_voxel_grid_empty(pfref):
    assert pfref.voxel_grid(np.zeros((0, 4), np.float32), 0.4).shape[0] == 0


def test_rgbds_keeps_max_r_g(pfref):
    """rgbds: voxel centroid, r = max r, g = max g (src/odomEstimationClass.cpp:86-131)."""
    xyz = np.array([[0.1, 0.1, 0.1], [0.2, 0.3, 0.1], [0.35, 0.05, 0.2], [5.1, 5.1, 5.1]], np.float32)
    pts = pfref.pack_rgb(xyz, r=[3, 9, 1, 7], g=[200, 4, 17, 0])
    out = pfref.rgbds(pts, 0.4, opts=pfref.VG_STABLE)
    assert out.shape[0] == 2
    xyz_o, r, g = pfref.unpack_rgb(out)
    np.testing.assert_allclose(xyz_o[0], xyz[:3].mean(0), rtol=1e-6)
    assert (r[0], g[0]) == (9, 200)
    assert (r[1], g[1]) == (7, 0)


def test_knn_kdtree_equals_brute_and_numpy(pfref):
    rng = np.random.default_rng(8)
    mp = np.zeros((4000, 4), np.float32)
    mp[:, :3] = rng.uniform(-10, 10, (4000, 3))
    mp[:1000, 2] = 0.0                                    # a plane: many equal distances
    q = np.zeros((500, 4), np.float32)
    q[:, :3] = rng.uniform(-10, 10, (500, 3))
    i_tree, d_tree = pfref.knn(mp, q, 5)
    i_brute, d_brute = pfref.knn(mp, q, 5, opts=pfref.KNN_BRUTE)
    np.testing.assert_array_equal(i_tree, i_brute)
    np.testing.assert_array_equal(d_tree.view(np.uint32), d_brute.view(np.uint32))
    d = mp[None, :, :3] - q[:, None, :3]
    d2 = ((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]).astype(np.float32)
    ref = np.lexsort((np.broadcast_to(np.arange(4000), d2.shape), d2), axis=1)[:, :5]
    np.testing.assert_array_equal(i_brute, ref)


def test_knn_cellpop_matches_numpy(pfref):
    """|C(q)| of SURVEY 8(d) (the algorithmic bytes' candidate set) against a numpy count."""
    rng = np.random.default_rng(3)
    mp = np.zeros((4000, 4), np.float32)
    mp[:, :3] = rng.uniform(-6, 6, (4000, 3))
    mp[:300, :3] = np.round(mp[:300, :3])                         # on cell faces
    q = np.zeros((500, 4), np.float32)
    q[:, :3] = rng.uniform(-8, 8, (500, 3))
    cm = np.floor(mp[:, :3]).astype(np.int64)
    cq = np.floor(q[:, :3]).astype(np.int64)
    want = 0
    for c in cq:
        want += int(np.all(np.abs(cm - c) <= 1, axis=1).sum())
    assert pfref.knn_cellpop(mp, q) == want


def _sort_inputs():
    rng = np.random.default_rng(11)
    yield np.zeros(0, np.uint32)
    yield np.array([5], np.uint32)
    for n in (2, 3, 15, 16, 17, 18, 33, 100, 1000, 20000):
        yield rng.integers(0, max(2, n // 7), n).astype(np.uint32)         # many ties (voxels)
        yield rng.integers(0, 1 << 30, n).astype(np.uint32)                # few ties
        yield np.sort(rng.integers(0, 50, n)).astype(np.uint32)            # sorted runs
        yield np.sort(rng.integers(0, 50, n))[::-1].astype(np.uint32).copy()
        yield np.full(n, 7, np.uint32)
    k = np.sort(rng.integers(0, 20000, 30000)).astype(np.uint32)           # a voxel-ordered map + a tail
    yield np.concatenate([k, rng.integers(0, 20000, 3000).astype(np.uint32)])
    n = 4096                                                               # organ pipe
    yield np.concatenate([np.arange(n // 2), np.arange(n // 2)[::-1]]).astype(np.uint32)


def test_introsort_restatements_equal_std_sort(pfref):
    """libstdc++ std::sort (the reference's VoxelGrid / rgbds sort, src/odomEstimationClass.cpp:74)
    leaves equal keys in an order only its algorithm defines. The literal restatement of its introsort
    and the level-synchronous form the device's reference-tie-order mode runs give exactly its
    permutation on tie-heavy, sorted, reversed, constant and map-like inputs."""
    for keys in _sort_inputs():
        want = pfref.sort_perm(keys, "std")
        np.testing.assert_array_equal(pfref.sort_perm(keys, "literal"), want)
        np.testing.assert_array_equal(pfref.sort_perm(keys, "levels"), want)
        assert np.all(np.diff(keys[want].astype(np.int64)) >= 0)


def test_introsort_levels_heap_branch(pfref):
    """The depth-limit branch (make_heap + sort_heap) of both restatements agrees at every small depth
    limit, where most segments end in it."""
    rng = np.random.default_rng(12)
    for n in (17, 40, 300, 5000):
        keys = rng.integers(0, max(2, n // 5), n).astype(np.uint32)
        for depth in (0, 1, 2, 3, 5):
            np.testing.assert_array_equal(pfref.sort_perm(keys, "levels", depth), pfref.sort_perm(keys, "literal", depth))
