"""CPU: the oracle's LaserMappingClass (src/laserMappingClass.cpp) — the global map of
src/laserMappingNode.cpp. Pinned by a numpy restatement (f32 transform in PCL's Transformer order,
50 m cubes, per-cube VoxelGrid of the 5x5x5 neighbourhood, getMap's cube order) and by properties:
a scan of one point per voxel at the identity pose comes back unchanged, repeated scans at the
same pose do not grow the map, points far from the pose land in allocated cubes or are refused."""
import numpy as np


def q2m(q):
    x, y, z, w = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz, txx, txy, txz = tx * w, ty * w, tz * w, tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy], [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]])


def voxel_np(P, leaf):
    leaf = np.float32(leaf)
    inv = np.float32(1) / leaf
    mn, mx = P[:, :3].min(0), P[:, :3].max(0)
    mb = np.floor(mn * inv).astype(np.int64)
    db = np.floor(mx * inv).astype(np.int64) - mb + 1
    ijk = (np.floor(P[:, :3] * inv) - mb.astype(np.float32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * db[0] + ijk[:, 2] * db[0] * db[1]
    order = np.argsort(idx, kind="stable")
    out = []
    s = 0
    while s < len(order):
        e = s
        while e < len(order) and idx[order[e]] == idx[order[s]]:
            e += 1
        acc = np.zeros(4, np.float32)
        for k in order[s:e]:
            acc = (acc + P[k]).astype(np.float32)
        out.append(acc / np.float32(e - s))
        s = e
    return np.array(out, np.float32).reshape(-1, 4)


class MapNp:
    def __init__(self, leaf):
        self.leaf, self.cubes = leaf, {}
        self._alloc(0, 0, 0)

    def _alloc(self, cx, cy, cz):
        for i in range(cx - 2, cx + 3):
            for j in range(cy - 2, cy + 3):
                for k in range(cz - 2, cz + 3):
                    self.cubes.setdefault((i, j, k), np.zeros((0, 4), np.float32))

    def update(self, xyzi, pose):
        c = lambda v: int(np.floor(v / 50.0 + 0.5))
        cx, cy, cz = c(pose[4]), c(pose[5]), c(pose[6])
        self._alloc(cx, cy, cz)
        R = q2m(pose[:4]).astype(np.float32)
        t = np.asarray(pose[4:], np.float64).astype(np.float32)
        p = xyzi[:, :3].astype(np.float32)
        w = np.empty((len(p), 4), np.float32)
        for a in range(3):
            w[:, a] = p[:, 0] * R[a, 0] + (p[:, 1] * R[a, 1] + (p[:, 2] * R[a, 2] + t[a]))
        w[:, 3] = np.minimum(1.0, np.maximum(p[:, 2].astype(np.float64) + 2.0, 0.0) / 5).astype(np.float32)
        for q in w:
            key = (c(float(q[0])), c(float(q[1])), c(float(q[2])))
            assert key in self.cubes
            self.cubes[key] = np.vstack([self.cubes[key], q[None]])
        for i in range(cx - 2, cx + 3):
            for j in range(cy - 2, cy + 3):
                for k in range(cz - 2, cz + 3):
                    if len(self.cubes[(i, j, k)]):
                        self.cubes[(i, j, k)] = voxel_np(self.cubes[(i, j, k)], self.leaf)

    def get(self):
        return np.vstack([self.cubes[k] for k in sorted(self.cubes)] + [np.zeros((0, 4), np.float32)])


def test_matches_numpy_restatement(pfref):
    rng = np.random.default_rng(3)
    m, ref = pfref.GlobalMap(1.0), MapNp(1.0)
    pose = np.array([0, 0, 0, 1, 0, 0, 0.0])
    for f in range(4):
        yaw = 0.3 * f
        pose = np.array([0, 0, np.sin(yaw / 2), np.cos(yaw / 2), 20.0 * f, 3.0 * f, 0.1])
        x = np.c_[rng.uniform(-60, 60, (400, 2)), rng.uniform(-3, 8, 400), rng.uniform(0, 1, 400)].astype(np.float32)
        assert m.update(x, pose) == 0
        ref.update(x, pose)
        np.testing.assert_array_equal(m.get(), ref.get())
    assert len(m.get()) > 600


def test_properties(pfref):
    m = pfref.GlobalMap(0.5)
    g = np.stack(np.meshgrid(np.arange(4), np.arange(4), np.arange(3), indexing="ij"), -1).reshape(-1, 3)
    x = np.c_[g * 0.5 + 0.25, np.zeros(len(g))].astype(np.float32)      # one point per 0.5 m voxel
    ident = np.array([0, 0, 0, 1, 0, 0, 0.0])
    assert m.update(x, ident) == 0
    out = m.get()
    assert out.shape == (len(g), 4)
    np.testing.assert_array_equal(np.sort(out[:, 0]), np.sort(x[:, 0]))
    n1 = len(out)
    assert m.update(x, ident) == 0 and len(m.get()) == n1                # same voxels: no growth
    far = np.array([[300.0, 0, 0, 0]], np.float32)                      # cube 6: never allocated
    assert m.update(far, ident) == -1 and len(m.get()) == n1
