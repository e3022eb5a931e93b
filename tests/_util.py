"""Helpers shared by the tests."""
import numpy as np


def pose_err(p, r):
    """(translation error m, rotation error rad) between poses {qx,qy,qz,qw,tx,ty,tz}."""
    dt = float(np.linalg.norm(np.asarray(p[4:7]) - np.asarray(r[4:7])))
    q = np.asarray(p[:4]) * (1.0 if float(np.dot(p[:4], r[:4])) >= 0 else -1.0)
    dr = float(2.0 * np.linalg.norm(q - np.asarray(r[:4])))
    return dt, dr


def quat_to_mat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def rand_quat(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    return q if q[3] >= 0 else -q


def as_bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a.view(np.uint64)
