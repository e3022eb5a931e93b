"""ctypes binding of the synthetic LiDAR workload generator (libpfsynth.so).

Workload input for tests and bench.py: S64 (KITTI-like 64-line),
S32 (campus 32-line) and S128 scans plus the config-5 dense map. Builds the library
on first use when it is missing (g++ is available on the build host and GPU box).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libpfsynth.so")


def build(force=False):
    src = os.path.join(_HERE, "scan_synth.cpp")
    hdr = os.path.join(_HERE, "scan_synth.h")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-fopenmp", "-fPIC", "-shared", "-o", _LIB, src])
    return _LIB


class Params(ctypes.Structure):
    _fields_ = [("lines", ctypes.c_int), ("az_steps", ctypes.c_int), ("speed", ctypes.c_double),
                ("scan_period", ctypes.c_double), ("yaw_amp", ctypes.c_double),
                ("yaw_period", ctypes.c_double), ("dropout", ctypes.c_double),
                ("range_noise", ctypes.c_double), ("max_range", ctypes.c_double),
                ("sensor_height", ctypes.c_double), ("building_prob", ctypes.c_double),
                ("setback_min", ctypes.c_double), ("setback_max", ctypes.c_double),
                ("seed", ctypes.c_int), ("vegetation", ctypes.c_double), ("terrain", ctypes.c_double),
                ("cross", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        _lib.pfsyn_create.restype = ctypes.c_void_p
        _lib.pfsyn_create.argtypes = [ctypes.POINTER(Params), ctypes.c_int]
        _lib.pfsyn_destroy.argtypes = [ctypes.c_void_p]
        _lib.pfsyn_frame.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
        _lib.pfsyn_frames.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        _lib.pfsyn_gt_pose.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        _lib.pfsyn_dense_map.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
        _lib.pfsyn_dense_queries.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_double, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.c_void_p]
    return _lib


PRESETS = {"S64": 0, "S32": 1, "S128": 2, "S64V": 3, "S64T": 4}


class Sequence:
    """A synthetic sequence: world built along the trajectory for n_frames frames."""

    def __init__(self, preset="S64", n_frames=100, seed=None, **overrides):
        L = lib()
        self.params = Params()
        L.pfsyn_default_params(PRESETS[preset], ctypes.byref(self.params))
        if seed is not None:
            self.params.seed = int(seed)
        for k, v in overrides.items():
            setattr(self.params, k, v)
        self.n_frames = int(n_frames)
        self._h = L.pfsyn_create(ctypes.byref(self.params), self.n_frames)
        if not self._h:
            raise RuntimeError("pfsyn_create failed")
        self.cap = self.params.lines * self.params.az_steps

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pfsyn_destroy(self._h)
            self._h = None

    def frame(self, k, with_ring=False):
        buf = np.empty((self.cap, 4), np.float32)
        ring = np.empty(self.cap, np.int32) if with_ring else None
        n = ctypes.c_size_t()
        rc = lib().pfsyn_frame(self._h, int(k), buf.ctypes.data, self.cap, ctypes.byref(n),
                               ring.ctypes.data if with_ring else None)
        if rc != 0:
            raise RuntimeError("pfsyn_frame overflow")
        if with_ring:
            return buf[:n.value].copy(), ring[:n.value].copy()
        return buf[:n.value].copy()

    def frames(self, f0, nf, threads=0):
        """Returns (buffer [nf, cap, 4] float32, counts [nf])."""
        buf = np.empty((nf, self.cap, 4), np.float32)
        counts = np.empty(nf, np.uint64)
        rc = lib().pfsyn_frames(self._h, int(f0), int(nf), buf.ctypes.data, self.cap, counts.ctypes.data,
                                int(threads))
        if rc != 0:
            raise RuntimeError("pfsyn_frames overflow")
        return buf, counts.astype(np.int64)

    def gt_pose(self, k):
        p = np.empty(7, np.float64)
        lib().pfsyn_gt_pose(self._h, int(k), p.ctypes.data)
        return p


def dense_map(n, seed=5):
    out = np.empty((n, 4), np.float32)
    lib().pfsyn_dense_map(int(seed), int(n), out.ctypes.data)
    return out


def voxel_map(n, leaf=0.8, seed=5, oversample=3.5):
    """configs[4]'s local map: n voxel centroids (float32 [n, 3]) of the dense synthetic block at `leaf`
    (the surf map's 0.8 m), in ascending voxel order (z, then y, then x), one point per voxel, so the
    map is a fixed point of the map update's re-voxelisation (rgbds) and keeps its size"""
    p = dense_map(int(n * oversample), seed=seed)[:, :3].astype(np.float64)
    ijk = np.floor(p / leaf).astype(np.int64)
    ijk -= ijk.min(axis=0)
    dims = ijk.max(axis=0) + 1
    key = ijk[:, 0] + dims[0] * (ijk[:, 1] + dims[1] * ijk[:, 2])
    order = np.argsort(key, kind="stable")
    ks = key[order]
    starts = np.r_[0, np.nonzero(np.diff(ks))[0] + 1]
    if starts.size < n:
        raise ValueError("the dense block has only %d voxels at leaf %g" % (starts.size, leaf))
    starts = starts[:n + 1]
    sums = np.add.reduceat(p[order[:starts[-1]]], starts[:-1], axis=0)
    cnt = np.diff(starts).astype(np.float64)
    return (sums[:n] / cnt[:n, None]).astype(np.float32)


def dense_queries(map_xyz4, nq, sigma=0.3, seed=6):
    q = np.empty((nq, 4), np.float32)
    m = np.ascontiguousarray(map_xyz4, np.float32)
    lib().pfsyn_dense_queries(int(seed), int(nq), float(sigma), m.ctypes.data, m.shape[0], q.ctypes.data)
    return q


def bpf_split(edge, surf, pillar_z=-1.0):
    """Beam / pillar / facade clouds for the BPF estimator from featureExtraction output.

    The reference feeds Odom_BPF_EstimationClass from its PCA feature classifier (include/preProcess.hpp,
    out of scope: SURVEY §8(f) rank 3). This stand-in is deterministic and keeps every feature point:
    edge points above `pillar_z` m in the sensor frame (vertical structures: poles, building corners)
    are pillars, the lower ones beams, and surf points are facades."""
    edge = np.asarray(edge, np.float32)
    up = edge[:, 2] > pillar_z
    return edge[~up].copy(), edge[up].copy(), np.asarray(surf, np.float32).copy()
