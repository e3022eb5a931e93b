"""ctypes binding of the pfref CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
See oracle/pfref.h for what is restated from the reference and where parity is unpinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "libpfref.so")

FE_STABLE_TIES = 1
FE_SQRT_DOUBLE = 2
VG_STABLE = 4
KNN_BRUTE = 8
LM_NORMAL_EQ = 16
DEV_HALFANGLE = 1024   # experiment: LM_NORMAL_EQ's SE(3) update by round 3's half-angle identities
DEV_LIBM = 512         # experiment: LM_NORMAL_EQ's SE(3) updates by libm sin / cos
COST_REVSUM = 256      # experiment: the faithful LM sums its cost in reverse order
LM_QUAD = 128          # experiment: LM_NORMAL_EQ's products and step in binary128
QR_REVSUM = 64         # experiment: the LM's Householder QR sums its rows in reverse order
LD_TRIG = 32           # experiment: the LM's sin / cos / cubes in long double (another libm's last bit)
GPU_EQUIV = FE_STABLE_TIES | VG_STABLE | LM_NORMAL_EQ


def build(force=False):
    srcs = [os.path.join(_HERE, f) for f in ("pfref_fe.cpp", "pfref_odom.cpp", "pfref_cls.cpp", "pfref_map.cpp",
                                              "pfref_dcvc.cpp", "pfref_sort.cpp", "pfref.h", "pfref_internal.h",
                                              "pfref_math.h", "Makefile")]
    newest = max(os.path.getmtime(s) for s in srcs)
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < newest:
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB


class Lidar(ctypes.Structure):
    _fields_ = [("num_lines", ctypes.c_int), ("min_distance", ctypes.c_double),
                ("max_distance", ctypes.c_double), ("scan_period", ctypes.c_double),
                ("ring_top", ctypes.c_double), ("ring_bottom", ctypes.c_double)]


class OdomParams(ctypes.Structure):
    _fields_ = [("map_resolution", ctypes.c_double), ("k_new", ctypes.c_int), ("theta_p", ctypes.c_float),
                ("theta_max", ctypes.c_int), ("weight_type", ctypes.c_double)]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("n_edge_in", "n_surf_in", "n_edge_ds", "n_surf_ds", "n_edge_map",
                                              "n_surf_map", "n_edge_res", "n_surf_res", "n_edge_valid",
                                              "n_surf_valid")] + \
               [(n, ctypes.c_int32) for n in ("outer_iterations", "lm_iterations", "map_too_small", "status")] + \
               [(n, ctypes.c_double) for n in ("t_downsample", "t_tree", "t_assoc", "t_solve", "t_mapupdate")] + \
               [(n, ctypes.c_int64 * 3) for n in ("n_in", "n_ds", "n_map", "n_res", "n_valid")]

    def as_dict(self):
        d = {}
        for f in self._fields_:
            v = getattr(self, f[0])
            d[f[0]] = list(v) if f[0] in ("n_in", "n_ds", "n_map", "n_res", "n_valid") else v
        return d


_lib = None
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t


class ClsParams(ctypes.Structure):
    """groundSeg / nongroundExtract parameters (include/preProcess.hpp:575-605, :703-715)."""
    _fields_ = [("ground_filter", ctypes.c_int), ("gf_min_grid_pts", ctypes.c_int),
                ("gf_grid_res", ctypes.c_float), ("gf_max_height_diff", ctypes.c_float),
                ("gf_neighbor_height_diff", ctypes.c_float), ("gf_max_ground_height", ctypes.c_float),
                ("gf_min_ground_height", ctypes.c_float), ("radius", ctypes.c_float), ("k", ctypes.c_int),
                ("k_min", ctypes.c_int), ("edge_thre", ctypes.c_float), ("planar_thre", ctypes.c_float),
                ("linear_vsin_high", ctypes.c_float), ("linear_vsin_low", ctypes.c_float),
                ("planar_vsin_low", ctypes.c_float), ("beam_h_max", ctypes.c_float), ("beam_h_min", ctypes.c_float)]


def cls_params(**kw):
    p = ClsParams()
    lib().pfref_cls_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class DcvcParams(ctypes.Structure):
    """curvedVoxel parameters (config/config.yaml:7-8, 49-54)."""
    _fields_ = [("start_r", ctypes.c_double), ("delta_r", ctypes.c_double), ("delta_p", ctypes.c_double),
                ("delta_a", ctypes.c_double), ("min_seg", ctypes.c_int), ("min_range", ctypes.c_double),
                ("max_range", ctypes.c_double)]


def dcvc_params(**kw):
    p = DcvcParams()
    lib().pfref_dcvc_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def dcvc(xyz, params=None, first_frame=False, components=False):
    """curvedVoxel::run: (input indices of the kept points in the published order, per-point cluster
    rank 1.. or 0 for dropped points). components=False: the serial reading of the reference;
    True: connected components of the same voxel neighbourhood (the device's reading)."""
    a = np.ascontiguousarray(xyz, dtype=np.float32)
    n = a.shape[0]
    p = params or dcvc_params()
    idx = np.empty(max(n, 1), np.int32)
    lab = np.empty(max(n, 1), np.int32)
    k = ctypes.c_size_t()
    rc = lib().pfref_dcvc_mode(a.ctypes.data, n, 4 * a.shape[1], ctypes.byref(p), int(bool(first_frame)),
                               int(bool(components)), idx.ctypes.data, ctypes.byref(k), lab.ctypes.data)
    assert rc == 0
    return idx[:k.value].copy(), lab[:n].copy()


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        L = _lib
        L.pfref_feature_extraction.argtypes = [ctypes.POINTER(Lidar), ctypes.c_int, _vp, _sz, _vp,
                                               ctypes.POINTER(_sz), _vp, ctypes.POINTER(_sz), _sz]
        L.pfref_voxel_grid.argtypes = [_vp, _sz, ctypes.c_float, ctypes.c_int, _vp, ctypes.POINTER(_sz)]
        L.pfref_rgbds.argtypes = [_vp, _sz, ctypes.c_float, ctypes.c_int, _vp, ctypes.POINTER(_sz)]
        L.pfref_knn.argtypes = [_vp, _sz, _vp, _sz, ctypes.c_int, ctypes.c_int, _vp, _vp]
        L.pfref_knn_cellpop.argtypes = [_vp, _sz, _vp, _sz]
        L.pfref_knn_cellpop.restype = ctypes.c_ulonglong
        L.pfref_eigen_sym3.argtypes = [_vp, _vp, _vp]
        L.pfref_plane_fit.argtypes = [_vp, _vp]
        L.pfref_se3_plus.argtypes = [_vp, _vp, _vp]
        L.pfref_se3_plus_half.argtypes = [_vp, _vp, _vp]
        L.pfref_det_sincos.argtypes = [ctypes.c_double, _vp, _vp]
        L.pfref_rotation_polar.argtypes = [_vp, _vp]
        L.pfref_edge_eval.argtypes = [_vp, _vp, _vp, _vp, ctypes.c_double, _vp]
        L.pfref_edge_eval.restype = ctypes.c_double
        L.pfref_surf_eval.argtypes = [_vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _vp]
        L.pfref_surf_eval.restype = ctypes.c_double
        L.pfref_odom_create.argtypes = [ctypes.POINTER(Lidar), ctypes.POINTER(OdomParams), ctypes.c_int]
        L.pfref_odom_create.restype = _vp
        L.pfref_odom_destroy.argtypes = [_vp]
        L.pfref_odom_init_map.argtypes = [_vp, _vp, _sz, _vp, _sz]
        L.pfref_odom_update.argtypes = [_vp, _vp, _sz, _vp, _sz, _vp]
        L.pfref_odom_get_pose.argtypes = [_vp, _vp]
        L.pfref_odom_get_map.argtypes = [_vp, ctypes.c_int, _vp, _vp, _sz, ctypes.POINTER(_sz)]
        L.pfref_odom_set_map.argtypes = [_vp, ctypes.c_int, _vp, _vp, _sz]
        L.pfref_odom_get_stats.argtypes = [_vp, ctypes.POINTER(Stats)]
        L.pfref_odom_frame.argtypes = [_vp, ctypes.POINTER(Lidar), _vp, _sz, _vp]
        L.pfref_odom_set_state.argtypes = [_vp, _vp, _vp]
        L.pfref_odom_set_opt_count.argtypes = [_vp, ctypes.c_int]
        L.pfref_bpf_create.argtypes = [ctypes.POINTER(Lidar), ctypes.POINTER(OdomParams), ctypes.c_int]
        L.pfref_bpf_create.restype = _vp
        L.pfref_odom_classes.argtypes = [_vp]
        L.pfref_odom_init_map_n.argtypes = [_vp, _vp, _vp]
        L.pfref_odom_update_n.argtypes = [_vp, _vp, _vp, _vp]
        L.pfref_cls_default_params.argtypes = [ctypes.POINTER(ClsParams)]
        L.pfref_ground_seg.argtypes = [_vp, _sz, _sz, ctypes.POINTER(ClsParams), _vp, ctypes.POINTER(_sz), _vp,
                                       ctypes.POINTER(_sz)]
        L.pfref_pca_classify.argtypes = [_vp, _sz, _sz, ctypes.POINTER(ClsParams), _vp, _vp]
        L.pfref_pca_classify_normals.argtypes = [_vp, _sz, _sz, ctypes.POINTER(ClsParams), _vp, _vp, _vp]
        L.pfref_dcvc.argtypes = [_vp, _sz, _sz, ctypes.POINTER(DcvcParams), ctypes.c_int, _vp, ctypes.POINTER(_sz), _vp]
        L.pfref_dcvc_default_params.argtypes = [ctypes.POINTER(DcvcParams)]
        L.pfref_dcvc_mode.argtypes = [_vp, _sz, _sz, ctypes.POINTER(DcvcParams), ctypes.c_int, ctypes.c_int, _vp,
                                      ctypes.POINTER(_sz), _vp]
        L.pfref_bpf_preprocess_dcvc.argtypes = [_vp, _sz, _sz, ctypes.POINTER(ClsParams), ctypes.POINTER(DcvcParams),
                                                ctypes.c_int, ctypes.c_int] + [_vp, ctypes.POINTER(_sz)] * 4
        L.pfref_map_create.argtypes = [ctypes.c_double]
        L.pfref_map_create.restype = _vp
        L.pfref_map_destroy.argtypes = [_vp]
        L.pfref_map_update.argtypes = [_vp, _vp, _sz, _sz, _vp]
        L.pfref_map_get.argtypes = [_vp, _vp, _sz, ctypes.POINTER(_sz)]
        L.pfref_bpf_preprocess.argtypes = [_vp, _sz, _sz, ctypes.POINTER(ClsParams)] + \
            [_vp, ctypes.POINTER(_sz)] * 4
        L.pfref_std_sort_perm.argtypes = [_vp, _sz, _vp]
        L.pfref_introsort_literal.argtypes = [_vp, _sz, ctypes.c_int, _vp]
        L.pfref_introsort_levels.argtypes = [_vp, _sz, ctypes.c_int, _vp]
    return _lib


def _f32(a, cols=4):
    a = np.ascontiguousarray(a, dtype=np.float32)
    assert a.ndim == 2 and a.shape[1] == cols
    return a


def make_lidar(num_lines=64, min_distance=3.0, max_distance=90.0, scan_period=0.1, ring_model=None):
    """ring_model=(top_deg, bottom_deg): the linear beam-model extension (S128)"""
    top, bottom = ring_model if ring_model else (0.0, 0.0)
    return Lidar(int(num_lines), float(min_distance), float(max_distance), float(scan_period), float(top),
                 float(bottom))


def feature_extraction(xyzi, lidar, opts=0):
    x = _f32(xyzi)
    n = x.shape[0]
    edge = np.empty((max(n, 1), 4), np.float32)
    surf = np.empty((max(n, 1), 4), np.float32)
    ne, ns = _sz(), _sz()
    rc = lib().pfref_feature_extraction(ctypes.byref(lidar), int(opts), x.ctypes.data, n, edge.ctypes.data,
                                        ctypes.byref(ne), surf.ctypes.data, ctypes.byref(ns), max(n, 1))
    if rc != 0:
        raise RuntimeError("pfref_feature_extraction failed")
    return edge[:ne.value].copy(), surf[:ns.value].copy()


def pack_rgb(xyz, r=None, g=None, b=None):
    n = xyz.shape[0]
    out = np.zeros((n, 4), np.float32)
    out[:, :3] = xyz[:, :3]
    r = np.zeros(n, np.uint32) if r is None else np.asarray(r, np.uint32)
    g = np.zeros(n, np.uint32) if g is None else np.asarray(g, np.uint32)
    b = np.zeros(n, np.uint32) if b is None else np.asarray(b, np.uint32)
    out[:, 3] = ((r << 16) | (g << 8) | b).view(np.float32)
    return out


def unpack_rgb(pts):
    rgb = np.ascontiguousarray(pts[:, 3]).view(np.uint32)
    return pts[:, :3].copy(), ((rgb >> 16) & 255).astype(np.uint8), ((rgb >> 8) & 255).astype(np.uint8)


def voxel_grid(pts, leaf, opts=0):
    p = _f32(pts)
    out = np.empty_like(p) if p.shape[0] else np.empty((1, 4), np.float32)
    n = _sz()
    lib().pfref_voxel_grid(p.ctypes.data, p.shape[0], float(leaf), int(opts), out.ctypes.data, ctypes.byref(n))
    return out[:n.value].copy()


def rgbds(pts, leaf, opts=0):
    p = _f32(pts)
    out = np.empty_like(p) if p.shape[0] else np.empty((1, 4), np.float32)
    n = _sz()
    lib().pfref_rgbds(p.ctypes.data, p.shape[0], float(leaf), int(opts), out.ctypes.data, ctypes.byref(n))
    return out[:n.value].copy()


def knn_cellpop(map_pts, queries):
    """sum over the queries of |C(q)| (map points in the 27 1 m cells around q)"""
    m = _f32(map_pts)
    q = _f32(queries)
    return int(lib().pfref_knn_cellpop(m.ctypes.data, m.shape[0], q.ctypes.data, q.shape[0]))


def knn(map_pts, queries, k=5, opts=0):
    m = _f32(map_pts)
    q = _f32(queries)
    idx = np.empty((q.shape[0], k), np.int32)
    d2 = np.empty((q.shape[0], k), np.float32)
    rc = lib().pfref_knn(m.ctypes.data, m.shape[0], q.ctypes.data, q.shape[0], int(k), int(opts),
                         idx.ctypes.data, d2.ctypes.data)
    if rc != 0:
        raise RuntimeError("pfref_knn failed")
    return idx, d2


def sort_perm(keys, how="std", depth=-1):
    """the permutation of (key, index) pairs sorted by key only: how = "std" (libstdc++ std::sort itself,
    as PCL's VoxelGrid and rgbds call it), "literal" (its line-by-line restatement, depth limit
    settable), "levels" (the level-synchronous form of the device's reference-tie-order mode)"""
    k = np.ascontiguousarray(keys, np.uint32)
    out = np.empty(max(k.size, 1), np.uint32)
    if how == "std":
        lib().pfref_std_sort_perm(k.ctypes.data, k.size, out.ctypes.data)
    elif how == "literal":
        lib().pfref_introsort_literal(k.ctypes.data, k.size, int(depth), out.ctypes.data)
    else:
        lib().pfref_introsort_levels(k.ctypes.data, k.size, int(depth), out.ctypes.data)
    return out[:k.size].copy()


def eigen_sym3(a6):
    a = np.ascontiguousarray(a6, np.float64)
    ev = np.empty(3)
    vec = np.empty(9)
    lib().pfref_eigen_sym3(a.ctypes.data, ev.ctypes.data, vec.ctypes.data)
    return ev, vec.reshape(3, 3).T  # columns are eigenvectors


def plane_fit(A):
    A = np.ascontiguousarray(A, np.float64).reshape(5, 3)
    n = np.empty(3)
    lib().pfref_plane_fit(A.ctypes.data, n.ctypes.data)
    return n


def se3_plus(x, delta):
    x = np.ascontiguousarray(x, np.float64)
    d = np.ascontiguousarray(delta, np.float64)
    out = np.empty(7)
    lib().pfref_se3_plus(x.ctypes.data, d.ctypes.data, out.ctypes.data)
    return out


def se3_plus_half(x, delta):
    """the GPU_EQUIV SE(3) update (pf_geom.h se3_exp: the source's form on the deterministic sincos)"""
    x = np.ascontiguousarray(x, np.float64)
    d = np.ascontiguousarray(delta, np.float64)
    out = np.empty(7)
    lib().pfref_se3_plus_half(x.ctypes.data, d.ctypes.data, out.ctypes.data)
    return out


def det_sincos(x):
    s = np.empty(1)
    c = np.empty(1)
    lib().pfref_det_sincos(float(x), s.ctypes.data, c.ctypes.data)
    return float(s[0]), float(c[0])


def rotation_polar(m):
    m = np.ascontiguousarray(m, np.float64).reshape(3, 3)
    out = np.empty((3, 3))
    lib().pfref_rotation_polar(m.ctypes.data, out.ctypes.data)
    return out


def edge_eval(x, cur, a, b, w=0.0):
    J = np.empty(7)
    arr = [np.ascontiguousarray(v, np.float64) for v in (x, cur, a, b)]
    r = lib().pfref_edge_eval(*(v.ctypes.data for v in arr), float(w), J.ctypes.data)
    return r, J


def surf_eval(x, cur, n, d, w=0.0):
    J = np.empty(7)
    arr = [np.ascontiguousarray(v, np.float64) for v in (x, cur, n)]
    r = lib().pfref_surf_eval(*(v.ctypes.data for v in arr), float(d), float(w), J.ctypes.data)
    return r, J


class Odom:
    """Odom_ES_EstimationClass restated on the CPU."""
    _create = "pfref_odom_create"

    def __init__(self, lidar=None, map_resolution=0.4, k_new=0, theta_p=0.4, theta_max=75, weight_type=0,
                 opts=0):
        self.lidar = lidar if lidar is not None else make_lidar()
        self.params = OdomParams(float(map_resolution), int(k_new), float(theta_p), int(theta_max),
                                 float(weight_type))
        self._h = getattr(lib(), self._create)(ctypes.byref(self.lidar), ctypes.byref(self.params), int(opts))
        if not self._h:
            raise ValueError("invalid odometry parameters")
        self.inited = False

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pfref_odom_destroy(self._h)
            self._h = None

    def init_map(self, edge, surf):
        e, s = _f32(edge), _f32(surf)
        lib().pfref_odom_init_map(self._h, e.ctypes.data, e.shape[0], s.ctypes.data, s.shape[0])
        self.inited = True

    def update(self, edge, surf):
        e, s = _f32(edge), _f32(surf)
        pose = np.empty(7)
        lib().pfref_odom_update(self._h, e.ctypes.data, e.shape[0], s.ctypes.data, s.shape[0], pose.ctypes.data)
        return pose

    def frame(self, xyzi):
        x = _f32(xyzi)
        pose = np.empty(7)
        rc = lib().pfref_odom_frame(self._h, ctypes.byref(self.lidar), x.ctypes.data, x.shape[0], pose.ctypes.data)
        if rc != 0:
            raise RuntimeError("pfref_odom_frame failed")
        self.inited = True
        return pose

    def pose(self):
        p = np.empty(7)
        lib().pfref_odom_get_pose(self._h, p.ctypes.data)
        return p

    def get_map(self, which):
        n = _sz()
        lib().pfref_odom_get_map(self._h, int(which), None, None, 0, ctypes.byref(n))
        xyz = np.empty((max(n.value, 1), 3), np.float32)
        rg = np.empty((max(n.value, 1), 2), np.uint8)
        lib().pfref_odom_get_map(self._h, int(which), xyz.ctypes.data, rg.ctypes.data, n.value, ctypes.byref(n))
        return xyz[:n.value].copy(), rg[:n.value].copy()

    def set_map(self, which, xyz, rg):
        xyz = np.ascontiguousarray(xyz, np.float32)
        rg = np.ascontiguousarray(rg, np.uint8)
        lib().pfref_odom_set_map(self._h, int(which), xyz.ctypes.data, rg.ctypes.data, xyz.shape[0])

    def set_state(self, odom_pose, last_pose=None):
        a = np.ascontiguousarray(odom_pose, np.float64)
        b = np.ascontiguousarray(odom_pose if last_pose is None else last_pose, np.float64)
        lib().pfref_odom_set_state(self._h, a.ctypes.data, b.ctypes.data)

    def set_opt_count(self, n):
        lib().pfref_odom_set_opt_count(self._h, int(n))

    def stats(self):
        s = Stats()
        lib().pfref_odom_get_stats(self._h, ctypes.byref(s))
        return s.as_dict()


def _clouds(clouds):
    arrs = [_f32(c) for c in clouds]
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    ns = (ctypes.c_size_t * len(arrs))(*[a.shape[0] for a in arrs])
    return arrs, ptrs, ns


class OdomBPF(Odom):
    """Odom_BPF_EstimationClass restated on the CPU (src/odomEstimationClass.cpp:649-1306): map
    classes 0 beam, 1 pillar (lines, leaf r) and 2 facade (plane, leaf 2r)."""
    _create = "pfref_bpf_create"

    def init_map(self, beam, pillar, facade):
        arrs, ptrs, ns = _clouds((beam, pillar, facade))
        lib().pfref_odom_init_map_n(self._h, ptrs, ns)
        self.inited = True

    def update(self, beam, pillar, facade):
        arrs, ptrs, ns = _clouds((beam, pillar, facade))
        pose = np.empty(7)
        lib().pfref_odom_update_n(self._h, ptrs, ns, pose.ctypes.data)
        return pose

    def frame(self, xyzi):
        raise NotImplementedError("the BPF estimator takes classified beam / pillar / facade clouds")


# ---- BPF front end (groundSeg + nongroundExtract; include/preProcess.hpp) ----

def ground_seg(xyz, params=None):
    """(ground, unground) input indices in the reference's push order."""
    a = np.ascontiguousarray(xyz, dtype=np.float32)
    n = a.shape[0]
    p = params or cls_params()
    g = np.empty(max(n, 1), np.int32)
    u = np.empty(max(n, 1), np.int32)
    ng, nu = ctypes.c_size_t(), ctypes.c_size_t()
    rc = lib().pfref_ground_seg(a.ctypes.data, n, 4 * a.shape[1], ctypes.byref(p), g.ctypes.data, ctypes.byref(ng),
                                u.ctypes.data, ctypes.byref(nu))
    assert rc == 0
    return g[:ng.value].copy(), u[:nu.value].copy()


def pca_classify(xyz, params=None, normals=False):
    """(class per point: 0 none / 1 pillar / 2 beam / 3 facade, neighbour count per point[, the normal
    assign_normal writes: [n, 4] float32])."""
    a = np.ascontiguousarray(xyz, dtype=np.float32)
    n = a.shape[0]
    p = params or cls_params()
    cls = np.empty(max(n, 1), np.uint8)
    num = np.empty(max(n, 1), np.int32)
    nrm = np.empty((max(n, 1), 4), np.float32)
    rc = lib().pfref_pca_classify_normals(a.ctypes.data, n, 4 * a.shape[1], ctypes.byref(p), cls.ctypes.data,
                                          num.ctypes.data, nrm.ctypes.data if normals else None)
    assert rc == 0
    if normals:
        return cls[:n].copy(), num[:n].copy(), nrm[:n].copy()
    return cls[:n].copy(), num[:n].copy()


def bpf_preprocess(xyz, params=None, dcvc=None, first_frame=False, components=False):
    """additionNode's chain: dict of beam / pillar / facade / ground input-index arrays. dcvc: DcvcParams
    to run curvedVoxel between ground_seg and featureExtract (curvedfilter on); components: its
    connected-components reading (the device's) instead of the serial one."""
    a = np.ascontiguousarray(xyz, dtype=np.float32)
    n = a.shape[0]
    p = params or cls_params()
    bufs = [np.empty(max(n, 1), np.int32) for _ in range(4)]
    cnt = [ctypes.c_size_t() for _ in range(4)]
    args = []
    for b, c in zip(bufs, cnt):
        args += [b.ctypes.data, ctypes.byref(c)]
    if dcvc is not None:
        rc = lib().pfref_bpf_preprocess_dcvc(a.ctypes.data, n, 4 * a.shape[1], ctypes.byref(p), ctypes.byref(dcvc),
                                             int(bool(first_frame)), int(bool(components)), *args)
    else:
        rc = lib().pfref_bpf_preprocess(a.ctypes.data, n, 4 * a.shape[1], ctypes.byref(p), *args)
    assert rc == 0
    return {k: b[:c.value].copy() for k, b, c in zip(("beam", "pillar", "facade", "ground"), bufs, cnt)}


class GlobalMap:
    """LaserMappingClass restated (src/laserMappingClass.cpp): update(xyzi, pose7), get() -> (n, 4)."""

    def __init__(self, map_resolution=0.4):
        self._h = lib().pfref_map_create(float(map_resolution))

    def update(self, xyzi, pose7):
        a = np.ascontiguousarray(xyzi, dtype=np.float32)
        pose = np.ascontiguousarray(pose7, dtype=np.float64)
        return lib().pfref_map_update(self._h, a.ctypes.data, a.shape[0], 4 * a.shape[1], pose.ctypes.data)

    def get(self):
        n = ctypes.c_size_t()
        lib().pfref_map_get(self._h, None, 0, ctypes.byref(n))
        out = np.empty((max(n.value, 1), 4), np.float32)
        lib().pfref_map_get(self._h, out.ctypes.data, n.value, ctypes.byref(n))
        return out[:n.value].copy()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pfref_map_destroy(self._h)
            self._h = None
