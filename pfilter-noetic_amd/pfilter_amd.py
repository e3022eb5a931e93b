"""ctypes binding of libpfilter_hip.so (include/pfilter_hip.h) for tests and bench.py.

Mirrors the reference classes used on the hot path, same method names and argument meaning:
  LaserProcessingClass.init / featureExtraction          include/laserProcessingClass.h:36-37
  Odom_ES_EstimationClass.init / initMapWithPoints /
      updatePointsToMap / getMap, members odom,
      laserCloudCornerMap, laserCloudSurfMap              include/odomEstimationClass.h:140-152
Point clouds are numpy float32 arrays [n, 4] (x, y, z, intensity).

There is no CPU fallback: if the HIP library is missing or fails to load, this module raises.
If PyTorch is also used in the process, import torch BEFORE this module so that one HIP runtime
(torch's, same SONAME) serves both.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PFILTER_HIP_LIB: development override (tools/ variant builds); the in-tree build otherwise
LIB_PATH = os.environ.get("PFILTER_HIP_LIB") or os.path.join(_HERE, "libpfilter_hip.so")

PF_OK = 0
PF_W_MAP_TOO_SMALL = 1
PF_W_FEW_CORRESPONDENCES = 2
PF_EINVAL = -1
PF_EHIP = -2
PF_ENOMEM = -3
PF_ECAPACITY = -4
PF_EUNSUPPORTED = -5


class PFError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__("%s failed with status %d" % (fn, code))
        self.code = code


def build():
    """Compile libpfilter_hip.so for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", "-j8", "-C", _HERE])
    return LIB_PATH


class LidarParams(ctypes.Structure):
    _fields_ = [("num_lines", ctypes.c_int), ("min_dist", ctypes.c_double), ("max_dist", ctypes.c_double),
                ("scan_period", ctypes.c_double)]


class OdomParams(ctypes.Structure):
    _fields_ = [("map_res", ctypes.c_double), ("k_new", ctypes.c_int), ("theta_p", ctypes.c_float),
                ("theta_max", ctypes.c_int), ("weight_type", ctypes.c_int)]


class OdomStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("n_edge_in", "n_surf_in", "n_edge_ds", "n_surf_ds", "n_edge_map",
                                              "n_surf_map", "n_edge_res", "n_surf_res", "n_edge_valid",
                                              "n_surf_valid")] + \
               [(n, ctypes.c_int32) for n in ("outer_iterations", "lm_iterations", "map_too_small", "status")] + \
               [(n, ctypes.c_int64 * 3) for n in ("n_in", "n_ds", "n_map", "n_res", "n_valid")] + \
               [("errors", ctypes.c_int32), ("pad_", ctypes.c_int32)]

    def as_dict(self):
        d = {}
        for f in self._fields_:
            v = getattr(self, f[0])
            d[f[0]] = list(v) if f[0] in ("n_in", "n_ds", "n_map", "n_res", "n_valid") else v
        return d


class DcvcParams(ctypes.Structure):
    """pf_dcvc_params: curvedVoxel (config/config.yaml:7-8, 49-54)."""
    _fields_ = [("start_r", ctypes.c_double), ("delta_r", ctypes.c_double), ("delta_p", ctypes.c_double),
                ("delta_a", ctypes.c_double), ("min_seg", ctypes.c_int), ("min_range", ctypes.c_double),
                ("max_range", ctypes.c_double)]


def dcvc_params(**kw):
    p = DcvcParams()
    lib().pf_dcvc_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class Dcvc:
    """curvedVoxel on the device (pf_dcvc_*): run(xyz) -> (kept input indices in the published order,
    per-point cluster rank 1.. / 0). The first call of a handle (or after reset) is a first frame."""

    def __init__(self, max_points=300000, device=0, **params):
        self._h = None
        h = _vp()
        _check("pf_dcvc_create", lib().pf_dcvc_create(ctypes.byref(dcvc_params(**params)), device, max_points,
                                                      ctypes.byref(h)), allow_warn=False)
        self._h = h

    def run(self, xyz):
        a = np.ascontiguousarray(xyz, dtype=np.float32)
        n = a.shape[0]
        idx = np.empty(max(n, 1), np.int32)
        lab = np.empty(max(n, 1), np.int32)
        k = _sz()
        _check("pf_dcvc_run", lib().pf_dcvc_run(self._h, a.ctypes.data, n, 4 * a.shape[1], idx.ctypes.data,
                                                ctypes.byref(k), lab.ctypes.data, max(n, 1)), allow_warn=False)
        return idx[:k.value].copy(), lab[:n].copy()

    def reset(self):
        _check("pf_dcvc_reset", lib().pf_dcvc_reset(self._h), allow_warn=False)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pf_dcvc_destroy(self._h)
            self._h = None


class ClsParams(ctypes.Structure):
    """pf_cls_params: groundSeg / nongroundExtract members (include/preProcess.hpp:575-605, :703-715)."""
    _fields_ = [("ground_filter", ctypes.c_int), ("gf_min_grid_pts", ctypes.c_int),
                ("gf_grid_res", ctypes.c_float), ("gf_max_height_diff", ctypes.c_float),
                ("gf_neighbor_height_diff", ctypes.c_float), ("gf_max_ground_height", ctypes.c_float),
                ("gf_min_ground_height", ctypes.c_float), ("radius", ctypes.c_float), ("k", ctypes.c_int),
                ("k_min", ctypes.c_int), ("edge_thre", ctypes.c_float), ("planar_thre", ctypes.c_float),
                ("linear_vsin_high", ctypes.c_float), ("linear_vsin_low", ctypes.c_float),
                ("planar_vsin_low", ctypes.c_float), ("beam_h_max", ctypes.c_float), ("beam_h_min", ctypes.c_float)]


EXPORTS = ["pf_fe_create", "pf_fe_destroy", "pf_fe_extract", "pf_odom_create", "pf_odom_destroy",
           "pf_odom_init_map", "pf_odom_update", "pf_odom_get_pose", "pf_odom_get_map", "pf_odom_set_map",
           "pf_odom_get_stats", "pf_odom_frame_device", "pf_odom_frame_host", "pf_odom_sync", "pf_odom_poses",
           "pf_odom_set_graph", "pf_device_count", "pf_dev_malloc", "pf_dev_free", "pf_memcpy_h2d",
           "pf_memcpy_d2h", "pf_knn_create", "pf_knn_destroy", "pf_knn_set_map", "pf_knn_query", "pf_knn_bench",
           "pf_bpf_create", "pf_bpf_init_map", "pf_bpf_update", "pf_bpf_frame_device", "pf_odom_classes",
           "pf_odom_reset", "pf_cls_default_params", "pf_cls_create", "pf_cls_destroy", "pf_cls_extract",
           "pf_cls_classify", "pf_cls_ground_seg", "pf_bpf_set_front_end", "pf_bpf_frame_scan_device", "pf_map_create", "pf_map_destroy", "pf_map_update",
           "pf_map_update_device", "pf_map_update_mat", "pf_map_get", "pf_odom_set_stage_a_reserve",
           "pf_fe_set_ring_model", "pf_odom_set_ring_model", "pf_odom_get_state", "pf_odom_snapshot",
           "pf_odom_restore", "pf_odom_set_map_export", "pf_odom_map_export", "pf_odom_set_stage_timing",
           "pf_odom_stage_times", "pf_odom_set_state", "pf_cls_normals", "pf_dcvc_default_params",
           "pf_dcvc_create", "pf_dcvc_destroy", "pf_dcvc_run", "pf_dcvc_reset", "pf_cls_set_dcvc", "pf_bpf_set_dcvc",
           "pf_host_alloc", "pf_host_free", "pf_odom_set_tie_order", "pf_odom_probe_assoc",
           "pf_odom_merge_stats", "pf_bpf_set_front_lanes", "pf_dcvc_reserve", "pf_fe_set_tie_order"]

_lib = None
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_i = ctypes.c_int


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError("libpfilter_hip.so not built (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    L.pf_fe_create.argtypes = [ctypes.POINTER(LidarParams), _i, _sz, ctypes.POINTER(_vp)]
    L.pf_fe_destroy.argtypes = [_vp]
    L.pf_fe_extract.argtypes = [_vp, _vp, _sz, _sz, _vp, ctypes.POINTER(_sz), _vp, ctypes.POINTER(_sz), _sz]
    L.pf_odom_create.argtypes = [ctypes.POINTER(LidarParams), ctypes.POINTER(OdomParams), _i, _sz, _sz,
                                 ctypes.POINTER(_vp)]
    L.pf_odom_destroy.argtypes = [_vp]
    L.pf_odom_init_map.argtypes = [_vp, _vp, _sz, _sz, _vp, _sz, _sz]
    L.pf_odom_update.argtypes = [_vp, _vp, _sz, _sz, _vp, _sz, _sz, _vp]
    L.pf_odom_get_pose.argtypes = [_vp, _vp]
    L.pf_odom_get_map.argtypes = [_vp, _i, _vp, _vp, _sz, ctypes.POINTER(_sz)]
    L.pf_odom_set_map.argtypes = [_vp, _i, _vp, _vp, _sz]
    L.pf_odom_get_stats.argtypes = [_vp, ctypes.POINTER(OdomStats)]
    L.pf_odom_frame_device.argtypes = [_vp, _vp, _sz, _vp]
    L.pf_odom_frame_host.argtypes = [_vp, _vp, _sz, _sz, _vp]
    L.pf_odom_sync.argtypes = [_vp]
    L.pf_odom_poses.argtypes = [_vp, _vp, _sz, ctypes.POINTER(_sz)]
    L.pf_odom_set_graph.argtypes = [_vp, _i]
    L.pf_odom_set_stage_timing.argtypes = [_vp, _i]
    L.pf_odom_set_state.argtypes = [_vp, _vp, _vp, _i]
    L.pf_cls_normals.argtypes = [_vp, _vp, _sz]
    L.pf_dcvc_default_params.argtypes = [ctypes.POINTER(DcvcParams)]
    L.pf_dcvc_create.argtypes = [ctypes.POINTER(DcvcParams), _i, _sz, ctypes.POINTER(_vp)]
    L.pf_dcvc_destroy.argtypes = [_vp]
    L.pf_dcvc_run.argtypes = [_vp, _vp, _sz, _sz, _vp, ctypes.POINTER(_sz), _vp, _sz]
    L.pf_dcvc_reset.argtypes = [_vp]
    L.pf_cls_set_dcvc.argtypes = [_vp, ctypes.POINTER(DcvcParams)]
    L.pf_bpf_set_dcvc.argtypes = [_vp, ctypes.POINTER(DcvcParams)]
    L.pf_bpf_set_front_lanes.argtypes = [_vp, ctypes.c_int]
    L.pf_odom_stage_times.argtypes = [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(_sz)]
    if hasattr(L, "pf_odom_set_stage_a_reserve"):
        L.pf_odom_set_stage_a_reserve.argtypes = [_vp, _i]
    L.pf_fe_set_ring_model.argtypes = [_vp, ctypes.c_double, ctypes.c_double]
    L.pf_fe_set_tie_order.argtypes = [_vp, _i]
    L.pf_odom_set_ring_model.argtypes = [_vp, ctypes.c_double, ctypes.c_double]
    L.pf_odom_get_state.argtypes = [_vp, _vp, _vp, ctypes.POINTER(_i)]
    L.pf_odom_snapshot.argtypes = [_vp, _vp, _sz, ctypes.POINTER(_sz)]
    L.pf_odom_restore.argtypes = [_vp, _vp, _sz]
    L.pf_odom_set_map_export.argtypes = [_vp, _i]
    L.pf_odom_map_export.argtypes = [_vp, _i, ctypes.POINTER(ctypes.POINTER(ctypes.c_float)), ctypes.POINTER(_sz)]
    L.pf_device_count.argtypes = [ctypes.POINTER(_i)]
    L.pf_dev_malloc.argtypes = [_i, _sz, ctypes.POINTER(_vp)]
    L.pf_dev_free.argtypes = [_i, _vp]
    L.pf_memcpy_h2d.argtypes = [_i, _vp, _vp, _sz]
    L.pf_memcpy_d2h.argtypes = [_i, _vp, _vp, _sz]
    L.pf_odom_set_tie_order.argtypes = [_vp, _i]
    L.pf_odom_probe_assoc.argtypes = [_vp, _i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(_sz), _vp, _sz]
    L.pf_odom_merge_stats.argtypes = [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i)]
    L.pf_dev_tie_sort.argtypes = [_i, _vp, _sz, _vp, ctypes.POINTER(_sz)]
    L.pf_dev_tie_sort2.argtypes = [_i, _vp, _sz, _i, _i, _vp, ctypes.POINTER(_sz)]
    L.pf_host_alloc.argtypes = [_sz, ctypes.POINTER(_vp)]
    L.pf_host_free.argtypes = [_vp]
    L.pf_knn_create.argtypes = [_i, _sz, _sz, ctypes.POINTER(_vp)]
    L.pf_knn_destroy.argtypes = [_vp]
    L.pf_knn_set_map.argtypes = [_vp, _vp, _sz]
    L.pf_knn_query.argtypes = [_vp, _vp, _sz, _vp, _vp]
    L.pf_knn_bench.argtypes = [_vp, _i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    if hasattr(L, "pf_bpf_create"):     # (absent only in an older library loaded for an A/B run)
        L.pf_bpf_create.argtypes = [ctypes.POINTER(LidarParams), ctypes.POINTER(OdomParams), _i, _sz, _sz,
                                    ctypes.POINTER(_vp)]
        L.pf_bpf_init_map.argtypes = [_vp, _vp, _sz, _sz, _vp, _sz, _sz, _vp, _sz, _sz]
        L.pf_bpf_update.argtypes = [_vp, _vp, _sz, _sz, _vp, _sz, _sz, _vp, _sz, _sz, _vp]
        L.pf_bpf_frame_device.argtypes = [_vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp]
        L.pf_odom_classes.argtypes = [_vp]
        L.pf_odom_reset.argtypes = [_vp]
    if hasattr(L, "pf_cls_create"):
        L.pf_cls_default_params.argtypes = [ctypes.POINTER(ClsParams)]
        L.pf_cls_default_params.restype = None
        L.pf_cls_create.argtypes = [ctypes.POINTER(ClsParams), _i, _sz, ctypes.POINTER(_vp)]
        L.pf_cls_destroy.argtypes = [_vp]
        L.pf_cls_extract.argtypes = [_vp, _vp, _sz, _sz] + [_vp, ctypes.POINTER(_sz)] * 4 + [_sz]
        L.pf_cls_classify.argtypes = [_vp, _vp, _sz, _sz, _vp, _vp]
        L.pf_cls_ground_seg.argtypes = [_vp, _vp, _sz, _sz, _vp, ctypes.POINTER(_sz), _vp, ctypes.POINTER(_sz), _sz]
        L.pf_bpf_set_front_end.argtypes = [_vp, ctypes.POINTER(ClsParams)]
    if hasattr(L, "pf_map_create"):
        L.pf_map_create.argtypes = [ctypes.c_double, _i, _sz, _sz, ctypes.POINTER(_vp)]
        L.pf_map_destroy.argtypes = [_vp]
        L.pf_map_update.argtypes = [_vp, _vp, _sz, _sz, _vp]
        L.pf_map_update_device.argtypes = [_vp, _vp, _sz, _vp]
        L.pf_map_update_mat.argtypes = [_vp, _vp, _sz, _sz, _vp]
        L.pf_map_get.argtypes = [_vp, _vp, _sz, ctypes.POINTER(_sz)]
        L.pf_bpf_frame_scan_device.argtypes = [_vp, _vp, _sz, _vp]
    _lib = L
    return L


def dev_errors(h):
    """development: the sticky device error words of a handle at their last report (ErrWord order)"""
    out = (ctypes.c_int * 8)()
    lib().pf_dev_errors(ctypes.c_void_p(h), out, 8)
    return list(out)


def _check(fn, rc, allow_warn=True):
    if rc < 0 or (rc > 0 and not allow_warn):
        raise PFError(fn, rc)
    return rc


def _f32x4(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] != 4:
        raise ValueError("expected an [n, 4] float32 array")
    return a


def make_lidar(num_lines=64, min_dist=3.0, max_dist=90.0, scan_period=0.1, ring_model=None):
    """lidar::Lidar. ring_model=(top_deg, bottom_deg): the linear beam-model EXTENSION
    (pf_fe_set_ring_model) for line counts the reference has no ring formula for (S128)."""
    lp = LidarParams(int(num_lines), float(min_dist), float(max_dist), float(scan_period))
    lp.ring_model = tuple(ring_model) if ring_model else None
    return lp


def tie_sort(keys, device=0, depth=-1, levels=2):
    """development probe pf_dev_tie_sort2: the input indices of the kept keys (not 0xFFFFFFFF) in the
    order the device's reference-tie-order sort (libstdc++ std::sort per class, bits 30-31, classes back
    to back) puts them. depth >= 0 replaces the depth limit 2 lg n (the heap-sort branch); levels = big
    levels before the single-workgroup fallback."""
    k = np.ascontiguousarray(keys, np.uint32)
    out = np.empty(max(k.size, 1), np.uint32)
    n = _sz()
    _check("pf_dev_tie_sort2", lib().pf_dev_tie_sort2(device, k.ctypes.data, k.size, int(depth), int(levels),
                                                      out.ctypes.data, ctypes.byref(n)), allow_warn=False)
    return out[:n.value].copy()


def device_count():
    n = _i()
    _check("pf_device_count", lib().pf_device_count(ctypes.byref(n)))
    return n.value


class DeviceBuffer:
    """Raw HBM allocation (scans staged once, read by the device pipeline)."""

    def __init__(self, nbytes, device=0):
        self.device, self.nbytes = device, int(nbytes)
        p = _vp()
        _check("pf_dev_malloc", lib().pf_dev_malloc(device, self.nbytes, ctypes.byref(p)))
        self.ptr = p.value

    def upload(self, arr, offset=0):
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        _check("pf_memcpy_h2d", lib().pf_memcpy_h2d(self.device, self.ptr + offset, a.ctypes.data, a.nbytes))

    def download(self, arr, offset=0):
        _check("pf_memcpy_d2h", lib().pf_memcpy_d2h(self.device, arr.ctypes.data, self.ptr + offset, arr.nbytes))
        return arr

    def free(self):
        if self.ptr:
            lib().pf_dev_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HostBuffer:
    """Pinned, device-mapped host memory (pf_host_alloc): what a caller keeps its scans in so that the
    host-input entry points DMA them without a repack. view() gives numpy arrays over it."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = _vp()
        _check("pf_host_alloc", lib().pf_host_alloc(self.nbytes, ctypes.byref(p)), allow_warn=False)
        self.ptr = p.value

    def view(self, shape, dtype=np.float32, offset=0):
        dt = np.dtype(dtype)
        count = int(np.prod(shape))
        assert offset + count * dt.itemsize <= self.nbytes
        raw = (ctypes.c_char * (count * dt.itemsize)).from_address(self.ptr + offset)
        return np.frombuffer(raw, dtype=dt, count=count).reshape(shape)

    def free(self):
        if self.ptr:
            lib().pf_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class LaserProcessingClass:
    """Drop-in for LaserProcessingClass (featureExtraction on the GPU)."""

    def __init__(self, device=0, max_points=300000, tie_order=None):
        """tie_order: None = the library default (the reference's std::sort order, on), False = the
        stable (value, ring position) order"""
        self.device, self.max_points, self.tie_order = device, max_points, tie_order
        self._h = None

    def init(self, lidar_param):
        h = _vp()
        _check("pf_fe_create", lib().pf_fe_create(ctypes.byref(lidar_param), self.device, self.max_points,
                                                  ctypes.byref(h)))
        self._h = h.value
        if self.tie_order is not None:
            self.set_tie_order(self.tie_order)
        self._rings = lidar_param.num_lines
        rm = getattr(lidar_param, "ring_model", None)
        if rm:
            _check("pf_fe_set_ring_model", lib().pf_fe_set_ring_model(self._h, float(rm[0]), float(rm[1])))

    def featureExtraction(self, pc_in):
        x = _f32x4(pc_in)
        n = x.shape[0]
        cap = max(n, 1)
        edge = np.empty((cap, 4), np.float32)
        surf = np.empty((cap, 4), np.float32)
        ne, ns = _sz(), _sz()
        _check("pf_fe_extract", lib().pf_fe_extract(self._h, x.ctypes.data, n, 16, edge.ctypes.data,
                                                    ctypes.byref(ne), surf.ctypes.data, ctypes.byref(ns), cap))
        return edge[:ne.value].copy(), surf[:ns.value].copy()

    def set_tie_order(self, enable):
        """reference tie order of the sector sort (pf_fe_set_tie_order): equal curvatures as
        libstdc++'s std::sort leaves them (src/laserProcessingClass.cpp:101-104)"""
        _check("pf_fe_set_tie_order", lib().pf_fe_set_tie_order(self._h, int(bool(enable))))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pf_fe_destroy(self._h)
            self._h = None


class Odom_ES_EstimationClass:
    """Drop-in for Odom_ES_EstimationClass (the whole update on the GPU)."""

    def __init__(self, device=0, max_points=300000, map_capacity=1 << 22, tie_order=None):
        """tie_order: None = the library default (the reference's std::sort order of equal keys, on:
        pf_odom_set_tie_order), False = the stable sorts (faster, centroids' last bits not the reference's)"""
        self.device, self.max_points, self.map_capacity = device, max_points, map_capacity
        self.tie_order = tie_order
        self._h = None
        self.last_status = PF_OK

    def _apply_order(self):
        if self.tie_order is not None:
            self.set_tie_order(self.tie_order)

    def init(self, lidar_param, map_resolution, k_new, theta_p, theta_max, weightType):
        self.lidar = lidar_param
        prm = OdomParams(float(map_resolution), int(k_new), float(theta_p), int(theta_max), int(weightType))
        h = _vp()
        _check("pf_odom_create", lib().pf_odom_create(ctypes.byref(lidar_param), ctypes.byref(prm), self.device,
                                                      self.max_points, self.map_capacity, ctypes.byref(h)))
        self._h = h.value
        self._apply_order()
        rm = getattr(lidar_param, "ring_model", None)
        if rm:
            _check("pf_odom_set_ring_model", lib().pf_odom_set_ring_model(self._h, float(rm[0]), float(rm[1])))

    def initMapWithPoints(self, edge_in, surf_in):
        e, s = _f32x4(edge_in), _f32x4(surf_in)
        _check("pf_odom_init_map", lib().pf_odom_init_map(self._h, e.ctypes.data, e.shape[0], 16, s.ctypes.data,
                                                          s.shape[0], 16))

    def updatePointsToMap(self, edge_in, surf_in):
        e, s = _f32x4(edge_in), _f32x4(surf_in)
        pose = np.empty(7)
        self.last_status = _check("pf_odom_update", lib().pf_odom_update(
            self._h, e.ctypes.data, e.shape[0], 16, s.ctypes.data, s.shape[0], 16, pose.ctypes.data))
        return pose

    @property
    def odom(self):
        """pose {qx, qy, qz, qw, tx, ty, tz} of the member `odom`"""
        p = np.empty(7)
        _check("pf_odom_get_pose", lib().pf_odom_get_pose(self._h, p.ctypes.data))
        return p

    def _map(self, which):
        n = _sz()
        _check("pf_odom_get_map", lib().pf_odom_get_map(self._h, which, None, None, 0, ctypes.byref(n)))
        xyz = np.empty((max(n.value, 1), 3), np.float32)
        rg = np.empty((max(n.value, 1), 2), np.uint8)
        _check("pf_odom_get_map", lib().pf_odom_get_map(self._h, which, xyz.ctypes.data, rg.ctypes.data, n.value,
                                                        ctypes.byref(n)))
        return xyz[:n.value].copy(), rg[:n.value].copy()

    @property
    def laserCloudCornerMap(self):
        return self._map(0)

    @property
    def laserCloudSurfMap(self):
        return self._map(1)

    def getMap(self):
        """surf map then corner map, appended (src/odomEstimationClass.cpp:210-215)"""
        s, c = self._map(1), self._map(0)
        return np.concatenate([s[0], c[0]]), np.concatenate([s[1], c[1]])

    def set_map(self, which, xyz, rg):
        xyz = np.ascontiguousarray(xyz, np.float32)
        rg = np.ascontiguousarray(rg, np.uint8)
        _check("pf_odom_set_map", lib().pf_odom_set_map(self._h, which, xyz.ctypes.data, rg.ctypes.data,
                                                        xyz.shape[0]))

    def stats(self):
        s = OdomStats()
        _check("pf_odom_get_stats", lib().pf_odom_get_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    # ---- whole-frame pipeline (featureExtraction -> init / update, all on the device) ----
    def frame_host(self, xyzi, want_pose=True):
        x = _f32x4(xyzi)
        pose = np.empty(7)
        _check("pf_odom_frame_host", lib().pf_odom_frame_host(self._h, x.ctypes.data, x.shape[0], 16,
                                                              pose.ctypes.data if want_pose else None))
        return pose if want_pose else None

    def frame_host_ptr(self, hptr, n, want_pose=False):
        """one packed float4 scan at a host address (a HostBuffer: DMA straight from it)"""
        pose = np.empty(7)
        _check("pf_odom_frame_host", lib().pf_odom_frame_host(self._h, hptr, int(n), 16,
                                                              pose.ctypes.data if want_pose else None))
        return pose if want_pose else None

    def frame_device(self, dptr, n, want_pose=False):
        pose = np.empty(7)
        _check("pf_odom_frame_device", lib().pf_odom_frame_device(self._h, dptr, int(n),
                                                                  pose.ctypes.data if want_pose else None))
        return pose if want_pose else None

    def sync(self):
        rc = lib().pf_odom_sync(self._h)
        if rc < 0:
            raise PFError("pf_odom_sync (device error words %s)" % dev_errors(self._h), rc)

    def poses(self):
        n = _sz()
        _check("pf_odom_poses", lib().pf_odom_poses(self._h, None, 0, ctypes.byref(n)))
        out = np.empty((max(n.value, 1), 7))
        _check("pf_odom_poses", lib().pf_odom_poses(self._h, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[:n.value].copy()

    def set_graph(self, mode):
        """hipGraph replay per stage (pf_odom_set_graph): 1 = stage A, 2 = stage B, 3 = both, 0 / False
        = eager launches, 4 / True = PF_GRAPH_AUTO (the default: stage A, and stage B when the process
        holds several handles)"""
        # this wrapper's numbering -> the C constants (PF_GRAPH_AUTO 1, PF_GRAPH_STAGE_A 2, _STAGE_B 4)
        m = 4 if mode is True else int(mode)
        if m not in (0, 1, 2, 3, 4):
            raise ValueError("graph mode %r" % (mode,))
        c = 1 if m == 4 else ((2 if m & 1 else 0) | (4 if m & 2 else 0))
        _check("pf_odom_set_graph", lib().pf_odom_set_graph(self._h, c))

    def set_stage_timing(self, enable):
        _check("pf_odom_set_stage_timing", lib().pf_odom_set_stage_timing(self._h, int(bool(enable))))

    def stage_times(self):
        """{a_us, b_us, frames}: mean device time of stage A (features + VoxelGrid) and stage B (odometry)
        per frame since set_stage_timing(True)"""
        a, b, n = ctypes.c_double(), ctypes.c_double(), _sz()
        _check("pf_odom_stage_times", lib().pf_odom_stage_times(self._h, ctypes.byref(a), ctypes.byref(b),
                                                                ctypes.byref(n)))
        return {"a_us": a.value, "b_us": b.value, "frames": n.value}

    # ---- OdomBaseClass public members and state capture ----
    def state(self):
        """{parameters (q_w_curr x, y, z, w, t_w_curr), last_odom (3 x 4 [R | t]), optimization_count}"""
        prm, last, oc = np.empty(7), np.empty(12), _i()
        _check("pf_odom_get_state", lib().pf_odom_get_state(self._h, prm.ctypes.data, last.ctypes.data,
                                                            ctypes.byref(oc)))
        return {"parameters": prm, "last_odom": last.reshape(3, 4), "optimization_count": oc.value}

    def set_state(self, odom_pose, last_pose=None, optimization_count=2):
        """odom = (R(q), t) of `odom_pose`, last_odom of `last_pose`, optimization_count (pf_odom_set_state)"""
        a = np.ascontiguousarray(odom_pose, np.float64)
        b = None if last_pose is None else np.ascontiguousarray(last_pose, np.float64)
        _check("pf_odom_set_state", lib().pf_odom_set_state(self._h, a.ctypes.data, None if b is None else b.ctypes.data,
                                                            int(optimization_count)))

    def snapshot(self):
        """the whole estimator state as bytes (pf_odom_snapshot)"""
        n = _sz()
        _check("pf_odom_snapshot", lib().pf_odom_snapshot(self._h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        _check("pf_odom_snapshot", lib().pf_odom_snapshot(self._h, buf, n.value, ctypes.byref(n)))
        return buf.raw

    def restore(self, blob):
        buf = ctypes.create_string_buffer(bytes(blob), len(blob))
        _check("pf_odom_restore", lib().pf_odom_restore(self._h, buf, len(blob)))

    def probe_assoc(self, iters=20, queries=False, cap=400000):
        """pf_odom_probe_assoc: (avg ms per launch of the association's kNN on the last frame, algorithmic
        bytes per launch, query count[, queries [nq, 4] float32: x, y, z, bits(class)])"""
        ms, b, n = ctypes.c_double(), ctypes.c_double(), _sz()
        q = np.empty((cap, 4), np.float32) if queries else None
        _check("pf_odom_probe_assoc", lib().pf_odom_probe_assoc(self._h, int(iters), ctypes.byref(ms), ctypes.byref(b),
                                                                ctypes.byref(n), q.ctypes.data if queries else None,
                                                                cap if queries else 0), allow_warn=False)
        if queries:
            return ms.value, b.value, n.value, q[:n.value].copy()
        return ms.value, b.value, n.value

    def set_rg_radix(self, enable):
        """development switch pf_dev_set_rg_radix: rgbds by the full radix sort instead of the merge"""
        L = lib()
        L.pf_dev_set_rg_radix.argtypes = [_vp, _i]
        _check("pf_dev_set_rg_radix", L.pf_dev_set_rg_radix(self._h, int(bool(enable))))

    def set_dep_full(self, enable):
        """development switch pf_dev_set_dep_full: every tie-order rgbds takes the full dependence table
        (each update as if the host had written the map) instead of the appended points' small table"""
        L = lib()
        L.pf_dev_set_dep_full.argtypes = [_vp, _i]
        _check("pf_dev_set_dep_full", L.pf_dev_set_dep_full(self._h, int(bool(enable))))

    def set_fuse_observe(self, enable):
        """development switch pf_dev_set_fuse_observe: False = the separate k_observe launch at weightType 0"""
        L = lib()
        L.pf_dev_set_fuse_observe.argtypes = [_vp, _i]
        _check("pf_dev_set_fuse_observe", L.pf_dev_set_fuse_observe(self._h, int(bool(enable))))

    def merge_stats(self):
        """pf_odom_merge_stats: (updates that sorted every element, largest appended-point count)"""
        f, m = _i(), _i()
        _check("pf_odom_merge_stats", lib().pf_odom_merge_stats(self._h, ctypes.byref(f), ctypes.byref(m)))
        return f.value, m.value

    def set_tie_order(self, enable):
        """pf_odom_set_tie_order: VoxelGrid / rgbds order equal keys as libstdc++ std::sort (parity mode)"""
        _check("pf_odom_set_tie_order", lib().pf_odom_set_tie_order(self._h, int(bool(enable))), allow_warn=False)

    def set_map_export(self, enable):
        _check("pf_odom_set_map_export", lib().pf_odom_set_map_export(self._h, int(bool(enable))))

    def map_export(self, which):
        """(xyz [n, 3] float32, rg [n, 2] uint8) of map `which` from the pinned export buffer"""
        ptr, n = ctypes.POINTER(ctypes.c_float)(), _sz()
        _check("pf_odom_map_export", lib().pf_odom_map_export(self._h, int(which), ctypes.byref(ptr), ctypes.byref(n)))
        a = np.ctypeslib.as_array(ptr, shape=(max(n.value, 1), 4))[:n.value].copy()
        w = a[:, 3].view(np.uint32)
        rg = np.stack([(w & 255), (w >> 8) & 255], 1).astype(np.uint8)
        return a[:, :3].copy(), rg

    def set_stage_a_reserve(self, cus):
        """CUs stage A stays off (default 128 ES / 32 BPF; 0 when several handles share the GPU)"""
        _check("pf_odom_set_stage_a_reserve", lib().pf_odom_set_stage_a_reserve(self._h, int(cus)))

    def reset(self):
        """state right after init (a new sequence on the same handle and buffers)"""
        _check("pf_odom_reset", lib().pf_odom_reset(self._h))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pf_odom_destroy(self._h)
            self._h = None


# the node-facing alias named by the north star
OdomEstimationClass = Odom_ES_EstimationClass


class Odom_BPF_EstimationClass(Odom_ES_EstimationClass):
    """Drop-in for Odom_BPF_EstimationClass (src/odomEstimationClass.cpp:649-1306): beam / pillar /
    facade maps, the whole update on the GPU. Map accessors by class: 0 beam, 1 pillar, 2 facade."""

    def init(self, lidar_param, map_resolution, k_new, theta_p, theta_max, weightType):
        self.lidar = lidar_param
        prm = OdomParams(float(map_resolution), int(k_new), float(theta_p), int(theta_max), int(weightType))
        h = _vp()
        _check("pf_bpf_create", lib().pf_bpf_create(ctypes.byref(lidar_param), ctypes.byref(prm), self.device,
                                                    self.max_points, self.map_capacity, ctypes.byref(h)))
        self._h = h.value
        self._apply_order()

    def initMapWithPoints(self, beam_in, pillar_in, facade_in):
        b, p, f = _f32x4(beam_in), _f32x4(pillar_in), _f32x4(facade_in)
        _check("pf_bpf_init_map", lib().pf_bpf_init_map(self._h, b.ctypes.data, b.shape[0], 16, p.ctypes.data,
                                                        p.shape[0], 16, f.ctypes.data, f.shape[0], 16))

    def updatePointsToMap(self, beam_in, pillar_in, facade_in):
        b, p, f = _f32x4(beam_in), _f32x4(pillar_in), _f32x4(facade_in)
        pose = np.empty(7)
        self.last_status = _check("pf_bpf_update", lib().pf_bpf_update(
            self._h, b.ctypes.data, b.shape[0], 16, p.ctypes.data, p.shape[0], 16, f.ctypes.data, f.shape[0], 16,
            pose.ctypes.data))
        return pose

    @property
    def laserCloudBeamMap(self):
        return self._map(0)

    @property
    def laserCloudPillarMap(self):
        return self._map(1)

    @property
    def laserCloudFacadeMap(self):
        return self._map(2)

    @property
    def laserCloudCornerMap(self):
        raise AttributeError("Odom_BPF_EstimationClass has beam / pillar / facade maps")

    laserCloudSurfMap = laserCloudCornerMap

    def getMap(self):
        """beam, pillar, then facade, appended (src/odomEstimationClass.cpp:683-689)"""
        parts = [self._map(c) for c in range(3)]
        return np.concatenate([m[0] for m in parts]), np.concatenate([m[1] for m in parts])

    def frame_device(self, d_clouds, counts, want_pose=False):
        """d_clouds: device pointers of the beam / pillar / facade clouds (packed float4), counts: sizes"""
        pose = np.empty(7)
        (b, p, f), (nb, np_, nf) = d_clouds, counts
        _check("pf_bpf_frame_device", lib().pf_bpf_frame_device(self._h, b, int(nb), p, int(np_), f, int(nf),
                                                                pose.ctypes.data if want_pose else None))
        return pose if want_pose else None

    # ---- raw-scan mode: the front end (ground_seg + featureExtract) in stage A, then the odometry ----
    def set_front_end(self, **params):
        """pf_cls_params of the front end (defaults: the reference's members, include/preProcess.hpp)"""
        self.front_params = cls_params(**params)
        _check("pf_bpf_set_front_end", lib().pf_bpf_set_front_end(self._h, ctypes.byref(self.front_params)),
               allow_warn=False)

    def set_dcvc(self, enable=True, **params):
        """curvedfilter (pf_bpf_set_dcvc): DCVC between ground_seg and featureExtract in raw-scan mode"""
        p = ctypes.byref(dcvc_params(**params)) if enable else None
        _check("pf_bpf_set_dcvc", lib().pf_bpf_set_dcvc(self._h, p), allow_warn=False)

    def set_front_lanes(self, lanes):
        """pf_bpf_set_front_lanes: 2 (default) overlaps consecutive frames' front ends, 1 runs it in line"""
        _check("pf_bpf_set_front_lanes", lib().pf_bpf_set_front_lanes(self._h, int(lanes)), allow_warn=False)

    def frame_scan_device(self, dptr, n, want_pose=False):
        """one raw scan already in HBM (packed float4) -> pose"""
        pose = np.empty(7)
        _check("pf_bpf_frame_scan_device", lib().pf_bpf_frame_scan_device(
            self._h, dptr, int(n), pose.ctypes.data if want_pose else None))
        return pose if want_pose else None

    def frame_host(self, xyzi, want_pose=True):
        """one raw scan from host memory (staged through a device buffer) -> pose"""
        x = _f32x4(xyzi)
        buf = getattr(self, "_scan_buf", None)
        if buf is None or buf.nbytes < max(x.nbytes, 16):
            if buf is not None:
                self.sync()
            buf = self._scan_buf = DeviceBuffer(max(x.nbytes, 16, 16 * self.max_points), self.device)
        self.sync()                   # the previous frame's stage A has consumed the buffer
        buf.upload(x)
        return self.frame_scan_device(buf.ptr, x.shape[0], want_pose)


class Knn:
    """Exact radius-gated 5-NN (the roofline kernel) on a resident map."""

    def __init__(self, map_capacity, query_capacity, device=0):
        h = _vp()
        _check("pf_knn_create", lib().pf_knn_create(device, int(map_capacity), int(query_capacity),
                                                    ctypes.byref(h)))
        self._h = h.value

    def set_map(self, xyz4):
        m = _f32x4(xyz4)
        _check("pf_knn_set_map", lib().pf_knn_set_map(self._h, m.ctypes.data, m.shape[0]), allow_warn=False)

    def query(self, q4):
        q = _f32x4(q4)
        idx = np.empty((q.shape[0], 5), np.int32)
        d2 = np.empty((q.shape[0], 5), np.float32)
        _check("pf_knn_query", lib().pf_knn_query(self._h, q.ctypes.data, q.shape[0], idx.ctypes.data,
                                                  d2.ctypes.data))
        return idx, d2

    def bench(self, iters=20):
        ms, b = ctypes.c_double(), ctypes.c_double()
        _check("pf_knn_bench", lib().pf_knn_bench(self._h, int(iters), ctypes.byref(ms), ctypes.byref(b)))
        return ms.value, b.value

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pf_knn_destroy(self._h)
            self._h = None


def cls_params(**kw):
    """The reference's defaults (pf_cls_default_params) with keyword overrides."""
    p = ClsParams()
    lib().pf_cls_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class BPFFrontEnd:
    """groundSeg::ground_seg + nongroundExtract::featureExtract as src/additionNode.cpp:21-45 chains them
    (include/preProcess.hpp:398-505, :646-689): a scan in, the beam / pillar / facade clouds (and the
    ground cloud) out, as indices into the scan in the published order."""

    def __init__(self, max_points=300000, device=0, **params):
        self.params = cls_params(**params)
        h = _vp()
        _check("pf_cls_create", lib().pf_cls_create(ctypes.byref(self.params), device, int(max_points),
                                                    ctypes.byref(h)), allow_warn=False)
        self._h = h.value

    def set_dcvc(self, enable=True, **params):
        """curvedfilter (pf_cls_set_dcvc): extract() runs DCVC on the non-ground cloud first"""
        p = ctypes.byref(dcvc_params(**params)) if enable else None
        _check("pf_cls_set_dcvc", lib().pf_cls_set_dcvc(self._h, p), allow_warn=False)

    def extract(self, xyz):
        a = np.ascontiguousarray(xyz, dtype=np.float32)
        n = a.shape[0]
        bufs = [np.empty(max(n, 1), np.int32) for _ in range(4)]
        cnt = [_sz() for _ in range(4)]
        args = []
        for b, c in zip(bufs, cnt):
            args += [b.ctypes.data, ctypes.byref(c)]
        _check("pf_cls_extract", lib().pf_cls_extract(self._h, a.ctypes.data, n, 4 * a.shape[1], *args, max(n, 1)),
               allow_warn=False)
        return {k: b[:c.value].copy() for k, b, c in zip(("beam", "pillar", "facade", "ground"), bufs, cnt)}

    def ground_seg(self, xyz):
        """ground_seg alone: (ground, non-ground) input indices in the reference's push order."""
        a = np.ascontiguousarray(xyz, dtype=np.float32)
        n = a.shape[0]
        g, u = np.empty(max(n, 1), np.int32), np.empty(max(n, 1), np.int32)
        ng, nu = _sz(), _sz()
        _check("pf_cls_ground_seg", lib().pf_cls_ground_seg(self._h, a.ctypes.data, n, 4 * a.shape[1], g.ctypes.data,
                                                            ctypes.byref(ng), u.ctypes.data, ctypes.byref(nu),
                                                            max(n, 1)), allow_warn=False)
        return g[:ng.value].copy(), u[:nu.value].copy()

    def classify(self, xyz, normals=False):
        """featureExtract alone: (index_with_feature code per point, neighbour count per point[, the
        normal assign_normal writes per point, [n, 4] float32])."""
        a = np.ascontiguousarray(xyz, dtype=np.float32)
        n = a.shape[0]
        cls = np.empty(max(n, 1), np.uint8)
        num = np.empty(max(n, 1), np.int32)
        _check("pf_cls_classify", lib().pf_cls_classify(self._h, a.ctypes.data, n, 4 * a.shape[1], cls.ctypes.data,
                                                        num.ctypes.data), allow_warn=False)
        if not normals:
            return cls[:n].copy(), num[:n].copy()
        nrm = np.empty((max(n, 1), 4), np.float32)
        _check("pf_cls_normals", lib().pf_cls_normals(self._h, nrm.ctypes.data, n), allow_warn=False)
        return cls[:n].copy(), num[:n].copy(), nrm[:n].copy()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pf_cls_destroy(self._h)
            self._h = None


class LaserMappingClass:
    """LaserMappingClass (src/laserMappingClass.cpp): init(map_resolution), updateCurrentPointsToMap(xyzi,
    pose7 = qx, qy, qz, qw, tx, ty, tz), getMap() -> (n, 4) x, y, z, intensity in the reference's order."""

    def __init__(self, device=0, max_points=1 << 24, max_scan=300000):
        self.device, self.max_points, self.max_scan = device, int(max_points), int(max_scan)
        self._h = None

    def init(self, map_resolution):
        h = _vp()
        _check("pf_map_create", lib().pf_map_create(float(map_resolution), self.device, self.max_points,
                                                    self.max_scan, ctypes.byref(h)), allow_warn=False)
        self._h = h.value

    def updateCurrentPointsToMap(self, xyzi, pose7):
        a = np.ascontiguousarray(xyzi, dtype=np.float32)
        pose = np.ascontiguousarray(pose7, dtype=np.float64)
        _check("pf_map_update", lib().pf_map_update(self._h, a.ctypes.data, a.shape[0], 4 * a.shape[1],
                                                    pose.ctypes.data), allow_warn=False)

    def getMap(self):
        n = _sz()
        _check("pf_map_get", lib().pf_map_get(self._h, None, 0, ctypes.byref(n)))
        out = np.empty((max(n.value, 1), 4), np.float32)
        _check("pf_map_get", lib().pf_map_get(self._h, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[:n.value].copy()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().pf_map_destroy(self._h)
            self._h = None
