"""GPU: the host-input entry points (include/pfilter_hip.h): scans and clouds arriving from host memory,
as the reference's nodes hand them over (src/laserProcessingNode.cpp:62-78, src/odomEstimationNode
copy.cpp:74-100). The upload goes by DMA on each handle's copy stream (pinned caller memory from
pf_host_alloc directly, other memory through pinned staging); the results must be the bits of the
HBM-resident pipeline, and a caller may reuse its buffer as soon as a call returns."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LID = (64, 3.0, 90.0)
CFG = (0.4, 0, 0.4, 75, 0)


def _odom(pa):
    od = pa.Odom_ES_EstimationClass(device=0)
    od.init(pa.make_lidar(*LID), *CFG)
    return od


def _device_run(pa, buf, counts, n):
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    od = _odom(pa)
    for k in range(n):
        od.frame_device(db.ptr + k * buf.shape[1] * 16, int(counts[k]))
    od.sync()
    p = od.poses()
    db.free()
    return p, od


def test_frame_host_pinned_and_pageable_equal_device_pipeline(pa, pfsynth):
    """pf_odom_frame_host over 30 frames, enqueue-only (pose_out NULL): from one pf_host_alloc buffer
    that is overwritten with the next scan right after every call returns, and from pageable numpy
    arrays; both give the HBM-resident pipeline's poses and final maps bit for bit."""
    n = 30
    seq = pfsynth.Sequence("S64", n_frames=n, az_steps=1500)
    buf, counts = seq.frames(0, n)
    want, ref = _device_run(pa, buf, counts, n)
    hb = pa.HostBuffer(buf.shape[1] * 16)
    view = hb.view((buf.shape[1], 4))
    od = _odom(pa)
    for k in range(n):
        view[:counts[k]] = buf[k, :counts[k]]
        od.frame_host_ptr(hb.ptr, int(counts[k]))
        view[:] = -1.0e30                                  # the caller's buffer is free on return
    od.sync()
    np.testing.assert_array_equal(od.poses(), want)
    for which in (0, 1):
        np.testing.assert_array_equal(od._map(which)[0], ref._map(which)[0])
        np.testing.assert_array_equal(od._map(which)[1], ref._map(which)[1])
    od2 = _odom(pa)
    for k in range(n):
        x = buf[k, :counts[k]].copy()
        od2.frame_host(x, want_pose=False)
        x[:] = np.nan
    od2.sync()
    np.testing.assert_array_equal(od2.poses(), want)


def test_frame_host_pcl_stride_and_pose_out(pa, pfsynth):
    """32-byte PCL PointXYZI records (intensity at byte 16) and the synchronous form with pose_out:
    the pose returned by every call is that frame's pose of the device pipeline."""
    n = 12
    seq = pfsynth.Sequence("S64", n_frames=n, az_steps=1200)
    buf, counts = seq.frames(0, n)
    want, _ = _device_run(pa, buf, counts, n)
    L = pa.lib()
    od = _odom(pa)
    pose = np.empty(7)
    for k in range(n):
        x = buf[k, :counts[k]]
        pcl = np.zeros((x.shape[0], 8), np.float32)
        pcl[:, :3] = x[:, :3]
        pcl[:, 4] = x[:, 3]
        assert L.pf_odom_frame_host(od._h, pcl.ctypes.data, x.shape[0], 32, pose.ctypes.data) >= 0
        np.testing.assert_array_equal(pose, want[k])


def test_fe_extract_pinned_outputs(pa, pfref, pfsynth):
    """pf_fe_extract with the scan and both outputs in pf_host_alloc memory (the kernel writes the clouds
    straight into the caller's buffers) equals the pageable call and the oracle bit for bit; a cap
    below the output size reports PF_ECAPACITY with the counts set."""
    seq = pfsynth.Sequence("S64", n_frames=3)
    x = seq.frame(2)
    fe = pa.LaserProcessingClass(device=0)
    fe.init(pa.make_lidar(*LID))
    ge, gs = fe.featureExtraction(x)
    re_, rs_ = pfref.feature_extraction(x, pfref.make_lidar(*LID), opts=0)
    np.testing.assert_array_equal(ge.view(np.uint32), re_.view(np.uint32))
    np.testing.assert_array_equal(gs.view(np.uint32), rs_.view(np.uint32))
    n = x.shape[0]
    hin, he, hs = pa.HostBuffer(n * 16), pa.HostBuffer(n * 16), pa.HostBuffer(n * 16)
    hin.view((n, 4))[:] = x
    ne, ns = ctypes.c_size_t(), ctypes.c_size_t()
    L = pa.lib()
    rc = L.pf_fe_extract(fe._h, hin.ptr, n, 16, he.ptr, ctypes.byref(ne), hs.ptr, ctypes.byref(ns), n)
    assert rc == 0 and (ne.value, ns.value) == (ge.shape[0], gs.shape[0])
    np.testing.assert_array_equal(he.view((ne.value, 4)).view(np.uint32), ge.view(np.uint32))
    np.testing.assert_array_equal(hs.view((ns.value, 4)).view(np.uint32), gs.view(np.uint32))
    rc = L.pf_fe_extract(fe._h, hin.ptr, n, 16, he.ptr, ctypes.byref(ne), hs.ptr, ctypes.byref(ns), 100)
    assert rc == pa.PF_ECAPACITY and (ne.value, ns.value) == (ge.shape[0], gs.shape[0])


def test_node_call_pattern_equals_device_pipeline(pa, pfsynth):
    """The nodes' synchronous pattern, pf_fe_extract -> pf_odom_init_map / pf_odom_update with the clouds
    in pinned host RAM (bench.py's node_pattern leg), gives the device pipeline's poses bit for bit."""
    n = 16
    seq = pfsynth.Sequence("S64", n_frames=n, az_steps=1500)
    buf, counts = seq.frames(0, n)
    want, _ = _device_run(pa, buf, counts, n)
    L = pa.lib()
    fe = pa.LaserProcessingClass(device=0)
    fe.init(pa.make_lidar(*LID))
    od = _odom(pa)
    cap = buf.shape[1]
    hin, he, hs = pa.HostBuffer(cap * 16), pa.HostBuffer(cap * 16), pa.HostBuffer(cap * 16)
    ne, ns = ctypes.c_size_t(), ctypes.c_size_t()
    pose = np.empty(7)
    for k in range(n):
        hin.view((cap, 4))[:counts[k]] = buf[k, :counts[k]]
        assert L.pf_fe_extract(fe._h, hin.ptr, int(counts[k]), 16, he.ptr, ctypes.byref(ne), hs.ptr,
                               ctypes.byref(ns), cap) == 0
        if k == 0:
            assert L.pf_odom_init_map(od._h, he.ptr, ne.value, 16, hs.ptr, ns.value, 16) == 0
        else:
            assert L.pf_odom_update(od._h, he.ptr, ne.value, 16, hs.ptr, ns.value, 16, pose.ctypes.data) >= 0
            np.testing.assert_array_equal(pose, want[k])
    np.testing.assert_array_equal(od.poses(), want)


def test_host_buffer_registry(pa):
    """pf_host_alloc / pf_host_free: a freed block is forgotten (a second free is PF_EINVAL), frees of
    unknown pointers are refused, and numpy views round-trip."""
    L = pa.lib()
    hb = pa.HostBuffer(4096)
    v = hb.view((256, 4))
    v[:] = np.arange(1024, dtype=np.float32).reshape(256, 4)
    np.testing.assert_array_equal(hb.view((256, 4)), np.arange(1024, dtype=np.float32).reshape(256, 4))
    ptr = hb.ptr
    hb.free()
    assert L.pf_host_free(ptr) == pa.PF_EINVAL
    x = np.zeros(16, np.float32)
    assert L.pf_host_free(x.ctypes.data) == pa.PF_EINVAL
