"""GPU: LaserProcessingClass::featureExtraction (src/laserProcessingClass.cpp:10-209) through
pf_fe_extract, bit-exact against the oracle.

Order and bits of every edge / surf point must equal the oracle: in the library's default order (the
reference's: equal curvatures in a sector as libstdc++'s std::sort leaves them) against opts=0, in the
stable order (pf_fe_set_tie_order off: equal curvatures by index) against FE_STABLE_TIES."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fe(pa, lines, mn=3.0, mx=90.0, order="tie"):
    fe = pa.LaserProcessingClass(device=0, tie_order=None if order == "tie" else False)
    fe.init(pa.make_lidar(lines, mn, mx))
    return fe


def _ref(pfref, x, lines, mn=3.0, mx=90.0, order="tie"):
    return pfref.feature_extraction(x, pfref.make_lidar(lines, mn, mx),
                                    opts=0 if order == "tie" else pfref.FE_STABLE_TIES)


def _same(a, b):
    assert a.shape == b.shape, (a.shape, b.shape)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("preset,lines,frames", [("S64", 64, (0, 9)), ("S32", 32, (4,)), ("S128", 64, (2,))])
def test_fe_bit_exact(pa, pfref, pfsynth, preset, lines, frames):
    """S128 fed to a 64-line config: rings above 63 follow the reference's 64-line binning."""
    seq = pfsynth.Sequence(preset, n_frames=12)
    fe = _fe(pa, lines)
    for k in frames:
        x = seq.frame(k)
        ge, gs = fe.featureExtraction(x)
        re_, rs_ = _ref(pfref, x, lines)
        assert re_.shape[0] > 100 and rs_.shape[0] > 1000
        _same(ge, re_)
        _same(gs, rs_)


def test_fe_16_lines_and_range_gate(pa, pfref, pfsynth):
    seq = pfsynth.Sequence("S32", n_frames=4, az_steps=700)
    x = seq.frame(1)
    fe = _fe(pa, 16, 5.0, 40.0)
    ge, gs = fe.featureExtraction(x)
    re_, rs_ = _ref(pfref, x, 16, 5.0, 40.0)
    _same(ge, re_)
    _same(gs, rs_)


def test_fe_pcl_stride(pa, pfref, pfsynth):
    """32-byte PCL PointXYZI layout (x, y, z, pad, intensity, pad x3)."""
    x = pfsynth.Sequence("S64", n_frames=2, az_steps=800).frame(1)
    pcl = np.zeros((x.shape[0], 8), np.float32)
    pcl[:, :3] = x[:, :3]
    pcl[:, 3] = 1.0
    pcl[:, 4] = x[:, 3]
    fe = _fe(pa, 64)
    n = x.shape[0]
    edge = np.empty((n, 4), np.float32)
    surf = np.empty((n, 4), np.float32)
    ne, ns = ctypes.c_size_t(), ctypes.c_size_t()
    rc = pa.lib().pf_fe_extract(fe._h, pcl.ctypes.data, n, 32, edge.ctypes.data, ctypes.byref(ne),
                                surf.ctypes.data, ctypes.byref(ns), n)
    assert rc == 0
    re_, rs_ = _ref(pfref, x, 64)
    _same(edge[:ne.value], re_)
    _same(surf[:ns.value], rs_)


def test_fe_empty_and_tiny(pa, pfref):
    fe = _fe(pa, 64)
    e, s = fe.featureExtraction(np.zeros((0, 4), np.float32))
    assert e.shape[0] == 0 and s.shape[0] == 0
    rng = np.random.default_rng(3)
    x = np.zeros((40, 4), np.float32)          # fewer than 131 points per ring: no sectors
    x[:, :3] = rng.uniform(-20, 20, (40, 3))
    x[:, 2] = rng.uniform(-1, 0.2, 40)
    ge, gs = fe.featureExtraction(x)
    re_, rs_ = _ref(pfref, x, 64)
    _same(ge, re_)
    _same(gs, rs_)


@pytest.mark.parametrize("order", ["tie", "stable"])
def test_fe_random_cloud_with_ties(pa, pfref, order):
    """Quantised coordinates: many equal curvatures, exercising both tie orders."""
    rng = np.random.default_rng(4)
    n = 60000
    az = rng.uniform(-np.pi, np.pi, n)
    el = np.radians(rng.uniform(-24.0, 2.0, n))
    r = np.round(rng.uniform(4, 60, n) * 4) / 4
    x = np.zeros((n, 4), np.float32)
    x[:, 0] = r * np.cos(el) * np.cos(az)
    x[:, 1] = r * np.cos(el) * np.sin(az)
    x[:, 2] = r * np.sin(el)
    x[:, 3] = rng.uniform(0, 1, n)
    fe = _fe(pa, 64, order=order)
    ge, gs = fe.featureExtraction(x)
    re_, rs_ = _ref(pfref, x, 64, order=order)
    _same(ge, re_)
    _same(gs, rs_)


def test_fe_capacity_error(pa):
    fe = pa.LaserProcessingClass(device=0, max_points=1000)
    fe.init(pa.make_lidar(64, 3.0, 90.0))
    with pytest.raises(pa.PFError) as ei:
        fe.featureExtraction(np.ones((1001, 4), np.float32))
    assert ei.value.code == pa.PF_ECAPACITY


def test_fe_golden(pa, pfsynth):
    """Against the committed oracle vectors (tests/golden/fe_s32_f3.npz, FE_STABLE_TIES)."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fe_s32_f3.npz"))
    x = pfsynth.Sequence("S32", n_frames=6, az_steps=600).frame(3)
    fe = _fe(pa, 32, order="stable")
    e, s = fe.featureExtraction(x)
    _same(e, g["edge"])
    _same(s, g["surf"])


def test_fe_s128_linear_ring_model(pa, pfref, pfsynth):
    """configs[4] scans (128 lines, -25..+15 deg) through the linear beam-model extension
    (pf_fe_set_ring_model), bit-exact against the oracle with the same model. Without the model the
    reference puts every point into ring 0 (src/laserProcessingClass.cpp:58-61): six sectors of
    ~25k points, far above the LDS sort's 2048 entries, which the device sorts in global scratch
    (any sector size, as the reference) — also bit-exact."""
    seq = pfsynth.Sequence("S128", n_frames=4)
    x = seq.frame(3)
    for model in ((15.0, -25.0), None):
        fe = pa.LaserProcessingClass(device=0)
        fe.init(pa.make_lidar(128, 3.0, 90.0, ring_model=model))
        ge, gs = fe.featureExtraction(x)
        re_, rs_ = pfref.feature_extraction(x, pfref.make_lidar(128, 3.0, 90.0, ring_model=model),
                                            opts=0)
        _same(ge, re_)
        _same(gs, rs_)
        assert ge.shape[0] > (128 * 6 * 5 if model else 6 * 5)


def test_fe_sector_sizes_around_the_lds_limit(pa, pfref, pfsynth):
    """Sectors on both sides of the 2048-entry LDS sort: S32 scans binned as 16 lines (the
    reference's 16-line formula folds beams together) at 2,000 to 9,000 azimuth steps give sectors
    of ~300 to ~3,900 entries in one scan; features bit-exact against the oracle."""
    for az in (2000, 6100, 9000):
        x = pfsynth.Sequence("S32", n_frames=1, az_steps=az).frame(0)
        fe = _fe(pa, 16)
        ge, gs = fe.featureExtraction(x)
        re_, rs_ = _ref(pfref, x, 16)
        _same(ge, re_)
        _same(gs, rs_)


def _tie_scan(pfsynth):
    """an S64 frame plus five rings that repeat two points in runs of 16 (A x16, B x16, ...): exact
    curvature ties, at 0 inside the runs (surf points) and at equal non-zero values on every A->B / B->A
    boundary (edge candidates above 0.1)"""
    x = pfsynth.Sequence("S64", n_frames=2, az_steps=800).frame(1)
    parts = [x]
    rng = np.random.default_rng(7)
    for r in (3, 8, 14, 20, 27):
        el = np.deg2rad(2.0 - r / 3.0)                       # ring r's centre (64-line formula, :38-39)
        th = rng.uniform(0, 2 * np.pi, 2)
        a = np.array([10 * np.cos(th[0]), 10 * np.sin(th[0]), 10 * np.tan(el), 0.5], np.float32)
        b = np.array([13 * np.cos(th[1]), 13 * np.sin(th[1]), 13 * np.tan(el), 0.7], np.float32)
        run = np.concatenate([np.repeat(a[None], 16, 0), np.repeat(b[None], 16, 0)])
        parts.append(np.tile(run, (20, 1)))
    return np.concatenate(parts).astype(np.float32)


def test_fe_tie_order_equal_curvatures(pa, pfref, pfsynth):
    """Reference tie order (pf_fe_set_tie_order): on a scan with exact curvature ties the device
    equals the faithful oracle (libstdc++ std::sort itself, opts=0) bit for bit, and the stable
    order still equals FE_STABLE_TIES; the two orders differ on this scan, so the check has teeth."""
    x = _tie_scan(pfsynth)
    lid = pfref.make_lidar(64, 3.0, 90.0)
    fe = _fe(pa, 64, order="stable")
    se, ss = fe.featureExtraction(x)
    _same(se, _ref(pfref, x, 64, order="stable")[0])
    _same(ss, _ref(pfref, x, 64, order="stable")[1])
    fe.set_tie_order(True)
    te, ts = fe.featureExtraction(x)
    re_, rs_ = pfref.feature_extraction(x, lid, opts=0)
    _same(te, re_)
    _same(ts, rs_)
    assert not np.array_equal(ts.view(np.uint32), ss.view(np.uint32)), "no tie changed the surf order"
    fe.set_tie_order(False)
    _same(fe.featureExtraction(x)[1], ss)
