"""GPU: the reference-tie-order sort (pf_tie.h, pf_odom_set_tie_order) against libstdc++'s std::sort
itself -- the reference's own VoxelGrid / rgbds sort (src/odomEstimationClass.cpp:74),
which leaves equal keys in an order only introsort defines. The device's permutation of the input
indices must be std::sort's exactly, per class (key bits 30-31), with 0xFFFFFFFF keys dropped."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _inputs():
    rng = np.random.default_rng(21)
    yield np.zeros(0, np.uint32)
    yield np.array([3], np.uint32)
    for n in (2, 16, 17, 18, 100, 5000, 65000):
        yield rng.integers(0, max(2, n // 7), n).astype(np.uint32)
        yield rng.integers(0, 1 << 30, n).astype(np.uint32)
        yield np.sort(rng.integers(0, 50, n)).astype(np.uint32)
        yield np.sort(rng.integers(0, 50, n))[::-1].astype(np.uint32).copy()
        yield np.full(n, 9, np.uint32)
    k = np.sort(rng.integers(0, 40000, 60000)).astype(np.uint32)            # voxel-ordered map + new points
    yield np.concatenate([k, rng.integers(0, 40000, 6000).astype(np.uint32)])


def _expected(pfref, keys):
    out = []
    for c in range(4):
        idx = np.nonzero((keys != 0xFFFFFFFF) & ((keys >> 30) == c))[0]
        out.append(idx[pfref.sort_perm(keys[idx], "std")])
    return np.concatenate(out).astype(np.uint32) if out else np.zeros(0, np.uint32)


def test_tie_sort_is_std_sort(pa, pfref):
    for keys in _inputs():
        np.testing.assert_array_equal(pa.tie_sort(keys), _expected(pfref, keys), err_msg="n=%d" % keys.size)


def test_tie_sort_classes_and_dropped_keys(pa, pfref):
    """rgbds / VoxelGrid batches: several classes back to back (the reference sorts each cloud on its
    own), cropped points (0xFFFFFFFF) interleaved and dropped, map-like tie-heavy keys."""
    rng = np.random.default_rng(22)
    for sizes in ((30000, 9000), (7000, 52000), (500, 800, 1200), (20, 5, 40000)):
        parts = []
        for c, n in enumerate(sizes):
            k = (rng.integers(0, max(2, n // 4), n).astype(np.uint32) & 0x3FFFFFFF) | np.uint32(c << 30)
            k[rng.random(n) < 0.05] = 0xFFFFFFFF
            parts.append(k)
        keys = np.concatenate(parts)
        np.testing.assert_array_equal(pa.tie_sort(keys), _expected(pfref, keys))


def test_tie_sort_big_levels_and_fallback(pa, pfref):
    """Classes above the LDS size (kTieLocal, 14336 keys) go through the big levels (tile-parallel
    partitions) and, past them, the single-workgroup partitions in global memory: every level count
    gives std::sort's permutation."""
    rng = np.random.default_rng(23)
    cases = [rng.integers(0, 3000, 200000).astype(np.uint32),                   # tie-heavy
             rng.integers(0, 1 << 30, 150000).astype(np.uint32),
             np.sort(rng.integers(0, 50000, 120000)).astype(np.uint32),
             np.full(90000, 5, np.uint32)]
    m = np.sort(rng.integers(0, 60000, 80000)).astype(np.uint32)               # rgbds: map + new points
    cases.append(np.concatenate([m, rng.integers(0, 60000, 12000).astype(np.uint32)]))
    for keys in cases:
        want = _expected(pfref, keys)
        for levels in (0, 1, 2, 4):
            np.testing.assert_array_equal(pa.tie_sort(keys, levels=levels), want,
                                          err_msg="n=%d levels=%d" % (keys.size, levels))


def test_tie_sort_depth_limit_heap_branch(pa, pfref):
    """The depth-limit branch (libstdc++'s make_heap + sort_heap) on the device against the oracle's
    restatement with the same settable depth limit (itself checked against std::sort's own branch in
    tests/test_oracle_units.py): segments at the limit from every tier, in LDS and (30000 keys at depth 0,
    above the 20352 the LDS holds) on the global scratch copy. Keys drawn with repeats (the heap sort
    itself: a segment with an equal pair) and without (the bitonic network, kept when no two keys are
    equal: random, sorted and reversed permutations, in LDS and across the global copy's 16384-key
    chunks)."""
    rng = np.random.default_rng(24)
    cases = [rng.integers(0, max(2, n // 5), n).astype(np.uint32) for n in (17, 40, 300, 5000, 20000, 30000)]
    for n in (17, 33, 1000, 16384, 20352, 20353, 40000, 70001):
        perm = rng.permutation(n).astype(np.uint32) * 3
        cases += [perm, np.sort(perm), np.sort(perm)[::-1].copy()]
    cases.append(np.r_[rng.permutation(50000), 7, 7].astype(np.uint32))   # one equal pair in 50002
    for keys in cases:
        n = keys.size
        for depth in ((0, 1, 2, 3, 5) if n <= 30000 else (0, 2)):
            want = pfref.sort_perm(keys, "literal", depth)
            np.testing.assert_array_equal(pa.tie_sort(keys, depth=depth), want, err_msg="n=%d depth=%d" % (n, depth))


def test_tie_sort_natural_depth_limit(pa, pfref):
    """rgbds inputs reach libstdc++'s own depth limit: a voxel-ordered map with a few new points
    appended sends median-of-three to one end, level after level, and leaves segments of thousands of
    keys (up to nearly the whole map) to the heap sort (k_tie_heap: LDS up to 20352 keys, a global
    scratch copy above)."""
    rng = np.random.default_rng(25)
    for nmap, napp in ((22000, 100), (12000, 60), (22000, 3700), (40000, 900)):
        m = np.sort(rng.choice(1 << 24, nmap, replace=False))
        keys = np.concatenate([m, rng.choice(m, napp)]).astype(np.uint32)
        want = _expected(pfref, keys)
        for levels in (0, 2):
            np.testing.assert_array_equal(pa.tie_sort(keys, levels=levels), want,
                                          err_msg="map %d + %d levels=%d" % (nmap, napp, levels))


def test_tie_sort_huge_segments_radix_then_heap(pa, pfref):
    """Sorts with big levels send depth-limit segments above the LDS size (20352 keys) to one device-wide
    radix sort of all of them (pf_tie.hip k_huge_*): kept where a segment holds no equal pair (its only
    sorted order), else the segment keeps its input and the heap tier sorts it. Several huge segments in
    one sort (depth limit 2: four pieces), one of them with an equal pair, in two classes."""
    rng = np.random.default_rng(26)
    perm = (rng.permutation(200000) * 3).astype(np.uint32)
    dup = perm.copy()
    dup[10] = dup[11]                                           # one equal pair: that segment heap-sorts
    two = np.concatenate([perm[:90000], (perm[90000:] & 0x3FFFFFFF) | np.uint32(1 << 30)])
    for keys in (perm, dup, two):
        for depth in (0, 2):
            want = np.concatenate([np.nonzero((keys >> 30) == c)[0][pfref.sort_perm(keys[(keys >> 30) == c],
                                                                                     "literal", depth)]
                                   for c in range(4) if np.any((keys >> 30) == c)]).astype(np.uint32)
            np.testing.assert_array_equal(pa.tie_sort(keys, depth=depth, levels=4), want,
                                          err_msg="n=%d depth=%d" % (keys.size, depth))


def test_tie_sort_deep_big_levels(pa, pfref):
    """tie_levels_for gives a class above kTieMed its whole depth limit in big levels (a segment that
    peels a few keys per level stays above kTieMed for tens of levels): rgbds-like inputs, a voxel-ordered
    map of 400k keys with new points appended, at 40 big levels and at 2."""
    rng = np.random.default_rng(27)
    m = np.sort(rng.choice(1 << 26, 400000, replace=False))
    for napp in (200, 8000):
        keys = np.concatenate([m, rng.choice(m, napp)]).astype(np.uint32)
        want = _expected(pfref, keys)
        for levels in (2, 40):
            np.testing.assert_array_equal(pa.tie_sort(keys, levels=levels), want,
                                          err_msg="map 400000 + %d levels=%d" % (napp, levels))
