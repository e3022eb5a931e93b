"""CPU: the curvedVoxel (DCVC) oracle (oracle/pfref_dcvc.cpp) against an independent pure-Python
transcription of src/additionClass.cpp:85-372 executed serially, and against known geometry.

The reference's loops run under OpenMP with shared temporaries (its output is not a function of its
input); the serial execution is the deterministic reading restated in both places. Equal-size clusters
are ordered by their first point (the reference's order there comes from an unordered_map: unpinned)."""
import math

import numpy as np


def _py_dcvc(P, startR=1.0, deltaR=0.003, deltaP=1.2, deltaA=1.2, minSeg=80, minR=1.0, maxR=120.0, first=False):
    n = len(P)
    polar = [(0.0, 0.0, 0.0)] * n
    minPitch = maxPitch = 0.0
    minPolar = maxPolar = 5.0 if first else 0.0
    for i in range(n):                                           # convertToPolar (:85-136)
        x, y, z = (float(v) for v in P[i])
        r = math.sqrt((x * x + y * y) + z * z)
        pitch = math.asin(z / r) * 180.0 / math.pi if r > 0 else 0.0
        ang = math.atan2(y, x)
        az = ang * 180 / math.pi if ang > 0.0 else (ang + 2 * math.pi) * 180 / math.pi
        if r >= maxR or r <= minR:
            continue
        minPitch, maxPitch = min(minPitch, pitch), max(maxPitch, pitch)
        minPolar, maxPolar = min(minPolar, r), max(maxPolar, r)
        polar[i] = (r, pitch, az)
    width = int(round(360.0 / deltaA) + 1)
    height = int((maxPitch - minPitch) / deltaP)
    bounds, rng, step = [], minPolar, 1
    while rng <= maxPolar:
        rng += (startR - step * deltaR)
        bounds.append(rng)
        step += 1
    PN = len(bounds)

    def pidx(r):
        for k in range(PN):
            if r < bounds[k]:
                return k
        return PN - 1

    def rnd(v):                                                  # std::round: half away from zero
        return int(math.floor(v + 0.5)) if v >= 0 else -int(math.floor(-v + 0.5))
    vox, vmap = [], {}
    for i in range(n):                                           # createHashTable (:143-177)
        r, pitch, az = polar[i]
        v = (pidx(r), rnd((pitch - minPitch) / deltaP), rnd(az / deltaA))
        vox.append(v)
        vmap.setdefault((v[2] * (PN + 1) + v[0]) + v[1] * (PN + 1) * (width + 1), []).append(i)
    lab = [-1] * n
    count = 0
    for i in range(n):                                           # voxelFilter (:232-318)
        if lab[i] != -1:
            continue
        p0, z0, a0 = vox[i]
        nb = []
        for z in (z0 - 1, z0, z0 + 1):                           # searchKNN (:196-225)
            if z < 0 or z > height:
                continue
            for y in (p0 - 1, p0, p0 + 1):
                if y < 0 or y > PN:
                    continue
                for x in (a0 - 1, a0, a0 + 1):
                    ax = width - 1 if x < 0 else x
                    ax = 300 if ax > 300 else ax
                    nb += vmap.get((ax * (PN + 1) + y) + z * (PN + 1) * (width + 1), [])
        for j in nb:
            cur, nei = lab[i], lab[j]
            if cur != -1 and nei != -1 and cur != nei:
                lab = [nei if s == cur else s for s in lab]
            elif nei != -1:
                lab[i] = nei
            elif cur != -1:
                lab[j] = cur
        if lab[i] == -1:
            count += 1
            lab[i] = count
            for j in nb:
                lab[j] = count
    groups = {}
    for i in range(n):
        groups.setdefault(lab[i], []).append(i)
    kept = sorted((g for g in groups.values() if len(g) > minSeg), key=lambda g: (-len(g), g[0]))
    out, label = [], np.zeros(n, np.int32)
    for c, g in enumerate(kept):
        out += g
        label[g] = c + 1
    return np.array(out, np.int32), label


def _scene(seed=0):
    rng = np.random.default_rng(seed)
    parts = [rng.normal([15, 0, 0.5], [0.3, 0.3, 0.5], (300, 3)),          # a bush
             rng.normal([-8, 6, 1.0], [0.1, 0.1, 1.0], (150, 3)),          # a pole
             rng.normal([0, -25, 2.0], [2.0, 0.05, 1.5], (400, 3)),        # a wall
             rng.normal([40, 40, 0.0], 0.5, (30, 3)),                      # a small blob (dropped at 80)
             [[0.1, 0.2, 0.0], [0.5, 0.1, 0.1], [150.0, 0.0, 0.0]]]        # out of range
    return np.concatenate(parts).astype(np.float32)


def test_dcvc_matches_python_transcription(pfref):
    for seed in range(3):
        P = _scene(seed)
        for first in (False, True):
            for min_seg in (80, 5):
                idx, lab = pfref.dcvc(P, pfref.dcvc_params(min_seg=min_seg), first_frame=first)
                pidx, plab = _py_dcvc(P, minSeg=min_seg, first=first)
                np.testing.assert_array_equal(idx, pidx)
                np.testing.assert_array_equal(lab, plab)


def test_dcvc_known_geometry(pfref):
    P = _scene(1)
    idx, lab = pfref.dcvc(P)
    assert set(np.unique(lab[:850])) - {0} and lab[850:880].max() == 0      # the 30-point blob is dropped
    sizes = np.bincount(lab[lab > 0])[1:]
    assert np.all(np.diff(sizes) <= 0)                                      # largest cluster first
    assert len(idx) == (lab > 0).sum() and np.all(np.diff(idx[lab[idx] == 1]) > 0)   # input order inside
    cidx, clab = pfref.dcvc(P, components=True)                            # components: never finer
    for c in np.unique(lab[lab > 0]):
        assert len(np.unique(clab[(lab == c) & (clab > 0)])) <= 1


def test_dcvc_curvedfilter_chain(pfref, pfsynth):
    x = pfsynth.Sequence("S32", n_frames=2, az_steps=600).frame(1)
    plain = pfref.bpf_preprocess(x)
    with_dc = pfref.bpf_preprocess(x, dcvc=pfref.dcvc_params())
    np.testing.assert_array_equal(plain["ground"], with_dc["ground"])
    assert sum(len(with_dc[k]) for k in ("beam", "pillar", "facade")) > 0
