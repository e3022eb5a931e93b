"""Development probe: the reference-tie-order sort alone (pf_dev_tie_sort2) on synthetic key sets shaped
like the pipeline's (VoxelGrid input: ~13 points per voxel; rgbds: a voxel-ordered map plus appended
points). Run under rocprofv3 --kernel-trace; tools/tie_trace.py splits the trace per call.
    python3 tools/tie_time.py [levels]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
import pfilter_amd as pa  # noqa: E402

levels = int(sys.argv[1]) if len(sys.argv) > 1 else 2
rng = np.random.default_rng(5)


def vg(n, per, runs):
    """VoxelGrid-like: n keys over n / per voxels; runs > 1 keeps scan locality (runs of equal keys)"""
    nv = max(1, n // per)
    if runs <= 1:
        return rng.integers(0, nv, n).astype(np.uint32)
    k = np.repeat(rng.integers(0, nv, n // runs + 1), runs)[:n]
    return k.astype(np.uint32)


def rg(nmap, napp):
    m = np.sort(rng.choice(1 << 24, nmap, replace=False))
    a = rng.choice(m, napp) if napp else np.empty(0, np.int64)
    return np.concatenate([m, a]).astype(np.uint32)


cases = [("vg11k_rand", vg(11000, 13, 1)), ("vg14k_rand", vg(14000, 13, 1)), ("vg45k_rand", vg(45000, 13, 1)),
         ("vg45k_runs4", vg(45000, 13, 4)), ("distinct11k", rng.permutation(11000).astype(np.uint32)),
         ("rg22k+3.7k", rg(22000, 3700)), ("rg10k+3.3k", rg(10000, 3300))]
for name, keys in cases:
    for r in range(3):
        out = pa.tie_sort(keys, levels=levels)
        assert out.size == keys.size
    print("case", name, keys.size, flush=True)
