"""kNN-only workload for profiling the standalone kNN (k_knn_thick; --layout grid: k_knn_query) (config 5: 2M-point dense map, 200k queries).

  python3 tools/knn_probe.py [--iters N]
Prints avg kernel ms (HIP events) and algorithmic bytes per launch. Run under
`rocprofv3 --kernel-trace --stats` or one `--pmc` counter per pass (see tools/gpu_round.sh)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--nmap", type=int, default=2_000_000)
    ap.add_argument("--nq", type=int, default=200_000)
    ap.add_argument("--team", type=int, default=0, help="lanes per query, 1..16 (development hook; 0 = default)")
    ap.add_argument("--layout", type=int, default=1, help="1: thick-row layout (default), 0: 9-row grid walk")
    ap.add_argument("--order", default="stratified", choices=["stratified", "cell", "random"],
                    help="query order: generator's, sorted by 1 m cell, or shuffled")
    a = ap.parse_args()
    import pfilter_amd as pa
    import pfsynth
    mp = pfsynth.dense_map(a.nmap, seed=5)
    q = pfsynth.dense_queries(mp, a.nq, sigma=0.3, seed=6)
    import numpy as np
    if a.order == "cell":
        c = np.floor(q[:, :3]).astype(np.int64)
        q = q[np.lexsort((c[:, 0], c[:, 1], c[:, 2]))].copy()
    elif a.order == "random":
        q = q[np.random.default_rng(1).permutation(q.shape[0])].copy()
    kn = pa.Knn(a.nmap, a.nq)
    import ctypes
    assert pa.lib().pf_knn_set_layout(ctypes.c_void_p(kn._h), a.layout) == 0
    kn.set_map(mp)
    if a.team:
        import ctypes
        assert pa.lib().pf_knn_set_team(ctypes.c_void_p(kn._h), a.team) == 0
    kn.query(q)
    ms, alg = kn.bench(a.iters)
    print(json.dumps({"avg_kernel_ms": ms, "alg_bytes_per_launch": alg, "launches": a.iters + 2,
                      "achieved_GBps": alg / (ms * 1e-3) / 1e9, "team": a.team, "order": a.order, "layout": a.layout}))


if __name__ == "__main__":
    main()
