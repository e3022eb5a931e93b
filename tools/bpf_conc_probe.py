"""Development probe: does the BPF chain leave the GPU idle? K handles on K host threads, each running
the same HBM-resident S64 scans through pf_bpf_frame_scan_device; prints the aggregate frames/s and
each handle's stage A / B device time. If K = 2 gives much more than K = 1, a second stage-A stream per
handle (two frames' front ends at once) would too.
  python3 tools/bpf_conc_probe.py [frames] [reserve]"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
RES = int(sys.argv[2]) if len(sys.argv) > 2 else -1
seq = pfsynth.Sequence("S64", n_frames=N + 20, seed=0)
stride = 128000 * 16
scans = pa.DeviceBuffer(stride * (N + 20))
counts = []
buf, cnt = seq.frames(0, N + 20, threads=16)
for i in range(N + 20):
    scans.upload(np.ascontiguousarray(buf[i, :cnt[i]], np.float32), i * stride)
    counts.append(int(cnt[i]))


def make():
    od = pa.Odom_BPF_EstimationClass(device=0, max_points=300000, map_capacity=1 << 22)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    if RES >= 0:
        od.set_stage_a_reserve(RES)
    for k in range(20):
        od.frame_scan_device(scans.ptr + k * stride, counts[k])
    od.sync()
    return od


for K in (1, 2, 3):
    ods = [make() for _ in range(K)]
    for od in ods:
        od.set_stage_timing(True)

    def work(od):
        for k in range(20, N + 20):
            od.frame_scan_device(scans.ptr + k * stride, counts[k])
        od.sync()

    th = [threading.Thread(target=work, args=(od,)) for od in ods]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    st = [od.stage_times() for od in ods]
    print("K=%d reserve=%d: %.1f frames/s aggregate; stage A/B us per handle: %s" % (
        K, RES, K * N / el, ["%.0f/%.0f" % (x["a_us"], x["b_us"]) for x in st]), flush=True)
    del ods
