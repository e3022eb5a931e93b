"""Development probe: ES pipeline frames/s and per-stage device time with the reference tie order off
and on (pf_odom_set_tie_order), same frames, same handle settings.  python3 tools/tie_probe.py [N]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
preset = sys.argv[2] if len(sys.argv) > 2 else "S64"
W = 20
seq = pfsynth.Sequence(preset, n_frames=N + W)
buf, cnt = seq.frames(0, N + W, threads=16)
db = pa.DeviceBuffer(buf.nbytes)
db.upload(buf)
ptrs = [(db.ptr + k * buf.shape[1] * 16, int(cnt[k])) for k in range(N + W)]


def run(tie, timing):
    od = pa.Odom_ES_EstimationClass(max_points=300000, map_capacity=1 << 22)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    od.set_graph(4)
    od.set_tie_order(tie)
    for k in range(W):
        od.frame_device(*ptrs[k])
    od.sync()
    if timing:
        od.set_stage_timing(True)
    t0 = time.perf_counter()
    for k in range(W, N + W):
        od.frame_device(*ptrs[k])
    od.sync()
    el = time.perf_counter() - t0
    st = od.stats()
    assert st["errors"] == 0
    out = {"tie": tie, "fps": round(N / el, 1), "n_map": st["n_map"], "n_ds": st["n_ds"]}
    if timing:
        s = od.stage_times()
        out.update(a_us=round(s["a_us"], 1), b_us=round(s["b_us"], 1))
    return out, od.poses()


modes = (True,) if len(sys.argv) > 3 and sys.argv[3] == "tie" else (False, True, False, True)
for tie in modes:
    r, p = run(tie, False)
    r2, _ = run(tie, True)
    r.update({k: r2[k] for k in ("a_us", "b_us")})
    print(r, flush=True)
