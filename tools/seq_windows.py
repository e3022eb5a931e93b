"""Development probe: the headline sequence (S64 seed 0, configs[1]) through pf_odom_frame_device in
windows of W frames; per window the wall time (synchronised at the window's end) and the mean stage
A / B device time (pf_odom_set_stage_timing, reset per window), so that the full-sequence rate can be
attributed to the frames that cost it.
  python3 tools/seq_windows.py [frames] [window] [tie|stable] [PF_DUMP_MAPS path]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4541
WIN = int(sys.argv[2]) if len(sys.argv) > 2 else 500
ORDER = sys.argv[3] if len(sys.argv) > 3 else "tie"
WARM = 20
seq = pfsynth.Sequence("S64", n_frames=N, seed=0)
bufs, ptrs = [], []
for f0 in range(0, N, 256):
    nf = min(256, N - f0)
    buf, cnt = seq.frames(f0, nf, threads=16)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    ptrs += [(db.ptr + i * buf.shape[1] * 16, int(cnt[i])) for i in range(nf)]
    bufs.append(db)
od = pa.Odom_ES_EstimationClass(max_points=300000, map_capacity=1 << 22)
od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
od.set_tie_order(ORDER == "tie")
for k in range(WARM):
    od.frame_device(*ptrs[k])
od.sync()
if len(sys.argv) > 4:
    with open("/proc/self/maps") as f, open(sys.argv[4], "w") as g:
        g.write(f.read())
rows = []
t_all = 0.0
for w0 in range(WARM, N, WIN):
    w1 = min(N, w0 + WIN)
    od.set_stage_timing(True)
    t0 = time.perf_counter()
    for k in range(w0, w1):
        od.frame_device(*ptrs[k])
    od.sync()
    el = time.perf_counter() - t0
    t_all += el
    s = od.stage_times()
    st = od.stats()
    r = {"frames": [w0, w1 - 1], "fps": round((w1 - w0) / el, 1), "a_us": round(s["a_us"], 1),
         "b_us": round(s["b_us"], 1), "n_map": st["n_map"], "n_ds": st["n_ds"]}
    rows.append(r)
    print(json.dumps(r), flush=True)
assert od.stats()["errors"] == 0
print(json.dumps({"order": ORDER, "frames": N - WARM, "fps_windows": round((N - WARM) / t_all, 1)}), flush=True)
