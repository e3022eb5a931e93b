"""Development: bisect the BPF create-after-edge-cases hang. python3 tools/repro_bpf_create.py <variant>"""
import ctypes, faulthandler, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd")); sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
import pfilter_amd as pa, pfsynth
faulthandler.dump_traceback_later(40, exit=True)
v = sys.argv[1]
od = pa.Odom_BPF_EstimationClass(device=0, max_points=200000)
od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
buf = pa.DeviceBuffer(16 * 200000)
x = pfsynth.Sequence("S64", n_frames=2, az_steps=800).frame(0)
buf.upload(x)
od.frame_scan_device(buf.ptr, x.shape[0])
print("seeded", flush=True)
if v in ("all", "n0"):
    pose = np.empty(7); print("n0 rc", pa.lib().pf_bpf_frame_scan_device(od._h, buf.ptr, 0, pose.ctypes.data), flush=True)
if v in ("all", "n5"):
    pose = np.empty(7); print("n5 rc", pa.lib().pf_bpf_frame_scan_device(od._h, buf.ptr, 5, pose.ctypes.data), flush=True)
if v in ("all", "cap"):
    print("cap rc", pa.lib().pf_bpf_frame_scan_device(od._h, buf.ptr, 200001, None), flush=True)
print("stats", od.stats()["errors"], flush=True)
del od, buf
print("destroyed", flush=True)
od2 = pa.Odom_BPF_EstimationClass(device=0)
od2.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
print("created OK", flush=True)
