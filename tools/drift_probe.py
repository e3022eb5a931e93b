"""CPU experiment (oracle only): how a difference of ~1e-12 m in the LM's linear algebra grows along a
free run of the faithful estimator (the S64T free run reaches 4.8e-5 m before a
count flips at frame 338 while synced frames differ by <= 2.7e-12 m). Runs the faithful oracle (opts=0:
std::sort ties, Householder-QR LM, kd-tree) and the same oracle with the normal-equation LDL^T step the
device takes (LM_NORMAL_EQ) side by side over the same frames, and prints the per-frame pose
difference and the first frame whose counts differ. Variant "ldtrig" instead perturbs only the libm:
the LM's sin / cos / cubes taken in long double and rounded once (PFREF_LD_TRIG), which differs from
glibc's double sin in the last bit now and then, as another C library would; "qrrev" keeps the QR
but sums its rows in reverse order (another QR implementation's rounding); "quad" is the device's
LM (LM_NORMAL_EQ) with its normal equations formed and solved in binary128; "costrev" is the faithful
LM with only its cost sums taken in reverse order; "devlibm" the device's LM with libm's sin / cos in its
SE(3) updates ("devlibmquad": and binary128 normal equations); "devhalf" the device's LM with round 3's
half-angle SE(3) update (2 sin^2(theta/2), 2 s c) instead of the reference's 1 - cos(theta),
theta - sin(theta): the variant that separates at frame 338 ("normaleq" is now the device's LM as it is,
in the reference's form).
    python3 tools/drift_probe.py [preset] [frames] [out.json] [variant]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "pfilter-noetic_amd", "synth"),
                os.path.join(ROOT, "tests")]
import pfref  # noqa: E402
import pfsynth  # noqa: E402
from _util import pose_err  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 else "S64T"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
out = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "-" else None
variant = sys.argv[4] if len(sys.argv) > 4 else "normaleq"
seq = pfsynth.Sequence(preset, n_frames=n)
lid = pfref.make_lidar(64, 3.0, 90.0)
a = pfref.Odom(lid, 0.4, 0, 0.4, 75, 0, opts=0)
b = pfref.Odom(lid, 0.4, 0, 0.4, 75, 0, opts={"normaleq": pfref.LM_NORMAL_EQ, "ldtrig": pfref.LD_TRIG,
                                               "qrrev": pfref.QR_REVSUM,
                                               "quad": pfref.LM_NORMAL_EQ | pfref.LM_QUAD,
                                               "costrev": pfref.COST_REVSUM,
                                               "devlibm": pfref.LM_NORMAL_EQ | pfref.DEV_LIBM,
                                               "devlibmquad": pfref.LM_NORMAL_EQ | pfref.DEV_LIBM | pfref.LM_QUAD,
                                               "devhalf": pfref.LM_NORMAL_EQ | pfref.DEV_HALFANGLE}[variant])
keys = ("n_edge_ds", "n_surf_ds", "n_edge_map", "n_surf_map", "n_edge_res", "n_surf_res", "outer_iterations",
        "lm_iterations")
rows, first_count = [], None
for k in range(n):
    x = seq.frame(k)
    pa_, pb = a.frame(x), b.frame(x)
    dt, dr = pose_err(pa_, pb)
    sa, sb = a.stats(), b.stats()
    diff = [c for c in keys if sa[c] != sb[c]]
    if diff and first_count is None:
        first_count = (k, {c: (sa[c], sb[c]) for c in diff})
    rows.append((k, dt, dr, len(diff)))
    if k % 25 == 0 or (diff and first_count[0] == k):
        print("frame %4d  dt %.3e m  dr %.3e rad  counts differ: %s" % (k, dt, dr, diff), flush=True)
first_jump = next((r for r in rows if r[1] > 1e-9), None)
res = {"preset": preset, "frames": n, "variant": variant, "first_frame_dt_above_1e-9": first_jump, "first_count_difference": first_count,
       "dt_at": {str(k): rows[k][1] for k in (1, 10, 50, 100, 200, 300, n - 1) if k < n},
       "max_dt_before_count_flip": max((r[1] for r in rows if first_count is None or r[0] < first_count[0]),
                                       default=0.0)}
print(json.dumps(res))
if out:
    with open(out, "w") as f:
        json.dump(dict(res, per_frame=rows), f)
