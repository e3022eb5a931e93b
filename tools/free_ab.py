"""Development: tests/test_gpu_parity_free.py's free run with handle options, to bisect a parity change.
  python3 tools/free_ab.py NAME PRESET fuse(0/1, -1 = leave) graph_mode(-1 = leave) [tie(0/1)]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402
import test_gpu_parity_free as tf  # noqa: E402

name, preset, fuse, gm = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
tie = int(sys.argv[5]) if len(sys.argv) > 5 else 1
Base = pa.Odom_ES_EstimationClass


class Opt(Base):
    def init(self, *a, **k):
        r = super().init(*a, **k)
        if fuse >= 0:
            self.set_fuse_observe(bool(fuse))
        if gm >= 0:
            self.set_graph(gm)
        return r


pa.Odom_ES_EstimationClass = Opt
rep = tf.free_run(pa, pfsynth, name, preset, (0.4, 75), tie_order=bool(tie))
print("fuse", fuse, "graph", gm, "->", rep["bit_identical_frames"], rep["worst_m_before_first_count_mismatch"],
      rep["first_count_mismatch"], flush=True)
