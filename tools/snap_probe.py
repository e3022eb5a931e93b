"""Development probe: a window of the headline sequence from a saved estimator state, so that a profiler
pass covers late frames without profiling (or wrapping the AQL ring with) the frames before them.

  python3 tools/snap_probe.py save K FILE          frames 0 .. K-1 (S64 seed 0, configs[1], library
                                                  default order), then pf_odom_snapshot -> FILE
  python3 tools/snap_probe.py run K N FILE [eager] pf_odom_restore FILE into a fresh handle, then frames
                                                  K .. K+N-1 (eager launches with "eager")"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd"))
sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
import pfilter_amd as pa  # noqa: E402
import pfsynth  # noqa: E402


def handle():
    od = pa.Odom_ES_EstimationClass(max_points=300000, map_capacity=1 << 22)
    od.init(pa.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0)
    return od


def frames(k0, n):
    seq = pfsynth.Sequence("S64", n_frames=k0 + n, seed=0)
    buf, cnt = seq.frames(k0, n, threads=16)
    db = pa.DeviceBuffer(buf.nbytes)
    db.upload(buf)
    return db, [(db.ptr + i * buf.shape[1] * 16, int(cnt[i])) for i in range(n)]


def main():
    mode = sys.argv[1]
    if mode == "save":
        k, path = int(sys.argv[2]), sys.argv[3]
        od = handle()
        for f0 in range(0, k, 256):
            db, ptrs = frames(f0, min(256, k - f0))
            for p in ptrs:
                od.frame_device(*p)
            od.sync()
            db.free()
        with open(path, "wb") as f:
            f.write(od.snapshot())
        print("saved state after %d frames: %s" % (k, path))
    else:
        k, n, path = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
        od = handle()
        if len(sys.argv) > 5 and sys.argv[5] == "eager":
            od.set_graph(0)
        od.restore(open(path, "rb").read())
        db, ptrs = frames(k, n)
        t0 = time.perf_counter()
        for p in ptrs:
            od.frame_device(*p)
        od.sync()
        el = time.perf_counter() - t0
        assert od.stats()["errors"] == 0
        print("frames %d..%d from the snapshot: %.1f frames/s" % (k, k + n - 1, n / el))


if __name__ == "__main__":
    main()
