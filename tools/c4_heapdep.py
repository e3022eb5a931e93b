"""Development study (oracle only, CPU): configs[4]'s depth-limit segments, as bench.py's configs4 leg
runs it (S128 at 1 m/s, a 2M-point voxel_map surf map seeded after frame 0, theta 0, weightType 0).

Runs the faithful oracle (opts=0) with PFREF_GROUP_STATS (oracle/pfref_sort.cpp pfref_introsort_heapdep)
and prints, per sorted call of each frame, the number of depth-limit segments, how many hold an
order-dependent group, the pops those need (sum, max) and the length of the longest segment, by size class
(<= 2048 k_tie_local, <= 20350 the LDS heap, above: the global path or the radix route):
python tools/c4_heapdep.py [frames]
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def child(n):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
    import numpy as np
    import pfref
    import pfsynth
    seq = pfsynth.Sequence("S128", n_frames=n, speed=1.0)
    orc = pfref.Odom(pfref.make_lidar(128, 3.0, 90.0, ring_model=(15.0, -25.0)), 0.4, 0, 0.0, 0, 0, opts=0)
    for k in range(n):
        os.write(2, b"frame %d\n" % k)
        orc.frame(seq.frame(k))
        if k == 0:
            m = pfsynth.voxel_map(2_000_000, 0.8, seed=5)
            orc.set_map(1, m, np.zeros((m.shape[0], 2), np.uint8))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    if os.environ.get("C4_HEAPDEP_CHILD"):
        child(n)
        return
    env = dict(os.environ, PFREF_GROUP_STATS="1", C4_HEAPDEP_CHILD="1")
    p = subprocess.Popen([sys.executable, __file__, str(n)], env=env, stderr=subprocess.PIPE, text=True)
    rx = re.compile(r"heapdep (\w+) len (\d+) distinct \d+ depkeys (\d+) depgroups \d+ pops (\d+)")
    frame, calls = -1, {}

    def flush():
        for tag, segs in calls.items():
            for lo, hi, name in ((0, 2048, "<=2048"), (2049, 20350, "<=20350"), (20351, 1 << 40, ">20350")):
                s = [x for x in segs if lo <= x[0] <= hi]
                if not s:
                    continue
                d = [x for x in s if x[1] > 0]
                print("frame %2d %-8s %-8s segs %5d dep %5d pops sum %8d max %6d  longest %7d  dep-longest %7d"
                      % (frame, tag, name, len(s), len(d), sum(x[2] for x in d), max([x[2] for x in d] or [0]),
                         max(x[0] for x in s), max([x[0] for x in d] or [0])), flush=True)

    for line in p.stderr:
        if line.startswith("frame "):
            flush()
            frame, calls = int(line.split()[1]), {}
            continue
        m = rx.search(line)
        if m:
            calls.setdefault(m.group(1), []).append((int(m.group(2)), int(m.group(3)), int(m.group(4))))
    flush()
    p.wait()


if __name__ == "__main__":
    main()
