"""Development study (oracle only, CPU): where the rgbds tie sort's depth-limit segments come from.

Runs the faithful oracle (opts=0) over the configs[1] S64 sequence with PFREF_GROUP_STATS, which prints
every depth-limit segment of every sorted call with the pops its order-dependent groups need
(oracle/pfref_sort.cpp pfref_introsort_heapdep). The device's tiers (csrc/pf_tie.hip) take a segment by
its length when it reaches the depth limit: > 14336 keys in k_tie_medium, > 2048 in k_tie_mid, else in
k_tie_local; every one is heap-sorted after k_tie_local. Per frame this prints the largest pop count of
the rgbds calls by origin tier, so the saving of starting a tier's heaps as soon as that tier ends can be
estimated: python tools/heap_origin.py [frames] [first] > out.txt
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def child(n, first):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "pfilter-noetic_amd", "synth"))
    import pfref
    import pfsynth
    seq = pfsynth.Sequence("S64", n_frames=4541, seed=0)
    orc = pfref.Odom(pfref.make_lidar(64, 3.0, 90.0), 0.4, 0, 0.4, 75, 0, opts=0)
    for k in range(first + n):
        os.write(2, b"frame %d\n" % k)
        orc.frame(seq.frame(k))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4541
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    if os.environ.get("HEAP_ORIGIN_CHILD"):
        child(n, first)
        return
    env = dict(os.environ, PFREF_GROUP_STATS="1", HEAP_ORIGIN_CHILD="1")
    p = subprocess.Popen([sys.executable, __file__, str(n), str(first)], env=env, stderr=subprocess.PIPE, text=True)
    rx = re.compile(r"heapdep (\w+) len (\d+) distinct \d+ depkeys \d+ depgroups \d+ pops (\d+)")
    frame, cls = -1, {}
    rows = []

    def flush():
        if frame >= first:
            rg = [v for k, v in cls.items() if k.startswith("rg")]
            best = {"med": 0, "mid": 0, "loc": 0}
            for segs in rg:
                for ln, pops in segs:
                    t = "med" if ln > 14336 else ("mid" if ln > 2048 else "loc")
                    best[t] = max(best[t], pops)
            rows.append((frame, best["med"], best["mid"], best["loc"]))
            print("%d %d %d %d" % rows[-1], flush=True)

    calls = 0
    for line in p.stderr:
        if line.startswith("frame "):
            flush()
            frame = int(line.split()[1])
            cls, calls = {}, 0
            continue
        if line.startswith("groups "):
            calls += 1
            continue
        m = rx.match(line)
        if m:
            key = "%s%d" % (m.group(1), calls)
            cls.setdefault(key, []).append((int(m.group(2)), int(m.group(3))))
    flush()
    p.wait()


if __name__ == "__main__":
    main()
