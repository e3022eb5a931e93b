"""Development study: the pipelined pop schedule of the heap tier on real depth-limit segments.
Reads segments dumped by the oracle (PFREF_HEAP_DUMP=<file>: int32 len, int32 pops, len keys, as each
segment reaches libstdc++'s heap sort) and replays __make_heap + __sort_heap sequentially to get every
pop's sift path, then schedules the pops as the device does: pop j starts >= 2 steps after pop j - 1 and
not while an earlier pop's hole is q_j (its value's position) or an ancestor of q_j.
    python3 tools/heap_sched.py <dump> [max segments]"""
import sys
import numpy as np


def sift_paths(keys, npops):
    a = list(keys)
    n = len(a)

    def sift(h, v, m):                       # top-down form of __adjust_heap + __push_heap
        path = [h]
        while True:
            c = 2 * h + 1
            if c >= m:
                break
            if c + 1 < m and not (a[c + 1] < a[c]):
                c += 1
            if a[c] < v:
                break
            a[h] = a[c]
            h = c
            path.append(h)
        a[h] = v
        return path

    for p in range((n - 2) // 2, -1, -1):
        sift(p, a[p], n)
    paths = []
    for j in range(npops):
        q = n - 1 - j
        v = a[q]
        a[q] = a[0]
        paths.append(sift(0, v, q))
    return paths


def anc_or_self(x, q):
    x += 1
    q += 1
    while q > x:
        q >>= 1
    return q == x


def schedule(paths, n, rule):
    """rule 'pair': starts on even steps only (the shipped engine); 'any': any step >= 2 after the last
    start; 'ideal': 'any', blocked only by a pop whose remaining path writes q_j"""
    starts = []
    t = 0
    blocked = 0
    for j, pj in enumerate(paths):
        q = n - 1 - j
        t = t if not starts else max(t, starts[-1] + 2)
        if rule == "pair" and t % 2:
            t += 1
        while True:
            blk = False
            for i in range(max(0, j - 32), j):
                d = t - starts[i]
                pi = paths[i]
                if d >= len(pi):
                    continue
                if rule == "ideal":
                    if q in pi[d:]:
                        blk = True
                        break
                elif anc_or_self(pi[d], q):
                    blk = True
                    break
            if not blk:
                break
            blocked += 1
            t += 2 if rule == "pair" else 1
        starts.append(t)
    end = max(s + len(p) for s, p in zip(starts, paths))
    return end, blocked


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.int32)
    lim = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    off = 0
    tot = {"pair": 0, "any": 0, "ideal": 0}
    npop_tot = 0
    seg = 0
    while off < len(raw) and seg < lim:
        n, pops = int(raw[off]), int(raw[off + 1])
        keys = raw[off + 2: off + 2 + n].view(np.uint32).tolist()
        off += 2 + n
        pops = min(pops, n - 1)
        paths = sift_paths(keys, pops)
        res = {r: schedule(paths, n, r) for r in tot}
        L = np.mean([len(p) for p in paths])
        asc = np.mean(np.diff(np.array(keys, dtype=np.int64)) >= 0)
        print("seg %3d n %6d pops %6d  mean path %.1f  ascending pairs %.2f  steps/pop: pair %.2f any %.2f ideal %.2f"
              % (seg, n, pops, L, asc, res["pair"][0] / pops, res["any"][0] / pops, res["ideal"][0] / pops), flush=True)
        for r in tot:
            tot[r] += res[r][0]
        npop_tot += pops
        seg += 1
    print("total: " + "  ".join("%s %.2f" % (r, tot[r] / npop_tot) for r in tot))


if __name__ == "__main__":
    main()
