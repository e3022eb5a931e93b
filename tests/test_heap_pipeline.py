"""CPU: the schedule k_tie_heap runs __sort_heap's pops on (csrc/pf_tie.hip heap_step), restated in
Python and checked against libstdc++'s heap sort (the oracle's line-by-line __make_heap + __sort_heap,
pfref.sort_perm(keys, "literal", depth=0): introsort whose depth limit is 0 heap-sorts the whole input).

The device pipelines the pops: each pop is a top-down sift (take the larger child, the right one unless
right < left; stop when it is less than the value), which equals __adjust_heap + __push_heap on a valid
heap; every pop in flight moves one tree level per step, reads happen before the step's writes, a pop
may start only on the first step of a pair and only while no hole in flight is its last element q or an
ancestor of q. The keys are compared as the device does: the low 30 bits << 1, the right child's + 1
under one max (ties to the right). This test runs the same schedule lane by lane."""
import numpy as np

NL = 64


def hlev(x):
    return (x + 1).bit_length() - 1


def make_heap(H, n):
    """__make_heap as the device runs it: a tree level at a time, top-down sifts"""
    for L in range(hlev((n - 2) // 2), -1, -1):
        for x in range((1 << L) - 1, min((2 << L) - 2, (n - 2) // 2) + 1):
            vk, h = H[x], x
            while 2 * h + 1 < n:
                c = 2 * h + 1
                if c + 1 < n and not (H[c + 1][0] < H[c][0]):
                    c += 1
                if H[c][0] < vk[0]:
                    break
                H[h] = H[c]
                h = c
            H[h] = vk


def pipelined_sort_heap(H, n, npops=None):
    """the first npops pops (default all, n - 1) of __sort_heap as heap_step schedules them"""
    last = n - 1
    npops = last if npops is None else npops
    act = [0] * NL
    h = [0] * NL
    m = [0] * NL
    vk = [None] * NL
    nxt = 0
    steps = 0

    def step(may):
        nonlocal nxt
        reads = {}
        for i in range(NL):                            # children of every hole (before this step's writes)
            if act[i]:
                c1 = 2 * h[i] + 1
                reads[i] = (c1, H[c1] if c1 < m[i] else None, H[c1 + 1] if c1 + 1 < m[i] else None)
        start = None
        if may and nxt < npops:
            q = last - nxt
            blk = False
            for i in range(NL):
                if act[i]:
                    sh = hlev(q) - hlev(h[i])
                    blk |= sh >= 0 and ((q + 1) >> sh) == h[i] + 1
            if not blk:
                s = nxt & (NL - 1)
                assert not act[s]
                vq, r0 = H[q], H[0]
                act[s], h[s], m[s], vk[s] = 1, 0, q, vq
                reads[s] = (1, H[1] if 1 < q else None, H[2] if 2 < q else None)
                start = (q, r0)
                nxt += 1
        writes = []
        for i, (c1, a, b) in reads.items():
            has = a is not None
            ak = (a[0] & 0x3FFFFFFF) << 1 if has else 0
            bk = (((b[0] & 0x3FFFFFFF) << 1) | 1) if b is not None else 0
            mx = max(ak, bk)
            right = mx & 1
            ch = (b if right else a) if has else None
            stop = (not has) or (mx ^ right) < ((vk[i][0] & 0x3FFFFFFF) << 1)
            writes.append((h[i], vk[i] if stop else ch))
            if stop:
                act[i] = 0
            else:
                h[i] = c1 + right
        if start:
            H[start[0]] = start[1]
        for pos, v in writes:
            H[pos] = v

    while True:
        step(True)
        step(False)
        steps += 2
        if nxt >= npops and not any(act):
            return steps


def device_heap_perm(keys):
    n = keys.size
    H = [(int(k), i) for i, k in enumerate(keys)]
    if n >= 2:
        make_heap(H, n)
        pipelined_sort_heap(H, n)
    return np.array([v for _, v in H], np.uint32)


def test_pipelined_heap_equals_libstdcxx(pfref):
    rng = np.random.default_rng(31)
    for trial in range(60):
        n = int(rng.choice([17, 18, 31, 64, 65, 100, 257, 500, 1200]))
        span = int(rng.choice([2, 5, 40, 1000, 1 << 30]))
        keys = rng.integers(0, span, n).astype(np.uint32)
        if trial % 5 == 0:
            keys = np.sort(keys)
        elif trial % 5 == 1:
            keys = np.sort(keys)[::-1].copy()
        want = pfref.sort_perm(keys, "literal", 0)
        np.testing.assert_array_equal(device_heap_perm(keys), want, err_msg="trial %d n=%d span=%d" % (trial, n, span))


def test_pipelined_heap_keeps_class_bits_out_of_the_compare(pfref):
    """a segment lies in one class (key bits 30-31): comparing the low 30 bits orders it the same"""
    rng = np.random.default_rng(32)
    keys = (rng.integers(0, 300, 700).astype(np.uint32) | np.uint32(2 << 30))
    np.testing.assert_array_equal(device_heap_perm(keys), pfref.sort_perm(keys, "literal", 0))


# the round-5 LDS engine (pf_tie.hip lds_pops / lds_pop_step_a / lds_pop_step_b), restated lane by lane:
# entries {position, key + 1}; H[n], H[n + 1] sentinels {_, 0}; a pop that starts writes {root's position,
# 0} at q (so the popped element keeps its name and reads as absent); the children of any hole h are read
# at min(2h + 1, n); idle lanes park on spare holes n + 2 + lane (children: the sentinels) with a value of
# key 1, so they stop every step; a pop may start only in the first step of a pair, by its own lane, with
# the value H[q] and the root's position prefetched after the previous pair's second step; the block mask
# for the next start is the second step's: not stopped, and the chosen child (right on !(b < a)) is q or
# an ancestor of q, q being the next pop's position
def _anc_or_self(x, q):
    x += 1
    q += 1
    while q > x:
        q >>= 1
    return q == x


def lds_pops_restated(keys, npops=None):
    n = keys.size
    last = n - 1
    npops = last if npops is None else npops
    H = [(i, int(k) + 1) for i, k in enumerate(keys)] + [(0, 0), (0, 0)] + [(0, 0)] * NL
    # __make_heap on key + 1 (the same order)
    for L in range(hlev((n - 2) // 2), -1, -1) if n >= 2 else []:
        for x in range((1 << L) - 1, min((2 << L) - 2, (n - 2) // 2) + 1):
            vk, h = H[x], x
            while 2 * h + 1 < n:
                c = 2 * h + 1
                if c + 1 < n and not (H[c + 1][1] < H[c][1]):
                    c += 1
                if H[c][1] < vk[1]:
                    break
                H[h] = H[c]
                h = c
            H[h] = vk
    spare = [n + 2 + l for l in range(NL)]
    h = list(spare)
    v = [(0, 1)] * NL
    nxt, blk = 0, 0
    vq, rp = H[last], H[0][0]

    def step(mine):
        """every lane one level; mine: the lane starting a pop this step (or None); returns the lanes whose
        new hole is q' or an ancestor of q' (q' = the next pop's position)"""
        if mine is not None:                          # the start, before the step's loads
            H[last - nxt] = (rp, 0)
            h[mine], v[mine] = 0, vq
        q2 = last - (nxt + (1 if mine is not None else 0))
        reads = []
        for l in range(NL):
            c1 = min(2 * h[l] + 1, n)
            reads.append((c1, H[c1], H[c1 + 1]))
        out = []
        for l in range(NL):
            c1, a, b = reads[l]
            right = not (b[1] < a[1])
            ch = b if right else a
            stop = ch[1] < v[l][1]
            H[h[l]] = v[l] if stop else ch
            child = 2 * h[l] + 1 + (1 if right else 0)
            out.append((not stop) and _anc_or_self(child, q2))
            h[l] = spare[l] if stop else child
        return any(out)

    steps = 0
    while True:
        for _ in range(4):
            start = nxt < npops and not blk
            step((nxt & (NL - 1)) if start else None)
            nxt += 1 if start else 0
            blk = step(None)
            vq, rp = H[last - nxt] if nxt <= last else (0, 0), H[0][0]
            steps += 2
        if nxt >= npops and all(h[l] == spare[l] for l in range(NL)):
            return H[:n], steps


def test_lds_engine_equals_libstdcxx(pfref):
    rng = np.random.default_rng(41)
    for trial in range(40):
        n = int(rng.choice([2, 3, 17, 18, 64, 65, 100, 257, 700]))
        span = int(rng.choice([2, 5, 40, 1000, 1 << 30]))
        keys = rng.integers(0, span, n).astype(np.uint32)
        if trial % 5 == 0:
            keys = np.sort(keys)
        elif trial % 5 == 1:
            keys = np.sort(keys)[::-1].copy()
        H, steps = lds_pops_restated(keys)
        got = np.array([p for p, _ in H], np.uint32)              # output positions (values = indices)
        want = pfref.sort_perm(keys, "literal", 0)
        np.testing.assert_array_equal(got, want, err_msg="trial %d n=%d span=%d" % (trial, n, span))
        assert steps <= 8 * n + 16


def test_lds_engine_partial_pops(pfref):
    """npops < n - 1: the popped tail is __sort_heap's after that many pops (pop_heap repeated)"""
    rng = np.random.default_rng(42)
    for trial in range(20):
        n = int(rng.choice([40, 200, 600]))
        keys = rng.integers(0, int(rng.choice([7, 300])), n).astype(np.uint32)
        npops = int(rng.integers(1, n - 1))
        H, _ = lds_pops_restated(keys, npops)
        want = pfref.sort_perm(keys, "literal", 0)                 # the full heap sort's order
        got_tail = [p for p, _ in H[n - npops:]]
        # the popped tail of a full heap sort is the same after npops pops (the later pops leave it alone)
        np.testing.assert_array_equal(np.array(got_tail, np.uint32), want[n - npops:], err_msg="trial %d" % trial)
        assert all(k == 0 for _, k in H[n - npops:])             # popped positions hold the sentinel key


# k_tie_heap's distinct-key path (pf_tie.hip lds_bitonic / glb_bitonic): the flip-form bitonic network
# with positions past the segment's end left out (+inf), run whole (LDS) or as chunks of C positions
# with the cross-chunk steps on the global copy; restated to check the index arithmetic at small C
def _p2(n):
    return 1 if n <= 1 else 1 << (n - 1).bit_length()


def _ce_step(S, nv, P, j, flip):
    for c in range(P >> 1):
        i = ((c & ~(j - 1)) << 1) | (c & (j - 1))
        q = (i ^ flip) if flip else i + j
        if q < nv and S[q][0] < S[i][0]:
            S[i], S[q] = S[q], S[i]


def _lds_bitonic(S, nv, P, k0, k1, jtop):
    if k0 == 0:
        j = jtop
        while j >= 1:
            _ce_step(S, nv, P, j, 0)
            j >>= 1
        return
    k = k0
    while k <= k1:
        _ce_step(S, nv, P, k >> 1, k - 1)
        j = k >> 2
        while j >= 1:
            _ce_step(S, nv, P, j, 0)
            j >>= 1
        k <<= 1


def _glb_bitonic(G, n, C):
    P = _p2(n)
    Pc = min(P, C)
    kk = 0
    while kk == 0 or (2 * C << (kk - 1)) <= P:
        k = 0 if kk == 0 else C << kk
        if k:
            _ce_step(G, n, P, k >> 1, k - 1)
            j = k >> 2
            while j >= C:
                _ce_step(G, n, P, j, 0)
                j >>= 1
        for c0 in range(0, n, C):
            nv = min(C, n - c0)
            S = G[c0:c0 + nv]
            if k:
                _lds_bitonic(S, nv, Pc, 0, 0, C >> 1)
            else:
                _lds_bitonic(S, nv, Pc, 2, Pc, 0)
            G[c0:c0 + nv] = S
        kk += 1


def test_bitonic_network_equals_heap_sort_on_distinct_keys(pfref):
    rng = np.random.default_rng(33)
    for n in (17, 33, 100, 129, 257, 600, 1025):
        for C in (16, 64, 4096):
            keys = (rng.permutation(n) * 5).astype(np.uint32)
            G = [(int(k), i) for i, k in enumerate(keys)]
            if C == 4096:
                _lds_bitonic(G, n, _p2(n), 2, _p2(n), 0)
            else:
                _glb_bitonic(G, n, C)
            got = np.array([v for _, v in G], np.uint32)
            np.testing.assert_array_equal(got, pfref.sort_perm(keys, "literal", 0), err_msg="n=%d C=%d" % (n, C))




# ---- k_tie_heap's pops with the dependence flags (pf_tie.hip heap_segment_pairs) ----------------------
# Only the pops down to the smallest key with an order-dependent element run; the rest of the heap is
# sorted by any order. Without flags every key with an equal neighbour counts (the exact permutation).
def segment_perm(keys, dep=None):
    n = keys.size
    sk = np.sort(keys)
    if dep is None:
        depk = [k for i, k in enumerate(sk) if (i > 0 and sk[i - 1] == k) or (i + 1 < n and sk[i + 1] == k)]
    else:
        depk = [int(keys[i]) for i in range(n) if dep[i]]
    if not depk:
        return np.argsort(keys, kind="stable").astype(np.uint32), 0
    kmin = min(depk)
    popsneed = int(np.sum(keys >= kmin))
    H = [(int(k), i) for i, k in enumerate(keys)]
    make_heap(H, n)
    npops = n - 1 if popsneed >= n else popsneed
    pipelined_sort_heap(H, n, npops)
    if npops < n - 1:
        H[:n - npops] = sorted(H[:n - npops])
    return np.array([v for _, v in H], np.uint32), npops


def test_early_termination_without_flags_is_libstdcxx(pfref):
    """without dependence flags every tie counts: the exact std::sort permutation of a depth-0 introsort,
    with the pops stopped below the smallest key that has an equal neighbour"""
    rng = np.random.default_rng(41)
    for trial in range(50):
        n = int(rng.choice([17, 18, 31, 64, 65, 100, 257, 500, 1200]))
        span = int(rng.choice([2, 5, 40, 1000, 1 << 30]))
        keys = rng.integers(0, span, n).astype(np.uint32)
        if trial % 5 == 0:
            keys = np.sort(keys)
        elif trial % 5 == 1:
            keys = np.sort(keys)[::-1].copy()
        got, _ = segment_perm(keys)
        np.testing.assert_array_equal(got, pfref.sort_perm(keys, "literal", 0),
                                      err_msg="trial %d n=%d span=%d" % (trial, n, span))


def test_early_termination_with_dependence_flags(pfref):
    """with flags: the order of every flagged group's elements is libstdc++'s, every key in order;
    unflagged groups may come in any order. Pops stop after the smallest flagged key (rgbds-like
    inputs: a sorted run with unsorted keys appended)."""
    rng = np.random.default_rng(42)
    saved = 0
    for trial in range(40):
        n = int(rng.choice([40, 300, 1500]))
        keys = np.sort(rng.integers(0, n, n).astype(np.uint32))
        keys = np.concatenate([keys[: n * 3 // 4], rng.permutation(keys[n * 3 // 4:])]).astype(np.uint32)
        groups = {}
        for i, k in enumerate(keys):
            groups.setdefault(int(k), []).append(i)
        flagged = {k for k, g in groups.items() if len(g) >= 3 and rng.random() < 0.3}
        dep = np.array([int(k) in flagged for k in keys])
        got, npops = segment_perm(keys, dep)
        saved += n - 1 - npops
        want = pfref.sort_perm(keys, "literal", 0)
        np.testing.assert_array_equal(keys[got], keys[want])                  # keys in order
        for k in flagged:                                                    # flagged groups: exact
            np.testing.assert_array_equal([i for i in got if keys[i] == k], [i for i in want if keys[i] == k])
    assert saved > 0
