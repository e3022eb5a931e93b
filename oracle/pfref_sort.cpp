// pfref — TEST INFRASTRUCTURE ONLY. libstdc++'s std::sort as the reference calls it, three ways:
//
//  * pfref_std_sort_perm: std::sort itself on (key, index) pairs compared by key only, exactly the
//    call of PCL 1.10's VoxelGrid (cloud_point_index_idx::operator<) and of rgbds
//    (src/odomEstimationClass.cpp:74). The oracle's VoxelGrid / rgbds (opts=0) use this call.
//  * pfref_introsort_literal: a line-by-line restatement of libstdc++'s introsort (bits/stl_algo.h,
//    unchanged from GCC 9 to 11: __introsort_loop with _S_threshold 16 and depth 2 * __lg(n),
//    __unguarded_partition_pivot with __move_median_to_first(first, first + 1, mid, last - 1),
//    __partial_sort = __make_heap + __sort_heap at the depth limit, __final_insertion_sort) with a
//    settable depth limit, so that its heap-sort branch can be exercised;
//  * pfref_introsort_levels: the level-synchronous form the device's reference-tie-order mode runs
//    (pfilter-noetic_amd/csrc/pf_tie.hip). Segments never interact, so all partitions of one
//    recursion level run at once; a Hoare partition [first + 1, last) around the pivot at first is
//    computed from the ascending positions L_1 < L_2 < ... of its left stops (key >= pivot, in
//    [first + 1, last)) and R_1 < R_2 < ... of its right stops (key <= pivot, in [first, last)): with
//    m the largest k for which L_k < R_(nR + 1 - k), the partition swaps L_k <-> R_(nR + 1 - k) for
//    k <= m and returns min(L_(m + 1), R_(nR + 1 - m)) (L_1 for m = 0); the final insertion sort is a
//    stable insertion sort inside every leaf (all keys of an earlier leaf are <= all keys of a later one).
// tests/test_oracle_units.py checks the three against each other.
#include <algorithm>
#include <climits>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <utility>
#include <vector>

namespace {

struct E {
    uint32_t key, val;
};
inline bool lt(const E& a, const E& b) { return a.key < b.key; }

int lg(size_t n) {
    int r = 0;
    while (n >>= 1) ++r;
    return r;
}

// ---- literal restatement -------------------------------------------------------------------------
void push_heap_(E* first, long hole, long top, E value) {
    long parent = (hole - 1) / 2;
    while (hole > top && lt(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

void adjust_heap(E* first, long hole, long len, E value) {
    const long top = hole;
    long child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (lt(first[child], first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    push_heap_(first, hole, top, value);
}

void make_heap_(E* first, E* last) {
    const long len = last - first;
    if (len < 2) return;
    long parent = (len - 2) / 2;
    while (true) {
        E value = first[parent];
        adjust_heap(first, parent, len, value);
        if (parent == 0) return;
        parent--;
    }
}

void sort_heap_(E* first, E* last) {
    while (last - first > 1) {
        --last;
        E value = *last;
        *last = *first;
        adjust_heap(first, 0, last - first, value);
    }
}

void move_median_to_first(E* result, E* a, E* b, E* c) {
    if (lt(*a, *b)) {
        if (lt(*b, *c)) std::swap(*result, *b);
        else if (lt(*a, *c)) std::swap(*result, *c);
        else std::swap(*result, *a);
    } else if (lt(*a, *c)) {
        std::swap(*result, *a);
    } else if (lt(*b, *c)) {
        std::swap(*result, *c);
    } else {
        std::swap(*result, *b);
    }
}

E* unguarded_partition(E* first, E* last, E* pivot) {
    while (true) {
        while (lt(*first, *pivot)) ++first;
        --last;
        while (lt(*pivot, *last)) --last;
        if (!(first < last)) return first;
        std::swap(*first, *last);
        ++first;
    }
}

void introsort_loop(E* first, E* last, long depth) {
    while (last - first > 16) {
        if (depth == 0) {
            make_heap_(first, last);
            sort_heap_(first, last);
            return;
        }
        --depth;
        E* mid = first + (last - first) / 2;
        move_median_to_first(first, first + 1, mid, last - 1);
        E* cut = unguarded_partition(first + 1, last, first);
        introsort_loop(cut, last, depth);
        last = cut;
    }
}

void unguarded_linear_insert(E* last) {
    E val = *last;
    E* next = last - 1;
    while (lt(val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

void insertion_sort(E* first, E* last) {
    if (first == last) return;
    for (E* i = first + 1; i != last; ++i) {
        if (lt(*i, *first)) {
            E val = *i;
            std::move_backward(first, i, i + 1);
            *first = val;
        } else {
            unguarded_linear_insert(i);
        }
    }
}

void final_insertion_sort(E* first, E* last) {
    if (last - first > 16) {
        insertion_sort(first, first + 16);
        for (E* i = first + 16; i != last; ++i) unguarded_linear_insert(i);
    } else {
        insertion_sort(first, last);
    }
}

// ---- level-synchronous form -----------------------------------------------------------------------
struct Seg {
    long first, last;
    int depth;
};

void sort_levels(E* a, long n, int depth0) {
    std::vector<Seg> cur, next, heaps, leaves;
    if (n > 16) cur.push_back(Seg{0, n, depth0});
    else if (n >= 2) leaves.push_back(Seg{0, n, 0});
    std::vector<long> L, R;
    while (!cur.empty()) {
        next.clear();
        for (const Seg& s : cur) {
            const long first = s.first, last = s.last;
            if (s.depth == 0) {
                heaps.push_back(s);
                continue;
            }
            const long mid = first + (last - first) / 2;
            move_median_to_first(a + first, a + first + 1, a + mid, a + last - 1);
            const uint32_t p = a[first].key;
            L.clear();
            R.clear();
            for (long i = first; i < last; ++i) {
                if (i > first && !(a[i].key < p)) L.push_back(i);
                if (!(p < a[i].key)) R.push_back(i);
            }
            const long nL = (long)L.size(), nR = (long)R.size();
            long lo = 0, hi = std::min(nL, nR);            // m: the last k with L_k < R_(nR + 1 - k)
            while (lo < hi) {
                const long k = (lo + hi + 1) / 2;
                if (L[k - 1] < R[nR - k]) lo = k;
                else hi = k - 1;
            }
            const long m = lo;
            long cut;
            if (m == 0) cut = nL ? L[0] : last;
            else cut = std::min(m < nL ? L[m] : LONG_MAX, R[nR - m]);
            for (long k = 0; k < m; ++k) std::swap(a[L[k]], a[R[nR - 1 - k]]);
            const Seg kids[2] = {Seg{first, cut, s.depth - 1}, Seg{cut, last, s.depth - 1}};
            for (const Seg& c : kids) {
                if (c.last - c.first > 16) next.push_back(c);
                else if (c.last - c.first >= 2) leaves.push_back(c);
            }
        }
        std::swap(cur, next);
    }
    for (const Seg& h : heaps) {
        make_heap_(a + h.first, a + h.last);
        sort_heap_(a + h.first, a + h.last);
    }
    for (const Seg& l : leaves)                                   // stable inside the leaf
        for (long i = l.first + 1; i < l.last; ++i) {
            const E v = a[i];
            long j = i;
            while (j > l.first && lt(v, a[j - 1])) {
                a[j] = a[j - 1];
                --j;
            }
            a[j] = v;
        }
}

std::vector<E> pairs(const uint32_t* keys, size_t n) {
    std::vector<E> a(n);
    for (size_t i = 0; i < n; ++i) a[i] = E{keys[i], (uint32_t)i};
    return a;
}

void perm(const std::vector<E>& a, uint32_t* out) {
    for (size_t i = 0; i < a.size(); ++i) out[i] = a[i].val;
}

}  // namespace

extern "C" {

void pfref_std_sort_perm(const uint32_t* keys, size_t n, uint32_t* out) {
    std::vector<E> a = pairs(keys, n);
    std::sort(a.begin(), a.end(), lt);
    perm(a, out);
}

// depth < 0: libstdc++'s own limit 2 * __lg(n)
void pfref_introsort_literal(const uint32_t* keys, size_t n, int depth, uint32_t* out) {
    std::vector<E> a = pairs(keys, n);
    if (n > 1) {
        introsort_loop(a.data(), a.data() + n, depth < 0 ? 2L * lg(n) : (long)depth);
        final_insertion_sort(a.data(), a.data() + n);
    }
    perm(a, out);
}

// development statistics of one std::sort call's introsort (the literal form): st = {partition
// levels reached, depth-limit segments, largest of them, their total keys, of those the segments holding
// three or more equal keys, the largest of those, the keys of the segments holding any equal pair}
void pfref_introsort_stats(const uint32_t* keys, size_t n, long* st) {
    std::vector<E> a = pairs(keys, n);
    for (int i = 0; i < 7; ++i) st[i] = 0;
    struct F { long f, l, d, lev; };
    std::vector<F> stack;
    const long d0 = n > 1 ? 2L * lg(n) : 0;
    if (n > 16) stack.push_back(F{0, (long)n, d0, 0});
    while (!stack.empty()) {
        F s = stack.back();
        stack.pop_back();
        E* first = a.data() + s.f;
        E* last = a.data() + s.l;
        long lev = s.lev, depth = s.d;
        while (last - first > 16) {
            st[0] = std::max(st[0], lev + 1);
            if (depth == 0) {
                const long len = last - first;
                ++st[1];
                st[2] = std::max(st[2], len);
                st[3] += len;
                std::vector<uint32_t> k(len);
                for (long i = 0; i < len; ++i) k[i] = first[i].key;
                std::sort(k.begin(), k.end());
                bool g3 = false, g2 = false;
                for (long i = 2; i < len; ++i) g3 |= k[i] == k[i - 2];
                for (long i = 1; i < len; ++i) g2 |= k[i] == k[i - 1];
                if (g2) st[6] += len;
                st[4] += g3;
                if (g3) st[5] = std::max(st[5], len);
                break;
            }
            --depth;
            E* mid = first + (last - first) / 2;
            move_median_to_first(first, first + 1, mid, last - 1);
            E* cut = unguarded_partition(first + 1, last, first);
            stack.push_back(F{cut - a.data(), last - a.data(), depth, lev + 1});
            last = cut;
            ++lev;
        }
    }
}

// development statistics: every depth-limit segment of one std::sort call with, per element, whether
// its voxel group's f32 sum depends on the order (dep[i] != 0, indexed by input position): prints the
// segment length, its distinct keys, the keys of order-dependent groups in it, those groups, and the
// heap pops needed before the smallest order-dependent key (pops run from the largest key down)
void pfref_introsort_heapdep(const uint32_t* keys, const uint8_t* dep, size_t n, const char* tag) {
    std::vector<E> a = pairs(keys, n);
    struct F { long f, l, d; };
    std::vector<F> stack;
    const long d0 = n > 1 ? 2L * lg(n) : 0;
    if (n > 16) stack.push_back(F{0, (long)n, d0});
    while (!stack.empty()) {
        F s = stack.back();
        stack.pop_back();
        E* first = a.data() + s.f;
        E* last = a.data() + s.l;
        long depth = s.d;
        while (last - first > 16) {
            if (depth == 0) {
                const long len = last - first;
                std::vector<E> seg(first, last);
                std::stable_sort(seg.begin(), seg.end(), lt);
                long ndk = 0, ndg = 0, distinct = 0, pops = 0;
                for (long i = 0; i < len; ++i) {
                    const bool head = i == 0 || seg[i].key != seg[i - 1].key;
                    distinct += head;
                    if (dep[seg[i].val]) {
                        ++ndk;
                        if (head || !dep[seg[i - 1].val]) ++ndg;
                        if (!pops) pops = len - i;
                    }
                }
                std::fprintf(stderr, "heapdep %s len %ld distinct %ld depkeys %ld depgroups %ld pops %ld\n", tag, len,
                             distinct, ndk, ndg, pops);
                // PFREF_HEAP_DUMP: the depth-limit segments needing more than 1000 pops, as they reach the heap
                // (int32 len, int32 pops, then len keys), for the pop-schedule studies in tools/
                static FILE* hd = std::getenv("PFREF_HEAP_DUMP") ? std::fopen(std::getenv("PFREF_HEAP_DUMP"), "ab") : nullptr;
                if (hd && pops > 1000) {
                    const int32_t hdr[2] = {(int32_t)len, (int32_t)pops};
                    std::fwrite(hdr, sizeof(hdr), 1, hd);
                    for (long i = 0; i < len; ++i) std::fwrite(&first[i].key, sizeof(uint32_t), 1, hd);
                    std::fflush(hd);
                }
                break;
            }
            --depth;
            E* mid = first + (last - first) / 2;
            move_median_to_first(first, first + 1, mid, last - 1);
            E* cut = unguarded_partition(first + 1, last, first);
            stack.push_back(F{cut - a.data(), last - a.data(), depth});
            last = cut;
        }
    }
}

void pfref_introsort_levels(const uint32_t* keys, size_t n, int depth, uint32_t* out) {
    std::vector<E> a = pairs(keys, n);
    sort_levels(a.data(), (long)n, depth < 0 ? 2 * lg(n) : depth);
    perm(a, out);
}

}  // extern "C"
