// Reference tie order (pf_odom_set_tie_order): the order libstdc++'s std::sort leaves equal keys in.
//
// The reference sorts (voxel index, point index) pairs by the voxel index alone with std::sort, in PCL
// 1.10's VoxelGrid and in rgbds (src/odomEstimationClass.cpp:74), then sums every voxel's
// points in f32 in the sorted order, so a centroid's last bits depend on how introsort happened to
// permute the points of its voxel. The pipeline's radix sorts are stable (points of a voxel in input
// order); this mode runs libstdc++'s introsort itself instead, so that VoxelGrid and rgbds centroids
// are the reference's bit for bit (the faithful oracle's, which calls std::sort itself).
//
// A Hoare partition of [first + 1, last) around the median-of-three pivot at first is computed from
// the ascending positions L_1 < L_2 < ... of its left stops (key >= pivot) and R_1 < R_2 < ... of its
// right stops (key <= pivot, first included): with m the largest k for which L_k < R_(nR + 1 - k), the
// partition swaps L_k <-> R_(nR + 1 - k) for k <= m and returns min(L_(m + 1), R_(nR + 1 - m)) (L_1 for
// m = 0). The test k <= m is local to the k-th left stop: L_k < R_(nR + 1 - k) holds exactly when at
// least k right stops lie after L_k, and the cut is the smallest of {R_(nR + 1 - k) : k <= m} and
// {L_k : k > m}, a minimum every left stop can contribute to. Introsort's segments never interact, so
// the recursion runs breadth-first, every segment of a level at once:
//   k_tie_medium  one 1024-thread workgroup per class (or per medium segment): drops the 0xFFFFFFFF
//                 keys (cropped points), then partitions in global memory, one sweep per level (tiles
//                 of 14336 keys ranked by ballots and a carried workgroup scan; the hit count m, the
//                 cut and the swaps in rank space), until every segment fits 14336 keys;
//   k_tie_mid     one workgroup per segment of 2049 .. 14336 keys: the same levels on the segment staged
//                 in LDS, until every piece fits 2048 keys (many CUs in parallel from here on);
//   k_tie_local   one workgroup per job of at most 2048 keys finishes the whole subtree in LDS: per
//                 level one pass ranks every segment's stops at once, one thread per segment searches
//                 m and the cut, a pass does the swaps, and one thread per segment files the children
//                 (median of three applied as it files them). Leaves of at most 16 keys are sorted
//                 stably at the end (libstdc++'s final insertion sort moves no key across a leaf);
//   k_tie_heap    the segments that reached the depth limit 2 lg n (in any tier) are written to the
//                 output as they stand and heap-sorted there as libstdc++'s __partial_sort does, one
//                 workgroup per segment: __make_heap a tree level at a time, __sort_heap's pops
//                 pipelined two tree levels apart in one wave (a pop every two LDS steps instead of one
//                 every 2 lg n); a segment above the LDS size runs the same on a global scratch copy.
// The levels are bound by VALU issue (about 50 instructions per 64 keys per level), so the tiers exist to
// spread a class over many CUs as early as the cost of a launch boundary allows: work handed from one
// workgroup to another inside a launch would pay an agent-scope release and acquire per hand-off.
//   big levels    (classes above kTieMed keys, e.g. a 2M-point rgbds map) first: k_tie_compact, then per
//                 level every tile of 4096 keys of every segment finds its stops in parallel (a
//                 look-back per segment ranks them) and one workgroup per segment swaps and files.
// oracle/pfref_sort.cpp holds the level-synchronous algorithm on the CPU next to a line-by-line
// restatement of libstdc++'s introsort, both checked against std::sort itself
// (tests/test_oracle_units.py).
#pragma once
#include "pf_prims.h"

namespace pf {

typedef unsigned char u8;

#ifndef PF_TIE_MED
#define PF_TIE_MED 65536
#endif
constexpr int kTieMed = PF_TIE_MED;   // classes above this run the multi-workgroup big levels first
constexpr int kTieTile = 4096;        // keys per tile of the compaction and the big levels

// class c of the input is its next cnt[ia + c] (+ cnt[ib + c] when ib >= 0) pairs, c < nc: the
// reference sorts every cloud with its own std::sort call
struct TieClasses {
    const int* cnt;
    int ia, ib, nc;
};

struct TieSort {
    u32 *k = nullptr, *v = nullptr;       // [cap] compacted pairs (the working copy)
    u32 *lp = nullptr, *rq = nullptr;     // [cap] left / right stop positions by rank
    u64* status = nullptr;                // [tiles] look-back words, zero between launches
    u32* arrive = nullptr;                // [8] arrival counters (look-backs, local-kernel / heap exits)
    int4* big = nullptr;                  // [2][bcap] big segments of a level {first, last, depth, tile base}
    u64* tot = nullptr;                   // [bcap] stop totals of a big segment (nL << 32 | nR)
    int4* med = nullptr;                  // [mcap] medium segments {first, last, depth, class}
    int4* mid = nullptr;                  // [midcap] mid-tier segments {first, last, depth, class}
    int4* jobs = nullptr;                 // [jcap] local jobs {first, last, depth (-1: at the limit), class}
    int2* heaps = nullptr;                // [hcap] depth-limit segments {output offset, length}
    int4* heapw = nullptr;                // [hcap] those the partition tiers filed (TieAux): {working offset,
                                          // length, class, 0}, heap-sorted beside k_tie_local
    u64* hbig = nullptr;                  // [cap + 64] heap entries of segments above the LDS size
    int* ctl = nullptr;                   // counters (pf_tie.hip)
    // sorts with big levels: depth-limit segments above the LDS size, and (with dependence flags) every
    // one without an order-dependent group, are sorted by one device-wide radix sort of all of them
    // (exact for a segment without an order-dependent group); the others go to the heap tier after it
    int2* huge = nullptr;                 // [hugecap] such segments {output offset, length}
    int2* heapf = nullptr;                // [hugecap] of those, the ones the heap tier still sorts
    u32* need = nullptr;                  // [hugecap] a segment's sorted copy holds an order-dependent group
    int2* hseg = nullptr;                 // [hugecap] the list in position order (k_huge_setup)
    int* hbase = nullptr;                 // [hugecap + 1] pairs of the segments before each
    u32* depn = nullptr;                  // [2][512] order-dependent elements of a level's big segments
    u32 *hk = nullptr, *hv = nullptr;     // [cap] their pairs, gathered
    PrimWork hprim;                       // the radix sort's scratch (cap)
    size_t cap = 0, tiles = 0;
    int bcap = 0, mcap = 0, midcap = 0, jcap = 0, hcap = 0, hugecap = 0;
    int max_levels = 0;                   // big levels the buffers are sized for
    int depth0 = -1;                      // test probe: >= 0 replaces every class's depth limit
};

constexpr int kMaxBigLevels = 48;     // big levels at most (the depth limit 2 lg n of a 16M-key class)

// cap: most pairs of one sort; max_levels < 0: as many big levels as cap can need
int tie_alloc(TieSort& t, size_t cap, int max_levels = -1);
void tie_free(TieSort& t);
// big levels for classes of up to `size_hint` keys: 0 up to kTieMed, else the class's depth limit
// 2 lg n (a segment that peels a few keys per level stays above kTieMed for tens of levels, and a big
// level spreads it over the device where a medium workgroup walks it on one CU); clamped to max_levels
int tie_levels_for(const TieSort& t, size_t size_hint);

// Sorts (keys, vals)[0 .. n) in place, n = the classes' total, each class as std::sort would (keys
// compared as whole 32-bit words), the 0xFFFFFFFF pairs dropped from the classes and the key array
// ended by them: keys[0 .. valid) sorted class after class, keys[valid .. n) = 0xFFFFFFFF (their
// vals too). Replaces a stable radix sort of the same pairs. levels: big levels to run first (0: every
// class goes straight to its medium workgroup, which handles any size, slowly above kTieMed). A
// look-back wait that gives up sets bit 2 of *err (the caller's sticky error word), a list overflow
// bit 4. freef (optional, indexed by val): nonzero when the element's voxel group is order-free (its f32
// centroid sum does not depend on the order of its points; pf_odom.hip k_rg_dep): the heap tier then
// runs only the pops the order-dependent groups need. NULL: every group counts as order-dependent.
// aux (optional, sorts without big levels): a second stream and two events. The depth-limit segments the
// partition tiers k_tie_medium / k_tie_mid produce are then heap-sorted by a k_tie_heap launch on aux that
// starts when k_tie_mid ends and runs beside k_tie_local (and the heap launch of the local tier's own
// depth-limit segments); s waits for it before the sort returns. Without aux every depth-limit segment
// goes through k_tie_local to the one heap launch after it.
// hs (optional, sorts with big levels and the radix route): the depth-limit and dependence-free segments
// above the LDS size that the big levels and k_tie_medium leave are filed by k_tie_medium straight from the
// working copy, and their radix sort (and the heap launch for those of them that need pops) runs on hs
// beside k_tie_mid / k_tie_local / k_tie_heap, joined before the sort returns (fork / join as above).
struct TieAux {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    hipStream_t hs = nullptr;
};
void tie_sort(TieSort& t, u32* keys, u32* vals, TieClasses cls, int* err, hipStream_t s, int levels = 0,
              const u8* freef = nullptr, const TieAux* aux = nullptr);
const int* tie_valid_count(const TieSort& t);   // device word: the valid pairs of the last sort

}  // namespace pf
