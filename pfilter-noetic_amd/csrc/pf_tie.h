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
// m = 0). Introsort's segments never interact, so the recursion runs breadth-first:
//   k_tie_compact   drops the 0xFFFFFFFF keys (cropped points) per class, one pass with a look-back;
//   big levels      segments above kTieLocal keys: every tile of 4096 keys of every segment finds its
//                   stops in parallel (a look-back per segment ranks them), then one workgroup per
//                   segment searches m, swaps the pairs and files the children;
//   k_tie_local     one workgroup per segment of at most kTieLocal keys finishes its whole subtree in
//                   LDS, one wavefront per segment per recursion level; leaves of at most 16 keys are
//                   sorted stably (libstdc++'s final insertion sort moves no key across a leaf), the
//                   depth limit 2 lg n hands a segment to libstdc++'s heap sort. Segments still above
//                   kTieLocal after the big levels (very large classes) are partitioned by their
//                   workgroup in global memory until they fit.
// oracle/pfref_sort.cpp holds the same algorithm on the CPU next to a line-by-line restatement of
// libstdc++'s introsort, both checked against std::sort itself (tests/test_oracle_units.py).
#pragma once
#include "pf_prims.h"

namespace pf {

constexpr int kTieLocal = 14336;      // largest segment sorted in LDS (10 B per key)
constexpr int kTieTile = 4096;        // keys per tile of the compaction and the big levels

// class c of the input is its next cnt[ia + c] (+ cnt[ib + c] when ib >= 0) pairs, c < nc: the
// reference sorts every cloud with its own std::sort call
struct TieClasses {
    const int* cnt;
    int ia, ib, nc;
};

struct TieSort {
    u32 *k = nullptr, *v = nullptr;       // [cap] compacted pairs, class-major (the working copy)
    u32 *lp = nullptr, *rq = nullptr;     // [cap] left / right stop positions of the big partitions
    u64* status = nullptr;                // [tiles] look-back words, zero between launches
    u32* arrive = nullptr;                // [2] look-back arrival counters
    int4* big = nullptr;                  // [2][bcap] big segments of a level {first, last, depth, tile base}
    u64* tot = nullptr;                   // [bcap] stop totals of a big segment (nL << 32 | nR)
    int4* jobs = nullptr;                 // [jcap] local jobs {first, last, depth, 0}
    int* ctl = nullptr;                   // counters (pf_tie.hip)
    size_t cap = 0, tiles = 0;
    int bcap = 0, jcap = 0;
    int levels = 0;                       // big levels launched per sort
    int depth0 = -1;                      // test probe: >= 0 replaces every class's depth limit
};

// cap: most pairs of one sort; levels: big levels per sort (classes up to about 2^levels x kTieLocal
// keys are sorted without the single-workgroup fallback)
int tie_alloc(TieSort& t, size_t cap, int levels = 2);
void tie_free(TieSort& t);

// Sorts (keys, vals)[0 .. n) in place, n = the classes' total, each class as std::sort would (keys
// compared as whole 32-bit words), the 0xFFFFFFFF pairs dropped from the classes and the key array
// ended by them: keys[0 .. valid) sorted class after class, keys[valid .. n) = 0xFFFFFFFF (their
// vals too). Replaces a stable radix sort of the same pairs. A look-back wait that gives up sets bit 2
// of *err (the caller's sticky error word).
void tie_sort(TieSort& t, u32* keys, u32* vals, TieClasses cls, int* err, hipStream_t s);
const int* tie_valid_count(const TieSort& t);   // device word: the valid pairs of the last sort

}  // namespace pf
