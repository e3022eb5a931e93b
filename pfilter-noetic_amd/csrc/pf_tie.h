// Reference tie order (pf_odom_set_tie_order): the order libstdc++'s std::sort leaves equal keys in.
//
// The reference sorts (voxel index, point index) pairs by the voxel index alone with std::sort, in PCL
// 1.10's VoxelGrid and in rgbds (src/odomEstimationClass.cpp:74), then sums every voxel's
// points in f32 in the sorted order, so a centroid's last bits depend on how introsort happened to
// permute the points of its voxel. The pipeline's radix sorts are stable (points of a voxel in input
// order); this mode reproduces introsort's permutation instead, so that VoxelGrid and rgbds centroids
// are the reference's bit for bit (the faithful oracle's, which calls std::sort itself).
//
// Introsort's segments never interact, so every partition of one recursion level runs at once (one
// wavefront per segment): a Hoare partition of [first + 1, last) around the median-of-three pivot at
// first is computed from the ascending positions L_1 < L_2 < ... of its left stops (key >= pivot) and
// R_1 < R_2 < ... of its right stops (key <= pivot, first included): with m the largest k for which
// L_k < R_(nR + 1 - k), the partition swaps L_k <-> R_(nR + 1 - k) for k <= m and returns
// min(L_(m + 1), R_(nR + 1 - m)) (L_1 for m = 0). Segments that reach the depth limit 2 lg(n) are
// heap-sorted by libstdc++'s make_heap / sort_heap (one thread each), and the final insertion sort is
// a stable insertion sort inside every leaf of at most 16 elements. oracle/pfref_sort.cpp holds the
// same algorithm on the CPU, checked against std::sort itself (tests/test_oracle_units.py).
#pragma once
#include "pf_prims.h"

namespace pf {

struct TieSort {
    u32 *k = nullptr, *v = nullptr;       // [cap] the pairs being sorted (compacted, class-major)
    u32 *flag = nullptr, *pos = nullptr;  // [cap + 1] compaction: valid flags and their exclusive scan
    int4* seg[3] = {};                    // [scap] segment lists {first, last, depth}, rotating per level
    int4* heap = nullptr;                 // [scap] segments at the depth limit
    int2* leaf = nullptr;                 // [cap / 2 + 8] leaves {first, last} of 2 .. 16 elements
    int *lp = nullptr, *rq = nullptr;     // [cap] left / right stop positions per segment
    int* cnt = nullptr;                   // [8]: segment counts 0-2, leaves 3, heaps 4, valid pairs 5
    size_t cap = 0, scap = 0;
    int levels = 0;                       // level launches: 2 floor(lg(cap)) + 2
};

int tie_alloc(TieSort& t, size_t cap);
void tie_free(TieSort& t);

// tie_sort_enqueue sorts the pairs (keys, vals)[0 .. *d_n) as std::sort would, each class (key bits
// 30-31) on its own (the reference's separate calls per cloud), 0xFFFFFFFF keys (cropped points)
// dropped: enqueue it before the pipeline's stable radix sort of the same pairs (it reads them
// unsorted). tie_sort_finish, enqueued after that sort, writes the result over its output's first
// (valid count) pairs: the same keys, the vals of equal keys in std::sort's order. `w`: the stream's
// sort / scan scratch (its scan words only).
void tie_sort_enqueue(TieSort& t, const u32* keys, const u32* vals, const int* d_n, PrimWork& w, hipStream_t s);
void tie_sort_finish(TieSort& t, u32* keys_out, u32* vals_out, hipStream_t s);

}  // namespace pf
