// Exact radius-gated 5-NN on a dense 1 m cell grid.
//
// The reference takes the 5 nearest map points from KdTreeFLANN::nearestKSearch and uses them only
// when the 5th squared distance is < 1 (src/odomEstimationClass.cpp:299-300, 447-451). Every point
// with d^2 < 1 of a query lies in the 3x3x3 block of 1 m cells around the query's cell (float
// subtraction is monotone, so |fl(px - qx)| < 1 implies |px - qx| < 1), hence scanning those 27
// cells with the same float distance (x, then y, then z, no FMA) gives bit-identical neighbours and
// distances for every query the reference keeps. Ties are broken by map index.
#pragma once
#include "pf_common.h"
#include "pf_prims.h"

namespace pf {

struct GridGPU {
    int* bounds = nullptr;      // [2][6]   min cell x,y,z / max cell x,y,z per map (atomics)
    int* dims = nullptr;        // [2][8]   minx,miny,minz, dx,dy,dz, base, valid
    int* d_ncells = nullptr;    // [1]      total cells + 1 (scan length)
    int* err = nullptr;         // [1]      cell capacity exceeded
    u32* arrive = nullptr;      // [1]      arrival counter of the bounds kernel
    u32* cell_count = nullptr;  // [cell_cap + 1]
    u32* cell_start = nullptr;  // [cell_cap + 1]
    u32* slot = nullptr;        // [pts_cap]
    float4* cpts = nullptr;     // [pts_cap] cell-ordered (x, y, z, bits(map index))
    size_t pts_cap = 0;
    size_t cell_cap = 0;
};

int grid_alloc(GridGPU& g, size_t pts_cap, size_t cell_cap);
void grid_free(GridGPU& g);
// Build the grids of up to two maps (map1 may be null). Counts are device-resident.
void grid_build(GridGPU& g, const float4* map0, const int* d_m0, const float4* map1, const int* d_m1, PrimWork& w,
                hipStream_t s);

struct GridView {
    const int* dims;
    const u32* cell_start;
    const float4* cpts;
};

__device__ __forceinline__ bool knn_lt(float da, int ia, float db, int ib) {
    return da < db || (da == db && ia < ib);
}

// 5 nearest neighbours with d2 < 1 of query q in map m. Returns the count found (0..5); d/id sorted.
__device__ __forceinline__ int knn5(const GridView& gv, int m, float qx, float qy, float qz, float (&d)[5],
                                    int (&id)[5]) {
#pragma unroll
    for (int k = 0; k < 5; ++k) { d[k] = 1.0f; id[k] = 0x7fffffff; }
    const int* dm = gv.dims + 8 * m;
    if (!dm[7]) return 0;
    const int cx = (int)floorf(qx), cy = (int)floorf(qy), cz = (int)floorf(qz);
    const int minx = dm[0], miny = dm[1], minz = dm[2], dx = dm[3], dy = dm[4], dz = dm[5], base = dm[6];
    for (int oz = -1; oz <= 1; ++oz) {
        const int z = cz + oz - minz;
        if (z < 0 || z >= dz) continue;
        for (int oy = -1; oy <= 1; ++oy) {
            const int y = cy + oy - miny;
            if (y < 0 || y >= dy) continue;
            for (int ox = -1; ox <= 1; ++ox) {
                const int x = cx + ox - minx;
                if (x < 0 || x >= dx) continue;
                const int cid = base + (z * dy + y) * dx + x;
                const u32 b0 = gv.cell_start[cid], b1 = gv.cell_start[cid + 1];
                for (u32 k = b0; k < b1; ++k) {
                    const float4 p = gv.cpts[k];
                    float r = 0.0f;
                    float t = qx - p.x; r += t * t;
                    t = qy - p.y; r += t * t;
                    t = qz - p.z; r += t * t;
                    if (!(r < 1.0f)) continue;
                    const int idx = __float_as_int(p.w);
                    if (!knn_lt(r, idx, d[4], id[4])) continue;
                    d[4] = r; id[4] = idx;
#pragma unroll
                    for (int q = 4; q > 0; --q) {
                        if (knn_lt(d[q], id[q], d[q - 1], id[q - 1])) {
                            float td = d[q]; d[q] = d[q - 1]; d[q - 1] = td;
                            int ti = id[q]; id[q] = id[q - 1]; id[q - 1] = ti;
                        }
                    }
                }
            }
        }
    }
    int found = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) found += (id[k] != 0x7fffffff) ? 1 : 0;
    return found;
}

// The same search by a team of T lanes (T a power of two <= 64, aligned within the wave). The 27
// cells form 9 x-rows of 3 cells that are contiguous in the cell-sorted point array, so the team
// reads 9 point ranges (18 cell_start words spread over the team's lanes); lane l takes points
// l, l + T, ... of every range (consecutive lanes, consecutive points: coalesced), keeping its own
// sorted 5 best, then the team merges its lists in 5 rounds of a (d^2 bits, index) minimum. Keys
// are unique (distinct map indices), so the merged 5 are exactly the sequential search's. Every
// lane of the wave must call this (the merge shuffles); `active` is uniform within a team. Results
// are valid on every lane.
#ifndef PF_KNN_GROUP
#define PF_KNN_GROUP 1
#endif
__device__ __forceinline__ u64 knn_key(float d, int i) {
    return ((u64)__float_as_uint(d) << 32) | (u64)(u32)i;
}
__device__ __forceinline__ void knn_insert(float qx, float qy, float qz, const float4& p, float (&d)[5],
                                           int (&id)[5]) {
    float r = 0.0f;
    float t = qx - p.x; r += t * t;
    t = qy - p.y; r += t * t;
    t = qz - p.z; r += t * t;
    if (!(r < 1.0f)) return;
    const int idx = __float_as_int(p.w);
    if (!knn_lt(r, idx, d[4], id[4])) return;
    d[4] = r; id[4] = idx;
#pragma unroll
    for (int q = 4; q > 0; --q) {
        if (knn_lt(d[q], id[q], d[q - 1], id[q - 1])) {
            float td = d[q]; d[q] = d[q - 1]; d[q - 1] = td;
            int ti = id[q]; id[q] = id[q - 1]; id[q - 1] = ti;
        }
    }
}
template <int T>
__device__ __forceinline__ int knn5_team(const GridView& gv, int m, float qx, float qy, float qz, bool active,
                                         float (&dout)[5], int (&iout)[5]) {
    static_assert(T >= 8 && T <= 64 && (T & (T - 1)) == 0, "team: a power of two, >= 5 result lanes");
    float d[5];
    int id[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) { d[k] = 1.0f; id[k] = 0x7fffffff; }
    const int* dm = gv.dims + 8 * m;
    if (active && dm[7]) {
        const int cx = (int)floorf(qx), cy = (int)floorf(qy), cz = (int)floorf(qz);
        const int minx = dm[0], miny = dm[1], minz = dm[2], dx = dm[3], dy = dm[4], dz = dm[5], base = dm[6];
        const int xlo = max(cx - 1 - minx, 0), xhi = min(cx + 1 - minx, dx - 1);
        if (xlo <= xhi) {
            const u32 tl = (u32)(lane_id() & (T - 1));
            const int tbase = lane_id() & ~(T - 1);
            // the 18 range words (row r: start of cell xlo, end of cell xhi) spread over the team's
            // lanes, a few loads per lane, then gathered on every lane with shuffles
            constexpr int K = (18 + T - 1) / T;
            u32 wv[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int w = (int)tl + T * k;
                const int r = w >> 1;
                const int y = cy + (r % 3) - 1 - miny, z = cz + r / 3 - 1 - minz;
                const bool ok = w < 18 && y >= 0 && y < dy && z >= 0 && z < dz;
                wv[k] = ok ? gv.cell_start[base + (z * dy + y) * dx + ((w & 1) ? xhi + 1 : xlo)] : 0u;
            }
            u32 b0[9], b1[9];
#pragma unroll
            for (int r = 0; r < 9; ++r) {
                b0[r] = (u32)__shfl((int)wv[(2 * r) / T], tbase + (2 * r) % T, 64);
                b1[r] = (u32)__shfl((int)wv[(2 * r + 1) / T], tbase + (2 * r + 1) % T, 64);
            }
            // rows in groups of G: the first point of each row of a group is loaded before any is
            // used. G = 1 measured fastest (config 5: 71 us vs 99 us for G = 9): full occupancy
            // (41 VGPRs, 8 waves / SIMD) hides more latency than loads in flight per wave
            constexpr int G = PF_KNN_GROUP;
#pragma unroll
            for (int g = 0; g < 9; g += G) {
                float4 pf[G];
#pragma unroll
                for (int r = 0; r < G; ++r)
                    if (g + r < 9 && b0[g + r] + tl < b1[g + r]) pf[r] = gv.cpts[b0[g + r] + tl];
#pragma unroll
                for (int r = 0; r < G; ++r) {
                    if (g + r >= 9 || b0[g + r] + tl >= b1[g + r]) continue;
                    knn_insert(qx, qy, qz, pf[r], d, id);
                    for (u32 k = b0[g + r] + tl + T; k < b1[g + r]; k += T) knn_insert(qx, qy, qz, gv.cpts[k], d, id);
                }
            }
        }
    }
    const u64 sentinel = knn_key(1.0f, 0x7fffffff);
    u64 head = knn_key(d[0], id[0]);
    int found = 0;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        u64 mn = head;
#pragma unroll
        for (int o = T / 2; o > 0; o >>= 1) {
            const u64 other = __shfl_xor(mn, o, 64);
            mn = other < mn ? other : mn;
        }
        dout[r] = __uint_as_float((u32)(mn >> 32));
        iout[r] = (int)(u32)(mn & 0xffffffffull);
        if (mn != sentinel) ++found;
        if (head == mn && mn != sentinel) {
#pragma unroll
            for (int k = 0; k < 4; ++k) { d[k] = d[k + 1]; id[k] = id[k + 1]; }
            d[4] = 1.0f; id[4] = 0x7fffffff;
            head = knn_key(d[0], id[0]);
        }
    }
    return found;
}

}  // namespace pf
