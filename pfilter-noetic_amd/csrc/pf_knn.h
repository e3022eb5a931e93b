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
    u32* ttot = nullptr;        // [ttiles] points per scan tile of kGridScanTile cells (k_grid_count)
    int ttiles = 0;
    size_t pts_cap = 0;
    size_t cell_cap = 0;
};
// cells per tile of the cell-count scan: k_grid_count also counts the points of each tile, so a
// tile's exclusive prefix is a sum of those totals (no look-back across workgroups)
constexpr int kGridScanPer = 32;
constexpr int kGridScanTile = 256 * kGridScanPer;

// up to kGridMaps maps share one cell array (map m's cells start at dims[8 m + 6])
constexpr int kGridMaps = 3;
struct GridPtrs {                 // maps and their device-resident point counts
    const float4* m[kGridMaps];
    const int* n[kGridMaps];
    int nm;
};

int grid_alloc(GridGPU& g, size_t pts_cap, size_t cell_cap);
void grid_free(GridGPU& g);

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ inline void grid_dims(const int* bounds, const int* npts, int* dims, int* d_ncells, long long cell_cap, int* err) {
    long long base = 0;
    for (int mi = 0; mi < kGridMaps; ++mi) {
        const int n = npts[mi];
        int* dm = dims + 8 * mi;
        if (n <= 0) {
            for (int k = 0; k < 8; ++k) dm[k] = 0;
            dm[6] = (int)base;
            continue;
        }
        const int* b = bounds + 6 * mi;
        const long long dx = (long long)b[3] - b[0] + 1, dy = (long long)b[4] - b[1] + 1, dz = (long long)b[5] - b[2] + 1;
        const long long nc = dx * dy * dz;
        if (base + nc > cell_cap) {           // grid too large for the handle: mark invalid
            for (int k = 0; k < 8; ++k) dm[k] = 0;
            dm[6] = (int)base;
            atomicOr(err, 1);
            continue;
        }
        dm[0] = b[0]; dm[1] = b[1]; dm[2] = b[2];
        dm[3] = (int)dx; dm[4] = (int)dy; dm[5] = (int)dz;
        dm[6] = (int)base;
        dm[7] = 1;
        base += nc;
    }
    *d_ncells = (int)(base + 1);
}

// the concatenation of the maps: point i belongs to map mi at local index li
struct GridIdx {
    int end[kGridMaps];
    int total;
    __device__ __forceinline__ int map_of(int i) const { return i < end[0] ? 0 : (i < end[1] ? 1 : 2); }
    __device__ __forceinline__ int start(int mi) const { return mi == 0 ? 0 : end[mi - 1]; }
};
__device__ __forceinline__ GridIdx grid_idx(const GridPtrs& gp) {
    GridIdx g;
    int acc = 0;
#pragma unroll
    for (int k = 0; k < kGridMaps; ++k) {
        acc += k < gp.nm ? *gp.n[k] : 0;
        g.end[k] = acc;
    }
    g.total = acc;
    return g;
}

// per-map min/max cell coordinates: wave then workgroup reduction, one atomic per workgroup. The
// last workgroup to arrive derives the grid dimensions and resets the bounds for the next build.
// A Tail with kActive runs on one extra workgroup (the last), which takes no part in the bounds: a
// caller's independent single-thread work (the odometry's pose prediction) overlaps the bounds
// instead of taking its own launch. Launch kGridBoundsBlocks + (Tail::kActive ? 1 : 0) workgroups.
struct GridBoundsArgs {
    GridPtrs gp;
    int* bounds;
    u32* arrive;
    int* dims;
    int* d_ncells;
    long long cell_cap;
    int* err;
};
struct NoTail {
    static constexpr bool kActive = false;
    __device__ void operator()(int) const {}
};
template <class Tail>
__global__ void __launch_bounds__(256) k_grid_bounds(GridBoundsArgs ga, Tail tail) {
    if (Tail::kActive && blockIdx.x == gridDim.x - 1) {
        tail((int)threadIdx.x);
        return;
    }
    const unsigned nblk = gridDim.x - (Tail::kActive ? 1u : 0u);   // workgroups sharing the bounds
    const GridPtrs& gp = ga.gp;
    int* bounds = ga.bounds;
    u32* arrive = ga.arrive;
    int* dims = ga.dims;
    int* d_ncells = ga.d_ncells;
    const long long cell_cap = ga.cell_cap;
    int* err = ga.err;
    constexpr int NB = 6 * kGridMaps;
    __shared__ int red[4][NB];
    __shared__ int last;
    __shared__ int lb[NB];
    const GridIdx gi = grid_idx(gp);
    const int l = lane_id(), w = threadIdx.x >> 6;
    int v[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) v[k] = ((k % 6) < 3) ? INT_MAX : INT_MIN;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < gi.total; i += nblk * blockDim.x) {
        const int mi = gi.map_of(i);
        const float4 p = gp.m[mi][i - gi.start(mi)];
        const int c[3] = {(int)floorf(p.x), (int)floorf(p.y), (int)floorf(p.z)};
#pragma unroll
        for (int mm = 0; mm < kGridMaps; ++mm) {      // branch-free: static register indices
            const bool mine = mm == mi;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                v[6 * mm + k] = mine ? min(v[6 * mm + k], c[k]) : v[6 * mm + k];
                v[6 * mm + 3 + k] = mine ? max(v[6 * mm + 3 + k], c[k]) : v[6 * mm + 3 + k];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        if (k >= 6 * gp.nm) break;                    // uniform: maps not built
        const int r = ((k % 6) < 3) ? wave_min_i(v[k]) : wave_max_i(v[k]);
        if (l == 0) red[w][k] = r;
    }
    __syncthreads();
    if (threadIdx.x < 6 * gp.nm) {
        const int k = threadIdx.x;
        const bool is_min = (k % 6) < 3;
        int r = red[0][k];
        for (int ww = 1; ww < 4; ++ww) r = is_min ? min(r, red[ww][k]) : max(r, red[ww][k]);
        if (is_min && r != INT_MAX) __hip_atomic_fetch_min(&bounds[k], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!is_min && r != INT_MIN) __hip_atomic_fetch_max(&bounds[k], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1;
    __syncthreads();
    if (!last) return;
    if (threadIdx.x < NB) {
        const int k = threadIdx.x;
        lb[k] = __hip_atomic_load(&bounds[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&bounds[k], ((k % 6) < 3) ? INT_MAX : INT_MIN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int nloc[kGridMaps];
        for (int k = 0; k < kGridMaps; ++k) nloc[k] = gi.end[k] - (k ? gi.end[k - 1] : 0);
        grid_dims(lb, nloc, dims, d_ncells, cell_cap, err);
        __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ int cell_of(const int* dm, float4 p) {
    const int x = (int)floorf(p.x) - dm[0], y = (int)floorf(p.y) - dm[1], z = (int)floorf(p.z) - dm[2];
    return dm[6] + (z * dm[4] + y) * dm[3] + x;
}
// the same, -1 for a point outside the grid's bounds (never, when the dims come from these points'
// own bounds: a guard that turns inconsistent dims into a reported error instead of stray writes)
__device__ __forceinline__ int cell_of_checked(const int* dm, float4 p) {
    const int x = (int)floorf(p.x) - dm[0], y = (int)floorf(p.y) - dm[1], z = (int)floorf(p.z) - dm[2];
    if ((unsigned)x >= (unsigned)dm[3] || (unsigned)y >= (unsigned)dm[4] || (unsigned)z >= (unsigned)dm[5]) return -1;
    return dm[6] + (z * dm[4] + y) * dm[3] + x;
}

// Agg: clouds whose consecutive points mostly share a cell (the front end's non-ground cloud, in
// 3 m ground-cell order) take one atomic per run of equal cells in a wave (up to 4 runs; the rest
// per lane) instead of serialising on the cell's counter. Slots inside a cell are arbitrary either
// way (the queries order candidates by (d^2, index)). Every point is also counted in its scan tile
// (ttot, one atomic per distinct tile in a wave: consecutive points share a tile).
// A Tail with kActive runs on one extra workgroup (the last), as in k_grid_bounds.
#ifndef PF_GRID_AGG_RUNS
#define PF_GRID_AGG_RUNS 4
#endif
constexpr int kGridAggRuns = PF_GRID_AGG_RUNS;   // runs of equal cells per wave taken by one atomic each
template <bool Agg, class Tail>
__global__ void __launch_bounds__(256) k_grid_count(GridPtrs gp, const int* __restrict__ dims, u32* __restrict__ cnt,
                                                     u32* __restrict__ slot, u32* __restrict__ ttot,
                                                     int* __restrict__ err, Tail tail) {
    if (Tail::kActive && blockIdx.x == gridDim.x - 1) {
        tail((int)threadIdx.x);
        return;
    }
    const GridIdx gi = grid_idx(gp);
    const int stride = (gridDim.x - (Tail::kActive ? 1 : 0)) * blockDim.x;
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = i0; i - (int)threadIdx.x % 64 < gi.total; i += stride) {   // trip count uniform per wave
        int cid = -1;
        if (i < gi.total) {
            const int mi = gi.map_of(i);
            const int* dm = dims + 8 * mi;
            if (dm[7]) {
                cid = cell_of_checked(dm, gp.m[mi][i - gi.start(mi)]);
                if (cid < 0) atomicOr(err, 1);
            }
        }
        {
            const int tt = cid >= 0 ? cid / kGridScanTile : -1;
            u64 todo = __ballot(tt >= 0);
            while (todo) {                                 // wave-uniform
                const int leader = __ffsll((unsigned long long)todo) - 1;
                const int c = __shfl(tt, leader, 64);
                const u64 m = __ballot(tt == c) & todo;
                if (lane_id() == leader) atomicAdd(&ttot[c], (u32)__popcll(m));
                todo &= ~m;
            }
        }
        if (!Agg) {
            if (cid >= 0) slot[i] = atomicAdd(&cnt[cid], 1u);
            continue;
        }
        u64 todo = __ballot(cid >= 0);
        for (int it = 0; it < kGridAggRuns && todo; ++it) {   // wave-uniform
            const int leader = __ffsll((unsigned long long)todo) - 1;
            const int c = __shfl(cid, leader, 64);
            const u64 m = __ballot(cid == c) & todo;
            u32 b = 0;
            if (lane_id() == leader) b = atomicAdd(&cnt[c], (u32)__popcll(m));
            b = (u32)__shfl((int)b, leader, 64);
            if ((m >> lane_id()) & 1ull) slot[i] = b + (u32)__popcll(m & lanemask_lt());
            todo &= ~m;
        }
        if ((todo >> lane_id()) & 1ull) slot[i] = atomicAdd(&cnt[cid], 1u);
    }
}

inline GridBoundsArgs grid_bounds_args(GridGPU& g, const GridPtrs& gp) {
    return GridBoundsArgs{gp, g.bounds, g.arrive, g.dims, g.d_ncells, (long long)g.cell_cap, g.err};
}
constexpr int kGridBoundsBlocks = 64;

// Build the grids of gp.nm maps (counts device-resident). pts_cap must hold all maps' points.
// bounds_launched: the caller already ran k_grid_bounds (with its own tail) on this stream.
// aggregate: one counter atomic per run of equal cells in a wave (clouds in spatially coherent order)
void grid_build(GridGPU& g, const GridPtrs& gp, PrimWork& w, hipStream_t s, bool bounds_launched = false,
                bool aggregate = false);

// the first half of a build: bounds, per-cell counts (wave-aggregated) and cell_start; the caller
// places the points itself (cell-major order, e.g. by a sort) and zeroes the counts it used
void grid_count_scan(GridGPU& g, const GridPtrs& gp, PrimWork& w, hipStream_t s);

// the second half of grid_build: the scan of the counts and the placement (after k_grid_count, which
// a caller launches itself with its own tail on dims computed elsewhere)
constexpr int kGridCountBlocks = 512;
void grid_scan_scatter(GridGPU& g, const GridPtrs& gp, hipStream_t s);

struct GridView {
    const int* dims;
    const u32* cell_start;
    const float4* cpts;
};

__device__ __forceinline__ u64 knn_key(float d, int i) {
    return ((u64)__float_as_uint(d) << 32) | (u64)(u32)i;
}
// d^2 in the reference's order (x, then y, then z; no FMA under -ffp-contract=off)
__device__ __forceinline__ float knn_d2(float qx, float qy, float qz, const float4& p) {
    float r = 0.0f;
    float t = qx - p.x; r += t * t;
    t = qy - p.y; r += t * t;
    t = qz - p.z; r += t * t;
    return r;
}
// Insert a candidate known to beat k[4] into a sorted 5-list of (d^2 bits, index) keys, branch-free:
// four independent compares, then every slot takes its left neighbour, the key, or itself. Keys are
// unique (distinct map indices).
__device__ __forceinline__ void knn_push(u64 key, u64 (&k)[5]) {
    bool c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = key < k[q];
#pragma unroll
    for (int q = 4; q > 0; --q) k[q] = c[q - 1] ? k[q - 1] : (q < 4 && !c[q] ? k[q] : key);
    k[0] = c[0] ? key : k[0];
}
// The empty-slot key is (1.0f, index 0): every candidate with d^2 >= 1 (or NaN) has a key >= it and
// never enters the list, so the radius gate (d^2 < 1) needs no compare / select of its own, and every
// candidate with d^2 < 1 has a key below it.
constexpr u64 kKnnEmpty = (u64)0x3f800000u << 32;
__device__ __forceinline__ void knn_consider(float qx, float qy, float qz, const float4& p, u64 (&k)[5]) {
    const u64 key = knn_key(knn_d2(qx, qy, qz, p), __float_as_int(p.w));
    if (key < k[4]) knn_push(key, k);
}

// Minimum of a u64 over an aligned team of T lanes, on every lane of the team. Teams of up to 16 use
// DPP lane moves (quad xor 1, quad xor 2, mirror within 8, mirror within 16): each step pairs every
// lane with one in the other half of its group, so after log2(T) steps all lanes hold the minimum.
template <int DPP>
__device__ __forceinline__ u64 dpp_u64(u64 v) {
    const int lo = __builtin_amdgcn_mov_dpp((int)(u32)v, DPP, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(u32)(v >> 32), DPP, 0xf, 0xf, false);
    return ((u64)(u32)hi << 32) | (u64)(u32)lo;
}
template <int T>
__device__ __forceinline__ u64 team_min(u64 v) {
    u64 o;
    if (T >= 2) { o = dpp_u64<0xB1>(v); v = o < v ? o : v; }      // quad_perm [1,0,3,2]
    if (T >= 4) { o = dpp_u64<0x4E>(v); v = o < v ? o : v; }      // quad_perm [2,3,0,1]
    if (T >= 8) { o = dpp_u64<0x141>(v); v = o < v ? o : v; }     // row_half_mirror
    if (T >= 16) { o = dpp_u64<0x140>(v); v = o < v ? o : v; }    // row_mirror
#pragma unroll
    for (int m = 16; m < T; m <<= 1) { o = __shfl_xor(v, m, 64); v = o < v ? o : v; }
    return v;
}

// Exact 5-NN with d^2 < 1 by a team of T lanes (T a power of two <= 64, aligned within the wave).
//
// Candidate set. The 27 cells around the query's cell form 9 x-rows of 3 cells, each contiguous in
// the cell-sorted point array. A row (oy, oz) or an end cell (ox = +-1) of a row is dropped when a
// float lower bound of d^2 for every point in it is already >= 1. The bound is exact in float: for a
// point in cell cy - 1, |fl(qy - py)| >= fl(qy - cy) and in cell cy + 1 >= fl((cy + 1) - qy) (float
// rounding is monotone), and squares and the x -> y -> z sums are monotone too, so the reference's
// own d^2 of every dropped point is >= 1 and the gate would reject it. That removes about a quarter
// of the block (27 cells against the 20.6-cell expected volume of a unit ball swept over a cell).
//
// Work split. The kept rows' point ranges are concatenated into one index space [0, total); lane l
// of the team takes indices l, l + T, ... (consecutive lanes, consecutive points: coalesced) and
// issues U loads before using any, so a lane has U requests in flight instead of one per row. Each
// lane keeps a sorted 5-list; the team then merges in 5 rounds of a key minimum. The merged 5 are
// exactly the sequential search's. Every lane of the wave must call this (the merge shuffles);
// `active` is uniform within a team. Results are valid on every lane.
#ifndef PF_KNN_UNROLL
#define PF_KNN_UNROLL 2
#endif
#ifndef PF_KNN_ROWS
#define PF_KNN_ROWS 0
#endif

template <int T>
__device__ __forceinline__ int knn5_team(const GridView& gv, int m, float qx, float qy, float qz, bool active,
                                         float (&dout)[5], int (&iout)[5]) {
    static_assert(T >= 1 && T <= 64 && (T & (T - 1)) == 0, "team: a power of two within a wave");
    constexpr int U = PF_KNN_UNROLL;
    const u64 sentinel = kKnnEmpty;
    u64 k[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) k[q] = sentinel;
    const int* dm = gv.dims + 8 * m;
    if (active && dm[7]) {
        const float fcx = floorf(qx), fcy = floorf(qy), fcz = floorf(qz);
        const int cx = (int)fcx, cy = (int)fcy, cz = (int)fcz;
        const int minx = dm[0], miny = dm[1], minz = dm[2], dx = dm[3], dy = dm[4], dz = dm[5], base = dm[6];
        // per-axis lower bounds of |q - p| for the cells at offset -1 / +1
        const float lx = qx - fcx, hx = (fcx + 1.0f) - qx;
        const float ly = qy - fcy, hy = (fcy + 1.0f) - qy;
        const float lz = qz - fcz, hz = (fcz + 1.0f) - qz;
        const u32 tl = (u32)(lane_id() & (T - 1));
        const int tbase = lane_id() & ~(T - 1);
        (void)tbase;
        // rows spread over the team's lanes: lane tl owns rows tl, tl + T, ... (row r: oy = r % 3 - 1,
        // oz = r / 3 - 1) and loads that row's two range words
        constexpr int K = (9 + T - 1) / T;
        u32 rs[K], rl[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int r = (int)tl + T * j;
            const int oy = r % 3 - 1, oz = r / 3 - 1;
            const float by = oy < 0 ? ly : (oy > 0 ? hy : 0.0f);
            const float bz = oz < 0 ? lz : (oz > 0 ? hz : 0.0f);
            const float brow = (0.0f + by * by) + bz * bz;       // bound with bx = 0
            const float bl = (lx * lx + by * by) + bz * bz;        // cell cx - 1
            const float bh = (hx * hx + by * by) + bz * bz;        // cell cx + 1
            const int y = cy + oy - miny, z = cz + oz - minz;
            const int x0 = max(cx - (bl < 1.0f ? 1 : 0) - minx, 0);
            const int x1 = min(cx + (bh < 1.0f ? 1 : 0) - minx, dx - 1);
            const bool ok = r < 9 && brow < 1.0f && y >= 0 && y < dy && z >= 0 && z < dz && x0 <= x1;
            u32 s = 0, e = 0;
            if (ok) {
                const int c = base + (z * dy + y) * dx;
                s = gv.cell_start[c + x0];
                e = gv.cell_start[c + x1 + 1];
            }
            rs[j] = s;
            rl[j] = e - s;
        }
#if PF_KNN_ROWS
        // every lane: the rows' starts and lengths. First the leading T points of every row, G rows'
        // loads in flight at a time, then the tails of rows longer than T.
        u32 b0[9], ln[9];
#pragma unroll
        for (int r = 0; r < 9; ++r) {
            b0[r] = rs[r / T];
            ln[r] = rl[r / T];
            if (T > 1) {
                b0[r] = (u32)__shfl((int)b0[r], tbase + r % T, 64);
                ln[r] = (u32)__shfl((int)ln[r], tbase + r % T, 64);
            }
        }
        constexpr int G = PF_KNN_ROWS;
#pragma unroll
        for (int g = 0; g < 9; g += G) {
            float4 p[G];
#pragma unroll
            for (int r = 0; r < G; ++r)
                if (g + r < 9 && tl < ln[g + r]) p[r] = gv.cpts[b0[g + r] + tl];
#pragma unroll
            for (int r = 0; r < G; ++r)
                if (g + r < 9 && tl < ln[g + r]) knn_consider(qx, qy, qz, p[r], k);
        }
#pragma unroll
        for (int r = 0; r < 9; ++r)
            for (u32 j = tl + T; j < ln[r]; j += T) knn_consider(qx, qy, qz, gv.cpts[b0[r] + j], k);
#else
        // every lane: the rows' starts and the running prefix of their lengths; point v of the
        // concatenation lives at v + off[r] for the last row r with pre[r] <= v
        int off[9];
        u32 pre[9];
        u32 total = 0;
#pragma unroll
        for (int r = 0; r < 9; ++r) {
            u32 s = rs[r / T], l = rl[r / T];
            if (T > 1) {
                s = (u32)__shfl((int)s, tbase + r % T, 64);
                l = (u32)__shfl((int)l, tbase + r % T, 64);
            }
            pre[r] = total;
            off[r] = (int)(s - total);
            total += l;
        }
        // branch-free body as in knn5_thick below: unconditional loads (an index past the end clamped
        // to the last point, whose copy gets a NaN x), all U loads issued before the first use
        for (u32 v0 = tl; v0 < total; v0 += T * U) {
            float4 p[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32 v = u == 0 ? v0 : min(v0 + T * u, total - 1);
                int o = off[0];
#pragma unroll
                for (int r = 1; r < 9; ++r) o = v >= pre[r] ? off[r] : o;
                p[u] = gv.cpts[(int)v + o];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 1; u < U; ++u)
                if (v0 + T * u >= total) p[u].x = __int_as_float(0x7fc00000);
#pragma unroll
            for (int u = 0; u < U; ++u) knn_consider(qx, qy, qz, p[u], k);
        }
#endif
    }
    int found = 0;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        const u64 mn = team_min<T>(k[0]);
        dout[r] = __uint_as_float((u32)(mn >> 32));
        iout[r] = (int)(u32)(mn & 0xffffffffull);
        if (mn != sentinel) ++found;
        if (k[0] == mn && mn != sentinel) {
#pragma unroll
            for (int q = 0; q < 4; ++q) k[q] = k[q + 1];
            k[4] = sentinel;
        }
    }
    return found;
}

// ---- thick-row layout (standalone queries against a static map) ------------------------------
// Every cell (x, y, z) of the thick layout holds the points of cells (x, y, z - 1), (x, y, z) and
// (x, y, z + 1), in that order, and consecutive x of one (y, z) are consecutive in memory, so the
// 27-cell block of a query is 3 contiguous ranges (oy = -1, 0, 1) instead of 9 x-rows: each point is
// stored three times (48 B per map point; 96 MB for config 5's 2M points), and the per-candidate
// 9-way row select becomes a 2-compare select. The end cells (ox = +-1) of a range are dropped by the
// same exact float bound as knn5_team's, taken with bz = 0 (every z layer of the range shares it).
struct ThickView {
    const int* dims;           // the cell grid's dims (map 0)
    const u32* tstart;         // [ncells + 1] exclusive scan of the thick cell sizes
    const float4* tpts;        // thick layout (x, y, z, bits(map index))
};

// loads in flight per lane (team 8, config 5, µs: U = 2 / 3 / 4 / 5 / 6 / 8 -> 34.4 / 33.1 / 32.6-32.8 /
// 32.6 / 32.7 / 32.9)
#ifndef PF_KNN_THICK_UNROLL
#define PF_KNN_THICK_UNROLL 4
#endif
template <int T>
__device__ __forceinline__ int knn5_thick(const ThickView& tv, float qx, float qy, float qz, bool active,
                                          float (&dout)[5], int (&iout)[5]) {
    static_assert(T >= 4 && T <= 64 && (T & (T - 1)) == 0, "team: a power of two >= 4 within a wave");
    constexpr int U = PF_KNN_THICK_UNROLL;
    const u64 sentinel = kKnnEmpty;
    u64 k[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) k[q] = sentinel;
    const int* dm = tv.dims;
    if (active && dm[7]) {
        const float fcx = floorf(qx), fcy = floorf(qy), fcz = floorf(qz);
        const int cx = (int)fcx, cy = (int)fcy, cz = (int)fcz;
        const int minx = dm[0], miny = dm[1], minz = dm[2], dx = dm[3], dy = dm[4], dz = dm[5];
        const float lx = qx - fcx, hx = (fcx + 1.0f) - qx;
        const float ly = qy - fcy, hy = (fcy + 1.0f) - qy;
        const u32 tl = (u32)(lane_id() & (T - 1));
        const int tbase = lane_id() & ~(T - 1);
        // lane tl < 3 owns range oy = tl - 1: thick cells cx - 1 .. cx + 1 of row (cy + oy, cz)
        u32 s = 0, e = 0;
        {
            const int oy = (int)tl - 1;
            const float by = oy < 0 ? ly : (oy > 0 ? hy : 0.0f);
            const float bl = (lx * lx + by * by) + 0.0f * 0.0f;
            const float bh = (hx * hx + by * by) + 0.0f * 0.0f;
            // a query one layer below / above the grid reads the nearest thick layer (its extra layer
            // lies >= 1 m away in z, so the gate rejects it)
            const int y = cy + oy - miny, zq = cz - minz, z = min(max(zq, 0), dz - 1);
            const int x0 = max(cx - (bl < 1.0f ? 1 : 0) - minx, 0);
            const int x1 = min(cx + (bh < 1.0f ? 1 : 0) - minx, dx - 1);
            if (tl < 3 && y >= 0 && y < dy && zq >= -1 && zq <= dz && x0 <= x1) {
                const int c = (z * dy + y) * dx;
                s = tv.tstart[c + x0];
                e = tv.tstart[c + x1 + 1];
            }
        }
        const u32 s0 = (u32)__shfl((int)s, tbase, 64), e0 = (u32)__shfl((int)e, tbase, 64);
        const u32 s1 = (u32)__shfl((int)s, tbase + 1, 64), e1 = (u32)__shfl((int)e, tbase + 1, 64);
        const u32 s2 = (u32)__shfl((int)s, tbase + 2, 64), e2 = (u32)__shfl((int)e, tbase + 2, 64);
        const u32 p1 = e0 - s0, p2 = p1 + (e1 - s1), total = p2 + (e2 - s2);
        const u32 o0 = s0, o1 = s1 - p1, o2 = s2 - p2;
        // branch-free body: the U loads are unconditional (an index past the end is clamped to the
        // last point, whose copy is then given a NaN x so its key can never enter the list), and the
        // addresses are 32-bit byte offsets from the layout's base (host: < 4 GB)
        const char* tb = reinterpret_cast<const char*>(tv.tpts);
        for (u32 v0 = tl; v0 < total; v0 += T * U) {
            float4 p[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32 v = u == 0 ? v0 : min(v0 + T * u, total - 1);
                const u32 o = v >= p2 ? o2 : (v >= p1 ? o1 : o0);
                p[u] = *reinterpret_cast<const float4*>(tb + ((v + o) << 4));
            }
            __builtin_amdgcn_sched_barrier(0);                   // all U loads issued before any use
#pragma unroll
            for (int u = 1; u < U; ++u)
                if (v0 + T * u >= total) p[u].x = __int_as_float(0x7fc00000);
#pragma unroll
            for (int u = 0; u < U; ++u) knn_consider(qx, qy, qz, p[u], k);
        }
    }
    int found = 0;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        const u64 mn = team_min<T>(k[0]);
        dout[r] = __uint_as_float((u32)(mn >> 32));
        iout[r] = (int)(u32)(mn & 0xffffffffull);
        if (mn != sentinel) ++found;
        if (k[0] == mn && mn != sentinel) {
#pragma unroll
            for (int q = 0; q < 4; ++q) k[q] = k[q + 1];
            k[4] = sentinel;
        }
    }
    return found;
}

}  // namespace pf
