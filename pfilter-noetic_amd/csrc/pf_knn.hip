// Dense 1 m cell grid build (counting sort) and the standalone exact 5-NN query API.
#include "pf_knn.h"

#include <climits>
#include <vector>

namespace pf {
namespace {

// exclusive scan of the cell counts (d_n = cells + 1 items): tile t's prefix is the sum of the point
// totals of tiles < t, so every workgroup scans its tiles independently
__global__ void __launch_bounds__(256) k_grid_scan(const u32* __restrict__ in, u32* __restrict__ out,
                                                    const int* __restrict__ d_n, const u32* __restrict__ ttot) {
    constexpr int PER = kGridScanPer;
    __shared__ u32 lw[4];
    __shared__ u32 lp[4];
    const int n = *d_n;
    const int ntiles = (n + kGridScanTile - 1) / kGridScanTile;
    const int t = threadIdx.x;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int base = tile * kGridScanTile + t * PER;
        u32 v[PER];
        if (base + PER <= n) {                                  // whole: 16-byte loads
#pragma unroll
            for (int k = 0; k < PER; k += 4) {
                const uint4 q = *reinterpret_cast<const uint4*>(in + base + k);
                v[k] = q.x; v[k + 1] = q.y; v[k + 2] = q.z; v[k + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < PER; ++k) v[k] = base + k < n ? in[base + k] : 0u;
        }
        u32 pre = 0;
        for (int j = t; j < tile; j += 256) pre += ttot[j];
        pre = (u32)wave_sum_i((int)pre);
        if (lane_id() == 0) lp[t >> 6] = pre;
        u32 sum = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) sum += v[k];
        u32 agg;
        const u32 tex = block_excl_scan256(sum, lw, agg);       // (its barriers publish lp)
        u32 r = lp[0] + lp[1] + lp[2] + lp[3] + tex;
        if (base + PER <= n) {
#pragma unroll
            for (int k = 0; k < PER; k += 4) {
                uint4 q;
                q.x = r; r += v[k];
                q.y = r; r += v[k + 1];
                q.z = r; r += v[k + 2];
                q.w = r; r += v[k + 3];
                *reinterpret_cast<uint4*>(out + base + k) = q;
            }
        } else {
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                if (base + k < n) out[base + k] = r;
                r += v[k];
            }
        }
        __syncthreads();                                        // lp reused by the next tile
    }
}

__global__ void __launch_bounds__(256) k_grid_scatter(GridPtrs gp, const int* __restrict__ dims,
                                                       const u32* __restrict__ start, const u32* __restrict__ slot,
                                                       float4* __restrict__ cpts, u32* __restrict__ cnt,
                                                       u32* __restrict__ ttot, int ttiles) {
    const GridIdx gi = grid_idx(gp);
    if (blockIdx.x == 0)                      // the tile totals of the next build (the scan has read them)
        for (int j = threadIdx.x; j < ttiles; j += blockDim.x) ttot[j] = 0u;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < gi.total; i += gridDim.x * blockDim.x) {
        const int mi = gi.map_of(i);
        const int* dm = dims + 8 * mi;
        if (!dm[7]) continue;
        const int li = i - gi.start(mi);
        const float4 p = gp.m[mi][li];
        const int cid = cell_of_checked(dm, p);
        if (cid < 0) continue;                // (counted as an error by k_grid_count)
        cpts[start[cid] + slot[i]] = make_float4(p.x, p.y, p.z, __int_as_float(li));
        cnt[cid] = 0u;                        // leaves the count array zero for the next build
    }
}

// standalone query: queries in map 0, a team of T lanes per query
#ifndef PF_KNN_MINW
#define PF_KNN_MINW 1
#endif
template <int T>
__global__ void __launch_bounds__(256, PF_KNN_MINW) k_knn_query(GridView gv, const float4* __restrict__ q, int nq,
                                                    int* __restrict__ idx, float* __restrict__ d2) {
#ifdef PF_KNN_NO_XCD
    const unsigned blk = blockIdx.x;
#else
    const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
#endif
    const int i = (int)((blk * blockDim.x + threadIdx.x) / T);
    const bool active = i < nq;
    const float4 p = active ? q[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float d[5];
    int id[5];
    const int found = knn5_team<T>(gv, 0, p.x, p.y, p.z, active, d, id);
    const int tl = lane_id() & (T - 1);
    if (active) {
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k % T != tl) continue;                       // result k written by lane k % T
            const bool f = k < found;
            idx[5 * i + k] = f ? id[k] : -1;
            d2[5 * i + k] = f ? d[k] : __int_as_float(0x7f800000);
        }
    }
}

// the thick-row layout of a built grid (pf_knn.h): sizes, then the triple copies
__global__ void __launch_bounds__(256) k_thick_count(const int* __restrict__ dims, const u32* __restrict__ start,
                                                      u32* __restrict__ tcount, int* __restrict__ d_n) {
    const int dx = dims[3], dy = dims[4], dz = dims[5];
    const int nc = dims[7] ? dx * dy * dz : 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *d_n = nc + 1;
        tcount[nc] = 0u;                      // the scan's last element: tstart[nc] = the total
    }
    const int L = dx * dy;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nc; c += gridDim.x * blockDim.x) {
        const int z = c / L;
        u32 n = start[c + 1] - start[c];
        if (z > 0) n += start[c - L + 1] - start[c - L];
        if (z + 1 < dz) n += start[c + L + 1] - start[c + L];
        tcount[c] = n;
    }
}
__global__ void __launch_bounds__(256) k_thick_scatter(const float4* __restrict__ pts, const int* __restrict__ d_m,
                                                        const int* __restrict__ dims, const u32* __restrict__ start,
                                                        const u32* __restrict__ slot, const u32* __restrict__ tstart,
                                                        float4* __restrict__ tpts) {
    const int n = *d_m;
    if (!dims[7]) return;
    const int L = dims[3] * dims[4], dz = dims[5];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        const int c = cell_of(dims, p);
        const int z = (c - dims[6]) / L;
        const u32 sl = slot[i];
        const float4 v = make_float4(p.x, p.y, p.z, __int_as_float(i));
        const u32 below = z > 0 ? start[c - L + 1] - start[c - L] : 0u;
        tpts[tstart[c] + below + sl] = v;                               // own layer: after z - 1
        if (z + 1 < dz) tpts[tstart[c + L] + sl] = v;                   // as layer z - 1 of cell z + 1
        if (z > 0) {                                                    // as layer z + 1 of cell z - 1
            const u32 b2 = z > 1 ? start[c - 2 * L + 1] - start[c - 2 * L] : 0u;
            tpts[tstart[c - L] + b2 + (start[c - L + 1] - start[c - L]) + sl] = v;
        }
    }
}

template <int T>
__global__ void __launch_bounds__(256, PF_KNN_MINW) k_knn_thick(ThickView tv, const float4* __restrict__ q, int nq,
                                                                int* __restrict__ idx, float* __restrict__ d2) {
    const unsigned blk = xcd_block(blockIdx.x, gridDim.x);
    const int i = (int)((blk * blockDim.x + threadIdx.x) / T);
    const bool active = i < nq;
    const float4 p = active ? q[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float d[5];
    int id[5];
    const int found = knn5_thick<T>(tv, p.x, p.y, p.z, active, d, id);
    const int tl = lane_id() & (T - 1);
    if (active) {
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k % T != tl) continue;
            const bool f = k < found;
            idx[5 * i + k] = f ? id[k] : -1;
            d2[5 * i + k] = f ? d[k] : __int_as_float(0x7f800000);
        }
    }
}

// |C(q)|: points in the 27 cells around each query (algorithmic byte count)
__global__ void __launch_bounds__(256) k_knn_cellpop(GridView gv, const float4* __restrict__ q, int nq,
                                                      unsigned long long* __restrict__ total) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long c = 0;
    if (i < nq) {
        const float4 p = q[i];
        const int* dm = gv.dims;
        if (dm[7]) {
            const int cx = (int)floorf(p.x), cy = (int)floorf(p.y), cz = (int)floorf(p.z);
            for (int oz = -1; oz <= 1; ++oz)
                for (int oy = -1; oy <= 1; ++oy)
                    for (int ox = -1; ox <= 1; ++ox) {
                        const int x = cx + ox - dm[0], y = cy + oy - dm[1], z = cz + oz - dm[2];
                        if (x < 0 || y < 0 || z < 0 || x >= dm[3] || y >= dm[4] || z >= dm[5]) continue;
                        const int cid = dm[6] + (z * dm[4] + y) * dm[3] + x;
                        c += gv.cell_start[cid + 1] - gv.cell_start[cid];
                    }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane_id() == 0 && c) atomicAdd(total, c);
}

}  // namespace

int grid_alloc(GridGPU& g, size_t pts_cap, size_t cell_cap) {
    g.pts_cap = pts_cap;
    g.cell_cap = cell_cap;
    if (hipMalloc(&g.bounds, sizeof(int) * 6 * kGridMaps) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&g.dims, sizeof(int) * 8 * kGridMaps) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&g.d_ncells, sizeof(int)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&g.err, sizeof(int)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&g.cell_count, sizeof(u32) * (cell_cap + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&g.cell_start, sizeof(u32) * (cell_cap + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&g.slot, sizeof(u32) * pts_cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&g.cpts, sizeof(float4) * pts_cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&g.arrive, sizeof(u32)) != hipSuccess) return PF_ENOMEM;
    g.ttiles = (int)((cell_cap + 1 + kGridScanTile - 1) / kGridScanTile);
    if (hipMalloc(&g.ttot, sizeof(u32) * g.ttiles) != hipSuccess) return PF_ENOMEM;
    if (hipMemset(g.ttot, 0, sizeof(u32) * g.ttiles) != hipSuccess) return PF_EHIP;
    if (hipMemset(g.err, 0, sizeof(int)) != hipSuccess) return PF_EHIP;
    if (hipMemset(g.arrive, 0, sizeof(u32)) != hipSuccess) return PF_EHIP;
    if (hipMemset(g.cell_count, 0, sizeof(u32) * (cell_cap + 1)) != hipSuccess) return PF_EHIP;
    int init[6 * kGridMaps];
    for (int k = 0; k < 6 * kGridMaps; ++k) init[k] = (k % 6) < 3 ? INT_MAX : INT_MIN;
    if (hipMemcpy(g.bounds, init, sizeof(init), hipMemcpyHostToDevice) != hipSuccess) return PF_EHIP;
    return PF_OK;
}

void grid_free(GridGPU& g) {
    (void)hipFree(g.bounds);
    (void)hipFree(g.dims);
    (void)hipFree(g.d_ncells);
    (void)hipFree(g.err);
    (void)hipFree(g.cell_count);
    (void)hipFree(g.cell_start);
    (void)hipFree(g.slot);
    (void)hipFree(g.cpts);
    (void)hipFree(g.arrive);
    (void)hipFree(g.ttot);
    g = GridGPU{};
}

static void grid_scan(GridGPU& g, hipStream_t s) {
    const int grid = g.ttiles < kSortMaxBlocks ? g.ttiles : kSortMaxBlocks;
    hipLaunchKernelGGL(k_grid_scan, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, g.cell_count, g.cell_start, g.d_ncells,
                       g.ttot);
}

void grid_count_scan(GridGPU& g, const GridPtrs& gp, PrimWork& w, hipStream_t s) {
    (void)w;
    hipLaunchKernelGGL(k_grid_bounds<NoTail>, dim3(kGridBoundsBlocks), dim3(256), 0, s, grid_bounds_args(g, gp), NoTail{});
    hipLaunchKernelGGL(k_grid_count<true>, dim3(512), dim3(256), 0, s, gp, g.dims, g.cell_count, g.slot, g.ttot, g.err, NoTail{});
    grid_scan(g, s);
}

void grid_build(GridGPU& g, const GridPtrs& gp, PrimWork& w, hipStream_t s, bool bounds_launched, bool aggregate) {
    (void)w;
    const int nb = kGridCountBlocks;
    if (!bounds_launched)
        hipLaunchKernelGGL(k_grid_bounds<NoTail>, dim3(kGridBoundsBlocks), dim3(256), 0, s, grid_bounds_args(g, gp),
                           NoTail{});
    if (aggregate)
        hipLaunchKernelGGL(k_grid_count<true>, dim3(nb), dim3(256), 0, s, gp, g.dims, g.cell_count, g.slot, g.ttot,
                           g.err, NoTail{});
    else
        hipLaunchKernelGGL(k_grid_count<false>, dim3(nb), dim3(256), 0, s, gp, g.dims, g.cell_count, g.slot, g.ttot,
                           g.err, NoTail{});
    grid_scan_scatter(g, gp, s);
}

void grid_scan_scatter(GridGPU& g, const GridPtrs& gp, hipStream_t s) {
    const int nb = kGridCountBlocks;
    grid_scan(g, s);
    hipLaunchKernelGGL(k_grid_scatter, dim3(nb), dim3(256), 0, s, gp, g.dims, g.cell_start, g.slot, g.cpts,
                       g.cell_count, g.ttot, g.ttiles);
}

}  // namespace pf

// ==================================================================================================
// standalone kNN C ABI
// ==================================================================================================
using namespace pf;

struct pf_knn {
    int device = 0;
    hipStream_t stream = nullptr;
    GridGPU grid;
    PrimWork prim;
    float4* d_map = nullptr;
    int* d_m = nullptr;
    float4* d_q = nullptr;
    int* d_idx = nullptr;
    float* d_d2 = nullptr;
    unsigned long long* d_pop = nullptr;
    size_t map_cap = 0, q_cap = 0;
    int nq = 0;
    int team = 8;                  // lanes per query
    bool thick = true;             // query the thick-row layout (pf_knn.h); false: the 9-row grid walk
    u32* tstart = nullptr;         // [cell_cap + 1]
    u32* tcount = nullptr;         // [cell_cap + 1]
    float4* tpts = nullptr;        // [3 * map_cap]
    int* d_nt = nullptr;           // thick scan length
};

namespace pf {
namespace {
void launch_knn(const pf_knn* h, const GridView& gv) {
    const unsigned blocks = (unsigned)(((size_t)h->nq * h->team + 255) / 256);
    if (h->thick) {
        const ThickView tv{h->grid.dims, h->tstart, h->tpts};
        switch (h->team) {
        case 4: hipLaunchKernelGGL(k_knn_thick<4>, dim3(blocks), dim3(256), 0, h->stream, tv, h->d_q, h->nq, h->d_idx, h->d_d2); break;
        case 16: hipLaunchKernelGGL(k_knn_thick<16>, dim3(blocks), dim3(256), 0, h->stream, tv, h->d_q, h->nq, h->d_idx, h->d_d2); break;
        default: hipLaunchKernelGGL(k_knn_thick<8>, dim3((unsigned)(((size_t)h->nq * 8 + 255) / 256)), dim3(256), 0, h->stream, tv, h->d_q, h->nq, h->d_idx, h->d_d2); break;
        }
        return;
    }
    switch (h->team) {
    case 1: hipLaunchKernelGGL(k_knn_query<1>, dim3(blocks), dim3(256), 0, h->stream, gv, h->d_q, h->nq, h->d_idx, h->d_d2); break;
    case 2: hipLaunchKernelGGL(k_knn_query<2>, dim3(blocks), dim3(256), 0, h->stream, gv, h->d_q, h->nq, h->d_idx, h->d_d2); break;
    case 4: hipLaunchKernelGGL(k_knn_query<4>, dim3(blocks), dim3(256), 0, h->stream, gv, h->d_q, h->nq, h->d_idx, h->d_d2); break;
    case 16: hipLaunchKernelGGL(k_knn_query<16>, dim3(blocks), dim3(256), 0, h->stream, gv, h->d_q, h->nq, h->d_idx, h->d_d2); break;
    default: hipLaunchKernelGGL(k_knn_query<8>, dim3(blocks), dim3(256), 0, h->stream, gv, h->d_q, h->nq, h->d_idx, h->d_d2); break;
    }
}
}  // namespace
}  // namespace pf

extern "C" {

int pf_knn_create(int device, size_t map_capacity, size_t query_capacity, pf_knn** out) {
    if (!out || map_capacity == 0 || query_capacity == 0) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(device));
    pf_knn* h = new pf_knn();
    h->device = device;
    h->map_cap = map_capacity;
    h->q_cap = query_capacity;
    int rc = PF_OK;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) rc = PF_EHIP;
    // cells: a 1 m grid over the map bounding box; 64M cells covers e.g. a 400 x 400 x 400 m block
    if (rc == PF_OK) rc = grid_alloc(h->grid, map_capacity, (size_t)1 << 26);
    if (rc == PF_OK) rc = prim_alloc(h->prim, 1, ((size_t)1 << 26) + 2);  // scans of the cell counts only
    if (rc == PF_OK && hipMalloc(&h->d_map, sizeof(float4) * map_capacity) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_m, sizeof(int) * 2) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_q, sizeof(float4) * query_capacity) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_idx, sizeof(int) * 5 * query_capacity) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_d2, sizeof(float) * 5 * query_capacity) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_pop, sizeof(unsigned long long)) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->tstart, sizeof(u32) * (((size_t)1 << 26) + 1)) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->tcount, sizeof(u32) * (((size_t)1 << 26) + 1)) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->tpts, sizeof(float4) * 3 * map_capacity) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_nt, sizeof(int)) != hipSuccess) rc = PF_ENOMEM;
    if (rc != PF_OK) {
        pf_knn_destroy(h);
        return rc;
    }
    *out = h;
    return PF_OK;
}

int pf_knn_destroy(pf_knn* h) {
    if (!h) return PF_OK;
    (void)hipSetDevice(h->device);
    grid_free(h->grid);
    prim_free(h->prim);
    (void)hipFree(h->d_map);
    (void)hipFree(h->d_m);
    (void)hipFree(h->d_q);
    (void)hipFree(h->d_idx);
    (void)hipFree(h->d_d2);
    (void)hipFree(h->d_pop);
    (void)hipFree(h->tstart);
    (void)hipFree(h->tcount);
    (void)hipFree(h->tpts);
    (void)hipFree(h->d_nt);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return PF_OK;
}

int pf_knn_set_map(pf_knn* h, const float* xyz4, size_t m) {
    if (!h || (!xyz4 && m)) return PF_EINVAL;
    if (m > h->map_cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(h->device));
    const int mm[2] = {(int)m, 0};
    if (m) PF_HIP_TRY(hipMemcpyAsync(h->d_map, xyz4, sizeof(float4) * m, hipMemcpyHostToDevice, h->stream));
    PF_HIP_TRY(hipMemcpyAsync(h->d_m, mm, sizeof(mm), hipMemcpyHostToDevice, h->stream));
    grid_build(h->grid, GridPtrs{{h->d_map, nullptr, nullptr}, {h->d_m, nullptr, nullptr}, 1}, h->prim, h->stream);
    // the thick-row copy: sizes, scan, triple scatter (the grid's slots and cell_start)
    hipLaunchKernelGGL(k_thick_count, dim3(1024), dim3(256), 0, h->stream, h->grid.dims, h->grid.cell_start, h->tcount,
                       h->d_nt);
    scan_exclusive(h->tcount, h->tstart, h->d_nt, nullptr, h->prim, h->stream);
    hipLaunchKernelGGL(k_thick_scatter, dim3(1024), dim3(256), 0, h->stream, h->d_map, h->d_m, h->grid.dims,
                       h->grid.cell_start, h->grid.slot, h->tstart, h->tpts);
    int err = 0;
    PF_HIP_TRY(hipMemcpyAsync(&err, h->grid.err, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    PF_HIP_TRY(hipGetLastError());
    return err ? PF_ECAPACITY : PF_OK;
}

int pf_knn_query(pf_knn* h, const float* q4, size_t nq, int32_t* idx, float* d2) {
    if (!h || (!q4 && nq)) return PF_EINVAL;
    if (nq > h->q_cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(h->device));
    h->nq = (int)nq;
    if (nq == 0) return PF_OK;
    PF_HIP_TRY(hipMemcpyAsync(h->d_q, q4, sizeof(float4) * nq, hipMemcpyHostToDevice, h->stream));
    GridView gv{h->grid.dims, h->grid.cell_start, h->grid.cpts};
    launch_knn(h, gv);
    if (idx) PF_HIP_TRY(hipMemcpyAsync(idx, h->d_idx, sizeof(int) * 5 * nq, hipMemcpyDeviceToHost, h->stream));
    if (d2) PF_HIP_TRY(hipMemcpyAsync(d2, h->d_d2, sizeof(float) * 5 * nq, hipMemcpyDeviceToHost, h->stream));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    PF_HIP_TRY(hipGetLastError());
    return PF_OK;
}

int pf_knn_bench(pf_knn* h, int iters, double* avg_ms, double* alg_bytes) {
    if (!h || iters <= 0 || h->nq <= 0) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->device));
    GridView gv{h->grid.dims, h->grid.cell_start, h->grid.cpts};
    PF_HIP_TRY(hipMemsetAsync(h->d_pop, 0, sizeof(unsigned long long), h->stream));
    hipLaunchKernelGGL(k_knn_cellpop, dim3((unsigned)((h->nq + 255) / 256)), dim3(256), 0, h->stream, gv, h->d_q,
                       h->nq, h->d_pop);
    unsigned long long pop = 0;
    PF_HIP_TRY(hipMemcpyAsync(&pop, h->d_pop, sizeof(pop), hipMemcpyDeviceToHost, h->stream));
    launch_knn(h, gv);  // warm
    hipEvent_t e0, e1;
    PF_HIP_TRY(hipEventCreate(&e0));
    PF_HIP_TRY(hipEventCreate(&e1));
    PF_HIP_TRY(hipEventRecord(e0, h->stream));
    for (int it = 0; it < iters; ++it)
        launch_knn(h, gv);
    PF_HIP_TRY(hipEventRecord(e1, h->stream));
    PF_HIP_TRY(hipEventSynchronize(e1));
    float ms = 0;
    PF_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    PF_HIP_TRY(hipGetLastError());
    if (avg_ms) *avg_ms = ms / iters;
    if (alg_bytes) *alg_bytes = (double)h->nq * (16.0 + 40.0 + 27.0 * 8.0) + 16.0 * (double)pop;
    return PF_OK;
}

// development: lanes per query of the standalone kernel (8 or 16; not part of the C ABI)
int pf_knn_set_team(pf_knn* h, int team) {
    if (!h || (team != 1 && team != 2 && team != 4 && team != 8 && team != 16)) return PF_EINVAL;
    h->team = team;
    return PF_OK;
}

// development: 1 = the thick-row layout (default), 0 = the 9-row walk of the cell grid
int pf_knn_set_layout(pf_knn* h, int thick) {
    if (!h) return PF_EINVAL;
    h->thick = thick != 0;
    if (!h->thick && h->team > 16) h->team = 8;
    return PF_OK;
}

}  // extern "C"
