// curvedVoxel (DCVC) on the device (see pf_dcvc.h) and its C ABI (pf_dcvc_*).
#include "pf_dcvc.h"

#include <cfloat>
#include <cstdlib>
#include <climits>
#include <cmath>
#include <vector>

namespace pf {
namespace {

constexpr double kPi = 3.14159265358979323846;   // M_PI

struct DcvcDev {
    pf_dcvc_params prm;
    u64* red;
    double* bounds;              // [kDcMaxBounds] + [kDcMaxBounds]: minPitch
    int* dim;
    double4* pol;
    u32 *keys, *vals, *segstart;
    int* seg_aux;
    u32 *parent, *csize, *cfirst, *crank, *okeys, *ovals, *plab;
    u32 *ukey, *ucount;
    int* vtab;
    long long vtab_cells;
    u32* edges;        // [cap][26] per voxel: the search edges it unions
    u32* ecount;       // [cap]
};

__device__ __forceinline__ u64 dord(double d) {       // order-preserving bits of a double
    const u64 b = (u64)__double_as_longlong(d);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ __forceinline__ double dord_inv(u64 o) {
    const u64 b = (o >> 63) ? (o & ~(1ull << 63)) : ~o;
    return __longlong_as_double((long long)b);
}

// convertToPolar (:85-136) and the grid dimensions (:121-135); the last workgroup forms the bounds
__global__ void __launch_bounds__(256) k_dc_polar(const float4* __restrict__ pts, const int* __restrict__ d_n, DcvcDev d) {
    __shared__ u64 red[4][4];
    __shared__ int last;
    const int n = *d_n;
    u64 mr = 0ull, mnp = ~0ull, mxp = 0ull, mnr = ~0ull;  // max range, min pitch, max pitch, min range (ordered)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        const double x = p.x, y = p.y, z = p.z;
        const double r = sqrt((x * x + y * y) + z * z);
        const double pitch = asin(z / r) * 180.0 / kPi;
        const double ang = atan2(y, x);
        const double az = ang > 0.0 ? ang * 180 / kPi : (ang + 2 * kPi) * 180 / kPi;
        const bool in = !(r >= d.prm.max_range || r <= d.prm.min_range);
        d.pol[i] = in ? make_double4(r, pitch, az, 0.0) : make_double4(0.0, 0.0, 0.0, 0.0);
        if (in) {
            mr = max(mr, dord(r));
            mnp = min(mnp, dord(pitch));
            mxp = max(mxp, dord(pitch));
            mnr = min(mnr, dord(r));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mr = max(mr, (u64)__shfl_xor((long long)mr, o, 64));
        mnp = min(mnp, (u64)__shfl_xor((long long)mnp, o, 64));
        mxp = max(mxp, (u64)__shfl_xor((long long)mxp, o, 64));
        mnr = min(mnr, (u64)__shfl_xor((long long)mnr, o, 64));
    }
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) { red[0][w] = mr; red[1][w] = mnp; red[2][w] = mxp; red[3][w] = mnr; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k) {
            mr = max(mr, red[0][k]);
            mnp = min(mnp, red[1][k]);
            mxp = max(mxp, red[2][k]);
            mnr = min(mnr, red[3][k]);
        }
        if (mr) __hip_atomic_fetch_max(&d.red[0], mr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mnp != ~0ull) __hip_atomic_fetch_min(&d.red[1], mnp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mxp) __hip_atomic_fetch_max(&d.red[2], mxp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mnr != ~0ull) __hip_atomic_fetch_min(&d.red[4], mnr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(&d.red[3], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        if (last) {
            const u64 gr = __hip_atomic_load(&d.red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const u64 gn = __hip_atomic_load(&d.red[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const u64 gx = __hip_atomic_load(&d.red[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const u64 gm = __hip_atomic_load(&d.red[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&d.red[4], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&d.red[0], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&d.red[1], ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&d.red[2], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&d.red[3], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool first = d.dim[D_CALLS] == 0;                 // member defaults: 5 m (.hpp:105-106)
            const double init = first ? 5.0 : 0.0;
            double maxPolar = init, minPolar = init, minPitch = 0.0, maxPitch = 0.0;
            if (gr) { const double v = dord_inv(gr); maxPolar = v > maxPolar ? v : maxPolar; }
            if (gm != ~0ull) { const double v = dord_inv(gm); minPolar = v < minPolar ? v : minPolar; }
            if (gn != ~0ull) { const double v = dord_inv(gn); minPitch = v < minPitch ? v : minPitch; }
            if (gx) { const double v = dord_inv(gx); maxPitch = v > maxPitch ? v : maxPitch; }
            const int width = (int)(round(360.0 / d.prm.delta_a) + 1);
            const int height = (int)((maxPitch - minPitch) / d.prm.delta_p);
            double range = minPolar;                        // :127-134
            int step = 1, k = 0;
            d.dim[D_ERR] = 0;                               // per call: a past overflow does not stick
            while (range <= maxPolar) {
                if (k >= kDcMaxBounds) { d.dim[D_ERR] = 1; break; }
                range += (d.prm.start_r - step * d.prm.delta_r);
                d.bounds[k++] = range;
                step++;
            }
            d.dim[D_POLAR] = k;
            d.dim[D_WIDTH] = width;
            d.dim[D_HEIGHT] = height;
            d.dim[D_N] = n;
            d.bounds[kDcMaxBounds] = minPitch;
            d.dim[D_CALLS] += 1;
        }
    }
}

// createHashTable (:143-177): polar / pitch / azimuth index and the voxel index of every point
// (the digit histograms of both sorts are fused into their key kernels, k_dc_keys and k_dc_label)
__global__ void __launch_bounds__(256) k_dc_keys(const int* __restrict__ d_n, DcvcDev d, SortHist sh) {
    __shared__ u32 lh[4][256];
    sort_hist_begin(lh);
    const int n = *d_n;
    const int P = d.dim[D_POLAR], W = d.dim[D_WIDTH];
    const double minPitch = d.bounds[kDcMaxBounds];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const double4 c = d.pol[i];
        int lo = 0, hi = P;                               // getPolarIndex (:69-78): first r < bound
        while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if (c.x < d.bounds[m]) hi = m; else lo = m + 1;
        }
        const int polar = lo < P ? lo : P - 1;
        const int pitch = (int)round((c.y - minPitch) / d.prm.delta_p);
        const int az = (int)round(c.z / d.prm.delta_a);
        const int vox = (az * (P + 1) + polar) + pitch * (P + 1) * (W + 1);
        d.keys[i] = (u32)vox;
        d.vals[i] = (u32)i;
        sort_hist_add(lh, (u32)vox, sh.passes);
    }
    sort_hist_end(lh, sh, n, n);
}

// per voxel (segment of the sorted keys): its key, point count; union-find and component state reset
__global__ void __launch_bounds__(256) k_dc_voxels(DcvcDev d) {
    const int nseg = d.seg_aux[0], nvalid = d.seg_aux[4];
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        const u32 b0 = d.segstart[s], b1 = s + 1 < nseg ? d.segstart[s + 1] : (u32)nvalid;
        const u32 key = d.keys[b0];
        d.ukey[s] = key;
        d.ucount[s] = b1 - b0;
        if ((long long)key < d.vtab_cells) d.vtab[key] = s;
        d.csize[s] = 0u;
        d.cfirst[s] = 0xFFFFFFFFu;
        d.crank[s] = 0u;
    }
}

__device__ __forceinline__ u32 dc_parent(const DcvcDev& d, u32 v) {
    return __hip_atomic_load(&d.parent[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// root of v, halving the path on the way (every store replaces a parent by one of its ancestors, so
// concurrent finds and hooks see a forest with the same roots)
__device__ __forceinline__ u32 dc_find(const DcvcDev& d, u32 v) {
    for (;;) {
        const u32 p = dc_parent(d, v);
        if (p == v) return v;
        const u32 gp = dc_parent(d, p);
        if (gp == p) return p;
        __hip_atomic_store(&d.parent[v], gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v = gp;
    }
}

// slot of the occupied voxel with key nk, or -1: the table, or a binary search over the sorted keys
__device__ __forceinline__ int dc_lookup(const DcvcDev& d, long long nk, int nseg) {
    if (nk < d.vtab_cells) return d.vtab[nk];
    int lo = 0, hi = nseg;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if ((long long)d.ukey[m] < nk) lo = m + 1; else hi = m;
    }
    return (lo < nseg && (long long)d.ukey[lo] == nk) ? lo : -1;
}

// the occupied search positions of voxel s (searchKNN :196-225: pitch layers above `height` skipped,
// azimuth -1 wrapped to width - 1, azimuth above 300 clamped to 300), -1 where empty
__device__ __forceinline__ void dc_search(const DcvcDev& d, int s, int nseg, int P, int W, int H, long long L,
                                          int (&nb)[27], int& x0, int& z0) {
    const long long key = d.ukey[s];
    z0 = (int)(key / L);
    const int rem = (int)(key % L);
    x0 = rem / (P + 1);
    const int y0 = rem % (P + 1);
#pragma unroll
    for (int k = 0; k < 27; ++k) {
        const int z = z0 - 1 + k / 9, y = y0 - 1 + (k / 3) % 3, x = x0 - 1 + k % 3;
        int ax = x;
        if (ax < 0) ax = W - 1;
        if (ax > 300) ax = 300;
        const long long nk = ((long long)ax * (P + 1) + y) + (long long)z * L;
        nb[k] = (z < 0 || z > H || y < 0 || y > P) ? -1 : dc_lookup(d, nk, nseg);
    }
}

// per voxel: its occupied search positions; the smallest (or itself) becomes its parent (ECL-CC style
// initialisation, so the trees the unions walk start shallow) and the other edges it must union are
// listed (an edge whose reverse is also a search edge is listed at its smaller end only)
__device__ __forceinline__ bool dc_take(const DcvcDev& d, int s, int v, int m, int x0, int z0, int P, int W, int H,
                                        long long L);
__global__ void __launch_bounds__(256) k_dc_link(DcvcDev d) {
    const int nseg = d.seg_aux[0];
    const int P = d.dim[D_POLAR], W = d.dim[D_WIDTH], H = d.dim[D_HEIGHT];
    const long long L = (long long)(P + 1) * (W + 1);
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        int nb[27], x0, z0;
        dc_search(d, s, nseg, P, W, H, L, nb, x0, z0);
        int m = s;
#pragma unroll
        for (int k = 0; k < 27; ++k)
            if (nb[k] >= 0 && nb[k] < m) m = nb[k];
        d.parent[s] = (u32)m;
        u32* e = d.edges + (size_t)s * 26;
        u32 ne = 0;
#pragma unroll
        for (int k = 0; k < 27; ++k)
            if (dc_take(d, s, nb[k], m, x0, z0, P, W, H, L)) e[ne++] = (u32)nb[k];
        d.ecount[s] = ne;
    }
}

// every search edge s -> nb unioned (lock-free, the smaller root wins, so the components do not depend
// on the order of the unions). An edge whose reverse nb -> s is also a search edge is taken from its
// smaller end only; the edge to the smallest position is the initial link already.
__device__ __forceinline__ bool dc_take(const DcvcDev& d, int s, int v, int m, int x0, int z0, int P, int W, int H,
                                        long long L) {
    if (v < 0 || v == s || v == m) return false;
    if (v < s && z0 <= H) {                                   // taken from v's side if v finds s
        const int x1 = (int)(((long long)d.ukey[v] % L) / (P + 1));
        int xl = x1 - 1, xr = x1 + 1;
        if (xl < 0) xl = W - 1;
        if (xl > 300) xl = 300;
        if (xr > 300) xr = 300;
        if (x0 == x1 || x0 == xl || x0 == xr) return false;
    }
    return true;
}

__global__ void __launch_bounds__(256) k_dc_union(DcvcDev d) {
    const int nseg = d.seg_aux[0];
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        const u32* e = d.edges + (size_t)s * 26;
        const u32 ne = d.ecount[s];
        u32 a = (u32)s;                                       // this voxel's root, refreshed per edge
        for (u32 j = 0; j < ne; ++j) {
            a = dc_find(d, a);
            u32 b = dc_find(d, e[j]);
            while (a != b) {
                if (a > b) { const u32 t = a; a = b; b = t; }
                u32 exp = b;
                if (__hip_atomic_compare_exchange_strong(&d.parent[b], &exp, a, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                    break;
                b = dc_find(d, exp);
                a = dc_find(d, a);
            }
        }
    }
}

// component point counts and first points at the roots: one atomic pair per distinct root of a wave
// (voxel s of this lane, r its root)
__device__ __forceinline__ void dc_sizes_wave(const DcvcDev& d, int s, int nseg, u32 r) {
    const int l = lane_id();
    bool todo = s < nseg;
    const u32 c = todo ? d.ucount[s] : 0u;
    const u32 f = todo ? d.vals[d.segstart[s]] : 0xFFFFFFFFu;   // points of a voxel in index order
    for (;;) {
        const u64 m = __ballot(todo);
        if (!m) break;
        const int lead = __ffsll((long long)m) - 1;
        const u32 r0 = __shfl(r, lead, 64);
        const bool mine = todo && r == r0;
        u32 cs = mine ? c : 0u, fm = mine ? f : 0xFFFFFFFFu;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            cs += __shfl_xor(cs, o, 64);
            fm = min(fm, (u32)__shfl_xor(fm, o, 64));
        }
        if (l == lead) {
            atomicAdd(&d.csize[r0], cs);
            atomicMin(&d.cfirst[r0], fm);
        }
        todo = todo && !mine;
    }
}

// full compression (every voxel's parent its root), each component's point count and first point at
// its root, and the voxel table emptied for the next call
__global__ void __launch_bounds__(256) k_dc_compress(DcvcDev d) {
    const int nseg = d.seg_aux[0];
    for (int s0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63); s0 < nseg; s0 += gridDim.x * blockDim.x) {
        const int s = s0 + lane_id();                          // uniform trip count per wave
        u32 v = (u32)s;
        if (s < nseg) {
            while (d.parent[v] != v) v = d.parent[v];
            d.parent[s] = v;
            const u32 key = d.ukey[s];
            if ((long long)key < d.vtab_cells) d.vtab[key] = -1;
        }
        dc_sizes_wave(d, s, nseg, v);
    }
}

// labelAnalysis (:325-355), one workgroup of 1024: the components larger than minSeg ranked by size
// (ties by first point); crank[root] = rank + 1. key: kDcMaxClusters LDS words; root(v): v's root;
// the sizes are read back with agent-scope loads (they were formed by atomics)
template <class RootF>
__device__ __forceinline__ void dc_rank(const DcvcDev& d, int nseg, u64* key, int& cnt, u32& kept, RootF root) {
    if (threadIdx.x == 0) { cnt = 0; kept = 0; }
    __syncthreads();
    for (int s = threadIdx.x; s < nseg; s += blockDim.x) {
        if (root(s) != (u32)s) continue;
        const u32 cs = __hip_atomic_load(&d.csize[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((int)cs <= d.prm.min_seg) continue;
        const u32 cf = __hip_atomic_load(&d.cfirst[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int k = atomicAdd(&cnt, 1);
        if (k < kDcMaxClusters) key[k] = ((u64)(~cs) << 32) | (u64)cf;
        else d.dim[D_ERR] = 2;
        atomicAdd(&kept, cs);
    }
    __syncthreads();
    const int m = cnt < kDcMaxClusters ? cnt : kDcMaxClusters;
    int np2 = 1;
    while (np2 < m) np2 <<= 1;
    for (int i = m + threadIdx.x; i < np2; i += blockDim.x) key[i] = ~0ull;
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1)                      // bitonic sort, ascending
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np2; i += blockDim.x) {
                const int o = i ^ j;
                if (o > i) {
                    const u64 a = key[i], b = key[o];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) { key[i] = b; key[o] = a; }
                }
            }
            __syncthreads();
        }
    // the root of the component with first point f: the voxel holding f (found through the point's key)
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const u32 f = (u32)(key[i] & 0xffffffffull);
        const u32 vk = d.okeys[f];                           // k_dc_pointvox: voxel slot of point f
        d.crank[root((int)vk)] = (u32)(i + 1);
    }
    if (threadIdx.x == 0) {
        d.dim[D_NCLUST] = m;
        d.dim[D_NKEPT] = (int)kept;
    }
}

__global__ void __launch_bounds__(1024) k_dc_rank(DcvcDev d) {
    __shared__ u64 key[kDcMaxClusters];
    __shared__ int cnt;
    __shared__ u32 kept;
    const int nseg = d.seg_aux[0];
    dc_rank(d, nseg, key, cnt, kept, [&](int v) { return d.parent[v]; });
}

// voxel slot of every point (okeys, reused before the final keys are written)
__global__ void __launch_bounds__(256) k_dc_pointvox(DcvcDev d) {
    const int nseg = d.seg_aux[0], nvalid = d.seg_aux[4];
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        const u32 b0 = d.segstart[s], b1 = s + 1 < nseg ? d.segstart[s + 1] : (u32)nvalid;
        for (u32 j = b0; j < b1; ++j) d.okeys[d.vals[j]] = (u32)s;
    }
}

// per point: sort key = its component's rank (published order) or dropped, label = rank + 1 or 0
__global__ void __launch_bounds__(256) k_dc_label(DcvcDev d, const int* __restrict__ d_n, SortHist sh) {
    __shared__ u32 lh[4][256];
    sort_hist_begin(lh);
    const int n = *d_n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32 r = d.crank[d.parent[d.okeys[i]]];
        const u32 key = r ? r - 1 : 0xFFFFFFFFu;
        d.plab[i] = r;
        d.okeys[i] = key;
        d.ovals[i] = (u32)i;
        sort_hist_add(lh, key, sh.passes);
    }
    sort_hist_end(lh, sh, n, n);
}

constexpr int kDcGrid = 256;

}  // namespace

int dcvc_alloc(DcvcGPU& g, size_t cap) {
    g.cap = cap;
    auto A = [&](auto** p, size_t bytes) { return hipMalloc((void**)p, bytes) == hipSuccess; };
    if (!A(&g.red, sizeof(u64) * 8) || !A(&g.bounds, sizeof(double) * (kDcMaxBounds + 2)) ||
        !A(&g.dim, sizeof(int) * 8) || !A(&g.pol, sizeof(double4) * cap) || !A(&g.keys, sizeof(u32) * cap) ||
        !A(&g.vals, sizeof(u32) * cap) || !A(&g.segstart, sizeof(u32) * (cap + 1)) || !A(&g.seg_aux, sizeof(int) * 8) ||
        !A(&g.parent, sizeof(u32) * cap) || !A(&g.csize, sizeof(u32) * cap) || !A(&g.cfirst, sizeof(u32) * cap) ||
        !A(&g.crank, sizeof(u32) * cap) || !A(&g.okeys, sizeof(u32) * cap) || !A(&g.ovals, sizeof(u32) * cap) ||
        !A(&g.plab, sizeof(u32) * cap) || !A(&g.ukey, sizeof(u32) * cap) || !A(&g.ucount, sizeof(u32) * cap) ||
        !A(&g.edges, sizeof(u32) * 26 * cap) || !A(&g.ecount, sizeof(u32) * cap))
        return PF_ENOMEM;
    const u64 r0[8] = {0ull, ~0ull, 0ull, 0ull, ~0ull, 0ull, 0ull, 0ull};
    if (hipMemcpy(g.red, r0, sizeof(r0), hipMemcpyHostToDevice) != hipSuccess) return PF_EHIP;
    if (hipMemset(g.dim, 0, sizeof(int) * 8) != hipSuccess) return PF_EHIP;
    return prim_alloc(g.w, cap);
}

void dcvc_free(DcvcGPU& g) {
    void* ps[] = {g.red, g.bounds, g.dim, g.pol, g.keys, g.vals, g.segstart, g.seg_aux, g.parent, g.csize,
                  g.cfirst, g.crank, g.okeys, g.ovals, g.plab, g.ukey, g.ucount, g.vtab, g.edges, g.ecount};
    for (void* p : ps) (void)hipFree(p);
    prim_free(g.w);
    g = DcvcGPU{};
}

int dcvc_reset(DcvcGPU& g, hipStream_t s) {
    PF_HIP_TRY(hipMemsetAsync(g.dim + D_CALLS, 0, sizeof(int), s));
    PF_HIP_TRY(hipMemsetAsync(g.dim + D_ERR, 0, sizeof(int), s));
    return PF_OK;
}

int dcvc_mark_called(DcvcGPU& g, hipStream_t s) {
    PF_HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g.dim + D_CALLS), 1, 1, s));
    PF_HIP_TRY(hipMemsetAsync(g.dim + D_ERR, 0, sizeof(int), s));
    return PF_OK;
}

// cells of the voxel index space: (polarNum + 1) (width + 1) (height + 3), polarNum bounded by the
// rings up to max(5 m, max_range) and the pitch layers (height + 1 of them, plus the top layer quirk)
// by 180 degrees
static long long dcvc_key_cells(const pf_dcvc_params& p) {
    double range = 0.0;
    long long P = 0;
    const double top = p.max_range > 5.0 ? p.max_range : 5.0;
    for (int step = 1; range <= top && P < kDcMaxBounds; ++step, ++P) range += (p.start_r - step * p.delta_r);
    const long long W = (long long)(std::round(360.0 / p.delta_a) + 1);
    const long long H = (long long)(180.0 / p.delta_p) + 2;
    return (P + 1) * (W + 1) * (H + 1);
}
static int dcvc_key_bits(const pf_dcvc_params& p) {
    const long long m = dcvc_key_cells(p);
    int b = 1;
    while (b < 32 && (1ll << b) < m) ++b;
    return b;
}

constexpr long long kDcTableMaxCells = 1ll << 26;          // 256 MB of table at most

int dcvc_set_params(DcvcGPU& g, const pf_dcvc_params& p) {
    g.prm = p;
    const long long m = dcvc_key_cells(p);
    if (m <= g.vtab_cells) return PF_OK;
    (void)hipFree(g.vtab);
    g.vtab = nullptr;
    g.vtab_cells = 0;
    if (m > kDcTableMaxCells) return PF_OK;                 // binary-search lookups
    if (hipMalloc(&g.vtab, sizeof(int) * (size_t)m) != hipSuccess) return PF_ENOMEM;
    if (hipMemset(g.vtab, 0xFF, sizeof(int) * (size_t)m) != hipSuccess) return PF_EHIP;
    if (hipDeviceSynchronize() != hipSuccess) return PF_EHIP;
    g.vtab_cells = m;
    return PF_OK;
}

void dcvc_enqueue(DcvcGPU& g, const float4* pts, const int* d_n, hipStream_t s, u32** out_idx) {
    DcvcDev d{g.prm, g.red, g.bounds, g.dim, g.pol, g.keys, g.vals, g.segstart, g.seg_aux, g.parent,
              g.csize, g.cfirst, g.crank, g.okeys, g.ovals, g.plab, g.ukey, g.ucount, g.vtab, g.vtab_cells, g.edges, g.ecount};
    hipLaunchKernelGGL(k_dc_polar, dim3(kDcGrid), dim3(256), 0, s, pts, d_n, d);
    hipLaunchKernelGGL(k_dc_keys, dim3(kDcGrid), dim3(256), 0, s, d_n, d, sort_hist(g.w, dcvc_key_bits(g.prm), false));
    u32 *ks = nullptr, *vs = nullptr;                       // sorted (voxel, point) pairs
    radix_sort_pairs(g.keys, g.vals, d_n, dcvc_key_bits(g.prm), g.w, s, &ks, &vs, true);
    d.keys = ks;
    d.vals = vs;
    segment_starts(ks, d_n, g.segstart, g.seg_aux, g.seg_aux + 1, g.seg_aux + 4, g.w, s);
    hipLaunchKernelGGL(k_dc_voxels, dim3(kDcGrid), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_dc_pointvox, dim3(kDcGrid), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_dc_link, dim3(kDcGrid), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_dc_union, dim3(kDcGrid), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_dc_compress, dim3(kDcGrid), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_dc_rank, dim3(1), dim3(1024), 0, s, d);
    hipLaunchKernelGGL(k_dc_label, dim3(kDcGrid), dim3(256), 0, s, d, d_n, sort_hist(g.w, 16, true));
    radix_sort_pairs(g.okeys, g.ovals, d_n, 16, g.w, s, nullptr, nullptr, true);
    if (out_idx) *out_idx = g.ovals;
}

}  // namespace pf

// ==================================================================================================
// pf_dcvc C ABI
// ==================================================================================================
using namespace pf;

struct pf_dcvc {
    int device = 0;
    hipStream_t stream = nullptr;
    DcvcGPU g;
    float4* d_pts = nullptr;
    int* d_n = nullptr;
    std::vector<float4> host;
};

namespace {
// The ring widths start_r - k delta_r (:127-134) must stay positive out to max(5 m, max_range) within
// kDcMaxBounds rings; otherwise the reference's loop never reaches the far points (an endless loop
// there, an overflow here), so such a parameter set is refused.
bool dcvc_params_ok(const pf_dcvc_params* p) {
    if (!(p && p->delta_p > 0 && p->delta_a > 0 && p->start_r > 0 && p->delta_r >= 0 && p->max_range > 0 &&
          p->max_range < 1e5 && p->min_seg >= 0))
        return false;
    const double top = p->max_range > 5.0 ? p->max_range : 5.0;
    double range = 0.0;
    for (int step = 1; range <= top; ++step) {
        const double w = p->start_r - step * p->delta_r;
        if (!(w > 0) || step > kDcMaxBounds) return false;
        range += w;
    }
    return true;
}
}  // namespace

namespace pf {
bool dcvc_params_valid(const pf_dcvc_params* p) { return dcvc_params_ok(p); }
}  // namespace pf

extern "C" {

void pf_dcvc_default_params(pf_dcvc_params* p) {
    if (!p) return;
    p->start_r = 1.0;       // config/config.yaml:50
    p->delta_r = 0.003;     // :51
    p->delta_p = 1.2;       // :52
    p->delta_a = 1.2;       // :53
    p->min_seg = 80;        // :54
    p->min_range = 1.0;     // :7
    p->max_range = 120.0;   // :8
}

int pf_dcvc_create(const pf_dcvc_params* p, int device, size_t max_points, pf_dcvc** out) {
    if (!out || !dcvc_params_ok(p) || max_points == 0 || max_points > (size_t)INT_MAX / 2) return PF_EINVAL;
    *out = nullptr;
    int ndev = 0;
    PF_HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(device));
    pf_dcvc* h = new pf_dcvc();
    h->device = device;
    h->g.prm = *p;
    int rc = PF_OK;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) rc = PF_EHIP;
    if (rc == PF_OK) rc = dcvc_alloc(h->g, max_points);
    if (rc == PF_OK) rc = dcvc_set_params(h->g, *p);
    if (rc == PF_OK && hipMalloc(&h->d_pts, sizeof(float4) * max_points) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMalloc(&h->d_n, sizeof(int)) != hipSuccess) rc = PF_ENOMEM;
    if (rc != PF_OK) {
        pf_dcvc_destroy(h);
        return rc;
    }
    *out = h;
    return PF_OK;
}

int pf_dcvc_destroy(pf_dcvc* h) {
    if (!h) return PF_EINVAL;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    dcvc_free(h->g);
    (void)hipFree(h->d_pts);
    (void)hipFree(h->d_n);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return PF_OK;
}

// development probe (not part of include/pfilter_hip.h): the grid of the last call
int pf_dcvc_debug(pf_dcvc* h, double* out8) {
    if (!h || !out8) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->device));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    int dim[8];
    double b0 = 0, mp = 0;
    PF_HIP_TRY(hipMemcpy(dim, h->g.dim, sizeof(dim), hipMemcpyDeviceToHost));
    PF_HIP_TRY(hipMemcpy(&b0, h->g.bounds, sizeof(double), hipMemcpyDeviceToHost));
    PF_HIP_TRY(hipMemcpy(&mp, h->g.bounds + kDcMaxBounds, sizeof(double), hipMemcpyDeviceToHost));
    out8[0] = b0; out8[1] = mp; out8[2] = dim[D_POLAR]; out8[3] = dim[D_WIDTH]; out8[4] = dim[D_HEIGHT];
    out8[5] = dim[D_CALLS]; out8[6] = dim[D_NKEPT]; out8[7] = dim[D_NCLUST];
    return PF_OK;
}

int pf_dcvc_reset(pf_dcvc* h) {
    if (!h) return PF_EINVAL;
    PF_HIP_TRY(hipSetDevice(h->device));
    int rc = dcvc_reset(h->g, h->stream);
    if (rc) return rc;
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    return PF_OK;
}

int pf_dcvc_reserve(pf_dcvc* h, size_t max_points) {
    if (!h || max_points == 0 || max_points > (size_t)INT_MAX / 2) return PF_EINVAL;
    if (max_points <= h->g.cap) return PF_OK;
    PF_HIP_TRY(hipSetDevice(h->device));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    int calls = 0;                                   // the call state survives the re-allocation
    PF_HIP_TRY(hipMemcpy(&calls, h->g.dim + D_CALLS, sizeof(int), hipMemcpyDeviceToHost));
    const pf_dcvc_params prm = h->g.prm;
    dcvc_free(h->g);
    (void)hipFree(h->d_pts);
    h->d_pts = nullptr;
    h->g.prm = prm;
    int rc = dcvc_alloc(h->g, max_points);
    if (rc == PF_OK) rc = dcvc_set_params(h->g, prm);
    if (rc == PF_OK && hipMalloc(&h->d_pts, sizeof(float4) * max_points) != hipSuccess) rc = PF_ENOMEM;
    if (rc == PF_OK && hipMemcpy(h->g.dim + D_CALLS, &calls, sizeof(int), hipMemcpyHostToDevice) != hipSuccess) rc = PF_EHIP;
    return rc;
}

int pf_dcvc_run(pf_dcvc* h, const float* xyz, size_t n, size_t stride_bytes, int32_t* out_idx, size_t* n_out,
                int32_t* label, size_t cap) {
    if (!h || (!xyz && n) || stride_bytes < 12) return PF_EINVAL;
    if (n > h->g.cap) return PF_ECAPACITY;
    PF_HIP_TRY(hipSetDevice(h->device));
    if (n_out) *n_out = 0;
    if (n == 0) return PF_OK;                                   // :462-466: nothing to convert
    h->host.resize(n);
    const char* b = reinterpret_cast<const char*>(xyz);
    for (size_t i = 0; i < n; ++i) {
        const float* q = reinterpret_cast<const float*>(b + i * stride_bytes);
        h->host[i] = make_float4(q[0], q[1], q[2], 0.f);
    }
    const int ni = (int)n;
    PF_HIP_TRY(hipMemcpyAsync(h->d_pts, h->host.data(), sizeof(float4) * n, hipMemcpyHostToDevice, h->stream));
    PF_HIP_TRY(hipMemcpyAsync(h->d_n, &ni, sizeof(int), hipMemcpyHostToDevice, h->stream));
    u32* idx = nullptr;
    dcvc_enqueue(h->g, h->d_pts, h->d_n, h->stream, &idx);
    PF_HIP_TRY(hipGetLastError());
    int dim[8];
    PF_HIP_TRY(hipMemcpyAsync(dim, h->g.dim, sizeof(dim), hipMemcpyDeviceToHost, h->stream));
    PF_HIP_TRY(hipStreamSynchronize(h->stream));
    if (dim[D_ERR]) {
        (void)hipMemset(h->g.dim + D_ERR, 0, sizeof(int));
        return PF_ECAPACITY;
    }
    const size_t k = (size_t)dim[D_NKEPT];
    if (n_out) *n_out = k;
    if (out_idx && k > cap) return PF_ECAPACITY;
    if (out_idx && k) PF_HIP_TRY(hipMemcpy(out_idx, idx, sizeof(int32_t) * k, hipMemcpyDeviceToHost));
    if (label) PF_HIP_TRY(hipMemcpy(label, h->g.plab, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    return PF_OK;
}

}  // extern "C"
