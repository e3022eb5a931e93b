// Feature extraction kernels (LaserProcessingClass::featureExtraction, src/laserProcessingClass.cpp:10-209).
//
//  k_fe_ring      ring id per point (range gate + elevation formula, :22-61) + per-block ring histogram
//  k_fe_ring_scan exclusive scan of the (ring, block) histogram -> stable ring partition offsets
//  k_fe_scatter   stable scatter into ring order (input order kept inside a ring, :62)
//  k_fe_sector    one workgroup per (ring, sector): 11-tap curvature (:73-77), LDS bitonic sort by
//                 (curvature, id), greedy edge pick with neighbour suppression (:110-148) and the
//                 ascending surf sweep (:198-205)
//  k_fe_out_scan  output offsets in ring -> sector order
//  k_fe_gather    bit-exact copies of the picked points
#include "pf_fe.h"

#include <cfloat>
#include <climits>

namespace pf {
namespace {

__device__ __forceinline__ int ring_of(const float4 p, int L, double mind, double maxd, int sqrt_double, double top,
                                       double scale) {
    const float sq = p.x * p.x + p.y * p.y;   // float expression (:23)
    const double distance = sqrt_double ? sqrt((double)sq) : (double)sqrtf(sq);
    if (distance < mind || distance > maxd) return -1;
    const double angle = atan(p.z / distance) * 180 / M_PI;
    int scanID = 0;
    if (scale > 0.0) {                       // extension: linear beam model (pf_fe_set_ring_model)
        scanID = int((top - angle) * scale);
        if (!(top - angle >= 0.0) || scanID > L - 1) return -1;
    } else if (L == 16) {
        scanID = int((angle + 15) / 2 + 0.5);
        if (scanID > (L - 1) || scanID < 0) return -1;
    } else if (L == 32) {
        scanID = int((angle + 92.0 / 3.0) * 3.0 / 4.0);
        if (scanID > (L - 1) || scanID < 0) return -1;
    } else if (L == 64) {
        if (angle >= -8.83)
            scanID = int((2 - angle) * 3.0 + 0.5);
        else
            scanID = L / 2 + int((-8.83 - angle) * 2.0 + 0.5);
        if (angle > 2 || angle < -24.33 || scanID > 63 || scanID < 0) return -1;
    } else {
        scanID = 0;  // "wrong scan number": every point lands in ring 0 (:58-61)
    }
    return scanID;
}

__global__ void __launch_bounds__(256) k_fe_ring(const float4* __restrict__ in, const int* __restrict__ d_n, int L,
                                                  double mind, double maxd, int sqrt_double, double top, double scale,
                                                  int* __restrict__ ring, u32* __restrict__ blkhist) {
    __shared__ u32 h[kMaxRings];
    const int n = *d_n;
    const int nblk = n > 0 ? (n + 255) / 256 : 1;
    if ((int)blockIdx.x >= nblk) return;
    const int t = threadIdx.x;
    for (int r = t; r < L; r += 256) h[r] = 0;
    __syncthreads();
    const int i = blockIdx.x * 256 + t;
    if (i < n) {
        const int r = ring_of(in[i], L, mind, maxd, sqrt_double, top, scale);
        ring[i] = r;
        if (r >= 0) atomicAdd(&h[r], 1u);
    }
    __syncthreads();
    for (int r = t; r < L; r += 256) blkhist[r * nblk + blockIdx.x] = h[r];
}

__device__ __forceinline__ u32 wave_incl_scan_u32(u32 v) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        u32 tt = __shfl_up(v, o, 64);
        if (l >= o) v += tt;
    }
    return v;
}

// Exclusive scan of data[0..total) in place by one 1024-thread workgroup: each wave owns a
// contiguous chunk read 64 entries at a time (coalesced). on_entry(e, prefix) sees every entry.
template <typename F>
__device__ __forceinline__ u32 block1024_scan_inplace(u32* data, int total, u32* lw, F on_entry) {
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    int chunk = (total + 15) / 16;
    chunk = (chunk + 63) & ~63;
    const int c0 = w * chunk;
    const int c1 = min(total, c0 + chunk);
    u32 s = 0;
    for (int e = c0 + l; e < c1; e += 64) s += data[e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (l == 0) lw[w] = s;
    __syncthreads();
    u32 run = 0, tot = 0;
    for (int k = 0; k < 16; ++k) {
        if (k < w) run += lw[k];
        tot += lw[k];
    }
    for (int base = c0; base < c1; base += 64) {
        const int e = base + l;
        const u32 v = e < c1 ? data[e] : 0u;
        const u32 inc = wave_incl_scan_u32(v);
        if (e < c1) {
            data[e] = run + inc - v;
            on_entry(e, run + inc - v);
        }
        run += __shfl(inc, 63, 64);
    }
    return tot;
}

// exclusive scan over (ring, block) in ring-major order; ring_start[r] = first offset of ring r
__global__ void __launch_bounds__(1024) k_fe_ring_scan(u32* __restrict__ blkhist, int L, const int* __restrict__ d_n,
                                                        int* __restrict__ ring_start) {
    __shared__ u32 lw[16];
    const int n = *d_n;
    const int nblk = n > 0 ? (n + 255) / 256 : 1;
    const u32 tot = block1024_scan_inplace(blkhist, L * nblk, lw, [&](int e, u32 pre) {
        if (e % nblk == 0) ring_start[e / nblk] = (int)pre;
    });
    if (threadIdx.x == 0) ring_start[L] = (int)tot;
}

__global__ void __launch_bounds__(256) k_fe_scatter(const float4* __restrict__ in, const int* __restrict__ d_n,
                                                     const int* __restrict__ ring, const u32* __restrict__ blkoff,
                                                     float4* __restrict__ rp) {
    __shared__ u32 wc[4][kMaxRings];
    const int n = *d_n;
    const int nblk = n > 0 ? (n + 255) / 256 : 1;
    if ((int)blockIdx.x >= nblk) return;
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    for (int r = l; r < kMaxRings; r += 64) wc[w][r] = 0;
    __syncthreads();
    const int i = blockIdx.x * 256 + t;
    const int r = i < n ? ring[i] : -1;
    const bool valid = r >= 0;
    const u64 peers = match_bits((u32)(valid ? r : 0), 7, valid);
    const u32 rank = (u32)__popcll(peers & lanemask_lt());
    if (valid && rank == 0) wc[w][r] = (u32)__popcll(peers);
    __syncthreads();
    if (valid) {
        u32 pos = blkoff[r * nblk + blockIdx.x] + rank;
        for (int ww = 0; ww < w; ++ww) pos += wc[ww][r];
        rp[pos] = in[i];
    }
}

// 11-tap curvature of ring point j (:73-77): float sums, left to right, widened, squared in double
__device__ __forceinline__ double curvature_at(const float4* __restrict__ rr, int j) {
    const float4 a = rr[j - 5], b = rr[j - 4], c = rr[j - 3], d = rr[j - 2], e = rr[j - 1], f = rr[j];
    const float4 g = rr[j + 1], h = rr[j + 2], k = rr[j + 3], m = rr[j + 4], o = rr[j + 5];
    const float dx = a.x + b.x + c.x + d.x + e.x - 10 * f.x + g.x + h.x + k.x + m.x + o.x;
    const float dy = a.y + b.y + c.y + d.y + e.y - 10 * f.y + g.y + h.y + k.y + m.y + o.y;
    const float dz = a.z + b.z + c.z + d.z + e.z - 10 * f.z + g.z + h.z + k.z + m.z + o.z;
    const double X = dx, Y = dy, Z = dz;
    return X * X + Y * Y + Z * Z;
}

__device__ __forceinline__ bool kv_greater(double va, int ia, double vb, int ib) {
    return va > vb || (va == vb && ia > ib);
}

__global__ void __launch_bounds__(256) k_fe_sector(const float4* __restrict__ rp, const int* __restrict__ ring_start,
                                                    int* __restrict__ sec_edge_ids, int* __restrict__ sec_surf_ids,
                                                    int* __restrict__ sec_cnt, int* __restrict__ err) {
    __shared__ double sval[kSecCap];
    __shared__ int sid[kSecCap];
    __shared__ unsigned char picked[kSecCap + 16];
    __shared__ unsigned char gapbig[kSecCap + 16];
    __shared__ int sedge[kEdgePerSector + 1];
    __shared__ int snedge;
    __shared__ u32 lw[4];

    const int sec = blockIdx.x;
    const int r = sec / 6, s = sec % 6;
    const int t = threadIdx.x;
    const int base = ring_start[r];
    const int nr = ring_start[r + 1] - base;
    if (nr < 131) {                                            // :67
        if (t == 0) { sec_cnt[2 * sec] = 0; sec_cnt[2 * sec + 1] = 0; }
        return;
    }
    const int total = nr - 10;                                 // :68
    const int len = total / 6;                                 // :82
    const int cs = len * s;
    const int ce = (s == 5) ? total - 1 : len * (s + 1) - 1;   // half-open (:84-88)
    const int size = ce - cs;
    if (size > kSecCap) {
        if (t == 0) { sec_cnt[2 * sec] = 0; sec_cnt[2 * sec + 1] = 0; atomicOr(err, 1); }
        return;
    }
    const float4* rr = rp + base;
    int P = 64;
    while (P < size) P <<= 1;
    for (int k = t; k < P; k += 256) {
        if (k < size) {
            const int j = cs + k + 5;      // curvature list index -> ring position (:77)
            sval[k] = curvature_at(rr, j);
            sid[k] = j;
        } else {
            sval[k] = DBL_MAX;
            sid[k] = INT_MAX;
        }
    }
    // window of ring positions [cs, cs + size + 10): picked flags and gaps to the previous point
    const int ws = cs;
    for (int w = t; w < size + 10; w += 256) {
        picked[w] = 0;
        unsigned char g = 0;
        if (w >= 1) {
            const float4 a = rr[ws + w], b = rr[ws + w - 1];
            const double dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;  // float differences (:129-131)
            g = (dx * dx + dy * dy + dz * dz > 0.05) ? 1 : 0;
        }
        gapbig[w] = g;
    }
    __syncthreads();
    // bitonic sort ascending by (curvature, id)
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = t; i < P; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const double vi = sval[i], vj = sval[ixj];
                    const int ii = sid[i], ij = sid[ixj];
                    const bool asc = (i & k) == 0;
                    if (asc == kv_greater(vi, ii, vj, ij)) {
                        sval[i] = vj; sval[ixj] = vi;
                        sid[i] = ij; sid[ixj] = ii;
                    }
                }
            }
            __syncthreads();
        }
    }
    // greedy edge pick from the largest curvature (:110-148)
    if (t == 0) {
        int count = 0, ne = 0;
        for (int i = size - 1; i >= 0; --i) {
            const int ind = sid[i];
            const int w = ind - ws;
            if (picked[w]) continue;
            if (sval[i] <= 0.1) break;
            ++count;
            picked[w] = 1;
            if (count <= kEdgePerSector) sedge[ne++] = ind;
            else break;
            for (int k = 1; k <= 5; ++k) {
                if (gapbig[w + k]) break;
                picked[w + k] = 1;
            }
            for (int k = 1; k <= 5; ++k) {
                if (gapbig[w - k + 1]) break;
                picked[w - k] = 1;
            }
        }
        snedge = ne;
    }
    __syncthreads();
    const int ne = snedge;
    if (t < ne) sec_edge_ids[sec * kEdgePerSector + t] = sedge[t];
    // surf sweep in ascending order (:198-205), order-preserving compaction
    u32 run = 0;
    for (int b0 = 0; b0 < size; b0 += 256) {
        const int i = b0 + t;
        const bool keep = (i < size) && !picked[sid[i] - ws];
        u32 tot;
        const int wv = t >> 6, l = lane_id();
        const u64 bal = __ballot(keep);
        const u32 inw = (u32)__popcll(bal & lanemask_lt());
        if (l == 0) lw[wv] = (u32)__popcll(bal);
        __syncthreads();
        u32 off = 0;
        tot = 0;
        for (int q = 0; q < 4; ++q) {
            if (q < wv) off += lw[q];
            tot += lw[q];
        }
        if (keep) sec_surf_ids[(size_t)sec * kSecCap + run + off + inw] = sid[i];
        run += tot;
        __syncthreads();
    }
    if (t == 0) {
        sec_cnt[2 * sec] = ne;
        sec_cnt[2 * sec + 1] = (int)run;
    }
}

// output offsets in ring -> sector order (nsec <= 768 fits one pass of the 1024-thread scan)
__global__ void __launch_bounds__(1024) k_fe_out_scan(const int* __restrict__ sec_cnt, int nsec,
                                                       int* __restrict__ sec_off, int* __restrict__ d_ne,
                                                       int* __restrict__ d_ns) {
    __shared__ u32 lw[2][16];
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const u32 ve = t < nsec ? (u32)sec_cnt[2 * t] : 0u;
    const u32 vs = t < nsec ? (u32)sec_cnt[2 * t + 1] : 0u;
    const u32 ie = wave_incl_scan_u32(ve), is = wave_incl_scan_u32(vs);
    if (l == 63) { lw[0][w] = ie; lw[1][w] = is; }
    __syncthreads();
    u32 oe = 0, os = 0, te = 0, ts = 0;
    for (int k = 0; k < 16; ++k) {
        if (k < w) { oe += lw[0][k]; os += lw[1][k]; }
        te += lw[0][k];
        ts += lw[1][k];
    }
    if (t < nsec) {
        sec_off[2 * t] = (int)(oe + ie - ve);
        sec_off[2 * t + 1] = (int)(os + is - vs);
    }
    if (t == 0) { *d_ne = (int)te; *d_ns = (int)ts; }
}

__global__ void __launch_bounds__(256) k_fe_gather(const float4* __restrict__ rp, const int* __restrict__ ring_start,
                                                    const int* __restrict__ sec_edge_ids,
                                                    const int* __restrict__ sec_surf_ids, const int* __restrict__ sec_cnt,
                                                    const int* __restrict__ sec_off, float4* __restrict__ edge,
                                                    float4* __restrict__ surf) {
    const int sec = blockIdx.x;
    const int base = ring_start[sec / 6];
    const int ne = sec_cnt[2 * sec], ns = sec_cnt[2 * sec + 1];
    const int eo = sec_off[2 * sec], so = sec_off[2 * sec + 1];
    for (int k = threadIdx.x; k < ne; k += 256) edge[eo + k] = rp[base + sec_edge_ids[sec * kEdgePerSector + k]];
    for (int k = threadIdx.x; k < ns; k += 256) surf[so + k] = rp[base + sec_surf_ids[(size_t)sec * kSecCap + k]];
}

}  // namespace

int fe_alloc(FeGPU& f, const pf_lidar_params& lidar, size_t cap) {
    f.lidar = lidar;
    f.cap = cap;
    f.rings = lidar.num_lines;
    if (f.rings <= 0) return PF_EINVAL;
    if (f.rings > kMaxRings) return PF_EUNSUPPORTED;
    f.nblk_cap = (int)((cap + 255) / 256);
    const int nsec = f.rings * 6;
    if (hipMalloc(&f.ring, sizeof(int) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.blkhist, sizeof(u32) * (size_t)f.rings * f.nblk_cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.ring_start, sizeof(int) * (kMaxRings + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.rp, sizeof(float4) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.sec_edge_ids, sizeof(int) * nsec * kEdgePerSector) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.sec_surf_ids, sizeof(int) * (size_t)nsec * kSecCap) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.sec_cnt, sizeof(int) * nsec * 2) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.sec_off, sizeof(int) * nsec * 2) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.err, sizeof(int)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.d_in_stage, sizeof(float4) * cap) != hipSuccess) return PF_ENOMEM;
    if (hipMemset(f.err, 0, sizeof(int)) != hipSuccess) return PF_EHIP;
    return PF_OK;
}

int fe_set_ring_model(FeGPU& f, double top_deg, double bottom_deg) {
    if (top_deg == 0.0 && bottom_deg == 0.0) {
        f.ring_top = f.ring_scale = 0.0;
        return PF_OK;
    }
    if (!(top_deg > bottom_deg) || !(top_deg - bottom_deg <= 180.0)) return PF_EINVAL;
    f.ring_top = top_deg;
    f.ring_scale = (double)f.rings / (top_deg - bottom_deg);
    return PF_OK;
}

void fe_free(FeGPU& f) {
    (void)hipFree(f.ring);
    (void)hipFree(f.blkhist);
    (void)hipFree(f.ring_start);
    (void)hipFree(f.rp);
    (void)hipFree(f.sec_edge_ids);
    (void)hipFree(f.sec_surf_ids);
    (void)hipFree(f.sec_cnt);
    (void)hipFree(f.sec_off);
    (void)hipFree(f.err);
    (void)hipFree(f.d_in_stage);
    f = FeGPU{};
}

void fe_enqueue(FeGPU& f, const float4* d_in, const int* d_n, float4* edge, int* d_ne, float4* surf, int* d_ns,
                hipStream_t s) {
    const int L = f.rings;
    hipLaunchKernelGGL(k_fe_ring, dim3(f.nblk_cap), dim3(256), 0, s, d_in, d_n, L, f.lidar.min_dist, f.lidar.max_dist,
                       f.sqrt_double, f.ring_top, f.ring_scale, f.ring, f.blkhist);
    hipLaunchKernelGGL(k_fe_ring_scan, dim3(1), dim3(1024), 0, s, f.blkhist, L, d_n, f.ring_start);
    hipLaunchKernelGGL(k_fe_scatter, dim3(f.nblk_cap), dim3(256), 0, s, d_in, d_n, f.ring, f.blkhist, f.rp);
    hipLaunchKernelGGL(k_fe_sector, dim3(L * 6), dim3(256), 0, s, f.rp, f.ring_start, f.sec_edge_ids,
                       f.sec_surf_ids, f.sec_cnt, f.err);
    hipLaunchKernelGGL(k_fe_out_scan, dim3(1), dim3(1024), 0, s, f.sec_cnt, L * 6, f.sec_off, d_ne, d_ns);
    hipLaunchKernelGGL(k_fe_gather, dim3(L * 6), dim3(256), 0, s, f.rp, f.ring_start, f.sec_edge_ids,
                       f.sec_surf_ids, f.sec_cnt, f.sec_off, edge, surf);
}

}  // namespace pf
