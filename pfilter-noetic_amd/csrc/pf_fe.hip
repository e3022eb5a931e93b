// Feature extraction kernels (LaserProcessingClass::featureExtraction, src/laserProcessingClass.cpp:10-209).
//
//  k_fe_ring      ring id per point (range gate + elevation formula, :22-61) + per-block ring histogram
//  k_fe_ring_scan exclusive scan of the (ring, block) histogram -> stable ring partition offsets
//  k_fe_scatter   stable scatter into ring order (input order kept inside a ring, :62)
//  k_fe_sector    one workgroup per (ring, sector): 11-tap curvature (:73-77), LDS bitonic sort by
//                 (curvature, id) (tie order: std::sort's own order for a sector with equal curvatures), greedy edge pick with neighbour suppression (:110-148) and the
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

// Exclusive scan of data[0..total) in place by one 1024-thread workgroup, in LDS chunks of
// kScanChunk entries: a chunk is loaded with every load in flight (entry t + 1024 i on thread t),
// each thread sums its 16 contiguous LDS entries, the 1024 sums are scanned across the waves, and
// the prefixes are written back coalesced. on_entry(e, prefix) sees every entry.
constexpr int kScanChunk = 16384;
__device__ __forceinline__ int scan_pad(int e) { return e + (e >> 4); }   // +1 word per 16: no bank conflicts
template <typename F>
__device__ __forceinline__ u32 block1024_scan_inplace(u32* data, int total, u32* buf, u32* lw, F on_entry) {
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    constexpr int kPer = kScanChunk / 1024;
    u32 carry = 0;
    for (int c0 = 0; c0 < total; c0 += kScanChunk) {
        const int n = min(kScanChunk, total - c0);
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int e = t + 1024 * i;
            buf[scan_pad(e)] = e < n ? data[c0 + e] : 0u;
        }
        __syncthreads();
        u32 v[kPer], s = 0;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            v[i] = buf[scan_pad(kPer * t + i)];
            s += v[i];
        }
        const u32 inc = wave_incl_scan_u32(s);
        if (l == 63) lw[w] = inc;
        __syncthreads();
        u32 run = carry, tot = carry;
        for (int k = 0; k < 16; ++k) {
            if (k < w) run += lw[k];
            tot += lw[k];
        }
        run += inc - s;                                   // exclusive prefix of this thread's segment
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            buf[scan_pad(kPer * t + i)] = run;
            run += v[i];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int e = t + 1024 * i;
            if (e < n) {
                const u32 pre = buf[scan_pad(e)];
                data[c0 + e] = pre;
                on_entry(c0 + e, pre);
            }
        }
        carry = tot;
        __syncthreads();                                  // buf and lw are reused by the next chunk
    }
    return carry;
}

// exclusive scan over (ring, block) in ring-major order; ring_start[r] = first offset of ring r
__global__ void __launch_bounds__(1024) k_fe_ring_scan(u32* __restrict__ blkhist, int L, const int* __restrict__ d_n,
                                                        int* __restrict__ ring_start) {
    __shared__ u32 buf[kScanChunk + kScanChunk / 16];
    __shared__ u32 lw[16];
    const int n = *d_n;
    const int nblk = n > 0 ? (n + 255) / 256 : 1;
    const u32 tot = block1024_scan_inplace(blkhist, L * nblk, buf, lw, [&](int e, u32 pre) {
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

// libstdc++'s std::sort (GCC 9-11 bits/stl_algo.h: __introsort_loop with _S_threshold 16 and depth
// 2 __lg(n), __move_median_to_first(first, first + 1, mid, last - 1), __unguarded_partition, heap sort
// at the depth limit, final insertion sort) on the pairs (val, id) compared by val alone -- the
// reference's sector sort (:101-104). One thread; stk: 3 * 64 ints of LDS for the pending right parts.
template <class VP, class IP>
__device__ void pair_swap(VP* val, IP* id, int a, int b) {
    const double va = val[a];
    const int ia = id[a];
    val[a] = val[b];
    id[a] = id[b];
    val[b] = va;
    id[b] = ia;
}
template <class VP, class IP>
__device__ void pair_adjust_heap(VP* val, IP* id, int base, int hole, int len, double vv, int vi) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (val[base + child] < val[base + child - 1]) child--;
        val[base + hole] = val[base + child];
        id[base + hole] = id[base + child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        val[base + hole] = val[base + child - 1];
        id[base + hole] = id[base + child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && val[base + parent] < vv) {
        val[base + hole] = val[base + parent];
        id[base + hole] = id[base + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    val[base + hole] = vv;
    id[base + hole] = vi;
}
template <class VP, class IP>
__device__ void std_sort_pairs(VP* val, IP* id, int n, int* stk) {
    if (n < 2) return;
    int sp = 0;
    stk[0] = 0;
    stk[1] = n;
    stk[2] = 2 * (31 - __clz(n));
    sp = 1;
    while (sp > 0) {
        --sp;
        int first = stk[3 * sp], last = stk[3 * sp + 1], depth = stk[3 * sp + 2];
        while (last - first > 16) {
            if (depth == 0) {                                   // __partial_sort: make_heap + sort_heap
                const int len = last - first;
                for (int parent = (len - 2) / 2;; --parent) {
                    pair_adjust_heap(val, id, first, parent, len, (double)val[first + parent], (int)id[first + parent]);
                    if (parent == 0) break;
                }
                for (int e = len; e > 1;) {
                    --e;
                    const double vv = val[first + e];
                    const int vi = id[first + e];
                    val[first + e] = val[first];
                    id[first + e] = id[first];
                    pair_adjust_heap(val, id, first, 0, e, vv, vi);
                }
                break;
            }
            --depth;
            const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
            const double va = val[a], vb = val[b], vc = val[c];
            int sel;
            if (va < vb) sel = vb < vc ? b : (va < vc ? c : a);
            else sel = va < vc ? a : (vb < vc ? c : b);
            pair_swap(val, id, first, sel);
            const double pv = val[first];
            int lo = first + 1, hi = last;
            for (;;) {                                          // __unguarded_partition
                while (val[lo] < pv) ++lo;
                --hi;
                while (pv < val[hi]) --hi;
                if (!(lo < hi)) break;
                pair_swap(val, id, lo, hi);
                ++lo;
            }
            stk[3 * sp] = lo;                                   // __introsort_loop(cut, last, depth)
            stk[3 * sp + 1] = last;
            stk[3 * sp + 2] = depth;
            ++sp;
            last = lo;
        }
    }
    for (int i = 1; i < n; ++i) {                               // final insertion sort (stable)
        const double vv = val[i];
        const int vi = id[i];
        int j = i;
        while (j > 0 && vv < val[j - 1]) {
            val[j] = val[j - 1];
            id[j] = id[j - 1];
            --j;
        }
        val[j] = vv;
        id[j] = vi;
    }
}

__device__ __forceinline__ bool kv_greater(double va, int ia, double vb, int ib) {
    return va > vb || (va == vb && ia > ib);
}

// One sector's selection (:99-209) on arrays that live in LDS (sectors up to kSecLds entries) or in
// global scratch (larger sectors: any size, as the reference). sval / sid: P >= size slots,
// picked / gapbig: the window of ring positions [cs, cs + size + 10). 256 threads.
template <bool kGlobal>
__device__ __forceinline__ void sector_select(const float4* __restrict__ rr, int cs, int size, int base, int sec,
                                              double* sval, int* sid, unsigned char* picked,
                                              unsigned char* gapbig, int* sedge, int* lw_int, int* ivl_lo, int* ivl_hi,
                                              int* __restrict__ sec_edge_ids, int* __restrict__ surf_ids,
                                              int* __restrict__ sec_cnt, int tie, int* stk) {
    const int t = threadIdx.x;
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
    for (int w = t; w < size + 10; w += 256) {
        picked[w] = 0;
        unsigned char g = 0;
        if (w >= 1) {
            const float4 a = rr[cs + w], b = rr[cs + w - 1];
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
    if (tie) {
        // reference tie order: libstdc++'s std::sort orders equal curvatures its own way (:101-104), so
        // a sector holding an exact tie is sorted again, from the unsorted list, by introsort itself
        // (one thread); without a tie both orders are the same
        bool has = false;
        for (int i = t; i + 1 < size; i += 256) has = has || sval[i] == sval[i + 1];
        if (__syncthreads_or(has)) {
            for (int k = t; k < size; k += 256) {
                sval[k] = curvature_at(rr, cs + k + 5);
                sid[k] = cs + k + 5;
            }
            __syncthreads();
            if (t == 0) std_sort_pairs(sval, sid, size, stk);
            __syncthreads();
        }
    }
    // Greedy edge pick from the largest curvature (:110-148), wave 0. The reference walks the sorted
    // list downwards: a picked point is skipped, the first unpicked point at curvature <= 0.1 ends
    // the walk, otherwise the point is picked (the 21st pick only marks itself and ends the walk)
    // and up to 5 neighbours on each side, up to the first big gap, are marked picked. Here 64
    // candidates at a time sit on the lanes (lane 0 = largest); a pick is the lowest lane that is
    // neither marked nor below the threshold, and every lane tests its own position against the
    // pick's marked interval [w - left, w + right] (and against every earlier pick's interval when a
    // new batch is loaded), so each pick costs a ballot and a broadcast instead of a walk.
    if (t < 64) {
        const int l = t;
        int count = 0, ne = 0;
        bool stop = false;
        for (int b0 = 0; b0 < size && !stop; b0 += 64) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the intervals stored by lane 0
            const int i = size - 1 - (b0 + l);
            bool live = i >= 0;
            int w = 0, lft = 0, rgt = 0, ind = 0;
            double v = 0.0;
            if (live) {
                v = sval[i];
                ind = sid[i];
                w = ind - cs;
                for (int k = 1; k <= 5 && !gapbig[w + k]; ++k) rgt = k;
                for (int k = 1; k <= 5 && !gapbig[w - k + 1]; ++k) lft = k;
                for (int p = 0; p < count; ++p) live = live && !(w >= ivl_lo[p] && w <= ivl_hi[p]);
            }
            for (;;) {
                const u64 m = __ballot(live);
                if (!m) break;
                const int pl = __ffsll((unsigned long long)m) - 1;
                const double pv = __shfl(v, pl, 64);
                if (pv <= 0.1) { stop = true; break; }                    // unpicked, below the threshold
                const int pw = __shfl(w, pl, 64), pind = __shfl(ind, pl, 64);
                ++count;
                int lo = pw, hi = pw;
                if (count <= kEdgePerSector) {
                    lo = pw - __shfl(lft, pl, 64);
                    hi = pw + __shfl(rgt, pl, 64);
                    if (l == 0) sedge[ne] = pind;
                    ++ne;
                }
                if (l == 0) {
                    ivl_lo[count - 1] = lo;
                    ivl_hi[count - 1] = hi;
                }
                live = live && !(w >= lo && w <= hi);
                if (count > kEdgePerSector) { stop = true; break; }
            }
        }
        // the marked positions, for the surf sweep
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int p = 0; p < count; ++p)
            if (l <= ivl_hi[p] - ivl_lo[p]) picked[ivl_lo[p] + l] = 1;
        if (l == 0) lw_int[4] = ne;
    }
    __syncthreads();
    const int ne = lw_int[4];
    if (t < ne) sec_edge_ids[sec * kEdgePerSector + t] = sedge[t];
    // surf sweep in ascending order (:198-205), order-preserving compaction
    u32 run = 0;
    for (int b0 = 0; b0 < size; b0 += 256) {
        const int i = b0 + t;
        const bool keep = (i < size) && !picked[sid[i] - cs];
        const int wv = t >> 6, l = lane_id();
        const u64 bal = __ballot(keep);
        const u32 inw = (u32)__popcll(bal & lanemask_lt());
        if (l == 0) lw_int[wv] = (int)__popcll(bal);
        __syncthreads();
        u32 off = 0, tot = 0;
        for (int q = 0; q < 4; ++q) {
            if (q < wv) off += (u32)lw_int[q];
            tot += (u32)lw_int[q];
        }
        if (keep) surf_ids[base + cs + run + off + inw] = sid[i];
        run += tot;
        __syncthreads();
    }
    if (t == 0) {
        sec_cnt[2 * sec] = ne;
        sec_cnt[2 * sec + 1] = (int)run;
    }
}

__global__ void __launch_bounds__(256) k_fe_sector(const float4* __restrict__ rp, const int* __restrict__ ring_start,
                                                    int* __restrict__ sec_edge_ids, int* __restrict__ surf_ids,
                                                    int* __restrict__ sec_cnt, double* __restrict__ g_val,
                                                    int* __restrict__ g_id, unsigned char* __restrict__ g_picked,
                                                    unsigned char* __restrict__ g_gap, int tie) {
    __shared__ double sval[kSecLds];
    __shared__ int stk[3 * 64];
    __shared__ int sid[kSecLds];
    __shared__ unsigned char picked[kSecLds + 16];
    __shared__ unsigned char gapbig[kSecLds + 16];
    __shared__ int sedge[kEdgePerSector + 1];
    __shared__ int lw_int[8];
    __shared__ int ivl_lo[kEdgePerSector + 1], ivl_hi[kEdgePerSector + 1];

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
    const float4* rr = rp + base;
    if (size <= kSecLds) {
        sector_select<false>(rr, cs, size, base, sec, sval, sid, picked, gapbig, sedge, lw_int, ivl_lo, ivl_hi,
                             sec_edge_ids, surf_ids, sec_cnt, tie, stk);
    } else {
        // a sector larger than LDS (e.g. every point in ring 0 for a line count without a ring
        // formula, :58-61): the same selection on global scratch; slots 2 (base + cs) .. of the
        // scratch arrays are this sector's own (P <= 2 size, windows of size + 10 <= 2 size bytes)
        const size_t o = 2 * (size_t)(base + cs);
        sector_select<true>(rr, cs, size, base, sec, g_val + o, g_id + o, g_picked + o, g_gap + o, sedge, lw_int, ivl_lo,
                            ivl_hi, sec_edge_ids, surf_ids, sec_cnt, tie, stk);
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
                                                    const int* __restrict__ surf_ids, const int* __restrict__ sec_cnt,
                                                    const int* __restrict__ sec_off, float4* __restrict__ edge,
                                                    float4* __restrict__ surf) {
    const int sec = blockIdx.x;
    const int r = sec / 6, s = sec % 6;
    const int base = ring_start[r];
    const int ne = sec_cnt[2 * sec], ns = sec_cnt[2 * sec + 1];
    const int eo = sec_off[2 * sec], so = sec_off[2 * sec + 1];
    const int cs = ((ring_start[r + 1] - base - 10) / 6) * s;    // the sector's surf ids start at base + cs
    for (int k = threadIdx.x; k < ne; k += 256) edge[eo + k] = rp[base + sec_edge_ids[sec * kEdgePerSector + k]];
    for (int k = threadIdx.x; k < ns; k += 256) surf[so + k] = rp[base + surf_ids[base + cs + k]];
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
    if (hipMalloc(&f.sec_surf_ids, sizeof(int) * cap) != hipSuccess) return PF_ENOMEM;
    // scratch of sectors larger than LDS: 2 slots per ring point (a sector's P <= 2 size)
    if (hipMalloc(&f.big_val, sizeof(double) * 2 * cap + 64) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.big_id, sizeof(int) * 2 * cap + 64) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.big_picked, 2 * cap + 64) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&f.big_gap, 2 * cap + 64) != hipSuccess) return PF_ENOMEM;
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
    (void)hipFree(f.big_val);
    (void)hipFree(f.big_id);
    (void)hipFree(f.big_picked);
    (void)hipFree(f.big_gap);
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
                       f.sec_surf_ids, f.sec_cnt, f.big_val, f.big_id, f.big_picked, f.big_gap, f.tie_order);
    hipLaunchKernelGGL(k_fe_out_scan, dim3(1), dim3(1024), 0, s, f.sec_cnt, L * 6, f.sec_off, d_ne, d_ns);
    hipLaunchKernelGGL(k_fe_gather, dim3(L * 6), dim3(256), 0, s, f.rp, f.ring_start, f.sec_edge_ids,
                       f.sec_surf_ids, f.sec_cnt, f.sec_off, edge, surf);
}

}  // namespace pf
