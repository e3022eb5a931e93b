// Reference tie order: libstdc++ introsort's permutation of equal keys, breadth-first (pf_tie.h).
#include <climits>

#include "pf_tie.h"

namespace pf {
namespace {

constexpr u32 kTieDrop = 0xFFFFFFFFu;
constexpr int kThreshold = 16;           // libstdc++ _S_threshold
constexpr int kMaxTieC = 4;              // classes of one sort (key bits 30-31)
constexpr int kTieGrid = 256;            // workgroups of the tile launches (co-resident, look-back)
constexpr int kTieSegLds = kTieLocal / (kThreshold + 1) + 4;   // segments of one LDS recursion level
constexpr int kTieStack = 128;           // pending big segments of the fallback
typedef unsigned short u16;

// control words (TieSort::ctl)
enum {
    T_VALID = 0,        // valid pairs (compacted)
    T_NJOBS = 1,        // local jobs
    T_CS = 2,           // [kMaxTieC] compacted start of every class
    T_BIG = 8,          // u64 [2]: big segments << 32 | their tiles, per level parity
    T_WORDS = 16
};
__device__ __forceinline__ u64* big_ctr(int* ctl, int p) { return reinterpret_cast<u64*>(ctl + T_BIG) + p; }

__device__ __forceinline__ int lg_floor(int n) { return 31 - __clz(n); }

// the class boundaries of the input: start[c], start[nc] = n
__device__ __forceinline__ int class_starts(const TieClasses& cls, int (&start)[kMaxTieC + 1]) {
    int acc = 0;
#pragma unroll
    for (int c = 0; c < kMaxTieC; ++c) {
        start[c] = acc;
        if (c < cls.nc) acc += cls.cnt[cls.ia + c] + (cls.ib >= 0 ? cls.cnt[cls.ib + c] : 0);
    }
    start[kMaxTieC] = acc;
    return acc;
}

// std::__move_median_to_first(first, first + 1, mid, last - 1): the position moved to first
__device__ __forceinline__ int median3(u32 ka, u32 kb, u32 kc, int a, int b, int c) {
    if (ka < kb) return kb < kc ? b : (ka < kc ? c : a);
    return ka < kc ? a : (kb < kc ? c : b);
}

__device__ __forceinline__ int tiles_of(int len) { return (len + kTieTile - 1) / kTieTile; }

// ------------------------------------------------------------------------------------------------
// compaction: the valid pairs of the input, class-major (the classes are contiguous in the input), one
// pass of 4096-pair tiles (16 rows of 256) with a decoupled look-back; the tile holding a class's first
// input element records where the class starts among the valid pairs
__global__ void __launch_bounds__(256) k_tie_compact(const u32* __restrict__ keys, const u32* __restrict__ vals,
                                                     TieClasses cls, u32* __restrict__ k, u32* __restrict__ v,
                                                     int* __restrict__ ctl, u64* __restrict__ status,
                                                     u32* __restrict__ arrive, int* __restrict__ err) {
    __shared__ u32 s_cnt[64];
    __shared__ u32 s_off[64];
    int start[kMaxTieC + 1];
    const int n = class_starts(cls, start);
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const u64 lt = lanemask_lt();
    const int ntiles = (n + kTieTile - 1) / kTieTile;
    if (n == 0) {
        if (blockIdx.x == 0 && t == 0) {
            ctl[T_VALID] = 0;
            for (int c = 0; c < kMaxTieC; ++c) ctl[T_CS + c] = 0;
        }
        return;
    }
    const int G = ntiles < (int)gridDim.x ? ntiles : (int)gridDim.x;
    if ((int)blockIdx.x >= G) return;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int base = tile * kTieTile;
        u32 kk[16], vv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = base + j * 256 + t;
            kk[j] = i < n ? keys[i] : kTieDrop;
            vv[j] = i < n ? vals[i] : 0u;
        }
        u64 m[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            m[j] = __ballot(kk[j] != kTieDrop);
            if (l == 0) s_cnt[j * 4 + w] = (u32)__popcll(m[j]);
        }
        __syncthreads();
        if (w == 0) {
            const u32 c = s_cnt[l];
            const u32 inc = wave_incl_scan_u32(c);
            const u32 agg = (u32)__shfl((int)inc, 63, 64);
            const u32 pre = tile_lookback(status, tile, agg, err);
            s_off[l] = pre + inc - c;
            if (tile == ntiles - 1 && l == 0) {
                ctl[T_VALID] = (int)(pre + agg);
                for (int c2 = 0; c2 < kMaxTieC; ++c2)
                    if (start[c2] >= n) ctl[T_CS + c2] = (int)(pre + agg);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = base + j * 256 + t;
            const u32 pos = s_off[j * 4 + w] + (u32)__popcll(m[j] & lt);
            if (kk[j] != kTieDrop) {
                k[pos] = kk[j];
                v[pos] = vv[j];
            }
#pragma unroll
            for (int c = 0; c < kMaxTieC; ++c)
                if (i == start[c] && i < n) ctl[T_CS + c] = (int)pos;
        }
        __syncthreads();
    }
    lookback_finish(status, ntiles, arrive, G);
}

// level 0: every class is one std::sort call; above kTieLocal keys it starts in the big levels
__global__ void k_tie_setup(TieClasses cls, int* __restrict__ ctl, int4* __restrict__ big, int4* __restrict__ jobs,
                            int levels, int depth0) {
    if (threadIdx.x != 0) return;
    const int nv = ctl[T_VALID];
    int cs[kMaxTieC + 1];
    for (int c = 0; c < kMaxTieC; ++c) cs[c] = c < cls.nc ? ctl[T_CS + c] : nv;
    cs[kMaxTieC] = nv;
    u64 ctr = 0;
    int nj = 0;
    for (int c = 0; c < kMaxTieC; ++c) {
        const int f = cs[c], e = cs[c + 1], len = e - f;
        if (len < 1) continue;
        const int depth = depth0 >= 0 ? depth0 : 2 * lg_floor(len);   // std::__lg(last - first) * 2
        if (levels > 0 && len > kTieLocal && depth > 0) {
            big[(int)(ctr >> 32)] = make_int4(f, e, depth, (int)(u32)ctr);
            ctr += (1ull << 32) | (u64)tiles_of(len);
        } else {
            jobs[nj++] = make_int4(f, e, depth, 0);
        }
    }
    *big_ctr(ctl, 0) = ctr;
    *big_ctr(ctl, 1) = 0;
    ctl[T_NJOBS] = nj;
}

// ------------------------------------------------------------------------------------------------
// big levels. Status word of a tile: tag << 62 | (left stops << 31 | right stops); the look-back of a
// tile stops at the first tile of its segment.
constexpr u64 kValMask = (1ull << 62) - 1;
__device__ __forceinline__ u64 seg_lookback(u64* status, int tile, int tfirst, u64 agg, int* err) {
    const int l = lane_id();
    if (l == 0 && tile > tfirst)
        __hip_atomic_store(&status[tile], (1ull << 62) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u64 excl = 0;
    int j = tile - 1;
    unsigned long long t0 = 0;
    while (j >= tfirst) {
        const int jj = j - l;
        const u64 sv = jj >= tfirst ? __hip_atomic_load(&status[jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : (2ull << 62);     // before the segment: an inclusive zero
        const u32 tag = (u32)(sv >> 62);
        const u64 incl = __ballot(tag == 2);
        const int first = incl ? __ffsll((long long)incl) - 1 : 64;
        const u64 upto = first >= 63 ? ~0ull : ((2ull << first) - 1);
        if (__ballot(tag == 0) & upto) {
            const unsigned long long now = rt_now();
            if (!t0) t0 = now;
            else if (now - t0 > kWaitTicks) { if (l == 0) atomicOr(err, 2); break; }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        u64 mine = (l <= first && jj >= tfirst) ? (sv & kValMask) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
        excl += mine;
        if (first < 64) break;
        j -= 64;
    }
    if (l == 0)
        __hip_atomic_store(&status[tile], (2ull << 62) | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}
__device__ __forceinline__ u64 pack2(u32 packed16) {              // (L << 16 | R) -> (L << 31 | R)
    return ((u64)(packed16 >> 16) << 31) | (u64)(packed16 & 0xffffu);
}

constexpr int kTieBigLds = 512;          // big segments of one level cached in LDS (bcap <= this)

// every tile of every big segment of level parity p: the stops of its 4096 keys ranked in position
// order. The median of three is applied virtually here (first holds the pivot, sel the old first key)
// and physically by k_tie_split, so no key moves during this launch.
__global__ void __launch_bounds__(256) k_tie_scan(const u32* __restrict__ k, const int4* __restrict__ big,
                                                  int* __restrict__ ctl, int p, u32* __restrict__ lp,
                                                  u32* __restrict__ rq, u64* __restrict__ tot,
                                                  u64* __restrict__ status, u32* __restrict__ arrive,
                                                  int* __restrict__ err) {
    __shared__ int4 s_big[kTieBigLds];
    __shared__ u32 s_cnt[64];
    __shared__ u64 s_off[64];
    const u64 cw = *big_ctr(ctl, p);
    const int nb = (int)(cw >> 32), ntiles = (int)(u32)cw;
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const u64 lt = lanemask_lt();
    if (blockIdx.x == 0 && t == 0) *big_ctr(ctl, p ^ 1) = 0;   // the next level's list (unread here)
    if (ntiles == 0) return;
    const int G = ntiles < (int)gridDim.x ? ntiles : (int)gridDim.x;
    if ((int)blockIdx.x >= G) return;
    for (int i = t; i < nb; i += 256) s_big[i] = big[i];
    __syncthreads();
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        int lo = 0, hi = nb - 1;                                 // last segment whose tile base <= tile
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_big[mid].w <= tile) lo = mid;
            else hi = mid - 1;
        }
        const int s = lo;
        const int first = s_big[s].x, last = s_big[s].y, tb = s_big[s].w;
        const int base = first + (tile - tb) * kTieTile;
        const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
        const u32 ka = k[a], kb = k[b], kc = k[c], kf = k[first];
        const int sel = median3(ka, kb, kc, a, b, c);
        const u32 pv = sel == a ? ka : (sel == b ? kb : kc);
        u32 fl = 0, fr = 0;                                      // this thread's stop flags, bit j = row j
        u64 mL[16], mR[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = base + j * 256 + t;
            const bool in = i < last;
            u32 key = in ? k[i] : 0u;
            key = i == first ? pv : (i == sel ? kf : key);
            const bool bl = in && i > first && !(key < pv);
            const bool br = in && !(pv < key);
            fl |= (u32)bl << j;
            fr |= (u32)br << j;
            mL[j] = __ballot(bl);
            mR[j] = __ballot(br);
            if (l == 0) s_cnt[j * 4 + w] = ((u32)__popcll(mL[j]) << 16) | (u32)__popcll(mR[j]);
        }
        __syncthreads();
        if (w == 0) {
            const u32 cc = s_cnt[l];
            const u32 inc = wave_incl_scan_u32(cc);
            const u32 agg = (u32)__shfl((int)inc, 63, 64);
            const u64 pre = seg_lookback(status, tile, tb, pack2(agg), err);
            s_off[l] = pre + pack2(inc - cc);
            if (l == 0 && tile == tb + tiles_of(last - first) - 1) {
                const u64 in = pre + pack2(agg);
                tot[s] = ((in >> 31) << 32) | (in & 0x7fffffffull);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = base + j * 256 + t;
            const u64 o = s_off[j * 4 + w];
            if ((fl >> j) & 1u) lp[first + (int)(o >> 31) + __popcll(mL[j] & lt)] = (u32)i;
            if ((fr >> j) & 1u) rq[first + (int)(o & 0x7fffffffull) + __popcll(mR[j] & lt)] = (u32)i;
        }
        __syncthreads();
    }
    lookback_finish(status, ntiles, arrive, G);
}

// m = the largest k <= min(nL, nR) with lp[first + k - 1] < rq[first + nR - k] (the predicate is
// monotone), searched by the whole workgroup (NT candidates per round)
template <int NT>
__device__ __forceinline__ int wg_msearch(const u32* lp, const u32* rq, int first, int nL, int nR) {
    int lo = 0, hi = nL < nR ? nL : nR;
    while (lo < hi) {
        const int step = (hi - lo + NT - 1) / NT;
        int kk = lo + ((int)threadIdx.x + 1) * step;
        kk = kk < hi ? kk : hi;
        const bool ok = lp[first + kk - 1] < rq[first + nR - kk];
        const int c = __syncthreads_count(ok);
        if (c == 0) {
            hi = lo + step - 1;
        } else {
            const int nlo = lo + c * step < hi ? lo + c * step : hi;
            const int nhi = c < NT ? (lo + (c + 1) * step < hi ? lo + (c + 1) * step : hi) - 1 : hi;
            lo = nlo;
            hi = nhi > lo ? nhi : lo;
        }
    }
    return lo;
}

// the cut of a partition with m swaps: min(L_(m+1), R_(nR+1-m)), L_1 for m = 0
template <class PA>
__device__ __forceinline__ int cut_of(const PA* lp, const PA* rq, int first, int nL, int nR, int m) {
    if (m == 0) return (int)lp[first];
    const int r = (int)rq[first + nR - m];
    const int lf = m < nL ? (int)lp[first + m] : INT_MAX;
    return lf < r ? lf : r;
}

__device__ __forceinline__ void file_child(int* ctl, int pn, int4* next, int4* jobs, int f, int e, int d,
                                           bool may_big) {
    const int len = e - f;
    if (len < 1) return;
    if (may_big && len > kTieLocal && d > 0) {
        const u64 r = atomicAdd((unsigned long long*)big_ctr(ctl, pn), (1ull << 32) | (u64)tiles_of(len));
        next[(int)(r >> 32)] = make_int4(f, e, d, (int)(u32)r);
    } else {
        jobs[atomicAdd(&ctl[T_NJOBS], 1)] = make_int4(f, e, d, 0);
    }
}

// one workgroup per big segment of level parity p: the median swap, m, the cut, the m swaps, and the
// two children filed as big segments of the next level or as local jobs
__global__ void __launch_bounds__(1024) k_tie_split(u32* __restrict__ k, u32* __restrict__ v,
                                                    const u32* __restrict__ lp, const u32* __restrict__ rq,
                                                    const int4* __restrict__ big, const u64* __restrict__ tot,
                                                    int* __restrict__ ctl, int p, int last_level,
                                                    int4* __restrict__ next, int4* __restrict__ jobs) {
    __shared__ int s_cut;
    const int nb = (int)(*big_ctr(ctl, p) >> 32);
    const int t = threadIdx.x;
    for (int s = blockIdx.x; s < nb; s += gridDim.x) {
        const int4 sg = big[s];
        const int first = sg.x, last = sg.y, depth = sg.z;
        if (t == 0) {
            const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
            const int sel = median3(k[a], k[b], k[c], a, b, c);
            const u32 kf = k[first], ks = k[sel], vf = v[first], vs = v[sel];
            k[first] = ks;
            k[sel] = kf;
            v[first] = vs;
            v[sel] = vf;
        }
        const u64 tt = tot[s];
        const int nL = (int)(tt >> 32), nR = (int)(u32)tt;
        const int m = wg_msearch<1024>(lp, rq, first, nL, nR);
        if (t == 0) s_cut = cut_of(lp, rq, first, nL, nR, m);
        __threadfence_block();
        __syncthreads();
        for (int q = t; q < m; q += 1024) {
            const int pl = (int)lp[first + q], pr = (int)rq[first + nR - 1 - q];
            const u32 kl = k[pl], kr = k[pr], vl = v[pl], vr = v[pr];
            k[pl] = kr;
            k[pr] = kl;
            v[pl] = vr;
            v[pr] = vl;
        }
        if (t == 0) {
            const int cut = s_cut;
            file_child(ctl, p ^ 1, next, jobs, first, cut, depth - 1, !last_level);
            file_child(ctl, p ^ 1, next, jobs, cut, last, depth - 1, !last_level);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// local sort: one workgroup of 1024 threads per job

// libstdc++ __adjust_heap + __push_heap on [base, base + len)
template <class KA, class VA>
__device__ void adjust_heap(KA* k, VA* v, int base, int hole, int len, u32 vk, VA vv) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (k[base + child] < k[base + child - 1]) child--;
        k[base + hole] = k[base + child];
        v[base + hole] = v[base + child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        k[base + hole] = k[base + child - 1];
        v[base + hole] = v[base + child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && k[base + parent] < vk) {
        k[base + hole] = k[base + parent];
        v[base + hole] = v[base + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    k[base + hole] = vk;
    v[base + hole] = vv;
}
// libstdc++'s __partial_sort(first, last, last) = __make_heap + __sort_heap (one thread)
template <class KA, class VA>
__device__ void heap_sort(KA* k, VA* v, int base, int len) {
    if (len >= 2)
        for (int parent = (len - 2) / 2;; --parent) {
            adjust_heap(k, v, base, parent, len, (u32)k[base + parent], v[base + parent]);
            if (parent == 0) break;
        }
    for (int last = len; last > 1;) {
        --last;
        const u32 vk = k[base + last];
        const VA vv = v[base + last];
        k[base + last] = k[base];
        v[base + last] = v[base];
        adjust_heap(k, v, base, 0, last, vk, vv);
    }
}

// stable sort of up to two leaves of <= 16 keys by one wavefront: lanes 16 g .. 16 g + 15 rank leaf g
// (final insertion sort: no key leaves its leaf, and insertion sort is stable)
template <class VA>
__device__ __forceinline__ void leaf_sort2(u32* K, VA* V, int f0, int e0, int f1, int e1) {
    const int l = lane_id(), g = l >> 4, j = l & 15;
    const int f = g == 0 ? f0 : f1, len = g == 0 ? e0 - f0 : (g == 1 ? e1 - f1 : 0);
    const bool leaf = g < 2 && len >= 2 && len <= kThreshold;
    const bool mine = leaf && j < len;
    const u32 key = mine ? K[f + j] : kTieDrop;
    const VA val = mine ? V[f + j] : (VA)0;
    int r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const u32 ki = (u32)__shfl((int)key, (l & ~15) + i, 64);
        r += (i < len) && (ki < key || (ki == key && i < j));
    }
    if (mine) {
        K[f + r] = key;
        V[f + r] = val;
    }
}

// one Hoare partition of [first, last) by one wavefront (median of three first); LP / RQ receive the
// stop positions at first + rank. Returns the cut.
template <class VA, class PA>
__device__ int wave_partition(u32* K, VA* V, PA* LP, PA* RQ, int first, int last) {
    const int l = lane_id();
    const u64 lt = lanemask_lt();
    const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
    const u32 ka = K[a], kb = K[b], kc = K[c];
    const int sel = median3(ka, kb, kc, a, b, c);
    const u32 pv = sel == a ? ka : (sel == b ? kb : kc);
    if (l == 0) {
        const u32 kf = K[first];
        const VA vf = V[first], vs = V[sel];
        K[first] = pv;
        K[sel] = kf;
        V[first] = vs;
        V[sel] = vf;
    }
    __builtin_amdgcn_wave_barrier();
    int nL = 0, nR = 0;
    for (int base = first; base < last; base += 256) {
        u32 kk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = base + 64 * u + l;
            kk[u] = i < last ? K[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = base + 64 * u + l;
            const bool in = i < last;
            const bool fl = in && i > first && !(kk[u] < pv);
            const bool fr = in && !(pv < kk[u]);
            const u64 bl = __ballot(fl), br = __ballot(fr);
            if (fl) LP[first + nL + __popcll(bl & lt)] = (PA)i;
            if (fr) RQ[first + nR + __popcll(br & lt)] = (PA)i;
            nL += __popcll(bl);
            nR += __popcll(br);
        }
    }
    __builtin_amdgcn_wave_barrier();
    int lo = 0, hi = nL < nR ? nL : nR;                  // m: 64 candidates per round
    while (lo < hi) {
        const int step = (hi - lo + 63) / 64;
        int kq = lo + (l + 1) * step;
        kq = kq < hi ? kq : hi;
        const bool ok = (int)LP[first + kq - 1] < (int)RQ[first + nR - kq];
        const int cnt = __popcll(__ballot(ok));
        if (cnt == 0) {
            hi = lo + step - 1;
        } else {
            const int nlo = lo + cnt * step < hi ? lo + cnt * step : hi;
            const int nhi = cnt < 64 ? (lo + (cnt + 1) * step < hi ? lo + (cnt + 1) * step : hi) - 1 : hi;
            lo = nlo;
            hi = nhi > lo ? nhi : lo;
        }
    }
    const int m = lo;
    const int cut = cut_of(LP, RQ, first, nL, nR, m);
    for (int q = l; q < m; q += 64) {
        const int pl = (int)LP[first + q], pr = (int)RQ[first + nR - 1 - q];
        const u32 kl = K[pl], kr = K[pr];
        const VA vl = V[pl], vr = V[pr];
        K[pl] = kr;
        K[pr] = kl;
        V[pl] = vr;
        V[pr] = vl;
    }
    __builtin_amdgcn_wave_barrier();
    return cut;
}

struct LocalLds {
    u32 K[kTieLocal];
    u16 I[kTieLocal], LP[kTieLocal], RQ[kTieLocal];
    u64 seg[2][kTieSegLds];        // first | last << 16 | depth << 32
    int nseg[2];
    int4 stk[kTieStack];           // fallback: pending big segments
    int nstk;
    int4 top;
    u32 cnt[64];                   // fallback: per-row-wave stop counts, then their prefixes
    u32 tot;
    int cut;
};

__device__ __forceinline__ u64 seg_pack(int f, int e, int d) {
    return (u64)(u32)f | ((u64)(u32)e << 16) | ((u64)(u32)d << 32);
}

// [f, f + len) of the compacted pairs, len <= kTieLocal: the whole subtree in LDS, then the sorted
// keys and the vals they carry to the output
__device__ void lds_sort(LocalLds& S, const u32* __restrict__ k, const u32* __restrict__ v, u32* __restrict__ keys,
                         u32* __restrict__ vals, int f, int len, int depth) {
    const int t = threadIdx.x, wv = t >> 6, l = lane_id();
    for (int i = t; i < len; i += 1024) {
        S.K[i] = k[f + i];
        S.I[i] = (u16)i;
    }
    if (t == 0) {
        S.nseg[0] = len > kThreshold ? 1 : 0;
        S.nseg[1] = 0;
        S.seg[0][0] = seg_pack(0, len, depth);
    }
    __syncthreads();
    if (len <= kThreshold) {
        if (wv == 0) leaf_sort2(S.K, S.I, 0, len, 0, 0);
    } else {
        int cur = 0;
        for (;;) {
            const int ns = S.nseg[cur];
            if (ns == 0) break;
            for (int s = wv; s < ns; s += 16) {
                const u64 e = S.seg[cur][s];
                const int first = (int)(e & 0xffff), last = (int)((e >> 16) & 0xffff), d = (int)(e >> 32);
                if (d == 0) {                                    // depth limit: __partial_sort
                    if (l == 0) heap_sort(S.K, S.I, first, last - first);
                    __builtin_amdgcn_wave_barrier();
                    continue;
                }
                const int cut = wave_partition(S.K, S.I, S.LP, S.RQ, first, last);
                if (l == 0) {
                    if (cut - first > kThreshold) S.seg[cur ^ 1][atomicAdd(&S.nseg[cur ^ 1], 1)] = seg_pack(first, cut, d - 1);
                    if (last - cut > kThreshold) S.seg[cur ^ 1][atomicAdd(&S.nseg[cur ^ 1], 1)] = seg_pack(cut, last, d - 1);
                }
                leaf_sort2(S.K, S.I, first, cut, cut, last);
                __builtin_amdgcn_wave_barrier();
            }
            __syncthreads();
            if (t == 0) S.nseg[cur] = 0;
            cur ^= 1;
            __syncthreads();
        }
    }
    __syncthreads();
    for (int i = t; i < len; i += 1024) {
        keys[f + i] = S.K[i];
        vals[f + i] = v[f + S.I[i]];
    }
    __syncthreads();
}

// fallback for a segment above kTieLocal left by the big levels: one Hoare partition of [first, last)
// by the whole workgroup in global memory (4 rows of 1024 keys per round); returns the cut
__device__ int wg_partition(LocalLds& S, u32* k, u32* v, u32* lp, u32* rq, int first, int last) {
    const int t = threadIdx.x, wv = t >> 6, l = lane_id();
    const u64 lt = lanemask_lt();
    if (t == 0) {
        const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
        const int sel = median3(k[a], k[b], k[c], a, b, c);
        const u32 kf = k[first], ks = k[sel], vf = v[first], vs = v[sel];
        k[first] = ks;
        k[sel] = kf;
        v[first] = vs;
        v[sel] = vf;
        S.tot = ks;
    }
    __threadfence_block();
    __syncthreads();
    const u32 pv = S.tot;
    int nL = 0, nR = 0;
    for (int base = first; base < last; base += 4096) {
        __syncthreads();                                         // S.tot / S.cnt reuse
        u64 mL[4], mR[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = base + j * 1024 + t;
            const bool in = i < last;
            const u32 key = in ? k[i] : 0u;
            mL[j] = __ballot(in && i > first && !(key < pv));
            mR[j] = __ballot(in && !(pv < key));
            if (l == 0) S.cnt[j * 16 + wv] = ((u32)__popcll(mL[j]) << 16) | (u32)__popcll(mR[j]);
        }
        __syncthreads();
        if (wv == 0) {
            const u32 cc = S.cnt[l];
            const u32 inc = wave_incl_scan_u32(cc);
            S.cnt[l] = inc - cc;
            if (l == 63) S.tot = inc;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = base + j * 1024 + t;
            const u32 o = S.cnt[j * 16 + wv];
            if ((mL[j] >> l) & 1ull) lp[first + nL + (int)(o >> 16) + __popcll(mL[j] & lt)] = (u32)i;
            if ((mR[j] >> l) & 1ull) rq[first + nR + (int)(o & 0xffffu) + __popcll(mR[j] & lt)] = (u32)i;
        }
        nL += (int)(S.tot >> 16);
        nR += (int)(S.tot & 0xffffu);
    }
    __threadfence_block();
    __syncthreads();
    const int m = wg_msearch<1024>(lp, rq, first, nL, nR);
    if (t == 0) S.cut = cut_of(lp, rq, first, nL, nR, m);
    for (int q = t; q < m; q += 1024) {
        const int pl = (int)lp[first + q], pr = (int)rq[first + nR - 1 - q];
        const u32 kl = k[pl], kr = k[pr], vl = v[pl], vr = v[pr];
        k[pl] = kr;
        k[pr] = kl;
        v[pl] = vr;
        v[pr] = vl;
    }
    __threadfence_block();
    __syncthreads();
    return S.cut;
}

// the local jobs; workgroup 0 also ends the key array with the dropped pairs
__global__ void __launch_bounds__(1024) k_tie_local(u32* __restrict__ k, u32* __restrict__ v, u32* __restrict__ lp,
                                                    u32* __restrict__ rq, const int4* __restrict__ jobs,
                                                    const int* __restrict__ ctl, u32* __restrict__ keys,
                                                    u32* __restrict__ vals, TieClasses cls) {
    __shared__ LocalLds S;
    const int t = threadIdx.x;
    const int nj = ctl[T_NJOBS];
    if (blockIdx.x == 0) {
        int start[kMaxTieC + 1];
        const int n = class_starts(cls, start);
        for (int i = ctl[T_VALID] + t; i < n; i += 1024) {
            keys[i] = kTieDrop;
            vals[i] = kTieDrop;
        }
    }
    for (int j = blockIdx.x; j < nj; j += gridDim.x) {
        const int4 jb = jobs[j];
        if (jb.y - jb.x <= kTieLocal) {
            lds_sort(S, k, v, keys, vals, jb.x, jb.y - jb.x, jb.z);
            continue;
        }
        if (t == 0) {
            S.stk[0] = make_int4(jb.x, jb.y, jb.z, 0);
            S.nstk = 1;
        }
        __syncthreads();
        while (S.nstk > 0) {
            __syncthreads();
            if (t == 0) S.top = S.stk[--S.nstk];
            __syncthreads();
            const int4 sg = S.top;
            const int first = sg.x, last = sg.y, len = sg.y - sg.x, d = sg.z;
            if (len <= kTieLocal) {
                lds_sort(S, k, v, keys, vals, first, len, d);
                continue;
            }
            if (d == 0) {                                        // depth limit on a big segment
                if (t == 0) heap_sort(k, v, first, len);
                __threadfence_block();
                __syncthreads();
                for (int i = t; i < len; i += 1024) {
                    keys[first + i] = k[first + i];
                    vals[first + i] = v[first + i];
                }
                __syncthreads();
                continue;
            }
            const int cut = wg_partition(S, k, v, lp, rq, first, last);
            if (t == 0) {
                S.stk[S.nstk++] = make_int4(cut, last, d - 1, 0);
                S.stk[S.nstk++] = make_int4(first, cut, d - 1, 0);
            }
            __syncthreads();
        }
        __syncthreads();
    }
}

}  // namespace

int tie_alloc(TieSort& t, size_t cap, int levels) {
    if (levels < 0) levels = 0;
    if (levels > 6) levels = 6;
    t.cap = cap;
    t.levels = levels;
    t.bcap = kMaxTieC << levels;
    t.jcap = kMaxTieC + 2 * (kMaxTieC << (levels + 1));
    t.tiles = cap / kTieTile + (size_t)t.bcap + 8;
#define PF_TALLOC(p, bytes) \
    if (hipMalloc(&(p), (bytes)) != hipSuccess) return PF_ENOMEM;
    PF_TALLOC(t.k, sizeof(u32) * cap);
    PF_TALLOC(t.v, sizeof(u32) * cap);
    PF_TALLOC(t.lp, sizeof(u32) * cap);
    PF_TALLOC(t.rq, sizeof(u32) * cap);
    PF_TALLOC(t.status, sizeof(u64) * t.tiles);
    PF_TALLOC(t.arrive, sizeof(u32) * 4);
    PF_TALLOC(t.big, sizeof(int4) * 2 * t.bcap);
    PF_TALLOC(t.tot, sizeof(u64) * t.bcap);
    PF_TALLOC(t.jobs, sizeof(int4) * t.jcap);
    PF_TALLOC(t.ctl, sizeof(int) * T_WORDS);
#undef PF_TALLOC
    if (hipMemset(t.status, 0, sizeof(u64) * t.tiles) != hipSuccess || hipMemset(t.arrive, 0, sizeof(u32) * 4) != hipSuccess ||
        hipMemset(t.ctl, 0, sizeof(int) * T_WORDS) != hipSuccess)
        return PF_EHIP;
    return PF_OK;
}

void tie_free(TieSort& t) {
    void* ptrs[] = {t.k, t.v, t.lp, t.rq, t.status, t.arrive, t.big, t.tot, t.jobs, t.ctl};
    for (void* p : ptrs) (void)hipFree(p);
    t = TieSort{};
}

void tie_sort(TieSort& t, u32* keys, u32* vals, TieClasses cls, int* err, hipStream_t s) {
    const int tg = (int)(t.tiles < (size_t)kTieGrid ? t.tiles : (size_t)kTieGrid);
    hipLaunchKernelGGL(k_tie_compact, dim3(tg), dim3(256), 0, s, keys, vals, cls, t.k, t.v, t.ctl, t.status, t.arrive, err);
    hipLaunchKernelGGL(k_tie_setup, dim3(1), dim3(64), 0, s, cls, t.ctl, t.big, t.jobs, t.levels, t.depth0);
    for (int lev = 0; lev < t.levels; ++lev) {
        const int p = lev & 1;
        hipLaunchKernelGGL(k_tie_scan, dim3(tg), dim3(256), 0, s, t.k, t.big + p * t.bcap, t.ctl, p, t.lp, t.rq, t.tot,
                           t.status, t.arrive + 1, err);
        hipLaunchKernelGGL(k_tie_split, dim3(t.bcap), dim3(1024), 0, s, t.k, t.v, t.lp, t.rq, t.big + p * t.bcap, t.tot,
                           t.ctl, p, lev == t.levels - 1 ? 1 : 0, t.big + (p ^ 1) * t.bcap, t.jobs);
    }
    hipLaunchKernelGGL(k_tie_local, dim3(t.jcap), dim3(1024), 0, s, t.k, t.v, t.lp, t.rq, t.jobs, t.ctl, keys, vals, cls);
}

const int* tie_valid_count(const TieSort& t) { return t.ctl + T_VALID; }

}  // namespace pf
