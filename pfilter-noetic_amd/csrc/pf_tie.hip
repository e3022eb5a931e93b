// Reference tie order: libstdc++ introsort's permutation of equal keys, breadth-first (pf_tie.h).
#include <climits>

#include "pf_tie.h"

namespace pf {
namespace {

constexpr u32 kTieDrop = 0xFFFFFFFFu;
constexpr int kThreshold = 16;           // libstdc++ _S_threshold
constexpr int kMaxTieC = 4;              // classes of one sort (key bits 30-31)
constexpr int kTieGrid = 256;            // workgroups of the tile launches (co-resident, look-back)
constexpr int kLocalGrid = 256;          // workgroups of k_tie_local (two per CU)
constexpr int kMidGrid = 128;            // workgroups of k_tie_mid (LDS-limited: one per CU)
constexpr int kMedGrid = 64;             // workgroups of k_tie_medium over a segment list
constexpr int kTieBigLds = 512;          // big segments of one level at most (cached in LDS by k_tie_scan)
constexpr int kDepFree = -2;             // a segment's depth word: no order-dependent group in it (routed)
constexpr int kHeapCap = 20480 - 128;    // longest depth-limit segment k_tie_heap stages in LDS (with the
                                         // spare slots: 160 KB less 512 B)
typedef unsigned short u16;

// control words (TieSort::ctl)
enum {
    T_VALID = 0,        // valid pairs (all classes)
    T_NJOBS = 1,        // local jobs
    T_CS = 2,           // [kMaxTieC] big path: compacted start of every class
    T_BIG = 8,          // u64 [2]: big segments << 32 | their tiles, per level parity
    T_NMED = 12,        // medium segments (big path)
    T_NMID = 13,        // mid-tier segments
    T_NHEAP = 14,       // depth-limit segments for k_tie_heap
    T_NHUGE = 15,       // of them, above the LDS size in a sort with big levels (TieSort::huge)
    T_VC = 16,          // [kMaxTieC] valid pairs of every class
    T_BASE = 20,        // [kMaxTieC] where class c starts in the working copy
    T_NHEAPF = 24,      // huge segments the heap tier still sorts (TieSort::heapf)
    T_HUGEN = 25,       // pairs of the huge segments
    T_NHEAPW = 26,      // depth-limit segments the partition tiers filed for the aux heap launch (TieAux)
    T_CLM_MED = 27,     // items claimed past the first gridDim.x (next_item) by k_tie_medium's segment list,
    T_CLM_MID = 28,     // k_tie_mid, k_tie_local (these three reset by k_tie_local's last workgroup),
    T_CLM_LOCAL = 29,
    T_CLM_HEAP = 30,    // the stream's k_tie_heap launches and the aux one (reset by their last workgroup)
    T_CLM_HEAPW = 31,
    T_CLM_HEAPF = 32,   // the heap launch of the radix route's segments that need pops (TieAux::hs: beside T_NHEAP's)
    T_WORDS = 40
};
__device__ __forceinline__ u64* big_ctr(int* ctl, int p) { return reinterpret_cast<u64*>(ctl + T_BIG) + p; }

__device__ __forceinline__ int lg_floor(int n) { return 31 - __clz(n); }

// The item after `cur` of a launch over n list items: workgroup b takes item b first, then claims the next
// unclaimed one (a counter from gridDim.x) when it is done, so a long item never holds back items dealt
// behind it (configs[4]'s lists hold thousands of segments, a few of them hundreds of times longer than
// the rest). No claim when the first round covers the list. Every thread of the workgroup calls it.
__device__ __forceinline__ int next_item(int n, int* ctr) {
    if (n <= (int)gridDim.x) return n;
    __shared__ int s_next;
    __syncthreads();
    if (threadIdx.x == 0) s_next = (int)gridDim.x + atomicAdd(ctr, 1);
    __syncthreads();
    return s_next;
}

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

__device__ __forceinline__ u32 wave_min_u32(u32 v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const u32 w = (u32)__shfl_xor((int)v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

// atomicMin of each active lane's value into slot[seg]: one atomic per wave when every active lane
// names the same segment (the common case above the deepest levels)
template <class A>
__device__ __forceinline__ void seg_min(A* slot, bool act, u32 seg, u32 val) {
    const u64 am = __ballot(act);
    if (!am) return;
    const u32 s0 = (u32)__shfl((int)seg, __ffsll((long long)am) - 1, 64);
    if (__ballot(act && seg != s0) == 0) {
        const u32 m = wave_min_u32(act ? val : 0xFFFFFFFFu);
        if (lane_id() == 0) atomicMin(&slot[s0], m);
    } else if (act) {
        atomicMin(&slot[seg], val);
    }
}

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

// the median of three moved to first (one thread); returns the pivot
template <class KA, class VA>
__device__ __forceinline__ u32 median_to_first(KA* k, VA* v, int first, int last) {
    const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
    const u32 ka = k[a], kb = k[b], kc = k[c];
    const int sel = median3(ka, kb, kc, a, b, c);
    const u32 pv = sel == a ? ka : (sel == b ? kb : kc);
    const u32 kf = k[first];
    const VA vf = v[first], vs = v[sel];
    k[first] = pv;
    k[sel] = kf;
    v[first] = vs;
    v[sel] = vf;
    return pv;
}

__device__ __forceinline__ void file_job(int* ctl, int4* jobs, int jcap, int* err, int f, int e, int d, int c) {
    if (e - f < 1) return;
    const int j = atomicAdd(&ctl[T_NJOBS], 1);
    if (j < jcap) jobs[j] = make_int4(f, e, d, c);
    else atomicOr(err, 4);
}

// a segment at the depth limit, already at its place in the output [off, off + len): k_tie_heap sorts it
// (with huge set, one above the LDS size goes to the device-wide radix sort first)
struct HeapList {
    int2* seg;
    int cap;
    int* err;
    int2* huge;            // the radix route's list (null: segments above the LDS size go to the heap list)
    int hugecap;
    bool route;            // dependence-free jobs leave k_tie_local unpartitioned (a sort with the radix route)
    // a segment without an order-dependent group: above the LDS size to the radix sort, else to k_tie_heap,
    // whose idle workgroups sort it in LDS beside the few segments that need pops (configs[4]: ~1200 such
    // segments per sort, half of the radix sort's keys, sorted off its critical path)
    __device__ __forceinline__ void file_free(int* ctl, long long off, int len) const {
        if (len <= kHeapCap || !huge) {
            const int j = atomicAdd(&ctl[T_NHEAP], 1);
            if (j < cap) seg[j] = make_int2((int)off, len);
            else atomicOr(err, 4);
            return;
        }
        const int j = atomicAdd(&ctl[T_NHUGE], 1);
        if (j < hugecap) huge[j] = make_int2((int)off, len);
        else atomicOr(err, 4);
    }
    __device__ __forceinline__ void file(int* ctl, long long off, int len) const {
        if (huge && len > kHeapCap) {
            const int j = atomicAdd(&ctl[T_NHUGE], 1);
            if (j < hugecap) huge[j] = make_int2((int)off, len);
            else atomicOr(err, 4);
            return;
        }
        const int j = atomicAdd(&ctl[T_NHEAP], 1);
        if (j < cap) seg[j] = make_int2((int)off, len);
        else atomicOr(err, 4);
    }
};

// ------------------------------------------------------------------------------------------------
// big path: compaction, one pass of 4096-pair tiles (16 rows of 256) with a decoupled look-back; the
// tile holding a class's first input element records where the class starts among the valid pairs
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

// level 0 of the big path: every class is one std::sort call; above kTieMed keys it starts in the
// big levels, otherwise in a medium workgroup
__global__ void k_tie_setup(TieClasses cls, int* __restrict__ ctl, int4* __restrict__ big, int4* __restrict__ med,
                            int levels, int depth0, u32* __restrict__ depn) {
    if (depn)
        for (int i = threadIdx.x; i < kTieBigLds; i += blockDim.x) depn[i] = 0u;
    if (threadIdx.x != 0) return;
    const int nv = ctl[T_VALID];
    int cs[kMaxTieC + 1];
    for (int c = 0; c < kMaxTieC; ++c) cs[c] = c < cls.nc ? ctl[T_CS + c] : nv;
    cs[kMaxTieC] = nv;
    u64 ctr = 0;
    int nm = 0;
    for (int c = 0; c < kMaxTieC; ++c) {
        const int f = cs[c], e = cs[c + 1], len = e - f;
        ctl[T_VC + c] = len > 0 ? len : 0;
        ctl[T_BASE + c] = f;
        if (len < 1) continue;
        const int depth = depth0 >= 0 ? depth0 : 2 * lg_floor(len);   // std::__lg(last - first) * 2
        if (levels > 0 && len > kTieMed && depth > 0) {
            big[(int)(ctr >> 32)] = make_int4(f, e, depth, (int)(u32)ctr);
            ctr += (1ull << 32) | (u64)tiles_of(len);
        } else {
            med[nm++] = make_int4(f, e, depth, c);
        }
    }
    *big_ctr(ctl, 0) = ctr;
    *big_ctr(ctl, 1) = 0;
    ctl[T_NMED] = nm;
    ctl[T_NJOBS] = 0;
}

// the class of a position of the compacted big-path layout
__device__ __forceinline__ int class_of(const int* ctl, int pos) {
    int c = 0;
#pragma unroll
    for (int q = 1; q < kMaxTieC; ++q)
        if (pos >= ctl[T_BASE + q] && ctl[T_VC + q] > 0) c = q;
    return c;
}

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


// every tile of every big segment of level parity p: the stops of its 4096 keys ranked in position
// order. The median of three is applied virtually here (first holds the pivot, sel the old first key)
// and physically by k_tie_split, so no key moves during this launch.
__global__ void __launch_bounds__(256) k_tie_scan(const u32* __restrict__ k, const int4* __restrict__ big,
                                                  int* __restrict__ ctl, int p, u32* __restrict__ lp,
                                                  u32* __restrict__ rq, u64* __restrict__ tot,
                                                  u64* __restrict__ status, u32* __restrict__ arrive,
                                                  int* __restrict__ err, const u32* __restrict__ v,
                                                  const u8* __restrict__ freef, u32* __restrict__ depn) {
    __shared__ int4 s_big[kTieBigLds];
    __shared__ u32 s_cnt[64];
    __shared__ u64 s_off[64];
    const u64 cw = *big_ctr(ctl, p);
    const int nb = (int)(cw >> 32), ntiles = (int)(u32)cw;
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const u64 lt = lanemask_lt();
    if (blockIdx.x == 0 && t == 0) *big_ctr(ctl, p ^ 1) = 0;   // the next level's list (unread here)
    if (freef && blockIdx.x == 0)                               // and its dependent counts
        for (int i = t; i < kTieBigLds; i += 256) depn[((p ^ 1) * kTieBigLds) + i] = 0u;
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
        if (freef) {                                             // order-dependent elements of the segment
            int dep = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int i = base + j * 256 + t;
                if (i < last) dep += freef[v[i]] ? 0 : 1;
            }
            dep = __syncthreads_count(dep);
            if (t == 0 && dep) atomicAdd(&depn[p * kTieBigLds + s], (u32)dep);
        }
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
__device__ __forceinline__ int cut_of(const u32* lp, const u32* rq, int first, int last, int nL, int nR, int m) {
    if (m == 0) return nL ? (int)lp[first] : last;
    const int r = (int)rq[first + nR - m];
    const int lf = m < nL ? (int)lp[first + m] : INT_MAX;
    return lf < r ? lf : r;
}

__device__ __forceinline__ void file_big_child(int* ctl, int pn, int4* next, int bcap, int4* med, int mcap, int* err,
                                               int f, int e, int d, bool may_big) {
    const int len = e - f;
    if (len < 1) return;
    if (may_big && len > kTieMed && d > 0) {
        const u64 r = atomicAdd((unsigned long long*)big_ctr(ctl, pn), (1ull << 32) | (u64)tiles_of(len));
        if ((int)(r >> 32) < bcap) next[(int)(r >> 32)] = make_int4(f, e, d, (int)(u32)r);
        else atomicOr(err, 4);
    } else {
        const int i = atomicAdd(&ctl[T_NMED], 1);
        if (i < mcap) med[i] = make_int4(f, e, d, class_of(ctl, f));
        else atomicOr(err, 4);
    }
}

// one workgroup per big segment of level parity p: the median swap, m, the cut, the m swaps, and the
// two children filed as big segments of the next level or as medium segments
__global__ void __launch_bounds__(1024) k_tie_split(u32* k, u32* v, const u32* __restrict__ lp,
                                                    const u32* __restrict__ rq, const int4* __restrict__ big,
                                                    const u64* __restrict__ tot, int* ctl, int p, int last_level,
                                                    int4* next, int bcap, int4* med, int mcap, int* err,
                                                    u32* __restrict__ depn) {
    __shared__ int s_cut;
    const int nb = (int)(*big_ctr(ctl, p) >> 32);
    const int t = threadIdx.x;
    for (int s = blockIdx.x; s < nb; s += gridDim.x) {
        const int4 sg = big[s];
        const int first = sg.x, last = sg.y, depth = sg.z;
        if (depn && depn[p * kTieBigLds + s] == 0u) {  // no order-dependent group: any order, no more levels
            if (t == 0) {
                const int i = atomicAdd(&ctl[T_NMED], 1);
                if (i < mcap) med[i] = make_int4(first, last, kDepFree, class_of(ctl, first));
                else atomicOr(err, 4);
            }
            continue;
        }
        if (t == 0) median_to_first(k, v, first, last);
        const u64 tt = tot[s];
        const int nL = (int)(tt >> 32), nR = (int)(u32)tt;
        const int m = wg_msearch<1024>(lp, rq, first, nL, nR);
        if (t == 0) s_cut = cut_of(lp, rq, first, last, nL, nR, m);
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
            file_big_child(ctl, p ^ 1, next, bcap, med, mcap, err, first, cut, depth - 1, !last_level);
            file_big_child(ctl, p ^ 1, next, bcap, med, mcap, err, cut, last, depth - 1, !last_level);
        }
        __syncthreads();
    }
}

#ifdef PF_TIE_PROF
// development build (-DPF_TIE_PROF): workgroup 0's first job records the real-time counter at every
// phase boundary of every level (pf_dev_tie_prof reads it back)
__device__ unsigned long long g_tie_prof[1024];
#define TIE_PROF(slot, val) \
    do { if (blockIdx.x == 0 && threadIdx.x == 0 && jb == 0 && (slot) < 1024) g_tie_prof[(slot)] = (val); } while (0)
#else
#define TIE_PROF(slot, val) do { } while (0)
#endif
#ifdef PF_TIE_PROF
#define PART_PROF(slot, val) \
    do { if (prof >= 0 && threadIdx.x == 0 && prof + (slot) < 1024) g_tie_prof[prof + (slot)] = (val); } while (0)
#else
#define PART_PROF(slot, val) do { } while (0)
#endif

// ------------------------------------------------------------------------------------------------
// Partition levels over an item whose active segments are all longer than a stop size (so a wave's 896
// positions meet at most two of them): per level one sweep ranks every active position's stops (tiles of
// 14336 positions, wave w owning rows 14 w .. 14 w + 13 of 64, ranks from ballots, a carried workgroup
// scan across tiles) and lists them by rank (LP / RP); in rank space every left stop then tests
// L_k < R_(nR + 1 - k) and the hits are counted per segment (m: the predicate is monotone), one thread
// per segment finds the cut, a second rank-space pass swaps L_k <-> R_(nR + 1 - k) for k <= m, and the
// children are filed in position order: longer than the stop into the next level (median of three moved
// to first), the others handed on. Two stores: the working copy in global memory (k_tie_medium, one
// workgroup per class) and an item staged in LDS (k_tie_mid).
constexpr int kMT = 1024;
constexpr int kMRows = 7;
constexpr int kMTile = kMT * kMRows;     // 7168
constexpr int kTieMid = 2 * kMTile;      // largest segment the LDS mid tier takes (14336)
constexpr int kTieSmall = 2048;          // largest local job
constexpr int kMBatch = 8;               // left stops per thread in flight in the rank-space passes

template <int NSEG>
struct MedTab {                          // one level's active segments, in position order
    int f[NSEG], e[NSEG], d[NSEG], cut[NSEG];
    u32 pv[NSEG], m[NSEG];
    u32 bl[NSEG], br[NSEG], el[NSEG], er[NSEG];   // stop ranks before first / up to last - 1
    u32 mp[NSEG];                                  // swap ranks before the segment's (prefix of m)
};
template <int NSEG>
struct MedWork {
    MedTab<NSEG> tab[2];
    u32 wt[2][16];
    u32 carry[2][2];
    int n[2];
    u32 msum;
};

// working copy in global memory; ranks listed at the item's own offset of t.lp / t.rq (round 6 measured
// an LDS cache of the ranks the rank-space passes read: no change, 845.2 vs 844.9 frames/s, not kept)
struct GStore {
    u32 *k, *v, *lp, *rq;
    int base;
    __device__ __forceinline__ u32 key(int p) const { return k[p]; }
    __device__ __forceinline__ void setL(u32 g, int p) { lp[base + g] = (u32)p; }
    __device__ __forceinline__ void setR(u32 g, int p) { rq[base + g] = (u32)p; }
    __device__ __forceinline__ int getL(u32 g) const { return (int)lp[base + g]; }
    __device__ __forceinline__ int getR(u32 g) const { return (int)rq[base + g]; }
    __device__ __forceinline__ void load2(int p, int q, u32 (&x)[4]) const {
        x[0] = k[p];
        x[1] = k[q];
        x[2] = v[p];
        x[3] = v[q];
    }
    __device__ __forceinline__ void store2(int p, int q, const u32 (&x)[4]) {
        k[p] = x[1];
        k[q] = x[0];
        v[p] = x[3];
        v[q] = x[2];
    }
    __device__ __forceinline__ u32 median(int f, int e) { return median_to_first(k, v, f, e); }
};
// an item staged in LDS, positions relative to the item
struct LStore {
    u32* K;
    u16 *I, *LP, *RP;
    __device__ __forceinline__ u32 key(int p) const { return K[p]; }
    __device__ __forceinline__ void setL(u32 g, int p) { LP[g] = (u16)p; }
    __device__ __forceinline__ void setR(u32 g, int p) { RP[g] = (u16)p; }
    __device__ __forceinline__ int getL(u32 g) const { return LP[g]; }
    __device__ __forceinline__ int getR(u32 g) const { return RP[g]; }
    __device__ __forceinline__ void load2(int p, int q, u32 (&x)[4]) const {
        x[0] = K[p];
        x[1] = K[q];
        x[2] = I[p];
        x[3] = I[q];
    }
    __device__ __forceinline__ void store2(int p, int q, const u32 (&x)[4]) {
        K[p] = x[1];
        K[q] = x[0];
        I[p] = (u16)x[3];
        I[q] = (u16)x[2];
    }
    __device__ __forceinline__ u32 median(int f, int e) { return median_to_first(K, I, f, e); }
};

// the last segment of T starting at or before p, -1 when none
template <int NSEG>
__device__ __forceinline__ int med_lo(const MedTab<NSEG>& T, int n, int p) {
    if (n == 0 || p < T.f[0]) return -1;
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (T.f[mid] <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
// the segment owning left-stop rank g (the last one whose first rank is <= g)
template <int NSEG>
__device__ __forceinline__ int med_rank_seg(const MedTab<NSEG>& T, int n, u32 g) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (T.bl[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
// atomicAdd of each active lane's 1 into slot[seg]: one atomic per wave when every active lane names
// the same segment
__device__ __forceinline__ void seg_count(u32* slot, bool act, int seg) {
    const u64 am = __ballot(act);
    if (!am) return;
    const int s0 = __shfl(seg, __ffsll((long long)am) - 1, 64);
    if (__ballot(act && seg != s0) == 0) {
        if (lane_id() == 0) atomicAdd(&slot[s0], (u32)__popcll(am));
    } else if (act) {
        atomicAdd(&slot[seg], 1u);
    }
}

// emit(f, e, d): a segment of at most `stop` keys (d >= 0) or one at the depth limit (d = -1: copied to
// the output as it stands by the locals, then heap-sorted there by k_tie_heap), or (d = kDepFree) one
// without an order-dependent group (copied as it stands, then sorted by the radix sort of k_huge_*)
template <int NSEG, class St, class Emit>
__device__ void part_levels(St& st, MedWork<NSEG>& S, int f0, int e0, int d0, int stop, Emit emit, int* err,
                            int prof = -1) {
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const u64 lt = lanemask_lt();
    if (e0 - f0 <= stop || d0 <= 0) {
        if (t == 0) {
            if (d0 == kDepFree) {
                emit(f0, e0, kDepFree);
            } else if (e0 - f0 > stop) {                            // the depth limit above the stop size
                emit(f0, e0, -1);
            } else {
                emit(f0, e0, d0);
            }
        }
        __syncthreads();
        return;
    }
    if (t == 0) {
        MedTab<NSEG>& T = S.tab[0];
        T.f[0] = f0;
        T.e[0] = e0;
        T.d[0] = d0;
        T.m[0] = 0;
        T.pv[0] = st.median(f0, e0);
        S.n[0] = 1;
    }
    __threadfence_block();
    __syncthreads();
    int cur = 0;
    [[maybe_unused]] int lev = 0;
    for (;;) {
        const int ns = S.n[cur];
        PART_PROF(8 * lev, rt_now());
        PART_PROF(8 * lev + 7, (unsigned long long)ns);
        if (ns == 0) break;
        MedTab<NSEG>& T = S.tab[cur];
        // 1. every active position's stops ranked (item-relative ranks), tile by tile
        if (t == 0) {
            S.carry[0][0] = 0;
            S.carry[0][1] = 0;
        }
        __syncthreads();
        int nt = 0;
        for (int tb = f0; tb < e0; tb += kMTile, ++nt) {
            const int par = nt & 1;
            const int wb = tb + w * kMRows * 64;
            const int sa = med_lo(T, ns, wb), sb = sa + 1 < ns ? sa + 1 : -1;
            const int fa = sa >= 0 ? T.f[sa] : 0, ea = sa >= 0 ? T.e[sa] : 0;
            const u32 pa = sa >= 0 ? T.pv[sa] : 0u;
            const int fb = sb >= 0 ? T.f[sb] : INT_MAX, eb = sb >= 0 ? T.e[sb] : 0;
            const u32 pb = sb >= 0 ? T.pv[sb] : 0u;
            // a wave whose positions lie in no active segment (handed on, or past the item) skips its rows
            const bool live = (sa >= 0 && wb < ea) || (sb >= 0 && fb < wb + kMRows * 64 && fb < e0);
            u32 kv[kMRows];
            u32 rk[kMRows];
            u32 bstop = 0, bend = 0, bsel = 0;   // bit j: left / right stop (j + 16); first / last - 1; segment b
            u32 cL = 0, cR = 0;
#pragma unroll
            for (int j = 0; j < kMRows; ++j) {
                kv[j] = 0u;
                rk[j] = 0u;
                if (live && wb + j * 64 + l < e0) kv[j] = st.key(wb + j * 64 + l);
            }
            // the common case: every position of the wave strictly inside segment a (neither its first nor
            // its last): no per-row segment selection
            const bool inner = sa >= 0 && wb > fa && wb + kMRows * 64 < ea && wb + kMRows * 64 <= e0;
            if (inner) {
#pragma unroll
                for (int j = 0; j < kMRows; ++j) {
                    const bool bl = !(kv[j] < pa), br = !(pa < kv[j]);
                    const u64 mL = __ballot(bl), mR = __ballot(br);
                    rk[j] = (cL + (u32)__popcll(mL & lt)) | ((cR + (u32)__popcll(mR & lt)) << 16);
                    bstop |= ((u32)bl << j) | ((u32)br << (j + 16));
                    cL += (u32)__popcll(mL);
                    cR += (u32)__popcll(mR);
                }
            }
#pragma unroll
            for (int j = 0; j < kMRows; ++j) {
                if (!live || inner) break;
                const int p = wb + j * 64 + l;
                const bool ina = p < e0 && sa >= 0 && p >= fa && p < ea;
                const bool inb = p < e0 && !ina && p >= fb && p < eb;
                const bool in = ina || inb;
                const int first = ina ? fa : fb, last = ina ? ea : eb;
                const u32 pv = ina ? pa : pb;
                const bool bl = in && p > first && !(kv[j] < pv);
                const bool br = in && !(pv < kv[j]);
                bend |= ((u32)(in && p == first) << j) | ((u32)(in && p == last - 1) << (j + 16));
                bsel |= (u32)inb << j;
                const u64 mL = __ballot(bl), mR = __ballot(br);
                rk[j] = (cL + (u32)__popcll(mL & lt)) | ((cR + (u32)__popcll(mR & lt)) << 16);
                bstop |= ((u32)bl << j) | ((u32)br << (j + 16));
                cL += (u32)__popcll(mL);
                cR += (u32)__popcll(mR);
            }
            if (l == 0) S.wt[par][w] = (cL << 16) | cR;
            __syncthreads();
            u32 oL = 0, oR = 0, tL = 0, tR = 0;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const u32 c = S.wt[par][q];
                oL += q < w ? (c >> 16) : 0u;
                oR += q < w ? (c & 0xffffu) : 0u;
                tL += c >> 16;
                tR += c & 0xffffu;
            }
            const u32 c0L = S.carry[par][0], c0R = S.carry[par][1];
            oL += c0L;
            oR += c0R;
            if (t == 0) {
                S.carry[par ^ 1][0] = c0L + tL;
                S.carry[par ^ 1][1] = c0R + tR;
            }
#pragma unroll
            for (int j = 0; j < kMRows; ++j) {
                if (!live) break;
                const int p = wb + j * 64 + l;
                const bool bl = (bstop >> j) & 1u, br = (bstop >> (j + 16)) & 1u;
                const u32 gL = oL + (rk[j] & 0xFFFFu), gR = oR + (rk[j] >> 16);
                const int sx = ((bsel >> j) & 1u) ? sb : sa;
                if (bl) st.setL(gL, p);
                if (br) st.setR(gR, p);
                if ((bend >> j) & 1u) {
                    T.bl[sx] = gL;
                    T.br[sx] = gR;
                }
                if ((bend >> (j + 16)) & 1u) {
                    T.el[sx] = gL + (bl ? 1u : 0u);
                    T.er[sx] = gR + (br ? 1u : 0u);
                }
            }
            __syncthreads();
        }
        __threadfence_block();
        __syncthreads();
        PART_PROF(8 * lev + 1, rt_now());
        // 2. m per segment: the largest k <= min(nL, nR) with L_k < R_(nR + 1 - k) (the predicate holds for
        // a prefix of k), one wave per segment searching 64 candidates per round (round 5: the hit count
        // over every left stop cost a pass over all of them, though a level that peels a few keys has
        // nL ~ n and m ~ 0)
        for (int i = w; i < ns; i += kMT / 64) {
            const int nL = (int)(T.el[i] - T.bl[i]), nR = (int)(T.er[i] - T.br[i]);
            int lo = 0, hi = nL < nR ? nL : nR;
            while (lo < hi) {
                const int step = (hi - lo + 63) >> 6;
                int kk = lo + (l + 1) * step;
                kk = kk < hi ? kk : hi;
                const bool ok = st.getL(T.bl[i] + (u32)(kk - 1)) < st.getR(T.br[i] + (u32)(nR - kk));
                const int c = __popcll(__ballot(ok));
                if (c == 0) {
                    hi = lo + step - 1;
                } else {
                    const int nlo = lo + c * step < hi ? lo + c * step : hi;
                    const int nhi = c < 64 ? (lo + (c + 1) * step < hi ? lo + (c + 1) * step : hi) - 1 : hi;
                    lo = nlo;
                    hi = nhi > lo ? nhi : lo;
                }
            }
            if (l == 0) T.m[i] = (u32)lo;
        }
        __threadfence_block();
        __syncthreads();
        PART_PROF(8 * lev + 2, rt_now());
        // 3. one thread per segment: the cut min(L_(m + 1), R_(nR + 1 - m)) (L_1 for m = 0); wave 0: the
        // segments' swap ranks (exclusive prefix of m)
        for (int i = t; i < ns; i += kMT) {
            const int m = (int)T.m[i];
            const int nL = (int)(T.el[i] - T.bl[i]), nR = (int)(T.er[i] - T.br[i]);
            int cut;
            if (m == 0) {
                cut = nL ? st.getL(T.bl[i]) : T.e[i];
            } else {
                const int r = st.getR(T.br[i] + (u32)(nR - m));
                const int lf = m < nL ? st.getL(T.bl[i] + (u32)m) : INT_MAX;
                cut = lf < r ? lf : r;
            }
            T.cut[i] = cut;
        }
        if (w == 0) {
            u32 carry = 0;
            for (int c0 = 0; c0 < ns; c0 += 64) {
                const u32 mv = c0 + l < ns ? T.m[c0 + l] : 0u;
                const u32 inc = wave_incl_scan_u32(mv);
                if (c0 + l < ns) T.mp[c0 + l] = carry + inc - mv;
                carry += (u32)__shfl((int)inc, 63, 64);
            }
            if (l == 0) S.msum = carry;
        }
        __syncthreads();
        PART_PROF(8 * lev + 3, rt_now());
        // 4. the swaps L_k <-> R_(nR + 1 - k), k <= m, over the m's of all segments
        const u32 SM = S.msum;
        for (u32 gb = 0; gb < SM; gb += kMT * kMBatch) {
            int pp[kMBatch], qq[kMBatch];
            u32 pr = 0;
#pragma unroll
            for (int i = 0; i < kMBatch; ++i) {
                const u32 g = gb + (u32)(i * kMT + t);
                pp[i] = 0;
                qq[i] = 0;
                if (g < SM) {
                    int lo = 0, hi = ns - 1;                 // the last segment whose first swap rank is <= g
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (T.mp[mid] <= g) lo = mid;
                        else hi = mid - 1;
                    }
                    const u32 k = g - T.mp[lo];
                    pr |= 1u << i;
                    pp[i] = st.getL(T.bl[lo] + k);
                    qq[i] = st.getR(T.er[lo] - 1u - k);
                }
            }
            u32 x[kMBatch][4];
#pragma unroll
            for (int i = 0; i < kMBatch; ++i)
                if ((pr >> i) & 1u) st.load2(pp[i], qq[i], x[i]);
#pragma unroll
            for (int i = 0; i < kMBatch; ++i)
                if ((pr >> i) & 1u) st.store2(pp[i], qq[i], x[i]);
        }
        __threadfence_block();
        __syncthreads();
        PART_PROF(8 * lev + 4, rt_now());
        // 5. children in position order: above the stop into the next table, the others handed on
        const int nx = cur ^ 1;
        if (w == 0) {
            MedTab<NSEG>& N = S.tab[nx];
            int nn = 0;
            for (int c0 = 0; c0 < ns; c0 += 64) {
                const int si = c0 + l;
                const bool ok = si < ns;
                int ff = 0, ee = 0, cut = 0, dd = 0;
                if (ok) {
                    ff = T.f[si];
                    ee = T.e[si];
                    cut = T.cut[si];
                    dd = T.d[si] - 1;
                }
                const bool bigL = ok && cut - ff > stop && dd > 0;
                const bool bigR = ok && ee - cut > stop && dd > 0;
                const u64 b1 = __ballot(bigL), b2 = __ballot(bigR);
                const int iL = nn + __popcll(b1 & lt) + __popcll(b2 & lt);
                const int iR = iL + (bigL ? 1 : 0);
                nn += __popcll(b1) + __popcll(b2);
                if (ok) {
                    const int cf[2] = {ff, cut}, ce[2] = {cut, ee};
                    const bool bg[2] = {bigL, bigR};
                    const int ix[2] = {iL, iR};
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int a = cf[h], b = ce[h];
                        if (b - a < 1) continue;
                        if (bg[h]) {
                            if (ix[h] < NSEG) {
                                N.f[ix[h]] = a;
                                N.e[ix[h]] = b;
                                N.d[ix[h]] = dd;
                                N.m[ix[h]] = 0;
                                N.pv[ix[h]] = st.median(a, b);
                            } else {
                                atomicOr(err, 4);
                            }
                        } else if (b - a > stop) {             // the depth limit above the stop size
                            emit(a, b, -1);
                        } else {
                            emit(a, b, dd);
                        }
                    }
                }
            }
            if (l == 0) S.n[nx] = nn < NSEG ? nn : NSEG;
        }
        __threadfence_block();
        __syncthreads();
        PART_PROF(8 * lev + 5, rt_now());
        cur = nx;
        ++lev;
    }
    __syncthreads();
}

// true when [f, e) of the working copy (values v) holds an element of an order-dependent group
__device__ __forceinline__ bool range_dep(const u32* v, const u8* freef, int f, int e) {
    int dep = 0;
    for (int i = f + (int)threadIdx.x; i < e && !dep; i += (int)blockDim.x) dep = freef[v[i]] ? 0 : 1;
    return __syncthreads_or(dep) != 0;
}

// hands a segment on: to the LDS mid tier above kTieSmall keys, else (and final segments) to the locals
// with a heap list (TieAux) a segment at the depth limit goes there, to be heap-sorted beside k_tie_local
__device__ __forceinline__ void file_heapw(int* ctl, int4* hw, int hwcap, int* err, int f, int e, int c) {
    const int j = atomicAdd(&ctl[T_NHEAPW], 1);
    if (j < hwcap) hw[j] = make_int4(f, e - f, c, 0);
    else atomicOr(err, 4);
}
struct EmitGlobal {
    int* ctl;
    int4 *mid, *jobs;
    int midcap, jcap, cls;
    int* err;
    int4* hw;
    int hwcap;
    int2* hg;              // TieAux::hs: segments above the LDS size with no levels left -> the radix route,
    int hgcap;             // in working-copy offsets (k_huge_gather reads the working copy)
    __device__ void operator()(int f, int e, int d) const {
        if (e - f < 1) return;
        if (hg && (d == -1 || d == kDepFree) && e - f > kHeapCap) {
            const int j = atomicAdd(&ctl[T_NHUGE], 1);
            if (j < hgcap) hg[j] = make_int2(f, e - f);
            else atomicOr(err, 4);
        } else if (d == -1 && hw) {
            file_heapw(ctl, hw, hwcap, err, f, e, cls);
        } else if (d >= 0 && e - f > kTieSmall) {
            const int j = atomicAdd(&ctl[T_NMID], 1);
            if (j < midcap) mid[j] = make_int4(f, e, d, cls);
            else atomicOr(err, 4);
        } else {
            file_job(ctl, jobs, jcap, err, f, e, d, cls);
        }
    }
};

// L1: one 1024-thread workgroup per class (from_classes: after moving the class's valid pairs into the
// working copy at its input offset) or per medium segment of the big path
__global__ void __launch_bounds__(1024) k_tie_medium(const u32* __restrict__ keys, const u32* __restrict__ vals,
                                                     TieClasses cls, int from_classes, int depth0, u32* k, u32* v,
                                                     u32* lp, u32* rq, int* ctl, const int4* __restrict__ med,
                                                     int4* mid, int midcap, int4* jobs, int jcap, int* err,
                                                     const u8* __restrict__ freef, int4* hw, int hwcap,
                                                     int2* hg, int hgcap) {
    __shared__ MedWork<512> S;
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const u64 lt = lanemask_lt();
    const int nitems = from_classes ? cls.nc : ctl[T_NMED];
    for (int it = blockIdx.x; it < nitems; it = next_item(nitems, &ctl[T_CLM_MED])) {
        int f0, e0, d0, cl;
        if (from_classes) {
            int start[kMaxTieC + 1];
            class_starts(cls, start);
            cl = it;
            const int a = start[cl], b = start[cl + 1];
            if (t == 0) S.carry[0][0] = 0;
            __syncthreads();
            int nt = 0;
            for (int tb = a; tb < b; tb += kMTile, ++nt) {
                const int par = nt & 1;
                u32 kk[kMRows], vv[kMRows], pos[kMRows];
                u32 cnt = 0;
                const int ib = tb + w * kMRows * 64 + l;           // one base, immediate row offsets
                const u32* kb = keys + ib;
                const u32* vb = vals + ib;
#pragma unroll
                for (int j = 0; j < kMRows; ++j) {
                    kk[j] = kTieDrop;
                    vv[j] = 0u;
                    if (ib + j * 64 < b) {
                        kk[j] = kb[j * 64];
                        vv[j] = vb[j * 64];
                    }
                }
#pragma unroll
                for (int j = 0; j < kMRows; ++j) {
                    const u64 m = __ballot(kk[j] != kTieDrop);
                    pos[j] = cnt + (u32)__popcll(m & lt);
                    cnt += (u32)__popcll(m);
                }
                if (l == 0) S.wt[par][w] = cnt;
                __syncthreads();
                u32 off = 0, tot = 0;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const u32 c = S.wt[par][q];
                    off += q < w ? c : 0u;
                    tot += c;
                }
                const u32 c0 = S.carry[par][0];
                off += c0;
                if (t == 0) S.carry[par ^ 1][0] = c0 + tot;
#pragma unroll
                for (int j = 0; j < kMRows; ++j)
                    if (kk[j] != kTieDrop) {
                        k[a + off + pos[j]] = kk[j];
                        v[a + off + pos[j]] = vv[j];
                    }
                __syncthreads();
            }
            const int vc = (int)S.carry[nt & 1][0];
            f0 = a;
            e0 = a + vc;
            d0 = vc > 0 ? (depth0 >= 0 ? depth0 : 2 * lg_floor(vc)) : 0;
            if (t == 0) {
                ctl[T_VC + cl] = vc;
                ctl[T_BASE + cl] = a;
            }
            __threadfence_block();
            __syncthreads();
        } else {
            const int4 mi = med[it];
            f0 = mi.x;
            e0 = mi.y;
            d0 = mi.z;
            cl = mi.w;
        }
        if (freef && d0 > 0 && e0 - f0 > kTieSmall && !range_dep(v, freef, f0, e0)) d0 = kDepFree;
        GStore st{k, v, lp, rq, f0};
        part_levels<512>(st, S, f0, e0, d0, kTieMid, EmitGlobal{ctl, mid, jobs, midcap, jcap, cl, err, hw, hwcap, hg, hgcap}, err,
                         blockIdx.x == 0 && it == 0 ? 256 : -1);
    }
}

// L2: one workgroup per segment of kTieSmall .. kTieMid keys, staged in LDS, partitioned until every
// segment fits kTieSmall, then written back
struct MidLds {
    u32 K[kTieMid];
    u16 I[kTieMid], LP[kTieMid], RP[kTieMid];   // LP and RP adjacent: u32[kTieMid] for the write-back
    MedWork<16> W;
};
struct EmitJob {
    int* ctl;
    int4* jobs;
    int jcap, cls, off;
    int* err;
    int4* hw;
    int hwcap;
    __device__ void operator()(int f, int e, int d) const {
        if (d == -1 && hw && e - f > 0) file_heapw(ctl, hw, hwcap, err, off + f, off + e, cls);
        else file_job(ctl, jobs, jcap, err, off + f, off + e, d, cls);
    }
};
__global__ void __launch_bounds__(1024) k_tie_mid(u32* k, u32* v, int* ctl, const int4* __restrict__ mid,
                                                  int4* jobs, int jcap, int* err, const u8* __restrict__ freef,
                                                  int4* hw, int hwcap) {
    __shared__ MidLds S;
    const int t = threadIdx.x;
    const int nm = ctl[T_NMID];
    for (int it = blockIdx.x; it < nm; it = next_item(nm, &ctl[T_CLM_MID])) {
        const int4 mi = mid[it];
        const int f = mi.x, len = mi.y - mi.x;
        if (freef && !range_dep(v, freef, f, f + len)) {         // no order-dependent group: as it stands
            if (t == 0) file_job(ctl, jobs, jcap, err, f, f + len, kDepFree, mi.w);
            continue;
        }
        for (int i = t; i < len; i += kMT) {
            S.K[i] = k[f + i];
            S.I[i] = (u16)i;
        }
        __syncthreads();
        LStore st{S.K, S.I, S.LP, S.RP};
        part_levels<16>(st, S.W, 0, len, mi.z, kTieSmall, EmitJob{ctl, jobs, jcap, mi.w, f, err, hw, hwcap}, err,
                        blockIdx.x == 0 && it == 0 ? 512 : -1);
        // back to the working copy: the values the keys carry gathered into the (now free) rank lists
        // first, since the gather reads the same range of v that is then written
        u32* VV = reinterpret_cast<u32*>(S.LP);
        for (int i = t; i < len; i += kMT) VV[i] = v[f + S.I[i]];
        __syncthreads();
        for (int i = t; i < len; i += kMT) {
            k[f + i] = S.K[i];
            v[f + i] = VV[i];
        }
        __syncthreads();
    }
}


// ------------------------------------------------------------------------------------------------
// L3 local: one 1024-thread workgroup per job of at most kTieSmall keys, the whole subtree in LDS, every
// segment of a level at once. Wave w owns rows 2 w, 2 w + 1 of 64 (ranks within a row from ballots).
constexpr int kLWaves = 16;
constexpr int kLRows = kTieSmall / (64 * kLWaves);
constexpr int kLSeg = kTieSmall / (kThreshold + 1) + 2;    // segments of one level (> 16 keys each)
constexpr int kWaveSeg = 64;                                // segments this short: finished by one wave
constexpr int kLSmall = kTieSmall / (kThreshold + 1) + 2;  // such segments of one job
// segment ids: a level's table index, or a terminal state (leaf, heap-sorted, finished by a wave)
constexpr u32 kSegLeaf = 0xFFFFu, kSegHeap = 0xFFFEu, kSegWave = 0xFFFDu, kSegLive = 0xFFFDu;
static_assert(kLRows * 64 * kLWaves == kTieSmall, "rows");

struct LocTab {
    u64 A[kLSeg];       // first | last << 16 | pivot << 32
    u32 cd[kLSeg];      // depth while the level runs, then the children: left | right << 16
    u32 cut[kLSeg];     // min of the cut candidates (starts at last)
    u32 base[kLSeg];    // L | R << 16: stop ranks before first
    u32 ends[kLSeg];    // R rank up to last - 1
};
struct LocalLds {
    u32 K[kTieSmall];
    u16 I[kTieSmall], RP[kTieSmall];
    LocTab tab[2];
    u32 lb[kTieSmall / 32];      // first positions of the leaves / heap segments
    u32 small[kLSmall];          // segments for the waves: first | length << 16 | depth << 24
    unsigned char SL[kLWaves][64], SR[kLWaves][64];   // a wave's rank lists while it finishes a segment
    u32 wl[kLWaves], wr[kLWaves];
    int n[2], nsmall;
};

__device__ __forceinline__ void lb_set(u32* lb, int p) { atomicOr(&lb[p >> 5], 1u << (p & 31)); }

// a row's position: wave w owns rows kLRows w .. kLRows w + kLRows - 1
__device__ __forceinline__ int lpos(int w, int j, int l) { return (w * kLRows + j) * 64 + l; }

// the segment id one level down: the child of the parent segment on p's side of its cut
__device__ __forceinline__ u32 child_of(const LocTab& P, u32 s, int p) {
    if (s >= kSegLive) return s;
    const u32 ch = P.cd[s];
    return p < (int)P.cut[s] ? (ch & 0xFFFFu) : (ch >> 16);
}

// one wave finishes a segment of 17 .. 64 keys [f, f + n) at depth d, one key per lane: every
// recursion level of its subtree at once in registers (a lane's segment [sf, se) in lane space), the
// rank lists in the wave's LDS bytes, the exchange of a partition by lane shuffles; then the leaves sorted
// stably and written back; a segment at the depth limit goes back as it stands and is filed for k_tie_heap
// (ofs: the output index of the job's position 0)
__device__ void wave_finish(LocalLds& S, int f, int n, int d, long long ofs, int* ctl, const HeapList& hl) {
    const int w = threadIdx.x >> 6, l = lane_id();
    const u64 lt = lanemask_lt(), le = lt | (1ull << l);
    const bool in = l < n;
    u32 key = in ? S.K[f + l] : 0xFFFFFFFFu;
    u32 idx = in ? S.I[f + l] : 0u;
    int sf = 0, se = n, dd = d;
    unsigned char* SL = S.SL[w];
    unsigned char* SR = S.SR[w];
    for (;;) {
        const bool act = in && se - sf > kThreshold && dd > 0;
        if (!__ballot(act)) break;
        const int a = sf + 1, b = sf + (se - sf) / 2, c = se - 1;
        const u32 ka = (u32)__shfl((int)key, a, 64), kb = (u32)__shfl((int)key, b, 64), kc = (u32)__shfl((int)key, c, 64);
        const int sel = median3(ka, kb, kc, a, b, c);
        const u32 ksel = (u32)__shfl((int)key, sel, 64), isel = (u32)__shfl((int)idx, sel, 64);
        const u32 kfst = (u32)__shfl((int)key, sf, 64), ifst = (u32)__shfl((int)idx, sf, 64);
        if (act && l == sf) {
            key = ksel;
            idx = isel;
        } else if (act && l == sel) {
            key = kfst;
            idx = ifst;
        }
        const u32 pv = ksel;
        const bool bl = act && l > sf && !(key < pv);
        const bool br = act && !(pv < key);
        const u64 ML = __ballot(bl), MR = __ballot(br);
        const u64 smask = (se >= 64 ? ~0ull : ((1ull << se) - 1)) & ~((1ull << sf) - 1);
        const int kL = __popcll(ML & smask & le);                 // 1-based rank of a left stop
        const int nL = __popcll(ML & smask), nR = __popcll(MR & smask);
        const int rlt = __popcll(MR & smask & lt);                // right stops before l
        const bool pred = bl && nR - (rlt + (br ? 1 : 0)) >= kL;  // L_k < R_(nR + 1 - k)
        if (bl) SL[sf + kL - 1] = (unsigned char)l;
        if (br) SR[sf + rlt] = (unsigned char)l;
        const int m = __popcll(__ballot(pred) & smask);
        __builtin_amdgcn_s_waitcnt(0xc07f);                       // lgkmcnt(0): the lists are written
        __builtin_amdgcn_wave_barrier();
        int src = l;
        const int kr = nR - rlt;                                  // a right stop's rank from the right
        if (pred) src = SR[sf + nR - kL];
        else if (br && kr <= m) src = SL[sf + kr - 1];
        int cut = se;
        if (act) {
            if (m == 0) cut = nL ? SL[sf] : se;
            else {
                const int r = SR[sf + nR - m];
                const int lf = m < nL ? SL[sf + m] : 64;
                cut = lf < r ? lf : r;
            }
        }
        key = (u32)__shfl((int)key, src, 64);
        idx = (u32)__shfl((int)idx, src, 64);
        if (act) {
            if (l < cut) se = cut;
            else sf = cut;
            --dd;
        }
        __builtin_amdgcn_wave_barrier();
    }
    // leaves: a stable rank inside [sf, se); heap segments (depth limit) go back as they are
    const bool heap = in && se - sf > kThreshold;
    int dest = l;
    if (!heap) {
        int r = 0;
#pragma unroll
        for (int i = 0; i < kThreshold; ++i) {
            const int q = sf + i;
            const u32 kq = (u32)__shfl((int)key, q < 64 ? q : 63, 64);
            r += (q < se && (kq < key || (kq == key && q < l))) ? 1 : 0;
        }
        dest = sf + r;
    }
    if (in) {
        S.K[f + dest] = key;
        S.I[f + dest] = (u16)idx;
    }
    if (heap && l == sf) hl.file(ctl, ofs + f + sf, se - sf);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
}

// the pass after the level loop: every key to its final place in the output. A leaf [st, en) (at most 16
// keys, bounded by the nearest set bits of lb) is sorted stably (libstdc++'s final insertion sort moves
// no key across a leaf); wave-finished segments are final, depth-limit ones stay as they are (k_tie_heap). The destinations go to RP
// (free after the levels), then every row's value is gathered at once.
__device__ __forceinline__ void local_output(LocalLds& S, int len, const u32 (&sg)[kLRows], const u32* v, int f,
                                             long long obase, u32* keys_out, u32* vals_out) {
    const int w = threadIdx.x >> 6, l = lane_id();
    constexpr int kW = kTieSmall / 32;
#pragma unroll 1
    for (int j = 0; j < kLRows; ++j) {
        const int p = lpos(w, j, l);
        if (w * kLRows * 64 + j * 64 >= len) break;          // rows past the job (uniform)
        if (sg[j] != kSegLeaf) {                              // final in place
            if (p < len) S.RP[p] = (u16)p;
            continue;
        }
        const int pc = p < len ? p : 0;
        const u32 key = S.K[pc];
        const int w0 = pc >> 5, b = pc & 31;
        const u32 m0 = S.lb[w0], mm = S.lb[w0 > 0 ? w0 - 1 : 0], mp = S.lb[w0 + 1 < kW ? w0 + 1 : w0];
        const u32 le = (b == 31) ? 0xFFFFFFFFu : ((2u << b) - 1u);
        const u32 lo = m0 & le, hi = m0 & ~le;
        const int st = lo ? (w0 << 5) + 31 - __clz(lo) : (mm ? ((w0 - 1) << 5) + 31 - __clz(mm) : 0);
        int en = hi ? (w0 << 5) + __ffs(hi) - 1 : ((w0 + 1 < kW && mp) ? ((w0 + 1) << 5) + __ffs(mp) - 1 : len);
        en = en < len ? en : len;
        u32 kq[kThreshold];
#pragma unroll
        for (int i = 0; i < kThreshold; ++i) {
            const int q = st + i;
            kq[i] = S.K[q < en ? q : st];
        }
        int r = 0;
#pragma unroll
        for (int i = 0; i < kThreshold; ++i) {
            const int q = st + i;
            r += (q < en && (kq[i] < key || (kq[i] == key && q < p))) ? 1 : 0;
        }
        if (p < len) S.RP[p] = (u16)(st + r);
    }
    u32 dst[kLRows], ky[kLRows], ip[kLRows];
#pragma unroll
    for (int j = 0; j < kLRows; ++j) {
        const int p = lpos(w, j, l), pc = p < len ? p : 0;
        dst[j] = S.RP[pc];
        ky[j] = S.K[pc];
        ip[j] = S.I[pc];
    }
#pragma unroll
    for (int j = 0; j < kLRows; ++j) ip[j] = v[f + (int)ip[j]];
#pragma unroll
    for (int j = 0; j < kLRows; ++j)
        if (lpos(w, j, l) < len) {
            const long long o = obase + f + (int)dst[j];
            keys_out[o] = ky[j];
            vals_out[o] = ip[j];
        }
}

__global__ void __launch_bounds__(1024) k_tie_local(const u32* __restrict__ k, const u32* __restrict__ v,
                                                    const int4* __restrict__ jobs, int* ctl, u32* __restrict__ arrive,
                                                    u32* __restrict__ keys, u32* __restrict__ vals, TieClasses cls,
                                                    HeapList hl, const u8* __restrict__ freef) {
    __shared__ LocalLds S;
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const u64 lt = lanemask_lt();
    const int nj = ctl[T_NJOBS];
#ifdef PF_TIE_PROF
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_tie_prof[6] = (unsigned long long)nj;
        g_tie_prof[7] = (unsigned long long)ctl[T_NMID];
    }
#endif
    int vcs[kMaxTieC], obase[kMaxTieC];
    int tot = 0;
#pragma unroll
    for (int c = 0; c < kMaxTieC; ++c) {
        vcs[c] = c < cls.nc ? ctl[T_VC + c] : 0;
        obase[c] = tot - ctl[T_BASE + c];           // output index = working-copy index + obase[class]
        tot += vcs[c];
    }
    if (blockIdx.x == 0) {                          // the dropped pairs end the arrays
        int start[kMaxTieC + 1];
        const int n = class_starts(cls, start);
        for (int i = tot + t; i < n; i += 1024) {
            keys[i] = kTieDrop;
            vals[i] = kTieDrop;
        }
        if (t == 0) ctl[T_VALID] = tot;
    }
    for (int jb = blockIdx.x; jb < nj; jb = next_item(nj, &ctl[T_CLM_LOCAL])) {
        const int4 job = jobs[jb];
        const int f = job.x, len = job.y - job.x, d = job.z;
        long long ob = 0;
#pragma unroll
        for (int c = 0; c < kMaxTieC; ++c)
            if (c == job.w) ob = obase[c];
        // at the depth limit in a partition tier, or (with the radix route) without an order-dependent
        // group: as it stands, for k_tie_heap or the radix sort
        const bool freej = d == kDepFree || (hl.route && freef && d >= 0 && len > kThreshold &&
                                             !range_dep(v, freef, f, f + len));
        if (d < 0 || freej) {
            for (int i = t; i < len; i += 1024) {
                keys[ob + f + i] = k[f + i];
                vals[ob + f + i] = v[f + i];
            }
            if (t == 0) {
                if (freej) hl.file_free(ctl, ob + f, len);
                else hl.file(ctl, ob + f, len);
            }
            continue;
        }
        // the segment id of every position this lane owns stays in its registers for the whole job;
        // ract: this wave's rows holding a position still in an active segment (wave-uniform)
        const u32 root = len <= kThreshold ? kSegLeaf : (d == 0 ? kSegHeap : (len <= kWaveSeg ? kSegWave : 0u));
        u32 sg[kLRows];
        u32 ract = 0;
#pragma unroll
        for (int j = 0; j < kLRows; ++j) {
            const int p = lpos(w, j, l);
            sg[j] = p < len ? root : kSegLeaf;
            if (p < len) {
                S.K[p] = k[f + p];
                S.I[p] = (u16)p;
            }
            ract |= (root == 0u && w * kLRows * 64 + j * 64 < len) ? (1u << j) : 0u;
        }
        for (int i = t; i < kTieSmall / 32; i += 1024) S.lb[i] = i == 0 ? 1u : 0u;
        __syncthreads();
        if (t == 0) {
            S.n[0] = root == 0u ? 1 : 0;
            S.n[1] = 0;
            S.nsmall = root == kSegWave ? 1 : 0;
            S.small[0] = (u32)len << 16 | (u32)d << 24;
            if (root == 0u) {
                LocTab& T = S.tab[0];
                const u32 pv = median_to_first(S.K, S.I, 0, len);
                T.A[0] = ((u64)pv << 32) | ((u32)len << 16);
                T.cd[0] = (u32)d;
                T.cut[0] = (u32)len;
            } else if (root == kSegHeap) {
                hl.file(ctl, ob + f, len);
            }
        }
        __syncthreads();
        int cur = 0;
        bool remap = false;
        [[maybe_unused]] int lev = 0;
        TIE_PROF(0, rt_now());
        TIE_PROF(4, __builtin_amdgcn_s_memtime());
        for (;;) {
            const int ns = S.n[cur];
            TIE_PROF(8 + 8 * lev, rt_now());
            TIE_PROF(8 + 8 * lev + 5, (unsigned long long)ns);
            if (ns == 0) break;
            LocTab& T = S.tab[cur];
            LocTab& P = S.tab[cur ^ 1];
            // 1. every active position: its segment (the parent's child on its side of the cut), its
            // stops, its wave-local ranks
            u32 rk[kLRows];
            u32 bstop = 0, bend = 0;           // bit j: left stop / right stop (j + 16); first / last - 1
            u32 rstop = 0;                     // rows with any stop (wave-uniform)
            {
                u32 cL = 0, cR = 0;
                u32 still = 0;
#pragma unroll
                for (int j = 0; j < kLRows; ++j) {
                    rk[j] = 0;
                    if (!((ract >> j) & 1u)) continue;
                    const int p = lpos(w, j, l);
                    const u32 key = S.K[p < len ? p : 0];
                    if (remap) sg[j] = child_of(P, sg[j], p);
                    const bool act = sg[j] < kSegLive;
                    const u64 a = T.A[act ? sg[j] : 0u];
                    const int first = (int)(a & 0xFFFFu), last = (int)((a >> 16) & 0xFFFFu);
                    const u32 pv = (u32)(a >> 32);
                    const bool bl = act && p > first && !(key < pv);
                    const bool br = act && !(pv < key);
                    bend |= ((u32)(act && p == first) << j) | ((u32)(act && p == last - 1) << (j + 16));
                    const u64 mL = __ballot(bl), mR = __ballot(br);
                    still |= __ballot(act) ? (1u << j) : 0u;
                    rstop |= (mL | mR) ? (1u << j) : 0u;
                    rk[j] = (cL + (u32)__popcll(mL & lt)) | ((cR + (u32)__popcll(mR & lt)) << 16);
                    bstop |= ((u32)bl << j) | ((u32)br << (j + 16));
                    cL += (u32)__popcll(mL);
                    cR += (u32)__popcll(mR);
                }
                ract = still;
                if (l == 0) {
                    S.wl[w] = cL;
                    S.wr[w] = cR;
                }
            }
            __syncthreads();
            TIE_PROF(8 + 8 * lev + 1, rt_now());
            // 2. ranks: the right stops listed by rank, every segment's ranks at its ends
            {
                u32 oL = 0, oR = 0;
#pragma unroll
                for (int q = 0; q < kLWaves; ++q) {
                    const u32 a = S.wl[q], b = S.wr[q];
                    oL += q < w ? a : 0u;
                    oR += q < w ? b : 0u;
                }
                const u32 off = oL | (oR << 16);
#pragma unroll
                for (int j = 0; j < kLRows; ++j) {
                    if (!((rstop >> j) & 1u) && !((bend >> j) & 1u) && !((bend >> (j + 16)) & 1u)) continue;
                    const int p = lpos(w, j, l);
                    rk[j] += off;
                    const u32 gR = rk[j] >> 16;
                    const bool br = (bstop >> (j + 16)) & 1u;
                    if (br) S.RP[gR] = (u16)p;
                    if ((bend >> j) & 1u) T.base[sg[j]] = rk[j];
                    if ((bend >> (j + 16)) & 1u) T.ends[sg[j]] = gR + (br ? 1u : 0u);
                }
            }
            __syncthreads();
            TIE_PROF(8 + 8 * lev + 2, rt_now());
            // 3. the swaps: left stop k of its segment with R_(nR + 1 - k) while that lies after it
            // (at least k right stops after L_k); every left stop offers the cut a candidate
#pragma unroll
            for (int j = 0; j < kLRows; ++j) {
                if (!((rstop >> j) & 1u)) continue;
                const bool bl = (bstop >> j) & 1u, br = (bstop >> (j + 16)) & 1u;
                const int p = lpos(w, j, l);
                u32 cand = (u32)p, s = 0;
                if (bl) {
                    s = sg[j];
                    const u32 bs = T.base[s];
                    const int bR = (int)(bs >> 16), eR = (int)T.ends[s];
                    const int kk = (int)(rk[j] & 0xFFFFu) - (int)(bs & 0xFFFFu) + 1;
                    const int rin = (int)(rk[j] >> 16) + (br ? 1 : 0) - bR;
                    if (eR - bR - rin >= kk) {
                        const int q = S.RP[eR - kk];
                        const u32 kq = S.K[q], kp = S.K[p];
                        const u16 iq = S.I[q], ip = S.I[p];
                        S.K[p] = kq;
                        S.I[p] = iq;
                        S.K[q] = kp;
                        S.I[q] = ip;
                        cand = (u32)q;
                    }
                }
                seg_min(T.cut, bl, s, cand);
            }
            __syncthreads();
            TIE_PROF(8 + 8 * lev + 3, rt_now());
            // 4. one thread per segment files its children: above 64 keys with depth left into the next
            // table (median of three moved to first), 17 .. 64 keys to the waves, a child at the depth
            // limit to k_tie_heap
            const int nx = cur ^ 1;
            LocTab& N = S.tab[nx];
            {
                const bool ok = t < ns;
                int ff = 0, ee = 0, cut = 0, dd = 0;
                if (ok) {
                    const u64 a = T.A[t];
                    ff = (int)(a & 0xFFFFu);
                    ee = (int)((a >> 16) & 0xFFFFu);
                    cut = (int)T.cut[t];
                    dd = (int)T.cd[t] - 1;
                }
                const bool aL = ok && cut - ff > kWaveSeg && dd > 0;
                const bool aR = ok && ee - cut > kWaveSeg && dd > 0;
                const u64 b1 = __ballot(aL), b2 = __ballot(aR);
                int wb = 0;
                if (l == 0 && (b1 | b2)) wb = atomicAdd(&S.n[nx], __popcll(b1) + __popcll(b2));
                wb = __shfl(wb, 0, 64);
                const int iL = wb + __popcll(b1 & lt) + __popcll(b2 & lt);
                const int iR = iL + (aL ? 1 : 0);
                if (ok) {
                    u32 ids[2];
                    const int cf[2] = {ff, cut}, ce[2] = {cut, ee};
                    const bool ac[2] = {aL, aR};
                    const int ix[2] = {iL, iR};
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int a = cf[h], b = ce[h];
                        if (ac[h]) {
                            const u32 pv = median_to_first(S.K, S.I, a, b);
                            N.A[ix[h]] = ((u64)pv << 32) | (u32)a | ((u32)b << 16);
                            N.cd[ix[h]] = (u32)dd;
                            N.cut[ix[h]] = (u32)b;
                            ids[h] = (u32)ix[h];
                        } else if (b - a > kThreshold && dd == 0) {
                            hl.file(ctl, ob + f + a, b - a);      // depth limit (__partial_sort)
                            ids[h] = kSegHeap;
                        } else if (b - a > kThreshold) {
                            S.small[atomicAdd(&S.nsmall, 1)] = (u32)a | ((u32)(b - a) << 16) | ((u32)dd << 24);
                            ids[h] = kSegWave;
                        } else {
                            ids[h] = kSegLeaf;
                        }
                    }
                    if (cut < ee && cut > ff) lb_set(S.lb, cut);
                    T.cd[t] = ids[0] | (ids[1] << 16);
                }
                if (t == 0) S.n[cur] = 0;
            }
            __syncthreads();
            TIE_PROF(8 + 8 * lev + 4, rt_now());
            TIE_PROF(8 + 8 * lev + 6, rt_now());
            cur = nx;
            remap = true;
            ++lev;
        }
        TIE_PROF(1, rt_now());
        TIE_PROF(5, __builtin_amdgcn_s_memtime());
        TIE_PROF(3, (unsigned long long)lev);
        if (remap) {
#pragma unroll
            for (int j = 0; j < kLRows; ++j)
                if ((ract >> j) & 1u) sg[j] = child_of(S.tab[cur ^ 1], sg[j], lpos(w, j, l));
        }
        // the short segments, one wave each
        for (int i = w; i < S.nsmall; i += kLWaves) {
            const u32 e = S.small[i];
            wave_finish(S, (int)(e & 0xFFFFu), (int)((e >> 16) & 0xFFu), (int)(e >> 24), ob + f, ctl, hl);
        }
        __syncthreads();
        local_output(S, len, sg, v, f, ob, keys, vals);
        __syncthreads();
        TIE_PROF(2, rt_now());
    }
    // the last workgroup out resets the job counter for the next sort
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        const u32 a = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a == gridDim.x - 1) {
            __hip_atomic_store(&ctl[T_NJOBS], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl[T_NMID], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int c = T_CLM_MED; c <= T_CLM_LOCAL; ++c) __hip_atomic_store(&ctl[c], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}


// ------------------------------------------------------------------------------------------------
// The depth-limit segments: libstdc++'s __partial_sort(first, last, last) = __make_heap + __sort_heap, on
// the output in place, one workgroup per segment staged in LDS as key << 32 | value.
//
// __adjust_heap walks the hole from its start to a leaf, always to the larger child (the right one unless
// right < left), moving each child up, then __push_heap lifts the value back while its parent is less than
// it. Along a max-heap path the values never increase, so the same result comes top-down: at each hole
// take the larger child as above; if it is less than the value, the value lands in the hole, else the
// child moves up. A sift then only reads the two children of its hole and writes the hole, one level per
// step, which is what lets __sort_heap's pops run as a pipeline: pop i + 1 reads the root's children
// once pop i has left level 1, so with pops started two steps apart every later pop stays two levels
// behind the one before it on any shared path and never reads a node that is still to change. A pop
// starts by taking the last element q (its value) and writing the root there; it waits while an earlier
// pop's hole is q or an ancestor of q, since that pop may still write q. __make_heap's sifts of one tree
// level touch disjoint subtrees and run in parallel, deepest level first.
// kHeapCap (top of the file): the longest segment staged in LDS; longer ones run the same schedule on a
// global scratch copy
constexpr int kHeapT = 1024;
constexpr int kHeapGrid = 256;
constexpr int kHeapGridW = 64;          // the aux launch (TieAux): a few depth-limit segments per sort

__device__ __forceinline__ int hlev(int x) { return 31 - __clz(x + 1); }

// where a segment's heap lives: LDS, or (above kHeapCap) a global scratch copy read and written at
// workgroup scope (one wave's lanes hand values to each other through it, and to the other waves of the
// workgroup during __make_heap; one workgroup owns the copy, so its CU's L1 and the XCD's L2 serve it:
// agent scope made every load go past the L1, 1.6 us per pop against 0.66), with the step's stores
// complete before the next step's loads (dropping that wait measured the same, 0.657 vs 0.658 us)
struct LdsHeap {
    uint2* H;
    __device__ __forceinline__ uint2 ld(int i) const { return H[i]; }
    __device__ __forceinline__ void st(int i, uint2 v) const { H[i] = v; }
    __device__ __forceinline__ void step_done() const { asm volatile("" ::: "memory"); }   // LDS: in order
};
struct GlbHeap {
    u64* H;
    __device__ __forceinline__ uint2 ld(int i) const {
        const u64 x = __hip_atomic_load(H + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return make_uint2((u32)x, (u32)(x >> 32));
    }
    __device__ __forceinline__ void st(int i, uint2 v) const {
        __hip_atomic_store(H + i, ((u64)v.y << 32) | v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ __forceinline__ void step_done() const { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
};

// one step of __sort_heap's pipelined pops (wave 0; entries {value, key}): every step reads the children
// of every hole in flight (and, on a step that may start a pop, the last element and the root) and
// writes every hole, with no branch on the lane (a lane with nothing to write writes its own spare slot)
struct HeapPops {
    int nxt;              // the next pop to start (wave-uniform)
    bool act;             // this lane's pop is in flight
    int h, m;             // its hole, its heap size
    uint2 vk;             // its value
};
template <bool MAY, class M>
__device__ __forceinline__ void heap_step(const M& H2, HeapPops& P, int npops, int l, int spare, int last) {
    bool start = false, mine = false;
    int q = 0;
    if (MAY) {
        q = last - P.nxt;                                     // the last element of the heap before pop nxt
        const int sh = hlev(q) - hlev(P.h);
        const bool blk = P.act && sh >= 0 && ((q + 1) >> sh) == P.h + 1;   // hole h is q or an ancestor
        start = P.nxt < npops && __ballot(blk) == 0;
        mine = start && l == (P.nxt & 63);
        P.h = mine ? 0 : P.h;
        P.m = mine ? q : P.m;
        P.act = P.act || mine;
    }
    const int c1 = 2 * P.h + 1;
    const bool has = P.act && c1 < P.m;                       // then c1 + 1 <= m < n
    const int cr = has ? c1 : 0;
    const uint2 a = H2.ld(cr), b = H2.ld(cr + 1);
    if (MAY) {
        const uint2 vq = H2.ld(q), r0 = H2.ld(0);
        P.vk = mine ? vq : P.vk;
        H2.st(mine ? q : spare, r0);
    }
    const bool right = c1 + 1 < P.m && !(b.y < a.y);
    const uint2 ch = right ? b : a;
    const bool stop = !has || ch.y < P.vk.y;
    H2.st(P.act ? P.h : spare, stop ? P.vk : ch);
    P.h = P.act ? (right ? c1 + 1 : c1) : P.h;
    P.act = P.act && !stop;
    P.nxt += start ? 1 : 0;
    H2.step_done();
}

// __make_heap (every thread) then __sort_heap (wave 0) on the n entries of H; spare: the index of lane
// 0's spare slot (lane l writes spare + l); jb: the job's index (the prof build records job 0)
// __make_heap: parents (n - 2) / 2 .. 0, a tree level at a time (the sifts of a level touch disjoint
// subtrees), each the top-down form of __adjust_heap + __push_heap; every thread
template <class M>
__device__ void heap_make(const M& H, int n) {
    const int t = threadIdx.x;
    for (int L = hlev((n - 2) / 2); n >= 2 && L >= 0; --L) {
        const int lo = (1 << L) - 1, hi = min((2 << L) - 2, (n - 2) / 2);
        for (int x = lo + t; x <= hi; x += kHeapT) {
            const uint2 vk = H.ld(x);
            int h = x;
            for (;;) {
                const int c1 = 2 * h + 1;
                if (c1 >= n) break;
                int c = c1;
                uint2 a = H.ld(c1);
                if (c1 + 1 < n) {
                    const uint2 b = H.ld(c1 + 1);
                    if (!(b.y < a.y)) {
                        a = b;
                        c = c1 + 1;
                    }
                }
                if (a.y < vk.y) break;
                H.st(h, a);
                h = c;
            }
            H.st(h, vk);
        }
        __syncthreads();
    }
}

template <class M>
__device__ void heap_sort_seg(const M& H, int n, int spare, [[maybe_unused]] int jb, int npops_in = -1) {
    const int t = threadIdx.x, l = lane_id();
    TIE_PROF(960, rt_now());
    TIE_PROF(965, __builtin_amdgcn_s_memtime());
    TIE_PROF(963, (unsigned long long)n);
    heap_make(H, n);
    // __sort_heap: pop i (i = 0 .. n - 2) in lane i % 64 of wave 0, steps in pairs, a pop starting only
    // on the first of a pair
    TIE_PROF(961, rt_now());
    [[maybe_unused]] unsigned long long steps = 0;
    if (t < 64) {
        const int npops = npops_in < 0 ? n - 1 : npops_in;
        HeapPops P{0, false, 0, 0, make_uint2(0u, 0u)};
        for (;;) {
            heap_step<true>(H, P, npops, l, spare + l, n - 1);
            heap_step<false>(H, P, npops, l, spare + l, n - 1);
#ifdef PF_TIE_PROF
            steps += 2;
#endif
            if (P.nxt >= npops && __ballot(P.act) == 0) break;
        }
    }
    TIE_PROF(962, rt_now());
    TIE_PROF(966, __builtin_amdgcn_s_memtime());
    TIE_PROF(964, steps);
    __syncthreads();
}

// __sort_heap's pops on a segment staged in LDS (round 5): the same pipeline with fewer instructions per
// step. Entries are {position in the segment, key + 1}; the pop that vacates position q writes {the
// root's position, 0} there, so the popped element keeps its name (the output is gathered through the
// positions at the end) and reads as absent to every later pop: no per-lane heap size, and H[n], H[n + 1]
// hold the same sentinel for the children of the last holes. A lane with no pop in flight parks its hole
// at its own spare slot n + 2 + lane, whose children are sentinels, so it stops every step and writes only
// there: no activity flag. A pop starts on the first step of a pair (as heap_step), by its own lane under
// its exec bit, with the value and the root prefetched after the previous pair's writes; the block test
// for the next start (an in-flight hole at q or an ancestor of q) is taken on both children of every hole
// while the second step's loads are in flight and selected by the step's own right / stop decisions. The
// steps are written out in gfx950 assembly, loads and waits included, the children read by one ds_read2_b64
// into four pinned registers (tools/mb/heap_pop.hip v27: 0.286 us per pop against 0.48 for heap_step, both
// checked there against std::make_heap + std::sort_heap).
// kHeapCapP: the longest segment this path takes (two sentinels and 64 spare slots after it)
constexpr int kHeapCapP = kHeapCap - 2;

// the first step of a pair: a pop may start (mine: its lane, by mask), then one level for every lane
__device__ __forceinline__ void lds_pop_step_a(u32 nbb, u32 base8, u32 base, int& h, u32& vx, u32& vy, int spare,
                                          unsigned long long mine, u32 q, u32 rp, u32 vqx, u32 vqy) {
    int hn;
    u32 ad, ax, ay, bx, by, tq, sa, rv, zz, t0, t1, t2, t3, t4;
    unsigned long long sm, tt, rm;
    asm volatile(
        "v_cndmask_b32_e64 %[h], %[h], 0, %[mine]\n\t"
        "v_mov_b32_e32 %[tq], %[q]\n\t"
        "v_mov_b32_e32 %[rv], %[rp]\n\t"
        "v_mov_b32_e32 %[zz], 0\n\t"
        "v_cndmask_b32_e64 %[sa], %[sp], %[tq], %[mine]\n\t"
        "v_lshl_add_u32 %[ad], %[h], 4, %[b8]\n\t"
        "v_lshl_add_u32 %[sa], %[sa], 3, %[base]\n\t"
        "v_min_u32_e32 %[ad], %[nbb], %[ad]\n\t"
        "ds_write2_b32 %[sa], %[rv], %[zz] offset1:1\n\t"
        "ds_read2_b64 v[40:43], %[ad] offset1:1\n\t"
        "v_cndmask_b32_e64 %[vx], %[vx], %[vqx], %[mine]\n\t"
        "v_cndmask_b32_e64 %[vy], %[vy], %[vqy], %[mine]\n\t"
        "v_lshl_add_u32 %[t3], %[h], 1, 1\n\t"
        "v_lshl_add_u32 %[t4], %[h], 3, %[base]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_ge_u32_e64 %[rm], v43, v41\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[t0], v40, v42, %[rm]\n\t"
        "v_cndmask_b32_e64 %[t1], v41, v43, %[rm]\n\t"
        "v_addc_co_u32_e64 %[t3], %[tt], 0, %[t3], %[rm]\n\t"
        "v_cmp_lt_u32_e64 %[sm], %[t1], %[vy]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[t0], %[t0], %[vx], %[sm]\n\t"
        "v_cndmask_b32_e64 %[t2], %[t1], %[vy], %[sm]\n\t"
        "v_cndmask_b32_e64 %[hn], %[t3], %[sp], %[sm]\n\t"
        "ds_write2_b32 %[t4], %[t0], %[t2] offset1:1\n\t"
        : [hn] "=&v"(hn), [h] "+v"(h), [vx] "+v"(vx), [vy] "+v"(vy), [ad] "=&v"(ad), [ax] "=&v"(ax),
          [tq] "=&v"(tq), [sa] "=&v"(sa), [rv] "=&v"(rv),
          [zz] "=&v"(zz), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [t4] "=&v"(t4),
          [sm] "=&s"(sm), [tt] "=&s"(tt), [rm] "=&s"(rm)
        : [sp] "v"(spare), [base] "s"(base), [b8] "s"(base8), [nbb] "s"(nbb), [mine] "s"(mine), [q] "s"(q),
          [rp] "s"(rp), [vqx] "v"(vqx), [vqy] "v"(vqy)
        : "memory", "v40", "v41", "v42", "v43");
    h = hn;
}
// the second step: one level for every lane, the ancestor test of both children of every hole (q1 = q + 1,
// cq = clz(q1)) between the loads' issue and their wait; returns the lanes whose new hole is q or an
// ancestor of q (the next start waits for none)
__device__ __forceinline__ unsigned long long lds_pop_step_b(u32 nbb, u32 base8, u32 base, int& h, u32 vx, u32 vy,
                                                        int spare, u32 q1, u32 cq) {
    int hn;
    u32 ad, ax, ay, bx, by, l1, r1, cl, cr, tl, tr, aLv, aRv, t0, t1, t2, t3, t4, t5;
    unsigned long long sm, blk, tt, rm, am, bm;
    asm volatile(
        "v_lshl_add_u32 %[ad], %[h], 4, %[b8]\n\t"
        "v_min_u32_e32 %[ad], %[nbb], %[ad]\n\t"
        "ds_read2_b64 v[40:43], %[ad] offset1:1\n\t"
        "v_lshl_add_u32 %[l1], %[h], 1, 2\n\t"
        "v_add_u32_e32 %[r1], 1, %[l1]\n\t"
        "v_ffbh_u32_e32 %[cl], %[l1]\n\t"
        "v_ffbh_u32_e32 %[cr], %[r1]\n\t"
        "v_sub_u32_e64 %[cl], %[cl], %[cq]\n\t"
        "v_sub_u32_e64 %[cr], %[cr], %[cq]\n\t"
        "v_lshrrev_b32_e64 %[tl], %[cl], %[q1]\n\t"
        "v_lshrrev_b32_e64 %[tr], %[cr], %[q1]\n\t"
        "v_cmp_eq_u32_e64 %[am], %[tl], %[l1]\n\t"
        "v_cmp_eq_u32_e64 %[bm], %[tr], %[r1]\n\t"
        "v_lshl_add_u32 %[t3], %[h], 1, 1\n\t"
        "v_lshl_add_u32 %[t4], %[h], 3, %[base]\n\t"
        "v_cndmask_b32_e64 %[aLv], 0, 1, %[am]\n\t"
        "v_cndmask_b32_e64 %[aRv], 0, 1, %[bm]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_ge_u32_e64 %[rm], v43, v41\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[t0], v40, v42, %[rm]\n\t"
        "v_cndmask_b32_e64 %[t1], v41, v43, %[rm]\n\t"
        "v_cndmask_b32_e64 %[t5], %[aLv], %[aRv], %[rm]\n\t"
        "v_addc_co_u32_e64 %[t3], %[tt], 0, %[t3], %[rm]\n\t"
        "v_cmp_lt_u32_e64 %[sm], %[t1], %[vy]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[t0], %[t0], %[vx], %[sm]\n\t"
        "v_cndmask_b32_e64 %[t2], %[t1], %[vy], %[sm]\n\t"
        "v_cndmask_b32_e64 %[hn], %[t3], %[sp], %[sm]\n\t"
        "v_cndmask_b32_e64 %[t5], %[t5], 0, %[sm]\n\t"
        "ds_write2_b32 %[t4], %[t0], %[t2] offset1:1\n\t"
        "v_cmp_ne_u32_e64 %[blk], 0, %[t5]\n\t"
        : [hn] "=&v"(hn), [ad] "=&v"(ad), [by] "=&v"(by),
          [l1] "=&v"(l1), [r1] "=&v"(r1), [cl] "=&v"(cl), [cr] "=&v"(cr), [tl] "=&v"(tl), [tr] "=&v"(tr),
          [aLv] "=&v"(aLv), [aRv] "=&v"(aRv), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),
          [t4] "=&v"(t4), [t5] "=&v"(t5), [sm] "=&s"(sm), [blk] "=&s"(blk), [tt] "=&s"(tt), [rm] "=&s"(rm),
          [am] "=&s"(am), [bm] "=&s"(bm)
        : [h] "v"(h), [vx] "v"(vx), [vy] "v"(vy), [sp] "v"(spare), [base] "s"(base), [b8] "s"(base8),
          [nbb] "s"(nbb), [q1] "s"(q1), [cq] "s"(cq)
        : "memory", "v40", "v41", "v42", "v43");
    h = hn;
    return blk;
}

// the pops of a heap built in H[0, n) (sentinel layout above), wave 0; four pairs per exit test
__device__ void lds_pops(uint2* H, int n, int npops) {
    n = __builtin_amdgcn_readfirstlane(n);                      // wave-uniform (the step's masks are scalar)
    npops = __builtin_amdgcn_readfirstlane(npops);
    const int l = lane_id();
    const int last = n - 1;
    const int spare = n + 2 + l;
    const u32 base = (u32)(size_t)H;
    const u32 nbb = base + (u32)n * 8u;
    int nxt = 0;
    int h = spare;
    u32 vx = 0u, vy = 1u;                                        // an idle lane's value: above the sentinels
    unsigned long long blk = 0;
    uint2 vq = H[last];
    u32 rp = H[0].x;
    for (;;) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool start = nxt < npops && blk == 0;          // wave-uniform
            const unsigned long long mine = start ? (1ull << (nxt & 63)) : 0ull;
            lds_pop_step_a(nbb, base + 8u, base, h, vx, vy, spare, mine, (u32)(last - nxt),
                           __builtin_amdgcn_readfirstlane(rp), vq.x, vq.y);
            nxt += start ? 1 : 0;
            const u32 q1 = (u32)(last - nxt + 1);
            blk = lds_pop_step_b(nbb, base + 8u, base, h, vx, vy, spare, q1, (u32)__clz(q1));
            vq = H[last - nxt];                                  // the next start's value and root
            rp = H[0].x;
        }
        if (nxt >= npops && __ballot(h != spare) == 0) break;
    }
}


// Round 6 engine (tools/mb/heap_pop.hip v38): the same pipelined pops with (1) every hole's children
// address carried from step to step (both candidates computed while the loads are in flight, selected by
// the step's own right / stop masks: the shift-add and the clamp leave the chain between a step's loads and
// the next step's), (2) the block test on the level of each hole: q's ancestor at the level of a lane's new
// hole is (q + 1) >> (lev(q) - lev) - 1, one shift taken while the loads are in flight, so the test after
// them is one compare with the new hole (a stopped lane's new hole is its spare, never an ancestor of q);
// 13 VALU of step B's block test become 5, (3) PF_POP_SHARED: every idle lane parks on one spare slot
// (their hole writes then hit one address; 64 distinct 8-byte slots put two lanes of a 32-lane store group
// on every even bank), (4) PF_POP_PERM: consecutive pops dealt to different 16-lane groups of ds_read2_b64
// (pop i on lane ((i & 3) << 4) | ((i >> 2) & 15)); (5) no LDS round trip between a pair's second step and
// the next pair's first: the root's position (broadcast to every lane) is read by step B beside its own
// loads, and the last element's entry by step A itself, first, consumed after step A's wait. Measured in
// the microbenchmark (one wave, s_memtime): 253 (round 5's engine) -> 239 ((1) + (2)) -> 226 cycles per
// step ((5)) -> 219.5 ((6): the block mask taken from the unselected hole, (ancestor == 2h + 1 + right),
// and the stop mask by one SALU and-not, so the next start's decision no longer waits for the hole's
// select; tools/mb/heap_pop.hip v40); (3) and (4) measured no gain and are off (PF_POP_SHARED / _PERM)
__device__ __forceinline__ void lds_pop_step_e(u32 base, u32 b24, u32 nbb, int& h, u32& ad, u32& lh, u32 vb8, u32 vnbb,
                                           u32& vx, u32& vy, int spare, u32 vsp8, u32 vzero,
                                           unsigned long long mine, u32 aq, u32 vrp) {
    int hn;
    u32 sa, t0, t1, t2, t3, t4, aL, aR, aN;
    unsigned long long sm, tt, rm;
    asm volatile(
        "ds_read_b64 v[44:45], %[aq]\n\t"
        "v_cndmask_b32_e64 %[sa], %[sp8], %[aq], %[mine]\n\t"
        "v_cndmask_b32_e64 %[ad], %[ad], %[vb8], %[mine]\n\t"
        "ds_write2_b32 %[sa], %[rp], %[zz] offset1:1\n\t"
        "ds_read2_b64 v[40:43], %[ad] offset1:1\n\t"
        "v_cndmask_b32_e64 %[h], %[h], 0, %[mine]\n\t"
        "v_cndmask_b32_e64 %[lh], %[lh], 0, %[mine]\n\t"
        "v_lshl_add_u32 %[t3], %[h], 1, 1\n\t"
        "v_lshl_add_u32 %[t4], %[h], 3, %[base]\n\t"
        "v_lshl_add_u32 %[aL], %[h], 5, %[b24]\n\t"
        "v_min_u32_e32 %[aL], %[nbb], %[aL]\n\t"
        "v_add_u32_e32 %[aR], 16, %[aL]\n\t"
        "v_min_u32_e32 %[aR], %[nbb], %[aR]\n\t"
        "v_add_u32_e32 %[lh], 1, %[lh]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_ge_u32_e64 %[rm], v43, v41\n\t"
        "v_cndmask_b32_e64 %[vx], %[vx], v44, %[mine]\n\t"
        "v_cndmask_b32_e64 %[vy], %[vy], v45, %[mine]\n\t"
        "v_cndmask_b32_e64 %[t1], v41, v43, %[rm]\n\t"
        "v_cndmask_b32_e64 %[t0], v40, v42, %[rm]\n\t"
        "v_cndmask_b32_e64 %[aN], %[aL], %[aR], %[rm]\n\t"
        "v_cmp_lt_u32_e64 %[sm], %[t1], %[vy]\n\t"
        "v_addc_co_u32_e64 %[t3], %[tt], 0, %[t3], %[rm]\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_e64 %[t0], %[t0], %[vx], %[sm]\n\t"
        "v_cndmask_b32_e64 %[t2], %[t1], %[vy], %[sm]\n\t"
        "v_cndmask_b32_e64 %[ad], %[aN], %[vnbb], %[sm]\n\t"
        "ds_write2_b32 %[t4], %[t0], %[t2] offset1:1\n\t"
        "v_cndmask_b32_e64 %[hn], %[t3], %[sp], %[sm]\n\t"
        : [hn] "=&v"(hn), [h] "+v"(h), [ad] "+v"(ad), [lh] "+v"(lh), [vx] "+v"(vx), [vy] "+v"(vy),
          [sa] "=&v"(sa), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2),
          [t3] "=&v"(t3), [t4] "=&v"(t4), [aL] "=&v"(aL), [aR] "=&v"(aR), [aN] "=&v"(aN),
          [sm] "=&s"(sm), [tt] "=&s"(tt), [rm] "=&s"(rm)
        : [sp] "v"(spare), [sp8] "v"(vsp8), [zz] "v"(vzero), [base] "s"(base), [b24] "s"(b24), [nbb] "s"(nbb),
          [vb8] "v"(vb8), [vnbb] "v"(vnbb), [mine] "s"(mine), [aq] "v"(aq), [rp] "v"(vrp)
        : "memory", "v40", "v41", "v42", "v43", "v44", "v45");
    h = hn;
}
__device__ __forceinline__ unsigned long long lds_pop_step_f(u32 base, u32 b24, u32 nbb, int& h, u32& ad, u32& lh,
                                                         u32 vnbb, u32 vx, u32 vy, int spare, u32 q1, u32 lq1,
                                                         u32 vbase, u32& vrp, u32 aqs, u32& aq) {
    int hn;
    u32 sh, an, t0, t1, t2, t3, t4, aL, aR, aN;
    unsigned long long sm, blk, tt, rm, bm;
    asm volatile(
        "ds_read2_b64 v[40:43], %[ad] offset1:1\n\t"
        "ds_read_b32 %[rp], %[vb]\n\t"
        "v_sub_u32_e32 %[sh], %[lq1], %[lh]\n\t"
        "v_lshl_add_u32 %[t3], %[h], 1, 1\n\t"
        "v_lshrrev_b32_e64 %[an], %[sh], %[q1]\n\t"
        "v_lshl_add_u32 %[t4], %[h], 3, %[base]\n\t"
        "v_lshl_add_u32 %[aL], %[h], 5, %[b24]\n\t"
        "v_add_u32_e32 %[an], -1, %[an]\n\t"
        "v_min_u32_e32 %[aL], %[nbb], %[aL]\n\t"
        "v_add_u32_e32 %[aR], 16, %[aL]\n\t"
        "v_min_u32_e32 %[aR], %[nbb], %[aR]\n\t"
        "v_add_u32_e32 %[lh], 1, %[lh]\n\t"
        "v_mov_b32_e32 %[aq], %[aqs]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_cmp_ge_u32_e64 %[rm], v43, v41\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[t1], v41, v43, %[rm]\n\t"
        "v_cndmask_b32_e64 %[t0], v40, v42, %[rm]\n\t"
        "v_cndmask_b32_e64 %[aN], %[aL], %[aR], %[rm]\n\t"
        "v_cmp_lt_u32_e64 %[sm], %[t1], %[vy]\n\t"
        "v_addc_co_u32_e64 %[t3], %[tt], 0, %[t3], %[rm]\n\t"
        "s_nop 0\n\t"
        "v_cndmask_b32_e64 %[t0], %[t0], %[vx], %[sm]\n\t"
        "v_cndmask_b32_e64 %[t2], %[t1], %[vy], %[sm]\n\t"
        "v_cmp_eq_u32_e64 %[bm], %[an], %[t3]\n\t"
        "ds_write2_b32 %[t4], %[t0], %[t2] offset1:1\n\t"
        "v_cndmask_b32_e64 %[ad], %[aN], %[vnbb], %[sm]\n\t"
        "v_cndmask_b32_e64 %[hn], %[t3], %[sp], %[sm]\n\t"
        "s_andn2_b64 %[blk], %[bm], %[sm]\n\t"
        : [hn] "=&v"(hn), [ad] "+v"(ad), [lh] "+v"(lh), [sh] "=&v"(sh), [an] "=&v"(an), [t0] "=&v"(t0),
          [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [t4] "=&v"(t4), [aL] "=&v"(aL), [aR] "=&v"(aR),
          [aN] "=&v"(aN), [sm] "=&s"(sm), [blk] "=&s"(blk), [tt] "=&s"(tt), [rm] "=&s"(rm), [bm] "=&s"(bm),
          [rp] "=&v"(vrp), [aq] "=&v"(aq)
        : [h] "v"(h), [vx] "v"(vx), [vy] "v"(vy), [sp] "v"(spare), [base] "s"(base), [b24] "s"(b24),
          [nbb] "s"(nbb), [vnbb] "v"(vnbb), [q1] "s"(q1), [lq1] "s"(lq1), [vb] "v"(vbase), [aqs] "s"(aqs)
        : "memory", "v40", "v41", "v42", "v43");
    h = hn;
    return blk;
}
template <bool SHARED, bool PERM>
__device__ void lds_pops2(uint2* H, int n, int npops) {
    n = __builtin_amdgcn_readfirstlane(n);
    npops = __builtin_amdgcn_readfirstlane(npops);
    const int l = lane_id();
    const int last = n - 1;
    const int spare = SHARED ? n + 2 : n + 2 + l;
    const u32 base = (u32)(size_t)H;
    const u32 nbb = base + (u32)n * 8u;
    const u32 b24 = base + 24u;                 // children of child c = 2h + 1 + r: base + 8 + 16 c
    // VGPR copies of loop constants (a VOP3 select reads one SGPR: the mask)
    u32 vb8 = base + 8u, vnbb = nbb, vbase = base, vsp8 = base + 8u * (u32)spare, vzero = 0u;
    asm volatile("" : "+v"(vb8), "+v"(vnbb), "+v"(vbase), "+v"(vsp8), "+v"(vzero));
    int nxt = 0;
    int h = spare;
    u32 ad = nbb, lh = 0u;
    u32 vx = 0u, vy = 1u;                       // an idle lane's value: above the sentinels
    unsigned long long blk = 0;
    u32 vrp = H[0].x;                           // the root's position (every lane)
    u32 aq = base + 8u * (u32)last;             // the address of the next start's q
    for (;;) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool start = nxt < npops && blk == 0;          // wave-uniform
            const int ln = PERM ? (((nxt & 3) << 4) | ((nxt >> 2) & 15)) : (nxt & 63);
            const unsigned long long mine = start ? (1ull << ln) : 0ull;
            lds_pop_step_e(base, b24, nbb, h, ad, lh, vb8, vnbb, vx, vy, spare, vsp8, vzero, mine, aq, vrp);
            nxt += start ? 1 : 0;
            const u32 q1 = (u32)(last - nxt + 1);
            blk = lds_pop_step_f(base, b24, nbb, h, ad, lh, vnbb, vx, vy, spare, q1, (u32)(30 - __clz(q1)), vbase,
                                 vrp, base + 8u * (u32)(last - nxt), aq);
        }
        if (nxt >= npops && __ballot(h != spare) == 0) break;
    }
}
#ifndef PF_HEAP_SIDE
#define PF_HEAP_SIDE 1        // development A/B: 0 = the rest sorted after the pops by the whole workgroup
#endif
#ifndef PF_POP_ENGINE
#define PF_POP_ENGINE 2       // 1: round 5's lds_pops; 2: lds_pops2 (round 6)
#endif
#ifndef PF_POP_SHARED
#define PF_POP_SHARED 0
#endif
#ifndef PF_POP_PERM
#define PF_POP_PERM 0
#endif

// A segment whose keys are all distinct has one sorted order, so whatever sorts it gives __sort_heap's
// exact result: the heap tier first sorts a copy with a bitonic network and keeps it when no two
// neighbours are equal; a segment with an equal pair is restored and heap-sorted. (The depth limit is
// reached mostly inside the voxel-ordered map part of an rgbds input: configs[4]'s ~820k-key segment,
// whose pipelined heap sort takes 0.54 s, holds distinct keys; at configs[1] 30 % of the heap-sorted
// keys do, oracle PFREF_SORT_STATS dupkeys.)
// The network is the flip form (every compare-exchange puts the smaller key first; phase k opens with
// partner i ^ (k - 1), then the half-cleaners i + j): positions at or past the segment's end act as +inf
// and are never touched, so no padding.
#ifndef PF_HEAP_U
#define PF_HEAP_U 4                   // loads in flight per thread in the long segments' global passes
#endif
constexpr int kBitChunk = 16384;      // chunk of a global segment staged in LDS (128 KB)

__device__ __forceinline__ int ce_lo(int c, int j) { return ((c & ~(j - 1)) << 1) | (c & (j - 1)); }
__device__ __forceinline__ int pow2_ceil(int n) { return n <= 1 ? 1 : 1 << (32 - __clz(n - 1)); }

// the flip step of phase k (flip) or the half-cleaner of distance j, on S[0, nv), over a network of size P
__device__ __forceinline__ void lds_ce_step(uint2* S, int nv, int P, int j, int flipmask) {
    for (int c = threadIdx.x; c < (P >> 1); c += kHeapT) {
        const int i = ce_lo(c, j);
        const int q = flipmask ? (i ^ flipmask) : i + j;
        if (q < nv) {
            const uint2 a = S[i], b = S[q];
            if (b.y < a.y) {
                S[i] = b;
                S[q] = a;
            }
        }
    }
    __syncthreads();
}
// phases k0 .. k1 in full (flip + half-cleaners), or (k0 = 0) only the half-cleaners from jtop down
__device__ void lds_bitonic(uint2* S, int nv, int P, int k0, int k1, int jtop) {
    if (k0 == 0) {
        for (int j = jtop; j >= 1; j >>= 1) lds_ce_step(S, nv, P, j, 0);
        return;
    }
    for (int k = k0; k <= k1; k <<= 1) {
        lds_ce_step(S, nv, P, k >> 1, k - 1);
        for (int j = k >> 2; j >= 1; j >>= 1) lds_ce_step(S, nv, P, j, 0);
    }
}
// one step of the network on the global copy (four compare-exchanges in flight per thread)
__device__ void glb_ce_step(const GlbHeap& G, int n, int P, int j, int flipmask) {
    constexpr int U = PF_HEAP_U;
    for (int c0 = threadIdx.x; c0 < (P >> 1); c0 += U * kHeapT) {
        int i[U], q[U];
        uint2 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = c0 + u * kHeapT;
            i[u] = ce_lo(c, j);
            q[u] = flipmask ? (i[u] ^ flipmask) : i[u] + j;
            if (c >= (P >> 1) || q[u] >= n) q[u] = -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (q[u] >= 0) {
                a[u] = G.ld(i[u]);
                b[u] = G.ld(q[u]);
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (q[u] >= 0 && b[u].y < a[u].y) {
                G.st(i[u], b[u]);
                G.st(q[u], a[u]);
            }
    }
    __syncthreads();
}
// i = 0 .. n - 1 over the workgroup, U loads in flight per thread before their stores (the global-side
// passes over a long segment are latency-bound otherwise)
template <int U, class Ld, class St>
__device__ __forceinline__ void copy_batched(int n, const Ld& load, const St& store) {
    for (int i0 = threadIdx.x; i0 < n; i0 += U * kHeapT) {
        uint2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * kHeapT < n) v[u] = load(i0 + u * kHeapT);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * kHeapT < n) store(i0 + u * kHeapT, v[u]);
    }
}
// true when two neighbours of the sorted G[0, n) hold the same key
__device__ bool glb_has_equal(const GlbHeap& G, int n) {
    int eq = 0;
    copy_batched<PF_HEAP_U>(n - 1, [&](int i) { return make_uint2(G.ld(i).y, G.ld(i + 1).y); },
                    [&](int, uint2 v) { eq |= v.x == v.y; });
    return __syncthreads_or(eq) != 0;
}
// the network on the global copy G[0, n): chunks of kBitChunk sorted in LDS, then per phase the steps whose
// partners lie in other chunks on G and the rest chunk by chunk in LDS
__device__ void glb_bitonic(const GlbHeap& G, uint2* S, int n) {
    const int P = pow2_ceil(n);
    const int Pc = P < kBitChunk ? P : kBitChunk;
    for (int kk = 0; kk == 0 || (2 * kBitChunk << (kk - 1)) <= P; ++kk) {
        const int k = kk == 0 ? 0 : kBitChunk << kk;
        if (k) {
            glb_ce_step(G, n, P, k >> 1, k - 1);
            for (int j = k >> 2; j >= kBitChunk; j >>= 1) glb_ce_step(G, n, P, j, 0);
        }
        for (int c0 = 0; c0 < n; c0 += kBitChunk) {
            const int nv = min(kBitChunk, n - c0);
            copy_batched<PF_HEAP_U>(nv, [&](int i) { return G.ld(c0 + i); }, [&](int i, uint2 v) { S[i] = v; });
            __syncthreads();
            if (k) lds_bitonic(S, nv, Pc, 0, 0, kBitChunk >> 1);
            else lds_bitonic(S, nv, Pc, 2, Pc, 0);
            copy_batched<PF_HEAP_U>(nv, [&](int i) { return S[i]; }, [&](int i, uint2 v) { G.st(c0 + i, v); });
            __syncthreads();
        }
    }
}

// ---- which pops are needed: the dependence flags (TieSort::free) ----------------------------------------
// Only the order of a voxel group whose f32 centroid sum depends on the order of its points is observable
// (a group of <= 2 points is order-free: 0 + a is exact and + commutes; of 3, when its three left folds
// agree; pf_odom.hip k_rg_dep). Pops run from the largest key down, so once the smallest key of an
// order-dependent group in the segment has been popped (P = the elements with a key >= it), the rest of
// the heap holds only order-free groups and any sort finishes it; a segment with no order-dependent
// group is the sorted copy itself. Without flags (the VoxelGrid sort, the tests of the permutation) an
// element counts as order-dependent when its key has an equal neighbour: the exact std::sort permutation.
// (A leaner pop engine on 32-bit rank words -- one 8-byte read per step, the ancestor test only on
// steps that may start a pop -- measured 0.48 us per pop against the pair engine's 0.39: a step is
// bound by the wave's VALU issue, about 350-460 cycles, not by the LDS round trip)
// The order-free rest beside the pops (round 6): after npops pops the heap's first r = n - npops entries are
// exactly the elements with a key below kmin (npops counts the keys >= kmin), in heap order, and any sort
// of them is exact (they belong to order-free groups). So the set is taken before __make_heap into its own
// LDS region, and waves 1-15 sort it (the flip-form bitonic network, 960 threads, a barrier of their own
// on an LDS counter) while wave 0 pops, instead of the whole workgroup sorting the heap's rest after the
// pops (34.9 us for r = 2600, 85.6 us for r = 7000 on the critical path, tools/mb/heap_pop.hip k_full).
// Used when the region fits beside the heap and the network's ~1.2 us per stage stays well below the pops.
constexpr int kSideT = kHeapT - 64;
// waves 1-15: arrive on the counter and wait for all 15 (the counter only grows: barrier b waits for 15 b)
__device__ __forceinline__ void side_barrier(u32* ctr, u32& gen) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    ++gen;
    if (lane_id() == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen * (kSideT / 64))
            __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void side_ce_step(uint2* S, int nv, int P, int j, int flipmask, u32* ctr, u32& gen) {
    for (int c = (int)threadIdx.x - 64; c < (P >> 1); c += kSideT) {
        const int i = ce_lo(c, j);
        const int q = flipmask ? (i ^ flipmask) : i + j;
        if (q < nv) {
            const uint2 a = S[i], b = S[q];
            if (b.y < a.y) {
                S[i] = b;
                S[q] = a;
            }
        }
    }
    side_barrier(ctr, gen);
}
__device__ __forceinline__ int bitonic_stages(int P) {
    const int lg = 31 - __clz(P);
    return lg * (lg + 1) / 2;
}

// the segment restored in LDS as {position, key + 1} (keys are below 0xFFFFFFFF: dropped keys never reach a
// segment), two sentinels after it, __make_heap, npops pops (lds_pops), the order-free rest (the keys below
// kmin) sorted, and the output gathered through the positions
__device__ void heap_pops_lds(u32* __restrict__ keys, u32* __restrict__ vals, int off, int n, int npops, uint2* H,
                              u32 kmin) {
    __shared__ u32 s_rc, s_bar;
    const int t = threadIdx.x;
    const int r = n - npops;
    const int Pr = pow2_ceil(r > 1 ? r : 1);
    const bool side = PF_HEAP_SIDE && r >= 2 && n + r + 2 <= kHeapCap && npops >= 6 * bitonic_stages(Pr);
    uint2* R = H + n + 66;                                       // past the sentinels and the spare slots
    if (t == 0) {
        s_rc = 0u;
        s_bar = 0u;
    }
    __syncthreads();
    for (int i = t; i < n; i += kHeapT) {
        const u32 k = keys[off + i];
        H[i] = make_uint2((u32)i, k + 1u);
        if (side && k < kmin) R[atomicAdd(&s_rc, 1u)] = make_uint2((u32)i, k + 1u);
    }
    if (t < 2) H[n + t] = make_uint2(0u, 0u);
    __syncthreads();
    heap_make(LdsHeap{H}, n);
    if (t < 64) {
        if (PF_POP_ENGINE == 2) lds_pops2<PF_POP_SHARED != 0, PF_POP_PERM != 0>(H, n, npops);
        else lds_pops(H, n, npops);
    } else if (side) {
        u32 gen = 0;
        for (int k = 2; k <= Pr; k <<= 1) {
            side_ce_step(R, r, Pr, k >> 1, k - 1, &s_bar, gen);
            for (int j = k >> 2; j >= 1; j >>= 1) side_ce_step(R, r, Pr, j, 0, &s_bar, gen);
        }
    }
    __syncthreads();
    if (!side && npops < n - 1) lds_bitonic(H, r, Pr, 2, Pr, 0);   // the rest: order-free groups only
    constexpr int kPer = (kHeapCapP + kHeapT - 1) / kHeapT;
    u32 gk[kPer], gv[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int i = t + j * kHeapT;
        if (i < n) {
            const u32 p = side && i < r ? R[i].x : H[i].x;
            gk[j] = keys[off + p];
            gv[j] = vals[off + p];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int i = t + j * kHeapT;
        if (i < n) {
            keys[off + i] = gk[j];
            vals[off + i] = gv[j];
        }
    }
}

// One depth-limit segment [off, off + n), n <= kHeapCap, in LDS as {val, key} entries: the sorted copy
// decides the pops, then the segment is restored and heap-sorted that far (heap_sort_seg)
__device__ void heap_segment_pairs(u32* __restrict__ keys, u32* __restrict__ vals, const u8* __restrict__ freef,
                                   int off, int n, uint2* H, int jb) {
    __shared__ u32 s_kmin2, s_pops2;
    const int t = threadIdx.x;
    if (t == 0) {
        s_kmin2 = 0xFFFFFFFFu;
        s_pops2 = 0u;
    }
    __syncthreads();
    if (freef && n <= kHeapCapP) {
        // with the dependence flags the pops needed come from two reductions, no sorted copy: the smallest
        // key of an order-dependent element, then the count of keys at or above it
        u32 km = 0xFFFFFFFFu;
        for (int i = t; i < n; i += kHeapT)
            if (!freef[vals[off + i]]) km = min(km, keys[off + i]);
        km = wave_min_u32(km);
        if (lane_id() == 0 && km != 0xFFFFFFFFu) atomicMin(&s_kmin2, km);
        __syncthreads();
        km = s_kmin2;
        if (km != 0xFFFFFFFFu) {
            u32 c = 0;
            for (int i = t; i < n; i += kHeapT) c += keys[off + i] >= km ? 1u : 0u;
            for (int o = 32; o > 0; o >>= 1) c += (u32)__shfl_xor((int)c, o, 64);
            if (lane_id() == 0) atomicAdd(&s_pops2, c);
            __syncthreads();
            const int popsneed = (int)s_pops2;
            heap_pops_lds(keys, vals, off, n, popsneed >= n ? n - 1 : popsneed, H, km);
            return;
        }
        s_kmin2 = 0xFFFFFFFFu;                          // no order-dependent element: sorted below
        __syncthreads();
    }
    for (int i = t; i < n; i += kHeapT) H[i] = make_uint2(vals[off + i], keys[off + i]);
    __syncthreads();
    const int P2 = pow2_ceil(n);
    lds_bitonic(H, n, P2, 2, P2, 0);
    u32 kmin = 0xFFFFFFFFu;
    for (int i = t; i < n; i += kHeapT) {
        const u32 k = H[i].y;
        const bool dep = freef ? !freef[H[i].x] : ((i > 0 && H[i - 1].y == k) || (i + 1 < n && H[i + 1].y == k));
        if (dep) kmin = min(kmin, k);
    }
    kmin = wave_min_u32(kmin);
    if (lane_id() == 0) atomicMin(&s_kmin2, kmin);
    __syncthreads();
    kmin = s_kmin2;
    if (kmin != 0xFFFFFFFFu) {
        for (int i = t; i < n; i += kHeapT)
            if (H[i].y == kmin && (i == 0 || H[i - 1].y != kmin)) s_pops2 = (u32)(n - i);
        __syncthreads();
        const int popsneed = (int)s_pops2;
        const int npops = popsneed >= n ? n - 1 : popsneed;
        if (n <= kHeapCapP) {
            __syncthreads();
            heap_pops_lds(keys, vals, off, n, npops, H, kmin);
            return;
        }
        for (int i = t; i < n; i += kHeapT) H[i] = make_uint2(vals[off + i], keys[off + i]);   // restore
        __syncthreads();
        heap_sort_seg(LdsHeap{H}, n, kHeapCap, jb, npops);
        if (npops < n - 1) {
            const int r = n - npops, Pr = pow2_ceil(r);
            lds_bitonic(H, r, Pr, 2, Pr, 0);                // the rest: order-free groups only
        }
    }
    for (int i = t; i < n; i += kHeapT) {
        const uint2 x = H[i];
        keys[off + i] = x.y;
        vals[off + i] = x.x;
    }
}

// which: the list's counter (T_NHEAP, or T_NHEAPF for the huge segments the radix sort could not finish);
// the last workgroup out zeroes it and, with also >= 0, that counter too
// wsegs (TieAux): the list holds working-copy segments {offset, length, class} of a partition tier,
// copied to their place in the output (working index + the class's output base, as k_tie_local places
// them) before they are sorted there
__global__ void __launch_bounds__(kHeapT) k_tie_heap(u32* __restrict__ keys, u32* __restrict__ vals, int* ctl,
                                                     const int2* __restrict__ segs, u64* __restrict__ big,
                                                     int bigcap, u32* __restrict__ arrive,
                                                     const u8* __restrict__ freef, int which, int also,
                                                     int2* __restrict__ route, int routecap, int* err,
                                                     const int4* __restrict__ wsegs, const u32* __restrict__ wk,
                                                     const u32* __restrict__ wv, int nc) {
    __shared__ uint2 H[kHeapCap + 64];             // + a spare slot per lane of wave 0
    const int t = threadIdx.x;
    const int nh = ctl[which];
    const int clm = which == T_NHEAPW ? T_CLM_HEAPW : (which == T_NHEAPF ? T_CLM_HEAPF : T_CLM_HEAP);
    for (int jb = blockIdx.x; jb < nh; jb = next_item(nh, &ctl[clm])) {
        int2 sg;
        if (wsegs) {
            const int4 w4 = wsegs[jb];
            int ob = -ctl[T_BASE + w4.z];
            for (int c = 0; c < nc && c < w4.z; ++c) ob += ctl[T_VC + c];
            sg = make_int2(w4.x + ob, w4.y);
            for (int i = t; i < w4.y; i += kHeapT) {
                keys[sg.x + i] = wk[w4.x + i];
                vals[sg.x + i] = wv[w4.x + i];
            }
            __syncthreads();
        } else {
            sg = segs[jb];
        }
        const int off = sg.x, n = sg.y;
        if (route && freef && n > kHeapCap) {   // no order-dependent element: the radix sort after this launch
            int dep = 0;
            for (int i = t; i < n; i += kHeapT) dep |= freef[vals[off + i]] ? 0 : 1;
            if (__syncthreads_or(dep) == 0) {
                if (t == 0) {
                    const int j = atomicAdd(&ctl[T_NHUGE], 1);
                    if (j < routecap) route[j] = sg;
                    else atomicOr(err, 4);
                }
                continue;
            }
        }
        if (n <= kHeapCap) {
            heap_segment_pairs(keys, vals, freef, off, n, H, jb);
        } else {                                              // the copy at the segment's own offset
            GlbHeap G{big + off};
            copy_batched<PF_HEAP_U>(n, [&](int i) { return make_uint2(vals[off + i], keys[off + i]); },
                            [&](int i, uint2 v) { G.st(i, v); });
            __syncthreads();
            glb_bitonic(G, H, n);
            // the sorted copy is the result when no two neighbours are equal or, with the dependence
            // flags, when no element belongs to an order-dependent group
            bool need;
            if (freef) {
                int dep = 0;
                copy_batched<PF_HEAP_U>(n, [&](int i) { return G.ld(i); },
                                        [&](int, uint2 v) { dep |= freef[v.x] ? 0 : 1; });
                need = __syncthreads_or(dep) != 0;
            } else {
                need = glb_has_equal(G, n);
            }
            if (need) {
                for (int i = t; i < n; i += kHeapT) G.st(i, make_uint2(vals[off + i], keys[off + i]));
                __syncthreads();
                heap_sort_seg(G, n, bigcap - off, jb);        // spares: big[bigcap .. bigcap + 64)
            }
            copy_batched<PF_HEAP_U>(n, [&](int i) { return G.ld(i); }, [&](int i, uint2 x) {
                keys[off + i] = x.y;
                vals[off + i] = x.x;
            });
        }
        __syncthreads();
    }
    // the last workgroup out resets the list for the next sort
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        const u32 a = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a == gridDim.x - 1) {
            __hip_atomic_store(&ctl[which], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (also >= 0) __hip_atomic_store(&ctl[also], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl[clm], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---- huge depth-limit segments (sorts with big levels): one device-wide radix sort --------------------
// A depth-limit segment above the LDS size would be sorted by one workgroup (the network, then maybe the
// heap on a global copy: configs[4]'s ~820k-key segment took 25 ms), and with the dependence flags a
// segment of any size that holds no order-dependent group needs no heap at all (configs[4]'s rgbds sort
// leaves ~1200 such segments per frame, 1.6M keys, and ~15 that need pops). Segments of one sort are
// disjoint and in key order (every key of a segment is >= every key of the segments before it, and the
// classes come in class order), so one stable radix sort of all of them gathered back to back in position
// order leaves every segment's keys sorted in its own range. Where that sorted copy is the result (no
// order-dependent group, as in k_tie_heap) it is written back; the other segments keep their input and go
// to the heap tier. The list is filed in any order: k_huge_setup ranks it by offset (O(nh^2)
// on one workgroup: since round 6 the list only holds segments above the LDS size, the shorter dependence-free
// ones being sorted by k_tie_heap's idle workgroups, so nh <= cap / 20352, about 200 at the default capacity).
constexpr int kHugeGrid = 256;
constexpr int kHugeLds = 4096;           // segment bases the gather / check / finish kernels stage in LDS
__global__ void __launch_bounds__(1024) k_huge_setup(int* ctl, const int2* __restrict__ huge, int hugecap,
                                                     int2* __restrict__ hseg, int* __restrict__ hbase,
                                                     u32* __restrict__ need) {
    __shared__ u32 ws[16];
    __shared__ u32 carry;
    __shared__ int s_off[kHugeLds];
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    int nh = ctl[T_NHUGE];
    nh = nh < hugecap ? nh : hugecap;
    const bool lds = nh <= kHugeLds;
    if (lds)
        for (int i = t; i < nh; i += 1024) s_off[i] = huge[i].x;
    __syncthreads();
    for (int i = t; i < nh; i += 1024) {                  // rank by offset (offsets are distinct)
        const int2 x = huge[i];
        int r = 0;
        if (lds)
            for (int j = 0; j < nh; ++j) r += s_off[j] < x.x ? 1 : 0;
        else
            for (int j = 0; j < nh; ++j) r += huge[j].x < x.x ? 1 : 0;
        hseg[r] = x;
        need[r] = 0u;
    }
    if (t == 0) carry = 0u;
    __threadfence_block();
    __syncthreads();
    for (int c0 = 0; c0 < nh; c0 += 1024) {              // exclusive prefix of the lengths in position order
        const int i = c0 + t;
        const u32 len = i < nh ? (u32)hseg[i].y : 0u;
        const u32 inc = wave_incl_scan_u32(len);
        if (l == 63) ws[w] = inc;
        __syncthreads();
        u32 off = carry;
        for (int q = 0; q < w; ++q) off += ws[q];
        if (i < nh) hbase[i] = (int)(off + inc - len);
        __syncthreads();
        if (t == 1023) carry = off + inc;
        __syncthreads();
    }
    if (t == 0) {
        hbase[nh] = (int)carry;
        ctl[T_HUGEN] = (int)carry;
    }
}
// the segment bases (position order) staged in LDS when they fit; returns nh
__device__ __forceinline__ int huge_stage(const int* ctl, int hugecap, const int* hbase, int* s_base) {
    int nh = ctl[T_NHUGE];
    nh = nh < hugecap ? nh : hugecap;
    if (nh < kHugeLds)
        for (int i = threadIdx.x; i <= nh; i += blockDim.x) s_base[i] = hbase[i];
    __syncthreads();
    return nh;
}
__device__ __forceinline__ int huge_seg_of(const int* s_base, const int* hbase, int nh, int i) {
    const int* b = nh < kHugeLds ? s_base : hbase;
    int lo = 0, hi = nh - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (b[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
__global__ void __launch_bounds__(256) k_huge_gather(const u32* __restrict__ keys, const u32* __restrict__ vals,
                                                     const int* ctl, int hugecap, const int2* __restrict__ hseg,
                                                     const int* __restrict__ hbase, u32* __restrict__ hk,
                                                     u32* __restrict__ hv, SortHist sh) {
    __shared__ int s_base[kHugeLds + 1];
    __shared__ u32 lh[4][256];
    sort_hist_begin(lh);
    const int nh = huge_stage(ctl, hugecap, hbase, s_base);
    const int n = ctl[T_HUGEN];
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int s = huge_seg_of(s_base, hbase, nh, i);
        const int p = hseg[s].x + (i - (nh < kHugeLds ? s_base[s] : hbase[s]));
        const u32 key = keys[p];
        hk[i] = key;
        hv[i] = vals[p];
        sort_hist_add(lh, key, sh.passes);
    }
    sort_hist_end(lh, sh, n, n);
}
// a huge segment needs the heap tier when its sorted copy holds an order-dependent element (flags) or,
// without flags, two equal neighbours
__global__ void __launch_bounds__(256) k_huge_check(const int* ctl, int hugecap, const int* __restrict__ hbase,
                                                    const u32* __restrict__ hk, const u32* __restrict__ hv,
                                                    const u8* __restrict__ freef, u32* __restrict__ need) {
    __shared__ int s_base[kHugeLds + 1];
    const int nh = huge_stage(ctl, hugecap, hbase, s_base);
    const int n = ctl[T_HUGEN];
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int s = huge_seg_of(s_base, hbase, nh, i);
        const int end = s + 1 < nh ? (nh < kHugeLds ? s_base[s + 1] : hbase[s + 1]) : n;
        const bool dep = freef ? freef[hv[i]] == 0 : (i + 1 < end && hk[i + 1] == hk[i]);
        if (dep && need[s] == 0u) atomicOr(&need[s], 1u);
    }
}
// the sorted copies written back; the segments that need the heap filed for it (block 0). wk / wv (TieAux::hs):
// the list is in working-copy offsets, so every segment goes to its output place (working offset + its class's
// output base, as k_tie_local places jobs), those that need the heap in their working-copy order
__device__ __forceinline__ int out_base(const int* ctl, int pos) {
    int ob = 0, tot = 0;
#pragma unroll
    for (int c = 0; c < kMaxTieC; ++c) {
        const int vc = ctl[T_VC + c];
        if (pos >= ctl[T_BASE + c] && vc > 0) ob = tot - ctl[T_BASE + c];
        tot += vc;
    }
    return ob;
}
__global__ void __launch_bounds__(256) k_huge_finish(u32* __restrict__ keys, u32* __restrict__ vals, int* ctl,
                                                     int hugecap, const int2* __restrict__ hseg,
                                                     const int* __restrict__ hbase, const u32* __restrict__ hk,
                                                     const u32* __restrict__ hv, const u32* __restrict__ need,
                                                     int2* __restrict__ heapf, const u32* __restrict__ wk,
                                                     const u32* __restrict__ wv) {
    __shared__ int s_base[kHugeLds + 1];
    __shared__ int s_nf;
    const int nh = huge_stage(ctl, hugecap, hbase, s_base);
    const int n = ctl[T_HUGEN];
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) s_nf = 0;
        __syncthreads();
        for (int s = threadIdx.x; s < nh; s += 256)
            if (need[s]) {
                int2 sg = hseg[s];
                if (wk) sg.x += out_base(ctl, sg.x);
                heapf[atomicAdd(&s_nf, 1)] = sg;
            }
        __syncthreads();
        if (threadIdx.x == 0) ctl[T_NHEAPF] = s_nf;
    }
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int s = huge_seg_of(s_base, hbase, nh, i);
        const int p = hseg[s].x + (i - (nh < kHugeLds ? s_base[s] : hbase[s]));
        if (wk) {
            const int o = p + out_base(ctl, hseg[s].x);
            const bool nd = need[s] != 0u;
            keys[o] = nd ? wk[p] : hk[i];
            vals[o] = nd ? wv[p] : hv[i];
            continue;
        }
        if (need[s]) continue;
        keys[p] = hk[i];
        vals[p] = hv[i];
    }
}

// the radix route on stream s: every segment of the huge list sorted by one device-wide radix sort, written
// back, and those that need pops heap-sorted (k_tie_heap's global path). work: the list holds working-copy
// offsets (TieAux::hs; read from t.k / t.v, written to keys / vals at their output places), else output ones
void huge_route(TieSort& t, u32* keys, u32* vals, int* err, const u8* freef, hipStream_t s, bool work, int nc) {
    PrimWork pw = t.hprim;
    pw.err = err;
    hipLaunchKernelGGL(k_huge_setup, dim3(1), dim3(1024), 0, s, t.ctl, t.huge, t.hugecap, t.hseg, t.hbase, t.need);
    hipLaunchKernelGGL(k_huge_gather, dim3(kHugeGrid), dim3(256), 0, s, work ? t.k : keys, work ? t.v : vals, t.ctl,
                       t.hugecap, t.hseg, t.hbase, t.hk, t.hv, sort_hist(pw, 32, true));
    radix_sort_pairs(t.hk, t.hv, t.ctl + T_HUGEN, 32, pw, s, nullptr, nullptr, true);
    hipLaunchKernelGGL(k_huge_check, dim3(kHugeGrid), dim3(256), 0, s, t.ctl, t.hugecap, t.hbase, t.hk, t.hv, freef,
                       t.need);
    hipLaunchKernelGGL(k_huge_finish, dim3(kHugeGrid), dim3(256), 0, s, keys, vals, t.ctl, t.hugecap, t.hseg, t.hbase,
                       t.hk, t.hv, t.need, t.heapf, work ? (const u32*)t.k : nullptr, work ? (const u32*)t.v : nullptr);
    hipLaunchKernelGGL(k_tie_heap, dim3(kHeapGrid), dim3(kHeapT), 0, s, keys, vals, t.ctl, t.heapf, t.hbig, (int)t.cap,
                       t.arrive + (work ? 5 : 3), freef, (int)T_NHEAPF, (int)T_NHUGE, (int2*)nullptr, 0, err,
                       (const int4*)nullptr, (const u32*)nullptr, (const u32*)nullptr, nc);
}

}  // namespace

int tie_alloc(TieSort& t, size_t cap, int max_levels) {
    if (cap < 1) cap = 1;
    if (max_levels < 0) max_levels = cap > (size_t)kTieMed ? 2 * (63 - __builtin_clzll((unsigned long long)cap)) : 0;
    if (max_levels > kMaxBigLevels) max_levels = kMaxBigLevels;
    t.cap = cap;
    t.max_levels = max_levels;
    // the big segments of one level are disjoint and longer than kTieMed (plus a short class of each
    // kind at level 0); every big segment files at most two medium segments
    t.bcap = (int)(cap / kTieMed) + 2 * kMaxTieC + 8;
    if (t.bcap > kTieBigLds) return PF_EINVAL;
    t.mcap = 2 * t.bcap * (max_levels > 0 ? max_levels : 1) + kMaxTieC + 8;
    t.hugecap = (int)(cap / (kThreshold + 1)) + 64;   // any depth-limit segment may be routed there
    // a partitioned segment files at most two pieces per level; the partitioned segments of a level
    // are disjoint and longer than the tier's stop size
    t.jcap = (int)(2 * 64 * (cap / kTieSmall + 1) + 64);
    t.midcap = (int)(2 * 64 * (cap / kTieMid + 1) + 64);
    t.hcap = (int)(cap / (kThreshold + 1) + 64);     // depth-limit segments are disjoint, > 16 keys each
    t.tiles = cap / kTieTile + (size_t)t.bcap + 8;
#define PF_TALLOC(p, bytes) \
    if (hipMalloc(&(p), (bytes)) != hipSuccess) return PF_ENOMEM;
    PF_TALLOC(t.k, sizeof(u32) * cap);
    PF_TALLOC(t.v, sizeof(u32) * cap);
    PF_TALLOC(t.lp, sizeof(u32) * cap);
    PF_TALLOC(t.rq, sizeof(u32) * cap);
    PF_TALLOC(t.status, sizeof(u64) * t.tiles);
    PF_TALLOC(t.arrive, sizeof(u32) * 8);
    PF_TALLOC(t.big, sizeof(int4) * 2 * t.bcap);
    PF_TALLOC(t.tot, sizeof(u64) * t.bcap);
    PF_TALLOC(t.med, sizeof(int4) * t.mcap);
    PF_TALLOC(t.mid, sizeof(int4) * t.midcap);
    PF_TALLOC(t.jobs, sizeof(int4) * t.jcap);
    PF_TALLOC(t.heaps, sizeof(int2) * t.hcap);
    PF_TALLOC(t.heapw, sizeof(int4) * t.hcap);
    PF_TALLOC(t.hbig, sizeof(u64) * (cap + 64));     // segments above the LDS size, at their own offsets
    PF_TALLOC(t.ctl, sizeof(int) * T_WORDS);
    if (max_levels > 0) {
        PF_TALLOC(t.huge, sizeof(int2) * t.hugecap);
        PF_TALLOC(t.heapf, sizeof(int2) * t.hugecap);
        PF_TALLOC(t.need, sizeof(u32) * t.hugecap);
        PF_TALLOC(t.hseg, sizeof(int2) * t.hugecap);
        PF_TALLOC(t.hbase, sizeof(int) * (t.hugecap + 1));
        PF_TALLOC(t.depn, sizeof(u32) * 2 * kTieBigLds);
        PF_TALLOC(t.hk, sizeof(u32) * cap);
        PF_TALLOC(t.hv, sizeof(u32) * cap);
        if (int rc = prim_alloc(t.hprim, cap)) return rc;
    }
#undef PF_TALLOC
    if (hipMemset(t.status, 0, sizeof(u64) * t.tiles) != hipSuccess || hipMemset(t.arrive, 0, sizeof(u32) * 8) != hipSuccess ||
        hipMemset(t.ctl, 0, sizeof(int) * T_WORDS) != hipSuccess)
        return PF_EHIP;
    return PF_OK;
}

void tie_free(TieSort& t) {
    void* ptrs[] = {t.k, t.v, t.lp, t.rq, t.status, t.arrive, t.big, t.tot, t.med, t.mid, t.jobs, t.heaps, t.heapw, t.hbig,
                    t.ctl, t.huge, t.heapf, t.need, t.hk, t.hv, t.hseg, t.hbase, t.depn};
    for (void* p : ptrs) (void)hipFree(p);
    if (t.hprim.cap) prim_free(t.hprim);
    t = TieSort{};
}

int tie_levels_for(const TieSort& t, size_t size_hint) {
    if (size_hint <= (size_t)kTieMed) return 0;
    const int lv = 2 * (63 - __builtin_clzll((unsigned long long)size_hint));
    return lv < t.max_levels ? lv : t.max_levels;
}

void tie_sort(TieSort& t, u32* keys, u32* vals, TieClasses cls, int* err, hipStream_t s, int levels,
              const u8* freef, const TieAux* aux) {
    if (levels > t.max_levels) levels = t.max_levels;
    // the radix route (sorts with big levels): huge depth-limit segments and, with dependence flags,
    // every segment without an order-dependent group, from any tier
    const bool huge = levels > 0 && t.huge;
    const u8* rf = huge ? freef : nullptr;
    u32* depn = rf ? t.depn : nullptr;
    // the partition tiers' depth-limit segments heap-sorted on aux beside k_tie_local (no big levels)
    const bool side = aux && aux->s && levels <= 0;
    // the radix route on aux->hs beside the tiers after k_tie_medium (big levels)
    const bool early = huge && aux && aux->hs;
    int4* hw = side ? t.heapw : nullptr;
    if (levels <= 0) {
        hipLaunchKernelGGL(k_tie_medium, dim3(kMaxTieC), dim3(kMT), 0, s, keys, vals, cls, 1, t.depth0, t.k, t.v,
                           t.lp, t.rq, t.ctl, t.med, t.mid, t.midcap, t.jobs, t.jcap, err, rf, hw, t.hcap,
                           (int2*)nullptr, 0);
    } else {
        const int tg = (int)(t.tiles < (size_t)kTieGrid ? t.tiles : (size_t)kTieGrid);
        hipLaunchKernelGGL(k_tie_compact, dim3(tg), dim3(256), 0, s, keys, vals, cls, t.k, t.v, t.ctl, t.status,
                           t.arrive, err);
        hipLaunchKernelGGL(k_tie_setup, dim3(1), dim3(64), 0, s, cls, t.ctl, t.big, t.med, levels, t.depth0, depn);
        for (int lev = 0; lev < levels; ++lev) {
            const int p = lev & 1;
            hipLaunchKernelGGL(k_tie_scan, dim3(tg), dim3(256), 0, s, t.k, t.big + p * t.bcap, t.ctl, p, t.lp, t.rq,
                               t.tot, t.status, t.arrive + 1, err, t.v, rf, depn);
            hipLaunchKernelGGL(k_tie_split, dim3(t.bcap), dim3(1024), 0, s, t.k, t.v, t.lp, t.rq, t.big + p * t.bcap,
                               t.tot, t.ctl, p, lev == levels - 1 ? 1 : 0, t.big + (p ^ 1) * t.bcap, t.bcap, t.med,
                               t.mcap, err, depn);
        }
        hipLaunchKernelGGL(k_tie_medium, dim3(kMedGrid), dim3(kMT), 0, s, keys, vals, cls, 0, t.depth0, t.k, t.v, t.lp,
                           t.rq, t.ctl, t.med, t.mid, t.midcap, t.jobs, t.jcap, err, rf, (int4*)nullptr, 0,
                           early ? t.huge : (int2*)nullptr, t.hugecap);
        if (early) {    // fork: the segments for the radix route are all filed
            (void)hipEventRecord(aux->fork, s);
            (void)hipStreamWaitEvent(aux->hs, aux->fork, 0);
            huge_route(t, keys, vals, err, freef, aux->hs, true, cls.nc);
            (void)hipEventRecord(aux->join, aux->hs);
        }
    }
    hipLaunchKernelGGL(k_tie_mid, dim3(kMidGrid), dim3(kMT), 0, s, t.k, t.v, t.ctl, t.mid, t.jobs, t.jcap, err, rf, hw,
                       t.hcap);
    if (side) {     // fork: the tiers' depth-limit segments are all filed, in the working copy
        (void)hipEventRecord(aux->fork, s);
        (void)hipStreamWaitEvent(aux->s, aux->fork, 0);
        hipLaunchKernelGGL(k_tie_heap, dim3(kHeapGridW), dim3(kHeapT), 0, aux->s, keys, vals, t.ctl, (const int2*)nullptr,
                           t.hbig, (int)t.cap, t.arrive + 4, freef, (int)T_NHEAPW, -1, (int2*)nullptr, 0, err,
                           (const int4*)t.heapw, (const u32*)t.k, (const u32*)t.v, cls.nc);
        (void)hipEventRecord(aux->join, aux->s);
    }
    hipLaunchKernelGGL(k_tie_local, dim3(kLocalGrid), dim3(1024), 0, s, t.k, t.v, t.jobs, t.ctl, t.arrive + 2, keys,
                       vals, cls, HeapList{t.heaps, t.hcap, err, huge && !early ? t.huge : nullptr, t.hugecap, huge}, rf);
    hipLaunchKernelGGL(k_tie_heap, dim3(kHeapGrid), dim3(kHeapT), 0, s, keys, vals, t.ctl, t.heaps, t.hbig,
                       (int)t.cap, t.arrive + 3, freef, (int)T_NHEAP, -1, huge && !early ? t.huge : nullptr, t.hugecap,
                       err, (const int4*)nullptr, (const u32*)nullptr, (const u32*)nullptr, cls.nc);
    if (side || early) (void)hipStreamWaitEvent(s, aux->join, 0);   // join
    else if (huge) huge_route(t, keys, vals, err, freef, s, false, cls.nc);
}

const int* tie_valid_count(const TieSort& t) { return t.ctl + T_VALID; }

#ifdef PF_TIE_PROF
extern "C" int pf_dev_tie_prof(unsigned long long* out, int n) {
    if (n > 1024) n = 1024;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tie_prof), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace pf
