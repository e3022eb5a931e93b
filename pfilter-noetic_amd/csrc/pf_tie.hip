// Reference tie order: libstdc++ introsort's permutation of equal keys, level-synchronously (pf_tie.h).
#include <climits>

#include "pf_tie.h"

namespace pf {
namespace {

constexpr u32 kTieDrop = 0xFFFFFFFFu;
constexpr int kTieGrid = 512;        // workgroups of a level launch (4 waves each, one segment per wave)
constexpr int kThreshold = 16;       // libstdc++ _S_threshold

__device__ __forceinline__ int lg_floor(int n) { return 31 - __clz(n); }

__global__ void __launch_bounds__(256) k_tie_flags(const u32* __restrict__ keys, const int* __restrict__ d_n,
                                                   u32* __restrict__ flag) {
    const int n = *d_n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        flag[i] = keys[i] != kTieDrop ? 1u : 0u;
}

__global__ void __launch_bounds__(256) k_tie_scatter(const u32* __restrict__ keys, const u32* __restrict__ vals,
                                                     const int* __restrict__ d_n, const u32* __restrict__ pos,
                                                     u32* __restrict__ k, u32* __restrict__ v) {
    const int n = *d_n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u32 key = keys[i];
        if (key == kTieDrop) continue;
        k[pos[i]] = key;
        v[pos[i]] = vals[i];
    }
}

// the initial segments: one per class present (the compacted pairs are class-major), depth 2 lg(n)
__global__ void k_tie_init(const u32* __restrict__ k, int* __restrict__ cnt, int4* __restrict__ seg0,
                           int2* __restrict__ leaf) {
    if (threadIdx.x != 0) return;
    const int n = (int)((const u32*)cnt)[5];
    cnt[0] = cnt[1] = cnt[2] = cnt[3] = cnt[4] = 0;
    int first = 0;
    for (int c = 0; c < 4 && first < n; ++c) {
        int lo = first, hi = n;                           // first index of a class above c
        while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if ((int)(k[m] >> 30) <= c) lo = m + 1;
            else hi = m;
        }
        const int last = lo, len = last - first;
        if (len > kThreshold) seg0[cnt[0]++] = make_int4(first, last, 2 * lg_floor(len), 0);
        else if (len >= 2) leaf[cnt[3]++] = make_int2(first, last);
        first = last;
    }
}

__device__ __forceinline__ void swap_at(u32* k, u32* v, int i, int j) {
    const u32 ki = k[i], kj = k[j], vi = v[i], vj = v[j];
    k[i] = kj;
    k[j] = ki;
    v[i] = vj;
    v[j] = vi;
}

// One recursion level: every segment of list `cur` is partitioned by one wavefront (or, at the depth
// limit, handed to the heap sort); the children go to list (cur + 1) % 3 or to the leaves. Lanes
// exchange the median swap and the stop positions through global memory inside one wave, so each
// exchange is fenced (device-scope fence: the stores are performed and the CU's L1 invalidated).
__global__ void __launch_bounds__(256) k_tie_level(u32* __restrict__ k, u32* __restrict__ v, int* __restrict__ cnt,
                                                   int4* __restrict__ cur_list, int4* __restrict__ next_list,
                                                   int cur, int4* __restrict__ heap, int2* __restrict__ leaf,
                                                   int* __restrict__ lp, int* __restrict__ rq) {
    const int l = lane_id();
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nwaves = (int)((gridDim.x * blockDim.x) >> 6);
    const int nseg = cnt[cur];
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(cur + 2) % 3] = 0;   // read by the previous level only
    for (int s = wave; s < nseg; s += nwaves) {
        const int4 sg = cur_list[s];
        const int first = sg.x, last = sg.y, depth = sg.z;
        if (depth == 0) {                                   // __partial_sort at the depth limit
            if (l == 0) heap[atomicAdd(&cnt[4], 1)] = sg;
            continue;
        }
        // __move_median_to_first(first, first + 1, mid, last - 1)
        u32 pv = 0;
        if (l == 0) {
            const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
            const u32 ka = k[a], kb = k[b], kc = k[c];
            int sel;
            if (ka < kb) sel = kb < kc ? b : (ka < kc ? c : a);
            else sel = ka < kc ? a : (kb < kc ? c : b);
            swap_at(k, v, first, sel);
            pv = sel == a ? ka : (sel == b ? kb : kc);
        }
        pv = (u32)__builtin_amdgcn_readfirstlane((int)pv);
        __threadfence();
        // stops: left (key >= pivot) in [first + 1, last), right (key <= pivot) in [first, last), in
        // ascending order, four chunks of 64 per round so that the loads overlap
        int nL = 0, nR = 0;
        const u64 lt = lanemask_lt();
        for (int base = first; base < last; base += 256) {
            u32 kk[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = base + 64 * j + l;
                kk[j] = i < last ? k[i] : 0u;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = base + 64 * j + l;
                const bool in = i < last;
                const bool fl = in && i > first && !(kk[j] < pv);
                const bool fr = in && !(pv < kk[j]);
                const u64 bl = __ballot(fl), br = __ballot(fr);
                if (fl) lp[first + nL + __popcll(bl & lt)] = i;
                if (fr) rq[first + nR + __popcll(br & lt)] = i;
                nL += __popcll(bl);
                nR += __popcll(br);
            }
        }
        __threadfence();
        // m = the last k with L_k < R_(nR + 1 - k): a binary search (the predicate is monotone)
        int lo = 0, hi = nL < nR ? nL : nR;
        while (lo < hi) {
            const int m = (lo + hi + 1) >> 1;
            if (lp[first + m - 1] < rq[first + nR - m]) lo = m;
            else hi = m - 1;
        }
        const int m = lo;
        int cut;
        if (m == 0) cut = nL ? lp[first] : last;
        else {
            const int r = rq[first + nR - m];
            const int lft = m < nL ? lp[first + m] : INT_MAX;
            cut = lft < r ? lft : r;
        }
        for (int t = l; t < m; t += 64) swap_at(k, v, lp[first + t], rq[first + nR - 1 - t]);
        if (l == 0) {
            const int kid[2][2] = {{first, cut}, {cut, last}};
            for (int q = 0; q < 2; ++q) {
                const int f = kid[q][0], e = kid[q][1];
                if (e - f > kThreshold) next_list[atomicAdd(&cnt[(cur + 1) % 3], 1)] = make_int4(f, e, depth - 1, 0);
                else if (e - f >= 2) leaf[atomicAdd(&cnt[3], 1)] = make_int2(f, e);
            }
        }
    }
}

__device__ __forceinline__ void adjust_heap(u32* k, u32* v, int base, int hole, int len, u32 vk, u32 vv) {
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
    int parent = (hole - 1) / 2;                          // __push_heap
    while (hole > top && k[base + parent] < vk) {
        k[base + hole] = k[base + parent];
        v[base + hole] = v[base + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    k[base + hole] = vk;
    v[base + hole] = vv;
}

// libstdc++'s __partial_sort(first, last, last) = __make_heap + __sort_heap, one thread per segment
__global__ void k_tie_heap(u32* __restrict__ k, u32* __restrict__ v, const int* __restrict__ cnt,
                           const int4* __restrict__ heap) {
    const int nh = cnt[4];
    for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < nh; h += gridDim.x * blockDim.x) {
        const int base = heap[h].x, len = heap[h].y - heap[h].x;
        if (len >= 2) {
            for (int parent = (len - 2) / 2;; --parent) {
                adjust_heap(k, v, base, parent, len, k[base + parent], v[base + parent]);
                if (parent == 0) break;
            }
        }
        for (int last = len; last > 1;) {
            --last;
            const u32 vk = k[base + last], vv = v[base + last];
            k[base + last] = k[base];
            v[base + last] = v[base];
            adjust_heap(k, v, base, 0, last, vk, vv);
        }
    }
}

// __final_insertion_sort: within every leaf a stable insertion sort (all keys of an earlier leaf are
// <= all keys of a later one, so no element crosses a leaf boundary)
__global__ void __launch_bounds__(256) k_tie_leaf(u32* __restrict__ k, u32* __restrict__ v, const int* __restrict__ cnt,
                                                  const int2* __restrict__ leaf) {
    const int nl = cnt[3];
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nl; q += gridDim.x * blockDim.x) {
        const int f = leaf[q].x, e = leaf[q].y;
        u32 kk[kThreshold], vv[kThreshold];
        const int len = e - f;
#pragma unroll
        for (int i = 0; i < kThreshold; ++i)
            if (i < len) { kk[i] = k[f + i]; vv[i] = v[f + i]; }
        for (int i = 1; i < len; ++i) {
            const u32 ck = kk[i], cv = vv[i];
            int j = i;
            while (j > 0 && ck < kk[j - 1]) {
                kk[j] = kk[j - 1];
                vv[j] = vv[j - 1];
                --j;
            }
            kk[j] = ck;
            vv[j] = cv;
        }
#pragma unroll
        for (int i = 0; i < kThreshold; ++i)
            if (i < len) { k[f + i] = kk[i]; v[f + i] = vv[i]; }
    }
}

__global__ void __launch_bounds__(256) k_tie_copy(const u32* __restrict__ k, const u32* __restrict__ v,
                                                  const int* __restrict__ cnt, u32* __restrict__ ko,
                                                  u32* __restrict__ vo) {
    const int n = (int)((const u32*)cnt)[5];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        ko[i] = k[i];
        vo[i] = v[i];
    }
}

}  // namespace

int tie_alloc(TieSort& t, size_t cap) {
    t.cap = cap;
    t.scap = cap / (kThreshold + 1) + 8;
    int lg = 0;
    while ((cap >> (lg + 1)) > 0) ++lg;
    t.levels = 2 * lg + 2;
#define PF_TALLOC(p, bytes) \
    if (hipMalloc(&(p), (bytes)) != hipSuccess) return PF_ENOMEM;
    PF_TALLOC(t.k, sizeof(u32) * cap);
    PF_TALLOC(t.v, sizeof(u32) * cap);
    PF_TALLOC(t.flag, sizeof(u32) * (cap + 1));
    PF_TALLOC(t.pos, sizeof(u32) * (cap + 1));
    for (int q = 0; q < 3; ++q) PF_TALLOC(t.seg[q], sizeof(int4) * t.scap);
    PF_TALLOC(t.heap, sizeof(int4) * t.scap);
    PF_TALLOC(t.leaf, sizeof(int2) * (cap / 2 + 8));
    PF_TALLOC(t.lp, sizeof(int) * cap);
    PF_TALLOC(t.rq, sizeof(int) * cap);
    PF_TALLOC(t.cnt, sizeof(int) * 8);
#undef PF_TALLOC
    if (hipMemset(t.cnt, 0, sizeof(int) * 8) != hipSuccess) return PF_EHIP;
    return PF_OK;
}

void tie_free(TieSort& t) {
    void* ptrs[] = {t.k, t.v, t.flag, t.pos, t.seg[0], t.seg[1], t.seg[2], t.heap, t.leaf, t.lp, t.rq, t.cnt};
    for (void* p : ptrs) (void)hipFree(p);
    t = TieSort{};
}

void tie_sort_enqueue(TieSort& t, const u32* keys, const u32* vals, const int* d_n, PrimWork& w, hipStream_t s) {
    hipLaunchKernelGGL(k_tie_flags, dim3(256), dim3(256), 0, s, keys, d_n, t.flag);
    scan_exclusive(t.flag, t.pos, d_n, reinterpret_cast<u32*>(t.cnt + 5), w, s);
    hipLaunchKernelGGL(k_tie_scatter, dim3(256), dim3(256), 0, s, keys, vals, d_n, t.pos, t.k, t.v);
    hipLaunchKernelGGL(k_tie_init, dim3(1), dim3(64), 0, s, t.k, t.cnt, t.seg[0], t.leaf);
    for (int lev = 0; lev < t.levels; ++lev) {
        const int cur = lev % 3, nxt = (lev + 1) % 3;
        hipLaunchKernelGGL(k_tie_level, dim3(kTieGrid), dim3(256), 0, s, t.k, t.v, t.cnt, t.seg[cur], t.seg[nxt], cur,
                           t.heap, t.leaf, t.lp, t.rq);
    }
    hipLaunchKernelGGL(k_tie_heap, dim3(64), dim3(64), 0, s, t.k, t.v, t.cnt, t.heap);
    hipLaunchKernelGGL(k_tie_leaf, dim3(256), dim3(256), 0, s, t.k, t.v, t.cnt, t.leaf);
}

void tie_sort_finish(TieSort& t, u32* keys_out, u32* vals_out, hipStream_t s) {
    hipLaunchKernelGGL(k_tie_copy, dim3(256), dim3(256), 0, s, t.k, t.v, t.cnt, keys_out, vals_out);
}

}  // namespace pf
