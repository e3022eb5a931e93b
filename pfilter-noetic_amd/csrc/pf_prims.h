// Device-wide primitives with device-resident element counts (no host round trip).
#pragma once
#include "pf_common.h"

namespace pf {

constexpr int kSortMaxBlocks = 256;   // max workgroups of the sort / scan grids
constexpr int kSortTile = 2048;       // keys per tile (256 threads x 8)

struct PrimWork {
    u32* keys_tmp = nullptr;   // cap
    u32* vals_tmp = nullptr;   // cap
    u32* bhist = nullptr;      // [4 passes][256] global digit counts (zero between sorts)
    u64* status = nullptr;     // [4 passes][max_tiles][256] look-back words
    u32* tickets = nullptr;    // [8]: [4] histogram arrivals, [5] scan arrivals
    u32* dbase = nullptr;      // [4 passes][256] exclusive digit bases
    u64* scan_status = nullptr;// [max_tiles] scan look-back words (zero between calls)
    int* err = nullptr;        // look-back spin limit hit (never expected)
    size_t cap = 0, max_tiles = 0, scan_tiles = 0;
};

// cap: largest sort; scan_cap: largest scan (defaults to cap)
int prim_alloc(PrimWork& w, size_t cap, size_t scan_cap = 0);
void prim_free(PrimWork& w);

// Stable sort of (keys, vals)[0 .. *d_n) by the low `bits` bits of keys (8-bit digits). With kout/vout
// null the pass count is rounded up to even so the result is back in keys/vals; otherwise *kout/*vout
// name the buffers holding the result (keys/vals or the PrimWork scratch). hist_fused: the kernel
// that produced the keys already ran the histogram prologue below (sort_hist_*), so the separate
// histogram launch is skipped.
void radix_sort_pairs(u32* keys, u32* vals, const int* d_n, int bits, PrimWork& w, hipStream_t s,
                      u32** kout = nullptr, u32** vout = nullptr, bool hist_fused = false);
inline int radix_passes(int bits, bool in_place) {
    int p = (bits + 7) / 8;
    if (p < 1) p = 1;
    if (p > 4) p = 4;
    if (in_place && (p & 1)) ++p;
    return p;
}

// exclusive scan across a 256-thread block; returns this thread's exclusive prefix
__device__ __forceinline__ u32 wave_incl_scan_u32(u32 v) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        u32 t = __shfl_up(v, o, 64);
        if (l >= o) v += t;
    }
    return v;
}
__device__ __forceinline__ u32 block_excl_scan256(u32 v, u32* lds_w, u32& total) {
    const int w = threadIdx.x >> 6, l = lane_id();
    u32 inc = wave_incl_scan_u32(v);
    if (l == 63) lds_w[w] = inc;
    __syncthreads();
    u32 off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        u32 t = lds_w[i];
        if (i < w) off += t;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return off + inc - v;
}

// ---- single-pass scans: decoupled look-back ----
// Blocks own 2048-item tiles b, b + G, ... (co-resident grid). A tile publishes its aggregate, wave 0
// looks back over up to 64 predecessors at once (agent-scope atomic words carrying tag << 32 |
// value), then publishes its inclusive prefix. The last block to finish clears the status words for
// the next call.
// wave 0 (all 64 lanes): publish `agg` for `tile`, return its exclusive prefix (all lanes)
__device__ __forceinline__ u32 tile_lookback(u64* status, int tile, u32 agg, int* err) {
    const int l = lane_id();
    if (l == 0 && tile > 0)
        __hip_atomic_store(&status[tile], (1ull << 32) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u32 excl = 0;
    int j = tile - 1;
    unsigned long long t0 = 0;
    while (j >= 0) {
        const int jj = j - l;
        const u64 sv = jj >= 0 ? __hip_atomic_load(&status[jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : (2ull << 32);                // before tile 0: an inclusive zero
        const u32 tag = (u32)(sv >> 32);
        const u64 incl = __ballot(tag == 2);
        const int first = incl ? __ffsll((long long)incl) - 1 : 64;       // nearest inclusive prefix
        const u64 upto = first >= 63 ? ~0ull : ((2ull << first) - 1);
        if (__ballot(tag == 0) & upto) {
            const unsigned long long now = rt_now();
            if (!t0) t0 = now;
            else if (now - t0 > kWaitTicks) { if (l == 0) atomicOr(err, 2); break; }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        u32 mine = (l <= first && jj >= 0) ? (u32)sv : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
        excl += mine;
        if (first < 64) break;
        j -= 64;
    }
    if (l == 0)
        __hip_atomic_store(&status[tile], (2ull << 32) | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// the last block of a look-back launch clears the status words and the arrival counter
__device__ __forceinline__ void lookback_finish(u64* status, int ntiles, u32* arrive, int G) {
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (u32)G - 1;
    __syncthreads();
    if (!last) return;
    for (int i = threadIdx.x; i < ntiles; i += blockDim.x)
        __hip_atomic_store(&status[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Histogram prologue fused into the kernel that writes a sort's keys (256-thread blocks; every block
// of the grid must reach sort_hist_end): per-block digit counts of every pass in LDS, added to the
// global counts; the last block to arrive forms the exclusive digit bases and resets the counts;
// every block clears its share of the pass kernels' look-back words.
struct SortHist {
    u32* ghist;     // [4][256], zero between sorts
    u32* dbase;     // [4][256]
    u64* status;    // [passes][ntiles][256]
    u32* arrive;
    int passes;
};
inline SortHist sort_hist(PrimWork& w, int bits, bool in_place) {
    return SortHist{w.bhist, w.dbase, w.status, w.tickets + 4, radix_passes(bits, in_place)};
}
__device__ __forceinline__ void sort_hist_begin(u32 (*lh)[256]) {
#pragma unroll
    for (int p = 0; p < 4; ++p) lh[p][threadIdx.x] = 0u;
    __syncthreads();
}
__device__ __forceinline__ void sort_hist_add(u32 (*lh)[256], u32 key, int passes) {
    for (int p = 0; p < passes; ++p) atomicAdd(&lh[p][(key >> (8 * p)) & 255u], 1u);
}
// items: the producer's grid-stride item count; blocks beyond ceil(items / 256) hold no keys and
// leave at once (only the others count as arrivals)
__device__ __forceinline__ int sort_hist_blocks(int items) {
    const int b = (items + 255) / 256;
    return b < (int)gridDim.x ? b : (int)gridDim.x;
}
__device__ __forceinline__ void sort_hist_end(u32 (*lh)[256], const SortHist& sh, int n, int items) {
    __shared__ u32 lw[4];
    __shared__ int last;
    const int t = threadIdx.x;
    const int G = sort_hist_blocks(items);
    if ((int)blockIdx.x >= G) return;
    const int ntiles = (n + kSortTile - 1) / kSortTile;
    for (size_t i = (size_t)blockIdx.x * 256 + t; i < (size_t)sh.passes * ntiles * 256; i += (size_t)G * 256)
        sh.status[i] = 0ull;
    __syncthreads();
    for (int p = 0; p < sh.passes; ++p)
        if (lh[p][t]) __hip_atomic_fetch_add(&sh.ghist[p * 256 + t], lh[p][t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) last = __hip_atomic_fetch_add(sh.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (u32)G - 1;
    __syncthreads();
    if (!last) return;
    u32 c[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
        c[p] = p < sh.passes ? __hip_atomic_load(&sh.ghist[p * 256 + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
    for (int p = 0; p < 4; ++p)
        if (p < sh.passes) __hip_atomic_store(&sh.ghist[p * 256 + t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int p = 0; p < sh.passes; ++p) {
        u32 tot;
        sh.dbase[p * 256 + t] = block_excl_scan256(c[p], lw, tot);
    }
    if (t == 0) __hip_atomic_store(sh.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Segments of stably sorted keys (bits 30-31 = cloud class 0..2, 0xFFFFFFFF = dropped entries, sorted
// last): segstart[s] = first index of segment s; *d_nseg = number of segments; d_nlt[b - 1] = segments
// of classes < b (b = 1, 2, 3); *d_nvalid = number of non-sentinel keys.
void segment_starts(const u32* keys, const int* d_n, u32* segstart, int* d_nseg, int* d_nlt, int* d_nvalid,
                    PrimWork& w, hipStream_t s);

// out[i] = sum(in[0..i)) for i < *d_n; *d_total = sum(in[0..n)) when d_total != nullptr. wide: tiles of
// 8192 items (32 per thread, 16-byte loads and stores; in / out 16-byte aligned) for long scans.
void scan_exclusive(const u32* in, u32* out, const int* d_n, u32* d_total, PrimWork& w, hipStream_t s,
                    bool wide = false);

}  // namespace pf
