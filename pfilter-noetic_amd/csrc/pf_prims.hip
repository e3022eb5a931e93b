// Stable LSD radix sort and exclusive scan over device-resident counts.
//
// Layout: a fixed grid of up to kSortMaxBlocks workgroups; each workgroup owns a contiguous run of
// tiles, so the per-(digit, workgroup) offsets of a digit-major scan give a stable scatter. The
// effective grid shrinks with n (read on the device), so small inputs touch only a few workgroups.
#include "pf_prims.h"

namespace pf {

namespace {

__device__ __forceinline__ int eff_blocks(int n, int tile) {
    int nt = (n + tile - 1) / tile;
    return nt < kSortMaxBlocks ? nt : kSortMaxBlocks;
}

constexpr int kOsThreads = 256;
constexpr int kOsPer = kSortTile / kOsThreads;   // 8 keys per thread per tile

__global__ void __launch_bounds__(256) k_os_hist(const u32* __restrict__ keys, const int* __restrict__ d_n, int passes,
                                                  u32* __restrict__ bhist, u32* __restrict__ dbase,
                                                  u64* __restrict__ status, u32* __restrict__ tickets) {
    __shared__ u32 lh[4][256];
    __shared__ u32 lw[4];
    __shared__ int last;
    const int n = *d_n;
    const int G = eff_blocks(n, kSortTile);
    const int b = blockIdx.x, t = threadIdx.x;
    const int ntiles = (n + kSortTile - 1) / kSortTile;
    // reset this sort's look-back state (visible to the pass kernels at the kernel boundary)
    for (size_t i = (size_t)b * 256 + t; i < (size_t)passes * ntiles * 256; i += (size_t)gridDim.x * 256)
        status[i] = 0ull;
    if (b >= G) return;
    for (int p = 0; p < 4; ++p) lh[p][t] = 0;
    __syncthreads();
    const int tpb = (ntiles + G - 1) / G;
    const int i0 = b * tpb * kSortTile;
    int i1 = (b + 1) * tpb * kSortTile;
    if (i1 > n) i1 = n;
    for (int i = i0 + t; i < i1; i += 256) {
        const u32 k = keys[i];
        for (int p = 0; p < passes; ++p) atomicAdd(&lh[p][(k >> (8 * p)) & 255u], 1u);
    }
    __syncthreads();
    // add this block's counts into the global histograms (agent-scope atomics), then the last block
    // to arrive forms the exclusive digit bases of every pass and clears the histograms for the next
    // sort (agent-scope loads / stores; no fence needed: G16 R2)
    for (int p = 0; p < passes; ++p)
        if (lh[p][t]) __hip_atomic_fetch_add(&bhist[p * 256 + t], lh[p][t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        const u32 tk = __hip_atomic_fetch_add(&tickets[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = tk == (u32)G - 1 ? 1 : 0;
    }
    __syncthreads();
    if (!last) return;
    u32 c[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
        c[p] = p < passes ? __hip_atomic_load(&bhist[p * 256 + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
    for (int p = 0; p < 4; ++p)
        if (p < passes) __hip_atomic_store(&bhist[p * 256 + t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int p = 0; p < passes; ++p) {
        u32 tot;
        dbase[p * 256 + t] = block_excl_scan256(c[p], lw, tot);
    }
    if (t == 0) __hip_atomic_store(&tickets[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One pass. Blocks own tiles b, b + G, ... (G <= kSortMaxBlocks co-resident blocks), so a tile's
// look-back only waits on tiles of running blocks. Inside a tile, wave w owns the contiguous 512
// keys w * 512 .. (lane l of round u: key w * 512 + 64 u + l), so the waves rank independently: a
// key's rank among equal digits of its wave is the wave's running count of that digit (a wave-
// private LDS row, updated by one leader lane per digit and round) plus the equal lanes below it;
// one block barrier then turns the four waves' digit counts into per-wave offsets. Stable: keys keep
// their index order within a digit. Two barriers per tile instead of four per round.
__global__ void __launch_bounds__(256) k_os_pass(const u32* __restrict__ kin, const u32* __restrict__ vin,
                                                         u32* __restrict__ kout, u32* __restrict__ vout,
                                                         const int* __restrict__ d_n, int pass,
                                                         const u32* __restrict__ dbase_g, u64* __restrict__ status,
                                                         int* __restrict__ err) {
    __shared__ u32 wcnt[4][256];                 // per wave: running digit counts, then its offsets
    __shared__ u32 off[256];
    const int n = *d_n;
    const int ntiles = (n + kSortTile - 1) / kSortTile;
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    if ((int)blockIdx.x >= ntiles) return;
    const int shift = 8 * pass;
    u64* st = status + (size_t)pass * ntiles * 256;
    const u32 dbase = dbase_g[pass * 256 + t];
    const u64 lt = lanemask_lt();
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int i0 = tile * kSortTile + w * (kSortTile / 4);
        u32 key[kOsPer], val[kOsPer], rk[kOsPer];
#pragma unroll
        for (int r = 0; r < kOsPer; ++r) {                      // the whole tile in flight at once
            const int i = i0 + r * 64 + l;
            key[r] = i < n ? kin[i] : 0xFFFFFFFFu;
            val[r] = i < n ? vin[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) wcnt[w][l + 64 * k] = 0;   // this wave's row only
#pragma unroll
        for (int r = 0; r < kOsPer; ++r) {
            const bool valid = i0 + r * 64 + l < n;
            const u32 d = (key[r] >> shift) & 255u;
            const u64 peers = match_bits(d, 8, valid);
            const u32 below = (u32)__popcll(peers & lt);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous round's leader updates
            const u32 run = valid ? wcnt[w][d] : 0u;
            rk[r] = valid ? run + below : 0xFFFFFFFFu;
            if (valid && below == 0) wcnt[w][d] = run + (u32)__popcll(peers);
        }
        __syncthreads();
        {   // digit t: the waves' counts -> per-wave exclusive offsets, the tile's count -> look-back
            u32 a = 0;
#pragma unroll
            for (int ww = 0; ww < 4; ++ww) {
                const u32 c = wcnt[ww][t];
                wcnt[ww][t] = a;
                a += c;
            }
            const u32 cnt = a;
            u64* mine = st + (size_t)tile * 256 + t;
            u32 excl = 0;
            if (tile > 0) {
                __hip_atomic_store(mine, (1ull << 32) | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                int j = tile - 1;
                unsigned long long t0 = 0;
                for (;;) {
                    const u64 v = __hip_atomic_load(st + (size_t)j * 256 + t, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
                    const u32 tag = (u32)(v >> 32);
                    if (tag == 0) {
                        const unsigned long long now = rt_now();
                        if (!t0) t0 = now;
                        else if (now - t0 > kWaitTicks) { atomicOr(err, 1); break; }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    excl += (u32)v;
                    if (tag == 2 || j == 0) break;
                    --j;
                }
            }
            __hip_atomic_store(mine, (2ull << 32) | (excl + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            off[t] = dbase + excl;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kOsPer; ++r) {
            if (rk[r] == 0xFFFFFFFFu) continue;
            const u32 d = (key[r] >> shift) & 255u;
            const u32 pos = off[d] + wcnt[w][d] + rk[r];
            kout[pos] = key[r];
            vout[pos] = val[r];
        }
        __syncthreads();
    }
}

constexpr int kScanPer = 8;

// PER items per thread, tiles of 256 * PER items (PER = 8: 2048, the sort tile; the cell-count scans
// of the kNN grids use 32: a few hundred tiles over a grid of up to 256 workgroups, so a workgroup
// scans about one tile with all of its loads in flight instead of a chain of look-backs)
template <int PER>
__global__ void __launch_bounds__(256) k_scan1(const u32* __restrict__ in, u32* __restrict__ out,
                                                const int* __restrict__ d_n, u32* __restrict__ d_total,
                                                u64* __restrict__ status, u32* __restrict__ arrive,
                                                int* __restrict__ err) {
    constexpr int kTile = 256 * PER;
    __shared__ u32 lw[4];
    __shared__ u32 s_excl;
    const int n = *d_n;
    const int ntiles = (n + kTile - 1) / kTile;
    const int t = threadIdx.x;
    const int G = ntiles < (int)gridDim.x ? ntiles : (int)gridDim.x;
    if (n == 0) {
        if (blockIdx.x == 0 && t == 0 && d_total) *d_total = 0u;
        return;
    }
    if ((int)blockIdx.x >= G) return;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int base = tile * kTile + t * PER;
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
        u32 sum = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) sum += v[k];
        u32 agg;
        const u32 tex = block_excl_scan256(sum, lw, agg);
        if (t < 64) {
            const u32 excl = tile_lookback(status, tile, agg, err);
            if (t == 0) {
                s_excl = excl;
                if (tile == ntiles - 1 && d_total) *d_total = excl + agg;
            }
        }
        __syncthreads();
        u32 r = s_excl + tex;
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
        __syncthreads();
    }
    lookback_finish(status, ntiles, arrive, G);
}

// Segments of sorted keys (bit 31 = cloud, 0xFFFFFFFF = dropped): segment starts, the number of
// segments, the number of cloud-0 segments and the number of non-sentinel keys, in one pass.
__global__ void __launch_bounds__(256) k_segments(const u32* __restrict__ keys, const int* __restrict__ d_n,
                                                   u32* __restrict__ segstart, int* __restrict__ d_nseg,
                                                   int* __restrict__ d_nlt, int* __restrict__ d_nvalid,
                                                   u64* __restrict__ status, u32* __restrict__ arrive,
                                                   int* __restrict__ err) {
    constexpr u32 kSent = 0xFFFFFFFFu;
    __shared__ u32 lw[4];
    __shared__ u32 s_excl;
    const int n = *d_n;
    const int ntiles = (n + kSortTile - 1) / kSortTile;
    const int t = threadIdx.x;
    const int G = ntiles < (int)gridDim.x ? ntiles : (int)gridDim.x;
    if (n == 0) {
        if (blockIdx.x == 0 && t == 0) { *d_nseg = 0; d_nlt[0] = d_nlt[1] = d_nlt[2] = 0; *d_nvalid = 0; }
        return;
    }
    if ((int)blockIdx.x >= G) return;
    if (blockIdx.x == 0 && t == 0) {                            // cases without an interior boundary
        const u32 k0 = keys[0], kl = keys[n - 1];
        if (k0 == kSent) *d_nvalid = 0;
        for (u32 b = 1; b <= 3; ++b)                            // classes below the first key's: none
            if ((k0 >> 30) >= b) d_nlt[b - 1] = 0;
        if (kl != kSent) *d_nvalid = n;
    }
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int base = tile * kSortTile + t * kScanPer;
        u32 k[kScanPer + 1];                                    // k[0] = predecessor of the first
        k[0] = base > 0 && base - 1 < n ? keys[base - 1] : kSent;
#pragma unroll
        for (int j = 0; j < kScanPer; ++j) k[j + 1] = base + j < n ? keys[base + j] : kSent;
        u32 sum = 0;
#pragma unroll
        for (int j = 0; j < kScanPer; ++j) {
            const bool head = base + j < n && k[j + 1] != kSent && (base + j == 0 || k[j] != k[j + 1]);
            sum += head ? 1u : 0u;
        }
        u32 agg;
        const u32 tex = block_excl_scan256(sum, lw, agg);
        if (t < 64) {
            const u32 excl = tile_lookback(status, tile, agg, err);
            if (t == 0) {
                s_excl = excl;
                if (tile == ntiles - 1) {
                    *d_nseg = (int)(excl + agg);
                    for (u32 b = 1; b <= 3; ++b)                // classes above the last key's: all
                        if ((keys[n - 1] >> 30) < b) d_nlt[b - 1] = (int)(excl + agg);
                }
            }
        }
        __syncthreads();
        u32 sid = s_excl + tex;                                 // segments before element base + j
#pragma unroll
        for (int j = 0; j < kScanPer; ++j) {
            const int i = base + j;
            if (i >= n) break;
            const u32 kp = k[j], kc = k[j + 1];
            if (i > 0 && (kp >> 30) < (kc >> 30))              // class boundary: segments before it
                for (u32 b = (kp >> 30) + 1; b <= (kc >> 30); ++b) d_nlt[b - 1] = (int)sid;
            if (i > 0 && kp != kSent && kc == kSent) *d_nvalid = i;
            if (kc != kSent && (i == 0 || kp != kc)) segstart[sid++] = (u32)i;
        }
        __syncthreads();
    }
    lookback_finish(status, ntiles, arrive, G);
}

}  // namespace

int prim_alloc(PrimWork& w, size_t cap, size_t scan_cap) {
    if (scan_cap < cap) scan_cap = cap;
    w.cap = cap;
    w.max_tiles = (cap + kSortTile - 1) / kSortTile;
    w.scan_tiles = (scan_cap + kSortTile - 1) / kSortTile;
    if (hipMalloc(&w.keys_tmp, sizeof(u32) * (cap + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&w.vals_tmp, sizeof(u32) * (cap + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&w.bhist, sizeof(u32) * 4 * 256) != hipSuccess) return PF_ENOMEM;
    if (hipMemset(w.bhist, 0, sizeof(u32) * 4 * 256) != hipSuccess) return PF_EHIP;
    if (hipMalloc(&w.status, sizeof(u64) * 4 * w.max_tiles * 256) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&w.tickets, sizeof(u32) * 8) != hipSuccess) return PF_ENOMEM;
    if (hipMemset(w.tickets, 0, sizeof(u32) * 8) != hipSuccess) return PF_EHIP;
    if (hipMalloc(&w.dbase, sizeof(u32) * 4 * 256) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&w.scan_status, sizeof(u64) * (w.scan_tiles + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMemset(w.scan_status, 0, sizeof(u64) * (w.scan_tiles + 1)) != hipSuccess) return PF_EHIP;
    if (hipMalloc(&w.err, sizeof(int)) != hipSuccess) return PF_ENOMEM;
    if (hipMemset(w.err, 0, sizeof(int)) != hipSuccess) return PF_EHIP;
    return PF_OK;
}

void prim_free(PrimWork& w) {
    (void)hipFree(w.keys_tmp);
    (void)hipFree(w.vals_tmp);
    (void)hipFree(w.bhist);
    (void)hipFree(w.status);
    (void)hipFree(w.tickets);
    (void)hipFree(w.dbase);
    (void)hipFree(w.scan_status);
    (void)hipFree(w.err);
    w = PrimWork{};
}

void radix_sort_pairs(u32* keys, u32* vals, const int* d_n, int bits, PrimWork& w, hipStream_t s, u32** kout,
                      u32** vout, bool hist_fused) {
    const int passes = radix_passes(bits, !kout);   // without kout the result goes back in place
    if (!hist_fused) hipLaunchKernelGGL(k_os_hist, dim3(kSortMaxBlocks), dim3(256), 0, s, keys, d_n, passes, w.bhist, w.dbase,
                       w.status, w.tickets);
    const unsigned grid = (unsigned)(w.max_tiles < (size_t)kSortMaxBlocks ? w.max_tiles : kSortMaxBlocks);
    u32 *ka = keys, *va = vals, *kb = w.keys_tmp, *vb = w.vals_tmp;
    for (int p = 0; p < passes; ++p) {
        hipLaunchKernelGGL(k_os_pass, dim3(grid), dim3(kOsThreads), 0, s, ka, va, kb, vb, d_n, p, w.dbase, w.status,
                           w.err);
        u32* t;
        t = ka; ka = kb; kb = t;
        t = va; va = vb; vb = t;
    }
    if (kout) *kout = ka;
    if (vout) *vout = va;
}

void segment_starts(const u32* keys, const int* d_n, u32* segstart, int* d_nseg, int* d_nlt, int* d_nvalid,
                    PrimWork& w, hipStream_t s) {
    const unsigned grid = (unsigned)(w.scan_tiles < (size_t)kSortMaxBlocks ? w.scan_tiles : kSortMaxBlocks);
    hipLaunchKernelGGL(k_segments, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, keys, d_n, segstart, d_nseg, d_nlt,
                       d_nvalid, w.scan_status, w.tickets + 5, w.err);
}

void scan_exclusive(const u32* in, u32* out, const int* d_n, u32* d_total, PrimWork& w, hipStream_t s, bool wide) {
    const unsigned grid = (unsigned)(w.scan_tiles < (size_t)kSortMaxBlocks ? w.scan_tiles : kSortMaxBlocks);
    if (wide)   // in and out 16-byte aligned (hipMalloc'd)
        hipLaunchKernelGGL(k_scan1<32>, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, in, out, d_n, d_total,
                           w.scan_status, w.tickets + 5, w.err);
    else
        hipLaunchKernelGGL(k_scan1<kScanPer>, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, in, out, d_n, d_total,
                           w.scan_status, w.tickets + 5, w.err);
}

}  // namespace pf
