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

__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        u32 t = __shfl_up(v, o, 64);
        if (l >= o) v += t;
    }
    return v;
}

// exclusive scan across a 256-thread block; returns this thread's exclusive prefix
__device__ __forceinline__ u32 block_excl_scan256(u32 v, u32* lds_w, u32& total) {
    const int w = threadIdx.x >> 6, l = lane_id();
    u32 inc = wave_incl_scan(v);
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

__global__ void __launch_bounds__(256) k_rs_hist(const u32* __restrict__ keys, const int* __restrict__ d_n, int shift,
                                                  u32* __restrict__ hist) {
    __shared__ u32 lh[256];
    const int n = *d_n;
    const int G = eff_blocks(n, kSortTile);
    const int b = blockIdx.x;
    if (b >= G) return;
    const int nt = (n + kSortTile - 1) / kSortTile;
    const int tpb = (nt + G - 1) / G;
    const int i0 = b * tpb * kSortTile;
    int i1 = (b + 1) * tpb * kSortTile;
    if (i1 > n) i1 = n;
    lh[threadIdx.x] = 0;
    __syncthreads();
    for (int i = i0 + threadIdx.x; i < i1; i += 256) atomicAdd(&lh[(keys[i] >> shift) & 255u], 1u);
    __syncthreads();
    hist[threadIdx.x * kSortMaxBlocks + b] = lh[threadIdx.x];
}

// exclusive scan of hist in (digit, block) order, in place
__global__ void __launch_bounds__(1024) k_rs_scan(u32* __restrict__ hist, const int* __restrict__ d_n) {
    __shared__ u32 lw[16];
    const int n = *d_n;
    const int G = eff_blocks(n, kSortTile);
    if (G == 0) return;
    const int total = 256 * G;
    const int per = (total + 1023) / 1024;
    const int t = threadIdx.x;
    const int e0 = t * per;
    u32 s = 0;
    for (int e = e0; e < e0 + per && e < total; ++e) s += hist[(e / G) * kSortMaxBlocks + (e % G)];
    // block scan of s (16 waves)
    const int w = t >> 6, l = lane_id();
    u32 inc = wave_incl_scan(s);
    if (l == 63) lw[w] = inc;
    __syncthreads();
    u32 off = 0;
    for (int i = 0; i < w; ++i) off += lw[i];
    u32 run = off + inc - s;
    for (int e = e0; e < e0 + per && e < total; ++e) {
        u32* p = &hist[(e / G) * kSortMaxBlocks + (e % G)];
        u32 c = *p;
        *p = run;
        run += c;
    }
}

__global__ void __launch_bounds__(256) k_rs_scatter(const u32* __restrict__ kin, const u32* __restrict__ vin,
                                                     u32* __restrict__ kout, u32* __restrict__ vout,
                                                     const int* __restrict__ d_n, int shift,
                                                     const u32* __restrict__ hist) {
    __shared__ u32 run[256];
    __shared__ u32 wcnt[4][256];
    const int n = *d_n;
    const int G = eff_blocks(n, kSortTile);
    const int b = blockIdx.x;
    if (b >= G) return;
    const int t = threadIdx.x, w = t >> 6, l = lane_id();
    const int nt = (n + kSortTile - 1) / kSortTile;
    const int tpb = (nt + G - 1) / G;
    const int i0 = b * tpb * kSortTile;
    int i1 = (b + 1) * tpb * kSortTile;
    if (i1 > n) i1 = n;
    run[t] = hist[t * kSortMaxBlocks + b];
    const u64 lt = lanemask_lt();
    for (int base = i0; base < i1; base += 256) {
        const int i = base + t;
        const bool valid = i < i1;
        const u32 key = valid ? kin[i] : 0u;
        const u32 val = valid ? vin[i] : 0u;
        const u32 d = (key >> shift) & 255u;
        wcnt[w][l] = 0; wcnt[w][l + 64] = 0; wcnt[w][l + 128] = 0; wcnt[w][l + 192] = 0;
        __syncthreads();
        const u64 peers = match_bits(d, 8, valid);
        const u32 rank = (u32)__popcll(peers & lt);
        if (valid && rank == 0) wcnt[w][d] = (u32)__popcll(peers);
        __syncthreads();
        {
            u32 r = run[t];
            for (int ww = 0; ww < 4; ++ww) {
                u32 c = wcnt[ww][t];
                wcnt[ww][t] = r;
                r += c;
            }
            run[t] = r;
        }
        __syncthreads();
        if (valid) {
            const u32 pos = wcnt[w][d] + rank;
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
    }
}

// ---- exclusive scan ----
__global__ void __launch_bounds__(256) k_sc_reduce(const u32* __restrict__ in, const int* __restrict__ d_n,
                                                    u32* __restrict__ partials) {
    __shared__ u32 lw[4];
    const int n = *d_n;
    const int G = eff_blocks(n, kScanTile);
    const int b = blockIdx.x;
    if (b >= G) return;
    const int nt = (n + kScanTile - 1) / kScanTile;
    const int tpb = (nt + G - 1) / G;
    const int i0 = b * tpb * kScanTile;
    int i1 = (b + 1) * tpb * kScanTile;
    if (i1 > n) i1 = n;
    u32 s = 0;
    for (int i = i0 + threadIdx.x; i < i1; i += 256) s += in[i];
    u32 tot;
    block_excl_scan256(s, lw, tot);
    if (threadIdx.x == 0) partials[b] = tot;
}

__global__ void __launch_bounds__(256) k_sc_top(u32* __restrict__ partials, const int* __restrict__ d_n,
                                                 u32* __restrict__ d_total) {
    __shared__ u32 lw[4];
    const int n = *d_n;
    const int G = eff_blocks(n, kScanTile);
    const int t = threadIdx.x;
    u32 v = t < G ? partials[t] : 0u;   // G <= 256
    u32 tot;
    u32 ex = block_excl_scan256(v, lw, tot);
    if (t < G) partials[t] = ex;
    if (t == 0 && d_total) *d_total = tot;
}

__global__ void __launch_bounds__(256) k_sc_down(const u32* __restrict__ in, u32* __restrict__ out,
                                                  const int* __restrict__ d_n, const u32* __restrict__ partials) {
    __shared__ u32 lw[4];
    const int n = *d_n;
    const int G = eff_blocks(n, kScanTile);
    const int b = blockIdx.x;
    if (b >= G) return;
    const int nt = (n + kScanTile - 1) / kScanTile;
    const int tpb = (nt + G - 1) / G;
    const int i0 = b * tpb * kScanTile;
    int i1 = (b + 1) * tpb * kScanTile;
    if (i1 > n) i1 = n;
    u32 run = partials[b];
    const int t = threadIdx.x;
    for (int base = i0; base < i1; base += kScanTile) {
        u32 v[4];
        u32 s = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = base + 4 * t + k;
            v[k] = i < i1 ? in[i] : 0u;
            s += v[k];
        }
        u32 tot;
        u32 ex = block_excl_scan256(s, lw, tot);
        u32 r = run + ex;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = base + 4 * t + k;
            if (i < i1) out[i] = r;
            r += v[k];
        }
        run += tot;
    }
}

}  // namespace

int prim_alloc(PrimWork& w, size_t cap) {
    w.cap = cap;
    if (hipMalloc(&w.hist, sizeof(u32) * 256 * kSortMaxBlocks) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&w.partials, sizeof(u32) * (kSortMaxBlocks + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&w.keys_tmp, sizeof(u32) * (cap + 1)) != hipSuccess) return PF_ENOMEM;
    if (hipMalloc(&w.vals_tmp, sizeof(u32) * (cap + 1)) != hipSuccess) return PF_ENOMEM;
    return PF_OK;
}

void prim_free(PrimWork& w) {
    (void)hipFree(w.hist);
    (void)hipFree(w.partials);
    (void)hipFree(w.keys_tmp);
    (void)hipFree(w.vals_tmp);
    w = PrimWork{};
}

void radix_sort_pairs(u32* keys, u32* vals, const int* d_n, int bits, PrimWork& w, hipStream_t s) {
    int passes = (bits + 7) / 8;
    if (passes & 1) ++passes;
    if (passes > 4) passes = 4;
    u32 *ka = keys, *va = vals, *kb = w.keys_tmp, *vb = w.vals_tmp;
    for (int p = 0; p < passes; ++p) {
        const int shift = 8 * p;
        hipLaunchKernelGGL(k_rs_hist, dim3(kSortMaxBlocks), dim3(256), 0, s, ka, d_n, shift, w.hist);
        hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, s, w.hist, d_n);
        hipLaunchKernelGGL(k_rs_scatter, dim3(kSortMaxBlocks), dim3(256), 0, s, ka, va, kb, vb, d_n, shift, w.hist);
        u32* t;
        t = ka; ka = kb; kb = t;
        t = va; va = vb; vb = t;
    }
}

void scan_exclusive(const u32* in, u32* out, const int* d_n, u32* d_total, PrimWork& w, hipStream_t s) {
    hipLaunchKernelGGL(k_sc_reduce, dim3(kSortMaxBlocks), dim3(256), 0, s, in, d_n, w.partials);
    hipLaunchKernelGGL(k_sc_top, dim3(1), dim3(256), 0, s, w.partials, d_n, d_total);
    hipLaunchKernelGGL(k_sc_down, dim3(kSortMaxBlocks), dim3(256), 0, s, in, out, d_n, w.partials);
}

}  // namespace pf
