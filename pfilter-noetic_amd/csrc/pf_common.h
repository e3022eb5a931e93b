// Common device/host helpers for the MI355X (gfx950) odometry path.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../../include/pfilter_hip.h"

#define PF_HIP_TRY(expr)                                                                      \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            std::fprintf(stderr, "pfilter_hip: %s failed: %s (%s:%d)\n", #expr,               \
                         hipGetErrorString(_e), __FILE__, __LINE__);                          \
            return PF_EHIP;                                                                   \
        }                                                                                     \
    } while (0)

namespace pf {

constexpr int kWave = 64;
typedef unsigned long long u64;
typedef uint32_t u32;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ u64 lanemask_lt() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}
// mask of active lanes whose `v` (first `bits` bits) equals this lane's
__device__ __forceinline__ u64 match_bits(u32 v, int bits, bool active) {
    u64 m = __ballot(active);
#pragma unroll
    for (int b = 0; b < 32; ++b) {
        if (b >= bits) break;
        const bool bit = (v >> b) & 1u;
        const u64 bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

// float <-> order-preserving uint (for atomic min/max on floats)
__device__ __forceinline__ u32 f2ord(float f) {
    u32 u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(u32 u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// XCD-aware block order. The dispatcher deals workgroups to the 8 XCDs round-robin (block b runs on
// XCD b % 8), and each XCD has its own L2. Renumbering so that XCD x owns one contiguous range of
// logical blocks keeps neighbouring work (spatially adjacent queries) inside one L2. Bijective for
// any grid size: XCD x owns q + (x < r) blocks, q = n / 8, r = n % 8.
constexpr int kXcds = 8;
__device__ __forceinline__ unsigned xcd_block(unsigned b, unsigned n) {
    const unsigned q = n / kXcds, r = n % kXcds, x = b % kXcds, l = b / kXcds;
    return x * q + (x < r ? x : r) + l;
}

// map point packing: float4(x, y, z, bits(r | g << 8))
__device__ __host__ __forceinline__ u32 pack_rg(u32 r, u32 g) { return (r & 255u) | ((g & 255u) << 8); }

// Bounded device waits: a wait that has not completed after kWaitTicks of the 100 MHz real-time
// counter (0.25 s, about 10^4 times the longest wait ever measured) gives up and latches a sticky
// error word instead of hanging the queue.
constexpr unsigned long long kWaitTicks = 25000000ull;
__device__ __forceinline__ unsigned long long rt_now() { return __builtin_amdgcn_s_memrealtime(); }

}  // namespace pf
