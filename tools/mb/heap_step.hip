// Microbenchmark: cycles per step of the pieces of a pipelined heap pop step in one wave (gfx950). Every lane
// walks a hole down a static heap of n entries in LDS and restarts at the root at the bottom, so each
// variant runs the same dependent chain shape as __sort_heap's pops; s_memtime brackets STEPS steps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb/heap_step.hip -o tools/mb/heap_step && tools/mb/heap_step
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32;
typedef unsigned long long u64;
constexpr int N = 16384, STEPS = 8192;

__device__ __forceinline__ bool anc_or_self(int x, int q) {
    const int sh = __clz(x + 1) - __clz(q + 1);
    return sh >= 0 && ((q + 1) >> sh) == x + 1;
}

template <int V>
__global__ void __launch_bounds__(64) k_step(u64* out, int lanes) {
    __shared__ uint2 H[N + 80];
    const int l = threadIdx.x;
    for (int i = l; i < N + 80; i += 64) H[i] = make_uint2((u32)i, i < N ? (u32)(N - i + (i * 7919u) % 5u) : 0u);
    __syncthreads();
    const int spare = N + 2 + l;
    int h = l < lanes ? (l * 37) % 64 : spare;
    uint2 v = make_uint2(0u, (u32)(l * 13 % 50) + 1u);
    const u32 nb = (u32)N * 8u;
    char* Hb = reinterpret_cast<char*>(H);
    int nxt = 0, since = 2;
    bool blk = false;
    u32 acc = 0;
    u64 t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < STEPS; ++it) {
        if (V == 4) {                                             // eligibility + ancestor test + ballot
            if (since >= 2 && nxt < 1000000) {
                const int q = N - 1 - (nxt & 1023);
                const bool b2 = anc_or_self(h, q);
                if (__ballot(b2) == 0) { ++nxt; since = 0; }
            }
            ++since;
        }
        const u32 ca = min((u32)h * 16u + 8u, nb);
        const uint2 a = *reinterpret_cast<const uint2*>(Hb + ca);
        const uint2 b = *reinterpret_cast<const uint2*>(Hb + ca + 8u);
        uint2 x1 = make_uint2(0u, 0u), x2 = make_uint2(0u, 0u);
        if (V == 5 || V == 6) x1 = H[N - 1 - (it & 1023)];
        if (V == 5) x2 = H[0];
        const bool right = !(b.y < a.y);
        const uint2 ch = right ? b : a;
        acc += x1.x + x2.y;
        if (V == 0) {                                             // read2 + select, no write
            acc += ch.x;
            h = 2 * h + 1 + (right ? 1 : 0);
            h = h < N ? h : 0;
        } else {
            const bool stop = V >= 2 ? ch.y < v.y : false;
            H[h] = stop ? v : ch;
            asm volatile("" ::: "memory");
            h = stop ? 0 : 2 * h + 1 + (right ? 1 : 0);
            h = h < N ? h : 0;
        }
        if (V == 8 && l == (it & 63) && (it % 3) == 0) {        // a start's writes, exec-masked
            H[N + 1 + 64] = ch;
            out[8 + l] = ((u64)ch.y << 32) | ch.x;
        }
        if ((V >= 3 && V <= 6) && __ballot(h != spare) == 0) break;   // loop control as the pops run it
        if (V >= 7 && (it & 3) == 3 && __ballot(h != spare) == 0) break;   // ... every fourth step
    }
    u64 t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) out[V] = t1 - t0;
    if (acc == 12345u) out[70] = acc + nxt;
}

int main() {
    u64* d;
    hipMalloc(&d, 128 * 8);
    u64 hv[16];
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_step<0>, 1, 64, 0, 0, d, 16);
        hipLaunchKernelGGL(k_step<1>, 1, 64, 0, 0, d, 16);
        hipLaunchKernelGGL(k_step<2>, 1, 64, 0, 0, d, 16);
        hipLaunchKernelGGL(k_step<3>, 1, 64, 0, 0, d, 16);
        hipLaunchKernelGGL(k_step<4>, 1, 64, 0, 0, d, 16);
        hipLaunchKernelGGL(k_step<5>, 1, 64, 0, 0, d, 16);
        hipLaunchKernelGGL(k_step<6>, 1, 64, 0, 0, d, 16);
        hipLaunchKernelGGL(k_step<7>, 1, 64, 0, 0, d, 16);
        hipLaunchKernelGGL(k_step<8>, 1, 64, 0, 0, d, 16);
        hipDeviceSynchronize();
    }
    hipMemcpy(hv, d, 9 * 8, hipMemcpyDeviceToHost);
    const char* nm[] = {"read2+select (no write)", "+ hole write", "+ stop test on the value", "+ ballot loop control",
                        "+ eligibility, ancestor test, ballot", "V3 + two broadcast reads (H[q], H[0])",
                        "V3 + one broadcast read", "V2 + loop control every 4th step", "V7 + exec-masked start writes"};
    for (int v = 0; v <= 8; ++v) std::printf("V%d %-40s %6.1f cycles/step\n", v, nm[v], (double)hv[v] / STEPS);
    return 0;
}
