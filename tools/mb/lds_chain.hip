// Microbenchmark: cycles per iteration of dependent LDS chains in one wave (gfx950), as the heap
// tier's pop pipeline runs them. Each variant loops N times; s_memtime brackets the loop.
//   hipcc --offload-arch=gfx950 -O3 tools/mb/lds_chain.hip -o /tmp/lds_chain && /tmp/lds_chain
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned long long u64;
constexpr int N = 4096, SZ = 8192;

template <int V>
__global__ void k_chain(u64* out, int lanes) {
    __shared__ uint2 H[SZ];
    const int l = threadIdx.x;
    for (int i = l; i < SZ; i += 64) H[i] = make_uint2((unsigned)((i * 7 + 3) % (SZ - 2)), (unsigned)i);
    __syncthreads();
    if (l >= lanes) return;
    int h = l;
    unsigned acc = 0;
    const u64 t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N; ++it) {
        if (V == 0) {                               // dependent ds_read_b64
            const uint2 a = H[h];
            h = (int)a.x;
        } else if (V == 1) {                        // dependent ds_read2_b64 + compare/select
            const uint2 a = H[h], b = H[h + 1];
            h = (int)(b.y < a.y ? a.x : b.x);
        } else if (V == 2) {                        // read2 + select + write of the hole
            const uint2 a = H[h], b = H[h + 1];
            const bool r = !(b.y < a.y);
            H[(h ^ 1) + 4096] = r ? b : a;
            h = (int)(r ? b.x : a.x);
        } else if (V == 3) {                        // V2 + 10 dependent VALU ops on the path
            const uint2 a = H[h], b = H[h + 1];
            const bool r = !(b.y < a.y);
            H[(h ^ 1) + 4096] = r ? b : a;
            int x = (int)(r ? b.x : a.x);
#pragma unroll
            for (int k = 0; k < 10; ++k) x = (x * 3 + k) & (SZ - 2);
            h = x;
        }
        asm volatile("" ::: "memory");
    }
    const u64 t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) out[0] = t1 - t0;
    if (h == -1) out[1] = acc;
}

int main() {
    u64* d;
    (void)hipMalloc(&d, 16);
    const char* names[] = {"ds_read_b64 chain", "read2_b64 + select", "read2 + select + write", "+ 10 VALU"};
    for (int lanes : {1, 16, 64}) {
        for (int v = 0; v < 4; ++v) {
            u64 c = 0;
            for (int rep = 0; rep < 3; ++rep) {
                switch (v) {
                    case 0: hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, d, lanes); break;
                    case 1: hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, d, lanes); break;
                    case 2: hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, d, lanes); break;
                    default: hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, d, lanes); break;
                }
                (void)hipDeviceSynchronize();
                (void)hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
            }
            // s_memtime counts at the shader clock here (tools/heap_prof.py measured 2.4 GHz)
            printf("lanes %2d  %-26s %6.1f cycles/iter\n", lanes, names[v], (double)c / N);
        }
    }
    return 0;
}
