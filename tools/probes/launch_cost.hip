// Development probe: per-kernel cost of a dependent chain of small kernels on one stream, replayed
// from a hipGraph, as a function of grid size and per-thread work (trivial / one dependent global
// load / grid-stride over 30k items). Prints microseconds per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_trivial(int* p) {
    if (blockIdx.x == 0 && threadIdx.x == 0) p[0] += 1;
}
__global__ void k_stride(const float4* __restrict__ in, float4* __restrict__ out, const int* __restrict__ d_n) {
    const int n = *d_n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        float4 v = in[i];
        v.x += 1.0f;
        out[i] = v;
    }
}

int main() {
    int* d;
    float4 *a, *b;
    int* dn;
    const int n = 30000;
    hipMalloc(&d, 64);
    hipMalloc(&a, sizeof(float4) * (1 << 20));
    hipMalloc(&b, sizeof(float4) * (1 << 20));
    hipMalloc(&dn, 4);
    hipMemcpy(dn, &n, 4, hipMemcpyHostToDevice);
    hipMemset(a, 0, sizeof(float4) * (1 << 20));
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const int chain = 40;
    int grids[] = {1, 32, 128, 256, 512, 1024};
    for (int kind = 0; kind < 2; ++kind) {
        for (int g : grids) {
            hipGraph_t gr;
            hipGraphExec_t ge;
            hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
            for (int i = 0; i < chain; ++i) {
                if (kind == 0) hipLaunchKernelGGL(k_trivial, dim3(g), dim3(256), 0, s, d);
                else hipLaunchKernelGGL(k_stride, dim3(g), dim3(256), 0, s, (i & 1) ? b : a, (i & 1) ? a : b, dn);
            }
            hipStreamEndCapture(s, &gr);
            hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
            for (int w = 0; w < 5; ++w) hipGraphLaunch(ge, s);
            hipStreamSynchronize(s);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            const int reps = 50;
            hipEventRecord(e0, s);
            for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, s);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("%s grid %5d blocks: %.2f us per kernel\n", kind == 0 ? "trivial " : "stride30k", g,
                   ms * 1000.0 / (reps * chain));
            hipGraphExecDestroy(ge);
            hipGraphDestroy(gr);
        }
    }
    return 0;
}
