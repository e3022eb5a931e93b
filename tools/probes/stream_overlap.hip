// Probe: do chains of small kernels on two streams (or two branches of one graph) overlap on gfx950?
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_small(float* p, int iters) {
    float v = p[threadIdx.x];
    for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;
    if (v == 12345.f) p[threadIdx.x] = v;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    float *a, *b;
    hipMalloc(&a, 4096); hipMalloc(&b, 4096);
    hipStream_t s1, s2;
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    const int N = 60, iters = 2000;
    for (int rep = 0; rep < 2; ++rep) {
        hipDeviceSynchronize();
        double t0 = now();
        for (int i = 0; i < 2 * N; ++i) hipLaunchKernelGGL(k_small, dim3(4), dim3(64), 0, s1, a, iters);
        hipStreamSynchronize(s1);
        double t1 = now();
        for (int i = 0; i < N; ++i) {
            hipLaunchKernelGGL(k_small, dim3(4), dim3(64), 0, s1, a, iters);
            hipLaunchKernelGGL(k_small, dim3(4), dim3(64), 0, s2, b, iters);
        }
        hipStreamSynchronize(s1); hipStreamSynchronize(s2);
        double t2 = now();
        // graph with two independent branches
        hipGraph_t g; hipGraphExec_t ge;
        hipEvent_t fork, join;
        hipEventCreateWithFlags(&fork, hipEventDisableTiming); hipEventCreateWithFlags(&join, hipEventDisableTiming);
        hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal);
        hipEventRecord(fork, s1);
        hipStreamWaitEvent(s2, fork, 0);
        for (int i = 0; i < N; ++i) {
            hipLaunchKernelGGL(k_small, dim3(4), dim3(64), 0, s1, a, iters);
            hipLaunchKernelGGL(k_small, dim3(4), dim3(64), 0, s2, b, iters);
        }
        hipEventRecord(join, s2);
        hipStreamWaitEvent(s1, join, 0);
        hipStreamEndCapture(s1, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        hipGraphLaunch(ge, s1); hipStreamSynchronize(s1);
        double t3 = now();
        hipGraphLaunch(ge, s1); hipStreamSynchronize(s1);
        double t4 = now();
        // single-stream graph of 2N
        hipGraph_t g2; hipGraphExec_t ge2;
        hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < 2 * N; ++i) hipLaunchKernelGGL(k_small, dim3(4), dim3(64), 0, s1, a, iters);
        hipStreamEndCapture(s1, &g2);
        hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0);
        hipGraphLaunch(ge2, s1); hipStreamSynchronize(s1);
        double t5 = now();
        hipGraphLaunch(ge2, s1); hipStreamSynchronize(s1);
        double t6 = now();
        printf("one stream %d launches: %.1f us/launch | two streams: %.1f us/pair | 2-branch graph: %.1f us/pair | 1-branch graph: %.1f us/launch\n",
               2 * N, (t1 - t0) / (2 * N) * 1e6, (t2 - t1) / N * 1e6, (t4 - t3) / N * 1e6, (t6 - t5) / (2 * N) * 1e6);
    }
    return 0;
}
