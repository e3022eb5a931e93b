// Development microbenchmark: the per-frame cost of the stage-B stream's packets around a graph.
// A graph of K short kernels (each spins ~T us on one workgroup) replayed N times on stream B:
//   mode 0: graphs back to back
//   mode 1: + hipEventRecord after each graph
//   mode 2: + hipStreamWaitEvent on an event recorded by stream A (one short kernel per frame on A)
//   mode 3: both (the odometry's pattern)
// prints us per replay and per kernel boundary.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_spin(unsigned long long ticks, int* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 1;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 11;
    const double T = argc > 2 ? atof(argv[2]) : 5.0;
    const int N = 2000;
    const unsigned evf = hipEventDisableTiming | (argc > 3 ? (unsigned)strtoul(argv[3], nullptr, 0) : 0u);
    printf("event flags 0x%x\n", evf);
    int* sink;
    CK(hipMalloc(&sink, 64));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    const unsigned long long ticks = (unsigned long long)(T * 100.0);   // 100 MHz realtime counter
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(sb, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, sb, ticks, sink);
    CK(hipStreamEndCapture(sb, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    std::vector<hipEvent_t> ea(3), eb(3);
    for (int i = 0; i < 3; ++i) {
        CK(hipEventCreateWithFlags(&ea[i], evf));
        CK(hipEventCreateWithFlags(&eb[i], evf));
    }
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, sb));
            for (int f = 0; f < N; ++f) {
                const int p = f % 3;
                if (mode & 2) {
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, sa, 10ull, sink);
                    CK(hipEventRecord(ea[p], sa));
                    CK(hipStreamWaitEvent(sb, ea[p], 0));
                }
                CK(hipGraphLaunch(ge, sb));
                if (mode & 1) CK(hipEventRecord(eb[p], sb));
            }
            CK(hipEventRecord(t1, sb));
            CK(hipEventSynchronize(t1));
            float ms;
            CK(hipEventElapsedTime(&ms, t0, t1));
            const double per = 1000.0 * ms / N;
            if (rep) printf("mode %d (record %d, wait %d): %.2f us per replay of %d x %.1f us kernels -> %.2f us overhead, %.2f per kernel\n",
                            mode, mode & 1, (mode >> 1) & 1, per, K, T, per - K * T, (per - K * T) / K);
        }
    }
    // eager launches for comparison
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(t0, sb));
        for (int f = 0; f < N; ++f)
            for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, sb, ticks, sink);
        CK(hipEventRecord(t1, sb));
        CK(hipEventSynchronize(t1));
        float ms;
        CK(hipEventElapsedTime(&ms, t0, t1));
        const double per = 1000.0 * ms / N;
        if (rep) printf("eager: %.2f us per %d kernels -> %.2f per kernel overhead\n", per, K, (per - K * T) / K);
    }
    return 0;
}
