// Development repro: host SIGSEGV inside hipGraphLaunch under `rocprofv3 --kernel-trace` (VERDICT r04
// weak 4; gpurun_out/r05a/traced.txt). The crashing read is made by librocprofiler-sdk.so from an HSA
// queue-intercept callback and runs off the end of a 1 MiB shared mapping: the size of an AQL ring of
// 16384 packets x 64 B. A graph's kernels are submitted as one batch of packets, and a batch that
// straddles the end of the ring is read linearly past it by the tool's callback.
// This program replays a graph of K trivial kernels R times on one stream (nothing of the pipeline):
//   K = 16 divides 16384, so no batch ever straddles the ring's end;
//   K = 15 (or 17) does, at the first wrap (about 16384 / K replays).
//   hipcc --offload-arch=gfx950 -O2 tools/mb/graph_ring.hip -o /tmp/graph_ring
//   rocprofv3 --kernel-trace -d out -- /tmp/graph_ring 15 3000
// prints a line every 200 replays and "done" at the end.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_touch(int* sink, int v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) sink[0] = v;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    const int K = argc > 1 ? std::atoi(argv[1]) : 15;
    const int R = argc > 2 ? std::atoi(argv[2]) : 3000;
    const bool eager = argc > 3 && std::atoi(argv[3]) != 0;
    int* sink;
    CK(hipMalloc(&sink, 64));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, sink, k);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < R; ++r) {
        if (eager) {
            for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, sink, k);
        } else {
            CK(hipGraphLaunch(ge, s));
        }
        if (r % 200 == 0) {
            CK(hipStreamSynchronize(s));
            std::fprintf(stderr, "K %d replay %d (%ld packets)\n", K, r, (long)r * K);
        }
    }
    CK(hipStreamSynchronize(s));
    std::printf("done K %d R %d %s\n", K, R, eager ? "eager" : "graph");
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
}
