// Development probe: which lane each DPP / permlane move reads from (prints 6 x 64 source lanes).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(int* out) {
    const int l = threadIdx.x;
    const int v = l;
    const auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    const auto r16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    out[0 * 64 + l] = r32[0];
    out[1 * 64 + l] = r32[1];
    out[2 * 64 + l] = r16[0];
    out[3 * 64 + l] = r16[1];
    out[4 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x124, 0xf, 0xf, false);   // row_ror:4
    out[5 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x12C, 0xf, 0xf, false);   // row_ror:12
    out[6 * 64 + l] = __builtin_amdgcn_update_dpp(-1, v, 0x128, 0xf, 0xf, false);   // row_ror:8
}

int main() {
    int* d;
    int h[7 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const char* names[7] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]", "ror4", "ror12", "ror8"};
    for (int r = 0; r < 7; ++r) {
        std::printf("%-7s", names[r]);
        for (int l = 0; l < 64; ++l) std::printf(" %d", h[r * 64 + l]);
        std::printf("\n");
    }
    return 0;
}
