// Probe of the gfx950 cross-lane primitives the k_front v2 FFT transposes rely on (semantics
// check on hardware): v_permlane32_swap, v_permlane16_swap, DPP row_ror / row_shl / row_shr.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
    const int l = threadIdx.x;
    int x = l, y = 100 + l;
    auto r32 = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    auto r16 = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    out[0 * 64 + l] = r32[0];
    out[1 * 64 + l] = r32[1];
    out[2 * 64 + l] = r16[0];
    out[3 * 64 + l] = r16[1];
    out[4 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x124, 0xf, 0xf, false);  // row_ror:4
    out[5 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x104, 0xf, 0xf, false);  // row_shl:4
    out[6 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    out[7 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x128, 0xf, 0xf, false);  // row_ror:8
}
int main() {
    int* d; hipMalloc(&d, 8 * 64 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[8 * 64]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[8] = {"pl32.x", "pl32.y", "pl16.x", "pl16.y", "ror4", "shl4", "shr4", "ror8"};
    for (int r = 0; r < 8; ++r) {
        printf("%s:", nm[r]);
        for (int l = 0; l < 64; ++l) printf(" %d", h[r * 64 + l]);
        printf("\n");
    }
    return 0;
}
