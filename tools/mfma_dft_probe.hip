// Bounded experiment: one radix-8 stage of k_front3's 512-point in-wave
// sub-FFT on the fp32 matrix cores instead of VALU + the LDS transpose T1.
//
// The stage as a GEMM: 64 independent 8-point complex DFTs per wave = a real [16 x 16] DFT matrix
// ([[Wr, -Wi], [Wi, Wr]]) times a [16 x 64] block of data: 4 column blocks x 4 k-steps of
// v_mfma_f32_16x16x4_f32 = 16 MFMAs per wave per stage (each lane feeds 16 B values = its 8
// complex inputs and receives 16 D values = 8 complex outputs). Timed here against the shipped
// VALU form of the same stage (radix-8 butterfly in packed FP32, 7 twiddle multiplies, the T1
// exchange through the wave's LDS region: 8 ds_write_b64 + 8 ds_read_b64), each as a chain of
// dependent stages per wave, at 16 waves per CU (k_front3's occupancy) and at 4 (one per SIMD).
// Timing only (the MFMA operand layout is not wired to the FFT's index maps); the result is the
// cost of the stage, which bounds what the substitution can gain.
//
//   hipcc -O3 --offload-arch=gfx950 -I mkids_sdr_amd/csrc -o build/mfma_dft_probe tools/mfma_dft_probe.hip
//   build/mfma_dft_probe            (prints one JSON line)
#include <hip/hip_runtime.h>

#include <cstdio>

#include "fft_common.h"

using namespace mkid;

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 2048;

__global__ __launch_bounds__(1024) void stage_valu(float2* out, int waves_per_block) {
    __shared__ float2 lds[16 * 576];
    const int wave = threadIdx.x >> 6, L = threadIdx.x & 63;
    if (wave >= waves_per_block) return;
    float2* reg = lds + wave * 576;
    float2 v[8], w[7];
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = make_float2(1.0f + 1e-3f * (L + r), 0.5f - 1e-3f * r);
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        float s, c;
        __sincosf(-6.2831853f * (float)(L * (k + 1)) / 512.0f, &s, &c);
        w[k] = make_float2(c, s);
    }
    for (int it = 0; it < kIters; ++it) {
        dft<8>(v);
#pragma unroll
        for (int k = 1; k < 8; ++k) v[k] = cmul_pk(v[k], w[k - 1]);
#pragma unroll
        for (int r = 0; r < 8; ++r) reg[72 * r + L] = v[r];
        __builtin_amdgcn_wave_barrier();
        const float2* rd = reg + 72 * (L >> 3) + (L & 7);
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = rd[8 * r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = make_float2(v[r].x * 0.125f, v[r].y * 0.125f);   // keep the values bounded
    }
    float2 s = make_float2(0.f, 0.f);
#pragma unroll
    for (int r = 0; r < 8; ++r) s = cadd(s, v[r]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(1024) void stage_mfma(float2* out, int waves_per_block) {
    const int wave = threadIdx.x >> 6, L = threadIdx.x & 63;
    if (wave >= waves_per_block) return;
    // A operand per k-step: this lane's element of the real DFT matrix, row L % 16, column 4 ks + L / 16
    float a[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const int row = L & 15, col = 4 * ks + (L >> 4);
        const int k = row >> 1, n = col >> 1;
        float s, c;
        __sincosf(-6.2831853f * (float)(k * n) / 8.0f, &s, &c);
        a[ks] = (row & 1) == (col & 1) ? c * 0.125f : ((row & 1) ? s : -s) * 0.125f;
    }
    f32x4 d[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
        d[nb] = f32x4{1.0f + 1e-3f * (L + nb), 0.5f, 0.25f, -0.5f};
    for (int it = 0; it < kIters; ++it) {
        f32x4 e[4];
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ks], d[nb][ks], acc, 0, 0, 0);
            e[nb] = acc;
        }
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) d[nb] = e[nb];
    }
    float2 s = make_float2(0.f, 0.f);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) s = cadd(s, make_float2(d[nb][0] + d[nb][2], d[nb][1] + d[nb][3]));
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static float time_kernel(void (*k)(float2*, int), float2* out, int blocks, int wpb) {
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1.f;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(1024), 0, 0, out, wpb);   // warm-up
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(1024), 0, 0, out, wpb);
    (void)hipEventRecord(e1, 0);
    float ms = -5.f;
    if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) ms = -5.f;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms / 5.f;
}

int main() {
    int ncu = 0, clk_khz = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || ncu <= 0) return 1;
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    float2* out = nullptr;
    if (hipMalloc(&out, (size_t)ncu * 1024 * sizeof(float2)) != hipSuccess) return 1;
    std::printf("{\"cus\": %d, \"iters\": %d, \"clock_mhz_attr\": %.0f", ncu, kIters, clk_khz / 1e3);
    for (int wpb : {16, 4}) {
        const float tv = time_kernel(stage_valu, out, ncu, wpb);
        const float tm = time_kernel(stage_mfma, out, ncu, wpb);
        // ns per stage per wave (each wave runs kIters dependent stages; all waves run together)
        std::printf(", \"waves_per_cu_%d\": {\"valu_lds_ns_per_stage\": %.2f, \"mfma_ns_per_stage\": %.2f, "
                    "\"mfma_over_valu\": %.3f}",
                    wpb, tv * 1e6 / kIters, tm * 1e6 / kIters, tm / tv);
    }
    std::printf("}\n");
    (void)hipFree(out);
    return 0;
}
